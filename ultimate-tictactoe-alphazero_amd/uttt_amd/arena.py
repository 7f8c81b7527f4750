"""Batched arena evaluation on the Python PV-MCTS semantics.

The reference's evaluate_network.py plays EN_GAME_COUNT games one after
another, each move a pv_mcts.py search (Python objects, one network call per
flush of <= 8 leaves). Here all games advance together: per move, the games
whose side to move plays model m form one batched search on engine m
(UTTT_SEMANTICS_PY: root evaluated by the first flush, expand replaces,
PUCT as NumPy 2 evaluates pv_mcts.py:120-130), and each round evaluates one
leaf per game in a single network call.

Game g draws its moves from RandomState(seed_base + g), so its record equals
the reference's play() after np.random.seed(seed_base + g) (same players).
"""
import numpy as np

from .engine import as_states
from .selfplay import BatchedSearch, NetworkEvaluator


def scores_from_visits(visits, temperature):
    """pv_mcts.py:175-181 on the root children's visit counts: one-hot first maximum
    (temperature 0, float64 array) or boltzman in Python floats (:190-192, a list;
    raises ZeroDivisionError like the reference when no child was visited)."""
    ns = [int(x) for x in visits]
    if temperature == 0:
        s = np.zeros(len(ns))
        s[int(np.argmax(ns))] = 1
        return s
    xs = [x ** (1 / temperature) for x in ns]
    return [x / sum(xs) for x in xs]


def first_player_point(state):
    """evaluate_network.py:26-30."""
    if state.is_lose():
        return 0 if state.is_first_player() else 1
    return 0.5


def _engine_state(state):
    import uttt_cpp
    if isinstance(state, uttt_cpp.State):
        return state
    return uttt_cpp.State(state.pieces, state.enemy_pieces, state.main_board_pieces, state.main_board_enemy_pieces,
                          state.active_board)


class PvMcts:
    """pv_mcts.py:133-181 for many root states at once (one tree each)."""

    def __init__(self, max_trees, max_sims=50, device=None):
        self.search = BatchedSearch(max_trees, max_sims, device)
        self.engine = self.search.engine

    def visits(self, states, evaluator, evaluate_count=50, batch_size=8):
        """states: uttt_cpp.State / game.State objects or a packed STATE_DTYPE array
        -> list of root-children visit counts (int arrays, legal-action order)."""
        roots = as_states(states) if isinstance(states, np.ndarray) else as_states([_engine_state(s) for s in states])
        self.search.run(roots, evaluator, evaluate_count, batch_size, semantics="py")
        v, L = self.search.visits()
        return [v[i, :L[i]].copy() for i in range(len(roots))]

    def scores(self, states, evaluator, temperature, evaluate_count=50, batch_size=8):
        return [scores_from_visits(v, temperature) for v in self.visits(states, evaluator, evaluate_count, batch_size)]


class ModelEvaluator:
    """A DualNetwork-shaped model (model(x) -> policies (N,81), values (N,1)) as an engine
    evaluator; inputs are moved to the model's device (models may live on the CPU)."""

    def __init__(self, model):
        import torch
        self.model = model.eval()
        self.dev = next((p.device for p in model.parameters()), None)
        self.torch = torch

    def __call__(self, x, n):
        with self.torch.no_grad():
            xi = x[:n] if self.dev is None else x[:n].to(self.dev)
            p, v = self.model(xi)
        return p.to(x.device).float(), v.to(x.device).float().reshape(n, -1)


def model_evaluator(model, max_batch=None, engine=None, kind=None):
    """Engine evaluator for a model: the fused HIP evaluator for a DualNetwork (given the engine;
    nnfast.evaluator_kind), else NetworkEvaluator when the model lives on the GPU (no copies),
    ModelEvaluator otherwise."""
    if engine is not None:
        from .nnfast import FusedNetworkEvaluator, evaluator_kind
        if evaluator_kind(model, kind) == "fused":
            return FusedNetworkEvaluator(model, engine)
    dev = next((p.device for p in model.parameters()), None)
    if dev is not None and dev.type == "cuda" and max_batch:
        model.eval()
        return NetworkEvaluator(model, max_batch)
    return ModelEvaluator(model)


def evaluate_network(model0, model1, game_count=50, temperature=1.0, seed_base=0, evaluate_count=50,
                     batch_size=8, device=None, make_evaluator=None, progress=None):
    """evaluate_network.py:58-104 with all games concurrent. Game g: model0 moves first when g is
    even, model1 when odd (:78-82). Returns (model0's average point, per-game first-player points,
    per-game action lists). make_evaluator(model, engine) -> engine evaluator (default: the model
    called on the engine's input batch; e.g. nnfast.FusedNetworkEvaluator for a DualNetwork)."""
    import uttt_cpp
    searches = [PvMcts(game_count, evaluate_count, device) for _ in range(2)]
    if make_evaluator is None:
        evaluators = (model_evaluator(model0, game_count, searches[0].engine),
                      model_evaluator(model1, game_count, searches[1].engine))
    else:
        evaluators = (make_evaluator(model0, searches[0].engine), make_evaluator(model1, searches[1].engine))
    states = [uttt_cpp.State() for _ in range(game_count)]
    rngs = [np.random.RandomState(seed_base + g) for g in range(game_count)]
    order = [(0, 1) if g % 2 == 0 else (1, 0) for g in range(game_count)]  # (first player, second player)
    actions = [[] for _ in range(game_count)]
    while True:
        live = [g for g in range(game_count) if not states[g].is_done()]
        if not live:
            break
        groups = [[g for g in live if order[g][0 if states[g].is_first_player() else 1] == m] for m in (0, 1)]
        for m, idx in enumerate(groups):  # one move per live game per iteration
            if not idx:
                continue
            vis = searches[m].visits([states[g] for g in idx], evaluators[m], evaluate_count, batch_size)
            for g, v in zip(idx, vis):
                legal = states[g].legal_actions()
                sc = scores_from_visits(v, temperature)
                if len(sc) != len(legal):
                    raise ValueError(f"Score size mismatch: scores={len(sc)}, legal_actions={len(legal)}")
                a = int(rngs[g].choice(legal, p=sc))
                actions[g].append(a)
                states[g] = states[g].next(a)
        if progress:
            progress(game_count - len(live), game_count)
    points = [first_player_point(s) for s in states]
    total = sum(p if g % 2 == 0 else 1 - p for g, p in enumerate(points))
    return total / game_count, points, actions


def first_player_value(state):
    """self_play.py:20-25."""
    if state.is_lose():
        return -1 if state.is_first_player() else 1
    return 0


def self_play_py(model, game_count, seed_base=0, temperature=1.0, evaluate_count=50, batch_size=8, device=None,
                 make_evaluator=None, progress=None):
    """self_play.py:66-99 (the Python self-play: pv_mcts.py searches) for game_count games at once.
    Game g draws from RandomState(seed_base + g) (= play(model) after np.random.seed(seed_base + g)).
    Returns one history per game: [input (9,9,3) float64, policies (81 Python floats, 0 for
    illegal actions), value (first_player_value at ply 0, then alternating)]."""
    import uttt_cpp
    search = PvMcts(game_count, evaluate_count, device)
    ev = make_evaluator(model, search.engine) if make_evaluator else model_evaluator(model, game_count, search.engine)
    states = [uttt_cpp.State() for _ in range(game_count)]
    rngs = [np.random.RandomState(seed_base + g) for g in range(game_count)]
    hist = [[] for _ in range(game_count)]
    while True:
        live = [g for g in range(game_count) if not states[g].is_done()]
        if not live:
            break
        vis = search.visits([states[g] for g in live], ev, evaluate_count, batch_size)
        for g, v in zip(live, vis):
            st = states[g]
            legal = st.legal_actions()
            scores = scores_from_visits(v, temperature)
            policies = [0] * 81
            for action, policy in zip(legal, scores):
                policies[action] = policy
            x = np.asarray(st.to_input_tensor(), dtype=np.float64).reshape(9, 9, 3)
            hist[g].append([x, policies, None])
            states[g] = st.next(int(rngs[g].choice(legal, p=scores)))
        if progress:
            progress(game_count - len(live), game_count)
    for g in range(game_count):
        value = first_player_value(states[g])
        for rec in hist[g]:
            rec[2] = value
            value = -value
    return hist


__all__ = ["ModelEvaluator", "first_player_value", "self_play_py", "PvMcts", "evaluate_network", "first_player_point", "model_evaluator",
           "scores_from_visits"]
