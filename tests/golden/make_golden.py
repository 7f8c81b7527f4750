"""Generate the golden fixtures under tests/golden/ from the REFERENCE itself.

Runs only in the build container (it needs /root/reference and oracle/_ref/,
built by ``make -C oracle``). The committed .npz files are data: inputs and the
reference's outputs on them. Nothing of the reference's source travels.

Sources of truth used here:
  * oracle/_ref/libuttt_ref.so — cpp/uttt_game.cpp + cpp/uttt_mcts.cpp compiled
    from the reference checkout (rules, pv_mcts_scores with the hash evaluator);
  * oracle/_ref/uttt_cpp*.so + the reference's self_play_cpp.py / pv_mcts_cpp.py
    imported from /root/reference (self-play with numpy's global RNG seeded
    per game), driven by oracle.hashnp.HashModel;
  * the reference's dual_network.py (DualNetwork under torch.manual_seed(0),
    CPU fp32) for the network I/O fixtures: network.npz (the seed-0 net as
    initialised, saturated) and netcal.npz (the same net with calibrated
    BatchNorm statistics: O(1) values, spread policies);
  * the reference's pv_mcts.py (Python PV-MCTS, its module constants set per
    case) and evaluate_network.py play() with two salted hash players, numpy's
    global RNG seeded per game (pvpy.npz, the arena path).

Usage:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py [--only pvpy|netcal]
"""
import json
import os
import random
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)

from oracle import ref  # noqa: E402

SEARCH_CONFIGS = [(50, 8), (50, 1), (50, 1024), (400, 8), (10, 2), (30, 3), (1, 1), (7, 100), (64, 64)]
TEMPERATURES = [1.0, 0.0, 0.5]


def initial():
    return (np.zeros((9, 9), np.int32), np.zeros((9, 9), np.int32), np.zeros(9, np.int32),
            np.zeros(9, np.int32), -1)


def pack(st):
    p, e, m, me, a = st
    return (np.asarray(p, np.uint8).reshape(81), np.asarray(e, np.uint8).reshape(81),
            np.asarray(m, np.uint8), np.asarray(me, np.uint8), np.int8(a))


def gen_rules(n_games=120, seed=7):
    rng = random.Random(seed)
    cols = {k: [] for k in ("pieces", "enemy", "main_p", "main_e", "active", "legal", "n_legal",
                            "flags", "tensor", "action", "game")}
    odd = {k: [] for k in ("pieces", "enemy", "main_p", "main_e", "active", "action",
                           "n_pieces", "n_enemy", "n_main_p", "n_main_e", "n_active")}
    strings = []
    q7 = 0
    for g in range(n_games):
        st = initial()
        while True:
            legal = ref.legal_actions(st)
            fl = ref.flags(st)
            p, e, m, me, a = pack(st)
            mask = np.zeros(81, np.uint8)
            mask[legal] = 1
            t = ref.tensor(st)
            act = rng.choice(legal) if legal else -1
            for k, v in (("pieces", p), ("enemy", e), ("main_p", m), ("main_e", me), ("active", a),
                         ("legal", mask), ("n_legal", len(legal)), ("flags", fl),
                         ("tensor", t.astype(np.uint8)), ("action", act), ("game", g)):
                cols[k].append(v)
            if (rng.random() < 0.02 or not legal) and len(strings) < 48:
                strings.append({"state": [p.tolist(), e.tolist(), m.tolist(), me.tolist(), int(a)],
                                "text": ref.to_string(st)})
            # next() on arbitrary in-range actions (occupied cells, closed boards): pin the
            # reference's unvalidated transition (uttt_game.cpp:97-145)
            if rng.random() < 0.15:
                ax = rng.randrange(81)
                nx = pack(ref.next_state(st, ax))
                for k, v in (("pieces", p), ("enemy", e), ("main_p", m), ("main_e", me), ("active", a),
                             ("action", ax), ("n_pieces", nx[0]), ("n_enemy", nx[1]), ("n_main_p", nx[2]),
                             ("n_main_e", nx[3]), ("n_active", nx[4])):
                    odd[k].append(v)
            if not legal:
                break
            nst = ref.next_state(st, act)
            b = act // 9
            if nst[2][b] == 1 and nst[3][b] == 1:
                q7 += 1
            st = nst
    out = {k: np.asarray(v) for k, v in cols.items()}
    out.update({"odd_" + k: np.asarray(v) for k, v in odd.items()})
    return out, strings, q7


def sample_positions(rules, n=40, seed=11):
    rng = np.random.RandomState(seed)
    live = np.nonzero(rules["n_legal"] > 0)[0]
    idx = rng.choice(live, size=n, replace=False)
    pos = []
    for i in sorted(idx.tolist()):
        pos.append((rules["pieces"][i].reshape(9, 9).astype(np.int32), rules["enemy"][i].reshape(9, 9).astype(np.int32),
                    rules["main_p"][i].astype(np.int32), rules["main_e"][i].astype(np.int32), int(rules["active"][i])))
    return pos


def win_in_one():
    """Side to move can win the game now (SURVEY App. A Q4 case)."""
    p, e, m, me, _ = initial()
    # side to move owns small boards 0 and 1; board 2 has own stones on cells 0,1
    m[0] = m[1] = 1
    for b in (0, 1):
        p[b, 0] = p[b, 1] = p[b, 2] = 1
    p[2, 0] = p[2, 1] = 1
    e[3, 0] = e[3, 4] = e[4, 4] = e[5, 8] = e[6, 2] = e[7, 5] = e[8, 1] = 1
    e[2, 4] = 1
    return (p, e, m, me, 2)


def gen_search(positions):
    out = {"pos_" + k: [] for k in ("pieces", "enemy", "main_p", "main_e", "active")}
    for st in positions:
        p, e, m, me, a = pack(st)
        for k, v in (("pieces", p), ("enemy", e), ("main_p", m), ("main_e", me), ("active", a)):
            out["pos_" + k].append(v)
    res = {"scores": [], "n": [], "pos": [], "sims": [], "batch": [], "temp": [], "flushes": [], "evals": [],
           "uniq": []}
    for pi, st in enumerate(positions):
        for (S, B) in SEARCH_CONFIGS:
            for tau in TEMPERATURES:
                sc, stats = ref.search_hash(st, tau, S, B)
                row = np.zeros(81, np.float32)
                row[:sc.size] = sc
                for k, v in (("scores", row), ("n", sc.size), ("pos", pi), ("sims", S), ("batch", B), ("temp", tau),
                             ("flushes", stats[0]), ("evals", stats[1]), ("uniq", stats[2])):
                    res[k].append(v)
    out = {k: np.asarray(v) for k, v in out.items()}
    out.update({k: np.asarray(v) for k, v in res.items()})
    return out


def gen_selfplay(n_games=12, base_seed=1234):
    sys.path[:0] = [ref.REF_DIR, REF]
    import self_play_cpp  # reference driver (imports the reference-built uttt_cpp)
    from oracle.hashnp import make_hash_model
    model = make_hash_model()
    T, P, A, V, L, S = [], [], [], [], [], []
    real_choice = np.random.choice

    def recording_choice(*args, **kw):  # same RNG stream; just records the pick
        r = real_choice(*args, **kw)
        A.append(int(r))
        return r

    np.random.choice = recording_choice
    try:
        for g in range(n_games):
            np.random.seed(base_seed + g)
            h = self_play_cpp.play(model, True)
            for rec in h:
                T.append(np.asarray(rec[0], np.float32).reshape(243).astype(np.uint8))
                P.append(np.asarray(rec[1], np.float64))
                V.append(int(rec[2]))
            L.append(len(h))
            S.append(base_seed + g)
    finally:
        np.random.choice = real_choice
    assert len(A) == len(T)
    return {"tensors": np.asarray(T), "policies": np.asarray(P), "actions": np.asarray(A, np.int8),
            "values": np.asarray(V, np.int8), "lengths": np.asarray(L, np.int32),
            "seeds": np.asarray(S, np.int64)}


def gen_network(n_states=24):
    sys.path[:0] = [REF]
    import torch
    import dual_network  # reference network definition
    torch.manual_seed(0)
    net = dual_network.DualNetwork().eval()
    rules = np.load(os.path.join(HERE, "rules.npz"))
    idx = np.linspace(0, len(rules["n_legal"]) - 1, n_states).astype(int)
    hwc = rules["tensor"][idx].astype(np.float32).reshape(-1, 9, 9, 3)
    x = torch.from_numpy(np.ascontiguousarray(hwc.transpose(0, 3, 1, 2)))
    with torch.no_grad():
        p, v = net(x)
    # a fingerprint of the seed-0 weights (sum per tensor, f64) pins the init order
    fp = np.asarray([t.double().sum().item() for t in net.state_dict().values()], np.float64)
    names = np.asarray(list(net.state_dict().keys()))
    return {"x": x.numpy(), "policy": p.numpy(), "value": v.numpy(), "param_sums": fp, "param_names": names}


NETCAL_VFC2_SCALE = 1.0 / 16  # exact power of two


def gen_netcal(n_states=256):
    """A NON-saturated DualNetwork (the seed-0 init saturates: v = -1, one-hot policies) and the
    reference's own CPU fp32 outputs on it. The net: the reference's DualNetwork under
    torch.manual_seed(0), BatchNorm running statistics calibrated on 1,024 positions of rules.npz
    (one train-mode pass with momentum None = the batch statistics, as a trained net would carry),
    value_fc2.weight scaled by 1/16 (exact). The calibrated buffers are stored, so the network is
    rebuilt from the seed-0 init + these arrays (uttt_amd.model.calibrated_network)."""
    sys.path[:0] = [REF]
    import torch
    import dual_network  # reference network definition
    torch.manual_seed(0)
    net = dual_network.DualNetwork()
    rules = np.load(os.path.join(HERE, "rules.npz"))
    n = len(rules["n_legal"])
    cal = np.random.RandomState(3).choice(n, 1024, replace=False)
    xc = rules["tensor"][cal].astype(np.float32).reshape(-1, 9, 9, 3).transpose(0, 3, 1, 2)
    bns = [(name, m) for name, m in net.named_modules() if isinstance(m, torch.nn.BatchNorm2d)]
    for _, m in bns:
        m.momentum = None
        m.reset_running_stats()
    net.train()
    with torch.no_grad():
        net(torch.from_numpy(np.ascontiguousarray(xc)))
    net.eval()
    with torch.no_grad():
        net.value_fc2.weight.mul_(NETCAL_VFC2_SCALE)
    live = np.nonzero(rules["n_legal"] > 0)[0]
    rest = np.setdiff1d(live, cal)
    idx = np.sort(np.random.RandomState(5).choice(rest, n_states, replace=False))
    x = np.ascontiguousarray(rules["tensor"][idx].astype(np.float32).reshape(-1, 9, 9, 3).transpose(0, 3, 1, 2))
    with torch.no_grad():
        p, v = net(torch.from_numpy(x))
    fp = np.asarray([t.double().sum().item() for t in net.state_dict().values()], np.float64)
    return {"bn_names": np.asarray([nm for nm, _ in bns]),
            "bn_mean": np.concatenate([m.running_mean.numpy() for _, m in bns]).astype(np.float32),
            "bn_var": np.concatenate([m.running_var.numpy() for _, m in bns]).astype(np.float32),
            "bn_sizes": np.asarray([m.num_features for _, m in bns], np.int32),
            "vfc2_scale": np.float64(NETCAL_VFC2_SCALE), "rules_index": idx.astype(np.int64),
            "x": x.astype(np.uint8), "policy": p.numpy(), "value": v.numpy().reshape(-1),
            "param_sums": fp}


PY_CONFIGS = [(50, 8), (50, 1), (30, 3), (10, 2), (1, 1), (7, 100), (64, 64)]
ARENA_SALTS = (0, 0x5EED5EED12345678)


def gen_pvpy(positions, n_games=8, base_seed=4321):
    """pv_mcts.py (Python semantics) scores + evaluate_network.play games."""
    sys.path[:0] = [ref.REF_DIR, REF]
    import uttt_cpp  # reference build
    import pv_mcts  # reference Python MCTS
    import evaluate_network  # reference arena
    from oracle.hashnp import make_hash_model
    model = make_hash_model(0)
    out = {"pos_" + k: [] for k in ("pieces", "enemy", "main_p", "main_e", "active")}
    for st in positions:
        p, e, m, me, a = pack(st)
        for k, v in (("pieces", p), ("enemy", e), ("main_p", m), ("main_e", me), ("active", a)):
            out["pos_" + k].append(v)
    res = {"scores": [], "n": [], "pos": [], "sims": [], "batch": [], "temp": []}
    saved = (pv_mcts.PV_EVALUATE_COUNT, pv_mcts.MCTS_BATCH_SIZE)
    try:
        for pi, st in enumerate(positions):
            state = uttt_cpp.State(st[0].tolist(), st[1].tolist(), st[2].tolist(), st[3].tolist(), int(st[4]))
            for (S, B) in PY_CONFIGS:
                pv_mcts.PV_EVALUATE_COUNT, pv_mcts.MCTS_BATCH_SIZE = S, B
                for tau in TEMPERATURES:
                    row = np.zeros(81, np.float64)
                    try:
                        sc = np.asarray(pv_mcts.pv_mcts_scores(model, state, tau), np.float64)
                        row[:sc.size] = sc
                    except ZeroDivisionError:  # boltzman over all-zero visits (S <= B: only the
                        sc = None              # root was ever reached); recorded as n = -1
                    if sc is None:
                        res["scores"].append(row)
                        for k, v in (("n", -1), ("pos", pi), ("sims", S), ("batch", B), ("temp", tau)):
                            res[k].append(v)
                        continue
                    for k, v in (("scores", row), ("n", sc.size), ("pos", pi), ("sims", S), ("batch", B),
                                 ("temp", tau)):
                        res[k].append(v)
    finally:
        pv_mcts.PV_EVALUATE_COUNT, pv_mcts.MCTS_BATCH_SIZE = saved
    out = {k: np.asarray(v) for k, v in out.items()}
    out.update({k: np.asarray(v) for k, v in res.items()})
    # arena: game g = evaluate_network.play after np.random.seed(base_seed + g); even games
    # start with player 0 (salt ARENA_SALTS[0]), odd games with player 1 (evaluate_network.py:78-82)
    players = [pv_mcts.pv_mcts_action(make_hash_model(s), 1.0) for s in ARENA_SALTS]
    A, L, PT, SD = [], [], [], []
    real_choice = np.random.choice

    def recording_choice(*args, **kw):
        r = real_choice(*args, **kw)
        A.append(int(r))
        return r

    np.random.choice = recording_choice
    try:
        for g in range(n_games):
            np.random.seed(base_seed + g)
            n0 = len(A)
            acts = players if g % 2 == 0 else list(reversed(players))
            PT.append(float(evaluate_network.play(acts)))
            L.append(len(A) - n0)
            SD.append(base_seed + g)
    finally:
        np.random.choice = real_choice
    out.update({"arena_actions": np.asarray(A, np.int8), "arena_lengths": np.asarray(L, np.int32),
                "arena_points": np.asarray(PT, np.float64), "arena_seeds": np.asarray(SD, np.int64),
                "arena_salts": np.asarray(ARENA_SALTS, np.uint64)})
    # self_play.py (the Python self-play, BASELINE configs[0]): play(model) after np.random.seed(seed + g)
    import self_play  # reference module
    T, P, V, SL, SS, DT = [], [], [], [], [], set()
    for g in range(6):
        np.random.seed(base_seed + 100 + g)
        h = self_play.play(model)
        for rec in h:
            x = np.asarray(rec[0])
            DT.add(str(x.dtype))
            T.append(x.reshape(243).astype(np.uint8))
            P.append(np.asarray(rec[1], np.float64))
            V.append(int(rec[2]))
        SL.append(len(h))
        SS.append(base_seed + 100 + g)
    assert DT == {"float64"}, DT
    out.update({"sp_tensors": np.asarray(T), "sp_policies": np.asarray(P), "sp_values": np.asarray(V, np.int8),
                "sp_lengths": np.asarray(SL, np.int32), "sp_seeds": np.asarray(SS, np.int64)})
    return out


def main():
    assert ref.available(), "build oracle/_ref first: make -C oracle"
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "netcal":
        nc = gen_netcal()
        np.savez_compressed(os.path.join(HERE, "netcal.npz"), **nc)
        print("netcal:", len(nc["value"]), "states; value range", float(nc["value"].min()), float(nc["value"].max()),
              "; median max policy", float(np.median(nc["policy"].max(1))))
        return
    if "--only" in sys.argv and sys.argv[sys.argv.index("--only") + 1] == "pvpy":
        rules = dict(np.load(os.path.join(HERE, "rules.npz")))
        positions = sample_positions(rules) + [initial(), win_in_one()]
        pv = gen_pvpy(positions)
        np.savez_compressed(os.path.join(HERE, "pvpy.npz"), **pv)
        print("pvpy:", len(pv["n"]), "searches;", len(pv["arena_lengths"]), "arena games,",
              int(pv["arena_lengths"].sum()), "moves; points", pv["arena_points"].tolist(), "; self_play.py:",
              len(pv["sp_lengths"]), "games,", int(pv["sp_lengths"].sum()), "plies")
        return
    rules, strings, q7 = gen_rules()
    np.savez_compressed(os.path.join(HERE, "rules.npz"), **rules)
    with open(os.path.join(HERE, "to_string.json"), "w") as f:
        json.dump(strings, f, indent=0)
    print("rules:", len(rules["n_legal"]), "states; drawn small boards (Q7):", q7, "; odd next():",
          len(rules["odd_action"]))
    positions = sample_positions(rules) + [initial(), win_in_one()]
    search = gen_search(positions)
    np.savez_compressed(os.path.join(HERE, "search.npz"), **search)
    print("search:", len(search["n"]), "cases; max unique leaves per flush:", int(search["uniq"].max()))
    sp = gen_selfplay()
    np.savez_compressed(os.path.join(HERE, "selfplay.npz"), **sp)
    print("selfplay:", len(sp["lengths"]), "games,", int(sp["lengths"].sum()), "plies")
    nn = gen_network()
    np.savez_compressed(os.path.join(HERE, "network.npz"), **nn)
    print("network:", nn["x"].shape[0], "states")
    pv = gen_pvpy(positions)
    np.savez_compressed(os.path.join(HERE, "pvpy.npz"), **pv)
    print("pvpy:", len(pv["n"]), "searches;", len(pv["arena_lengths"]), "arena games")
    nc = gen_netcal()
    np.savez_compressed(os.path.join(HERE, "netcal.npz"), **nc)
    print("netcal:", len(nc["value"]), "states")


if __name__ == "__main__":
    main()
