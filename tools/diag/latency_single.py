#!/usr/bin/env python3
"""Per-call latency of the single-tree search paths a reference caller uses one move at a time
(INTEGRATION.md Option A): pv_mcts_cpp.pv_mcts_scores_cpp (the engine with the fused HIP evaluator,
one tree, 50 sims, batch 8) and pv_mcts.pv_mcts_scores (Python-search semantics on the engine), on
positions along one game; plus the conv alone at small batches. One JSON line."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    import pv_mcts_cpp
    import uttt_cpp
    from uttt_amd.model import random_network
    net = random_network(0, "cuda")
    rng = np.random.RandomState(0)
    states = []
    s = uttt_cpp.State()
    while not s.is_done() and len(states) < 40:
        states.append(s)
        s = s.next(int(rng.choice(s.legal_actions())))
    out = {"metric": "single-tree search latency (ms per call, one move, 50 sims, batch 8)"}
    # Option A: the reference's pv_mcts_cpp / self_play_cpp drivers unchanged over this
    # uttt_cpp. "torch": the reference's own flush glue (pv_mcts_cpp.py:37-87: to_input_tensor per state, NCHW
    # torch tensor, model(x), .cpu()) with the PyTorch DualNetwork; "fused": this build's pv_mcts_cpp, whose
    # callback hands the states to the fused HIP evaluator instead.
    for name, kind in (("pv_mcts_scores_cpp_fused", "auto"), ("pv_mcts_scores_cpp_torch", "torch")):
        os.environ["UTTT_EVALUATOR"] = kind
        fn = lambda st: pv_mcts_cpp.pv_mcts_scores_cpp(net, st, 1.0, 50, 8)  # noqa: E731
        for st in states[:3]:
            fn(st)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for st in states:
            fn(st)
        torch.cuda.synchronize()
        out[name] = round((time.perf_counter() - t) * 1e3 / len(states), 3)
    os.environ.pop("UTTT_EVALUATOR")
    # the same searches on the reference's own uttt_cpp (oracle/_ref, compiled from its sources; present where
    # the build ran __graft_entry__.build() beside /root/reference) with the reference's own flush glue
    # (pv_mcts_cpp.py:37-87: k states per flush, to_input_tensor each, NCHW torch tensor, model, .cpu()), and
    # this build's uttt_cpp under the same glue: the per-search difference is the module's own cost
    ref_dir = os.path.join(REPO, "oracle", "_ref")
    glue_calls = {"n": 0, "states": 0, "s": 0.0}

    def ref_glue(states_list):
        t0 = time.perf_counter()
        x = np.asarray([s.to_input_tensor() for s in states_list], dtype=np.float32).reshape(-1, 9, 9, 3)
        x = torch.from_numpy(np.ascontiguousarray(x.transpose(0, 3, 1, 2))).to("cuda")
        with torch.no_grad():
            p, v = net(x)
        p, v = p.cpu().numpy(), v.cpu().numpy()
        res = [(p[i], float(v[i][0])) for i in range(len(states_list))]
        glue_calls["n"] += 1
        glue_calls["states"] += len(states_list)
        glue_calls["s"] += time.perf_counter() - t0
        return res

    mods = [("this_uttt_cpp_reference_glue", uttt_cpp, {"dedup": False}),
            ("this_uttt_cpp_reference_glue_dedup", uttt_cpp, {"dedup": True})]
    if os.path.isdir(ref_dir):
        import importlib.machinery
        import importlib.util
        path = [os.path.join(ref_dir, f) for f in os.listdir(ref_dir) if f.startswith("uttt_cpp")][0]
        # the reference module's init function is PyInit_uttt_cpp: load it under that name, outside sys.modules
        loader = importlib.machinery.ExtensionFileLoader("uttt_cpp", path)
        spec = importlib.util.spec_from_file_location("uttt_cpp", path, loader=loader)
        ref_mod = importlib.util.module_from_spec(spec)
        loader.exec_module(ref_mod)
        mods.insert(0, ("reference_uttt_cpp_reference_glue", ref_mod, {}))
    out["same_glue"] = {}
    for name, mod, kw in mods:
        sts = [mod.State(s.pieces, s.enemy_pieces, s.main_board_pieces, s.main_board_enemy_pieces, s.active_board)
               for s in states]
        for st in sts[:3]:
            mod.pv_mcts_scores(model=ref_glue, state=st, temperature=1.0, evaluate_count=50, batch_size=8, **kw)
        torch.cuda.synchronize()
        glue_calls.update(n=0, states=0, s=0.0)
        t = time.perf_counter()
        for st in sts:
            mod.pv_mcts_scores(model=ref_glue, state=st, temperature=1.0, evaluate_count=50, batch_size=8, **kw)
        torch.cuda.synchronize()
        tot = (time.perf_counter() - t) * 1e3 / len(sts)
        out["same_glue"][name] = {"ms_per_search": round(tot, 3), "sims_per_s": round(50e3 / tot, 1),
                                  "flushes_per_search": round(glue_calls["n"] / len(sts), 2),
                                  "states_per_flush": round(glue_calls["states"] / max(glue_calls["n"], 1), 2),
                                  "glue_ms_per_search": round(glue_calls["s"] * 1e3 / len(sts), 3),
                                  "module_ms_per_search": round(tot - glue_calls["s"] * 1e3 / len(sts), 3)}
    # the modules alone: a model that returns fixed arrays (no device work), so a search's time is the module's
    # own (the reference's CPU tree; this build's select / apply kernels and the per-flush host round trip)
    fixed_p, fixed_v = np.full(81, 1.0 / 81, np.float32), 0.0
    out["module_only"] = {}
    for name, mod, kw in mods:
        sts = [mod.State(s.pieces, s.enemy_pieces, s.main_board_pieces, s.main_board_enemy_pieces, s.active_board)
               for s in states]
        fixed = lambda sl: [(fixed_p, fixed_v)] * len(sl)  # noqa: E731
        for st in sts[:3]:
            mod.pv_mcts_scores(model=fixed, state=st, temperature=1.0, evaluate_count=50, batch_size=8, **kw)
        t = time.perf_counter()
        for st in sts:
            mod.pv_mcts_scores(model=fixed, state=st, temperature=1.0, evaluate_count=50, batch_size=8, **kw)
        out["module_only"][name] = round((time.perf_counter() - t) * 1e3 / len(sts), 4)
    out["positions"] = len(states)
    # self_play_cpp.self_play's 500 games one move at a time: 26,651 plies in the build's 500-game cycle
    # (profiles/r3/cycle_fp32_final.json), i.e. 53.3 moves per game
    plies = 26651
    out["projected_500_games_s"] = {k: round(out[k] * plies / 1e3, 1) for k in
                                    ("pv_mcts_scores_cpp_fused", "pv_mcts_scores_cpp_torch")}
    out["projected_sims_per_s"] = {k: round(50 * 1e3 / out[k], 1) for k in
                                   ("pv_mcts_scores_cpp_fused", "pv_mcts_scores_cpp_torch")}
    out["reference_published_ms"] = {"mcts_50_sims": 50.0, "source": "README.md:290 (4070 Ti + 5800X)"}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
