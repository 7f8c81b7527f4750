#!/usr/bin/env python3
"""Cost of the end-of-cycle .history path at C4 scale: rank 0's work after
the gather for --games games x ~58 plies of synthetic compact records (690 B per ply, the PLY_DTYPE
the ranks send): unpack (sort by game id), rebuild the (9,9,3) inputs from the packed states on the
host rules, build the reference's list schema (self_play_cpp.py:95-99) and pickle it to a file
(self_play_cpp.py:125-130). One JSON line.
usage: python tools/bench_history.py [--games 32768] [--plies 58] [--out /tmp/x.history]
"""
import argparse
import json
import os
import pickle
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=32768)
    ap.add_argument("--plies", type=int, default=58)
    import tempfile
    ap.add_argument("--out", default=os.path.join(tempfile.gettempdir(), "bench_history.history"))
    ap.add_argument("--keep", action="store_true")
    args = ap.parse_args()
    import numpy as np
    from uttt_amd import distributed as D
    from uttt_amd import history as H
    from uttt_amd.selfplay import history_from_records

    rng = np.random.RandomState(0)
    n = args.games * args.plies
    plies = np.zeros(n, D.PLY_DTYPE)
    plies["game"] = np.repeat(np.arange(args.games, dtype=np.int64), args.plies)
    st = plies["state"]
    st["own"] = rng.randint(0, 1 << 27, size=(n, 3)) & rng.randint(0, 1 << 27, size=(n, 3))
    st["opp"] = rng.randint(0, 1 << 27, size=(n, 3)) & ~st["own"] & ((1 << 27) - 1)
    st["active"] = rng.randint(-1, 9, size=n)
    plies["policy"] = rng.dirichlet(np.ones(81), size=n)
    plies["action"] = rng.randint(0, 81, size=n)
    plies["value"] = rng.randint(-1, 2, size=n)
    perm = rng.permutation(args.games)  # ranks deliver blocks in rank order; shuffle game blocks
    plies = plies.reshape(args.games, args.plies)[perm].reshape(-1)
    out = {"metric": ".history path on rank 0 after the gather (seconds)", "games": args.games, "plies": n,
           "compact_bytes": int(plies.nbytes)}
    t = time.perf_counter()
    recs = D.unpack_records(plies)
    out["unpack_s"] = round(time.perf_counter() - t, 3)
    t = time.perf_counter()
    recs = D.records_to_inputs(recs)
    out["inputs_s"] = round(time.perf_counter() - t, 3)
    t = time.perf_counter()
    hist = history_from_records(recs)
    out["list_build_s"] = round(time.perf_counter() - t, 3)
    t = time.perf_counter()
    with open(args.out, "wb") as f:
        pickle.dump(hist, f)
    out["pickle_dump_s"] = round(time.perf_counter() - t, 3)
    out["pickle_bytes"] = os.path.getsize(args.out)
    del hist
    t = time.perf_counter()
    H.write_history_file(recs, args.out + ".fast")
    out["fast_writer_s"] = round(time.perf_counter() - t, 3)
    out["fast_writer_bytes"] = os.path.getsize(args.out + ".fast")
    out["fast_equals_pickle_bytes"] = H.files_equal(args.out, args.out + ".fast")
    if not args.keep:
        os.remove(args.out)
        os.remove(args.out + ".fast")
    out["reference_path_s"] = round(out["unpack_s"] + out["inputs_s"] + out["list_build_s"] + out["pickle_dump_s"], 3)
    out["fast_path_s"] = round(out["unpack_s"] + out["inputs_s"] + out["fast_writer_s"], 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
