#!/usr/bin/env python3
"""bench.py — self-play MCTS simulations/s on MI355X (BASELINE.json metric).

A step = one move of every concurrent game on this GPU: each game's search
runs `sims` simulations (uttt_mcts.cpp:109 iterations) with the leaf
evaluator = DualNetwork 128f x16 (random init, torch.manual_seed(0), fp32,
PyTorch-ROCm), then the move is sampled and recorded on device. Finished games
are replaced by new ones, so every step keeps `games` trees in flight.

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU; games sharded, no collective
                                                       on the data path — weak scaling)

Prints one JSON line (rank 0) with the select-kernel roofline (algorithmic
bytes / HIP-event time on the engine's stream) and the reference's own C++
search timed on the host cores (cpu_baseline).
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")
METRIC = "MCTS simulations/sec (whole node), 4096 games × 50 sims/move; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
FP32_PEAK_TFLOPS = 157.3       # MI355X_MICROARCH.md: FP32 (vector = matrix) peak


def select_traffic(trees_per_launch):
    """HBM bytes per k_select launch from the committed PMC summary (tools/pmc_select.sh ->
    tools/pmc_summary.py; FETCH_SIZE + WRITE_SIZE, separate passes, raw - see that file),
    when it was taken at this launch size; else None. A live bench run cannot read PMC."""
    import glob
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "pmc_select.json")), reverse=True):
        with open(f) as fh:
            d = json.load(fh)
        if d.get("trees_per_launch") == trees_per_launch:
            return {"bytes_per_launch": round(d["traffic_bytes_raw"]),
                    "read_bytes": round(d["fetch_bytes"]), "write_bytes": round(d["write_bytes"]),
                    "source": os.path.relpath(f, REPO)}
    return None


def nn_macs():
    f, k, r = 128, 9, 81
    macs = r * f * 3 * k + 32 * r * f * f * k          # stem + 16 blocks x 2 convs
    macs += r * 2 * f + 162 * 81 + r * 1 * f + 81 * 256 + 256  # heads
    return macs


NN_FLOP_PER_STATE = 2 * nn_macs()  # 0.765 GFLOP per evaluated position
# residual-tower MFMA flops actually executed per board / direct-equivalent flops per state
TOWER_MFMA_FRACTION = {"fused": 3 * 32 * 9 * 25 * 128 * 128 * 2 / NN_FLOP_PER_STATE,      # F(3x3,3x3), 3 f16 products
                       "fused-f32": 32 * 9 * 25 * 128 * 128 * 2 / NN_FLOP_PER_STATE}      # F(3x3,3x3), f32


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--games", type=int, default=4096, help="concurrent games per GPU")
    ap.add_argument("--sims", type=int, default=50)
    ap.add_argument("--batch", type=int, default=8, help="MCTS_BATCH_SIZE (per-tree flush size)")
    ap.add_argument("--evaluator", choices=["fused", "fused-f32", "nn", "nn-plain", "hash"],
                    default="fused")
    ap.add_argument("--age", type=int, default=100,
                    help="moves played before warmup so the timed population mixes all game phases")
    ap.add_argument("--cudnn-benchmark", type=int, default=1)
    ap.add_argument("--lanes", type=int, default=2,
                    help="engines per GPU, each on its own stream; their network evaluations overlap")
    ap.add_argument("--cache-log2", type=int, default=21, help="evaluation cache entries (log2); 0 = off")
    ap.add_argument("--tag", default="", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-baseline-child", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args()


# ------------------------------------------------------------- CPU baseline --
def cpu_baseline_child(seconds):
    """Reference C++ PV-MCTS (oracle/_ref: cpp/uttt_game.cpp + uttt_mcts.cpp + python_bindings.cpp
    compiled from the reference sources) driven like self_play_cpp.play, leaf evaluator = the same
    DualNetwork on the host cores (torch CPU fp32). Falls back to the C oracle port if _ref is absent."""
    import numpy as np
    import torch

    sys.path.insert(0, PKG)
    from uttt_amd.model import random_network

    net = random_network(0, "cpu")
    threads = torch.get_num_threads()
    ref_dir = os.path.join(REPO, "oracle", "_ref")
    kind = "reference"
    try:
        sys.path.insert(0, ref_dir)
        import uttt_cpp as ref_uttt  # the reference's own module, built from its sources
        assert os.path.dirname(os.path.abspath(ref_uttt.__file__)) == ref_dir
    except Exception:
        kind = "port"
        ref_uttt = None

    def infer(states):  # pv_mcts_cpp.py:37-78 glue
        x = np.stack([np.asarray(s.to_input_tensor(), np.float32).reshape(9, 9, 3) for s in states])
        x = torch.from_numpy(np.ascontiguousarray(x.transpose(0, 3, 1, 2)))
        with torch.no_grad():
            p, v = net(x)
        p, v = p.numpy(), v.numpy()
        return [(p[i], float(v[i][0])) for i in range(len(states))]

    rng = np.random.RandomState(1234)
    sims = moves = 0
    tree_only = None
    t0 = time.perf_counter()
    if ref_uttt is not None:
        state = ref_uttt.State()
        while time.perf_counter() - t0 < seconds:
            if state.is_done():
                state = ref_uttt.State()
            sc = np.array(ref_uttt.pv_mcts_scores(model=infer, state=state, temperature=1.0, evaluate_count=50,
                                                  batch_size=8), np.float64)
            legal = state.legal_actions()
            sc = sc / np.sum(sc)
            state = state.next(int(rng.choice(legal, p=sc)))
            sims += 50
            moves += 1
        dt = time.perf_counter() - t0
        from oracle import ref as refdrv
        if refdrv.available():
            tree_only, _ = refdrv.bench_tree(50, 8, 2000)
    else:
        from oracle import core
        s = core.OrState.initial()

        def ev(x):
            with torch.no_grad():
                p, v = net(torch.from_numpy(np.asarray(x, np.float32).reshape(1, 3, 9, 9)))
            return p.numpy()[0], float(v.numpy()[0, 0])

        while time.perf_counter() - t0 < seconds:
            if s.is_done():
                s = core.OrState.initial()
            sc, _, _ = core.pv_mcts_scores(s, 1.0, 50, 8, ev)
            legal = s.legal_actions()
            s = s.next(legal[int(np.argmax(sc))])
            sims += 50
            moves += 1
        dt = time.perf_counter() - t0
    print(json.dumps({"value": sims / dt, "unit": "simulations/s", "cores": threads, "kind": kind,
                      "sample": f"{moves} consecutive self-play moves (50 sims, MCTS_BATCH_SIZE 8, tau 1) of "
                                f"the reference C++ search + DualNetwork fp32 on {threads} CPU threads, "
                                f"{dt:.1f} s",
                      "tree_only_1core": tree_only}))


def run_cpu_baseline(seconds):
    env = dict(os.environ)
    env["HIP_VISIBLE_DEVICES"] = ""
    env["CUDA_VISIBLE_DEVICES"] = ""
    env["PYTHONPATH"] = REPO
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", "--cpu-seconds",
                        str(seconds)], capture_output=True, text=True, env=env, cwd=REPO, timeout=seconds * 20 + 300)
    for line in reversed(r.stdout.strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return {"value": None, "error": (r.stderr or r.stdout)[-400:]}


# ----------------------------------------------------------------- GPU bench --
def main():
    args = parse()
    if args.cpu_baseline_child:
        cpu_baseline_child(args.cpu_seconds)
        return
    import torch
    import torch.distributed as dist

    sys.path.insert(0, REPO)
    sys.path.insert(0, PKG)
    from uttt_amd import HashEvaluator, NetworkEvaluator, SelfPlay
    from uttt_amd.model import FoldedDualNetwork, random_network
    from uttt_amd.nnfast import FusedNetworkEvaluator

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)
    torch.backends.cudnn.benchmark = bool(args.cudnn_benchmark)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False

    G, S, B = args.games, args.sims, args.batch
    net = random_network(0, dev)
    model = FoldedDualNetwork(net).to(dev) if args.evaluator == "nn" else net
    sp = SelfPlay(G, S, B, 1.0, device=local, cache_log2=args.cache_log2, lanes=args.lanes)
    if args.evaluator == "hash":
        make_inner = HashEvaluator
    elif args.evaluator.startswith("fused"):
        conv = {"fused": "wino3h", "fused-f32": "wino3"}[args.evaluator]
        make_inner = lambda eng: FusedNetworkEvaluator(net, eng, conv=conv)  # noqa: E731
    else:
        make_inner = lambda eng: NetworkEvaluator(model, eng.max_trees)  # noqa: E731

    # NN timing: events around every evaluation on the stream it runs on (lanes
    # overlap, so busy time is the union of the intervals), and useful rows
    nn_stats = {"ms": 0.0, "rows": 0, "padded_rows": 0}
    ev_pairs = []
    pads = args.evaluator in ("nn", "nn-plain")

    def make_timed(eng):
        inner = make_inner(eng)

        def timed_eval(x, n):
            a = torch.cuda.Event(enable_timing=True)
            b = torch.cuda.Event(enable_timing=True)
            a.record()
            out = inner(x, n)
            b.record()
            ev_pairs.append((a, b))
            nn_stats["rows"] += n
            if pads:
                from uttt_amd.selfplay import _bucket
                nn_stats["padded_rows"] += _bucket(n, eng.max_trees)
            else:
                nn_stats["padded_rows"] += n
            return out

        timed_eval.needs_input = getattr(inner, "needs_input", True)
        return timed_eval

    sp.set_evaluator(make_timed)
    games_per_rank = 10**9
    arena = (args.age + args.warmup + args.steps + 2) * G
    sp.begin(rank * games_per_rank, (rank + 1) * games_per_rank, 1234, arena_plies=arena)

    # Setup (not warmup, not timed): age the population. All games start together
    # from the initial position; refilling finished slots with new games spreads
    # the slots over every phase of a game (openings, middle games with wide
    # child lists, endgames with terminal simulations) like continuous self-play.
    for _ in range(args.age):
        sp.step()
    for _ in range(args.warmup):
        sp.step()
    torch.cuda.synchronize()
    ev_pairs.clear()
    nn_stats.update(ms=0.0, rows=0, padded_rows=0)
    sp.reset_stats()
    sp.set_timing(True)
    rounds0, finished0 = sp.rounds, sp.finished

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    base = torch.cuda.Event(enable_timing=True)
    base.record()
    t0 = time.perf_counter()
    sims = 0
    for _ in range(args.steps):
        sims += sp.step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    torch.cuda.synchronize()
    ivs = sorted((base.elapsed_time(a), base.elapsed_time(b)) for a, b in ev_pairs)
    busy, cur = 0.0, None
    for lo, hi in ivs:
        if cur is None or lo > cur[1]:
            if cur is not None:
                busy += cur[1] - cur[0]
            cur = [lo, hi]
        else:
            cur[1] = max(cur[1], hi)
    if cur is not None:
        busy += cur[1] - cur[0]
    nn_stats["ms"] = busy
    nn_stats["sum_ms"] = sum(hi - lo for lo, hi in ivs)
    sel = sp.kernel_stats("select")
    app = sp.kernel_stats("apply")
    enc = sp.kernel_stats("encode")
    scan = sp.kernel_stats("scan")
    mend = sp.kernel_stats("move_end")
    rounds = sp.rounds - rounds0
    cache = sp.cache_stats() if args.cache_log2 else None

    tot = torch.tensor([float(sims), elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        s = tot[:1].clone()
        m = tot[1:].clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        tot = torch.cat([s, m])
    total_sims, max_elapsed = float(tot[0].item()), float(tot[1].item())

    if rank == 0:
        value = total_sims / max_elapsed
        sel_ms = sel["ms"]
        achieved = (sel["bytes"] / 1e9) / (sel_ms / 1e3) if sel_ms > 0 else 0.0
        flops = NN_FLOP_PER_STATE * nn_stats["rows"]
        nn_tflops = flops / (nn_stats["ms"] / 1e3) / 1e12 if nn_stats["ms"] > 0 else 0.0
        out = {
            "metric": METRIC,
            "value": round(value, 1),
            "unit": "simulations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(max_elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic: self-play from the initial position, games refilled as they end; "
                    "random-init DualNetwork (torch.manual_seed(0)); no checkpoint",
            "config": {
                "workload": f"{G} concurrent self-play games per GPU x {S} sims/move, MCTS_BATCH_SIZE {B}, "
                            f"tau 1.0, continuous self-play (finished games refilled; population aged "
                            f"{args.age} moves before warmup); one step = one move of every game",
                "games_per_gpu": G, "sims_per_move": S, "mcts_batch_size": B, "aged_moves": args.age,
                "eval_cache_log2": args.cache_log2,
                "lanes_per_gpu": args.lanes,
                "evaluator": {"fused": "DualNetwork 128f x16, f32 activations/accumulation, BN folded; residual-tower "
                                       "convs as a fused Winograd F(3x3,3x3) HIP kernel whose point GEMMs run as "
                                       "3-term split-f16 products on the f16 MFMA with f32 accumulation "
                                       "(csrc/wino3h_conv.hip; f32-level error, 1.4e-6 rel vs f64 per conv, tested "
                                       "at 1e-5), stem/heads HIP kernels (csrc/nn_kernels.hip)",
                              "fused-f32": "DualNetwork 128f x16 fp32, BN folded; residual-tower convs as a fused "
                                           "Winograd F(3x3,3x3) f32-MFMA HIP kernel (csrc/wino3_conv.hip), stem/heads "
                                           "HIP kernels (csrc/nn_kernels.hip)",
                              "nn": "DualNetwork 128f x16 fp32, BN folded, channels-last (PyTorch-ROCm/MIOpen)",
                              "nn-plain": "DualNetwork 128f x16 fp32 (PyTorch-ROCm/MIOpen)",
                              "hash": "device hash evaluator (no network)"}[args.evaluator],
                "parallelism": f"games sharded over {world} GPU(s), no data-path collective",
            },
            "roofline": {
                "kernel": "k_select (PUCT descent, one wave per tree)",
                "bound": "hbm",
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": (select_traffic(G // args.lanes) or {}).get("bytes_per_launch"),
                "traffic_detail": select_traffic(G // args.lanes),
                "algo_bytes_per_launch": round(sel["bytes"] / max(sel["launches"], 1)),
                "avg_launch_us": round(sel_ms * 1e3 / max(sel["launches"], 1), 2),
                "launches": sel["launches"],
            },
            "nn": {
                "rows_evaluated": nn_stats["rows"], "rows_padded": nn_stats["padded_rows"],
                "ms": round(nn_stats["ms"], 2), "share_of_step": round(nn_stats["ms"] / 1e3 / elapsed, 4),
                "lane_sum_ms": round(nn_stats["sum_ms"], 2),
                "achieved_tflops": round(nn_tflops, 2), "peak_tflops": FP32_PEAK_TFLOPS,
                "frac": round(nn_tflops / FP32_PEAK_TFLOPS, 4),
                "flops_basis": "direct-conv equivalent, 2 x MACs of dual_network.py per evaluated row "
                               "(Winograd kernels execute fewer MFMA flops; see mfma_executed_tflops)",
                "mfma_executed_tflops": (round(nn_tflops * TOWER_MFMA_FRACTION[args.evaluator], 2)
                                         if args.evaluator in TOWER_MFMA_FRACTION else None),
            },
            "breakdown_ms": {"select": round(sel_ms, 2), "apply": round(app["ms"], 2), "encode": round(enc["ms"], 2),
                             "scan": round(scan["ms"], 2), "move_end": round(mend["ms"], 2),
                             "nn": round(nn_stats["ms"], 2), "wall": round(elapsed * 1e3, 2)},
            "rounds_per_step": round(rounds / args.steps, 2),
            "games_finished_in_timed_steps": int(sp.finished - finished0),
            "eval_cache": (dict(cache, hit_rate=round(cache["hits"] / max(cache["hits"] + cache["misses"], 1), 4),
                                log2_capacity=args.cache_log2) if cache else None),
        }
        if not args.no_cpu_baseline:
            cb = run_cpu_baseline(args.cpu_seconds)
            out["cpu_baseline"] = cb
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
