#!/usr/bin/env python3
"""bench.py — self-play MCTS simulations/s on MI355X (BASELINE.json metric).

A step = one move of every concurrent game on this GPU: each game's search
runs `sims` simulations (uttt_mcts.cpp:109 iterations) with the leaf
evaluator = DualNetwork 128f x16 (random init, torch.manual_seed(0): the
network the reference's dual_network() writes as best.pth), then the move is
sampled and recorded on device. Finished games are replaced by new ones, so
every step keeps `games` trees in flight.

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU; games sharded by global id in
                                                       contiguous blocks, no collective on the data path)

Rank 0 prints ONE JSON line: the headline (BASELINE.json's 4096 x 50 config), the
roofline of the dominant kernel (the residual-tower conv, MFMA), the north star's
select and backup kernels against HBM, and - at N=1 - extra configurations
(`variants`: non-saturated network, evaluation cache off, C3 4096 x 400) and
the CPU baselines (`cpu_baseline`: the reference's own C++ search with its
DualNetwork on the host cores; `cpu_baselines`: BASELINE.md's B-tree and B-e2e).
"""
import argparse
import ctypes
import glob
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")
METRIC = "MCTS simulations/sec (whole node), 4096 games × 50 sims/move; 1/2/4/8 GPU"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
F16_DENSE_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: BF16/F16 MFMA ~2.5 PF dense
NETCAL = os.path.join(REPO, "tests", "golden", "netcal.npz")

# residual-tower conv, per board: MFMA flops the kernels issue, and the direct 3x3 conv's flops
CONV_EXEC_FLOP = {"wino3h": 3 * 9 * 25 * 128 * 128 * 2,  # F(3x3,3x3): 9 tiles x 25 points, 3 f16 products
                  "wino3h_f16": 9 * 25 * 128 * 128 * 2}   # the f16 mode: one product
CONV_DIRECT_FLOP = 2 * 81 * 128 * 1152
CONV_PEAK = {"wino3h": F16_DENSE_PEAK_TFLOPS, "wino3h_f16": F16_DENSE_PEAK_TFLOPS}
# residual-tower conv, algorithmic HBM bytes per board: read x, write y (+ read the residual on
# every second conv); the transformed weights (1.6 MB) are read once per launch, L2/MALL-resident
CONV_BYTES_PER_BOARD = 81 * 128 * 4 * 2.5


def nn_macs():
    f, k, r = 128, 9, 81
    macs = r * f * 3 * k + 32 * r * f * f * k          # stem + 16 blocks x 2 convs
    macs += r * 2 * f + 162 * 81 + r * 1 * f + 81 * 256 + 256  # heads
    return macs


NN_FLOP_PER_STATE = 2 * nn_macs()  # 0.765 GFLOP per evaluated position


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)  # ~1.8 s timed: resolution below 1%
    ap.add_argument("--warmup", type=int, default=6)
    ap.add_argument("--games", type=int, default=4096, help="concurrent games per GPU")
    ap.add_argument("--sims", type=int, default=50)
    ap.add_argument("--batch", type=int, default=8, help="MCTS_BATCH_SIZE (per-tree flush size)")
    ap.add_argument("--evaluator", choices=["fused", "nn", "hash", "fused_f16"], default="fused",
                    help="fused: the HIP network at f32-level accuracy (the measurement); fused_f16: its optional "
                         "one-product f16 mode (not the reference's numerics; a variant line only)")
    ap.add_argument("--net", choices=["seed0", "calibrated"], default="seed0",
                    help="seed0: the reference's initial best.pth; calibrated: tests/golden/netcal.npz")
    ap.add_argument("--age", type=int, default=300,
                    help="moves played before warmup so the timed population mixes all game phases and the "
                         "evaluation cache is at its steady state (hit rate 35.7%% at 100 moves, 30.1%% at 300, "
                         "31.8%% at 700)")
    ap.add_argument("--lanes", type=int, default=2,
                    help="engines per GPU, each on its own stream; their network evaluations overlap")
    ap.add_argument("--cache-log2", type=int, default=23, help="evaluation cache entries (log2); 0 = off")
    ap.add_argument("--cache-clear-every", type=int, default=0,
                    help="moves between evaluation-cache clears (0: never; full probe windows replace entries)")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-variants", action="store_true")
    ap.add_argument("--no-isolated", action="store_true",
                    help="skip the isolated conv timing after the timed region (rocprof window runs)")
    # rehearsal of the multi-rank path on a one-GPU box: every rank on device 0, gloo instead of RCCL
    ap.add_argument("--rehearse-shared-gpu", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--cpu-baseline-child", choices=["cpu-nn", "tree", "device-nn"], help=argparse.SUPPRESS)
    return ap.parse_args()


def newest_profile(name, match):
    """The newest committed profiles/r*/<name> JSON whose fields equal `match` (PMC summaries:
    a live bench cannot read counters)."""
    for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", name)), reverse=True):
        try:
            with open(f) as fh:
                d = json.load(fh)
        except (OSError, ValueError):  # unreadable: never let a stray file stop the measurement
            continue
        if isinstance(d, dict) and all(d.get(k) == v for k, v in match.items()):
            d["source"] = os.path.relpath(f, REPO)
            return d
    return None


# ------------------------------------------------------------- CPU baselines --
def _ref_uttt():
    """The reference's own uttt_cpp (oracle/_ref, compiled from its sources by oracle/Makefile)."""
    ref_dir = os.path.join(REPO, "oracle", "_ref")
    sys.path.insert(0, ref_dir)
    import uttt_cpp as ref_uttt
    assert os.path.dirname(os.path.abspath(ref_uttt.__file__)) == ref_dir
    return ref_uttt


def _serial_selfplay(ref_uttt, infer, seconds, rng):
    """self_play_cpp.play's loop (self_play_cpp.py:47-93) on the reference search: moves until the
    time is up, games restarted as they end. Returns (sims, moves, seconds)."""
    import numpy as np
    sims = moves = 0
    state = ref_uttt.State()
    t0 = time.perf_counter()
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
    return sims, moves, time.perf_counter() - t0


def cpu_baseline_child(kind, seconds):
    import numpy as np

    sys.path[:0] = [REPO, PKG]
    if kind == "tree":
        # B-tree: the reference's C++ search alone (hash evaluator, no network),
        # one game per process on the box's host cores
        import multiprocessing as mp
        from oracle import ref as refdrv
        procs = max(1, min(16, os.cpu_count() or 1))
        moves = max(200, int(seconds * 3000))
        with mp.get_context("fork").Pool(procs) as pool:
            t0 = time.perf_counter()
            res = pool.starmap(refdrv.bench_tree, [(50, 8, moves)] * procs)
            dt = time.perf_counter() - t0
        # the processes run concurrently: the node's rate is the sum of their own rates
        print(json.dumps({"value": round(sum(r for r, _ in res), 1), "unit": "simulations/s", "cores": procs,
                          "kind": "reference",
                          "sample": f"{procs} processes x {moves} consecutive 50-sim moves (MCTS_BATCH_SIZE 8) of the "
                                    f"reference's C++ search with the deterministic hash evaluator, {dt:.1f} s",
                          "per_core": round(float(np.mean([r for r, _ in res])), 1)}))
        return
    import torch
    from uttt_amd.model import random_network
    ref_uttt = _ref_uttt()
    if kind == "cpu-nn":
        dev = torch.device("cpu")
    else:
        dev = torch.device("cuda", 0)
    net = random_network(0, dev)
    threads = torch.get_num_threads()

    def infer(states):  # pv_mcts_cpp.py:37-78 glue
        x = np.stack([np.asarray(s.to_input_tensor(), np.float32).reshape(9, 9, 3) for s in states])
        x = torch.from_numpy(np.ascontiguousarray(x.transpose(0, 3, 1, 2))).to(dev)
        with torch.no_grad():
            p, v = net(x)
        p, v = p.cpu().numpy(), v.cpu().numpy()
        return [(p[i], float(v[i][0])) for i in range(len(states))]

    if kind == "device-nn":
        _serial_selfplay(ref_uttt, infer, 2.0, np.random.RandomState(0))  # MIOpen / allocator warmup
    sims, moves, dt = _serial_selfplay(ref_uttt, infer, seconds, np.random.RandomState(1234))
    where = f"DualNetwork fp32 on {threads} CPU threads" if kind == "cpu-nn" else \
        "DualNetwork fp32 on the MI355X (PyTorch-ROCm, one flush of <= 8 states per call)"
    print(json.dumps({"value": sims / dt, "unit": "simulations/s", "cores": threads if kind == "cpu-nn" else 1,
                      "kind": "reference",
                      "sample": f"{moves} consecutive self-play moves (50 sims, MCTS_BATCH_SIZE 8, tau 1) of the "
                                f"reference's C++ search (oracle/_ref, built from its sources) + {where}, {dt:.1f} s"}))


def run_cpu_baseline(kind, seconds):
    env = dict(os.environ, PYTHONPATH=REPO)
    if kind != "device-nn":
        env["HIP_VISIBLE_DEVICES"] = ""
        env["CUDA_VISIBLE_DEVICES"] = ""
    r = subprocess.run([sys.executable, os.path.abspath(__file__), "--cpu-baseline-child", kind, "--cpu-seconds",
                        str(seconds)], capture_output=True, text=True, env=env, cwd=REPO, timeout=seconds * 20 + 300)
    for line in reversed(r.stdout.strip().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    return {"value": None, "error": (r.stderr or r.stdout)[-400:]}


# ----------------------------------------------------------------- GPU bench --
def union_ms(intervals):
    busy, cur = 0.0, None
    for lo, hi in sorted(intervals):
        if cur is None or lo > cur[1]:
            if cur is not None:
                busy += cur[1] - cur[0]
            cur = [lo, hi]
        else:
            cur[1] = max(cur[1], hi)
    return busy + (cur[1] - cur[0] if cur is not None else 0.0)


def run_config(net, local, rank, world, games, sims, batch, lanes, cache_log2, age, warmup, steps, evaluator,
               cache_clear_every=0, instrument=True):
    """Continuous self-play of `games` slots on this GPU; returns the timed-window statistics."""
    import torch
    import torch.distributed as dist
    from uttt_amd import HashEvaluator, NetworkEvaluator, SelfPlay
    from uttt_amd.distributed import shard
    from uttt_amd.model import FoldedDualNetwork
    from uttt_amd.nnfast import FusedNetworkEvaluator

    dev = torch.device("cuda", local)
    sp = SelfPlay(games, sims, batch, 1.0, device=local, cache_log2=cache_log2, lanes=lanes,
                  cache_clear_every=cache_clear_every)
    conv = {"fused": "wino3h", "fused_f16": "wino3h"}.get(evaluator)
    tower_events = []
    if evaluator == "hash":
        make_inner = HashEvaluator
    elif conv:
        def make_inner(eng):
            fe = FusedNetworkEvaluator(net, eng, conv=conv, precision="f16" if evaluator == "fused_f16" else "f32")
            fe.tower_events = tower_events
            return fe
    else:
        folded = FoldedDualNetwork(net).to(dev)
        make_inner = lambda eng: NetworkEvaluator(folded, eng.max_trees)  # noqa: E731
    ev_pairs = []
    rows = []  # per network call: n, or the RoundCount the async round loop fills in

    def make_timed(eng):
        inner = make_inner(eng)

        def timed_eval(x, n):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            out = inner(x, n)
            b.record()
            ev_pairs.append((a, b))
            rows.append(n)
            return out

        timed_eval.needs_input = getattr(inner, "needs_input", True)
        timed_eval.device_count = getattr(inner, "device_count", False)
        return timed_eval

    # the hash evaluator runs inside the engine's one-call rounds (Engine.round_hash_async): no per-round
    # Python evaluator call to wrap; its time is the engine's own dispatch-event telemetry ("hash_eval")
    # instrument=False: no events anywhere in the timed region (the engine's per-dispatch events cost the
    # tree-only configuration a quarter of its rate); the kernel statistics then come from
    # a separate instrumented pass
    if instrument:
        sp.set_evaluator(HashEvaluator if evaluator == "hash" else make_timed)
    else:  # no events anywhere in the timed region (no evaluator wrapper, no tower events)
        def make_plain(eng):
            ev = make_inner(eng)
            if hasattr(ev, "tower_events"):
                ev.tower_events = None
            return ev
        sp.set_evaluator(HashEvaluator if evaluator == "hash" else make_plain)
    # continuous self-play: rank r owns the contiguous block r of global game ids (the same
    # scheme as self_play_cpp's torchrun sharding), large enough for every game it can start
    per_rank = (age + warmup + steps + 2) * games
    gb, ge = shard(per_rank * world, rank, world)
    sp.begin(gb, ge, 1234, arena_plies=per_rank)
    sp.steps(age + warmup)
    torch.cuda.synchronize()
    ev_pairs.clear()
    tower_events.clear()
    rows.clear()
    sp.reset_stats()
    # UTTT_BENCH_KERNEL_TIMING=0: no per-dispatch events in the timed region (the value without their cost;
    # the kernel rooflines then have no times)
    sp.set_timing(instrument)
    rounds0, finished0, leaves0 = sp.rounds, sp.finished, sp.leaves
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    base = torch.cuda.Event(enable_timing=True)
    base.record()
    t0 = time.perf_counter()
    done = sp.steps(steps)  # every lane plays `steps` moves (lanes pipelined across moves)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    torch.cuda.synchronize()
    ivs = [(base.elapsed_time(a), base.elapsed_time(b)) for a, b in ev_pairs]
    # rounds enqueued before their count was known may have had no leaf (the move's last select)
    tower = [(int(n), a.elapsed_time(b)) for n, a, b in tower_events if int(n) > 0]
    st = {k: sp.kernel_stats(k) for k in ("select", "apply", "scan", "move_end", "select_levels", "select_trees",
                                          "select_max_levels_sum", "select_trips", "select_max_trips_sum", "hash_eval")}
    if evaluator == "hash":
        n_rows, nn_ms, nn_sum = sp.leaves - leaves0, st["hash_eval"]["ms"], st["hash_eval"]["ms"]
    else:
        n_rows, nn_ms, nn_sum = sum(int(n) for n in rows), union_ms(ivs), sum(hi - lo for lo, hi in ivs)
    out = {"sims": done, "elapsed": elapsed, "rows": n_rows, "nn_ms": nn_ms,
           "nn_lane_sum_ms": nn_sum, "tower": tower, "stats": st,
           "rounds": sp.rounds - rounds0, "finished": sp.finished - finished0,
           "conv": "wino3h_f16" if evaluator == "fused_f16" else conv,
           "cache": sp.cache_stats() if cache_log2 else None, "trees_per_launch": games // lanes}
    del sp
    torch.cuda.empty_cache()
    return out


def summarize(r, steps):
    """Compact statistics of one run_config result (rank-local)."""
    out = {"value": round(r["sims"] / r["elapsed"], 1), "ms_per_step": round(r["elapsed"] / steps * 1e3, 3),
           "nn_share_of_step": round(r["nn_ms"] / 1e3 / r["elapsed"], 4), "rows_per_step": round(r["rows"] / steps, 1),
           "rounds_per_step": round(r["rounds"] / steps, 2)}
    if r["cache"]:
        c = r["cache"]
        out["eval_cache_hit_rate"] = round(c["hits"] / max(c["hits"] + c["misses"], 1), 4)
    return out


def conv_roofline(r, steps):
    """The dominant kernel: one residual-tower conv launch. achieved = executed MFMA flops per launch
    / the launch's average duration, from HIP events recorded on the lane's stream around each forward's
    32 launches (so the few-us launch gaps are included: conservative). Two lanes' launches overlap, so
    that per-launch figure is not the kernel's share of the chip: chip_frac = every conv's executed flops
    in the timed steps / the steps' wall time / peak, beside the per-step sum of conv launch time (which
    exceeds ms_per_step by the overlap)."""
    conv = r["conv"]
    if not conv or not r["tower"]:
        return None
    ncv = 32
    boards = sum(n for n, _ in r["tower"])
    ms = sum(t for _, t in r["tower"])
    launches = ncv * len(r["tower"])
    chip_tflops = CONV_EXEC_FLOP[conv] * ncv * boards / r["elapsed"] / 1e12
    avg_us = ms * 1e3 / launches
    boards_per_launch = boards / len(r["tower"])
    flop = CONV_EXEC_FLOP[conv] * boards_per_launch
    achieved = flop / (avg_us * 1e-6) / 1e12
    dataflow = conv == "wino3h" and os.environ.get("UTTT_NN_TOWER", "layers") == "dataflow"
    kname = "k_wino3t_tower" if dataflow else "k_wino3h_conv"
    pmc = newest_profile("pmc_conv.json", {"kernel": kname}) if conv == "wino3h" else None
    traffic = round(pmc["hbm_bytes_per_board"] * boards_per_launch) if pmc else None
    algo_bytes = CONV_BYTES_PER_BOARD * boards_per_launch + U_BYTES_PER_SET // (2 if conv == "wino3h_f16" else 1)
    arith = 'f16 MFMA, 3-term split-f16 products, f32 accumulation' if conv == 'wino3h' else 'f16 MFMA, one product'
    label = (f"k_wino3t_tower (the residual tower's 32 3x3 convs as ONE persistent dataflow launch, Winograd "
             f"F(3x3,3x3) on the {arith}; per conv-equivalent: a launch's duration / 32)" if dataflow else
             f"k_wino3h_conv (residual-tower 3x3 conv, Winograd F(3x3,3x3) on the {arith})")
    return {"kernel": label,
            "bound": "mfma", "achieved": round(achieved, 2), "peak": CONV_PEAK[conv], "unit": "TFLOP/s",
            "frac": round(achieved / CONV_PEAK[conv], 4),
            "chip_achieved": round(chip_tflops, 2), "chip_frac": round(chip_tflops / CONV_PEAK[conv], 4),
            "conv_launch_ms_per_step": round(ms / steps, 3), "ms_per_step": round(r["elapsed"] / steps * 1e3, 3),
            "frac_basis": ("frac: per conv-equivalent (HIP events around each forward's tower launch on its lane's "
                           "stream, / 32; the other lane's launches share the CUs meanwhile)" if dataflow else
                           "frac: per launch (HIP events around a forward's 32 launches on its lane's stream; the "
                           "other lane's launches share the CUs meanwhile)") +
                          "; chip_frac: all conv flops of the timed steps / their wall time (conv_launch_ms_per_step / "
                          "ms_per_step = the lanes' overlap)",
            "tower_launches": len(r["tower"]) if dataflow else None,
            "tower_avg_launch_us": round(ms * 1e3 / len(r["tower"]), 1) if dataflow else None,
            "traffic": traffic,
            "traffic_detail": ({k: pmc[k] for k in ("hbm_bytes_per_board", "fetch_bytes_per_board_x2",
                                                    "write_bytes_per_board", "source") if k in pmc} if pmc else None),
            "algo_hbm_bytes_per_launch": round(algo_bytes),
            "avg_launch_us": round(avg_us, 2), "launches": launches, "boards_per_launch": round(boards_per_launch, 1),
            "executed_flop_per_board": CONV_EXEC_FLOP[conv], "direct_equiv_flop_per_board": CONV_DIRECT_FLOP,
            "direct_equiv_tflops": round(CONV_DIRECT_FLOP * boards_per_launch / (avg_us * 1e-6) / 1e12, 1),
            "vmem_stream": conv_vmem_roofline(r["tower"], avg_us, r["nn_ms"],
                                              U_BYTES_PER_SET // (2 if conv == "wino3h_f16" else 1)),
            "note": "two lanes' conv launches overlap on the GPU, so each launch's duration includes the time it "
                    "shares the CUs with the other lane's; aggregate = nn.mfma_executed_tflops"}


def isolated_conv(net, boards_list, reps=20):
    """The dominant kernel alone on the GPU (after the timed region, no other lane): the product
    launch of one tower conv (block 8's conv1 weights, plain and residual forms alternating as in
    the tower) on random post-ReLU inputs of n boards, HIP events on the launching stream around
    `reps` launches. Gives the kernel's own roofline beside the in-bench figure, whose launches
    share the CUs with the other lane's."""
    import torch
    from uttt_amd.model import fold_bn
    from uttt_amd.nnfast import board_amax, wino3h_weights, _p
    from uttt_amd import _lib
    lib = _lib.load()
    w, b = fold_bn(net.residual_blocks[8].conv1, net.residual_blocks[8].bn1)
    uh, su = wino3h_weights(w)
    uh, b = uh.cuda(), b.float().contiguous().cuda()
    stream = torch.cuda.current_stream()
    st = ctypes.c_void_p(stream.cuda_stream)
    out = []
    for n in boards_list:
        g = torch.Generator(device="cuda").manual_seed(n)
        x = torch.relu(torch.randn(n, 81, 128, device="cuda", generator=g))
        res = torch.relu(torch.randn(n, 81, 128, device="cuda", generator=g))
        y = torch.empty_like(x)
        ba = board_amax(x)

        def launch(i):
            rc = lib.uttt_nn_conv3x3_wino3h(_p(x), _p(uh), ctypes.c_float(su), _p(b), _p(res) if i & 1 else None,
                                            _p(y), _p(ba), 1, None, None, 0, n, st)
            if rc != 0:
                raise RuntimeError(f"uttt_nn_conv3x3_wino3h failed ({rc})")
        for i in range(4):
            launch(i)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        for i in range(reps):
            launch(i)
        e1.record(stream)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        tf = CONV_EXEC_FLOP["wino3h"] * n / (us * 1e-6) / 1e12
        out.append({"boards": n, "avg_launch_us": round(us, 2), "achieved": round(tf, 2),
                    "frac": round(tf / CONV_PEAK["wino3h"], 4)})
        del x, res, y
    return {"unit": "TFLOP/s", "peak": CONV_PEAK["wino3h"], "points": out,
            "basis": "one launch at a time, no other lane (block 8 conv1 weights, random post-ReLU inputs, plain and "
                     "residual forms alternating); the headline roofline above is the in-bench figure"}


def isolated_tower(net, boards_list, reps=10):
    """The dataflow tower (k_wino3t_tower, UTTT_NN_TOWER=dataflow) alone on the GPU after the timed region:
    HIP events around `reps` launches over n boards' stem outputs (opening positions), per conv-equivalent
    (launch / 32) beside the per-conv kernel's isolated figure."""
    import torch
    import uttt_amd
    from uttt_amd.nnfast import FusedNetworkEvaluator
    out = []
    for n in boards_list:
        fe = FusedNetworkEvaluator(net, None, max_batch=n, tower="dataflow")
        fe.forward_states(uttt_amd.initial_states(n))
        stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
        for _ in range(2):
            fe._tower_dataflow(stream, None, n)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fe._tower_dataflow(stream, None, n)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / reps
        tf = CONV_EXEC_FLOP["wino3h"] * 32 * n / (us * 1e-6) / 1e12
        out.append({"boards": n, "avg_launch_us": round(us, 1), "per_conv_us": round(us / 32, 2),
                    "achieved": round(tf, 2), "frac": round(tf / CONV_PEAK["wino3h"], 4)})
        del fe
        torch.cuda.empty_cache()
    return {"unit": "TFLOP/s", "peak": CONV_PEAK["wino3h"], "points": out,
            "basis": "one tower launch at a time, no other lane (opening positions' stem outputs, the run's network)"}


# Measured ceiling of the L2 -> CU vector-memory path for 16-byte lane-linear loads, every CU
# streaming (tools/diag/u_stream.hip: 95-108 GB/s per CU x 256 CUs); what bounds the conv's
# point GEMMs
L2_STREAM_CEILING_TBS = 27.7
U_BYTES_PER_SET = 25 * 128 * 128 * 4   # every 32-tile set streams all of U (f16 hi + lo) from L2


def conv_sets(n):
    """k_wino3h_conv sets of n boards: two per full group of 7, one or two for a partial group."""
    return 2 * (n // 7) + (0 if n % 7 == 0 else (1 if n % 7 <= 3 else 2))


def conv_vmem_roofline(tower, avg_us, nn_ms, u_bytes=U_BYTES_PER_SET):
    """The conv's binding resource: bytes through each CU's vector-memory path per launch (U once
    per set, inputs, outputs and residual per board) / launch time, against the measured ceiling.
    aggregate_*: every conv's bytes over the union of the lanes' forward intervals (stem and heads
    included, so conservative) -- the rate the chip sustains while two lanes' launches overlap."""
    per_fwd = [conv_sets(n) * u_bytes + CONV_BYTES_PER_BOARD * n for n, _ in tower]
    per_launch = sum(per_fwd) / len(tower)
    achieved = per_launch / (avg_us * 1e-6) / 1e12
    agg = 32 * sum(per_fwd) / (nn_ms * 1e-3) / 1e12 if nn_ms > 0 else 0.0
    return {"bytes_per_launch": round(per_launch), "achieved": round(achieved, 2), "ceiling": L2_STREAM_CEILING_TBS,
            "unit": "TB/s", "frac": round(achieved / L2_STREAM_CEILING_TBS, 4),
            "aggregate_achieved": round(agg, 2), "aggregate_frac": round(agg / L2_STREAM_CEILING_TBS, 4),
            "basis": "U (1.6 MB) streamed from L2 by every 32-tile set + 103.7 KB per board of activations; ceiling "
                     "= lane-linear 16-B loads with every CU streaming (tools/diag/u_stream.hip)"}


def chase_latency(chase):
    """tools/diag/chase.hip's dependent-load latency at k_select's concurrency (2,048 waves, loads
    missing the XCD's L2): the unit of the select latency model."""
    if not chase:
        return None
    for c in chase["configs"]:
        if c["waves"] == 2048 and c["loads"] == "plain" and c["span_bytes"] >= 1 << 30:
            return {"us": c.get("us_per_step_events", c["us_mean"]), "source": chase["source"]}
    return None


def fetch_factor():
    """FETCH_SIZE correction for the tree kernels' reads, measured on their own load shapes
    (tools/diag/fetch_cal.hip at k_select's concurrency, profiles/r*/fetch_cal.json): FETCH_SIZE counts 64 B
    per L2 read request whatever its size, so 16-B-per-lane loads of L consecutive 16-B records (a child-scan
    group; L uniform over 1..64) read 1/0.554 of what it reports, full 1-KB groups 2x, and a lone 16-B
    record 1/4 of it."""
    cal = newest_profile("fetch_cal.json", {})
    if not cal:
        return None
    sh = cal["shapes"]
    return {"factor": sh["partial_group_Lx16B"]["correction_factor"], "shape": "partial_group_Lx16B",
            "bounds": [sh["single_record_16B"]["correction_factor"], sh["group64_dwordx4_1KB"]["correction_factor"]],
            "source": cal["source"]}


def hbm_roofline(name, stat, trees_per_launch, pmc_name=None, evaluator=None, sims=None):
    """A tree kernel against HBM. achieved = algorithmic bytes per launch of THIS run / this run's average
    launch duration from each dispatch's own events (hipExtLaunchKernelGGL; the code being benchmarked,
    ADVICE r5). The newest committed rocprof kernel trace of the same command (profiles/r*/prof_*.json,
    matched on evaluator, trees per launch and sims; it may predate this build) is kept beside it as a
    labelled secondary figure (rocprof_*), ~5 us per launch below the events. traffic = PMC reads x the
    FETCH_SIZE factor measured on the kernels' load shape + writes; traffic_over_algo divides it by the
    algorithmic bytes of the SAME PMC run (not of this run, whose step count and population differ)."""
    ms, launches, byts = stat["ms"], max(stat["launches"], 1), stat["bytes"]
    ev_us = ms * 1e3 / launches
    kname = name.split()[0]
    prof = None
    if evaluator is not None:
        for f in sorted(glob.glob(os.path.join(REPO, "profiles", "r*", "prof_*.json")), reverse=True):
            try:
                with open(f) as fh:
                    d = json.load(fh)
            except (OSError, ValueError):  # not a kernel-trace summary of this form: skip it
                continue
            if not isinstance(d, dict) or "checks" not in d:
                continue
            if (d.get("evaluator") == evaluator and d.get("trees_per_launch") == trees_per_launch
                    and d.get("sims_per_move") == sims and any(c["kernel"] == kname for c in d["checks"].values())):
                prof = d
                prof["source"] = os.path.relpath(f, REPO)
                break
    rp_us = None
    if prof:
        rp_us = next(c["rocprof_avg_us"] for c in prof["checks"].values() if c["kernel"] == kname)
    us = ev_us
    achieved = (byts / launches / 1e9) / (us * 1e-6) if us > 0 else 0.0
    rp_achieved = (byts / launches / 1e9) / (rp_us * 1e-6) if rp_us else None
    pmc = newest_profile(pmc_name, {"trees_per_launch": trees_per_launch}) if pmc_name else None
    ff = fetch_factor()
    traffic, detail = None, None
    if pmc:
        k = ff["factor"] if ff else 1.0
        traffic = round(pmc["fetch_bytes"] * k + pmc["write_bytes"])
        pmc_algo = pmc.get("algo_bytes_per_launch_bench")
        detail = {"read_bytes_fetch_size": round(pmc["fetch_bytes"]), "write_bytes": round(pmc["write_bytes"]),
                  "read_correction": ff, "traffic_bounds": ([round(pmc["fetch_bytes"] * b + pmc["write_bytes"])
                                                             for b in ff["bounds"]] if ff else None),
                  "algo_bytes_per_launch_pmc_run": pmc_algo,
                  "traffic_over_algo": round(traffic / pmc_algo, 3) if pmc_algo else None,
                  "writes_over_traffic": round(pmc["write_bytes"] / traffic, 3) if traffic else None,
                  "source": pmc["source"]}
    return {"kernel": name, "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 5), "traffic": traffic, "traffic_detail": detail,
            "algo_bytes_per_launch": round(byts / launches), "avg_launch_us": round(us, 2),
            "avg_launch_us_basis": "dispatch events of this run",
            "rocprof_avg_launch_us": round(rp_us, 2) if rp_us else None,
            "rocprof_achieved": round(rp_achieved, 2) if rp_achieved else None,
            "rocprof_source": ("committed kernel trace of the same command (may predate this build): " +
                               prof["source"]) if prof else None,
            "event_avg_launch_us": round(ev_us, 2), "launches": stat["launches"]}


def fused_rounds(evaluator):
    """Hash-evaluator rounds run the previous round's apply and this round's select as one k_round launch
    (uttt_round_hash_async; UTTT_FUSED_ROUNDS=0 keeps k_select and k_apply apart)."""
    return evaluator == "hash" and os.environ.get("UTTT_FUSED_ROUNDS", "1") != "0"


def tree_rooflines(stats, trees, evaluator, sims, pmc_sel, pmc_app):
    """(select roofline, backup roofline) of the tree kernels. Fused rounds: one roofline for k_round, whose
    launches carry both kernels' algorithmic bytes (the first round of a move is a plain k_select and the
    move's last staged apply a plain k_apply; their launches are included, a move's 1 of ~9)."""
    sel, app = stats["select"], stats["apply"]
    if not fused_rounds(evaluator):
        return (hbm_roofline("k_select (PUCT descent, one wave per tree)", sel, trees, pmc_sel, evaluator, sims),
                hbm_roofline("k_apply (expand + backup, one wave per pending leaf)", app, trees, pmc_app, evaluator,
                             sims))
    merged = {"ms": sel["ms"] + app["ms"], "launches": sel["launches"] + app["launches"],
              "bytes": sel["bytes"] + app["bytes"]}
    rf = hbm_roofline("k_round (the previous round's expand + backup, then this round's PUCT descent; one wave "
                      "per tree)", merged, trees, "pmc_round_tree.json" if pmc_sel else None, evaluator, sims)
    rf["fused"] = {"select_bytes": sel["bytes"], "apply_bytes": app["bytes"], "k_select_or_round_launches":
                   sel["launches"], "k_apply_launches": app["launches"]}
    return rf, {"kernel": "k_apply", "fused_into": "k_round", "algo_bytes_per_round": round(app["bytes"] / max(
        sel["launches"], 1)), "note": "hash-evaluator rounds apply inside k_round (roofline_select); "
                                      "UTTT_FUSED_ROUNDS=0 measures k_apply on its own"}


def main():
    args = parse()
    if args.cpu_baseline_child:
        cpu_baseline_child(args.cpu_baseline_child, args.cpu_seconds)
        return
    import torch
    import torch.distributed as dist

    sys.path[:0] = [REPO, PKG]
    from uttt_amd.model import calibrated_network, random_network

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = 0 if args.rehearse_shared_gpu else int(os.environ.get("LOCAL_RANK", 0))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        if args.rehearse_shared_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=dev)
    torch.backends.cuda.matmul.allow_tf32 = False
    torch.backends.cudnn.allow_tf32 = False

    G, S, B = args.games, args.sims, args.batch
    net0 = random_network(0, dev) if args.net == "seed0" else calibrated_network(NETCAL, dev)
    # the measurement: K steps with no per-dispatch events in the timed region; then a separate instrumented
    # pass (every kernel timed by its own dispatch's events, the network's forwards by events) whose statistics
    # give the rooflines and breakdowns (UTTT_BENCH_ONE_PASS=1: one instrumented pass gives both, as in round 4)
    one_pass = os.environ.get("UTTT_BENCH_ONE_PASS", "0") == "1"
    r_val = run_config(net0, local, rank, world, G, S, B, args.lanes, args.cache_log2, args.age, args.warmup,
                       args.steps, args.evaluator, args.cache_clear_every, instrument=one_pass)
    inst_steps = args.steps if one_pass else min(args.steps, 10)
    r = r_val if one_pass else run_config(net0, local, rank, world, G, S, B, args.lanes, args.cache_log2, args.age,
                                          min(args.warmup, 2), inst_steps, args.evaluator, args.cache_clear_every,
                                          instrument=True)

    tot = torch.tensor([float(r_val["sims"]), r_val["elapsed"]], dtype=torch.float64,
                       device="cpu" if args.rehearse_shared_gpu else dev)
    if world > 1:
        s = tot[:1].clone()
        m = tot[1:].clone()
        dist.all_reduce(s, op=dist.ReduceOp.SUM)
        dist.all_reduce(m, op=dist.ReduceOp.MAX)
        tot = torch.cat([s, m])
    total_sims, max_elapsed = float(tot[0].item()), float(tot[1].item())

    variants = None
    if world == 1 and not args.no_variants and args.evaluator.startswith("fused"):
        variants = {}
        for key, kw in (("calibrated_net", dict(net=calibrated_network(NETCAL, dev))),
                        ("cache_off", dict(cache_log2=0)),
                        ("c3_4096x400", dict(sims=400, age=30, warmup=2, steps=4)),
                        # BASELINE configs[1]: 1,024 games x 50 sims, MCTS_BATCH_SIZE 1024 (one flush per move):
                        # each move is one network call on 1,024 boards. Measured with the evaluation cache
                        # OFF: with B >= S every tree flushes one leaf per move and the one-hot scores make
                        # every game play the same line, so a cache would answer every leaf and the line
                        # would time no network at all (that degenerate form is kept beside it, labelled)
                        ("c2_1024x50_b1024", dict(games=1024, batch=1024, age=100, cache_log2=0)),
                        ("c2_1024x50_b1024_cache_on_degenerate", dict(games=1024, batch=1024, age=100)),
                        # SURVEY §8(d) kernel microbench: the search kernels alone (hash evaluator, no network),
                        # one lane: with no network to overlap, one launch per round over every tree is the
                        # fastest shape (1 / 2 / 4 lanes: 170.6M / 141M / 82M sims/s, profiles/r3/ab/hashlanes.log)
                        # 60 timed moves (as the standalone tree-only runs): 10 are a 3 ms window, where the
                        # window's own start and end set a tenth of the rate
                        ("tree_only_4096x50", dict(evaluator="hash", age=100, lanes=1, steps=60)),
                        # SURVEY §8(f) rank 1's optional fast evaluator: the tower conv with one f16 product per
                        # point (uttt_nn_conv3x3_wino3h_f16, ~1e-3 relative): not the reference's numerics, so a
                        # variant line beside the f32-level headline, never the headline
                        ("f16_mode", dict(evaluator="fused_f16")),
                        ("tree_only_4096x400", dict(evaluator="hash", sims=400, age=30, warmup=2, steps=4, lanes=1))):
            cfg = dict(net=net0, games=G, sims=S, batch=B, lanes=args.lanes, cache_log2=args.cache_log2,
                       age=args.age, warmup=3, steps=10, evaluator=args.evaluator)
            cfg.update(kw)
            rv = run_config(cfg["net"], local, 0, 1, cfg["games"], cfg["sims"], cfg["batch"], cfg["lanes"],
                            cfg["cache_log2"], cfg["age"], cfg["warmup"], cfg["steps"], cfg["evaluator"])
            sv = summarize(rv, cfg["steps"])
            if cfg["evaluator"] == "hash" and not one_pass:
                # the search kernels' own rate without the per-dispatch events (a quarter of it at 4,096 x 50);
                # the rooflines below come from the instrumented pass rv
                rv_val = run_config(cfg["net"], local, 0, 1, cfg["games"], cfg["sims"], cfg["batch"], cfg["lanes"],
                                    cfg["cache_log2"], cfg["age"], cfg["warmup"], cfg["steps"], cfg["evaluator"],
                                    instrument=False)
                sv_inst = summarize(rv, cfg["steps"])
                sv = summarize(rv_val, cfg["steps"])
                sv["instrumented_pass"] = {k: sv_inst[k] for k in ("value", "ms_per_step")}
            sv["config"] = {k: cfg[k] for k in ("games", "sims", "batch", "lanes", "cache_log2", "age", "steps",
                                                "evaluator")}
            sv["net"] = "calibrated (tests/golden/netcal.npz)" if key == "calibrated_net" else args.net
            # every line says whether its timed steps ran the network at all
            sv["evaluates_network"] = cfg["evaluator"] != "hash" and sv["rows_per_step"] > 0
            if key.endswith("_degenerate"):
                sv["degenerate"] = True
                sv["note"] = ("configs[1] with the evaluation cache on: B >= S gives one flush per tree per move and "
                              "one-hot scores, every game plays the same line and the cache answers every leaf, so "
                              "this line times the search kernels only (rows_per_step 0); variants.c2_1024x50_b1024 "
                              "(cache off) is the configs[1] measurement")
            if cfg["evaluator"] == "hash":
                sv["net"] = None
                sv["roofline_select"], sv["roofline_backup"] = tree_rooflines(
                    rv["stats"], rv["trees_per_launch"], "hash", cfg["sims"],
                    "pmc_select_tree.json" if cfg["sims"] == S else None,
                    "pmc_apply_tree.json" if cfg["sims"] == S else None)
                sv["breakdown_ms"] = {k: round(rv["stats"][k]["ms"], 2) for k in ("select", "apply", "scan", "move_end")}
                sv["breakdown_ms"]["evaluator"] = round(rv["nn_ms"], 2)
                sv["breakdown_ms"]["wall"] = round(rv["elapsed"] * 1e3, 2)
                sv["note"] = ("hash evaluator in place of the network: the search kernels' own rate, to set beside "
                              "cpu_baselines.b_tree_all_cores (the reference's C++ search with the same evaluator)")
            elif cfg["evaluator"] == "fused_f16":
                sv["precision"] = "f16: one f16 MFMA product per Winograd point (not f32-level; DESIGN.md §5)"
            else:
                cr = conv_roofline(rv, cfg["steps"]) or {}
                sv["conv_roofline_frac"] = cr.get("frac")
                sv["conv_chip_frac"] = cr.get("chip_frac")
            variants[key] = sv

    iso = None
    if world == 1 and not args.no_isolated and r["conv"] == "wino3h" and r["tower"]:
        nb = round(sum(n for n, _ in r["tower"]) / len(r["tower"]))
        iso = isolated_conv(net0, [nb, 16384])
        # the optional dataflow tower alone (the two-lane headline keeps the per-conv launches: DESIGN §5)
        iso["tower_dataflow"] = isolated_tower(net0, [nb, 16384])

    if rank == 0:
        value = total_sims / max_elapsed
        st = r["stats"]
        flops_direct = NN_FLOP_PER_STATE * r["rows"]
        nn_direct_tflops = flops_direct / (r["nn_ms"] / 1e3) / 1e12 if r["nn_ms"] > 0 else 0.0
        conv = r["conv"]
        exec_tower = (CONV_EXEC_FLOP[conv] * 32 * r["rows"] / (r["nn_ms"] / 1e3) / 1e12) if conv and r["nn_ms"] else None
        sel = st["select"]
        sel_launches = max(sel["launches"], 1)
        lev_trees = max(st["select_trees"]["bytes"], 1)
        max_lev = st["select_max_levels_sum"]["bytes"] / sel_launches
        max_trips = st["select_max_trips_sum"]["bytes"] / sel_launches
        sel_us = sel["ms"] * 1e3 / sel_launches
        chase_lat = chase_latency(newest_profile("chase.json", {}))
        tree = args.evaluator == "hash"
        pmc_sel = "pmc_select_tree.json" if tree else "pmc_select.json"
        pmc_app = "pmc_apply_tree.json" if tree else "pmc_apply.json"
        tree_rf = tree_rooflines(st, r["trees_per_launch"], args.evaluator, S, pmc_sel, pmc_app)
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
            "dtype": {"fused": "f32 activations and accumulation; tower point GEMMs as 3-term split-f16 products "
                               "on the f16 MFMA (f32-level accuracy: within 1e-5 of the reference's fp32 network)",
                      "fused_f16": "f32 activations and accumulation; tower point GEMMs as ONE f16 product (the "
                                   "optional f16 mode: ~1e-2 on the network's outputs, not the reference's numerics)",
                      "nn": "f32", "hash": "f32 (hash evaluator)"}[args.evaluator],
            "data": "synthetic: self-play from the initial position, games refilled as they end; DualNetwork "
                    + ("random init torch.manual_seed(0) (the reference's initial best.pth)" if args.net == "seed0"
                       else "with calibrated BatchNorm statistics (tests/golden/netcal.npz)") + "; no checkpoint",
            "config": {
                "workload": f"{G} concurrent self-play games per GPU x {S} sims/move, MCTS_BATCH_SIZE {B}, "
                            f"tau 1.0, continuous self-play (finished games refilled; population aged "
                            f"{args.age} moves before warmup); one step = one move of every game",
                "games_per_gpu": G, "sims_per_move": S, "mcts_batch_size": B, "aged_moves": args.age,
                "eval_cache_log2": args.cache_log2, "eval_cache_clear_every": args.cache_clear_every,
                "lanes_per_gpu": args.lanes,
                "evaluator": {"fused": "DualNetwork 128f x16 on HIP kernels: stem from bitboards, residual tower as "
                                       "fused Winograd F(3x3,3x3) convs (csrc/wino3h_conv.hip, split-f16 MFMA, f32 "
                                       "accumulation, per-board scaling), heads (csrc/nn_kernels.hip)",
                              "fused_f16": "DualNetwork 128f x16 on HIP kernels in the optional f16 mode: the "
                                           "Winograd tower conv with one f16 MFMA product per point "
                                           "(uttt_nn_conv3x3_wino3h_f16)",
                              "nn": "DualNetwork 128f x16 fp32, BN folded, PyTorch-ROCm/MIOpen",
                              "hash": "device hash evaluator (no network)"}[args.evaluator],
                "parallelism": f"games sharded over {world} GPU(s) by contiguous global-id blocks, "
                               f"no data-path collective",
            },
            "roofline": conv_roofline(r, inst_steps) if conv else tree_rf[0],
            "roofline_select": dict(tree_rf[0],
                                    latency_model={
                                        "levels_per_tree_per_launch": round(st["select_levels"]["bytes"] / lev_trees, 2),
                                        "slowest_tree_levels_per_launch": round(max_lev, 1),
                                        "us_per_level_of_slowest_tree": round(sel_us / max(max_lev, 1e-9), 3),
                                        "trips_per_tree_per_launch": round(st["select_trips"]["bytes"] / lev_trees, 2),
                                        "slowest_tree_trips_per_launch": round(max_trips, 1),
                                        "us_per_trip_of_slowest_tree": round(sel_us / max(max_trips, 1e-9), 3),
                                        "dependent_load_us": chase_lat,
                                        "predicted_launch_us": (round(max_trips * chase_lat["us"], 1)
                                                                if chase_lat else None),
                                        "note": "a launch lasts as long as its slowest tree's chain of dependent "
                                                "memory round trips (per descent the root's link and visits, one per "
                                                "64-lane child-scan group, per completion in place the cache probe, "
                                                "payload, re-check, path update and fence); predicted = that chain x "
                                                "the dependent-load latency of tools/diag/chase.hip (2,048 waves, "
                                                "random 256-B loads that miss L2)"}),
            "roofline_backup": tree_rf[1],
            "nn": {"rows_evaluated": r["rows"], "ms": round(r["nn_ms"], 2),
                   "share_of_step": round(r["nn_ms"] / 1e3 / r["elapsed"], 4),
                   "lane_sum_ms": round(r["nn_lane_sum_ms"], 2),
                   "mfma_executed_tflops": round(exec_tower, 2) if exec_tower else None,
                   "frac": round(exec_tower / CONV_PEAK[conv], 4) if exec_tower else None,
                   "peak_tflops": CONV_PEAK[conv] if conv else None,
                   "frac_basis": "residual-tower MFMA flops actually issued (Winograd, 3 f16 products) per evaluated "
                                 "row / union of NN-call time (stem and heads included), over the dtype's dense peak",
                   "direct_equiv_tflops": round(nn_direct_tflops, 2),
                   "direct_equiv_basis": "2 x MACs of dual_network.py per evaluated row (what the reference's "
                                         "network costs as direct convs)"},
            "breakdown_ms": {"select": round(sel["ms"], 2), "apply": round(st["apply"]["ms"], 2),
                             "scan": round(st["scan"]["ms"], 2), "move_end": round(st["move_end"]["ms"], 2),
                             "nn": round(r["nn_ms"], 2), "wall": round(r["elapsed"] * 1e3, 2)},
            "rounds_per_step": round(r["rounds"] / inst_steps, 2),
            "instrumented_pass": {"steps": inst_steps, "value": round(r["sims"] / r["elapsed"], 1),
                                  "ms_per_step": round(r["elapsed"] / inst_steps * 1e3, 3),
                                  "note": "value and ms_per_step above: the timed steps with no events in them; the "
                                          "rooflines, nn, breakdown_ms and eval_cache: this separate pass, every "
                                          "kernel timed by its own dispatch's events" if not one_pass else
                                          "one pass: value measured with the events on"},
            "games_finished_in_timed_steps": int(r["finished"]),
            "eval_cache": (dict(r["cache"], hit_rate=round(r["cache"]["hits"] / max(r["cache"]["hits"] +
                                                                                     r["cache"]["misses"], 1), 4),
                                log2_capacity=args.cache_log2) if r["cache"] else None),
            "variants": variants,
        }
        if iso and out.get("roofline") and out["roofline"].get("bound") == "mfma":
            out["roofline"]["isolated"] = iso
        if args.rehearse_shared_gpu:
            out["config"]["rehearsal"] = f"{world} ranks sharing one GPU over gloo (not a scaling measurement)"
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = run_cpu_baseline("cpu-nn", args.cpu_seconds)
            out["cpu_baselines"] = {"b_tree_all_cores": run_cpu_baseline("tree", 10.0),
                                    "b_e2e_nn_on_device": run_cpu_baseline("device-nn", 10.0)}
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
