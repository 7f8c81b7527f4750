#!/usr/bin/env python3
"""The data-parallel training step on ONE rank (torchrun --nproc-per-node 1, nccl = RCCL), the two forms
train_network can run per rank (train_network.py:41-125):

  eager DDP + SyncBatchNorm (UTTT_TRAIN_DP=ddp): ~600 kernel launches per step, DDP's bucketed all-reduce;
      SyncBatchNorm adds two collectives per BatchNorm layer (35 layers) per step on >= 2 ranks (at one
      rank torch runs plain BatchNorm, so they are priced here, not measured);
  the flat graphed step (DPGraphedStep, UTTT_TRAIN_DP=flat, the default): graph(forward + backward into a
      flat gradient buffer) -> one all_reduce of that buffer -> graph(fused Adam); per-rank BatchNorm.

Both at the per-rank batch of the 8-GPU split of the reference's global batch 128 (16) and at 128, beside
the single-process graphed step (GraphedStep) at 128. Then the DP8 projection of each form from the
measured per-rank step and a modelled all-reduce of the 19.1 MB gradient over 8 ranks.

usage: torchrun --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port P tools/bench_train_dp.py --out F
"""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

GRAD_BYTES = 4765338 * 4
# all-reduce model for 8 ranks (no 8-GPU node available to this build): ring, 2 x 7/8 x bytes per rank at an
# assumed 100 GB/s bus bandwidth per rank (xGMI: 7 links x ~153 GB/s peak, MI355X_MICROARCH.md) + 8 steps x 2 x
# 5 us latency; small collectives (SyncBatchNorm's stats all-gather / all-reduce) at 20 us each on 8 ranks
ALLREDUCE_8_MS = 2 * 7 / 8 * GRAD_BYTES / 100e9 * 1e3 + 2 * 8 * 5e-3
SMALL_COLLECTIVE_8_MS = 0.020
SYNCBN_COLLECTIVES = 2 * 35  # forward stats all-gather + backward all-reduce per BatchNorm layer


def history(n, seed=0):
    import numpy as np
    rng = np.random.RandomState(seed)
    xs = (rng.rand(n, 9, 9, 3) < 0.3).astype(np.float64)
    ps = rng.rand(n, 81)
    ps /= ps.sum(axis=1, keepdims=True)
    vs = rng.randint(-1, 2, size=n)
    return [[xs[i], ps[i], int(vs[i])] for i in range(n)]


def timeit(fn, steps, warm=5):
    import torch
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    from uttt_amd import train
    from uttt_amd.model import random_network
    torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", 0)))
    dist.init_process_group("nccl")
    dev = torch.device("cuda", torch.cuda.current_device())
    x, p, v = (torch.from_numpy(a).to(dev) for a in train.history_arrays(history(4096)))
    g = torch.Generator(device="cpu").manual_seed(0)
    res = {"metric": "train_network step time per rank (DualNetwork 128f x16 fp32, Adam)", "unit": "ms",
           "backend": dist.get_backend(), "world_size": dist.get_world_size(), "steps": args.steps, "forms": {}}
    for batch in (16, 128):
        idx = [torch.randperm(len(x), generator=g)[:batch].to(dev) for _ in range(8)]
        it = iter(range(10 ** 9))

        # eager DDP + SyncBatchNorm, fused Adam (train_network's "ddp" form)
        net = torch.nn.SyncBatchNorm.convert_sync_batchnorm(random_network(0).to(dev))
        ddp = torch.nn.parallel.DistributedDataParallel(net, device_ids=[dev.index], bucket_cap_mb=25)
        opt = torch.optim.Adam(ddp.parameters(), lr=1e-3, fused=True)

        def eager():
            i = idx[next(it) % 8]
            train.train_step(ddp, opt, x[i], p[i], v[i])
        res["forms"][f"eager_ddp_syncbn_b{batch}"] = round(timeit(eager, args.steps), 3)
        del ddp, net, opt

        # the flat graphed step (DPGraphedStep), this rank's slice = the whole batch at world 1
        net = random_network(0).to(dev).train()
        lr_t = torch.tensor(1e-3, device=dev)
        opt = torch.optim.Adam(net.parameters(), lr=lr_t, capturable=True, fused=True)
        step = train.DPGraphedStep(net, opt, x, p, v, batch, 1.0, graph=True, tune=True)

        def flat():
            step.step(idx[next(it) % 8], 1.0)
        res["forms"][f"flat_graph_b{batch}"] = round(timeit(flat, args.steps), 3)
        # the same without the collective: the graphs alone
        ar = dist.all_reduce

        def no_ar(*a, **k):
            return None
        dist.all_reduce = no_ar
        res["forms"][f"flat_graph_no_allreduce_b{batch}"] = round(timeit(flat, args.steps), 3)
        dist.all_reduce = ar
        del step, net, opt

    # single process, the whole step in one graph (GraphedStep, train_network's one-GPU form) at 128
    net = random_network(0).to(dev).train()
    lr_t = torch.tensor(1e-3, device=dev)
    opt = torch.optim.Adam(net.parameters(), lr=lr_t, capturable=True, fused=True)
    gs = train.GraphedStep(net, opt, x, p, v, 128, tune=True)
    idx = [torch.randperm(len(x), generator=g)[:128].to(dev) for _ in range(8)]
    it = iter(range(10 ** 9))
    res["forms"]["single_gpu_graph_b128"] = round(timeit(lambda: gs.step(idx[next(it) % 8]), args.steps), 3)
    # the flat gradient all-reduce at this world size (one rank: RCCL's own path, no peer)
    buf = torch.zeros(GRAD_BYTES // 4, device=dev)
    res["allreduce_19MB_ms_this_world"] = round(timeit(lambda: dist.all_reduce(buf), 20), 4)

    f = res["forms"]
    one = f["single_gpu_graph_b128"]
    proj = {
        "allreduce_19MB_8ranks_ms_modelled": round(ALLREDUCE_8_MS, 3),
        "syncbn_collectives_ms_modelled": round(SYNCBN_COLLECTIVES * SMALL_COLLECTIVE_8_MS, 3),
        "model_basis": "ring all-reduce 2 x 7/8 x 19.1 MB per rank at 100 GB/s + 16 x 5 us latency; SyncBatchNorm: "
                       f"{SYNCBN_COLLECTIVES} small collectives per step at {SMALL_COLLECTIVE_8_MS * 1e3:.0f} us each on 8 ranks "
                       "(not measured: no multi-GPU node)",
        "single_gpu_b128": {"step_ms": one, "samples_per_s": round(128 / one * 1e3, 1)},
    }
    fl = f["flat_graph_no_allreduce_b16"] + ALLREDUCE_8_MS
    ed = f["eager_ddp_syncbn_b16"] + SYNCBN_COLLECTIVES * SMALL_COLLECTIVE_8_MS  # DDP overlaps its all-reduce
    proj["dp8_flat_graph"] = {"step_ms": round(fl, 3), "samples_per_s": round(128 / fl * 1e3, 1),
                              "vs_single_gpu": round(one / fl, 3),
                              "numerics": "per-rank BatchNorm statistics (16 samples per rank)"}
    proj["dp8_eager_ddp_syncbn"] = {"step_ms": round(ed, 3), "samples_per_s": round(128 / ed * 1e3, 1),
                                    "vs_single_gpu": round(one / ed, 3),
                                    "numerics": "the reference's batch-128 BatchNorm statistics (SyncBatchNorm)"}
    res["dp8_projection"] = proj
    if args.out:
        with open(args.out, "w") as fh:
            json.dump(res, fh, indent=1)
    print(json.dumps(res), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
