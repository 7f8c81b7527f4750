"""Launched by tests/test_dropins_gpu.py under torch.distributed.run with ONE rank and the nccl
(RCCL) backend (not a test module): the RCCL branches of the data path and of data-parallel
training on the real device. self_play_sharded's gather_records (device-tensor all_gather of the
byte counts), broadcast_int, and DDP steps whose gradient all-reduce runs over RCCL. Two RCCL ranks
cannot share one device, so this is the most of the 8-GPU path one GPU can run. Prints RCCL-OK."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

if __name__ == "__main__":
    torch.cuda.set_device(0)
    dist.init_process_group("nccl")
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    from oracle.hashnp import make_hash_model
    from uttt_amd import SelfPlay
    from uttt_amd.distributed import broadcast_int, self_play_sharded
    from uttt_amd.model import random_network
    from uttt_amd.train import train_step

    n_games, seed = 6, 77
    out = self_play_sharded(make_hash_model(), n_games, 3, seed, evaluate_count=20, batch_size=4)
    sp = SelfPlay(3, 20, 4, 1.0)
    sp.run(0, n_games, seed)
    ref = sp.records()
    assert len(out) == n_games, len(out)
    for a, b in zip(sorted(out, key=lambda r: r["game"]), ref):
        assert a["game"] == b["game"]
        assert np.array_equal(np.asarray(a["actions"]), np.asarray(b["actions"]))
        assert np.array_equal(np.asarray(a["policies"]).view(np.uint64), np.asarray(b["policies"]).view(np.uint64))
        assert np.array_equal(np.asarray(a["values"]), np.asarray(b["values"]))
    assert broadcast_int(123457) == 123457

    net = random_network(0).cuda()
    ddp = torch.nn.parallel.DistributedDataParallel(net, device_ids=[0], bucket_cap_mb=25)
    opt = torch.optim.Adam(ddp.parameters(), lr=1e-3, fused=True)
    g = torch.Generator(device="cpu").manual_seed(0)
    x = (torch.rand(16, 3, 9, 9, generator=g) > 0.5).float().cuda()
    p = torch.softmax(torch.randn(16, 81, generator=g), 1).cuda()
    v = (torch.rand(16, 1, generator=g) * 2 - 1).cuda()
    losses = [float(train_step(ddp, opt, x, p, v)) for _ in range(3)]
    assert all(np.isfinite(losses)) and losses[-1] < losses[0], losses

    # round 5: the flat graphed data-parallel step (train.DPGraphedStep: graph(forward + backward into one
    # flat gradient buffer) -> RCCL all_reduce of it -> graph(fused Adam)) against the eager DDP step on the
    # same batch from the same weights: the same loss and the same all-reduced gradient (up to the rounding
    # of the convolution kernels MIOpen picks inside and outside a capture). Later steps are not compared
    # bit for bit: Adam's first updates are ~lr * sign(g) per element, so rounding-level gradient
    # differences flip single elements by 2 lr and the trajectories part (a CPU run of the same phases,
    # tests/test_distributed.py, matches the eager step exactly).
    from uttt_amd.train import DPGraphedStep
    X = (torch.rand(64, 3, 9, 9, generator=g) > 0.5).float().cuda()
    P = torch.softmax(torch.randn(64, 81, generator=g), 1).cuda()
    V = (torch.rand(64, 1, generator=g) * 2 - 1).cuda()
    i0 = torch.randperm(64, generator=g)[:16].cuda()
    net_a = random_network(0).cuda().train()
    opt_a = torch.optim.Adam(net_a.parameters(), lr=torch.tensor(1e-3, device="cuda"), capturable=True, fused=True)
    step = DPGraphedStep(net_a, opt_a, X, P, V, 16, 1.0, graph=True, tune=False)
    net_b = random_network(0).cuda().train()
    ddp_b = torch.nn.parallel.DistributedDataParallel(net_b, device_ids=[0], bucket_cap_mb=25)
    opt_b = torch.optim.Adam(ddp_b.parameters(), lr=1e-3, fused=True)
    step.step(i0, 1.0)
    la = float(step.loss_sum)
    lb = float(train_step(ddp_b, opt_b, X[i0], P[i0], V[i0]))
    assert abs(la - lb) <= 1e-5 * abs(lb), (la, lb)
    for (k, qa), qb in zip(net_a.named_parameters(), net_b.parameters()):
        scale = max(qb.grad.abs().max().item(), 1e-12)
        err = (qa.grad - qb.grad).abs().max().item()
        assert err <= 1e-3 * scale, (k, err, scale)

    # Graph replays against the same phases run eagerly, over 12 steps: a new random
    # slice every step (the index copy into the graph's input), the learning-rate tensor changed at step 6
    # (read by the replay), Adam's step counter and bias correction advancing inside graph B. A replay bug (a
    # stale flat gradient, a stale lr or step, the warm-up undo leaving state behind) moves the graph's weights
    # by O(update) from the eager ones. The comparison is made well-conditioned on purpose: BatchNorm in eval
    # mode (the calibrated running statistics; in train mode a channel with near-zero batch variance over 16
    # samples multiplies rounding by up to 1/sqrt(eps) = 316, and the graph and eager runs, whose MIOpen
    # kernels differ in rounding, part by 10% of an update within 4 steps), and Adam with eps = 1e3 and lr 10,
    # so each update is ~1e-2 m_hat, linear in the gradient (no lr * sign(g) amplification). Bounds: the
    # distance at 1% of how far the weights moved, each step's update difference at 2% of that update; a
    # stale lr (x3.3 at step 6), step counter or gradient breaks the second by an O(1) factor. (Train mode,
    # the per-rank BatchNorm path, is pinned at step 1 above and in tests/dp_flat_two_ranks_main.py.)
    from uttt_amd.model import calibrated_network
    netcal = os.path.join(REPO, "tests", "golden", "netcal.npz")
    nets, steps, lrs = [], [], []
    for graph in (True, False):
        net = calibrated_network(netcal, "cuda").eval()
        lr_t = torch.tensor(10.0, device="cuda")
        opt = torch.optim.Adam(net.parameters(), lr=lr_t, eps=1e3, capturable=True, fused=True)
        nets.append(net)
        lrs.append(lr_t)
        steps.append(DPGraphedStep(net, opt, X, P, V, 16, 1.0, graph=graph, tune=False))
    assert steps[0].graph and not steps[1].graph
    w0 = [q.detach().clone() for q in nets[1].parameters()]
    prev = [[q.detach().clone() for q in n.parameters()] for n in nets]
    gg = torch.Generator(device="cpu").manual_seed(11)
    hist = []
    for t in range(12):
        if t == 6:
            for lr_t in lrs:
                lr_t.fill_(3.0)
        idx = torch.randperm(64, generator=gg)[:16].cuda()
        for st in steps:
            st.loss_sum.zero_()
            st.step(idx, 1.0)
        lg, le = float(steps[0].loss_sum), float(steps[1].loss_sum)
        assert np.isfinite(lg) and abs(lg - le) <= 1e-4 * abs(le), (t, lg, le, hist)
        moved = max((qe.detach() - q0).abs().max().item() for qe, q0 in zip(nets[1].parameters(), w0))
        diff = max((qg.detach() - qe.detach()).abs().max().item()
                   for qg, qe in zip(nets[0].parameters(), nets[1].parameters()))
        # this step's update, graph against eager
        inc = [[q.detach() - p0 for q, p0 in zip(n.parameters(), pr)] for n, pr in zip(nets, prev)]
        step_e = max(d.abs().max().item() for d in inc[1])
        step_d = max((a - b).abs().max().item() for a, b in zip(inc[0], inc[1]))
        prev = [[q.detach().clone() for q in n.parameters()] for n in nets]
        assert diff <= 1e-2 * moved and step_d <= 2e-2 * step_e, (t, diff, moved, step_d, step_e, hist)
        hist.append((round(lg, 6), round(le, 6), round(diff / moved, 5), round(step_d / step_e, 5)))
    dist.destroy_process_group()
    print("RCCL-OK", losses, "flat-graph DP", la, "eager DDP", lb, flush=True)
    print("GRAPH-VS-EAGER", hist, flush=True)
