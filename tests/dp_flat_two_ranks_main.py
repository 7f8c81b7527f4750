"""Launched by tests/test_dropins_gpu.py under torch.distributed.run with 2 ranks sharing the box's GPU
(gloo, as uttt_amd.distributed.init_from_env picks when ranks outnumber GPUs; not a test module):
train_network's opt-in GPU data-parallel form (UTTT_TRAIN_DP=flat: train.DPGraphedStep, two captured
graphs around one flat gradient all-reduce per step) on a small history with an uneven last batch. Each rank
saves its weights and losses into argv[1]; the test checks that the replicas are identical."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

if __name__ == "__main__":
    from uttt_amd import train
    from uttt_amd.distributed import init_from_env
    from uttt_amd.model import random_network
    rank, world, local = init_from_env()
    rng = np.random.RandomState(5)
    n = 150  # batches of 32: four full ones (16 + 16 per rank) and a last one of 22 (11 + 11)
    xs = (rng.rand(n, 9, 9, 3) < 0.3).astype(np.float64)
    ps = rng.rand(n, 81)
    ps /= ps.sum(axis=1, keepdims=True)
    hist = [[xs[i], ps[i], int(v)] for i, v in enumerate(rng.randint(-1, 2, size=n))]
    model = random_network(1 + rank)  # different start weights: rank 0's are broadcast
    losses = train.train_network(model, hist, epochs=3, batch_size=32, device=torch.device("cuda", local), log=None,
                                 dp="flat")
    torch.save({"sd": {k: t.detach().cpu() for k, t in model.state_dict().items()}, "losses": losses},
               os.path.join(sys.argv[1], f"m{rank}.pt"))

    # The graphed step at world size 2 against a single-process emulation of the same job:
    # per step, each rank's slice forward, share x its loss backward, the gradients summed, one Adam step.
    # (a) Train mode, one step: BatchNorm over each rank's 16 samples (the per-rank statistics of the flat
    # form); the all-reduced flat gradient equals the emulation's summed gradient and the losses agree.
    # (b) Ten steps, BatchNorm in eval mode (train mode over 16 samples amplifies rounding by up to 316 through
    # near-zero-variance channels, tests/rccl_one_rank_main.py), Adam with eps = 1e3 and lr 10 (updates ~1e-2
    # m_hat, linear in the gradient): weights within 1% of their motion, each update within 2%.
    from uttt_amd.model import calibrated_network
    from uttt_amd.train import DPGraphedStep, all_reduce_sum, local_slice, policy_loss_fn
    dev = torch.device("cuda", local)
    netcal = os.path.join(REPO, "tests", "golden", "netcal.npz")
    g = torch.Generator(device="cpu").manual_seed(3)
    X = (torch.rand(64, 3, 9, 9, generator=g) > 0.5).float().to(dev)
    P = torch.softmax(torch.randn(64, 81, generator=g), 1).to(dev)
    V = (torch.rand(64, 1, generator=g) * 2 - 1).to(dev)
    full = local_slice(torch.arange(32), rank, world)

    def emulate(ref, idx):
        le = 0.0
        for r in range(world):
            sl = local_slice(idx, r, world).to(dev)
            pp, pv = ref(X[sl])
            loss = policy_loss_fn(pp, P[sl]) + torch.nn.functional.mse_loss(pv, V[sl])
            (loss * (len(sl) / 32)).backward()
            le += float(loss) * len(sl) / 32
        return le

    for mode in ("train", "eval"):
        net = calibrated_network(netcal, dev)
        ref = calibrated_network(netcal, dev)
        net.train(mode == "train")
        ref.train(mode == "train")
        opt = torch.optim.Adam(net.parameters(), lr=torch.tensor(10.0, device=dev), eps=1e3, capturable=True,
                               fused=True)
        step = DPGraphedStep(net, opt, X, P, V, len(full), len(full) / 32, graph=True, tune=False)
        assert step.graph
        opt_r = torch.optim.Adam(ref.parameters(), lr=10.0, eps=1e3)
        w0 = [q.detach().clone() for q in ref.parameters()]
        prev = [[q.detach().clone() for q in m.parameters()] for m in (net, ref)]
        hist = []
        for t in range(1 if mode == "train" else 10):
            idx = torch.randperm(64, generator=g)[:32]
            mine = local_slice(idx, rank, world).to(dev)
            step.loss_sum.zero_()
            step.step(mine, len(mine) / 32)
            lt = step.loss_sum.clone()
            all_reduce_sum(lt)
            opt_r.zero_grad()
            le = emulate(ref, idx)
            lg = float(lt)
            assert abs(lg - le) <= 1e-4 * abs(le), (mode, t, lg, le, hist)
            if mode == "train":  # the all-reduced gradient (the flat buffer after the step) against the summed one
                gref = torch.cat([q.grad.reshape(-1) for q in ref.parameters() if q.requires_grad])
                scale = max(gref.abs().max().item(), 1e-12)
                err = (step.flat - gref).abs().max().item()
                # train-mode BatchNorm over 16-sample rank batches amplifies the GPU's reduction-order rounding
                # (max error / max gradient measured 0.8e-3 .. 1.6e-3 across boxes); a replay or all-reduce
                # fault (a stale flat buffer, one rank's half missing) is an O(1) relative error
                assert err <= 1e-2 * scale, (err, scale)
                hist.append((round(lg, 6), round(le, 6), round(err / scale, 7)))
                continue
            opt_r.step()
            moved = max((qe.detach() - q0).abs().max().item() for qe, q0 in zip(ref.parameters(), w0))
            diff = max((qg.detach() - qe.detach()).abs().max().item()
                       for qg, qe in zip(net.parameters(), ref.parameters()))
            inc = [[q.detach() - p0 for q, p0 in zip(m.parameters(), pr)] for m, pr in zip((net, ref), prev)]
            step_e = max(d.abs().max().item() for d in inc[1])
            step_d = max((a - b).abs().max().item() for a, b in zip(inc[0], inc[1]))
            prev = [[q.detach().clone() for q in m.parameters()] for m in (net, ref)]
            assert diff <= 1e-2 * moved and step_d <= 2e-2 * step_e, (t, diff, moved, step_d, step_e, hist)
            hist.append((round(lg, 6), round(le, 6), round(diff / moved, 5), round(step_d / step_e, 5)))
        if rank == 0:
            print("DP-GRAPH-VS-EMULATION", mode, hist, flush=True)
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
    print("DP-FLAT-OK", rank, losses, flush=True)
