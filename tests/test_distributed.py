"""Multi-process (gloo, world_size 2, CPU) tests of the sharded self-play plumbing:
game-id sharding covers [0, n) exactly once and the record gather reassembles
rank-local games into one id-ordered set, identical to a single-rank run."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from uttt_amd.distributed import PLY_DTYPE, gather_records, pack_records, shard, unpack_records


def _fake_records(ids):
    recs = []
    for g in ids:
        rng = np.random.RandomState(g)
        n = 5 + g % 7
        st = np.zeros(n, PLY_DTYPE.fields["state"][0])
        st["own"][:, 0] = rng.randint(0, 2**27, size=n)
        st["active"] = -1
        recs.append({"game": g, "states": st, "policies": rng.rand(n, 81), "actions": rng.randint(0, 81, n),
                     "values": rng.randint(-1, 2, n)})
    return recs


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, n_games, out_dir):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b, e = shard(n_games, rank, world)
    merged = gather_records(_fake_records(range(b, e)))
    if rank == 0:
        np.save(os.path.join(out_dir, "merged.npy"), pack_records(merged))
    dist.barrier()
    dist.destroy_process_group()


def test_shard_partitions_ids():
    for n in (0, 1, 7, 500, 32768):
        for w in (1, 2, 3, 8):
            ranges = [shard(n, r, w) for r in range(w)]
            assert ranges[0][0] == 0 and ranges[-1][1] == n
            assert all(ranges[i][1] == ranges[i + 1][0] for i in range(w - 1))
            sizes = [e - b for b, e in ranges]
            assert max(sizes) - min(sizes) <= 1


def test_pack_roundtrip():
    recs = _fake_records([3, 1, 2])
    back = unpack_records(pack_records(recs))
    assert [r["game"] for r in back] == [1, 2, 3]
    for r in back:
        src = next(x for x in recs if x["game"] == r["game"])
        assert np.array_equal(r["policies"], src["policies"]) and np.array_equal(r["actions"], src["actions"])


def test_gloo_gather_two_ranks(tmp_path):
    n_games = 23
    mp.spawn(_worker, args=(2, _free_port(), n_games, str(tmp_path)), nprocs=2, join=True)
    merged = np.load(tmp_path / "merged.npy")
    single = pack_records(_fake_records(range(n_games)))
    assert np.array_equal(merged, single)


# ------------------------------------------------- data-parallel train_network --
def _history(n, seed):
    rng = np.random.RandomState(seed)
    xs = (rng.rand(n, 9, 9, 3) < 0.3).astype(np.float64)
    ps = rng.rand(n, 81)
    ps /= ps.sum(axis=1, keepdims=True)
    vs = rng.randint(-1, 2, size=n)
    return [[xs[i], ps[i].tolist(), int(vs[i])] for i in range(n)]


def _grad_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    from uttt_amd import train
    from uttt_amd.model import random_network
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    model = random_network(0).eval()  # BatchNorm on running statistics: per-sample losses
    net = train.prepare(model, torch.device("cpu"), sync_bn=False)
    x, p, v = (torch.from_numpy(a) for a in train.history_arrays(_history(8, 3)))
    li = train.local_slice(torch.arange(8), rank, world)
    pp, pv = net(x[li])
    loss = train.policy_loss_fn(pp, p[li]) + torch.nn.functional.mse_loss(pv, v[li])
    loss.backward()
    if rank == 0:
        torch.save({k: q.grad.clone() for k, q in model.named_parameters()}, os.path.join(out_dir, "g.pt"))
    # a short train-mode run: replicas stay identical
    model2 = random_network(1)
    losses = train.train_network(model2, _history(24, 5), epochs=2, batch_size=8, device=torch.device("cpu"),
                                 log=None, sync_bn=False)
    params = {k: q.detach().clone() for k, q in model2.named_parameters()}  # BN running stats stay per
    torch.save({"sd": params, "losses": losses}, os.path.join(out_dir, f"m{rank}.pt"))  # rank without SyncBN
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_step_equals_single_process(tmp_path):
    """DDP over 2 gloo ranks, each half of a global batch: the averaged gradients equal the
    single-process gradients of the whole batch (train_network.py:97-113 loss); a short
    train-mode run keeps both replicas' parameters identical."""
    import torch
    from uttt_amd import train
    from uttt_amd.model import random_network
    mp.spawn(_grad_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    model = random_network(0).eval()
    x, p, v = (torch.from_numpy(a) for a in train.history_arrays(_history(8, 3)))
    pp, pv = model(x)
    loss = train.policy_loss_fn(pp, p) + torch.nn.functional.mse_loss(pv, v)
    loss.backward()
    g = torch.load(os.path.join(tmp_path, "g.pt"), weights_only=True)
    for k, q in model.named_parameters():
        scale = max(q.grad.abs().max().item(), 1e-12)
        assert (g[k] - q.grad).abs().max().item() <= 1e-4 * scale, k  # f32, different summation order
    m0 = torch.load(os.path.join(tmp_path, "m0.pt"), weights_only=True)
    m1 = torch.load(os.path.join(tmp_path, "m1.pt"), weights_only=True)
    for k in m0["sd"]:
        assert torch.equal(m0["sd"][k], m1["sd"][k]), k
    assert m0["losses"] == m1["losses"] and all(np.isfinite(m0["losses"]))


# ------------------------------- data-parallel step around one flat gradient all-reduce --
def _flat_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    from uttt_amd import train
    from uttt_amd.model import random_network
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(2)
    # one step of DPGraphedStep's phases (eager form: graph A's body, the flat all-reduce, Adam) on an
    # uneven split of a global batch of 7 (4 + 3 samples): BatchNorm on running statistics, so the
    # per-sample losses and the reduced gradient equal the single-process ones up to summation order
    model = random_network(0).eval()
    x, p, v = (torch.from_numpy(a) for a in train.history_arrays(_history(7, 3)))
    li = train.local_slice(torch.arange(7), rank, world)
    opt = torch.optim.Adam(model.parameters(), lr=1e-3)
    step = train.DPGraphedStep(model, opt, x, p, v, len(li), len(li) / 7, graph=False)
    step.step(li, len(li) / 7)
    if rank == 0:
        torch.save({k: q.grad.clone() for k, q in model.named_parameters()}, os.path.join(out_dir, "g.pt"))
    # train mode (BatchNorm on each rank's own slice): the all-reduced gradient of one flat step
    mt = random_network(2).train()
    opt_t = torch.optim.Adam(mt.parameters(), lr=1e-3)
    step_t = train.DPGraphedStep(mt, opt_t, x, p, v, len(li), len(li) / 7, graph=False)
    step_t.step(li, len(li) / 7)
    tl = step_t.loss_sum.clone()
    dist.all_reduce(tl)  # the ranks' shares -> the global mean loss
    if rank == 0:
        torch.save({"g": {k: q.grad.clone() for k, q in mt.named_parameters()}, "loss": float(tl)},
                   os.path.join(out_dir, "gt.pt"))
    # sync_buffers pools the ranks' running statistics: mean of means, E[var + mean^2] - mean^2
    bn = mt.bn_input
    with torch.no_grad():
        bn.running_mean.fill_(1.0 + 2.0 * rank)
        bn.running_var.fill_(0.5 + rank)
    step_t.sync_buffers()
    if rank == 0:  # ranks: means 1, 3 (mean 2); variances 0.5, 1.5 -> 1.0 + spread 1.0 = 2.0
        assert torch.allclose(bn.running_mean, torch.full_like(bn.running_mean, 2.0)), bn.running_mean
        assert torch.allclose(bn.running_var, torch.full_like(bn.running_var, 2.0)), bn.running_var
    # train mode through train_network(dp="flat"): 21 plies in batches of 8 (the last one 5 = 3 + 2):
    # parameters and the rank-averaged BatchNorm running statistics identical on both ranks
    model2 = random_network(1)
    losses = train.train_network(model2, _history(21, 5), epochs=2, batch_size=8, device=torch.device("cpu"),
                                 log=None, dp="flat")
    sd = {k: t.detach().clone() for k, t in model2.state_dict().items()}
    torch.save({"sd": sd, "losses": losses}, os.path.join(out_dir, f"m{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


def test_flat_data_parallel_step_equals_single_process(tmp_path):
    """train.DPGraphedStep (round 5: the GPU data-parallel path's step as two graphs around one flat
    gradient all-reduce), its phases run eagerly over 2 gloo ranks with an uneven split: the all-reduced
    gradient equals the single-process gradient of the whole batch; train_network(dp="flat") keeps the
    replicas' parameters and averaged BatchNorm statistics identical."""
    import torch
    from uttt_amd import train
    from uttt_amd.model import random_network
    mp.spawn(_flat_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    # the seed-0 network is saturated (near one-hot softmax), so f32 gradients carry ~2e-4 relative error
    # against f64: the bound is the single-process f32 gradient's own distance from f64, doubled
    x, p, v = (torch.from_numpy(a) for a in train.history_arrays(_history(7, 3)))
    ref = {}
    for dt in (torch.float32, torch.float64):
        model = random_network(0).eval().to(dt)
        pp, pv = model(x.to(dt))
        loss = train.policy_loss_fn(pp, p.to(dt)) + torch.nn.functional.mse_loss(pv, v.to(dt))
        loss.backward()
        ref[dt] = {k: q.grad.double() for k, q in model.named_parameters()}
    g = torch.load(os.path.join(tmp_path, "g.pt"), weights_only=True)
    for k, g64 in ref[torch.float64].items():
        scale = max(g64.abs().max().item(), 1e-12)
        own = (ref[torch.float32][k] - g64).abs().max().item()
        assert (g[k].double() - g64).abs().max().item() <= 2 * own + 1e-6 * scale, k
    # train mode: the flat step's gradient is the sum over the ranks' slices of share x the gradient of
    # that slice's loss with BatchNorm over the slice alone (per-rank statistics; train.DPGraphedStep)
    # BatchNorm over 3-4 samples amplifies rounding: the single-process f32 gradient of the input conv
    # lands 2e-4 to 2.3e-2 (of 5.4) from f64 depending on the host thread count alone, so the bound is
    # 1e-2 of the gradient's scale, below any one rank's missing contribution (rank 1's part is 8% of it)
    ref, loss_ref = {}, {}
    for dt in (torch.float32, torch.float64):
        mt = random_network(2).train().to(dt)
        loss_ref[dt] = 0.0
        for r in range(2):
            lr_ = train.local_slice(torch.arange(7), r, 2)
            pp, pv = mt(x[lr_].to(dt))
            loss = train.policy_loss_fn(pp, p[lr_].to(dt)) + torch.nn.functional.mse_loss(pv, v[lr_].to(dt))
            (loss * (len(lr_) / 7)).backward()
            loss_ref[dt] += float(loss) * len(lr_) / 7
        ref[dt] = {k: q.grad.double() for k, q in mt.named_parameters()}
    gt = torch.load(os.path.join(tmp_path, "gt.pt"), weights_only=True)
    l64 = loss_ref[torch.float64]
    assert abs(gt["loss"] - l64) <= 1e-5 * abs(l64), (gt["loss"], l64)
    for k, g64 in ref[torch.float64].items():
        scale = max(g64.abs().max().item(), 1e-12)
        err = (gt["g"][k].double() - g64).abs().max().item()
        assert err <= 1e-2 * scale, (k, err, scale)
    # train mode: the flat step's gradient is the sum over the ranks' slices of share x the gradient of
    # that slice's loss with BatchNorm over the slice alone (per-rank statistics; train.DPGraphedStep)
    # BatchNorm over 3-4 samples amplifies rounding: the single-process f32 gradient of the input conv
    # lands 2e-4 to 2.3e-2 (of 5.4) from f64 depending on the host thread count alone, so the bound is
    # 1e-2 of the gradient's scale, below any one rank's missing contribution (rank 1's part is 8% of it)
    ref, loss_ref = {}, {}
    for dt in (torch.float32, torch.float64):
        mt = random_network(2).train().to(dt)
        loss_ref[dt] = 0.0
        for r in range(2):
            lr_ = train.local_slice(torch.arange(7), r, 2)
            pp, pv = mt(x[lr_].to(dt))
            loss = train.policy_loss_fn(pp, p[lr_].to(dt)) + torch.nn.functional.mse_loss(pv, v[lr_].to(dt))
            (loss * (len(lr_) / 7)).backward()
            loss_ref[dt] += float(loss) * len(lr_) / 7
        ref[dt] = {k: q.grad.double() for k, q in mt.named_parameters()}
    gt = torch.load(os.path.join(tmp_path, "gt.pt"), weights_only=True)
    l64 = loss_ref[torch.float64]
    assert abs(gt["loss"] - l64) <= 1e-5 * abs(l64), (gt["loss"], l64)
    for k, g64 in ref[torch.float64].items():
        scale = max(g64.abs().max().item(), 1e-12)
        err = (gt["g"][k].double() - g64).abs().max().item()
        assert err <= 1e-2 * scale, (k, err, scale)
    m0 = torch.load(os.path.join(tmp_path, "m0.pt"), weights_only=True)
    m1 = torch.load(os.path.join(tmp_path, "m1.pt"), weights_only=True)
    for k in m0["sd"]:
        assert torch.equal(m0["sd"][k], m1["sd"][k]), k
    assert m0["losses"] == m1["losses"] and all(np.isfinite(m0["losses"]))
