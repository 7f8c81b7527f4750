"""train_network.py as data-parallel training, one process per GPU.

The reference trains DualNetwork on the newest .history for RN_EPOCHS epochs,
batch 128, shuffled, Adam(lr 1e-3) with LambdaLR (x0.5 from epoch 50, x0.25
from 80), loss = -sum(target * log(pred + 1e-8)) / N + MSE(value)
(train_network.py:41-125). Here the same global batch of 128 is split evenly
over the ranks (so W ranks run the reference's optimisation, not a W-times
larger batch): every rank draws the epoch's permutation from the same seeded
generator and takes its slice of each global batch; gradients are averaged by
DDP's bucketed all-reduce (RCCL over xGMI on MI355X, overlapped with the
backward); BatchNorm statistics span the global batch through SyncBatchNorm on
GPU. With one process this is the reference's loop on the GPU.

Equal-size shards make the averaged per-rank mean losses equal the global mean
loss, so one data-parallel step equals the single-process step up to
floating-point summation order (tests/test_distributed.py).
"""
import numpy as np
import torch
import torch.distributed as dist
import torch.nn as nn

RN_EPOCHS = 100
BATCH_SIZE = 128


def history_arrays(history):
    """[[x (9,9,3), policy (81,), value], ...] -> (x NCHW f32, policies f32, values f32 (N,1))
    exactly as HistoryDataset prepares them (train_network.py:27-36)."""
    xs, ps, vs = zip(*history)
    x = np.transpose(np.array(xs), (0, 3, 1, 2)).astype(np.float32)
    return x, np.array(ps).astype(np.float32), np.array(vs).astype(np.float32).reshape(-1, 1)


def policy_loss_fn(pred, target):
    """train_network.py:70-74 (pred is softmax output)."""
    return -torch.sum(target * torch.log(pred + 1e-8)) / pred.size(0)


def lr_lambda(epoch):
    """train_network.py:80-86."""
    if epoch >= 80:
        return 0.25
    if epoch >= 50:
        return 0.5
    return 1.0


def _world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def prepare(model, device, sync_bn=None):
    """Move to device; for W > 1 wrap in DDP (SyncBatchNorm on GPU unless sync_bn=False)."""
    rank, world = _world()
    model = model.to(device)
    if world == 1:
        return model
    if sync_bn is None:
        sync_bn = device.type == "cuda"
    if sync_bn:
        model = nn.SyncBatchNorm.convert_sync_batchnorm(model)
    ids = [device.index] if device.type == "cuda" else None
    return nn.parallel.DistributedDataParallel(model, device_ids=ids, bucket_cap_mb=25)


def train_step(model, optimizer, x, p, v):
    """One optimiser step on this rank's shard; returns the (local) loss."""
    optimizer.zero_grad()
    pred_p, pred_v = model(x)
    loss = policy_loss_fn(pred_p, p) + nn.functional.mse_loss(pred_v, v)
    loss.backward()
    optimizer.step()
    return loss


def batches(n, batch_size, epoch, seed):
    """The epoch's shuffled global batches (same on every rank)."""
    g = torch.Generator().manual_seed(seed * 1000003 + epoch)
    perm = torch.randperm(n, generator=g)
    return [perm[i:i + batch_size] for i in range(0, n, batch_size)]


def local_slice(idx, rank, world):
    """Rank's contiguous share of one global batch (sizes differ by at most one)."""
    base, extra = divmod(len(idx), world)
    b = rank * base + min(rank, extra)
    return idx[b:b + base + (1 if rank < extra else 0)]


def train_network(model, history, epochs=RN_EPOCHS, batch_size=BATCH_SIZE, device=None, seed=0, lr=0.001,
                  log=print, sync_bn=None):
    """Train `model` (a DualNetwork) on `history` in place; returns the per-epoch mean losses.
    In a torch.distributed job every rank calls this with the same history and seed."""
    rank, world = _world()
    device = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
                        else torch.device("cpu"))
    x, p, v = (torch.from_numpy(a).to(device) for a in history_arrays(history))  # resident in HBM
    net = prepare(model, device, sync_bn)
    opt = torch.optim.Adam(net.parameters(), lr=lr)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, lr_lambda=lr_lambda)
    net.train()
    losses = []
    for epoch in range(epochs):
        total = torch.zeros((), device=device)
        nb = 0
        for idx in batches(len(x), batch_size, epoch, seed):
            li = local_slice(idx, rank, world).to(device)
            loss = train_step(net, opt, x[li], p[li], v[li])
            total += loss.detach() * (len(li) / len(idx)) * world  # local mean -> share of the global mean
            nb += 1
        if world > 1:
            dist.all_reduce(total)
            total /= world
        sched.step()
        losses.append(float(total) / nb)
        if log and rank == 0:
            log(f"Epoch {epoch + 1}/{epochs}, Loss: {losses[-1]:.4f}, LR: {sched.get_last_lr()[0]:.6f}")
    return losses


__all__ = ["BATCH_SIZE", "RN_EPOCHS", "batches", "history_arrays", "local_slice", "lr_lambda", "policy_loss_fn",
           "prepare", "train_network", "train_step"]
