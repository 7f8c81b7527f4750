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


class GraphedStep:
    """One optimiser step of the static global batch (gather from the resident dataset, forward,
    loss, backward, Adam) captured once in a HIP graph and replayed per batch: ~300 kernels per
    step become one graph launch, so the step is no longer bound by host launch overhead.

    Adam runs with capturable=True and a device-tensor learning rate (the epoch's LambdaLR factor
    is written into it, not baked into the graph). The warm-up steps the capture needs are undone
    (parameters, buffers and optimiser state restored in place), so training starts from the
    caller's weights exactly as the eager loop does. The graph adds the step's loss to a device
    accumulator; batches of another size (an epoch's last) run the same body eagerly."""

    def __init__(self, model, opt, x, p, v, batch_size, channels_last=False, precision="fp32", tune=False):
        self.model, self.opt, self.x, self.p, self.v = model, opt, x, p, v
        self.channels_last = channels_last
        if precision not in PRECISIONS:
            raise ValueError(f"precision must be one of {PRECISIONS}")
        self.precision = precision
        dev = x.device
        self.idx = torch.zeros(batch_size, dtype=torch.long, device=dev)
        self.loss_sum = torch.zeros((), device=dev)
        if precision == "f16":
            # static loss scale; a step whose unscaled gradients hold an inf / nan is skipped on the
            # device (fused Adam reads found_inf), so nothing in the step needs the host
            self.scale = float(F16_LOSS_SCALE)
            self.inv_scale = torch.full((), 1.0 / F16_LOSS_SCALE, device=dev)
            self.found_inf = torch.zeros((), device=dev)
            opt.found_inf = self.found_inf
        snap = {k: t.detach().clone() for k, t in model.state_dict().items()}
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        # MIOpen's immediate mode (heuristic kernel choice), whatever torch.backends.cudnn.benchmark
        # says (the reference's dual_network.py sets it at import): with find mode the captured step
        # ran 7x slower and trained to a different loss (round 3, tools/bench_train.py), because find
        # then ran inside the warm-up on the side stream. tune=True (round 4, train_network's default):
        # MIOpen's find runs first, in two eager steps on the current stream outside any capture, and the
        # warm-up and capture reuse its choices (benchmark mode, results cached per shape): graph fp32
        # 13.0k -> 16.3k samples/s, the same losses (tools/bench_train.py, profiles/r4/train_bench.json)
        if tune:
            with torch.backends.cudnn.flags(enabled=True, benchmark=True, deterministic=False):
                for _ in range(2):
                    opt.zero_grad(set_to_none=True)
                    self._body(self.idx)
            torch.cuda.synchronize(dev)
        with torch.backends.cudnn.flags(enabled=True, benchmark=bool(tune), deterministic=False):
            with torch.cuda.stream(side):
                for _ in range(3):  # allocator, MIOpen kernel choice, optimiser state
                    opt.zero_grad(set_to_none=True)
                    self._body(self.idx)
            torch.cuda.current_stream(dev).wait_stream(side)
            self.graph = torch.cuda.CUDAGraph()
            opt.zero_grad(set_to_none=True)
            with torch.cuda.graph(self.graph):
                self._body(self.idx)
        # undo the warm-up: the same tensors (the graph's addresses), the caller's values
        with torch.no_grad():
            for k, t in model.state_dict().items():
                t.copy_(snap[k])
            for st in opt.state.values():
                for name, t in st.items():
                    if torch.is_tensor(t):
                        t.zero_()
        self.loss_sum.zero_()

    def _body(self, idx):
        xb = self.x.index_select(0, idx)
        if self.channels_last:
            xb = xb.contiguous(memory_format=torch.channels_last)
        if self.precision == "f16":
            with torch.autocast("cuda", dtype=torch.float16):
                pred_p, pred_v = self.model(xb)
            pred_p, pred_v = pred_p.float(), pred_v.float()
        else:
            pred_p, pred_v = self.model(xb)
        loss = policy_loss_fn(pred_p, self.p.index_select(0, idx)) + \
            nn.functional.mse_loss(pred_v, self.v.index_select(0, idx))
        if self.precision == "f16":
            (loss * self.scale).backward()
            self.found_inf.zero_()
            grads = [q.grad for q in self.model.parameters() if q.grad is not None]
            torch._amp_foreach_non_finite_check_and_unscale_(grads, self.found_inf, self.inv_scale)
        else:
            loss.backward()
        self.opt.step()
        self.loss_sum += loss.detach()
        return loss

    def step(self, idx):
        if idx.numel() == self.idx.numel():
            self.idx.copy_(idx, non_blocking=True)
            self.graph.replay()
        else:
            self.opt.zero_grad(set_to_none=False)
            with torch.backends.cudnn.flags(enabled=True, benchmark=False, deterministic=False):
                self._body(idx)


def all_reduce_sum(t):
    """dist.all_reduce(t) (SUM) in place. gloo with a device tensor (ranks sharing a GPU: the multi-rank GPU
    tests' form) goes through an explicit, synchronous host copy, so the collective never depends on gloo's
    own device streams and pinned staging buffers (round 6: one run in ~30 of tests/dp_flat_two_ranks_main.py
    read a NaN loss there, cause not found). RCCL and host tensors take dist.all_reduce directly."""
    if t.is_cuda and dist.get_backend() == "gloo":
        h = t.cpu()
        dist.all_reduce(h)
        t.copy_(h)
    else:
        dist.all_reduce(t)


class DPGraphedStep:
    """The data-parallel step of a torchrun rank as two HIP graphs around ONE collective (round 5):

      graph A: gather this rank's slice of the global batch from the HBM-resident dataset, forward,
               loss x this rank's share of the global batch (n_r / N), backward into one flat
               gradient buffer (every parameter's .grad is a view of it, so autograd accumulates in
               place and nothing is copied);
      all_reduce(SUM) of that buffer (RCCL over xGMI; 4.77 M f32 = 19.1 MB), enqueued on the current
               stream between the replays: the averaged gradient of the global mean loss;
      graph B: fused Adam (capturable, device-tensor learning rate).

    ~600 kernel launches per step become two graph launches and one collective. DDP's bucketed
    all-reduce overlaps the backward, but a captured graph cannot interleave host-issued collectives,
    and the step at the per-rank batch of 16 is launch-bound, so one flat all-reduce
    after the graph is the cheaper form. BatchNorm runs on each rank's own slice (per-rank batch
    statistics, as plain DDP does): a numerics change against the reference's batch-128 statistics
    (train_network.py:88-113 on one device), which SyncBatchNorm (UTTT_TRAIN_DP=ddp) keeps at ~70
    small collectives per step. The running statistics are averaged over the ranks after every
    epoch (train_network's caller sees one model on every rank).

    graph=False runs the same three phases eagerly (the CPU / gloo form the multi-rank tests run)."""

    def __init__(self, model, opt, x, p, v, local_batch, share, graph=True, tune=False):
        """local_batch / share: this rank's slice of a full global batch and its n_r / N (the graphs')."""
        self.model, self.opt, self.x, self.p, self.v = model, opt, x, p, v
        self.rank, self.world = _world()
        # the collective runs whenever a process group exists (one rank too: RCCL's path on one GPU)
        self.collective = dist.is_available() and dist.is_initialized()
        dev = x.device
        params = [q for q in model.parameters() if q.requires_grad]
        self.flat = torch.zeros(sum(q.numel() for q in params), device=dev)
        o = 0
        for q in params:  # .grad as views of one buffer: backward accumulates into it in place
            q.grad = self.flat[o:o + q.numel()].view_as(q)
            o += q.numel()
        self.idx = torch.zeros(local_batch, dtype=torch.long, device=dev)
        self.share_f = float(share)
        self.share = torch.full((), self.share_f, device=dev)  # n_r / N of the static batch
        self.loss_sum = torch.zeros((), device=dev)
        self.graph = bool(graph) and dev.type == "cuda"
        if not self.graph:
            return
        snap = {k: t.detach().clone() for k, t in model.state_dict().items()}
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        if tune:  # MIOpen's find on the current stream, outside any capture (as GraphedStep)
            with torch.backends.cudnn.flags(enabled=True, benchmark=True, deterministic=False):
                for _ in range(2):
                    self._fb(self.idx, self.share)
                    self.opt.step()
            torch.cuda.synchronize(dev)
        with torch.backends.cudnn.flags(enabled=True, benchmark=bool(tune), deterministic=False):
            with torch.cuda.stream(side):
                for _ in range(3):  # allocator, kernel choice, optimiser state
                    self._fb(self.idx, self.share)
                    self.opt.step()
            torch.cuda.current_stream(dev).wait_stream(side)
            self.g_fb, self.g_opt = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.g_fb):
                self._fb(self.idx, self.share)
            with torch.cuda.graph(self.g_opt, pool=self.g_fb.pool()):
                self.opt.step()
        with torch.no_grad():  # undo the warm-up: the graphs' tensors, the caller's values
            for k, t in model.state_dict().items():
                t.copy_(snap[k])
            for st in opt.state.values():
                for t in st.values():
                    if torch.is_tensor(t):
                        t.zero_()
            self.flat.zero_()
        self.loss_sum.zero_()

    def _fb(self, idx, share):
        self.flat.zero_()
        if idx.numel():
            pred_p, pred_v = self.model(self.x.index_select(0, idx))
            loss = policy_loss_fn(pred_p, self.p.index_select(0, idx)) + \
                nn.functional.mse_loss(pred_v, self.v.index_select(0, idx))
            (loss * share).backward()
            self.loss_sum += loss.detach() * share  # this rank's share of the global mean loss

    def step(self, idx, share):
        """One global-batch step: idx = this rank's slice (device tensor), share = its n_r / N."""
        if self.graph and idx.numel() == self.idx.numel() and share == self.share_f:
            self.idx.copy_(idx, non_blocking=True)
            self.g_fb.replay()
            if self.collective:
                all_reduce_sum(self.flat)
            self.g_opt.replay()
            return
        sh = torch.full((), float(share), device=self.flat.device)
        with torch.backends.cudnn.flags(enabled=True, benchmark=False, deterministic=False):
            self._fb(idx, sh)
        if self.collective:
            all_reduce_sum(self.flat)
        self.opt.step()

    def sync_buffers(self):
        """Combine the BatchNorm running statistics of the ranks (one all_reduce of a flat copy): the
        running means are averaged, and the running variances combined as a pooled variance, E[var_r +
        mean_r^2] - mean^2, so the spread between the ranks' means is counted (averaging the variances
        alone leaves it out and biases the eval-time statistics low)."""
        if self.world == 1:
            return
        bns = [m for m in self.model.modules() if isinstance(m, nn.modules.batchnorm._BatchNorm)
               and m.running_mean is not None]
        with torch.no_grad():
            parts = []
            for m in bns:
                parts += [m.running_mean.reshape(-1), (m.running_var + m.running_mean * m.running_mean).reshape(-1)]
            flat = torch.cat(parts)
            all_reduce_sum(flat)
            flat /= self.world
            o = 0
            for m in bns:
                c = m.running_mean.numel()
                mean, ex2 = flat[o:o + c], flat[o + c:o + 2 * c]
                m.running_mean.copy_(mean.view_as(m.running_mean))
                m.running_var.copy_((ex2 - mean * mean).clamp_min(0).view_as(m.running_var))
                o += 2 * c


PRECISIONS = ("fp32", "f16")
# "f16": convolutions and linear layers on f16 operands (10-bit mantissa, the reference's cuDNN TF32
# default on its NVIDIA card has the same), f32 accumulation, BatchNorm / softmax / loss in f32
F16_LOSS_SCALE = 2.0 ** 12


def _use_graph(graph, device, world):
    if graph is None:
        import os
        graph = os.environ.get("UTTT_TRAIN_GRAPH", "1") != "0"
    return bool(graph) and world == 1 and device.type == "cuda"


def train_network(model, history, epochs=RN_EPOCHS, batch_size=BATCH_SIZE, device=None, seed=0, lr=0.001,
                  log=print, sync_bn=None, graph=None, channels_last=False, precision=None, tune=None, adam=None,
                  dp=None):
    """Train `model` (a DualNetwork) on `history` in place; returns the per-epoch mean losses.
    In a torch.distributed job every rank calls this with the same history and seed.
    graph (default on for one GPU; UTTT_TRAIN_GRAPH=0 disables): replay the step as a HIP graph
    (GraphedStep); the eager loop otherwise.
    dp (UTTT_TRAIN_DP; data-parallel jobs only): "ddp" (the default) = the eager DDP loop, with
    SyncBatchNorm on GPUs unless sync_bn=False, so BatchNorm normalises over the whole global batch of
    128 as the reference's one-device loop does (~70 small collectives per step); "flat" (opt-in) =
    DPGraphedStep, two graphs around one flat gradient all-reduce, with per-rank BatchNorm statistics (a
    numerics change: 16 samples per rank at 8 GPUs)."""
    import os
    rank, world = _world()
    device = device or (torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available()
                        else torch.device("cpu"))
    x, p, v = (torch.from_numpy(a).to(device) for a in history_arrays(history))  # resident in HBM
    if precision is None:
        precision = os.environ.get("UTTT_TRAIN_PRECISION", "fp32")
    if tune is None:  # MIOpen find before the capture (round 4: graph fp32 13.0k -> 16.3k samples/s)
        tune = os.environ.get("UTTT_TRAIN_TUNE", "1") != "0"
    if adam is None:  # the graph step's Adam: "fused" (default) or "foreach" (rounds 1-3 for fp32)
        adam = os.environ.get("UTTT_TRAIN_ADAM", "fused")
    if dp is None:
        dp = os.environ.get("UTTT_TRAIN_DP", "ddp")
    if dp not in ("flat", "ddp"):
        raise ValueError("dp must be 'flat' or 'ddp'")
    if _use_graph(graph, device, world):
        return _train_graphed(model, x, p, v, epochs, batch_size, device, seed, lr, log, channels_last, precision, tune,
                              adam)
    if world > 1 and dp == "flat":
        if precision != "fp32":
            raise ValueError("the data-parallel step trains in fp32")
        return _train_dp_flat(model, x, p, v, epochs, batch_size, device, seed, lr, log,
                              graph=graph is not False and device.type == "cuda", tune=tune)
    if precision != "fp32":
        raise ValueError("precision other than fp32 needs the graph step (one GPU)")
    net = prepare(model, device, sync_bn)
    # on the GPU the fused Adam kernel (same update; the per-parameter foreach kernels were ~1 ms of a
    # 128-sample step on one MI355X, §7c), the reference's default Adam on the CPU
    opt = torch.optim.Adam(net.parameters(), lr=lr, fused=True) if device.type == "cuda" and adam == "fused" \
        else torch.optim.Adam(net.parameters(), lr=lr)
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


def _train_dp_flat(model, x, p, v, epochs, batch_size, device, seed, lr, log, graph=True, tune=False):
    """The data-parallel loop on DPGraphedStep (see there): every rank draws the epoch's permutation from
    the same generator and steps on its slice of each global batch."""
    rank, world = _world()
    net = model.to(device)
    with torch.no_grad():  # one set of weights on every rank (DDP broadcasts rank 0's at construction)
        for t in net.state_dict().values():
            dist.broadcast(t, 0)
    net.train()
    if device.type == "cuda":
        lr_t = torch.tensor(lr, dtype=torch.float32, device=device)
        opt = torch.optim.Adam(net.parameters(), lr=lr_t, capturable=True, fused=True)
    else:  # the reference's default Adam on the host
        lr_t = None
        opt = torch.optim.Adam(net.parameters(), lr=lr)
    full = local_slice(torch.arange(batch_size), rank, world)
    step = DPGraphedStep(net, opt, x, p, v, len(full), len(full) / batch_size, graph=graph, tune=tune)
    losses = []
    for epoch in range(epochs):
        f = lr * lr_lambda(epoch)
        if lr_t is not None:
            lr_t.fill_(f)
        else:
            for g in opt.param_groups:
                g["lr"] = f
        step.loss_sum.zero_()
        idxs = batches(len(x), batch_size, epoch, seed)
        mine = [local_slice(b, rank, world) for b in idxs]
        perm = torch.cat(mine).to(device, non_blocking=True)
        o = 0
        for b, li in zip(idxs, mine):
            step.step(perm[o:o + len(li)], len(li) / len(b))
            o += len(li)
        total = step.loss_sum.clone()
        if world > 1:
            all_reduce_sum(total)
        step.sync_buffers()
        losses.append(float(total) / len(idxs))
        if log and rank == 0:
            log(f"Epoch {epoch + 1}/{epochs}, Loss: {losses[-1]:.4f}, LR: {lr * lr_lambda(epoch + 1):.6f}")
    return losses


def _train_graphed(model, x, p, v, epochs, batch_size, device, seed, lr, log, channels_last, precision="fp32",
                   tune=False, adam="fused"):
    net = model.to(device)
    if channels_last:
        net = net.to(memory_format=torch.channels_last)
    net.train()
    lr_t = torch.tensor(lr, dtype=torch.float32, device=device)
    # the fused Adam kernel for both precisions (f16: it also takes found_inf and skips the step on the
    # device). Round 4: the fp32 step used foreach=True, which with capturable=True and a tensor lr ran
    # ~800 per-parameter kernels per step (222 of them divisions, ~1 ms of the 7.9 ms step in the trace,
    # profiles/r4/train_fp32_graph_tuned_kernel_stats.csv); the update is the same algorithm
    if adam not in ("fused", "foreach"):
        raise ValueError("adam must be 'fused' or 'foreach'")
    if adam == "fused" or precision == "f16":
        opt = torch.optim.Adam(net.parameters(), lr=lr_t, capturable=True, fused=True)
    else:
        opt = torch.optim.Adam(net.parameters(), lr=lr_t, capturable=True, foreach=True)
    step = GraphedStep(net, opt, x, p, v, batch_size, channels_last, precision, tune)
    losses = []
    for epoch in range(epochs):
        lr_t.fill_(lr * lr_lambda(epoch))
        step.loss_sum.zero_()
        idxs = batches(len(x), batch_size, epoch, seed)
        perm = torch.cat(idxs).to(device, non_blocking=True)
        o = 0
        for b in idxs:
            step.step(perm[o:o + len(b)])
            o += len(b)
        losses.append(float(step.loss_sum) / len(idxs))
        if log:
            log(f"Epoch {epoch + 1}/{epochs}, Loss: {losses[-1]:.4f}, LR: {lr * lr_lambda(epoch + 1):.6f}")
    if channels_last:
        net.to(memory_format=torch.contiguous_format)
    return losses


__all__ = ["BATCH_SIZE", "DPGraphedStep", "F16_LOSS_SCALE", "GraphedStep", "PRECISIONS", "RN_EPOCHS", "batches", "history_arrays", "local_slice", "lr_lambda",
           "policy_loss_fn", "prepare", "train_network", "train_step"]
