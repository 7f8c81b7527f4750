"""FusedNetworkEvaluator: the DualNetwork leaf evaluator as gfx950 kernels
(csrc/nn_kernels.hip, csrc/wino3h_conv.hip, include/uttt_nn.h):

  leaves --k_stem--> act (n,81,128 NHWC, relu(conv_input+bn) applied, straight from bitboards)
  16 x [ conv3x3 + b1 + ReLU            (Winograd F(3x3,3x3), point GEMMs as split-f16 products
         conv3x3 + b2 + residual + ReLU ]  on the f16 MFMA, f32 accumulation)
  --k_heads--> policy (n,81) softmax, value (n,)

BatchNorm is folded (eval mode), so the function is the reference's
dual_network.py:89-121 up to fp32 rounding order (tests/test_engine_gpu.py
bounds value and post-softmax policy at 1e-5 against the reference's own CPU
fp32 outputs on a non-saturated network). Every kernel computes a board from
that board's inputs alone (the split-f16 V scale is per board), so a position's
outputs are bit-identical whatever batch it is evaluated in - the premise of
the engine's evaluation cache and of lane/GPU-count invariance.
"""
import ctypes
import weakref

import torch

from . import _lib
from ._lib import check
from .engine import RoundCount
from .model import fold_bn

HEAD = {}


def _head_layout():
    if not HEAD:
        o = 0
        for name, size in (("pconv_w", 2 * 128), ("pconv_b", 2), ("vconv_w", 128), ("vconv_b", 1),
                           ("pfc_w", 81 * 162), ("pfc_b", 81), ("vfc1_w", 256 * 81), ("vfc1_b", 256),
                           ("vfc2_w", 256), ("vfc2_b", 1)):
            HEAD[name] = (o, size)
            o += size
        HEAD["size"] = o
    return HEAD


def pack_heads(net, device):
    lay = _head_layout()
    buf = torch.zeros(lay["size"], dtype=torch.float32)
    pw, pb = fold_bn(net.policy_conv, net.policy_bn)
    vw, vb = fold_bn(net.value_conv, net.value_bn)
    parts = {"pconv_w": pw.reshape(-1), "pconv_b": pb, "vconv_w": vw.reshape(-1), "vconv_b": vb,
             "pfc_w": net.policy_fc.weight.t().reshape(-1), "pfc_b": net.policy_fc.bias,
             "vfc1_w": net.value_fc1.weight.t().reshape(-1), "vfc1_b": net.value_fc1.bias,
             "vfc2_w": net.value_fc2.weight.reshape(-1), "vfc2_b": net.value_fc2.bias}
    for k, v in parts.items():
        o, n = lay[k]
        assert v.numel() == n, (k, v.numel(), n)
        buf[o:o + n] = v.detach().float().cpu()
    return buf.to(device)


def _p(t):
    return ctypes.c_void_p(t.data_ptr())


_WEIGHTS = weakref.WeakKeyDictionary()  # model -> {(device, conv): (fingerprint, prepared weights)}


def _fingerprint(net):
    """Changes whenever a parameter or buffer is replaced or modified in place (optimizer
    steps, load_state_dict): tensors' version counters are shared with their detached views."""
    return tuple((t.data_ptr(), t._version) for t in net.state_dict().values())


@torch.no_grad()
def _prepared_weights(net, dev, conv):
    """BN-folded, kernel-ordered weights of a DualNetwork on `dev` (cached per model, device and
    kernel; rebuilt when the model's weights change)."""
    fp = _fingerprint(net)
    per = _WEIGHTS.setdefault(net, {})
    key = (str(dev), conv)
    hit = per.get(key)
    if hit is not None and hit[0] == fp:
        return hit[1]
    sw, sb = fold_bn(net.conv_input, net.bn_input)            # (128,3,3,3)
    out = {"stem_w": sw.permute(1, 2, 3, 0).reshape(27, 128).contiguous().to(dev),
           "stem_b": sb.contiguous().to(dev), "heads": pack_heads(net, dev), "wino": []}
    us, sus, bs = [], [], []
    for b in net.residual_blocks:
        for cv, bn in ((b.conv1, b.bn1), (b.conv2, b.bn2)):
            w, bb = fold_bn(cv, bn)
            u, su = wino3h_weights(w)
            us.append(u)
            sus.append(su)
            bs.append(bb.float())
    # the tower's weights back to back (uttt_nn_tower_wino3h_dev); the per-conv entries are views of them
    out["u_all"] = torch.stack(us).to(dev)
    out["bias_all"] = torch.stack(bs).contiguous().to(dev)
    out["scale_all"] = torch.tensor(sus, dtype=torch.float32, device=dev)
    for i in range(0, len(us), 2):
        out["wino"].append(((out["u_all"][i], sus[i], out["bias_all"][i]),
                            (out["u_all"][i + 1], sus[i + 1], out["bias_all"][i + 1])))
    # the stem's output bound for every board: relu(b + sum of the positive weight rows), inputs 0/1
    out["stem_bound"] = float(torch.relu(out["stem_b"].double().cpu() +
                                         out["stem_w"].double().cpu().clamp_min(0).sum(0)).max())
    per[key] = (fp, out)
    return out


class FusedNetworkEvaluator:
    """Leaf evaluator over an engine's pending leaves (needs_input = False: the stem reads
    the leaves' bitboards, the engine never builds the NCHW tensor). device_count: called
    with a RoundCount (after Engine.select_async) it reads the leaf count on the device, so
    the round needs no host synchronisation.

    precision: "f32" (default; the split-f16 tower, within 1e-5 of the fp32 DualNetwork) or "f16"
    (uttt_nn_conv3x3_wino3h_f16: one f16 product per point, ~1e-3 relative: the optional fast
    evaluator, not the reference's numerics); None reads UTTT_NN_PRECISION (default f32).

    tower: "layers" (default) launches the 32 tower convs one by one; "dataflow" runs them as ONE persistent
    launch (uttt_nn_tower_wino3h_dev: work items (conv, set) handed out in conv-major order, each waiting
    only for its own board group's previous conv; split-f16 only). Same output bits. The dataflow launch is
    1.2-1.3x faster alone on the GPU at 1.4k-2.7k boards, but holds every CU for the whole forward, so two
    lanes' towers run one after the other instead of interleaving; in the two-lane headline it is no
    faster. None reads UTTT_NN_TOWER."""
    needs_input = False
    device_count = True
    NROW = 4  # per-board max rows, rotated over the 32 convs (see __init__, _tower_heads)

    def __init__(self, net, engine=None, max_batch=None, conv="wino3h", device=None, precision=None, tower=None):
        import os
        net = net.eval()
        if conv != "wino3h":
            raise ValueError("conv must be 'wino3h' (the split-f16 Winograd tower; the f32-MFMA kernel was retired)")
        self.conv = conv
        self.precision = precision or os.environ.get("UTTT_NN_PRECISION", "f32")
        if self.precision not in ("f32", "f16"):
            raise ValueError("precision must be 'f32' (split-f16, f32-level) or 'f16' (one f16 product)")
        self.engine = engine
        self.lib = _lib.load()
        if engine is not None:
            dev = torch.device("cuda", engine.device)
            self.max_batch = max_batch or engine.max_trees
            if self.max_batch < engine.max_trees:
                # the stem writes one row per pending leaf (up to every tree of the engine; in
                # device-count rounds its grid covers them all) and k_apply reads as many rows
                raise ValueError(f"max_batch {self.max_batch} < the engine's {engine.max_trees} trees")
        else:
            dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
            if max_batch is None:
                raise ValueError("max_batch is required without an engine")
            self.max_batch = max_batch
        self.device = dev
        self.nconv = 2 * len(net.residual_blocks)
        if self.nconv % self.NROW:
            raise ValueError("the max-row rotation needs a multiple of 4 convolutions")
        w = _prepared_weights(net, dev, conv)
        self.stem_w, self.stem_b, self.heads, self.wino = w["stem_w"], w["stem_b"], w["heads"], w["wino"]
        self.u_all, self.bias_all, self.scale_all = w["u_all"], w["bias_all"], w["scale_all"]
        self.tower = tower or os.environ.get("UTTT_NN_TOWER", "layers")
        if self.tower not in ("dataflow", "layers"):
            raise ValueError("tower must be 'dataflow' (one persistent launch) or 'layers' (a launch per conv)")
        if self.precision == "f16":
            self.tower = "layers"  # the dataflow kernel is the split-f16 (f32-level) form only
        # X_even, t, X_odd of the tower as one allocation (the dataflow kernel addresses them by offset)
        self.act = torch.zeros((3, self.max_batch, 81, 128), dtype=torch.float32, device=dev)
        self.buf = [self.act[0], self.act[1], self.act[2]]
        # the dataflow launches' counters: two blocks (ticket, items done, done per 7-board group) used by
        # alternate launches, each launch resetting the other block
        self.ctl = torch.zeros(2 * self.lib.uttt_nn_tower_ctl_words(self.max_batch), dtype=torch.int32, device=dev)
        self.ctl_parity = 0
        # The stem's output is bounded for every board by relu(b + sum of the positive weight
        # rows) (its inputs are 0/1 planes): one scale for all boards. Conv i then reads the
        # per-board maxima of its input from row (i-1) % 4, atomically maxes its own output
        # into row i % 4 and zeroes row (i+1) % 4 for conv i+1; 32 convs per forward keep
        # the rotation aligned across forwards, so no fill kernel is ever needed.
        self.stem_bound = w["stem_bound"]
        self.stem_amax = torch.tensor([self.stem_bound], dtype=torch.float32, device=dev).view(torch.int32)
        self.bamax = torch.zeros((self.NROW, self.max_batch), dtype=torch.int32, device=dev)
        self.policy = torch.zeros((self.max_batch, 81), dtype=torch.float32, device=dev)
        self.value = torch.zeros((self.max_batch,), dtype=torch.float32, device=dev)
        self.states = None
        # bench telemetry: when a list, every forward appends (n, start event, end event) recorded
        # on its stream around the residual tower (2 x blocks conv launches)
        self.tower_events = None

    def _stream(self):
        return ctypes.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)

    @torch.no_grad()
    def forward(self, n, softmax=True):
        """Evaluate the engine's n pending leaves; returns (policy or logits (n,81), value (n,)).
        n a RoundCount: the count is read on the device (Engine.select_async), and the full
        (max_batch, 81) / (max_batch,) buffers are returned (rows past the count untouched)."""
        check(self.lib.uttt_nn_stem(self.engine.h, _p(self.stem_w), _p(self.stem_b), _p(self.buf[0])))
        if isinstance(n, RoundCount):
            return self._tower_heads(n, softmax, n_dev=self.engine.count_ptr())
        return self._tower_heads(n, softmax)

    @torch.no_grad()
    def forward_states(self, states, softmax=True):
        """Evaluate packed states (a STATE_DTYPE numpy array, any count <= max_batch)."""
        import numpy as np
        n = len(states)
        if n > self.max_batch:
            raise ValueError(f"{n} states > max_batch {self.max_batch}")
        if self.states is None:
            self.states = torch.zeros((self.max_batch, 8), dtype=torch.int32, device=self.device)
        if n == 0:
            return self.policy[:0], self.value[:0]
        st = np.ascontiguousarray(states).view(np.int32).reshape(n, 8)
        self.states[:n].copy_(torch.from_numpy(st))
        check(self.lib.uttt_nn_stem_states(_p(self.states), n, _p(self.stem_w), _p(self.stem_b), _p(self.buf[0]),
                                           self._stream()))
        return self._tower_heads(n, softmax)

    def _dev_plan(self, stream, n_dev):
        """The device-count forward's 32 conv argument tuples (fixed buffers and weights), built
        once per (stream, count): the per-round host cost is then one ctypes call per kernel."""
        key = (stream.value, n_dev.value)
        if getattr(self, "_plan", None) is None or self._plan[0] != key:
            rows = [ctypes.c_void_p(self.bamax[r].data_ptr()) for r in range(self.NROW)]
            cap = self.max_batch
            x, t, y = (ctypes.c_void_p(b.data_ptr()) for b in self.buf)
            calls, i = [], 0
            for (u1, s1, b1), (u2, s2, b2) in self.wino:
                src = (_p(self.stem_amax), 0) if i == 0 else (rows[(i - 1) % 4], 1)
                calls.append((x, _p(u1), ctypes.c_float(s1), _p(b1), None, t, src[0], src[1], rows[i % 4],
                              rows[(i + 1) % 4], cap, n_dev, cap, stream))
                i += 1
                calls.append((t, _p(u2), ctypes.c_float(s2), _p(b2), x, y, rows[(i - 1) % 4], 1, rows[i % 4],
                              rows[(i + 1) % 4], cap, n_dev, cap, stream))
                i += 1
                x, y = y, x
            heads = (x, _p(self.heads), n_dev, cap, _p(self.policy), _p(self.value))
            self._plan = (key, calls, heads)
        return self._plan

    def _tower_dataflow(self, stream, n_dev, max_boards):
        check(self.lib.uttt_nn_tower_wino3h_dev(_p(self.act), ctypes.c_int64(self.act[0].numel()), _p(self.u_all),
                                                _p(self.scale_all), _p(self.bias_all), self.nconv, _p(self.stem_amax),
                                                _p(self.bamax), self.max_batch, _p(self.ctl), self.ctl_parity, n_dev,
                                                int(max_boards), stream))
        self.ctl_parity ^= 1

    def _tower_heads(self, n, softmax, n_dev=None):
        stream = self._stream()
        if self.tower == "dataflow" and (n_dev is not None or n > 28):
            # one persistent launch for the whole tower (small host-count batches keep the per-conv kernels'
            # channel split); the final activation is X_even = buf[0]
            if self.tower_events is not None:
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
            self._tower_dataflow(stream, n_dev, self.max_batch if n_dev is not None else n)
            if self.tower_events is not None:
                ev1.record()
                self.tower_events.append((n, ev0, ev1))
            if n_dev is not None:
                check(self.lib.uttt_nn_heads_dev(_p(self.buf[0]), _p(self.heads), n_dev, self.max_batch,
                                                 _p(self.policy), _p(self.value), 1 if softmax else 0, stream))
                return self.policy, self.value
            check(self.lib.uttt_nn_heads(_p(self.buf[0]), _p(self.heads), n, _p(self.policy), _p(self.value),
                                         1 if softmax else 0, stream))
            return self.policy[:n], self.value[:n]
        if n_dev is not None:
            _, calls, heads = self._dev_plan(stream, n_dev)
            if self.tower_events is not None:
                ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                ev0.record()
            fn = self.lib.uttt_nn_conv3x3_wino3h_f16_dev if self.precision == "f16" else \
                self.lib.uttt_nn_conv3x3_wino3h_dev
            for a in calls:
                check(fn(*a))
            if self.tower_events is not None:
                ev1.record()
                self.tower_events.append((n, ev0, ev1))
            check(self.lib.uttt_nn_heads_dev(*heads, 1 if softmax else 0, stream))
            return self.policy, self.value
        x, t, y = self.buf
        if self.tower_events is not None:
            ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ev0.record()
        rows = [ctypes.c_void_p(self.bamax[r].data_ptr()) for r in range(self.NROW)]
        cap = self.max_batch
        fn = self.lib.uttt_nn_conv3x3_wino3h_f16 if self.precision == "f16" else self.lib.uttt_nn_conv3x3_wino3h
        i = 0
        for (u1, s1, b1), (u2, s2, b2) in self.wino:
            src = (_p(self.stem_amax), 0) if i == 0 else (rows[(i - 1) % 4], 1)
            check(fn(_p(x), _p(u1), ctypes.c_float(s1), _p(b1), None, _p(t), src[0], src[1], rows[i % 4],
                     rows[(i + 1) % 4], cap, n, stream))
            i += 1
            check(fn(_p(t), _p(u2), ctypes.c_float(s2), _p(b2), _p(x), _p(y), rows[(i - 1) % 4], 1, rows[i % 4],
                     rows[(i + 1) % 4], cap, n, stream))
            i += 1
            x, y = y, x
        if self.tower_events is not None:
            ev1.record()
            self.tower_events.append((n, ev0, ev1))
        check(self.lib.uttt_nn_heads(_p(x), _p(self.heads), n, _p(self.policy), _p(self.value),
                                     1 if softmax else 0, stream))
        return self.policy[:n], self.value[:n]

    def __call__(self, x, n):
        return self.forward(n, True)


def wino3h_weights(w):
    """Folded conv weight (128,128,3,3) -> (U as f16 hi/lo pairs, 25*128*128*2 int16 in kernel order, su):
    the split-f16 F(3x3,3x3) kernel's weights, scaled by the power of two su (host, double)."""
    import numpy as np
    wc = np.ascontiguousarray(w.detach().float().cpu().numpy())
    u = np.zeros((25 * 128 * 128 * 2,), np.uint16)
    su = ctypes.c_float(0.0)
    lib = _lib.load()
    check(lib.uttt_nn_wino3h_weights(wc.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                     ctypes.c_void_p(u.ctypes.data), ctypes.byref(su)))
    return torch.from_numpy(u.view(np.int16)), su.value


def set_conv_split(split):
    """The tower conv's channel split for small batches (uttt_nn_wino3h_set_split): -1 automatic
    (default: split 2 up to 28 boards), 1 the persistent kernel only, 2 forced. Every choice gives the
    same output bits."""
    check(_lib.load().uttt_nn_wino3h_set_split(int(split)))


def amax(x, out=None):
    """max |x| as a (1,) int32 tensor of float bits on x's device (uttt_nn_amax)."""
    if out is None:
        out = torch.zeros(1, dtype=torch.int32, device=x.device)
    check(_lib.load().uttt_nn_amax(_p(x), x.numel(), _p(out), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    return out


def board_amax(x):
    """Per-board max |x| of (n,81,128) activations as int32 float bits (the y_amax row form)."""
    return x.abs().reshape(x.shape[0], -1).amax(dim=1).contiguous().view(torch.int32)


def conv3x3_wino3h(x, u, su, bias, residual=None, y_amax=None, x_amax=None, precision="f32"):
    """Test/utility wrapper for the split-f16 F(3x3,3x3) kernel: x (n,81,128) f32 cuda ->
    relu(conv3x3(x) + bias (+ residual)); u, su from wino3h_weights(). x_amax: per-board
    max rows (default: computed from x); y_amax: optional (n,) int32 row receiving max(y) per board.
    precision "f16": the one-product f16 mode (uttt_nn_conv3x3_wino3h_f16)."""
    y = torch.empty_like(x)
    xa = board_amax(x) if x_amax is None else x_amax
    lib = _lib.load()
    fn = lib.uttt_nn_conv3x3_wino3h_f16 if precision == "f16" else lib.uttt_nn_conv3x3_wino3h
    check(fn(_p(x), _p(u), ctypes.c_float(su), _p(bias), _p(residual) if residual is not None else None, _p(y), _p(xa),
             1, _p(y_amax) if y_amax is not None else None, None, 0, x.shape[0],
             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    return y


_DUAL_ATTRS = ("conv_input", "bn_input", "residual_blocks", "policy_conv", "policy_bn", "policy_fc", "value_conv",
               "value_bn", "value_fc1", "value_fc2")


def is_dual_network(model):
    """True for a DualNetwork (this package's or the reference's dual_network.DualNetwork: same
    module names, dual_network.py:47-87) of the shape the fused kernels compute: 128 filters,
    3x3 convs, a multiple of 2 residual blocks, 81 policy outputs, eval mode."""
    try:
        if not all(hasattr(model, a) for a in _DUAL_ATTRS) or getattr(model, "training", False):
            return False
        if tuple(model.conv_input.weight.shape) != (128, 3, 3, 3):
            return False
        blocks = list(model.residual_blocks)
        if not blocks or (2 * len(blocks)) % FusedNetworkEvaluator.NROW:
            return False
        for b in blocks:
            if tuple(b.conv1.weight.shape) != (128, 128, 3, 3) or tuple(b.conv2.weight.shape) != (128, 128, 3, 3):
                return False
        return (tuple(model.policy_fc.weight.shape) == (81, 162) and tuple(model.value_fc1.weight.shape) == (256, 81)
                and tuple(model.value_fc2.weight.shape) == (1, 256))
    except (AttributeError, TypeError):
        return False


def evaluator_kind(model, kind=None):
    """Which leaf evaluator the drop-ins use for `model`: "fused" (the HIP kernels, default for
    a DualNetwork), or "torch" (model(x) under PyTorch-ROCm: any other callable, or forced by
    kind="torch" / the environment variable UTTT_EVALUATOR=torch)."""
    import os
    kind = kind or os.environ.get("UTTT_EVALUATOR", "auto")
    if kind not in ("auto", "fused", "torch"):
        raise ValueError("evaluator kind must be 'auto', 'fused' or 'torch'")
    if kind == "auto":
        return "fused" if is_dual_network(model) else "torch"
    if kind == "fused" and not is_dual_network(model):
        raise ValueError("the fused evaluator needs a DualNetwork (128 filters, 3x3, eval mode)")
    return kind
