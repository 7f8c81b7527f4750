"""FusedNetworkEvaluator: the DualNetwork leaf evaluator as gfx950 kernels
(csrc/nn_kernels.hip, csrc/wino_conv.hip, include/uttt_nn.h):

  leaves --k_stem--> act (n,9,9,128 NHWC, relu(conv_input+bn) applied)
  16 x [ conv3x3 + b1 + ReLU            (conv="wino3h": Winograd F(3x3,3x3), split-f16 MFMA,
         conv3x3 + b2 + residual + ReLU ]  conv="wino3": the same on f32 MFMA,
                                           conv="wino": Winograd F(2x2,3x3), f32 MFMA,
                                           conv="miopen": MIOpen NHWC conv + k_epilogue)
  --k_heads--> policy (n,81) softmax, value (n,)

Replaces, per forward, the engine's NCHW encode, MIOpen's stem conv (naive /
ck grouped kernels for 3 input channels), every separate bias / ReLU / add
pass, and the head convs + FCs. BatchNorm is folded (eval mode), so the
function is the reference's dual_network.py:89-121 up to fp32 rounding order.
"""
import ctypes

import torch
import torch.nn.functional as F

from . import _lib
from ._lib import check
from .model import fold_bn
from .selfplay import _bucket

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


class FusedNetworkEvaluator:
    needs_input = False
    AMAX_RING = 64

    def __init__(self, net, engine, max_batch=None, conv="wino3h"):
        net = net.eval()
        assert conv in ("wino3h", "wino3", "wino", "miopen")
        self.conv = conv
        self.engine = engine
        self.lib = _lib.load()
        dev = torch.device("cuda", engine.device)
        self.max_batch = max_batch or engine.max_trees
        with torch.no_grad():
            sw, sb = fold_bn(net.conv_input, net.bn_input)            # (128,3,3,3)
            self.stem_w = sw.permute(1, 2, 3, 0).reshape(27, 128).contiguous().to(dev)
            self.stem_b = sb.contiguous().to(dev)
            cl = torch.channels_last
            self.blocks = []
            for b in net.residual_blocks:
                w1, b1 = fold_bn(b.conv1, b.bn1)
                w2, b2 = fold_bn(b.conv2, b.bn2)
                self.blocks.append((w1.to(dev).contiguous(memory_format=cl), b1.to(dev),
                                    w2.to(dev).contiguous(memory_format=cl), b2.to(dev)))
            self.heads = pack_heads(net, dev)
            if conv == "wino3h":
                self.wino = []
                for b in net.residual_blocks:
                    pair = []
                    for cv, bn in ((b.conv1, b.bn1), (b.conv2, b.bn2)):
                        w, bb = fold_bn(cv, bn)
                        u, su = wino3h_weights(w)
                        pair.append((u.to(dev), su, bb.to(dev)))
                    self.wino.append(tuple(pair))
                self.buf = [torch.zeros((self.max_batch, 81, 128), dtype=torch.float32, device=dev) for _ in range(3)]
                # per-forward maxima: slot 0 bounds the stem output (inputs are 0/1 planes:
                # relu(b + sum of the positive weight rows)), slot i+1 = max of conv i's output.
                # Forwards take fresh slots from a ring that is zeroed once per AMAX_RING
                # forwards: a per-forward fill kernel would wait for a free CU behind the
                # other lanes' persistent convolutions.
                nconv = 2 * len(self.wino)
                self.amax_stride = nconv + 1
                self.amax = torch.zeros(self.AMAX_RING * self.amax_stride, dtype=torch.float32, device=dev)
                self.stem_bound = float(torch.relu(self.stem_b.double().cpu() +
                                                   self.stem_w.double().cpu().clamp_min(0).sum(0)).max())
                self.amax[::self.amax_stride] = self.stem_bound
                self.amax = self.amax.view(torch.int32)
                self.amax_pos = 0
            elif conv in ("wino", "wino3"):
                wfn = wino3_weights if conv == "wino3" else wino_weights
                self.conv_fn = self.lib.uttt_nn_conv3x3_wino3 if conv == "wino3" else self.lib.uttt_nn_conv3x3_wino
                self.wino = []
                for b in net.residual_blocks:
                    pair = []
                    for cv, bn in ((b.conv1, b.bn1), (b.conv2, b.bn2)):
                        w, bb = fold_bn(cv, bn)
                        pair += [wfn(w).to(dev), bb.to(dev)]
                    self.wino.append(tuple(pair))
                self.buf = [torch.zeros((self.max_batch, 81, 128), dtype=torch.float32, device=dev) for _ in range(3)]
        self.act = torch.zeros((self.max_batch, 9, 9, 128), dtype=torch.float32, device=dev)
        self.policy = torch.zeros((self.max_batch, 81), dtype=torch.float32, device=dev)
        self.value = torch.zeros((self.max_batch,), dtype=torch.float32, device=dev)

    def _epilogue(self, x, bias, res, out, stream):
        check(self.lib.uttt_nn_epilogue(_p(x), _p(bias), _p(res) if res is not None else None, _p(out),
                                        x.numel() // 128, 128, ctypes.c_void_p(stream)))

    @torch.no_grad()
    def forward(self, n, softmax=True):
        """Evaluate the engine's n pending leaves; returns (policy or logits (n,81), value (n,))."""
        if self.conv != "miopen":
            return self._forward_wino(n, softmax)
        stream = torch.cuda.current_stream(self.engine.device).cuda_stream
        nb = _bucket(n, self.max_batch)
        check(self.lib.uttt_nn_stem(self.engine.h, _p(self.stem_w), _p(self.stem_b), _p(self.act)))
        a = self.act[:nb].permute(0, 3, 1, 2)  # NCHW view, channels-last strides
        for w1, b1, w2, b2 in self.blocks:
            y = F.conv2d(a, w1, None, padding=1)
            assert y.is_contiguous(memory_format=torch.channels_last)
            self._epilogue(y, b1, None, y, stream)
            z = F.conv2d(y, w2, None, padding=1)
            self._epilogue(z, b2, a, z, stream)
            a = z
        check(self.lib.uttt_nn_heads(_p(a), _p(self.heads), n, _p(self.policy), _p(self.value),
                                     1 if softmax else 0, ctypes.c_void_p(stream)))
        return self.policy[:n], self.value[:n]

    def _forward_wino(self, n, softmax):
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.engine.device).cuda_stream)
        x, t, y = self.buf
        check(self.lib.uttt_nn_stem(self.engine.h, _p(self.stem_w), _p(self.stem_b), _p(x)))
        if self.conv == "wino3h":
            if self.amax_pos == self.AMAX_RING:
                self.amax.view(torch.float32).zero_()[::self.amax_stride] = self.stem_bound
                self.amax_pos = 0
            base = self.amax.data_ptr() + 4 * self.amax_stride * self.amax_pos
            self.amax_pos += 1
            slot = lambda i: ctypes.c_void_p(base + 4 * i)  # noqa: E731
            fn = self.lib.uttt_nn_conv3x3_wino3h
            for i, ((u1, s1, b1), (u2, s2, b2)) in enumerate(self.wino):
                check(fn(_p(x), _p(u1), ctypes.c_float(s1), _p(b1), None, _p(t), slot(2 * i), slot(2 * i + 1), n,
                         stream))
                check(fn(_p(t), _p(u2), ctypes.c_float(s2), _p(b2), _p(x), _p(y), slot(2 * i + 1), slot(2 * i + 2),
                         n, stream))
                x, y = y, x
            check(self.lib.uttt_nn_heads(_p(x), _p(self.heads), n, _p(self.policy), _p(self.value),
                                         1 if softmax else 0, stream))
            return self.policy[:n], self.value[:n]
        for u1, b1, u2, b2 in self.wino:
            check(self.conv_fn(_p(x), _p(u1), _p(b1), None, _p(t), n, stream))
            check(self.conv_fn(_p(t), _p(u2), _p(b2), _p(x), _p(y), n, stream))
            x, y = y, x
        check(self.lib.uttt_nn_heads(_p(x), _p(self.heads), n, _p(self.policy), _p(self.value),
                                     1 if softmax else 0, stream))
        return self.policy[:n], self.value[:n]

    def __call__(self, x, n):
        return self.forward(n, True)


def wino_weights(w):
    """Folded conv weight (128,128,3,3) -> Winograd U (16,128,128) [xi][ci][co] (host, double precision)."""
    import numpy as np
    wc = np.ascontiguousarray(w.detach().float().cpu().numpy())
    u = np.zeros((16, 128, 128), np.float32)
    lib = _lib.load()
    check(lib.uttt_nn_wino_weights(wc.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                   u.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
    return torch.from_numpy(u)


def wino3_weights(w):
    """Folded conv weight (128,128,3,3) -> Winograd F(3x3,3x3) U, 25*128*128 floats in kernel order (host, double)."""
    import numpy as np
    wc = np.ascontiguousarray(w.detach().float().cpu().numpy())
    u = np.zeros((25, 128, 128), np.float32)
    lib = _lib.load()
    check(lib.uttt_nn_wino3_weights(wc.ctypes.data_as(ctypes.POINTER(ctypes.c_float)),
                                    u.ctypes.data_as(ctypes.POINTER(ctypes.c_float))))
    return torch.from_numpy(u)


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


def amax(x, out=None):
    """max |x| as a (1,) int32 tensor of float bits on x's device (uttt_nn_amax)."""
    if out is None:
        out = torch.zeros(1, dtype=torch.int32, device=x.device)
    check(_lib.load().uttt_nn_amax(_p(x), x.numel(), _p(out), ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    return out


def conv3x3_wino3h(x, u, su, bias, residual=None, y_amax=None):
    """Test/utility wrapper for the split-f16 F(3x3,3x3) kernel: x (n,81,128) f32 cuda ->
    relu(conv3x3(x) + bias (+ residual)); u, su from wino3h_weights()."""
    y = torch.empty_like(x)
    xa = amax(x)
    check(_lib.load().uttt_nn_conv3x3_wino3h(_p(x), _p(u), ctypes.c_float(su), _p(bias),
                                             _p(residual) if residual is not None else None, _p(y), _p(xa),
                                             _p(y_amax) if y_amax is not None else None, x.shape[0],
                                             ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    return y


def conv3x3_wino(x, u, bias, residual=None, f3=False):
    """Test/utility wrapper: x (n,81,128) f32 cuda -> relu(conv3x3(x) + bias (+ residual)).
    f3: u is a wino3_weights() transform (F(3x3,3x3) kernel), else wino_weights() (F(2x2,3x3))."""
    y = torch.empty_like(x)
    lib = _lib.load()
    fn = lib.uttt_nn_conv3x3_wino3 if f3 else lib.uttt_nn_conv3x3_wino
    check(fn(_p(x), _p(u), _p(bias), _p(residual) if residual is not None else None, _p(y),
             x.shape[0], ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)))
    return y
