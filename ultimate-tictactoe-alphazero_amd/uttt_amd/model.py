"""The leaf evaluator: the reference's ResNet dual head (dual_network.py:28-121),
kept in PyTorch-ROCm as the north star asks, plus the glue that feeds it the
engine's NCHW leaf batches.

``DualNetwork`` has the reference's parameter names (so ``./model/best.pth``
state dicts load unchanged) and builds its layers in the reference's order, so
``torch.manual_seed(s); DualNetwork()`` draws the same random weights
(checked against tests/golden/network.npz).
"""
import torch
import torch.nn as nn
import torch.nn.functional as F

DN_FILTERS = 128
DN_RESIDUAL_NUM = 16
DN_INPUT_SHAPE = (9, 9, 3)
DN_OUTPUT_SIZE = 81


class ResidualBlock(nn.Module):
    def __init__(self, filters):
        super().__init__()
        self.conv1 = nn.Conv2d(filters, filters, 3, padding=1, bias=False)
        self.bn1 = nn.BatchNorm2d(filters)
        self.conv2 = nn.Conv2d(filters, filters, 3, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(filters)

    def forward(self, x):
        y = F.relu(self.bn1(self.conv1(x)))
        return F.relu(self.bn2(self.conv2(y)) + x)


class DualNetwork(nn.Module):
    """(N,3,9,9) -> (softmax policy (N,81), tanh value (N,1))."""

    def __init__(self, input_shape=DN_INPUT_SHAPE, filters=DN_FILTERS, residual_num=DN_RESIDUAL_NUM,
                 output_size=DN_OUTPUT_SIZE):
        super().__init__()
        cin = input_shape[2]
        self.conv_input = nn.Conv2d(cin, filters, 3, padding=1, bias=False)
        self.bn_input = nn.BatchNorm2d(filters)
        self.residual_blocks = nn.ModuleList(ResidualBlock(filters) for _ in range(residual_num))
        self.policy_conv = nn.Conv2d(filters, 2, 1, bias=False)
        self.policy_bn = nn.BatchNorm2d(2)
        self.policy_fc = nn.Linear(2 * 81, output_size)
        self.value_conv = nn.Conv2d(filters, 1, 1, bias=False)
        self.value_bn = nn.BatchNorm2d(1)
        self.value_fc1 = nn.Linear(81, 256)
        self.value_fc2 = nn.Linear(256, 1)
        for m in self.modules():  # same re-initialisation pass, same module order
            if isinstance(m, (nn.Conv2d, nn.Linear)):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.constant_(m.weight, 1)
                nn.init.constant_(m.bias, 0)

    def forward(self, x):
        x = F.relu(self.bn_input(self.conv_input(x)))
        for blk in self.residual_blocks:
            x = blk(x)
        p = F.relu(self.policy_bn(self.policy_conv(x)))
        p = F.softmax(self.policy_fc(torch.flatten(p, 1)), dim=1)
        v = F.relu(self.value_bn(self.value_conv(x)))
        v = torch.tanh(self.value_fc2(F.relu(self.value_fc1(torch.flatten(v, 1)))))
        return p, v


def fold_bn(conv, bn):
    """Eval-mode conv+BN -> (weight, bias) of one conv (exact algebra, f32 rounding)."""
    scale = bn.weight / torch.sqrt(bn.running_var + bn.eps)
    w = conv.weight * scale.reshape(-1, 1, 1, 1)
    b = bn.bias - bn.running_mean * scale
    return w.detach().contiguous(), b.detach().contiguous()


class FoldedDualNetwork(nn.Module):
    """Inference form of a DualNetwork: BN folded into the convolutions,
    channels-last activations (MIOpen NHWC kernels). Same function; f32
    rounding differs from the unfolded net at the 1e-6 level."""

    def __init__(self, net):
        super().__init__()
        net = net.eval()
        self.stem = fold_bn(net.conv_input, net.bn_input)
        self.blocks = [(fold_bn(b.conv1, b.bn1), fold_bn(b.conv2, b.bn2)) for b in net.residual_blocks]
        self.pconv = fold_bn(net.policy_conv, net.policy_bn)
        self.vconv = fold_bn(net.value_conv, net.value_bn)
        self.pfc = (net.policy_fc.weight.detach(), net.policy_fc.bias.detach())
        self.vfc1 = (net.value_fc1.weight.detach(), net.value_fc1.bias.detach())
        self.vfc2 = (net.value_fc2.weight.detach(), net.value_fc2.bias.detach())
        self.channels_last = True
        self._to_cl()

    def _to_cl(self):
        cl = torch.channels_last
        self.stem = (self.stem[0].contiguous(memory_format=cl), self.stem[1])
        self.blocks = [((a[0].contiguous(memory_format=cl), a[1]), (b[0].contiguous(memory_format=cl), b[1]))
                       for a, b in self.blocks]

    def to(self, *args, **kw):
        mv = lambda t: t.to(*args, **kw)  # noqa: E731
        self.stem = tuple(map(mv, self.stem))
        self.blocks = [(tuple(map(mv, a)), tuple(map(mv, b))) for a, b in self.blocks]
        for n in ("pconv", "vconv", "pfc", "vfc1", "vfc2"):
            setattr(self, n, tuple(map(mv, getattr(self, n))))
        self._to_cl()
        return self

    @torch.no_grad()
    def forward(self, x):
        logits, v = self.forward_logits(x)
        return F.softmax(logits, dim=1), v

    @torch.no_grad()
    def forward_logits(self, x):
        x = x.contiguous(memory_format=torch.channels_last)
        x = F.relu(F.conv2d(x, self.stem[0], self.stem[1], padding=1))
        for (w1, b1), (w2, b2) in self.blocks:
            y = F.relu(F.conv2d(x, w1, b1, padding=1))
            x = F.relu(F.conv2d(y, w2, b2, padding=1) + x)
        p = F.relu(F.conv2d(x, self.pconv[0], self.pconv[1]))
        p = torch.flatten(p.contiguous(), 1)
        logits = F.linear(p, *self.pfc)
        v = F.relu(F.conv2d(x, self.vconv[0], self.vconv[1]))
        v = torch.flatten(v.contiguous(), 1)
        v = torch.tanh(F.linear(F.relu(F.linear(v, *self.vfc1)), *self.vfc2))
        return logits, v


def policy_logits(net, x):
    """(pre-softmax policy logits, value) of a DualNetwork (hook on policy_fc)."""
    if hasattr(net, "forward_logits"):
        return net.forward_logits(x)
    box = {}
    h = net.policy_fc.register_forward_hook(lambda m, i, o: box.setdefault("z", o))
    try:
        with torch.no_grad():
            _, v = net(x)
    finally:
        h.remove()
    return box["z"], v


def random_network(seed=0, device="cpu"):
    torch.manual_seed(seed)
    return DualNetwork().to(device).eval()


def calibrated_network(npz_path, device="cpu"):
    """The non-saturated test/bench network of tests/golden/netcal.npz: the seed-0 DualNetwork
    (as the reference initialises it) with the fixture's calibrated BatchNorm running statistics
    and value_fc2.weight scaled by the fixture's power of two (tests/golden/make_golden.py
    gen_netcal). Its outputs are O(1) values and spread policies, so network parity is not
    hidden behind tanh/softmax saturation."""
    import numpy as np
    with np.load(npz_path) as z:
        names = [str(s) for s in z["bn_names"]]
        mean, var, sizes = z["bn_mean"], z["bn_var"], z["bn_sizes"]
        scale = float(z["vfc2_scale"])
    torch.manual_seed(0)
    net = DualNetwork()
    mods = dict(net.named_modules())
    o = 0
    with torch.no_grad():
        for name, k in zip(names, sizes.tolist()):
            bn = mods[name]
            bn.running_mean.copy_(torch.from_numpy(mean[o:o + k]))
            bn.running_var.copy_(torch.from_numpy(var[o:o + k]))
            o += k
        net.value_fc2.weight.mul_(scale)
    return net.to(device).eval()
