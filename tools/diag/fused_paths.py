"""Diagnostic: fused evaluator wino vs miopen vs CPU on real pending leaves."""
import sys, random
import numpy as np
import torch
sys.path[:0] = ['.', 'ultimate-tictactoe-alphazero_amd', 'tests']
import uttt_amd
from uttt_amd.model import policy_logits, random_network
from uttt_amd.nnfast import FusedNetworkEvaluator
from oracle import core
from test_engine_gpu import _random_positions

roots, _ = _random_positions(core, 300, seed=13)
net = random_network(0, "cuda")
cpu = random_network(0)
bs = uttt_amd.BatchedSearch(len(roots), 50)
fw = FusedNetworkEvaluator(net, bs.engine, conv="wino")
fm = FusedNetworkEvaluator(net, bs.engine, conv="miopen")
e = bs.engine
e.use_stream()
e.search_begin(roots, 50, 8)
for rnd in range(3):
    n = e.select(bs.x)
    zw, vw = [t.clone() for t in fw.forward(n, softmax=False)]
    zm, vm = [t.clone() for t in fm.forward(n, softmax=False)]
    zc, vc = policy_logits(cpu, bs.x[:n].cpu())
    vc = vc.reshape(-1)
    for name, z, v in (("wino", zw, vw), ("miopen", zm, vm)):
        dv = (v.cpu() - vc).abs()
        dz = ((z.cpu() - zc).abs() / zc.abs().amax(1, keepdim=True).clamp_min(1)).amax(1)
        bad = (dv > 1e-5).nonzero().flatten().tolist()
        print(f"round {rnd} n={n} {name}: max dv {dv.max().item():.3e} max dz {dz.max().item():.3e} bad rows {bad[:20]} (#{len(bad)})", flush=True)
        if bad:
            i = bad[0]
            print("   v", v[i].item(), "cpu", vc[i].item(), "logits", z[i, :5].tolist(), zc[i, :5].tolist())
    # also: value pre-activations from the acts? print wino vs miopen final activation diff
    xw = fw.buf[0]  # not necessarily final; skip
    p, v2 = fm.forward(n, softmax=True)
    e.apply(p, v2)
