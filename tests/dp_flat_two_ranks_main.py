"""Launched by tests/test_dropins_gpu.py under torch.distributed.run with 2 ranks sharing the box's GPU
(gloo, as uttt_amd.distributed.init_from_env picks when ranks outnumber GPUs; not a test module):
train_network's default GPU data-parallel form (UTTT_TRAIN_DP=flat: train.DPGraphedStep, two captured
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
    torch.distributed.barrier()
    torch.distributed.destroy_process_group()
    print("DP-FLAT-OK", rank, losses, flush=True)
