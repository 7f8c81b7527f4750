"""Launched by tests/test_dropins_gpu.py under torch.distributed.run (not a test module):
self_play_cpp.self_play() with the hash model on WORLD_SIZE ranks that share the box's GPU(s),
gloo for the gather; rank 0 writes the .history into argv[1]."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ultimate-tictactoe-alphazero_amd")]

import self_play_cpp  # noqa: E402
from oracle.hashnp import make_hash_model  # noqa: E402

if __name__ == "__main__":
    out_dir, n_games, seed = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    path = self_play_cpp.self_play(n_games=n_games, seed_base=seed, model=make_hash_model(), out_dir=out_dir,
                                   slots=5)
    if path:
        print("HISTORY", path, flush=True)
