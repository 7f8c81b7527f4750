"""Drop-in for the reference's train_network.py (same names and constants):
load the newest ./data/*.history, train ./model/best.pth for RN_EPOCHS epochs
(batch 128, Adam 1e-3, LambdaLR), save ./model/latest.pth. Run directly it
trains on one GPU; under `torchrun --nproc-per-node N` (backend nccl = RCCL) it
trains data-parallel over N GPUs with the same global batch (uttt_amd.train:
eager DDP with SyncBatchNorm, the reference's batch-128 statistics, by default;
UTTT_TRAIN_DP=flat for two captured graphs per rank around one flat gradient
all-reduce, with per-rank BatchNorm statistics).
The dataset is resident in HBM; no DataLoader workers.
"""
import os
import pickle
import sys
import time
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from uttt_amd import train as _train  # noqa: E402
from uttt_amd.model import DN_INPUT_SHAPE, DualNetwork  # noqa: E402,F401

RN_EPOCHS = _train.RN_EPOCHS
BATCH_SIZE = _train.BATCH_SIZE
NUM_WORKERS = 0

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


def load_data():
    history_path = sorted(Path("./data").glob("*.history"))[-1]
    with history_path.open(mode="rb") as f:
        return pickle.load(f)  # the file this pipeline wrote (self_play*.write_data)


class HistoryDataset(torch.utils.data.Dataset):
    def __init__(self, xs, y_policies, y_values):
        self.xs = np.transpose(xs, (0, 3, 1, 2)).astype(np.float32)
        self.y_policies = y_policies.astype(np.float32)
        self.y_values = y_values.astype(np.float32).reshape(-1, 1)

    def __len__(self):
        return len(self.xs)

    def __getitem__(self, idx):
        return self.xs[idx], self.y_policies[idx], self.y_values[idx]


# wall-clock seconds of the last train_network() call's phases (tools/bench_cycle.py)
LAST_TIMINGS = {}


def train_network():
    distributed = int(os.environ.get("WORLD_SIZE", "1")) > 1
    if distributed and not dist.is_initialized():
        from uttt_amd.distributed import init_from_env
        init_from_env()  # RCCL, one rank per GPU (gloo where ranks share a GPU)
    dev = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu")
    LAST_TIMINGS.clear()
    t0 = time.perf_counter()
    history = load_data()
    t1 = time.perf_counter()
    model = DualNetwork().to(dev)
    model.load_state_dict(torch.load("./model/best.pth", map_location=dev, weights_only=True))
    losses = _train.train_network(model, history, RN_EPOCHS, BATCH_SIZE, dev)
    if dev.type == "cuda":
        torch.cuda.synchronize(dev)
    t2 = time.perf_counter()
    if not distributed or dist.get_rank() == 0:
        torch.save(model.state_dict(), "./model/latest.pth")
        print("Model saved to ./model/latest.pth")
    LAST_TIMINGS.update(load_s=t1 - t0, train_s=t2 - t1, save_s=time.perf_counter() - t2, samples=len(history),
                        epochs=RN_EPOCHS, first_loss=losses[0] if losses else None,
                        last_loss=losses[-1] if losses else None)
    del model


if __name__ == "__main__":
    train_network()
