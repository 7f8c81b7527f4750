"""Drop-in for the reference's dual_network.py: the same DualNetwork (parameter names, layer
order, seed-for-seed initialisation: uttt_amd.model), constants, device, and dual_network()
which writes ./model/best.pth once (dual_network.py:125-135). Leaf evaluation of this network
inside the self-play / arena drop-ins runs on the fused HIP kernels (uttt_amd.nnfast)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from uttt_amd.model import (DN_FILTERS, DN_INPUT_SHAPE, DN_OUTPUT_SIZE, DN_RESIDUAL_NUM,  # noqa: E402,F401
                            DualNetwork, ResidualBlock)

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")


def dual_network():
    if os.path.exists("./model/best.pth"):
        return
    model = DualNetwork().to(device)
    os.makedirs("./model/", exist_ok=True)
    torch.save(model.state_dict(), "./model/best.pth")
    print("Model saved to './model/best.pth'")


if __name__ == "__main__":
    dual_network()
