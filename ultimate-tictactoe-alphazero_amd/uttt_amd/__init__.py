"""uttt_amd — MI355X-native batched PV-MCTS self-play for Ultimate Tic-Tac-Toe.

Layout of the package directory (ultimate-tictactoe-alphazero_amd/):
  csrc/               HIP kernels (engine.hip), host rules (rules_api.cpp),
                      shared bitboards (uttt_bits.h), pybind11 module source
  libuttt_engine.so   the C ABI of include/uttt_engine.h (built in-tree)
  uttt_cpp*.so        drop-in for the reference's `uttt_cpp` module
  pv_mcts_cpp.py, self_play_cpp.py   drop-in mirrors of the reference drivers
  uttt_amd/           this package: engine handle, network, batched drivers
"""
import os
import sys

PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if PKG_ROOT not in sys.path:  # makes `import uttt_cpp` resolve to the in-tree module
    sys.path.insert(0, PKG_ROOT)

from .engine import Engine, as_states, initial_states  # noqa: E402
from .selfplay import (BatchedSearch, HashEvaluator, NetworkEvaluator, SelfPlay,  # noqa: E402
                       history_from_records)

__all__ = ["Engine", "as_states", "initial_states", "BatchedSearch", "SelfPlay", "HashEvaluator",
           "NetworkEvaluator", "history_from_records", "PKG_ROOT"]
