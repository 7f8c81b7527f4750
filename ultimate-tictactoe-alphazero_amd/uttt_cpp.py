"""`uttt_cpp` — drop-in for the reference's pybind11 module (cpp/python_bindings.cpp:49-107).

The compiled module is `_uttt_cpp` (csrc/uttt_cpp_module.cpp over the C ABI in
include/uttt_engine.h). torch is imported first so that the engine binds the
same HIP runtime (libamdhip64.so.7) torch uses: engine launches then share
torch's streams and device pointers.
"""
import torch  # noqa: F401  (must precede _uttt_cpp: one HIP runtime per process)

from _uttt_cpp import InferenceResult, State, boltzman, pv_mcts_scores  # noqa: E402,F401
from _uttt_cpp import __version__, backend  # noqa: E402,F401

__all__ = ["State", "InferenceResult", "pv_mcts_scores", "boltzman"]
