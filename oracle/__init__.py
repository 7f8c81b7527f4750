"""TEST INFRASTRUCTURE ONLY — the parity checker for the MI355X self-play engine.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package. The product (ultimate-tictactoe-alphazero_amd/) never does.

* :mod:`oracle.core`  — ctypes wrapper over ``liboracle.so`` (plain-C restatement
  of cpp/uttt_game.cpp, cpp/uttt_mcts.cpp and the self_play_cpp.py arithmetic).
* :mod:`oracle.hashnp` — numpy twin of the deterministic hash evaluator, used to
  drive the reference Python self-play when generating fixtures.
* :mod:`oracle.ref`   — ctypes wrapper over ``_ref/libuttt_ref.so`` (the
  reference's own C++ compiled from its sources by oracle/Makefile).
"""
import os
import subprocess

ORACLE_DIR = os.path.dirname(os.path.abspath(__file__))


def build(quiet=True):
    """Compile liboracle.so (and _ref/ when the reference checkout is present)."""
    out = subprocess.run(["make", "-C", ORACLE_DIR, "all"], capture_output=True, text=True)
    if out.returncode != 0:
        raise RuntimeError("oracle build failed:\n" + out.stdout + out.stderr)
    if not quiet:
        print(out.stdout)
