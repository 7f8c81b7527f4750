"""Host sanitizer run: the product's rules (csrc/rules_api.cpp) and the
oracle (oracle/uttt_oracle.c) built with AddressSanitizer + UBSan and played against
each other over 3,000 random games (tests/asan/rules_asan.cpp). CPU only."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))


@pytest.mark.skipif(shutil.which("g++") is None or shutil.which("make") is None, reason="needs g++ and make")
def test_rules_and_oracle_under_asan_ubsan(tmp_path):
    r = subprocess.run(["make", "-C", os.path.join(HERE, "asan"), f"OUT={tmp_path}"], capture_output=True, text=True,
                       timeout=600)
    out = r.stdout + r.stderr
    assert r.returncode == 0, out[-4000:]
    assert "0 failures" in out and "ERROR: AddressSanitizer" not in out and "runtime error" not in out, out[-4000:]
