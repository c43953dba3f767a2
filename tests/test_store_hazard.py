"""The compiled kernels leave two wait states between every store of more than 8 bytes and a VALU
rewrite of its data registers (tools/store_hazard_audit.py).  Without them gfx950 stored boards
whose first word was already overwritten by the next instruction (k_rollout_lean at 1M+ boards,
under store-queue back-pressure; tests/test_fullsize_gpu.py::test_rollout_large_n_vs_oracle).
CPU-only: hipcc cross-compiles the library's HIP sources to gfx950 assembly."""
import os
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "reinforcement-learning-2048_amd", "csrc")
sys.path.insert(0, os.path.join(ROOT, "tools"))


@pytest.mark.skipif(shutil.which("hipcc") is None, reason="hipcc not in this image")
@pytest.mark.timeout(900)
def test_no_store_data_hazard(tmp_path):
    import store_hazard_audit

    out = []
    for f in sorted(os.listdir(CSRC)):
        if not f.endswith(".hip"):
            continue
        s = str(tmp_path / (f + ".s"))
        subprocess.run(["hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only",
                        "-S", os.path.join(CSRC, f), "-o", s], check=True, capture_output=True)
        out.append(s)
    assert sum(store_hazard_audit.audit(s) for s in out) == 0
