"""The plain-C ABI client (examples/abi_demo.c, built by __graft_entry__.build()) run on the GPU:
a caller that binds the C ABI the way a cgo / JNI / N-API host would, with no Python in the
loop.  Its final boards and meta must equal the CPU oracle's after the same random-policy steps
+ rollout (src/board.py / src/dqn_lib.py:91-107 restated in oracle/oracle2048.c)."""
import os
import subprocess

import numpy as np
import pytest

from oracle import oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
DEMO = os.path.join(ROOT, "examples", "abi_demo")


@pytest.mark.gpu
def test_c_client_matches_oracle(tmp_path):
    if not os.path.exists(DEMO):
        pytest.fail("examples/abi_demo is not built: run __graft_entry__.build()")
    n, steps, k = 3000, 5, 11
    out = tmp_path / "boards.bin"
    res = subprocess.run([DEMO, str(n), str(steps), str(k), str(out)], capture_output=True,
                         text=True, timeout=120)
    assert res.returncode == 0, res.stderr
    assert "0 input errors" in res.stdout
    raw = np.fromfile(out, np.uint8)
    board = raw[:16 * n].reshape(n, 16)
    meta = raw[16 * n:].view(np.uint32).reshape(n, 2)
    ref = O.OracleEnv(n, seed=0x2048)
    for _ in range(steps + k):
        ref.step(O.MODE_RANDOM)
    assert np.array_equal(board, ref.board)
    assert np.array_equal(meta, ref.meta)
