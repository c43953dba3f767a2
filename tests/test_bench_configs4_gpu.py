"""BASELINE configs[4] as a workload: 512k boards sharded 8 ways, conv Double
DQN with the gradient all-reduce, run through bench.py itself -- the driver's 8-GPU SCALE leg.
Here on ONE GPU: 8 ranks (processes) share it over gloo collectives (RCCL refuses two ranks on one
device), each with 65 536 boards, a 1M-row ring and the fused conv learner in fp64 and fp32.
Checked: the JSON line's world size and global boards, the fused path, and that all 8 replicas'
online and target weights are bitwise equal after the timed updates (bench.py all-gathers them).
Reference semantics: src/dqn_lib.py:119-164 (train_step), :227-228 (target sync)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(900)
def test_bench_configs4_eight_ranks_on_one_gpu():
    env = dict(os.environ, G2048_BENCH_BACKEND="gloo", PYTHONUNBUFFERED="1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--boards", "65536",
           "--train", "conv", "--train-dtypes", "fp64,fp32", "--train-updates", "10",
           "--step-steps", "0", "--steps", "20", "--warmup", "5", "--rollout-k-extra", "",
           "--large-n", "", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=900)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 8
    assert rec["config"]["global_boards"] == 8 * 65536 == 524288
    assert rec["value"] > 0 and rec["scaling"] == "weak"
    # the ranks' global board ranges tile [0, 8 * 65536) without overlap: board g owns Philox
    # subsequence g, so no two ranks share one
    ranges = sorted(tuple(r) for r in rec["config"]["rank_boards"])
    assert len(ranges) == 8 and all(n == 65536 for _, n in ranges)
    assert [o for o, _ in ranges] == [r * 65536 for r in range(8)]
    for dt in ("fp64", "fp32"):
        L = rec["learner"][f"conv.{dt}"]
        assert L["path"] == "fused HIP kernels", L
        assert L["ranks_lockstep"] is True, dt
        assert L["batch"] == 8192 and L["replay"] == (1 << 20) // 65536 * 65536
        assert L["updates_per_s"] > 0
