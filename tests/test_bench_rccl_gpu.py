"""bench.py's RCCL branch on the one-GPU box: G2048_BENCH_DIST=1 builds a
one-rank RCCL process group (plus the gloo side group), so the paths the driver's multi-GPU run
takes execute once before it -- the RCCL barrier and max-over-ranks around every timed region,
thread-local hipGraph captures next to ProcessGroupNCCL's watchdog, the learner's data-parallel
update with the SUM all-reduce captured in its graph and 1 / world in Adam, the fixed-count settle,
the GPU all_gather of the lockstep check and the side-group agreement after each learner leg.
No sleep guards a capture (g2048/dist.py: capture_error_mode)."""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.timeout(600)
def test_bench_rccl_world1():
    env = dict(os.environ, G2048_BENCH_DIST="1", PYTHONUNBUFFERED="1")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "20", "--warmup", "5",
           "--step-steps", "200", "--rollout-k-extra", "", "--large-n", "",
           "--hbm-ring-launches", "0", "--train", "conv,dense64,dense@512",
           "--train-dtypes", "fp32,fp64", "--train-updates", "20", "--no-cpu-baseline"]
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [x for x in out.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, out.stdout[-2000:]
    rec = json.loads(lines[0])
    assert rec["dist"] == {"process_group": True, "backend": "nccl",
                           "capture_error_mode": "thread_local"}
    assert rec["n_gpus"] == 1 and rec["value"] > 0 and rec["step_kernel"]["env_steps_per_s"] > 0
    for leg in ("conv.fp32", "conv.fp64", "dense64.fp32", "dense64.fp64", "dense@512.fp32",
                "dense@512.fp64"):
        L = rec["learner"][leg]
        assert "error" not in L, (leg, L)
        assert L["path"] == "fused HIP kernels", leg
        assert L["data_parallel"] is True and L["captured_allreduce"] is True, leg
        assert L["ranks_lockstep"] is True, leg
        assert L["updates_per_s"] > 0 and L["loop_iter_ms"] > 0, leg
    assert "Traceback" not in out.stderr, out.stderr[-3000:]
