#!/bin/bash
# round 6 (r): the start row prefetched with the board in k_step / the dense-64 fused steps --
# env GPU tests, then the default bench line
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06r
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_env_gpu.py tests/test_boundary_gpu.py tests/test_abi_gpu.py tests/test_fullsize_gpu.py tests/test_player_gpu.py > gpurun_out/r06r/tests.log 2>&1
rc=$?
tail -2 gpurun_out/r06r/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --train "" > gpurun_out/r06r/bench.json 2> gpurun_out/r06r/bench.err || { tail -20 gpurun_out/r06r/bench.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06r/bench.json").read().strip().splitlines()[-1])
print(round(d["value"] / 1e9, 1), "G", round(d["roofline"]["frac"], 3), "step", round(d["step_kernel"]["launch_us_graph"], 2), "floor", round(d["step_kernel"]["launch_floor_us"], 2))
PY
