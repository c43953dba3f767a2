#!/bin/bash
# round 6 (e): the dense-ref forward's 16-row remainder tiles (B = 5000): parity + A/B timing
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06e
B="python bench.py --steps 20 --warmup 5 --step-steps 0 --rollout-k-extra '' --large-n '' --hbm-ring-launches 0 --train dense@5000,dense --train-updates 100 --no-cpu-baseline"
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_dense_gpu.py tests/test_learner_gpu.py -k "dense" > gpurun_out/r06e/tests.log 2>&1 \
&& timeout -k 10 300 bash -c "G2048_DENSE_FWD_ONE_TILE=1 $B" > gpurun_out/r06e/old.json 2> gpurun_out/r06e/old.err \
&& timeout -k 10 300 bash -c "$B" > gpurun_out/r06e/new.json 2> gpurun_out/r06e/new.err
rc=$?
tail -3 gpurun_out/r06e/tests.log
python - <<'PY'
import json
for f in ("old", "new"):
    try:
        d = json.load(open(f"gpurun_out/r06e/{f}.json"))
        for k, v in d["learner"].items():
            print(f, k, round(v["update_ms"] * 1e3, 1), "us", round(v["flop_frac"], 3))
    except Exception as e:
        print(f, "no line", e)
PY
exit $rc
