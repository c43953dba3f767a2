#!/bin/bash
# round 6 (a): RCCL capture mode + bench RCCL branch (world-1 group), scaled Adam, round-4 dense
# resume, one-launch dense-64 update (bitwise vs two launches, A/B timing).  Run while the
# one-launch form was the default and G2048_DENSE64_TWO_LAUNCH=1 selected the two launches (since
# reversed: G2048_DENSE64_ONE_LAUNCH=1 selects the one-launch form)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
B="python bench.py --steps 20 --warmup 5 --step-steps 0 --rollout-k-extra '' --large-n '' --hbm-ring-launches 0 --train dense64 --train-updates 400 --no-cpu-baseline"
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_qnet_gpu.py -k "dense64" tests/test_adam_scaled_gpu.py \
  tests/test_train_gpu.py::test_resume_round4_dense_checkpoint > gpurun_out/r06a_1.log 2>&1 \
&& timeout -k 10 300 bash -c "G2048_DENSE64_TWO_LAUNCH=1 $B" > gpurun_out/r06a_two.json 2> gpurun_out/r06a_two.err \
&& timeout -k 10 300 bash -c "$B" > gpurun_out/r06a_one.json 2> gpurun_out/r06a_one.err \
&& timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread \
  tests/test_bench_rccl_gpu.py tests/test_dist_gpu.py tests/test_learner_gpu.py -k "dense64 or rccl or lockstep or graphed_dp or bench" > gpurun_out/r06a_2.log 2>&1
rc=$?
tail -5 gpurun_out/r06a_1.log; tail -25 gpurun_out/r06a_2.log
python - <<'PY'
import json
for f in ("two", "one"):
    try:
        d = json.load(open(f"gpurun_out/r06a_{f}.json"))
        for k, v in d["learner"].items():
            print(f, k, round(v["update_ms"] * 1e3, 2), "us", round(v["updates_per_s"]), "upd/s")
    except Exception as e:
        print(f, "no line", e)
PY
exit $rc
