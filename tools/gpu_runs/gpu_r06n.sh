#!/bin/bash
# round 6 (n): HBM bytes of the GEMM-form conv64 kernels (FETCH / WRITE passes)
set -o pipefail
mkdir -p gpurun_out/r06n
bash tools/gpu_pmc_learner.sh conv:fp64:8192 > gpurun_out/r06n/pmc.log 2>&1 || { tail -20 gpurun_out/r06n/pmc.log; exit 1; }
cp gpurun_out/pmc_learner.json gpurun_out/r06n/pmc_learner.json
python - <<'PY'
import json
d = json.load(open("gpurun_out/r06n/pmc_learner.json"))
for k, v in d.items():
    if k.startswith("_"): continue
    c = v.get("counters", {})
    print(k, {x: v.get(x) for x in ("traffic", "mfma_busy_frac")}, {x: c.get(x) for x in ("FETCH_SIZE", "WRITE_SIZE")})
PY
