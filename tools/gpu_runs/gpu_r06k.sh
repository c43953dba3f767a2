#!/bin/bash
# round 6 (k): wait split and MFMA busy of the GEMM-form conv64 kernels
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06k
bash tools/gpu_pmc_waits.sh conv:fp64:8192 || exit 1
cp gpurun_out/pmc_waits.json gpurun_out/r06k/pmc_waits.json
export TMPDIR=/tmp
d=/tmp/pmcm
timeout -s KILL 180 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F64 SQ_BUSY_CYCLES --kernel-trace --output-format csv -d $d -o m \
   -- python tools/prof_learner.py conv fp64 10 8192 > gpurun_out/r06k/mfma.log 2>&1 || exit 1
python tools/pmc_learner.py gpurun_out/r06k/pmc_mfma.json $d:conv.fp64@8192 > /dev/null
python - <<'PY'
import json
for f in ("gpurun_out/r06k/pmc_waits.json", "gpurun_out/r06k/pmc_mfma.json"):
    d = json.load(open(f))
    print(json.dumps(d)[:3000])
PY
