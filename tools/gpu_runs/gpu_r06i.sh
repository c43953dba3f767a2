#!/bin/bash
# round 6 (i): kernel-trace summary of the float64 conv update in GEMM (GW) and slab modes
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06i
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
G2048_CONV64_WGRAD=gemm timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06i/gemm -o run -- python tools/learner_ab.py "" conv > gpurun_out/r06i/gemm.log 2>&1 && \
G2048_CONV64_WGRAD=slab timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06i/slab -o run -- python tools/learner_ab.py "" conv > gpurun_out/r06i/slab.log 2>&1
rc=$?
for m in gemm slab; do
  f=$(ls gpurun_out/r06i/$m/*/run_kernel_stats.csv gpurun_out/r06i/$m/run_kernel_stats.csv 2>/dev/null | head -1)
  echo "== $m $f"
  [ -n "$f" ] && grep -E "conv64|Name" "$f" | cut -c1-160
done
exit $rc
