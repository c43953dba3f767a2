#!/bin/bash
# round 6 (l): k_conv64_wgrad's time without its GEMM MFMAs / without its staging (timing-only
# variant libraries from tools/conv64_wgrad_probe.sh) against the library
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06l
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for v in lib:"" nogemm:tools/variants/libg2048_wg_nogemm.so noput:tools/variants/libg2048_wg_noput.so; do
  n=${v%%:*}; f=${v#*:}
  G2048_CONV64_WGRAD=gemm timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r06l/$n -o run -- python tools/learner_ab.py "$f" conv > gpurun_out/r06l/$n.log 2>&1 || exit 1
  echo "== $n"; grep -h "float64" gpurun_out/r06l/$n.log
  grep -E "conv64" gpurun_out/r06l/$n/run_kernel_stats.csv | awk -F, '{print $1, $4}' | cut -c1-160
done
