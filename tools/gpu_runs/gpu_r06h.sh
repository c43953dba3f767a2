#!/bin/bash
# round 6 (h): the float64 conv update's weight gradients as K = B GEMMs (k_conv64_wgrad) --
# parity (reference fixtures, torch path, GEMM vs slabs, guard regions) and timing vs the slabs
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06h
timeout -k 10 900 python -u -m pytest -x -q --timeout 600 --timeout-method thread \
  tests/test_learner_gpu.py -k "conv64 or f64 or conv" > gpurun_out/r06h/tests.log 2>&1
rc=$?
tail -5 gpurun_out/r06h/tests.log
[ $rc -eq 0 ] || exit $rc
G2048_CONV64_WGRAD=gemm timeout -k 10 300 python tools/learner_ab.py "" conv > gpurun_out/r06h/gemm.txt 2>&1 && \
G2048_CONV64_WGRAD=slab timeout -k 10 300 python tools/learner_ab.py "" conv > gpurun_out/r06h/slab.txt 2>&1
rc=$?
grep -h "us/update" gpurun_out/r06h/gemm.txt gpurun_out/r06h/slab.txt
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" && \
G2048_CONV64_WGRAD=gemm timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r06h/prof -o run -- python tools/learner_ab.py "" conv > gpurun_out/r06h/prof.log 2>&1
rc=$?
f=$(ls gpurun_out/r06h/prof/*/run_kernel_stats.csv 2>/dev/null | head -1)
[ -n "$f" ] && grep -E "conv64" "$f" | cut -c1-200
exit $rc
