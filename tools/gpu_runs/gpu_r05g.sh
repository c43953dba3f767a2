#!/bin/bash
# GPU box: dense-ref update tuning (weight-gradient splits; f32 targets on 32-row tiles), the
# graph-hazard tests in their final form, the DP/RCCL tests
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_dense_gpu.py -x -q -m gpu --timeout 300 --timeout-method thread -k "fused" > gpurun_out/dense_tests2.log 2>&1; echo "dense rc=$?"; tail -2 gpurun_out/dense_tests2.log
timeout -k 10 300 python -u tools/dense_nsplit.py > gpurun_out/dense_nsplit.txt 2>&1; echo "nsplit rc=$?"; cat gpurun_out/dense_nsplit.txt | grep -v amdgpu.ids
timeout -k 10 900 python -u -m pytest tests/test_graph_hazards_gpu.py -v -m gpu --timeout 300 --timeout-method thread -k "not dim0_sum" > gpurun_out/hazards3.log 2>&1; echo "hazards rc=$?"; grep -E "PASSED|FAILED|XFAIL|ERROR" gpurun_out/hazards3.log | cut -c1-140 | tail -50
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -v -m gpu --timeout 300 --timeout-method thread -k "rccl or lockstep" > gpurun_out/rccl2.log 2>&1; echo "rccl rc=$?"; grep -E "PASSED|FAILED|ERROR" gpurun_out/rccl2.log | cut -c1-140
