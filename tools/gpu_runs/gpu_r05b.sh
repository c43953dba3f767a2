#!/bin/bash
# GPU box: the graph-hazard diagnostics (all cases, no -x) and the captured-RCCL tests
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_graph_hazards_gpu.py -v -s -m gpu --timeout 300 --timeout-method thread -k "bounds or old_bias" > gpurun_out/hazards2.log 2>&1
echo "hazards rc=$?"; grep -E "PASS|FAIL|ERROR|errors:|previous" gpurun_out/hazards2.log | tail -60
timeout -k 10 600 python -u -m pytest tests/test_dist_gpu.py -v -m gpu --timeout 300 --timeout-method thread -k "rccl or lockstep or graphed_dp" > gpurun_out/rccl.log 2>&1
echo "rccl rc=$?"; grep -E "PASS|FAIL|ERROR|Error" gpurun_out/rccl.log | tail -40
