#!/bin/bash
# GPU box, round 5 first call: the graph-hazard diagnostics (all cases, no -x), the full GPU
# suite, and the PMC passes with the fixed per-step normalisation
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_graph_hazards_gpu.py -v -s -m gpu --timeout 300 --timeout-method thread > gpurun_out/hazards.log 2>&1
echo "hazards rc=$?"; grep -E "PASS|FAIL|ERROR|errors:" gpurun_out/hazards.log | tail -60
timeout -k 10 1200 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --deselect tests/test_graph_hazards_gpu.py > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -30 gpurun_out/pmc.log; exit 1; }
