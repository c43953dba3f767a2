#!/bin/bash
# GPU box: which HIP graph mechanism the stale torch reduction depends on
mkdir -p gpurun_out
set -o pipefail
export TMPDIR=/tmp
run() {  # name, env...
    local name=$1; shift
    env "$@" timeout -k 10 300 python -u -m pytest tests/test_graph_hazards_gpu.py -v -s -m gpu --timeout 200 --timeout-method thread -k "old_bias and (torchcap or none)" > gpurun_out/hz_$name.log 2>&1
    echo "== $name rc=$?"; grep -E "PASSED|FAILED" gpurun_out/hz_$name.log | grep -v "^E" | cut -c1-160 | head -8
}
run default
run nopkt DEBUG_CLR_GRAPH_PACKET_CAPTURE=0
run noblitkarg DEBUG_CLR_BLIT_KERNARG_OPT=0
run nokargcopy DEBUG_HIP_KERNARG_COPY_OPT=0
timeout -k 10 300 python -u -m pytest tests/test_graph_hazards_gpu.py -v -m gpu --timeout 200 --timeout-method thread -k "dim0_sum and torchcap" > gpurun_out/hz_sum.log 2>&1
echo "== standalone sum rc=$?"; grep -E "PASSED|FAILED" gpurun_out/hz_sum.log | grep -v "^E" | cut -c1-160
