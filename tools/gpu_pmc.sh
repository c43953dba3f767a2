#!/bin/bash
# GPU box: two separate PMC passes (FETCH_SIZE, WRITE_SIZE), kernel-trace only, no sys/runtime trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_fetch -o fetch -- python tools/pmc_step.py > gpurun_out/pmc_fetch.log 2>&1 || { tail -30 gpurun_out/pmc_fetch.log; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/pmc_write -o write -- python tools/pmc_step.py > gpurun_out/pmc_write.log 2>&1 || { tail -30 gpurun_out/pmc_write.log; exit 1; }
find gpurun_out/pmc_fetch gpurun_out/pmc_write -name "*.csv" | head
python tools/pmc_summary.py 'gpurun_out/pmc_fetch/**/*counter_collection.csv' 'gpurun_out/pmc_write/**/*counter_collection.csv' gpurun_out/pmc_step.json
