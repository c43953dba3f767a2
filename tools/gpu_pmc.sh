#!/bin/bash
# GPU box: three separate PMC passes over tools/pmc_step.py (FETCH_SIZE; WRITE_SIZE; SQ issue
# counters), kernel-trace only, no sys/runtime trace; summary -> gpurun_out/pmc.json
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
run_pass() {  # name, workload arg ("" or r8), counters...
    local name=$1 arg=$2; shift 2
    timeout -s KILL 120 rocprofv3 --pmc "$@" --kernel-trace --output-format csv \
        -d /tmp/pmc_$name -o $name -- python tools/pmc_step.py $arg > gpurun_out/pmc_$name.log 2>&1 \
        || { tail -30 gpurun_out/pmc_$name.log; return 1; }
}
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA"
run_pass fetch "" FETCH_SIZE && run_pass write "" WRITE_SIZE && run_pass sq "" $SQ && \
run_pass fetch_r8 r8 FETCH_SIZE && run_pass write_r8 r8 WRITE_SIZE && run_pass sq_r8 r8 $SQ && \
python tools/pmc_summary.py gpurun_out/pmc.json /tmp/pmc_fetch /tmp/pmc_write /tmp/pmc_sq \
    /tmp/pmc_fetch_r8:r8 /tmp/pmc_write_r8:r8 /tmp/pmc_sq_r8:r8
