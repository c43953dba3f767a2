#!/bin/bash
# GPU box: PMC passes over the learner updates (tools/prof_learner.py <net> <dtype> <updates>
# <batch>), one counter group per rocprofv3 run, kernel-trace only (no sys/runtime trace);
# summary -> gpurun_out/pmc_learner.json.  Usage: gpu_pmc_learner.sh [workload ...]
#   workload = net:dtype:batch (default: every learner leg of bench.py)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
WL=${*:-"conv:fp64:8192 conv:fp32:8192 dense:fp64:8192 dense:fp32:8192 dense:fp64:5000 dense:fp32:5000 dense64:fp32:8192 dense64:fp64:8192"}
timeout -s KILL 60 rocprofv3 -L > gpurun_out/pmc_counter_list.txt 2>&1 || true
have() { grep -qw "$1" gpurun_out/pmc_counter_list.txt; }
SQ=""
for c in SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_VALU_MFMA_MOPS_F64 \
         SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES; do
    have $c && SQ="$SQ $c"
done
echo "SQ pass counters:$SQ"
SPECS=""
for w in $WL; do
    IFS=: read net dt b <<< "$w"
    tag="$net.$dt@$b"
    for pass in fetch write sq; do
        case $pass in fetch) C=FETCH_SIZE;; write) C=WRITE_SIZE;; sq) C=$SQ;; esac
        d=/tmp/pmcl_${net}_${dt}_${b}_$pass
        timeout -s KILL 180 rocprofv3 --pmc $C --kernel-trace --output-format csv -d $d \
            -o $pass -- python tools/prof_learner.py $net $dt 10 $b \
            > gpurun_out/pmcl_${net}_${dt}_${b}_$pass.log 2>&1 \
            || { tail -30 gpurun_out/pmcl_${net}_${dt}_${b}_$pass.log; exit 1; }
        SPECS="$SPECS $d:$tag"
    done
done
python tools/pmc_learner.py gpurun_out/pmc_learner.json $SPECS
