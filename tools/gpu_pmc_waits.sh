#!/bin/bash
# GPU box: where the conv learner kernels wait -- one SQ pass per workload (wave cycles split into
# waiting on counters / barriers, issue stalls, LDS issue stalls, active; LDS bank conflicts),
# kernel trace only; summary -> gpurun_out/pmc_waits.json
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SQ="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS"
SPECS=""
for w in ${*:-conv:fp64:8192 conv:fp32:8192}; do
    IFS=: read net dt b <<< "$w"
    d=/tmp/pmcw_${net}_${dt}_${b}
    timeout -s KILL 180 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $d -o sq \
        -- python tools/prof_learner.py $net $dt 10 $b > gpurun_out/pmcw_${net}_${dt}_${b}.log 2>&1 \
        || { tail -30 gpurun_out/pmcw_${net}_${dt}_${b}.log; exit 1; }
    SPECS="$SPECS $d:$net.$dt@$b"
done
python tools/pmc_learner.py gpurun_out/pmc_waits.json $SPECS > /dev/null && python - <<'PY'
import json
d = json.load(open("gpurun_out/pmc_waits.json"))
for k, v in d.items():
    if k.startswith("_"):
        continue
    c = v["counters"]
    wc = c.get("SQ_WAVE_CYCLES", 0) or 1
    print(f"{k:45s} wait_any {c.get('SQ_WAIT_ANY',0)/wc:.2f} wait_inst {c.get('SQ_WAIT_INST_ANY',0)/wc:.2f} "
          f"wait_lds {c.get('SQ_WAIT_INST_LDS',0)/wc:.2f} active {c.get('SQ_ACTIVE_INST_ANY',0)/wc:.2f} "
          f"lds_active {c.get('SQ_ACTIVE_INST_LDS',0)/wc:.2f} bank_conf/wave {c.get('SQ_LDS_BANK_CONFLICT',0)/max(c.get('SQ_WAVES',1),1):.0f}")
PY
