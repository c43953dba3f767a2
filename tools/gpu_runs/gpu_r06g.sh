#!/bin/bash
# round 6 (g): the driver's bench command on the committed tree (the learner roofline objects
# reading profiles/r06/pmc_learner.json, the env legs profiles/r06/pmc.json)
set -o pipefail
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out/r06g
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > gpurun_out/r06g/bench_driver_cmd.json 2> gpurun_out/r06g/bench_driver_cmd.err || { tail -20 gpurun_out/r06g/bench_driver_cmd.err; exit 1; }
python - <<'PY'
import json
d = json.loads(open("gpurun_out/r06g/bench_driver_cmd.json").read().strip().splitlines()[-1])
r = d["roofline"]
print(round(d["value"] / 1e9, 1), "G", round(r["frac"], 3), round(r["frac_wall"], 3), r["traffic_source"][:40])
for k, v in d["learner"].items():
    ro = v["roofline"]
    print(k, round(v["update_ms"] * 1e3, 1), round(ro["frac"], 3), ro.get("executed_mfma_frac"), ro.get("traffic"), ro.get("traffic_over_algorithmic"))
print(d["dist"])
PY
