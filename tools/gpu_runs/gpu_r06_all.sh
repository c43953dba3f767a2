#!/bin/bash
# GPU box: the whole GPU suite, smoke, the default bench line and the driver's command line
mkdir -p gpurun_out/prof
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 400 python bench.py > gpurun_out/prof/bench.json 2> gpurun_out/prof/bench.err || { tail -20 gpurun_out/prof/bench.err; exit 1; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/prof/bench_driver_cmd.json 2> gpurun_out/prof/bench_driver_cmd.err || { tail -20 gpurun_out/prof/bench_driver_cmd.err; exit 1; }
python - <<'PY'
import json
for f in ("bench", "bench_driver_cmd"):
    d = json.loads(open(f"gpurun_out/prof/{f}.json").read().strip().splitlines()[-1])
    r = d["roofline"]
    print(f, round(d["value"] / 1e9, 1), "G", "frac", round(r["frac"], 3), "frac_wall", round(r["frac_wall"], 3),
          "issue", r.get("issue", {}).get("valu_insts_per_wave_step"))
    for k, v in d.get("learner", {}).items():
        print(" ", k, round(v["update_ms"] * 1e3, 1), "us", round(v["flop_frac"], 3), "traffic", v.get("roofline", {}).get("traffic"), "loop", round(v["loop_iter_ms"] * 1e3, 1), round(v["loop_late_iter_ms"] * 1e3, 1))
    if "step_kernel" in d: print("  step", round(d["step_kernel"]["launch_us_graph"], 2), "floor", round(d["step_kernel"]["launch_floor_us"], 2))
    if "rollout_large_n" in d: print("  large", round(d["rollout_large_n"]["frac"], 3))
    if "rollout_64k_hbm" in d: print("  64k hbm", round(d["rollout_64k_hbm"]["roofline"]["frac"], 3))
PY
