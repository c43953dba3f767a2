# GPU box: the large-N leg of bench.py under different settle / length settings, beside rollexp
mkdir -p gpurun_out; set -o pipefail
for cfg in "0 40" "0 400" "60 40" "200 200"; do set -- $cfg
timeout -k 10 200 python bench.py --no-cpu-baseline --train '' --rollout-k-extra '' --step-steps 0 --settle-ms $1 --steps $2 --warmup 2 > gpurun_out/bl_$1_$2.json 2> gpurun_out/bl_$1_$2.err || exit 1
python -c "import json;d=json.load(open('gpurun_out/bl_$1_$2.json'));print('settle $1 steps $2', d['roofline']['launch_us'], d['rollout_large_n']['launch_us'])"; done
timeout -k 10 150 tools/rollexp 4194304 16 > gpurun_out/rx4m.txt 2>&1 && grep -E "ws2: pair ring 8 steps, nt" gpurun_out/rx4m.txt
