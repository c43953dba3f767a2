# GPU box: the bench-driven tests, one default bench line (timed), the rollout kernels' rocprof
# stats (64k lean + 4M warp-specialised) and the PMC passes
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_dist_gpu.py tests/test_bench_configs4_gpu.py -x -v --timeout 800 --timeout-method thread -k "bench" > gpurun_out/tb.log 2>&1 || { tail -30 gpurun_out/tb.log; exit 1; }
tail -4 gpurun_out/tb.log
bash tools/gpu_pmc.sh > gpurun_out/pmc.log 2>&1 || { tail -30 gpurun_out/pmc.log; exit 1; }
s=$(date +%s); timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }; echo "bench wall $(( $(date +%s) - s )) s"
python -c "import json;d=json.load(open('gpurun_out/bench.json'));print(d['value'],d['roofline']['frac'],d['rollout_large_n'])"
rm -rf /tmp/prk && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d /tmp/prk -o r --output-format csv -- python bench.py --train '' --no-cpu-baseline > gpurun_out/prk.log 2>&1 && cp $(find /tmp/prk -name "*kernel_stats.csv") gpurun_out/bench_kernel_stats.csv && cut -d, -f1-4 gpurun_out/bench_kernel_stats.csv | head -5
