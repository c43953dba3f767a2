# GPU box: rocprofv3 kernel trace of the dense-ref learner legs (torch path) at B = 5000
mkdir -p gpurun_out
export TMPDIR=/tmp
set -o pipefail
for dt in fp64 fp32; do
rm -rf /tmp/prd && timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prd -o p -- python bench.py --steps 5 --warmup 2 --step-steps 0 --rollout-k-extra '' --train dense@5000 --train-dtypes $dt --train-updates 50 --no-cpu-baseline > gpurun_out/pd_$dt.log 2>&1 && cp $(find /tmp/prd -name '*kernel_stats.csv') gpurun_out/dense5000_${dt}_kernel_stats.csv || exit 1
done
