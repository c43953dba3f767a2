# GPU box: GFX-clock cycles per dispatch (GRBM_GUI_ACTIVE) of the 4M-board rollout variants, to
# tell a power/clock limit from an issue-interleaving one (large N)
set -o pipefail
mkdir -p gpurun_out/clk
export TMPDIR=/tmp
rm -rf /tmp/clk
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d /tmp/clk -o clk -- tools/rollexp 4194304 16 > gpurun_out/clk/rollexp.txt 2>&1
cp "$(find /tmp/clk -name '*counter_collection.csv' | head -1)" gpurun_out/clk/counters.csv
cp "$(find /tmp/clk -name '*kernel_trace.csv' | head -1)" gpurun_out/clk/trace.csv 2>/dev/null || true
