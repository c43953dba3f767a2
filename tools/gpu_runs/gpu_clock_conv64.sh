# GPU box: GFX-clock cycles per dispatch (GRBM_GUI_ACTIVE) of the float64 conv update kernels and
# of the f64 MFMA microbenchmark, to tell a clock limit from an issue one
set -o pipefail
mkdir -p gpurun_out/clk64
export TMPDIR=/tmp
for t in prof_conv64 mfma64_feed; do
  rm -rf /tmp/clk64
  timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d /tmp/clk64 -o clk -- tools/$t > gpurun_out/clk64/$t.txt 2>&1 || exit 1
  cp "$(find /tmp/clk64 -name '*counter_collection.csv' | head -1)" gpurun_out/clk64/${t}_counters.csv
  cp "$(find /tmp/clk64 -name '*kernel_trace.csv' | head -1)" gpurun_out/clk64/${t}_trace.csv
done
