#!/bin/bash
# Effective clock of k_delta_page per DELTA block shape (verdict r05: 512 / 4x128 vs 128 / 4x32):
# one GRBM_GUI_ACTIVE pass per shape, each its own process -> gpurun_out/dclk/<shape>/clock.txt
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for shape in "512 4" "128 4"; do
  set -- $shape
  O=$R/gpurun_out/dclk/b$1
  mkdir -p "$O"
  timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d "$O/clk" -o run --output-format csv -- \
      python3 "$R/bench.py" --config delta --steps 10 --warmup 2 --variants 0 --cpu-baseline 0 --pcie 0 \
      --block-size $1 --mini-blocks $2 > "$O/bench.log" 2>&1 || exit 1
  d=$(dirname "$(find "$O/clk" -name 'run_kernel_trace.csv' | head -1)")
  python3 "$R/tools/diag/clock.py" "$d" > "$O/clock.txt" || exit 1
done
