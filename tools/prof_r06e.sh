#!/bin/bash
# Round-6 last: p_null 0.1 level profile and the default bench line after the k_d1_tab grid change.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/profile.sh levels r06_p10 --p-null 0.1 --variants 0 --pcie 0 --cpu-baseline 0 || exit 1
mkdir -p gpurun_out/r06_bench3
timeout -k 10 600 python bench.py > gpurun_out/r06_bench3/bench.json 2> gpurun_out/r06_bench3/bench.err || exit 1
