#!/bin/bash
# Round-6: the default bench line (every config) and the alltypes profile after the D1 routing change.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
mkdir -p gpurun_out/r06_bench
timeout -k 10 600 python bench.py > gpurun_out/r06_bench/bench.json 2> gpurun_out/r06_bench/bench.err || exit 1
bash tools/profile.sh alltypes r06_at --variants 0 --pcie 0 --cpu-baseline 0 || exit 1
