#!/bin/bash
# Round-6 final: GPU suite, smoke, the default bench line and the dictionary profile.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_tests.sh r06_final || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_final/smoke.log 2>&1 || exit 1
mkdir -p gpurun_out/r06_bench2
timeout -k 10 600 python bench.py > gpurun_out/r06_bench2/bench.json 2> gpurun_out/r06_bench2/bench.err || exit 1
bash tools/profile.sh dict r06_dict --variants 0 --pcie 0 --cpu-baseline 0 || exit 1
