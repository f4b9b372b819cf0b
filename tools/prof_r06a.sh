#!/bin/bash
# Round-6 profiles, part 1: GPU suite, smoke, level configs (kernel stats + PMC traffic + SQ counters).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/gpu_tests.sh r06_final || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r06_final/smoke.log 2>&1 || exit 1
bash tools/profile.sh levels r06_p10 --p-null 0.1 --variants 0 --pcie 0 --cpu-baseline 0 || exit 1
bash tools/profile.sh levels r06_p50 --p-null 0.5 --variants 0 --pcie 0 --cpu-baseline 0 || exit 1
bash tools/profile.sh levels r06_p00 --variants 0 --pcie 0 --cpu-baseline 0 || exit 1
bash tools/sq_counters.sh levels r06_p10_sq --p-null 0.1 || exit 1
