#!/bin/bash
# Profile one bench config on the GPU box:
#   1. bench.py (the JSON line)                      -> gpurun_out/<tag>/bench.json
#   2. rocprofv3 --kernel-trace --stats              -> gpurun_out/<tag>/trace/
#   3. rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE   -> gpurun_out/<tag>/pmc_{fetch,write}/
#      (separate passes: the two TCC counters do not fit one pass on gfx950)
# Usage: tools/profile.sh <config> <tag> [extra bench args...]
set -o pipefail
cfg=$1; tag=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 "$R/bench.py" --config "$cfg" "$@" > "$O/bench.json" 2> "$O/bench.err" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace" -o run --output-format csv -- \
    python3 "$R/bench.py" --config "$cfg" --steps 5 --warmup 1 --cpu-baseline 0 --variants 0 "$@" > "$O/trace.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d "$O/pmc_fetch" -o run --output-format csv -- \
    python3 "$R/bench.py" --config "$cfg" --steps 2 --warmup 1 --cpu-baseline 0 --variants 0 "$@" > "$O/pmc_fetch.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d "$O/pmc_write" -o run --output-format csv -- \
    python3 "$R/bench.py" --config "$cfg" --steps 2 --warmup 1 --cpu-baseline 0 --variants 0 "$@" > "$O/pmc_write.log" 2>&1
