#!/bin/bash
# Quick kernel stats of one bench config: rocprofv3 --kernel-trace --stats -> gpurun_out/<tag>/kq/
# Usage: tools/kq.sh <tag> [bench args...]
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kq" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 3 --warmup 1 --cpu-baseline 0 --variants 0 --pcie 0 "$@" > "$O/kq.log" 2>&1
rc=$?
f=$(find "$O/kq" -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && python3 "$R/tools/kstat_csv.py" "$f" 2>/dev/null | head -25
exit $rc
