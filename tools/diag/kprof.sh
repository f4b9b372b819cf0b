#!/bin/bash
# Kernel averages (rocprofv3 --kernel-trace --stats) of one bench config for each experiment build:
# kprof.sh <tag> <config> <lib> [<lib> ...] [-- bench args]; prints the kernels above 20 us.
set -o pipefail
tag=$1; cfg=$2; shift 2
libs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done; [ "$1" == "--" ] && shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in "${libs[@]}"; do
  O=$R/gpurun_out/$tag/$v
  mkdir -p "$O"
  PQG_LIBDIR=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O" -o run --output-format csv -- \
    python3 "$R/bench.py" --config "$cfg" --steps 5 --warmup 1 --cpu-baseline 0 --pcie 0 --variants 0 "$@" > "$O/trace.log" 2>&1 || exit 1
  python3 - "$O/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    a = float(r["AverageNs"]) / 1e3
    if a > 20 and "copy16" not in r["Name"] and "rocclr" not in r["Name"]:
        print(sys.argv[2], f"{r['Name'][:56]:56s} {int(r['Calls']):4d} {a:9.1f} us")
PY
done
