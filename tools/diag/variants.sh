#!/bin/bash
# Time one bench config under several PQG_DEBUG diagnostics variants (kernel-trace stats each).
#   tools/diag/variants.sh <tag> <config> <debug values...>
set -o pipefail
tag=$1; cfg=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
for m in "$@"; do
  PQG_DEBUG=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_$m" -o run --output-format csv -- \
    python3 "$R/bench.py" --config $cfg --steps 10 --warmup 2 --cpu-baseline 0 --pcie 0 --variants 0 > "$O/bench_$m.json" 2> "$O/bench_$m.err" || { tail -5 "$O/bench_$m.err"; exit 1; }
  echo "== PQG_DEBUG=$m"
  python3 - "$O/trace_$m/run_kernel_stats.csv" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0].replace("void ", "")
    if n.startswith("pqg") and float(r["AverageNs"]) > 20000:
        print("   %-36s %4s  %9.1f us" % (n[:36], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
