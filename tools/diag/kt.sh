#!/bin/bash
# Kernel-trace one or more bench runs on the GPU box and print per-kernel average times.
#   tools/diag/kt.sh <tag> "<bench args 1>" ["<bench args 2>" ...]
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
i=0
for a in "$@"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/kt_$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --steps 10 --warmup 2 --cpu-baseline 0 --pcie 0 --variants 0 $a > "$O/kt_$i.json" 2> "$O/kt_$i.err" || { echo "FAILED: $a"; tail -5 "$O/kt_$i.err"; exit 1; }
  python3 - "$O/kt_$i/run_kernel_stats.csv" "$O/kt_$i.json" "$a" <<'PY'
import csv, json, sys
b = json.load(open(sys.argv[2]))
print("== %s: ms/step %.3f" % (sys.argv[3], b["ms_per_step"]))
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0].replace("void ", "")
    if n.startswith("pqg"):
        print("   %-40s %4s  %9.1f us" % (n[:40], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
