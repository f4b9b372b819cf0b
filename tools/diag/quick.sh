#!/bin/bash
# GPU-box check used while iterating: gpu parity tests, then bench + kernel-trace stats per config.
#   tools/diag/quick.sh <tag> [configs...]
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd "$R"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > "$O/pytest.log" 2>&1
rc=$?
tail -5 "$O/pytest.log"
[ $rc -eq 0 ] || exit $rc
cd /tmp && export TMPDIR=/tmp
for c in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$O/trace_$c" -o run --output-format csv -- \
    python3 "$R/bench.py" --config $c --steps 10 --warmup 2 --cpu-baseline 0 --pcie 0 --variants 0 > "$O/bench_$c.json" 2> "$O/bench_$c.err" || exit 1
  python3 - "$O/trace_$c/run_kernel_stats.csv" "$O/bench_$c.json" <<'PY'
import csv, json, sys
b = json.load(open(sys.argv[2]))
print(b["config"]["workload"], "ms/step %.3f" % b["ms_per_step"], "GB/s %.0f" % b["gbps"])
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Name"].split("(")[0].replace("void ", "")
    if n.startswith("pqg"):
        print("   %-32s %4s  %9.1f us" % (n[:32], r["Calls"], float(r["AverageNs"]) / 1e3))
PY
done
