#!/bin/bash
# A/B of experiment builds on one bench config: ab.sh <tag> <config> <lib> <lib> ... [-- bench args]
# (PQG_LIBDIR selects lib_<variant>/, Makefile VARIANT=...). Each build twice, interleaved.
set -o pipefail
tag=$1; cfg=$2; shift 2
libs=(); while [ $# -gt 0 ] && [ "$1" != "--" ]; do libs+=("$1"); shift; done; [ "$1" == "--" ] && shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/$tag"
for i in 1 2; do
  for v in "${libs[@]}"; do
    PQG_LIBDIR=$v timeout -k 10 300 python "$R/bench.py" --config "$cfg" --steps 10 --warmup 3 --cpu-baseline 0 --pcie 0 "$@" \
      > "$R/gpurun_out/$tag/$v.$i.json" 2>/dev/null || exit 1
    python3 - "$R/gpurun_out/$tag/$v.$i.json" "$v" <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
c = d.get("configs", {d.get("config", {}).get("workload", "?"): d})
for k, v in (c.items() if isinstance(c, dict) else []):
    r = v.get("roofline") or {}
    print(sys.argv[2], k[:28], round(v["ms_per_step"], 4), "kernel", round(r.get("avg_ms") or 0, 4),
          " ".join(f"{n}:{round(x['ms_per_step'], 4)}" for n, x in (v.get("variants") or {}).items()))
PY
  done
done
