#!/bin/bash
# A/B timing on the GPU box: bench.py once per argument set (no profiler), one summary line each.
#   tools/diag/ab.sh <tag> "<bench args 1>" "<bench args 2>" ...
# An argument "VAR=value ...|<bench args>" runs that set with the environment assignments first
# (e.g. "PQG_LIBDIR=lib_spk2|--config levels": an experiment build).
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
i=0
for a in "$@"; do
  i=$((i + 1))
  envs=""; args=$a
  case "$a" in *"|"*) envs=${a%%|*}; args=${a#*|} ;; esac
  env $envs timeout -k 10 300 python3 "$R/bench.py" --cpu-baseline 0 --pcie 0 $args > "$O/ab_$i.json" 2> "$O/ab_$i.err" || { echo "FAILED: $a"; tail -5 "$O/ab_$i.err"; exit 1; }
  python3 - "$O/ab_$i.json" "$a" <<'PY'
import json, sys
b = json.load(open(sys.argv[1]))
out = ["%-40s ms/step %.3f" % (sys.argv[2], b["ms_per_step"])]
st = b.get("stages_ms") or {}
if st:
    out.append("lv %.3f val %.3f" % (st.get("levels_kernel", 0), st.get("values_kernel", 0)))
for k, v in (b.get("variants") or {}).items():
    s = v.get("stages_ms") or {}
    out.append("| %s %.3f (lv %.3f val %.3f)" % (k, v["ms_per_step"], s.get("levels_kernel", 0), s.get("values_kernel", 0)))
print("  ".join(out))
PY
done
