#!/bin/bash
# Config-2 profiles at p_null 0, 0.1 and 0.5 (tools/profile.sh each), into gpurun_out/<prefix>_levels_pXX;
# tools/pmc_traffic.py then writes profiles/<round>/levels_pXX (the directories bench.py's
# pmc_traffic() looks up).  Usage: tools/prof_levels.sh <prefix> [extra bench args...]
set -o pipefail
pre=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
for p in 0.0 0.1 0.5; do
  t=$(printf 'p%02d' "$(python3 -c "print(round($p*100))")")
  bash "$R/tools/profile.sh" levels "${pre}_levels_$t" --p-null "$p" --variants 0 --cpu-baseline 0 --pcie 0 "$@" || exit $?
done
