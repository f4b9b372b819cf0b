#!/bin/bash
# Round-6 profiles, part 2: dictionary, DELTA and alltypes configs (kernel stats + PMC traffic).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
bash tools/profile.sh dict r06_dict --variants 0 --pcie 0 --cpu-baseline 0 || exit 1
bash tools/profile.sh delta r06_delta --variants 0 --pcie 0 --cpu-baseline 0 || exit 1
bash tools/profile.sh alltypes r06_at --variants 0 --pcie 0 --cpu-baseline 0 || exit 1
