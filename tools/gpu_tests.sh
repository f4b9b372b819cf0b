#!/bin/bash
# GPU parity tests (one process), log under gpurun_out/<tag>/pytest.log; extra args go to pytest.
set -o pipefail
tag=$1; shift
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p "$R/gpurun_out/$tag"
cd "$R" && timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > "gpurun_out/$tag/pytest.log" 2>&1
rc=$?
tail -5 "gpurun_out/$tag/pytest.log"
exit $rc
