#!/bin/bash
# LDS counters per kernel for one bench config (diagnostics): instructions, bank conflicts,
# active / waiting cycles. Usage: tools/lds_counters.sh <config> <tag> [extra bench args]
set -o pipefail
cfg=$1; tag=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU -d "$O/p1" -o run --output-format csv -- \
    python3 "$R/bench.py" --config "$cfg" --steps 1 --warmup 0 --cpu-baseline 0 --variants 0 --pcie 0 "$@" > "$O/p1.log" 2>&1
