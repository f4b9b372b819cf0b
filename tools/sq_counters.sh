#!/bin/bash
# SQ instruction / wait counters per kernel for one bench config (diagnostics).
# Usage: tools/sq_counters.sh <config> <tag> [extra bench args]
set -o pipefail
cfg=$1; tag=$2; shift 2
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE -d "$O/p1" -o run --output-format csv -- \
    python3 "$R/bench.py" --config "$cfg" --steps 1 --warmup 0 --cpu-baseline 0 --variants 0 --pcie 0 "$@" > "$O/p1.log" 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_BRANCH SQ_INSTS_SENDMSG -d "$O/p2" -o run --output-format csv -- \
    python3 "$R/bench.py" --config "$cfg" --steps 1 --warmup 0 --cpu-baseline 0 --variants 0 --pcie 0 "$@" > "$O/p2.log" 2>&1
