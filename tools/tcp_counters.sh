#!/bin/bash
# L1 (TCP) / texture-address (TA) counters of config 3's dictionary expand and of the gather
# micro-benchmark (tools/ubench/gather_ubench.hip: the same random 8-byte gathers from a 512 KiB
# table, nothing else), two --pmc passes each (TCP: 4 counters, TA + GRBM: 3).
#   tools/tcp_counters.sh <tag>
set -o pipefail
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p "$O"
make -s -C "$R/tools/ubench" gather_ubench || exit 1
cd /tmp && export TMPDIR=/tmp
P1="TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_LATENCY_sum TCP_PENDING_STALL_CYCLES_sum"
P2="TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE"
for i in 1 2; do
  eval P=\$P$i
  timeout -k 10 120 rocprofv3 --pmc $P -d "$O/dict_p$i" -o run --output-format csv -- \
    python3 "$R/bench.py" --config dict --steps 1 --warmup 0 --cpu-baseline 0 --variants 0 --pcie 0 > "$O/dict_p$i.log" 2>&1 || exit 1
  timeout -k 10 120 rocprofv3 --pmc $P -d "$O/gather_p$i" -o run --output-format csv -- \
    "$R/tools/ubench/gather_ubench" > "$O/gather_p$i.log" 2>&1 || exit 1
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d "$O/gather_kt" -o run --output-format csv -- \
  "$R/tools/ubench/gather_ubench" > "$O/gather_kt.log" 2>&1 || exit 1
echo ok
