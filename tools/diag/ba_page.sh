set -o pipefail
R=$(pwd)
mkdir -p gpurun_out/bap
timeout -k 10 120 python tools/diag/ba_page.py > gpurun_out/bap/run.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/bap/kq -o run --output-format csv -- python3 $R/tools/diag/ba_page.py > $R/gpurun_out/bap/kq.log 2>&1
f=$(find $R/gpurun_out/bap/kq -name '*kernel_stats.csv' | head -1)
python3 $R/tools/kstat_csv.py "$f" > $R/gpurun_out/bap/kstat.txt
