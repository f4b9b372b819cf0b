set -o pipefail
R=$GRAFT_REPO_ROOT; cd $R
bash tools/profile.sh levels r02g_levels || exit 1; echo "levels done"
O=$R/gpurun_out/r02g_alltypes; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 python3 $R/bench.py --config alltypes --streams 16 > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --config alltypes --streams 16 --steps 3 --warmup 1 --cpu-baseline 0 --pcie 0 > $O/trace.log 2>&1 || exit 1
cd $R && python3 tools/conc.py $O/trace/run_kernel_trace.csv 17 > $O/concurrency.txt
echo alltypes done
