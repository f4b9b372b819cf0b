set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
bash tools/profile.sh levels $1_levels || exit $?
python -c "import json;b=json.load(open('$R/gpurun_out/$1_levels/bench.json'));print(b['value'], b['ms_per_step'], b['roofline']['frac'], b['cpu_baseline']['value'])"
cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/at -o run --output-format csv -- python3 bench.py --config alltypes --steps 5 --warmup 1 --cpu-baseline 0 --pcie 0 > $O/at_trace.json 2>$O/at_trace.err || exit $?
timeout -k 10 600 python bench.py --config alltypes > $O/bench_alltypes.json 2> $O/bench_alltypes.err || { tail -5 $O/bench_alltypes.err; exit 1; }
python -c "import json;b=json.load(open('$O/bench_alltypes.json'));print(b['value'], b['ms_per_step'], b['pcie_inclusive']['ms'])"
