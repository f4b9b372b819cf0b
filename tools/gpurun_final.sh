set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python bench.py > $O/bench_default.json 2> $O/bench_default.err || { tail -5 $O/bench_default.err; exit 1; }
python -c "import json;b=json.load(open('$O/bench_default.json'));print(b['value'], b['ms_per_step'], b['roofline']['frac'], b['roofline']['traffic'], b['cpu_baseline']['value'])"
timeout -k 10 600 python bench.py --config alltypes > $O/bench_alltypes.json 2> $O/bench_alltypes.err || { tail -5 $O/bench_alltypes.err; exit 1; }
python -c "import json;b=json.load(open('$O/bench_alltypes.json'));print(b['value'], b['ms_per_step'], b['config']['streams'], b['pcie_inclusive']['ms'])"
