set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
cd /tmp; export TMPDIR=/tmp
for pn in 0.05 0.5; do
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $O/p$pn -o run --output-format csv -- python3 $R/bench.py --config levels --p-null $pn --variants 0 --steps 5 --warmup 1 --cpu-baseline 0 --pcie 0 > $O/lv$pn.json 2>$O/lv$pn.err || exit $?
python3 -c "import json;b=json.load(open('$O/lv$pn.json'));print('levels', $pn, b['ms_per_step'], b['stages_ms']['levels_kernel'])"
python3 -c "
import csv,glob
f=glob.glob('$O/p$pn/**/run_kernel_stats.csv',recursive=True)[0]
for x in list(csv.DictReader(open(f)))[:8]: print('  ',x['Name'][:50], x['Calls'], x['AverageNs'])
"
done
cd $R
timeout -k 10 300 python bench.py --config alltypes --steps 10 --warmup 2 --cpu-baseline 0 --pcie 0 --streams 16 > $O/at.json 2>$O/at.err && python -c "import json;b=json.load(open('$O/at.json'));print('alltypes', b['ms_per_step'])"
