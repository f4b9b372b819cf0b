set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config levels --steps 10 --warmup 2 --cpu-baseline 0 --pcie 0 --variants 0 > $O/lv.json 2>$O/lv.err || exit $?
python -c "import json;b=json.load(open('$O/lv.json'));print('levels', b['ms_per_step'], b['stages_ms']['levels_kernel'])"
for i in 1 2 3; do
timeout -k 10 300 python bench.py --config alltypes --steps 10 --warmup 2 --cpu-baseline 0 --pcie 0 --streams 16 > $O/at$i.json 2>$O/at$i.err || exit $?
python -c "import json;b=json.load(open('$O/at$i.json'));print('alltypes', b['ms_per_step'])"
done
