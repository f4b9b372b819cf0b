set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; cd $R
for i in 1 2 3; do
timeout -k 10 300 python bench.py --config alltypes --steps 10 --warmup 2 --cpu-baseline 0 --pcie 0 --streams 16 > $O/at$i.json 2>$O/at$i.err || exit $?
python -c "import json;b=json.load(open('$O/at$i.json'));print('alltypes', b['ms_per_step'])"
done
