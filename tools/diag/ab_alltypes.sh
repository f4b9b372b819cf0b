set -o pipefail
R=$GRAFT_REPO_ROOT
TAG=${TAG:-r05k}; mkdir -p $R/gpurun_out/$TAG
for i in 1 2; do
for v in lib lib_nofork; do
PQG_LIBDIR=$v timeout -k 10 300 python bench.py --config alltypes --steps 10 --warmup 3 --cpu-baseline 0 --pcie 0 > $R/gpurun_out/$TAG/$v.$i.json 2>/dev/null || exit 1
python3 -c "import json;d=json.load(open('$R/gpurun_out/$TAG/$v.$i.json'));print('$v', d['ms_per_step'], d['value_check']['status'] if 'value_check' in d else '')"
done; done
