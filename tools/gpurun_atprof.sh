set -o pipefail
R=$GRAFT_REPO_ROOT; O=$R/gpurun_out/$1; mkdir -p $O; cd /tmp; export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/at -o run --output-format csv -- python3 $R/bench.py --config alltypes --steps 5 --warmup 1 --cpu-baseline 0 --pcie 0 > $O/at.json 2>$O/at.err || exit $?
python3 -c "import json;b=json.load(open('$O/at.json'));print('alltypes', b['ms_per_step'])"
python3 -c "
import csv,glob
f=glob.glob('$O/at/**/run_kernel_stats.csv',recursive=True)[0]
for x in list(csv.DictReader(open(f)))[:24]: print('  ',x['Name'][:50], x['Calls'], x['AverageNs'], x['TotalDurationNs'])
"
