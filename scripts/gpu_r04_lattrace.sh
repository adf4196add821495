# round 4: kernel trace of 300 single-frame cache-0 reads (latency probe)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04lattrace
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python scripts/latency_probe.py 300 > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
grep p50 $O/probe.log
python3 -c "
import csv,glob
f=glob.glob('$O/trace/*/*_kernel_stats.csv')[0]
for r in csv.DictReader(open(f)):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1), 'us')
"
