# round 4: the chunk parse's emit with folded checks -- parity tests, the
# one-frame parse phase cycles (tuning build), 4 KiB latency and its trace
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/emit
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py tests/test_gpu_block_route.py -x -q --timeout 120 --timeout-method thread -m gpu -p no:cacheprovider > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/libzseek_tune.so ZSEEK_CHUNK_TIMERS=1 timeout -k 10 300 python scripts/latency_probe.py 300 > $O/ctimers.log 2>&1 || { tail -5 $O/ctimers.log; exit 1; }
grep -E "chunk one-route" $O/ctimers.log | tail -1
timeout -k 10 300 python scripts/latency_probe.py 300 > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
grep p50 $O/probe.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python scripts/latency_probe.py 300 > $O/probe_tr.log 2>&1 || { tail -5 $O/probe_tr.log; exit 1; }
python3 -c "
import csv,glob
f=max(glob.glob('$O/trace/*/*_kernel_stats.csv'))
for r in csv.DictReader(open(f)):
    print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1000,1), 'us')
"
