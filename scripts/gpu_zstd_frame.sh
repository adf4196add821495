# zstd frame-kernel change: parity (zstd GPU tests), per-kernel times with the
# kernels serialized (one chunk), then the default bench line
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/zfr
mkdir -p $O
timeout -k 10 400 python -u -X faulthandler -m pytest -x -v tests/test_gpu_zstd.py > $O/tests.log 2>&1 || { tail -60 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ZSEEK_ZSTD_CHUNKS=1 ZSEEK_ZSTD_SERIAL=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -- python bench.py --codec zstd --profile --steps 3 --warmup 1 > $O/tr.log 2>&1 || { tail -20 $O/tr.log; exit 1; }
python3 -c "
import csv,glob
f=max(glob.glob('$O/tr/*/*_kernel_stats.csv'))
for r in csv.DictReader(open(f)):
    if 'zstd' in r['Name'] or 'seq_exec' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3))"
timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-latency > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/b.json'));print('zstd', d['ms_per_step'], d['value'], d['verified_bit_exact'])"
