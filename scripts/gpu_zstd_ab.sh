# zstd: tests, the default bench line, and the SQ pass (pipeline off)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/zab
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 200 --timeout-method thread > $O/t.log 2>&1 || { grep -B5 -A40 "FAILED\|Error" $O/t.log | head -80; exit 1; }
tail -1 $O/t.log
timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-latency > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/b.json'));print('zstd', d['ms_per_step'], d['value'], d['verified_bit_exact'])"
ZSEEK_ZSTD_CHUNKS=1 ZSEEK_ZSTD_SERIAL=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr -- python bench.py --codec zstd --profile --steps 3 --warmup 1 > $O/tr.log 2>&1 || { tail -20 $O/tr.log; exit 1; }
ZSEEK_ZSTD_CHUNKS=1 ZSEEK_ZSTD_SERIAL=1 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $O/p1 -- python bench.py --codec zstd --profile --steps 2 --warmup 1 > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
python3 scripts/pmc_summary.py $O > $O/summary.txt 2>&1; grep -A24 "zstd_seq_kernel" $O/summary.txt | grep "per-wave"
python3 -c "
import csv,glob
f=max(glob.glob('$O/tr/*/*_kernel_stats.csv'))
for r in csv.DictReader(open(f)):
    if 'zstd' in r['Name'] or 'seq_exec' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3))"
