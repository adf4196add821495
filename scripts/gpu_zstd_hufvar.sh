# zstd A/B (tuning library): Huffman 64-byte store bursts (production) vs
# 128-byte bursts at three waves per SIMD, default 4-chunk pipeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/zhv
mkdir -p $O
export ZSEEK_AMD_LIB=$GRAFT_REPO_ROOT/libzseek_amd/lib/libzseek_tune.so
i=0
for v in 0 100 0 100; do
i=$((i+1))
ZSEEK_ZSTD_HUF_DIAG=$v timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-latency > $O/v$v.$i.json 2> $O/v$v.$i.err || { tail -20 $O/v$v.$i.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/v$v.$i.json'));print('huf variant $v', d['ms_per_step'], d['value'], d['verified_bit_exact'])"
done
ZSEEK_ZSTD_HUF_DIAG=100 ZSEEK_ZSTD_CHUNKS=1 ZSEEK_ZSTD_SERIAL=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr100 -- python bench.py --codec zstd --profile --steps 3 --warmup 1 > $O/tr100.log 2>&1 || { tail -20 $O/tr100.log; exit 1; }
python3 -c "
import csv,glob
f=max(glob.glob('$O/tr100/*/*_kernel_stats.csv'))
for r in csv.DictReader(open(f)):
    if 'zstd' in r['Name'] or 'seq_exec' in r['Name']: print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e6,3))"
