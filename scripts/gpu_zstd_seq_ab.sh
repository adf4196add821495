# zstd sequence-kernel layouts, same box (tuning build, ZSEEK_ZSTD_SEQ
# variants, default "0 3"): 0 = production, see zstd_decode.hip for the rest
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/zsab
mkdir -p $O
export ZSEEK_AMD_LIB=$GRAFT_REPO_ROOT/libzseek_amd/lib/libzseek_tune.so
V=${1:-0 3}
for v in $V $V; do
ZSEEK_ZSTD_SEQ=$v timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-latency > $O/b$v.json 2> $O/b$v.err || { tail -20 $O/b$v.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/b$v.json'));print('seq layout $v', d['ms_per_step'], d['value'], d['verified_bit_exact'])"
done
for v in $V; do
ZSEEK_ZSTD_SEQ=$v ZSEEK_ZSTD_CHUNKS=1 ZSEEK_ZSTD_SERIAL=1 timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr$v -- python bench.py --codec zstd --profile --steps 3 --warmup 1 > $O/tr$v.log 2>&1 || { tail -20 $O/tr$v.log; exit 1; }
python3 -c "
import csv,glob
f=max(glob.glob('$O/tr$v/*/*_kernel_stats.csv'))
for r in csv.DictReader(open(f)):
    if 'seq_kernel' in r['Name']: print('serial, layout $v:', r['Name'][:60], round(float(r['AverageNs'])/1e6,3))"
done
