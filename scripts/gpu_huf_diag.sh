# Huffman kernel elisions (tuning build, kernels serialized, one chunk):
# 8 = counters only, 1 = no literal stores, 3 = also no ring refills,
# 7 = also no table lookups
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/hdiag
mkdir -p $O
export ZSEEK_AMD_LIB=$GRAFT_REPO_ROOT/libzseek_amd/lib/libzseek_tune.so ZSEEK_ZSTD_CHUNKS=1 ZSEEK_ZSTD_SERIAL=1
for v in 0 8 1 3 7; do
ZSEEK_ZSTD_HUF_DIAG=$v timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $O/v$v -- python bench.py --codec zstd --profile --no-verify --steps 3 --warmup 1 > $O/v$v.log 2>&1 || { tail -20 $O/v$v.log; exit 1; }
grep -m2 "huf diag" $O/v$v.log || true
python3 -c "
import csv,glob
f=max(glob.glob('$O/v$v/*/*_kernel_stats.csv'))
for r in csv.DictReader(open(f)):
    if 'huf' in r['Name']: print('variant $v', r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e6,3))"
done
