# zstd A/B (tuning library): sequence kernel with tables in LDS (production)
# vs from the table slots (no LDS), under the default 4-chunk pipeline
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/zsv
mkdir -p $O
export ZSEEK_AMD_LIB=$GRAFT_REPO_ROOT/libzseek_amd/lib/libzseek_tune.so
for v in 0 1 2 0; do
ZSEEK_ZSTD_SEQ=$v timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-latency > $O/v$v.json 2> $O/v$v.err || { tail -20 $O/v$v.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/v$v.json'));print('seq variant $v', d['ms_per_step'], d['value'], d['verified_bit_exact'])"
done
