set -o pipefail
# zstd sequence-kernel variants A/B (ZSEEK_ZSTD_SEQ=0..3): config-5 bench and
# a kernel-trace profile each
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/zab
for v in 0 2 3 0; do
  ZSEEK_ZSTD_SEQ=$v timeout -k 10 300 python bench.py --codec zstd --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/zab/b$v.json 2> gpurun_out/zab/b$v.err || exit $?
  echo "v$v $(python -c "import json;d=json.load(open('gpurun_out/zab/b$v.json'));print(d['ms_per_step'], d['verified_bit_exact'])")"
done
for v in 2 3; do
  ZSEEK_ZSTD_SEQ=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/zab/p$v -o run -- python3 bench.py --codec zstd --profile --steps 3 --warmup 1 > gpurun_out/zab/p$v.log 2>&1 || exit $?
done
echo done
