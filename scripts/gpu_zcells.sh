set -o pipefail
# zstd sequence kernel: more LDS cells per frame (ZSEEK_ZSTD_SEQ=4: 16 x 1312,
# 5: 24 x 1056) vs the default 32 x 800
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/zc
run() {
  timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/zc/b.json 2> gpurun_out/zc/b.err || exit $?
  echo "$1 $(python -c "import json;d=json.load(open('gpurun_out/zc/b.json'));print(d['ms_per_step'], d['verified_bit_exact'])")"
}
for k in 1 2; do
  for v in 0 6 7; do ZSEEK_ZSTD_SEQ=$v run "seq$v"; done
done
