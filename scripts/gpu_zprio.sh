set -o pipefail
# zstd: Huffman side-stream priority (ZSEEK_ZSTD_SIDE_PRIO=-1/0/1) and launch
# order (ZSEEK_ZSTD_SEQ_FIRST) A/B
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/zpr
run() {
  timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/zpr/b.json 2> gpurun_out/zpr/b.err || exit $?
  echo "$1 $(python -c "import json;d=json.load(open('gpurun_out/zpr/b.json'));print(d['ms_per_step'], d['verified_bit_exact'])")"
}
for k in 1 2; do
  ZSEEK_ZSTD_SIDE_PRIO=0 run "prio0"
  ZSEEK_ZSTD_SIDE_PRIO=-1 run "prio-1"
  ZSEEK_ZSTD_SIDE_PRIO=0 ZSEEK_ZSTD_SEQ_FIRST=1 run "seqfirst"
  ZSEEK_ZSTD_SIDE_PRIO=-1 ZSEEK_ZSTD_SEQ_FIRST=1 run "seqfirst+prio-1"
done
