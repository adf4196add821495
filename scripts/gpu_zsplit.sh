set -o pipefail
# zstd: two-part frame/sequence overlap A/B (ZSEEK_ZSTD_SPLIT = first part %)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/zsp
ZSEEK_ZSTD_SPLIT=50 timeout -k 10 300 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/zsp/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/zsp/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {
  timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/zsp/b.json 2> gpurun_out/zsp/b.err || exit $?
  echo "$1 $(python -c "import json;d=json.load(open('gpurun_out/zsp/b.json'));print(d['ms_per_step'], d['verified_bit_exact'])")"
}
for k in 1 2; do
  for v in 0 50 35 65; do ZSEEK_ZSTD_SPLIT=$v run "split$v"; done
done
