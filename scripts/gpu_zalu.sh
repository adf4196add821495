set -o pipefail
# zstd sequence kernel: LL/ML code tables from LDS vs computed (ZSEEK_ZSTD_ALU)
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/za
ZSEEK_ZSTD_ALU=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/za/pytest.log 2>&1; rc=$?; tail -3 gpurun_out/za/pytest.log; [ $rc -eq 0 ] || exit $rc
run() {
  timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/za/b.json 2> gpurun_out/za/b.err || exit $?
  echo "$1 $(python -c "import json;d=json.load(open('gpurun_out/za/b.json'));print(d['ms_per_step'], d['verified_bit_exact'])")"
}
for k in 1 2 3; do
  run "lds"
  ZSEEK_ZSTD_ALU=1 run "alu"
done
