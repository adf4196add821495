set -o pipefail
# zstd phase-kernel check: GPU zstd parity tests, then the config-5 bench and a
# rocprofv3 kernel-trace summary.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/zstd
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 120 --timeout-method thread > gpurun_out/zstd/pytest.log 2>&1; rc=$?; tail -30 gpurun_out/zstd/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --codec zstd --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/zstd/bench.json 2> gpurun_out/zstd/bench.err; rc=$?; cat gpurun_out/zstd/bench.json; tail -3 gpurun_out/zstd/bench.err; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/zstd/prof -o run -- python3 bench.py --codec zstd --profile --steps 3 --warmup 1 > gpurun_out/zstd/prof.log 2>&1; rc=$?; tail -3 gpurun_out/zstd/prof.log; exit $rc
