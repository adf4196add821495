# smoke + full GPU test suite + short benches (config 2, config 3 at 1 MiB).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -3 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== pytest gpu"; timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?; cat gpurun_out/bench1.json; tail -3 gpurun_out/bench1.err; [ $rc -eq 0 ] || exit $rc
echo "== bench 1 MiB"; timeout -k 10 600 python bench.py --steps 5 --warmup 2 --frame 1048576 --no-cpu-baseline > gpurun_out/bench1m.json 2> gpurun_out/bench1m.err; rc=$?; cat gpurun_out/bench1m.json; tail -3 gpurun_out/bench1m.err; exit $rc
