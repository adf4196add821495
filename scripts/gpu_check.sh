set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
echo "== smoke"; timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; tail -5 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
echo "== pytest gpu"; timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
echo "== bench"; timeout -k 10 600 python bench.py --steps 5 --warmup 2 > gpurun_out/bench1.json 2> gpurun_out/bench1.err; rc=$?; cat gpurun_out/bench1.json; tail -5 gpurun_out/bench1.err; exit $rc
