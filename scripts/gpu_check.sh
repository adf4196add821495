set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/g1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g1/pytest.log 2>&1; rc=$?
tail -5 gpurun_out/g1/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > gpurun_out/g1/bench.json 2> gpurun_out/g1/bench.err && cat gpurun_out/g1/bench.json
