set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/check
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > $O/pytest.log 2>&1; rc=$?
grep -E "passed|failed|error" $O/pytest.log | tail -5
[ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error\|error" $O/pytest.log | head -120; exit $rc; }
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err && cat $O/bench.json
