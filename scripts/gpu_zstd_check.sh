# zstd GPU tests (one process), then the config-5 bench line.  Output dir: $1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-zstd_check}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_zstd.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/suite.log | tail -3
[ $rc -eq 0 ] || { grep -E "FAIL|Error|assert" $O/suite.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py --codec zstd --no-e2e > $O/bench.json 2> $O/bench.err && cat $O/bench.json
