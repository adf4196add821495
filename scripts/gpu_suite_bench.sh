# the whole GPU suite (one process, as the driver runs it), then the default
# bench line (config 2 + cpu_baseline + end_to_end + latency).  Output dir: $1.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/${1:-suite_bench}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/suite.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err && cat $O/bench.json
