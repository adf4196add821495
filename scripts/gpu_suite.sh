# the whole GPU suite, one process, as the driver runs it (plus -v)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/suite
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v > $O/suite.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/suite.log | tail -3
exit $rc
