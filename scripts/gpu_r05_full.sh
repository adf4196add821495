# round 5 evidence: the GPU suite first (production build, one process, as
# the driver runs it), smoke, then scripts/gpu_round5.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/round5
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/round5/suite.log 2>&1 || { tail -30 gpurun_out/round5/suite.log; exit 1; }
tail -2 gpurun_out/round5/suite.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" 2>&1 | tail -2 &&
bash scripts/gpu_round5.sh c2
