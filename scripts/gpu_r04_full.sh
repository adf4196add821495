# round 4 evidence: the GPU suite first (production build), then the round
# evidence script (bench lines, kernel traces, PMC traffic and SQ counters,
# config 3 / 5 lines, compression lines, PCIe probe).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/round4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/round4/suite.log 2>&1 || { tail -30 gpurun_out/round4/suite.log; exit 1; }
tail -2 gpurun_out/round4/suite.log
bash scripts/gpu_round4.sh
