set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
true
timeout -k 10 300 python scripts/kbench.py --size 4294967296 --variants 61,73,60,74 --rounds 7 > gpurun_out/kb.log 2>&1; rc=$?; grep -v "^$" gpurun_out/kb.log | tail -4; exit $rc
