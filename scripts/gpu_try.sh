set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pt_all.log 2>&1; rc=$?; tail -3 gpurun_out/pt_all.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python scripts/kbench.py --size 4294967296 --variants 61,73 --rounds 5 > gpurun_out/kb.log 2>&1; rc=$?; grep -v "^$" gpurun_out/kb.log | tail -2; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --codec zstd --steps 2 --warmup 1 --profile > gpurun_out/bz.json 2>&1; rc=$?; grep -o '"value": [0-9.]*' gpurun_out/bz.json; exit $rc
