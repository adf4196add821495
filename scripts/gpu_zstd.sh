set -o pipefail
# zstd (config 5) evidence: the full bench line (with the reference CPU
# baseline) and a rocprofv3 kernel-trace summary of a short profile run.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/zstd
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --codec zstd --steps 3 --warmup 1 > gpurun_out/zstd/bench.json 2> gpurun_out/zstd/bench.err; rc=$?; cat gpurun_out/zstd/bench.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/zstd/prof -o run -- python3 bench.py --codec zstd --profile --steps 3 --warmup 1 > gpurun_out/zstd/prof.log 2>&1; rc=$?; tail -3 gpurun_out/zstd/prof.log; exit $rc
