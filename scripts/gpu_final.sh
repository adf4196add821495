set -o pipefail
# round-end evidence: the default bench line (as the driver runs it) and the
# config-5 line
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/final
timeout -k 10 600 python bench.py > gpurun_out/final/bench.json 2> gpurun_out/final/bench.err || exit $?
cat gpurun_out/final/bench.json
timeout -k 10 600 python bench.py --codec zstd > gpurun_out/final/zstd.json 2> gpurun_out/final/zstd.err || exit $?
cat gpurun_out/final/zstd.json
