# kernel timeline of the default (pipelined) zstd launch at config 5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ztl
mkdir -p $O
timeout -s KILL 240 rocprofv3 --kernel-trace --output-format csv -d $O/tr -- python bench.py --codec zstd --profile --steps 3 --warmup 1 > $O/tr.log 2>&1 || { tail -20 $O/tr.log; exit 1; }
python3 scripts/trace_timeline.py $O/tr/*/*_kernel_trace.csv
