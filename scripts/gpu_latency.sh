set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/lat
mkdir -p $O
timeout -k 10 300 python scripts/latency_probe.py 300 > $O/probe.txt 2>&1 && cat $O/probe.txt &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python scripts/latency_probe.py 300 > $O/trace.log 2>&1 && tail -2 $O/trace.log &&
find $O/trace -name "*kernel_stats.csv" -exec cat {} \;
