set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/bench
mkdir -p $O
timeout -k 10 600 python bench.py > $O/n1.json 2> $O/n1.err || { tail -20 $O/n1.err; exit 1; }
cat $O/n1.json
timeout -k 10 600 python bench.py --total-size 64G --no-cpu-baseline --no-e2e --no-latency > $O/c4n1.json 2> $O/c4n1.err || { tail -20 $O/c4n1.err; exit 1; }
cat $O/c4n1.json
