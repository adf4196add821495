# multi-rank bench path on a one-GPU box: 2 ranks sharing device 0 (gloo
# collective), contiguous and round-robin shards of a fixed total
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/multi
mkdir -p $O
export ZSEEK_BENCH_SHARE_GPU=1
timeout -k 10 400 python bench.py --gpus 2 --total-size 16G --steps 3 --warmup 1 > $O/c.json 2> $O/c.err || { tail -30 $O/c.err; exit 1; }
cat $O/c.json
timeout -k 10 400 python bench.py --gpus 2 --total-size 8G --steps 3 --warmup 1 --partition round_robin > $O/rr.json 2> $O/rr.err || { tail -30 $O/rr.err; exit 1; }
cat $O/rr.json
