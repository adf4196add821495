# zstd pipeline chunk count, same box: ZSEEK_ZSTD_CHUNKS in $1 (default "2 3 4 6")
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/zchunks
mkdir -p $O
for k in ${1:-2 3 4 6} ${1:-2 3 4 6}; do
ZSEEK_ZSTD_CHUNKS=$k timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-latency > $O/k$k.json 2> $O/k$k.err || { tail -20 $O/k$k.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/k$k.json'));print('chunks $k', d['ms_per_step'], d['value'], d['verified_bit_exact'])"
done
