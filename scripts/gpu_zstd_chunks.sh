# zstd chunked pipeline: tests (default and forced 3 chunks), then config 5
# at 1 / 2 / 4 / 8 chunks
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/zc
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 200 --timeout-method thread > $O/t1.log 2>&1 || { grep -B5 -A40 "FAILED\|Error" $O/t1.log | head -80; exit 1; }
tail -1 $O/t1.log
ZSEEK_ZSTD_CHUNKS=3 timeout -k 10 400 python -u -m pytest tests/test_gpu_zstd.py -x -q --timeout 200 --timeout-method thread > $O/t3.log 2>&1 || { grep -B5 -A40 "FAILED\|Error" $O/t3.log | head -80; exit 1; }
tail -1 $O/t3.log
for k in 1 2 4 8; do
ZSEEK_ZSTD_CHUNKS=$k timeout -k 10 300 python bench.py --codec zstd --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-latency > $O/k$k.json 2> $O/k$k.err || { tail -20 $O/k$k.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/k$k.json'));print('chunks $k', d['ms_per_step'], d['value'], d['verified_bit_exact'])"
done
