# block route: its tests, the parity tests through it, config 3 (1 MiB) and
# config 2 (64 KiB, the route off) bench lines
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/block
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_block_route.py -x -v --timeout 200 --timeout-method thread > $O/t1.log 2>&1 || { tail -60 $O/t1.log; exit 1; }
tail -3 $O/t1.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "block or None" > $O/t2.log 2>&1 || { grep -B5 -A40 "FAILED\|Error" $O/t2.log | head -100; exit 1; }
tail -2 $O/t2.log
timeout -k 10 400 python bench.py --frame 1048576 --steps 5 --warmup 2 --no-e2e --no-cpu-baseline > $O/f1m.json 2> $O/f1m.err || { tail -20 $O/f1m.err; exit 1; }
cat $O/f1m.json
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-e2e --no-cpu-baseline > $O/f64k.json 2> $O/f64k.err || { tail -20 $O/f64k.err; exit 1; }
cat $O/f64k.json
