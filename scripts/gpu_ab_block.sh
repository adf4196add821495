# block route: its tests + the parity tests through it, then A/B at config 3
# (ZSEEK_BLOCK_ROUTE=0 turns it off), same box
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_block_route.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "block" > $O/t.log 2>&1 || { grep -B5 -A40 "FAILED\|Error" $O/t.log | head -100; exit 1; }
tail -2 $O/t.log
timeout -k 10 400 python bench.py --frame 1048576 --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-latency > $O/on.json 2> $O/on.err || { tail -20 $O/on.err; exit 1; }
ZSEEK_BLOCK_ROUTE=0 timeout -k 10 400 python bench.py --frame 1048576 --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-latency > $O/off.json 2> $O/off.err || { tail -20 $O/off.err; exit 1; }
for f in on off; do python3 -c "
import json;d=json.load(open('$O/$f.json'));r=d['roofline'];print('$f',d['ms_per_step'],d['verified_bit_exact'],{k:(v['kernel'][:22],v['avg_ms']) for k,v in r['stages'].items()})"; done
