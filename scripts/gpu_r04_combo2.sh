# round 4: production execute stage (3,584 bytes) against the 4,096 one, the
# GPU suite (writer min-batch fix, linked-frame compression), the destroy
# probe, and the compressor at 64 KiB (frames per wave) and 1 MiB frames.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04combo2
mkdir -p $O
timeout -k 10 300 python scripts/kbench.py --variants 0,321 --rounds 5 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep -v amdgpu.ids $O/kb.log | grep "median\|MISMATCH\|bit-exact"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
ZSEEK_HIP_DESTROY=1 timeout -k 10 400 python -u scripts/hang_probe.py both 250 > $O/probe_destroy.log 2>&1
rc=$?
tail -3 $O/probe_destroy.log
echo "probe rc=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit 0
timeout -k 10 240 python bench.py --codec lz4c --frame 65536 --steps 3 --warmup 1 --no-cpu-baseline > $O/c64.json 2> $O/c64.err || { tail -5 $O/c64.err; exit 1; }
ZSEEK_LZ4C_WAVES=1024 timeout -k 10 240 python bench.py --codec lz4c --frame 65536 --steps 3 --warmup 1 --no-cpu-baseline > $O/c64w1024.json 2> $O/c64w1024.err || { tail -5 $O/c64w1024.err; exit 1; }
timeout -k 10 300 python bench.py --codec lz4c --frame 1048576 --size 1073741824 --steps 3 --warmup 1 > $O/c1m.json 2> $O/c1m.err || { tail -5 $O/c1m.err; exit 1; }
for f in c64 c64w1024 c1m; do python -c "
import json,sys; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
print('$f', d['value'], d['unit'], d['ms_per_step'], 'ms', d.get('launch_by_frames'), (d.get('cpu_baseline') or {}).get('value'), d.get('verified_bit_exact'))"; done
exit 0
