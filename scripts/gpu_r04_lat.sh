# round 4: the one-frame route's workgroup execute (seq_exec_frame_kernel):
# GPU suite, then the config-2 line's 4 KiB read latency with it and with
# the wave execute (ZSEEK_ONE_EXEC=wave), and a kernel trace of the reads.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04lat
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-verify > $O/l1.json 2> $O/l1.err || { tail -5 $O/l1.err; exit 1; }
ZSEEK_ONE_EXEC=wave timeout -k 10 400 python bench.py --steps 3 --warmup 1 --no-e2e --no-cpu-baseline --no-verify > $O/l2.json 2> $O/l2.err || { tail -5 $O/l2.err; exit 1; }
for f in l1 l2; do python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d['latency_4k_us'])"; done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python scripts/latency_probe.py 300 > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
tail -2 $O/probe.log
