# round 4: launches with no work trimmed (plan workgroups capped, hand-off
# and chunk kernels group frames per wave): GPU suite, then config 2 and the
# 4 KiB sweep line with a kernel trace of each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04empty
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-e2e --no-cpu-baseline > $O/c2.json 2> $O/c2.err && tail -c 300 $O/c2.json &&
timeout -k 10 400 python bench.py --frame 4096 --steps 5 --warmup 2 --no-e2e --no-cpu-baseline > $O/f4096.json 2> $O/f4096.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace4k -- python bench.py --frame 4096 --profile --steps 5 --warmup 1 > $O/trace4k.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -- python bench.py --profile --steps 5 --warmup 1 > $O/trace.log 2>&1
rc=$?
for f in c2 f4096; do python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in (r.get('stages') or {}).items()})"; done
exit $rc
