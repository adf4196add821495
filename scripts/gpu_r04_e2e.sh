# round 4: registered host destinations (direct D2H): GPU suite, then the
# config-2 bench line with its end-to-end figures (no CPU baseline).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04e2e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-latency > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['end_to_end'])"
