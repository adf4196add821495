# round 4: two sequences per lean sub-step in production: GPU suite, the
# config-2 line, plan + parse variants (12 = production, 0x220 = one per sub-step)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04lean2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python scripts/kbench.py --variants 12,544,0 --rounds 5 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep "median\|bit-exact\|MISMATCH" $O/kb.log
timeout -k 10 400 python bench.py --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-latency > $O/c2.json 2> $O/c2.err || { tail -5 $O/c2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/c2.json').read().strip().splitlines()[-1]); r=d['roofline']; print(d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in r['stages'].items()}, d['verified_bit_exact'])"
