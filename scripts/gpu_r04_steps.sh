# round 4: why bench.py's config-2 step (3.72 ms) is longer than the kernel
# trace's (3.57 ms): kbench's variant 0 (tuning build, event pair around 3
# launches) and bench.py with the product and with the tuning library.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04steps
mkdir -p $O
timeout -k 10 300 python scripts/kbench.py --variants 0 --rounds 5 > $O/kb.log 2>&1 || { tail -20 $O/kb.log; exit 1; }
grep median $O/kb.log
timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --no-verify --no-latency > $O/b1.json 2> $O/b1.err || { tail -5 $O/b1.err; exit 1; }
ZSEEK_AMD_LIB=$PWD/libzseek_amd/lib/libzseek_tune.so timeout -k 10 300 python bench.py --steps 20 --warmup 3 --no-e2e --no-cpu-baseline --no-verify --no-latency > $O/b2.json 2> $O/b2.err || { tail -5 $O/b2.err; exit 1; }
for f in b1 b2; do python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], d['ms_per_step'], {k:v['avg_ms'] for k,v in (r.get('stages') or {}).items()})"; done
# zstd's execute on the seven-wave 3,072-byte stage against the 4,096 one
timeout -k 10 400 python bench.py --codec zstd --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-verify --no-latency > $O/z1.json 2> $O/z1.err || { tail -5 $O/z1.err; exit 1; }
ZSEEK_ZSTD_STAGE=3072 timeout -k 10 400 python bench.py --codec zstd --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-verify --no-latency > $O/z2.json 2> $O/z2.err || { tail -5 $O/z2.err; exit 1; }
for f in z1 z2; do python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$f', d['value'], d['ms_per_step'])"; done
