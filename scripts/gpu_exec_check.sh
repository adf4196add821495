# execute-kernel change: the whole GPU suite, then the default bench line
# (config 2) and config 5
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/xchk
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
for c in lz4 zstd lz4 zstd; do
timeout -k 10 300 python bench.py --codec $c --steps 10 --warmup 3 --no-e2e --no-cpu-baseline --no-latency > $O/b_$c.json 2> $O/b_$c.err || { tail -20 $O/b_$c.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/b_$c.json'));r=d['roofline'];print('$c', d['ms_per_step'], d['value'], d['verified_bit_exact'], {k: v['avg_ms'] for k, v in r['stages'].items()})"
done
