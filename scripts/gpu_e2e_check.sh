# reader pipeline change: the GPU suite, then end-to-end zseek_pread rates
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/e2e
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
for c in lz4 zstd; do
timeout -k 10 400 python bench.py --codec $c --steps 5 --warmup 2 --no-cpu-baseline --no-latency > $O/b_$c.json 2> $O/b_$c.err || { tail -20 $O/b_$c.err; exit 1; }
python3 -c "
import json;d=json.load(open('$O/b_$c.json'));print('$c', d['ms_per_step'], d['value'], d['end_to_end'])"
done
