# round 4: the whole GPU suite, single-frame latency (LZ4 and zstd) and a
# bench line (end to end included) -- a check after host-side changes
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/check
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 300 python scripts/latency_probe.py 300 > $O/probe.log 2>&1 || { tail -5 $O/probe.log; exit 1; }
grep p50 $O/probe.log
timeout -k 10 300 python scripts/latency_probe.py 300 zstd > $O/probez.log 2>&1 || { tail -5 $O/probez.log; exit 1; }
grep p50 $O/probez.log
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.load(open('$O/bench.json')); print(d['ms_per_step'], d['value'], d.get('latency_4k_us'), d.get('end_to_end'))"
