# round 4: linked frames compressed with the stream table in LDS: the
# compression GPU tests, then the 1 MiB and 64 KiB compression lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04lz4c
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_lz4_compress.py tests/test_gpu_writer_compress.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -2 $O/suite.log
timeout -k 10 400 python bench.py --codec lz4c --frame 1048576 --size 1073741824 --steps 3 --warmup 1 > $O/c1m.json 2> $O/c1m.err || { tail -5 $O/c1m.err; exit 1; }
timeout -k 10 400 python bench.py --codec lz4c --frame 1048576 --steps 3 --warmup 1 --no-cpu-baseline > $O/c1m4g.json 2> $O/c1m4g.err || { tail -5 $O/c1m4g.err; exit 1; }
for f in c1m c1m4g; do python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d.get('launch_by_frames'), (d.get('cpu_baseline') or {}).get('value'), d.get('writer_end_to_end'), d.get('verified_bit_exact'))"; done
