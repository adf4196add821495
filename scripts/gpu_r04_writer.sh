# round 4: writer GPU mode end to end at 64 KiB and 1 MiB frames (staging
# growth only for linked frames), and the writer GPU tests
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r04writer
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_writer_compress.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/suite.log 2>&1 || { tail -30 $O/suite.log; exit 1; }
tail -1 $O/suite.log
timeout -k 10 400 python bench.py --codec lz4c --size 1073741824 --steps 2 --warmup 1 --no-cpu-baseline > $O/c64.json 2> $O/c64.err || { tail -5 $O/c64.err; exit 1; }
timeout -k 10 400 python bench.py --codec lz4c --frame 1048576 --size 1073741824 --steps 2 --warmup 1 --no-cpu-baseline > $O/c1m.json 2> $O/c1m.err || { tail -5 $O/c1m.err; exit 1; }
for f in c64 c1m; do python3 -c "
import json; d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]); print('$f', d['value'], d.get('writer_end_to_end'))"; done
