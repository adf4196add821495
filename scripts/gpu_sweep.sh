# Config 3: LZ4 frame-size sweep (4 KiB / 64 KiB / 1 MiB frames on the 4 GiB
# synthetic), one bench line per frame size, each next to the reference CPU
# path on the same image.  Each GPU step has its own time limit; steps are
# chained with &&.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/sweep
mkdir -p $O
timeout -k 10 400 python bench.py --frame 4096 --steps 5 --warmup 2 --no-e2e > $O/f4096.json 2> $O/f4096.err && cat $O/f4096.json &&
timeout -k 10 400 python bench.py --frame 65536 --steps 5 --warmup 2 --no-e2e > $O/f65536.json 2> $O/f65536.err && cat $O/f65536.json &&
timeout -k 10 400 python bench.py --frame 1048576 --steps 5 --warmup 2 --no-e2e > $O/f1048576.json 2> $O/f1048576.err && cat $O/f1048576.json
