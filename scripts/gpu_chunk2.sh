# Chunk parse where the lane-per-frame scan lacks frames: 1 MiB frames (config 3)
# and 256 MiB batches of 64 KiB frames (the reader's batch), vs the wave kernel (20).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u scripts/kbench.py --frame 1048576 --variants 20,80,82 --rounds 3 --reps 2 2>&1 | tee gpurun_out/chunk2_1m.log &&
timeout -k 10 120 python -u scripts/kbench.py --size 268435456 --variants 20,80,81,82,83 --rounds 3 --reps 3 2>&1 | tee gpurun_out/chunk2_256m.log
