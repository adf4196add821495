# Chunk-parse bring-up: parity through the split decoder with the chunk parse,
# then parse / decoder A/B on config 2 (kbench variants: 79 default, 80 chunk
# parse for every frame, 81 scan parse for every frame, 82/83 plan + parse only).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
    -k "chunk or scanparse or split or None" 2>&1 | tee gpurun_out/chunk_pytest.log &&
timeout -k 10 300 python -u scripts/kbench.py --variants ${VARIANTS:-79,80,81,82,83} --rounds 3 --reps 3 ${KARGS} 2>&1 | tee gpurun_out/chunk_kbench.log
