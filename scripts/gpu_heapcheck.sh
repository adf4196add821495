# zstd GPU tests under glibc's malloc checker (host heap: a double free or a
# write past a block aborts at once with its stack; the harness's own preload,
# if any, is kept)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/heap
mkdir -p $O
export MALLOC_CHECK_=3 GLIBC_TUNABLES=glibc.malloc.tcache_count=0
export LD_PRELOAD="${LD_PRELOAD:+$LD_PRELOAD:}/usr/lib/x86_64-linux-gnu/libc_malloc_debug.so.0"
timeout -k 10 400 python -u -X faulthandler -m pytest -x -v tests/test_gpu_zstd.py > $O/tests.log 2>&1
rc=$?
tail -40 $O/tests.log
exit $rc
