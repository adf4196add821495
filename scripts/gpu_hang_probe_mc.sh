# the probe under glibc's malloc checker (the harness's preload, if any, kept)
export MALLOC_CHECK_=3 GLIBC_TUNABLES=glibc.malloc.tcache_count=0
export LD_PRELOAD="${LD_PRELOAD:+$LD_PRELOAD:}/usr/lib/x86_64-linux-gnu/libc_malloc_debug.so.0"
exec bash scripts/gpu_hang_probe.sh "$@"
