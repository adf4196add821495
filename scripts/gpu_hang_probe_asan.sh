# the probe against the host-ASan build of the library (GCC runtime; device code
# unsanitized; the harness's preload, if any, kept first)
export ASAN_OPTIONS=verify_asan_link_order=0:detect_leaks=0:halt_on_error=1:protect_shadow_gap=0
export LD_PRELOAD="${LD_PRELOAD:+$LD_PRELOAD:}/usr/lib/x86_64-linux-gnu/libasan.so.6"
export ZSEEK_AMD_LIB=$GRAFT_REPO_ROOT/libzseek_amd/lib/libzseek_asan.so
exec bash scripts/gpu_hang_probe.sh "$@"
