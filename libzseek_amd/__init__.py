"""libzseek_amd — MI355X-native random-access decode path of libzseek.

The product is the C-ABI shared library ``libzseek_amd/lib/libzseek.so``
(include/zseek.h + include/zseek_hip.h); this package is its Python host
mirror (``libzseek_amd.zseek``) used by tests and bench.py.
"""
from .zseek import (  # noqa: F401
    ZSEEK_LZ4, ZSEEK_ZSTD, FRAME_DESC_DTYPE, COMPRESS_DESC_DTYPE, LibraryNotBuilt, Reader, Writer, ZseekError,
    decode_frames, frame_batch, kernel_times, kernel_timing, lib, lz4_seekable, parse_kernel_name,
    seek_table_of, status_string, lz4_compress_bound, lz4_compress_frames, lz4_compress_layout,
    lz4_compress_scratch_size,
    synth_buffer, tools, verify_frame_checksums, with_frame_checksums, zstd_decode_frames,
    zstd_seekable, zstd_tool_version,
)
