"""Python host mirror of the libzseek C API (include/zseek.h, include/zseek_hip.h).

Thin ctypes layer over the in-tree ``libzseek_amd/lib/libzseek.so``: the
class and method names follow the reference's reader/writer API
(/root/reference/src/zseek.h:225-443) — ``Reader.pread`` is ``zseek_pread``,
``Reader.stats`` is ``zseek_reader_stats`` and so on, with the same return
conventions (bytes returned may be short; -1 becomes ``ZseekError`` carrying
the library's 80-byte error string).  There is no Python or CPU fallback: if
the shared library is missing this module raises on import of the library.
"""
from __future__ import annotations

import ctypes as C
import os
from dataclasses import dataclass

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# ZSEEK_AMD_LIB: a tuning build (libzseek_tune.so, same exports plus A/B
# variants) for scripts/ A/B runs; the product library otherwise
LIB_PATH = os.environ.get("ZSEEK_AMD_LIB") or os.path.join(HERE, "lib", "libzseek.so")
TOOLS_PATH = os.path.join(HERE, "lib", "libzseek_tools.so")

ERRBUF = 80
ZSEEK_ZSTD, ZSEEK_LZ4 = 0, 1
ZSK_OK = 0
ZSK_ERR_SEEK_CHECKSUM = 104

WRITE_FN = C.CFUNCTYPE(C.c_bool, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p)
PREAD_FN = C.CFUNCTYPE(C.c_ssize_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_void_p)
FSIZE_FN = C.CFUNCTYPE(C.c_ssize_t, C.c_void_p, C.c_void_p)


class ZseekError(RuntimeError):
    """A libzseek call failed; ``str(err)`` is the library's error buffer."""


class LibraryNotBuilt(ImportError):
    pass


class WriteFile(C.Structure):
    _fields_ = [("user_data", C.c_void_p), ("write", WRITE_FN)]


class ReadFile(C.Structure):
    _fields_ = [("user_data", C.c_void_p), ("pread", PREAD_FN), ("fsize", FSIZE_FN)]


class ZstdParam(C.Structure):
    _fields_ = [("nb_workers", C.c_int), ("cpusetsize", C.c_size_t), ("cpuset", C.c_void_p),
                ("compression_level", C.c_int), ("strategy", C.c_int)]


class Lz4Param(C.Structure):
    _fields_ = [("compression_level", C.c_int)]


class ParamUnion(C.Union):
    _fields_ = [("zstd_params", ZstdParam), ("lz4_params", Lz4Param)]


class CompressionParam(C.Structure):
    _fields_ = [("type", C.c_int), ("params", ParamUnion)]


class ReaderStatsC(C.Structure):
    _fields_ = [(n, C.c_size_t) for n in ("seek_table_memory", "frames", "decompressed_size",
                                          "cache_memory", "cached_frames", "buffer_size")]


class WriterStatsC(C.Structure):
    _fields_ = [(n, C.c_size_t) for n in ("seek_table_size", "seek_table_memory", "frames",
                                          "compressed_size", "buffer_size")]


class GpuStatsC(C.Structure):
    _fields_ = [("batches", C.c_uint64), ("frames_decoded", C.c_uint64),
                ("bytes_decoded", C.c_uint64), ("bytes_uploaded", C.c_uint64),
                ("device_memory", C.c_uint64), ("device", C.c_int), ("copy_threads", C.c_int),
                ("io_parts", C.c_int)]


# zsk_frame_desc_t
FRAME_DESC_DTYPE = np.dtype([("c_off", "<u8"), ("d_off", "<u8"), ("c_size", "<u4"),
                             ("d_size", "<u4")])
assert FRAME_DESC_DTYPE.itemsize == 24
# zsk_compress_desc_t (include/zseek_hip.h)
COMPRESS_DESC_DTYPE = np.dtype([("src_off", "<u8"), ("dst_off", "<u8"), ("src_size", "<u4"),
                                ("flags", "<u4")])
assert COMPRESS_DESC_DTYPE.itemsize == 24
COMPRESS_CONTENT_SIZE = 1

# exported C symbols that include/zseek.h and include/zseek_hip.h declare
EXPORTED = [
    "zseek_writer_open_full", "zseek_writer_open", "zseek_writer_close", "zseek_write",
    "zseek_writer_stats", "zseek_reader_open_full", "zseek_reader_open", "zseek_reader_close",
    "zseek_pread", "zseek_read", "zseek_reader_stats",
    "zsk_lz4_decode_frames", "zsk_lz4_decode_frames_ex", "zsk_status_string", "zsk_lz4_kernel_name",
    "zsk_lz4_parse_kernel_name", "zsk_reader_frames", "zsk_reader_type",
    "zsk_pread_device", "zsk_reader_gpu_stats", "zsk_reader_gpu_stats_ex", "zsk_reader_set_batch_bytes",
    "zsk_kernel_timing", "zsk_kernel_times", "zsk_zstd_decode_frames",
    "zsk_verify_frame_checksums", "zsk_reader_set_verify_checksums",
    "zsk_reader_set_devices", "zsk_reader_devices", "zsk_reader_set_io_threads",
    "zsk_lz4_compress_scratch_size", "zsk_lz4_compress_frames", "zsk_writer_set_gpu_compress",
]

_lib = None
_tools = None


def lib() -> C.CDLL:
    """Load libzseek.so (once).  Raises LibraryNotBuilt when it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LibraryNotBuilt(f"{LIB_PATH} not built: run __graft_entry__.build() "
                              "(make -C libzseek_amd/csrc)")
    L = C.CDLL(LIB_PATH)
    L.zseek_writer_open_full.restype = C.c_void_p
    L.zseek_writer_open_full.argtypes = [WriteFile, C.POINTER(CompressionParam), C.c_size_t,
                                         C.c_void_p, C.c_char_p]
    L.zseek_write.restype = C.c_bool
    L.zseek_write.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_char_p]
    L.zseek_writer_close.restype = C.c_bool
    L.zseek_writer_close.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p]
    L.zseek_writer_stats.restype = C.c_bool
    L.zseek_writer_stats.argtypes = [C.c_void_p, C.POINTER(WriterStatsC), C.c_char_p]
    L.zseek_reader_open_full.restype = C.c_void_p
    L.zseek_reader_open_full.argtypes = [ReadFile, C.c_size_t, C.c_void_p, C.c_char_p]
    L.zseek_reader_close.restype = C.c_bool
    L.zseek_reader_close.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p]
    L.zseek_pread.restype = C.c_ssize_t
    L.zseek_pread.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p,
                              C.c_char_p]
    L.zseek_read.restype = C.c_ssize_t
    L.zseek_read.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_char_p]
    L.zseek_reader_stats.restype = C.c_bool
    L.zseek_reader_stats.argtypes = [C.c_void_p, C.POINTER(ReaderStatsC), C.c_char_p]
    L.zsk_lz4_decode_frames.restype = C.c_int
    L.zsk_lz4_decode_frames.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_void_p]
    L.zsk_zstd_decode_frames.restype = C.c_int
    L.zsk_zstd_decode_frames.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                         C.c_void_p, C.c_void_p]
    L.zsk_lz4_decode_frames_ex.restype = C.c_int
    L.zsk_lz4_decode_frames_ex.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.c_int]
    L.zsk_lz4_kernel_name.restype = C.c_char_p
    L.zsk_lz4_kernel_name.argtypes = [C.c_uint32]
    L.zsk_lz4_parse_kernel_name.restype = C.c_char_p
    L.zsk_lz4_parse_kernel_name.argtypes = [C.c_uint32, C.c_uint32]
    L.zsk_kernel_timing.restype = C.c_int
    L.zsk_kernel_timing.argtypes = [C.c_int]
    L.zsk_kernel_times.restype = C.c_int
    L.zsk_kernel_times.argtypes = [C.POINTER(C.c_double), C.c_int]
    L.zsk_status_string.restype = C.c_char_p
    L.zsk_status_string.argtypes = [C.c_int32]
    L.zsk_reader_frames.restype = C.c_ssize_t
    L.zsk_reader_frames.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p]
    L.zsk_reader_type.restype = C.c_int
    L.zsk_reader_type.argtypes = [C.c_void_p]
    L.zsk_pread_device.restype = C.c_ssize_t
    L.zsk_pread_device.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p,
                                   C.c_char_p]
    L.zsk_reader_gpu_stats.restype = C.c_bool
    L.zsk_reader_gpu_stats.argtypes = [C.c_void_p, C.POINTER(GpuStatsC)]
    L.zsk_reader_gpu_stats_ex.restype = C.c_bool
    L.zsk_reader_gpu_stats_ex.argtypes = [C.c_void_p, C.POINTER(GpuStatsC), C.c_size_t]
    L.zsk_reader_set_batch_bytes.restype = C.c_bool
    L.zsk_reader_set_batch_bytes.argtypes = [C.c_void_p, C.c_size_t]
    L.zsk_verify_frame_checksums.restype = C.c_int
    L.zsk_verify_frame_checksums.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                             C.c_void_p, C.c_void_p]
    L.zsk_reader_set_verify_checksums.restype = C.c_bool
    L.zsk_reader_set_verify_checksums.argtypes = [C.c_void_p, C.c_bool]
    L.zsk_reader_set_devices.restype = C.c_bool
    L.zsk_reader_set_devices.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int]
    L.zsk_reader_set_io_threads.restype = C.c_bool
    L.zsk_reader_set_io_threads.argtypes = [C.c_void_p, C.c_int]
    L.zsk_reader_devices.restype = C.c_int
    L.zsk_reader_devices.argtypes = [C.c_void_p, C.POINTER(C.c_int), C.c_int]
    L.zsk_writer_set_gpu_compress.restype = C.c_bool
    L.zsk_writer_set_gpu_compress.argtypes = [C.c_void_p, C.c_size_t]
    L.zsk_lz4_compress_scratch_size.restype = C.c_size_t
    L.zsk_lz4_compress_scratch_size.argtypes = [C.c_uint32]
    L.zsk_lz4_compress_frames.restype = C.c_int
    L.zsk_lz4_compress_frames.argtypes = [C.c_void_p, C.c_uint32, C.c_void_p, C.c_void_p,
                                          C.c_void_p, C.c_int, C.c_void_p, C.c_void_p]
    _lib = L
    return L


def tools() -> C.CDLL:
    """Bench/test input helpers (libzseek_tools.so)."""
    global _tools
    if _tools is not None:
        return _tools
    if not os.path.exists(TOOLS_PATH):
        raise LibraryNotBuilt(f"{TOOLS_PATH} not built")
    T = C.CDLL(TOOLS_PATH)
    T.zsk_tool_install_backtrace.restype = C.c_int
    T.zsk_tool_install_backtrace.argtypes = []
    T.zsk_tool_synth.restype = None
    T.zsk_tool_synth.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    T.zsk_tool_gen.restype = None
    T.zsk_tool_gen.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
    T.zsk_tool_lz4_seekable_bound.restype = C.c_size_t
    T.zsk_tool_lz4_seekable_bound.argtypes = [C.c_size_t, C.c_size_t]
    T.zsk_tool_lz4_seekable.restype = C.c_int
    T.zsk_tool_lz4_seekable.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_int, C.c_int,
                                        C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
    T.zsk_tool_zstd_version.restype = C.c_uint
    T.zsk_tool_zstd_version.argtypes = []
    T.zsk_tool_zstd_seekable_bound.restype = C.c_size_t
    T.zsk_tool_zstd_seekable_bound.argtypes = [C.c_size_t, C.c_size_t]
    T.zsk_tool_zstd_seekable.restype = C.c_int
    T.zsk_tool_zstd_seekable.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_int, C.c_int,
                                         C.c_int, C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
    T.zsk_tool_lz4_seekable_ex.restype = C.c_int
    T.zsk_tool_lz4_seekable_ex.argtypes = [C.c_void_p, C.c_size_t, C.c_size_t, C.c_int, C.c_int,
                                           C.c_int, C.c_int, C.c_int, C.c_int, C.c_uint, C.c_int,
                                           C.c_void_p, C.c_size_t, C.POINTER(C.c_size_t)]
    T.zsk_tool_open_mem.restype = C.c_void_p
    T.zsk_tool_open_mem.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_char_p]
    T.zsk_tool_close_mem.restype = C.c_bool
    T.zsk_tool_close_mem.argtypes = [C.c_void_p, C.c_void_p]
    T.zsk_tool_latency.restype = C.c_int
    T.zsk_tool_latency.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t,
                                   C.c_void_p, C.c_void_p, C.POINTER(C.c_size_t)]
    T.zsk_tool_read_all.restype = C.c_double
    T.zsk_tool_read_all.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_size_t,
                                    C.POINTER(C.c_size_t)]
    _tools = T
    return T


def status_string(status: int) -> str:
    return lib().zsk_status_string(status).decode()


def parse_kernel_name(nframes: int, c_size: int) -> str:
    """The parse kernel the library routes a frame of c_size compressed bytes
    to in a batch of nframes frames (zsk_lz4_parse_kernel_name)."""
    return lib().zsk_lz4_parse_kernel_name(nframes, c_size).decode()


# ---------------------------------------------------------------------------
# inputs (bench tooling)
# ---------------------------------------------------------------------------
def synth_buffer(n: int, threads: int = 16) -> np.ndarray:
    """SURVEY.md §8d buffer(N) (64 MiB chunks, seed = 1 + chunk)."""
    out = np.empty(n, np.uint8)
    tools().zsk_tool_synth(out.ctypes.data, n, threads)
    return out


def lz4_seekable(data: np.ndarray, frame_size: int, level: int = 0, threads: int = 16) -> np.ndarray:
    """Seekable LZ4 image of `data`, identical to the writer fed frame_size writes."""
    T = tools()
    cap = T.zsk_tool_lz4_seekable_bound(data.size, frame_size)
    out = np.empty(cap, np.uint8)
    n = C.c_size_t(0)
    if T.zsk_tool_lz4_seekable(data.ctypes.data, data.size, frame_size, level, threads,
                               out.ctypes.data, cap, C.byref(n)) != 0:
        raise ZseekError("lz4 seekable compression failed")
    return out[: n.value]


def lz4_seekable_ex(data: np.ndarray, frame_size: int, *, level: int = 0, bsid: int = 4,
                    independent: bool = False, content_checksum: bool = False,
                    block_checksum: bool = False, content_size: bool = False, dict_id: int = 0,
                    threads: int = 16) -> np.ndarray:
    """Seekable LZ4 image with LZ4F frame options the reference writer never
    sets but its reader accepts (block size id 4..7, linked / independent
    blocks, content / block checksums, content size, dictID)."""
    T = tools()
    data = np.ascontiguousarray(data, dtype=np.uint8)
    nf = max(1, -(-data.size // frame_size))
    cap = nf * (frame_size + frame_size // 64 + (1 << 16)) + 8 * nf + 64
    out = np.empty(cap, np.uint8)
    n = C.c_size_t(0)
    if T.zsk_tool_lz4_seekable_ex(data.ctypes.data, data.size, frame_size, level, bsid,
                                  int(independent), int(content_checksum), int(block_checksum),
                                  int(content_size), dict_id, threads, out.ctypes.data, cap,
                                  C.byref(n)) != 0:
        raise ZseekError("lz4 seekable compression failed")
    return out[: n.value]


def zstd_tool_version() -> str:
    """The libzstd zstd_seekable compresses with ("1.4.9": the reference
    writer's pinned version)."""
    v = int(tools().zsk_tool_zstd_version())
    return f"{v // 10000}.{v // 100 % 100}.{v % 100}"


def zstd_seekable(data: np.ndarray, frame_size: int, level: int = 3, strategy: int = 1,
                  threads: int = 16) -> np.ndarray:
    T = tools()
    cap = T.zsk_tool_zstd_seekable_bound(data.size, frame_size)
    out = np.empty(cap, np.uint8)
    n = C.c_size_t(0)
    if T.zsk_tool_zstd_seekable(data.ctypes.data, data.size, frame_size, level, strategy,
                                threads, out.ctypes.data, cap, C.byref(n)) != 0:
        raise ZseekError("zstd seekable compression failed")
    return out[: n.value]


# ---------------------------------------------------------------------------
# writer (zseek_writer_*)
# ---------------------------------------------------------------------------
class Writer:
    """zseek_writer over an in-memory sink (``getvalue()`` returns the file)."""

    def __init__(self, ctype: int = ZSEEK_LZ4, min_frame_size: int = 1 << 20,
                 level: int | None = None, strategy: int = 1, nb_workers: int = 1,
                 fail_on_callback: int | None = None):
        self._out = bytearray()
        self.callbacks = 0          # write callbacks so far
        self.call_data_seen = []    # call_data of each callback (None or int)

        def _w(ptr, size, ud, cd):
            self.callbacks += 1
            self.call_data_seen.append(cd)
            if fail_on_callback is not None and self.callbacks == fail_on_callback:
                return False
            self._out.extend(C.string_at(ptr, size))
            return True

        self._cb = WRITE_FN(_w)
        p = CompressionParam()
        p.type = ctype
        if ctype == ZSEEK_LZ4:
            p.params.lz4_params.compression_level = 0 if level is None else level
        else:
            p.params.zstd_params.nb_workers = nb_workers
            p.params.zstd_params.compression_level = 3 if level is None else level
            p.params.zstd_params.strategy = strategy
        self._err = C.create_string_buffer(ERRBUF)
        self._h = lib().zseek_writer_open_full(WriteFile(None, self._cb), C.byref(p),
                                               min_frame_size, None, self._err)
        if not self._h:
            raise ZseekError(self._err.value.decode())

    def write(self, data, call_data: int | None = None) -> None:
        b = bytes(data)
        buf = C.create_string_buffer(b, max(len(b), 1))
        if not lib().zseek_write(self._h, buf, len(b), call_data, self._err):
            raise ZseekError(self._err.value.decode())

    def set_gpu_compress(self, batch_bytes: int = 0) -> bool:
        """zsk_writer_set_gpu_compress: LZ4 frames of <= 4 MiB compressed on
        the GPU in batches (0 = 1 GiB, -1 = off)."""
        return bool(lib().zsk_writer_set_gpu_compress(self._h, batch_bytes & ((1 << 64) - 1)))

    def stats(self) -> dict:
        s = WriterStatsC()
        if not lib().zseek_writer_stats(self._h, C.byref(s), self._err):
            raise ZseekError(self._err.value.decode())
        return {k: getattr(s, k) for k, _ in WriterStatsC._fields_}

    def close(self) -> bytes:
        if self._h:
            ok = lib().zseek_writer_close(self._h, None, self._err)
            self._h = None
            if not ok:
                raise ZseekError(self._err.value.decode())
        return bytes(self._out)


# ---------------------------------------------------------------------------
# reader (zseek_reader_*, zseek_pread, zsk_* GPU extensions)
# ---------------------------------------------------------------------------
class Reader:
    """zseek_reader over an in-memory file image (bytes / numpy uint8)."""

    def __init__(self, image, cache_size: int = 0):
        arr = np.frombuffer(image, np.uint8) if isinstance(image, (bytes, bytearray)) else image
        self.image = np.ascontiguousarray(arr, dtype=np.uint8)
        self.size = self.image.size
        base = self.image.ctypes.data
        self.npreads = 0

        def _pread(ptr, size, offset, ud, cd):
            self.npreads += 1
            if offset >= self.size:
                return 0
            n = min(size, self.size - offset)
            C.memmove(ptr, base + offset, n)
            return n

        def _fsize(ud, cd):
            return self.size

        self._cbs = (PREAD_FN(_pread), FSIZE_FN(_fsize))
        self._err = C.create_string_buffer(ERRBUF)
        self._h = lib().zseek_reader_open_full(ReadFile(None, *self._cbs), cache_size, None,
                                               self._err)
        if not self._h:
            raise ZseekError(self._err.value.decode())

    @property
    def error(self) -> str:
        return self._err.value.decode(errors="replace")

    @property
    def handle(self):
        return self._h

    def pread_raw(self, buf_ptr: int, count: int, offset: int) -> int:
        """zseek_pread into raw memory; returns the C return value."""
        return lib().zseek_pread(self._h, buf_ptr, count, offset, None, self._err)

    def pread(self, count: int, offset: int) -> bytes:
        out = np.empty(max(count, 1), np.uint8)
        r = self.pread_raw(out.ctypes.data, count, offset)
        if r < 0:
            raise ZseekError(self.error)
        return out[:r].tobytes()

    def read_all(self, count: int, offset: int, chunk: int | None = None) -> bytes:
        """Loop zseek_pread until `count` bytes or EOF (what callers do)."""
        out = np.empty(max(count, 1), np.uint8)
        done = 0
        while done < count:
            want = count - done if chunk is None else min(chunk, count - done)
            r = self.pread_raw(out.ctypes.data + done, want, offset + done)
            if r < 0:
                raise ZseekError(self.error)
            if r == 0:
                break
            done += r
        return out[:done].tobytes()

    def read(self, count: int) -> bytes:
        out = np.empty(max(count, 1), np.uint8)
        r = lib().zseek_read(self._h, out.ctypes.data, count, None, self._err)
        if r < 0:
            raise ZseekError(self.error)
        return out[:r].tobytes()

    def pread_device(self, dev_ptr: int, count: int, offset: int) -> int:
        r = lib().zsk_pread_device(self._h, dev_ptr, count, offset, None, self._err)
        if r < 0:
            raise ZseekError(self.error)
        return r

    def stats(self) -> dict:
        s = ReaderStatsC()
        if not lib().zseek_reader_stats(self._h, C.byref(s), self._err):
            raise ZseekError(self.error)
        return {k: getattr(s, k) for k, _ in ReaderStatsC._fields_}

    def gpu_stats(self) -> dict:
        s = GpuStatsC()
        lib().zsk_reader_gpu_stats_ex(self._h, C.byref(s), C.sizeof(s))
        return {k: getattr(s, k) for k, _ in GpuStatsC._fields_}

    def frames(self):
        """(c_off, d_off) prefix sums, n+1 entries each."""
        n = lib().zsk_reader_frames(self._h, None, None)
        c_off = np.zeros(n + 1, np.uint64)
        d_off = np.zeros(n + 1, np.uint64)
        lib().zsk_reader_frames(self._h, c_off.ctypes.data, d_off.ctypes.data)
        return c_off, d_off

    @property
    def type(self) -> int:
        return lib().zsk_reader_type(self._h)

    def set_batch_bytes(self, n: int) -> None:
        lib().zsk_reader_set_batch_bytes(self._h, n)

    def set_devices(self, devices) -> None:
        """zsk_reader_set_devices: one decode lane per entry (may repeat)."""
        arr = (C.c_int * len(devices))(*devices)
        if not lib().zsk_reader_set_devices(self._h, arr, len(devices)):
            raise ZseekError("invalid device list")

    def set_io_threads(self, n: int) -> None:
        """zsk_reader_set_io_threads: concurrent pread callbacks (this class's
        in-memory callback is safe for it)."""
        if not lib().zsk_reader_set_io_threads(self._h, n):
            raise ZseekError("invalid io thread count")

    def devices(self) -> list:
        n = lib().zsk_reader_devices(self._h, None, 0)
        arr = (C.c_int * max(n, 1))()
        lib().zsk_reader_devices(self._h, arr, n)
        return list(arr[:n])

    def set_verify_checksums(self, on: bool = True) -> None:
        """zsk_reader_set_verify_checksums: check seek-table frame checksums."""
        lib().zsk_reader_set_verify_checksums(self._h, bool(on))

    def close(self) -> None:
        if self._h:
            lib().zseek_reader_close(self._h, None, self._err)
            self._h = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ---------------------------------------------------------------------------
# device batch API (zsk_lz4_decode_frames) on torch tensors
# ---------------------------------------------------------------------------
@dataclass
class FrameBatch:
    """Descriptors for decoding frames [f0, f1) of a seek table in one grid."""
    desc: np.ndarray       # FRAME_DESC_DTYPE, one per frame
    comp_begin: int        # compressed byte range of the batch in the file
    comp_end: int
    out_bytes: int         # decoded bytes of the batch


def frame_batch(c_off: np.ndarray, d_off: np.ndarray, f0: int, f1: int) -> FrameBatch:
    d = np.empty(f1 - f0, FRAME_DESC_DTYPE)
    d["c_off"] = c_off[f0:f1] - c_off[f0]
    d["d_off"] = d_off[f0:f1] - d_off[f0]
    d["c_size"] = (c_off[f0 + 1:f1 + 1] - c_off[f0:f1]).astype(np.uint32)
    d["d_size"] = (d_off[f0 + 1:f1 + 1] - d_off[f0:f1]).astype(np.uint32)
    return FrameBatch(d, int(c_off[f0]), int(c_off[f1]), int(d_off[f1] - d_off[f0]))


def seek_table_of(image: np.ndarray):
    """(c_off, d_off) of an in-memory seekable file, parsed by the library."""
    r = Reader(image, 0)
    try:
        return r.frames()
    finally:
        r.close()


# The library's production decoders, forced for every frame through
# zsk_lz4_decode_frames_ex (ZSK_DECODER_*): each one complete incl. hand-offs.
DECODERS = {"auto": 0, "wave": 1, "lean": 2, "scan": 3, "chunk": 4, "block": 5, "one": 6}


def decode_frames(desc, comp, out, status, stream: int | None = None,
                  engine: str | None = None) -> None:
    """Launch zsk_lz4_decode_frames on torch CUDA(HIP) tensors (async).

    desc: uint8 tensor holding N x 24-byte zsk_frame_desc_t; comp / out: uint8
    tensors; status: int32 tensor of N.  `stream` is a raw hipStream_t
    (torch.cuda.Stream.cuda_stream); None = the current torch stream.
    `engine` forces one production decoder (DECODERS; None = the library's
    choice).
    """
    import torch
    n = status.numel()
    if desc.numel() != n * 24:
        raise ValueError("desc must hold 24 bytes per frame")
    for t in (desc, comp, out, status):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("decode_frames needs contiguous device tensors")
    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    if engine is None:
        rc = lib().zsk_lz4_decode_frames(desc.data_ptr(), n, comp.data_ptr(), out.data_ptr(),
                                         status.data_ptr(), stream)
    else:
        rc = lib().zsk_lz4_decode_frames_ex(desc.data_ptr(), n, comp.data_ptr(), out.data_ptr(),
                                            status.data_ptr(), stream, DECODERS[engine])
    if rc != 0:
        raise ZseekError("zsk_lz4_decode_frames launch failed")


def zstd_decode_frames(desc, comp, out, status, stream: int | None = None) -> None:
    """zsk_zstd_decode_frames on torch device tensors (same layout as
    decode_frames; synchronizes the stream once, after its planning kernel)."""
    import torch
    n = status.numel()
    if desc.numel() != n * 24:
        raise ValueError("desc must hold 24 bytes per frame")
    for t in (desc, comp, out, status):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("zstd_decode_frames needs contiguous device tensors")
    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    rc = lib().zsk_zstd_decode_frames(desc.data_ptr(), n, comp.data_ptr(), out.data_ptr(),
                                      status.data_ptr(), stream)
    if rc != 0:
        raise ZseekError("zsk_zstd_decode_frames launch failed")


def verify_frame_checksums(desc, out, checksums, status, stream: int | None = None) -> None:
    """zsk_verify_frame_checksums on torch device tensors (async): checksums
    holds N expected XXH64-low-32 values (int32/uint32); a frame whose status
    is ZSK_OK and whose decoded bytes hash differently gets
    ZSK_ERR_SEEK_CHECKSUM."""
    import torch
    n = status.numel()
    if desc.numel() != n * 24 or checksums.numel() != n:
        raise ValueError("desc must hold 24 bytes and checksums one value per frame")
    for t in (desc, out, checksums, status):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("verify_frame_checksums needs contiguous device tensors")
    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    if lib().zsk_verify_frame_checksums(desc.data_ptr(), n, out.data_ptr(), checksums.data_ptr(),
                                        status.data_ptr(), stream) != 0:
        raise ZseekError("zsk_verify_frame_checksums launch failed")


def lz4_compress_bound(n: int) -> int:
    """ZSK_LZ4_COMPRESS_BOUND: output slot bytes for a frame of n bytes."""
    return (n + 24 + 15) & ~15


def lz4_compress_layout(sizes, src_offsets=None, flags=None) -> tuple[np.ndarray, int]:
    """Descriptors for zsk_lz4_compress_frames: frame f reads
    src[src_offsets[f], +sizes[f]) (default: the frames back to back) and
    writes its slot at a 16-byte aligned dst_off.  -> (COMPRESS_DESC_DTYPE
    array, dst bytes needed)."""
    sizes = np.asarray(sizes, np.uint64)
    n = sizes.size
    d = np.zeros(n, COMPRESS_DESC_DTYPE)
    d["src_size"] = sizes
    if src_offsets is None:
        src_offsets = np.concatenate(([0], np.cumsum(sizes)[:-1])) if n else sizes
    d["src_off"] = src_offsets
    slots = (sizes + 4 * (sizes >> np.uint64(16)) + 24 + 15) & ~np.uint64(15)   # ZSK_LZ4_COMPRESS_BOUND
    d["dst_off"] = np.concatenate(([0], np.cumsum(slots)[:-1])) if n else slots
    if flags is not None:
        d["flags"] = flags
    return d, int(slots.sum())


def lz4_compress_scratch_size(nframes: int) -> int:
    return int(lib().zsk_lz4_compress_scratch_size(nframes))


def lz4_compress_frames(desc, src, dst, csize, level: int = 0, scratch=None,
                        stream: int | None = None) -> None:
    """zsk_lz4_compress_frames on torch device tensors (async on the current
    stream): desc = COMPRESS_DESC_DTYPE bytes (uint8), src / dst uint8,
    csize one int32 per frame (frame sizes out; 0 = refused descriptor)."""
    import torch
    n = csize.numel()
    if desc.numel() != n * 24:
        raise ValueError("desc must hold 24 bytes per frame")
    if scratch is None:
        scratch = torch.empty(max(lz4_compress_scratch_size(n), 1), dtype=torch.uint8,
                              device=csize.device)
    for t in (desc, src, dst, csize, scratch):
        if not t.is_cuda or not t.is_contiguous():
            raise ValueError("lz4_compress_frames needs contiguous device tensors")
    if scratch.numel() < lz4_compress_scratch_size(n):
        raise ValueError("scratch too small")
    if stream is None:
        stream = torch.cuda.current_stream().cuda_stream
    if lib().zsk_lz4_compress_frames(desc.data_ptr(), n, src.data_ptr(), dst.data_ptr(),
                                     csize.data_ptr(), level, scratch.data_ptr(), stream) != 0:
        raise ZseekError("zsk_lz4_compress_frames launch failed")


def with_frame_checksums(image, checksums) -> np.ndarray:
    """Copy of a seekable image whose seek table carries per-frame checksums
    (descriptor bit 7; 12-byte entries cSize, dSize, checksum - the layout
    ZSTD_seekable_writeSeekTable writes, /root/reference/src/seek_table.c:365-419).
    `checksums`: one value per frame (low 32 bits kept)."""
    import struct
    img = np.frombuffer(image, np.uint8) if isinstance(image, (bytes, bytearray)) else image
    img = np.ascontiguousarray(img, dtype=np.uint8)
    c_off, d_off = seek_table_of(img)
    n = len(c_off) - 1
    ent = np.empty((n, 3), "<u4")
    ent[:, 0] = np.diff(c_off)
    ent[:, 1] = np.diff(d_off)
    ent[:, 2] = np.asarray(checksums, np.uint64) & 0xFFFFFFFF
    body = ent.tobytes()
    foot = (struct.pack("<II", 0x184D2A5E, len(body) + 9) + body +
            struct.pack("<IBI", n, 0x80, 0x8F92EAB1))
    return np.concatenate([img[: int(c_off[n])], np.frombuffer(foot, np.uint8)])


STAGES = ("plan", "parse", "execute", "hand-off")


def kernel_timing(on: bool) -> None:
    """Switch per-stage event timing of the two-phase decoder (and clear it)."""
    lib().zsk_kernel_timing(1 if on else 0)


ZSTD_KERNEL_SPANS = ("zstd_frame_kernel", "zstd_seq_kernel", "zstd_huf_kernel", "seq_exec_kernel")


def kernel_times(spans: bool = False) -> tuple[int, dict]:
    """(launches recorded, {stage: median ms}) since kernel_timing(True);
    spans=True adds the zstd per-kernel spans (summed over a launch's
    chunks, each on its own stream)."""
    ms = (C.c_double * 8)()
    n = lib().zsk_kernel_times(ms, 8)
    out = {k: float(ms[i]) for i, k in enumerate(STAGES)}
    if spans:
        out.update({k: float(ms[4 + i]) for i, k in enumerate(ZSTD_KERNEL_SPANS)})
    return n, out
