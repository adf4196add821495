"""ctypes front-end to the CPU oracle — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker.  The product (libzseek_amd) never does.

Two backends:
  * ``Oracle``     — our C restatement (oracle/build/liboracle.so): LZ4-frame
                     decode, seek-table parse, XXH32/64, the §8d synthetic.
  * ``RefZseek``   — the reference library itself (oracle/_ref/libzseek_ref.so,
                     compiled from /root/reference/src by oracle/Makefile),
                     driven through its public zseek.h API.

``pread_model`` restates the reference reader's per-call semantics
(/root/reference/src/decompress.c:576-804): a call returns at most the rest of
ONE frame; offset >= size -> 0.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "build", "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libzseek_ref.so")
REF_BENCH_SO = os.path.join(HERE, "_ref", "libref_bench.so")

# LZ4F error names, lz4frame.h LZ4F_LIST_ERRORS order (liblz4 1.9.3).
LZ4F_ERROR_NAMES = [
    "OK_NoError", "ERROR_GENERIC", "ERROR_maxBlockSize_invalid",
    "ERROR_blockMode_invalid", "ERROR_contentChecksumFlag_invalid",
    "ERROR_compressionLevel_invalid", "ERROR_headerVersion_wrong",
    "ERROR_blockChecksum_invalid", "ERROR_reservedFlag_set",
    "ERROR_allocation_failed", "ERROR_srcSize_tooLarge",
    "ERROR_dstMaxSize_tooSmall", "ERROR_frameHeader_incomplete",
    "ERROR_frameType_unknown", "ERROR_frameSize_wrong", "ERROR_srcPtr_wrong",
    "ERROR_decompressionFailed", "ERROR_headerChecksum_invalid",
    "ERROR_contentChecksum_invalid", "ERROR_frameDecoding_alreadyStarted",
]
ORC_ERROR_DST_OVERFLOW = 100
ORC_ERROR_SHORT_FRAME = 101
ORC_ERROR_TRUNCATED = 102

SYNTH_CHUNK = 64 << 20

# The reference's dependency pins (/root/reference/meson.build:10-11 floors;
# built against /opt/conda's liblz4 1.9.3 / libzstd 1.4.9).
REF_ZSTD_VERSION = 10409
REF_LZ4_VERSION = 10903

_RTLD_NOW = 2
_LM_ID_NEWLM = -1
_RTLD_DI_LMID = 1
_ref_lmid = None


def ref_cdll(path: str) -> C.CDLL:
    """Load a reference build (oracle/_ref/*.so) into the reference's OWN link
    namespace (dlmopen), shared by every reference library of this process.

    Loaded with a plain dlopen, libzseek_ref.so's DT_NEEDED libzstd.so.1 is
    satisfied by whichever libzstd.so.1 the process already mapped -- the
    system 1.4.8 our libzseek.so / libzseek_tools.so link -- so the reference
    would run against a libzstd it was not compiled for.  In its own namespace
    its RUNPATH (/opt/conda/lib) decides: liblz4 1.9.3 and libzstd 1.4.9, the
    versions SURVEY.md §8c pins.  The namespace has its own libc (and malloc
    arena); the reference never frees memory this process allocated, nor the
    reverse, so nothing crosses heaps."""
    global _ref_lmid
    libc = C.CDLL(None)
    libc.dlmopen.restype = C.c_void_p
    libc.dlmopen.argtypes = [C.c_long, C.c_char_p, C.c_int]
    libc.dlerror.restype = C.c_char_p
    libc.dlinfo.argtypes = [C.c_void_p, C.c_int, C.c_void_p]
    lmid = _LM_ID_NEWLM if _ref_lmid is None else _ref_lmid
    h = libc.dlmopen(lmid, os.fsencode(path), _RTLD_NOW)
    if not h:
        raise OSError(f"dlmopen {path}: {(libc.dlerror() or b'?').decode(errors='replace')}")
    if _ref_lmid is None:
        out = C.c_long(0)
        if libc.dlinfo(h, _RTLD_DI_LMID, C.byref(out)) != 0:
            raise OSError("dlinfo(RTLD_DI_LMID) failed")
        _ref_lmid = out.value
    return C.CDLL(os.path.basename(path), handle=h)


def ref_dependency_versions(lib: C.CDLL) -> dict:
    """The libzstd / liblz4 versions a reference library actually runs
    against (dlsym through its own dependency tree)."""
    lib.ZSTD_versionNumber.restype = C.c_uint
    lib.LZ4_versionNumber.restype = C.c_int
    return {"zstd": int(lib.ZSTD_versionNumber()), "lz4": int(lib.LZ4_versionNumber())}


def _u8p(buf):
    return C.cast(buf.ctypes.data, C.POINTER(C.c_uint8))


class Oracle:
    """Our scalar C restatement of the decode path."""

    def __init__(self, path: str = ORACLE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle restatement`")
        L = self.lib = C.CDLL(path)
        L.orc_xxh32.restype = C.c_uint32
        L.orc_xxh32.argtypes = [C.c_void_p, C.c_size_t, C.c_uint32]
        L.orc_xxh64.restype = C.c_uint64
        L.orc_xxh64.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.orc_lz4f_decode.restype = C.c_int
        L.orc_lz4f_decode.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                      C.POINTER(C.c_size_t), C.POINTER(C.c_size_t),
                                      C.POINTER(C.c_size_t), C.POINTER(C.c_int),
                                      C.POINTER(C.c_size_t)]
        L.orc_seek_table_parse.restype = C.c_int64
        L.orc_seek_table_parse.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p,
                                           C.c_void_p, C.c_void_p, C.POINTER(C.c_int)]
        L.orc_synth_gen.restype = None
        L.orc_synth_gen.argtypes = [C.c_void_p, C.c_size_t, C.c_uint64]
        L.orc_zstd_decode.restype = C.c_longlong
        L.orc_zstd_decode.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.orc_zstd_decode_at.restype = C.c_longlong
        L.orc_zstd_decode_at.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                         C.POINTER(C.c_size_t)]
        L.orc_huf_select_x2.restype = C.c_int
        L.orc_huf_select_x2.argtypes = [C.c_size_t, C.c_size_t]
        L.orc_huf_decompress.restype = C.c_long
        L.orc_huf_decompress.argtypes = [C.c_int, C.c_int, C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t]
        L.orc_zstd_x1_only.restype = None
        L.orc_zstd_x1_only.argtypes = [C.c_int]
        L.orc_lz4f_compress_frame.restype = C.c_longlong
        L.orc_lz4f_compress_frame.argtypes = [C.c_void_p, C.c_size_t, C.c_void_p, C.c_size_t,
                                              C.c_int, C.c_int]

    # -- LZ4 frame compression (the reference writer's, lz4c_oracle.c) ------
    def lz4f_compress_frame(self, data, level: int = 0, content_size: bool = False) -> bytes:
        """LZ4F_compressFrame(level, autoFlush, 64 KiB blocks) of one frame,
        as compress.c:750 / :483 call it (linked blocks above 64 KiB)."""
        s = np.frombuffer(bytes(data), np.uint8)
        out = np.empty(s.size + 4 * (s.size // 65536 + 1) + 32, np.uint8)
        r = self.lib.orc_lz4f_compress_frame(s.ctypes.data if s.size else None, s.size,
                                             out.ctypes.data, out.size, level, int(content_size))
        if r < 0:
            raise ValueError("orc_lz4f_compress_frame: unsupported input")
        return out[:r].tobytes()

    # -- hashes -----------------------------------------------------------
    def xxh32(self, data: bytes, seed: int = 0) -> int:
        b = np.frombuffer(data, np.uint8)
        return self.lib.orc_xxh32(b.ctypes.data, b.size, seed)

    def xxh64(self, data: bytes, seed: int = 0) -> int:
        b = np.frombuffer(data, np.uint8)
        return self.lib.orc_xxh64(b.ctypes.data, b.size, seed)

    # -- synthetic --------------------------------------------------------
    def synth(self, n: int, seed: int) -> np.ndarray:
        out = np.empty(n, np.uint8)
        self.lib.orc_synth_gen(out.ctypes.data, n, seed)
        return out

    def synth_buffer(self, n: int) -> np.ndarray:
        """SURVEY.md §8d buffer(N): concat of gen(64 MiB, seed=1+c) chunks."""
        out = np.empty(n, np.uint8)
        for c, start in enumerate(range(0, n, SYNTH_CHUNK)):
            m = min(SYNTH_CHUNK, n - start)
            self.lib.orc_synth_gen(out[start:].ctypes.data, m, 1 + c)
        return out

    # -- frames -----------------------------------------------------------
    def decode_frame(self, src: bytes, dst_cap: int):
        """-> (status, decoded bytes, src_used, info) with info = dict(fail_at,
        block_fail, max_block) describing where a failure happened."""
        s = np.frombuffer(src, np.uint8)
        d = np.empty(max(dst_cap, 1), np.uint8)
        dl, su, fa, mb = C.c_size_t(0), C.c_size_t(0), C.c_size_t(0), C.c_size_t(0)
        bf = C.c_int(0)
        st = self.lib.orc_lz4f_decode(s.ctypes.data, s.size, d.ctypes.data, dst_cap,
                                      C.byref(dl), C.byref(su), C.byref(fa), C.byref(bf),
                                      C.byref(mb))
        info = {"fail_at": fa.value, "block_fail": bool(bf.value), "max_block": mb.value}
        # a failed frame: the bytes of its blocks before the failing one
        return st, d[: dl.value if st == 0 else fa.value].tobytes(), su.value, info

    def zstd_decode(self, src: bytes, dst_cap: int):
        """ZSTD_decompressDCtx restated -> (decoded bytes, 0) or (b"", zstd error code)."""
        s = np.frombuffer(src, np.uint8)
        d = np.empty(max(dst_cap, 1), np.uint8)
        r = self.lib.orc_zstd_decode(s.ctypes.data, s.size, d.ctypes.data, dst_cap)
        if r < 0:
            return b"", -r
        return d[:r].tobytes(), 0

    def huf_select_x2(self, dst_size: int, csrc_size: int) -> bool:
        """HUF_selectDecoder restated: True = the double-symbol decoder (X2)."""
        return bool(self.lib.orc_huf_select_x2(dst_size, csrc_size))

    def huf_decompress(self, x2: bool, four: bool, src: bytes, cnt: int):
        """HUF_decompress{1,4}X{1,2}_DCtx restated -> (ok, cnt bytes written)."""
        s = np.frombuffer(src, np.uint8)
        d = np.zeros(cnt + 64, np.uint8)
        r = self.lib.orc_huf_decompress(int(x2), int(four), s.ctypes.data, s.size, d.ctypes.data, cnt)
        return r >= 0, d[:cnt].tobytes()

    def zstd_decode_at(self, src: bytes, dst_cap: int):
        """-> (decoded bytes, 0, None) or (bytes before the failing block, zstd
        error code, fail_at): fail_at = output offset of the failing block's
        start (frame end for the content-size / checksum checks)."""
        s = np.frombuffer(src, np.uint8)
        d = np.zeros(max(dst_cap, 1), np.uint8)
        fa = C.c_size_t(0)
        r = self.lib.orc_zstd_decode_at(s.ctypes.data, s.size, d.ctypes.data, dst_cap, C.byref(fa))
        if r < 0:
            return d[: fa.value].tobytes(), -r, fa.value
        return d[:r].tobytes(), 0, None

    def seek_table(self, file: bytes):
        """-> dict(c_off, d_off, checksum, checksum_flag) or None."""
        f = np.frombuffer(file, np.uint8)
        ck = C.c_int(0)
        n = self.lib.orc_seek_table_parse(f.ctypes.data, f.size, None, None, None, C.byref(ck))
        if n < 0:
            return None
        c_off = np.zeros(n + 1, np.uint64)
        d_off = np.zeros(n + 1, np.uint64)
        cks = np.zeros(max(n, 1), np.uint32)
        self.lib.orc_seek_table_parse(f.ctypes.data, f.size, c_off.ctypes.data,
                                      d_off.ctypes.data, cks.ctypes.data, C.byref(ck))
        return {"c_off": c_off, "d_off": d_off, "checksum": cks[:n],
                "checksum_flag": bool(ck.value), "frames": int(n)}

    def decode_file(self, file: bytes):
        """Decode every frame of a seekable LZ4 file -> bytes (raises on error)."""
        st = self.seek_table(file)
        if st is None:
            raise ValueError("read_seek_table failed")
        parts = []
        for i in range(st["frames"]):
            c0, c1 = int(st["c_off"][i]), int(st["c_off"][i + 1])
            dsz = int(st["d_off"][i + 1] - st["d_off"][i])
            status, data, _, _ = self.decode_frame(file[c0:c1], dsz)
            if status != 0:
                raise ValueError(f"frame {i}: {self.error_name(status)}")
            if len(data) != dsz:
                raise ValueError(f"frame {i}: short frame")
            parts.append(data)
        return b"".join(parts)

    @staticmethod
    def error_name(code: int) -> str:
        if 0 <= code < len(LZ4F_ERROR_NAMES):
            return LZ4F_ERROR_NAMES[code]
        return {ORC_ERROR_DST_OVERFLOW: "decoded data exceeds frame size",
                ORC_ERROR_SHORT_FRAME: "decoded data shorter than frame size",
                ORC_ERROR_TRUNCATED: "truncated frame"}.get(code, "?")

    def pread_model(self, file: bytes, count: int, offset: int):
        """Reference zseek_pread result for a valid file: bytes of ONE frame."""
        st = self.seek_table(file)
        d_off = st["d_off"]
        n = st["frames"]
        if count == 0 or offset >= int(d_off[n]):
            return b""
        i = int(np.searchsorted(d_off, np.uint64(offset), side="right") - 1)
        c0, c1 = int(st["c_off"][i]), int(st["c_off"][i + 1])
        dsz = int(d_off[i + 1] - d_off[i])
        status, data, _, _ = self.decode_frame(file[c0:c1], dsz)
        assert status == 0
        rel = offset - int(d_off[i])
        return data[rel: rel + min(count, dsz - rel)]


# ---------------------------------------------------------------------------
# The reference library, driven through zseek.h (test infrastructure only).
# ---------------------------------------------------------------------------
ERRBUF = 80
WRITE_FN = C.CFUNCTYPE(C.c_bool, C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p)
PREAD_FN = C.CFUNCTYPE(C.c_ssize_t, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p, C.c_void_p)
FSIZE_FN = C.CFUNCTYPE(C.c_ssize_t, C.c_void_p, C.c_void_p)


class _WriteFile(C.Structure):
    _fields_ = [("user_data", C.c_void_p), ("write", WRITE_FN)]


class _ReadFile(C.Structure):
    _fields_ = [("user_data", C.c_void_p), ("pread", PREAD_FN), ("fsize", FSIZE_FN)]


class _ZstdParam(C.Structure):
    _fields_ = [("nb_workers", C.c_int), ("cpusetsize", C.c_size_t),
                ("cpuset", C.c_void_p), ("compression_level", C.c_int),
                ("strategy", C.c_int)]


class _Lz4Param(C.Structure):
    _fields_ = [("compression_level", C.c_int)]


class _ParamUnion(C.Union):
    _fields_ = [("zstd_params", _ZstdParam), ("lz4_params", _Lz4Param)]


class _CompParam(C.Structure):
    _fields_ = [("type", C.c_int), ("params", _ParamUnion)]


class _ReaderStats(C.Structure):
    _fields_ = [(n, C.c_size_t) for n in ("seek_table_memory", "frames", "decompressed_size",
                                          "cache_memory", "cached_frames", "buffer_size")]


ZSEEK_ZSTD, ZSEEK_LZ4 = 0, 1


class RefZseek:
    """The reference libzseek (oracle/_ref/libzseek_ref.so) via its public API."""

    def __init__(self, path: str = REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle ref` where /root/reference exists")
        L = self.lib = ref_cdll(path)
        self.versions = ref_dependency_versions(L)
        L.zseek_writer_open_full.restype = C.c_void_p
        L.zseek_writer_open_full.argtypes = [_WriteFile, C.POINTER(_CompParam), C.c_size_t,
                                             C.c_void_p, C.c_char_p]
        L.zseek_write.restype = C.c_bool
        L.zseek_write.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_void_p, C.c_char_p]
        L.zseek_writer_close.restype = C.c_bool
        L.zseek_writer_close.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p]
        L.zseek_reader_open_full.restype = C.c_void_p
        L.zseek_reader_open_full.argtypes = [_ReadFile, C.c_size_t, C.c_void_p, C.c_char_p]
        L.zseek_reader_close.restype = C.c_bool
        L.zseek_reader_close.argtypes = [C.c_void_p, C.c_void_p, C.c_char_p]
        L.zseek_pread.restype = C.c_ssize_t
        L.zseek_pread.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_size_t, C.c_void_p,
                                  C.c_char_p]
        L.zseek_reader_stats.restype = C.c_bool
        L.zseek_reader_stats.argtypes = [C.c_void_p, C.POINTER(_ReaderStats), C.c_char_p]

    # -- writer -------------------------------------------------------------
    def compress(self, data: bytes, ctype: int, min_frame_size: int, write_size: int,
                 level: int | None = None) -> bytes:
        """zseek_writer over `data`, fed in `write_size` chunks -> file bytes."""
        out = bytearray()

        def _w(ptr, size, ud, cd):
            out.extend(C.string_at(ptr, size))
            return True

        wf = _WriteFile(None, WRITE_FN(_w))
        p = _CompParam()
        p.type = ctype
        if ctype == ZSEEK_LZ4:
            p.params.lz4_params.compression_level = 0 if level is None else level
        else:
            p.params.zstd_params.nb_workers = 1
            p.params.zstd_params.compression_level = 3 if level is None else level
            p.params.zstd_params.strategy = 1
        err = C.create_string_buffer(ERRBUF)
        w = self.lib.zseek_writer_open_full(wf, C.byref(p), min_frame_size, None, err)
        if not w:
            raise RuntimeError(err.value.decode())
        buf = C.create_string_buffer(bytes(data), len(data)) if len(data) else None
        base = C.addressof(buf) if buf is not None else 0
        for s in range(0, len(data), write_size):
            n = min(write_size, len(data) - s)
            if not self.lib.zseek_write(w, base + s, n, None, err):
                raise RuntimeError(err.value.decode())
        if not self.lib.zseek_writer_close(w, None, err):
            raise RuntimeError(err.value.decode())
        return bytes(out)

    # -- reader ------------------------------------------------------------
    def open(self, file: bytes, cache_size: int):
        return _RefReader(self, file, cache_size)


class _RefReader:
    def __init__(self, ref: RefZseek, file: bytes, cache_size: int):
        self.ref = ref
        self.buf = C.create_string_buffer(bytes(file), max(len(file), 1))
        self.size = len(file)
        base = C.addressof(self.buf)

        def _pread(ptr, size, offset, ud, cd):
            if offset >= self.size:
                return 0
            n = min(size, self.size - offset)
            C.memmove(ptr, base + offset, n)
            return n

        def _fsize(ud, cd):
            return self.size

        self._cb = (PREAD_FN(_pread), FSIZE_FN(_fsize))
        rf = _ReadFile(None, self._cb[0], self._cb[1])
        self.err = C.create_string_buffer(ERRBUF)
        self.h = ref.lib.zseek_reader_open_full(rf, cache_size, None, self.err)

    @property
    def error(self) -> str:
        return self.err.value.decode(errors="replace")

    def pread(self, count: int, offset: int):
        out = C.create_string_buffer(max(count, 1))
        r = self.ref.lib.zseek_pread(self.h, out, count, offset, None, self.err)
        return r, (out.raw[: r] if r > 0 else b"")

    def stats(self):
        s = _ReaderStats()
        ok = self.ref.lib.zseek_reader_stats(self.h, C.byref(s), self.err)
        return ok, {k: getattr(s, k) for k, _ in _ReaderStats._fields_}

    def close(self):
        if self.h:
            self.ref.lib.zseek_reader_close(self.h, None, self.err)
            self.h = None


class RefBench:
    """T-thread reference CPU decode (oracle/ref_bench.c over libzseek_ref.so)."""

    def __init__(self, path: str = REF_BENCH_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = self.lib = ref_cdll(path)
        self.versions = ref_dependency_versions(L)
        L.ref_bench_run.restype = C.c_int
        L.ref_bench_run.argtypes = [C.c_void_p, C.c_size_t, C.c_int, C.c_uint64, C.c_uint64,
                                    C.c_uint64, C.c_size_t, C.c_size_t, C.c_void_p,
                                    C.POINTER(C.c_double), C.POINTER(C.c_uint64), C.c_char_p]

    def run(self, img: np.ndarray, threads: int, d_begin: int, d_end: int, align: int,
            req: int, cache_size: int = 0, out: np.ndarray | None = None):
        secs, nbytes = C.c_double(0), C.c_uint64(0)
        err = C.create_string_buffer(ERRBUF)
        rc = self.lib.ref_bench_run(img.ctypes.data, img.size, threads, d_begin, d_end, align,
                                    req, cache_size, None if out is None else out.ctypes.data,
                                    C.byref(secs), C.byref(nbytes), err)
        if rc != 0:
            raise RuntimeError("reference decode failed: " + err.value.decode(errors="replace"))
        return secs.value, nbytes.value
