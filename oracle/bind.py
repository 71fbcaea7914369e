"""TEST INFRASTRUCTURE ONLY -- ctypes access to the oracle.

* `Oracle`    : the C restatement (oracle/liboracle_snappy.so).
* `Reference` : the reference's own snappy.cc compiled by oracle/Makefile
                (oracle/_ref/libsnappy_ref.so), present wherever it was built
                in the dev container (it travels with the repo snapshot).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module.  It is the checker, never the product path.
"""
from __future__ import annotations

import ctypes
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
ORACLE_LIB = ORACLE_DIR / "liboracle_snappy.so"
REF_LIB = ORACLE_DIR / "_ref" / "libsnappy_ref.so"

_vp, _sz, _u32, _c = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes


def _buf(b: bytes):
    return ctypes.create_string_buffer(b, max(len(b), 1))


def _iovec_call(fn, comp: bytes, iov_lens, fill: int):
    bufs = [ctypes.create_string_buffer(bytes([fill]) * max(int(n), 1)) for n in iov_lens]
    cnt = len(bufs)
    base = (ctypes.c_void_p * max(cnt, 1))(*[ctypes.addressof(b) for b in bufs])
    lens = (ctypes.c_size_t * max(cnt, 1))(*[int(n) for n in iov_lens])
    ok = fn(_buf(comp), len(comp), base, lens, cnt)
    return bool(ok), [b.raw[:int(n)] for b, n in zip(bufs, iov_lens)]


class Oracle:
    def __init__(self, path: Path = ORACLE_LIB):
        if not Path(path).exists():
            raise RuntimeError(f"oracle library missing: {path}")
        L = ctypes.CDLL(str(path))
        L.so_max_compressed_length.argtypes = [_sz]
        L.so_max_compressed_length.restype = _sz
        L.so_header_strict.argtypes = [_vp, _sz, _c.POINTER(_u32)]
        L.so_header_lenient.argtypes = [_vp, _sz, _c.POINTER(_u32)]
        L.so_compress.argtypes = [_vp, _sz, _vp]
        L.so_compress.restype = _sz
        L.so_uncompress.argtypes = [_vp, _sz, _vp, _sz, _c.POINTER(_u32)]
        L.so_is_valid.argtypes = [_vp, _sz]
        L.so_compress_batch.argtypes = [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _c.c_int]
        L.so_compress_batch.restype = _c.c_double
        L.so_uncompress_batch.argtypes = [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _c.c_int]
        L.so_uncompress_batch.restype = _c.c_double
        L.so_uncompress_as_much.argtypes = [_vp, _sz, _sz, _vp, _sz, _c.POINTER(_sz)]
        L.so_uncompress_as_much.restype = _sz
        L.so_uncompress_iovec.argtypes = [_vp, _sz, _vp, _vp, _sz]
        self.L = L

    def max_compressed_length(self, n: int) -> int:
        return self.L.so_max_compressed_length(n)

    def compress(self, data: bytes) -> bytes:
        out = ctypes.create_string_buffer(self.max_compressed_length(len(data)) + 1)
        n = self.L.so_compress(_buf(data), len(data), out)
        return out.raw[:n]

    def uncompress(self, comp: bytes, cap: int | None = None):
        """Returns (ok: bool, ulen, output bytes or None).  ok None = slot too small."""
        ulen = _u32(0)
        h = self.L.so_header_lenient(_buf(comp), len(comp), ctypes.byref(ulen))
        if not h:
            return False, 0, None
        cap = ulen.value if cap is None else cap
        if cap > 1 << 31:
            return None, ulen.value, None
        out = ctypes.create_string_buffer(max(cap, 1))
        r = self.L.so_uncompress(_buf(comp), len(comp), out, cap, ctypes.byref(ulen))
        if r < 0:
            return None, ulen.value, None
        return bool(r), ulen.value, (out.raw[:ulen.value] if r == 1 else None)

    def header(self, comp: bytes, lenient: bool = True):
        ulen = _u32(0)
        fn = self.L.so_header_lenient if lenient else self.L.so_header_strict
        h = fn(_buf(comp), len(comp), ctypes.byref(ulen))
        return h, ulen.value

    def is_valid(self, comp: bytes) -> bool:
        return bool(self.L.so_is_valid(_buf(comp), len(comp)))

    def uncompress_as_much(self, comp: bytes, cap: int, frag: int = 0):
        """UncompressAsMuchAsPossible restated: (its return value, the bytes the sink gets)."""
        out = ctypes.create_string_buffer(max(cap, 1))
        got = _sz(0)
        r = self.L.so_uncompress_as_much(_buf(comp), len(comp), frag, out, cap, ctypes.byref(got))
        return r, out.raw[:min(got.value, cap)]

    def uncompress_iovec(self, comp: bytes, iov_lens, fill: int = 0xA5):
        """RawUncompressToIOVec restated: (ok, the iovecs' bytes after the call)."""
        return _iovec_call(self.L.so_uncompress_iovec, comp, iov_lens, fill)

    def compress_batch(self, data, offs, lens, out, out_offs, out_lens, threads=1) -> float:
        return self.L.so_compress_batch(data.ctypes.data, offs.ctypes.data, lens.ctypes.data, len(lens),
                                        out.ctypes.data, out_offs.ctypes.data, out_lens.ctypes.data,
                                        threads)

    def uncompress_batch(self, data, offs, lens, out, out_offs, out_caps, out_lens, status,
                         threads=1) -> float:
        return self.L.so_uncompress_batch(data.ctypes.data, offs.ctypes.data, lens.ctypes.data,
                                          len(lens), out.ctypes.data, out_offs.ctypes.data,
                                          out_caps.ctypes.data, out_lens.ctypes.data,
                                          status.ctypes.data, threads)


class Reference:
    """The reference's own flare/io/snappy compiled in place (oracle/Makefile)."""

    FRAG = 8160  # cord_buf block payload, flare/io/cord_buf.h:67

    def __init__(self, path: Path = REF_LIB):
        if not Path(path).exists():
            raise RuntimeError(f"reference build missing: {path}")
        L = ctypes.CDLL(str(path))
        L.ref_max_compressed_length.argtypes = [_sz]
        L.ref_max_compressed_length.restype = _sz
        L.ref_compress.argtypes = [_vp, _sz, _vp, _sz]
        L.ref_compress.restype = _sz
        L.ref_uncompress.argtypes = [_vp, _sz, _vp, _sz, _c.POINTER(_sz), _sz]
        L.ref_get_uncompressed_length.argtypes = [_vp, _sz, _c.POINTER(_sz)]
        L.ref_get_uncompressed_length_source.argtypes = [_vp, _sz, _c.POINTER(_u32)]
        L.ref_raw_uncompress.argtypes = [_vp, _sz, _vp]
        L.ref_is_valid.argtypes = [_vp, _sz]
        L.ref_uncompress_as_much.argtypes = [_vp, _sz, _vp, _sz, _sz, _c.POINTER(_sz)]
        L.ref_uncompress_as_much.restype = _sz
        L.ref_batch.argtypes = [_c.c_int, _vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _c.c_int, _sz]
        L.ref_batch.restype = _c.c_double
        L.ref_uncompress_iovec.argtypes = [_vp, _sz, _vp, _vp, _sz]
        self.L = L

    @staticmethod
    def available() -> bool:
        return REF_LIB.exists()

    def compress(self, data: bytes, frag: int = FRAG) -> bytes:
        out = ctypes.create_string_buffer(self.L.ref_max_compressed_length(len(data)) + 1)
        n = self.L.ref_compress(_buf(data), len(data), out, frag)
        return out.raw[:n]

    def uncompress(self, comp: bytes, cap: int, frag: int = FRAG):
        out = ctypes.create_string_buffer(max(cap, 1))
        prod = _sz(0)
        ok = self.L.ref_uncompress(_buf(comp), len(comp), out, cap, ctypes.byref(prod), frag)
        return bool(ok), out.raw[:min(prod.value, cap)]

    def uncompress_as_much(self, comp: bytes, cap: int, frag: int = FRAG):
        """UncompressAsMuchAsPossible: (its return value, the bytes the sink received)."""
        out = ctypes.create_string_buffer(max(cap, 1))
        got = _sz(0)
        r = self.L.ref_uncompress_as_much(_buf(comp), len(comp), out, cap, frag, ctypes.byref(got))
        assert got.value <= cap
        return r, out.raw[:got.value]

    def uncompress_iovec(self, comp: bytes, iov_lens, fill: int = 0xA5):
        """RawUncompressToIOVec: (its bool, the iovecs' bytes after the call)."""
        return _iovec_call(self.L.ref_uncompress_iovec, comp, iov_lens, fill)

    def header_source(self, comp: bytes):
        u = _u32(0)
        ok = self.L.ref_get_uncompressed_length_source(_buf(comp), len(comp), ctypes.byref(u))
        return bool(ok), u.value

    def header_strict(self, comp: bytes):
        u = _sz(0)
        ok = self.L.ref_get_uncompressed_length(_buf(comp), len(comp), ctypes.byref(u))
        return bool(ok), u.value

    def is_valid(self, comp: bytes) -> bool:
        return bool(self.L.ref_is_valid(_buf(comp), len(comp)))

    def batch(self, mode, data, offs, lens, out, out_offs, out_caps, out_lens, threads=1,
              frag: int = FRAG) -> float:
        return self.L.ref_batch(mode, data.ctypes.data, offs.ctypes.data, lens.ctypes.data, len(lens),
                                out.ctypes.data, out_offs.ctypes.data,
                                out_caps.ctypes.data if out_caps is not None else None,
                                out_lens.ctypes.data, threads, frag)


LZ4_ORACLE_LIB = ORACLE_DIR / "liboracle_lz4.so"


class Lz4Oracle:
    """The LZ4 block restatement (oracle/liboracle_lz4.so).  RPC body = varint32
    uncompressed length + one LZ4 block."""

    def __init__(self, path: Path = LZ4_ORACLE_LIB):
        if not Path(path).exists():
            raise RuntimeError(f"oracle library missing: {path}")
        L = ctypes.CDLL(str(path))
        L.lz4o_max_compressed_length.argtypes = [_sz]
        L.lz4o_max_compressed_length.restype = _sz
        L.lz4o_compress_block.argtypes = [_vp, _sz, _vp]
        L.lz4o_compress_block.restype = _sz
        L.lz4o_decompress_block.argtypes = [_vp, _sz, _vp, _sz]
        L.lz4o_compress.argtypes = [_vp, _sz, _vp]
        L.lz4o_compress.restype = _sz
        L.lz4o_decompress.argtypes = [_vp, _sz, _vp, _sz, _c.POINTER(_u32)]
        self.L = L

    def bound(self, n: int) -> int:
        return self.L.lz4o_max_compressed_length(n)

    def compress_block(self, data: bytes) -> bytes:
        out = ctypes.create_string_buffer(self.bound(len(data)) + 1)
        n = self.L.lz4o_compress_block(_buf(data), len(data), out)
        return out.raw[:n]

    def decompress_block(self, block: bytes, ulen: int):
        out = ctypes.create_string_buffer(max(ulen, 1))
        ok = self.L.lz4o_decompress_block(_buf(block), len(block), out, ulen)
        return bool(ok), (out.raw[:ulen] if ok else None)

    def compress(self, data: bytes) -> bytes:
        out = ctypes.create_string_buffer(self.bound(len(data)) + 6)
        n = self.L.lz4o_compress(_buf(data), len(data), out)
        return out.raw[:n]

    def uncompress(self, body: bytes, cap: int = 1 << 30):
        """(status, ulen, bytes): status 1 ok, 0 corrupt, -1 bad header, -2 above cap."""
        ulen = _u32(0)
        out = ctypes.create_string_buffer(max(min(cap, 1 << 30), 1))
        r = self.L.lz4o_decompress(_buf(body), len(body), out, cap, ctypes.byref(ulen))
        return r, ulen.value, (out.raw[:ulen.value] if r == 1 else None)
