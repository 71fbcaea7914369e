"""TEST INFRASTRUCTURE ONLY: the image's system liblz4 (1.9.3, Ubuntu
package, /usr/lib/x86_64-linux-gnu/liblz4.so.1) through ctypes, to pin the
LZ4 oracle.  Not part of the reference and never loaded by the product."""
import ctypes
import ctypes.util


def load():
    for name in ("liblz4.so.1", ctypes.util.find_library("lz4")):
        if not name:
            continue
        try:
            L = ctypes.CDLL(name)
        except OSError:
            continue
        L.LZ4_compress_default.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.LZ4_decompress_safe.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_int, ctypes.c_int]
        L.LZ4_compressBound.argtypes = [ctypes.c_int]
        L.LZ4_versionNumber.restype = ctypes.c_int
        return L
    return None


class SysLz4:
    def __init__(self, L):
        self.L = L
        self.version = L.LZ4_versionNumber()

    def compress(self, data: bytes) -> bytes:
        cap = self.L.LZ4_compressBound(len(data))
        out = ctypes.create_string_buffer(max(cap, 1))
        n = self.L.LZ4_compress_default(data, out, len(data), cap)
        return out.raw[:n]

    def decompress(self, block: bytes, ulen: int):
        out = ctypes.create_string_buffer(max(ulen, 1))
        n = self.L.LZ4_decompress_safe(block, out, len(block), ulen)
        return n, (out.raw[:n] if n >= 0 else None)
