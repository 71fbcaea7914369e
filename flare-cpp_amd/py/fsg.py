"""ctypes binding of libflare_snappy_gpu.so (include/flare_snappy_gpu.h) and of
the synthetic-data generator, for the Python test suite and bench.py.

The product path is the C ABI; this module only marshals device pointers
(torch tensors on cuda:N are used as plain device allocations) and never
falls back to anything else: if the HIP library is missing, loading raises.
"""
from __future__ import annotations

import ctypes
import os
from pathlib import Path

import numpy as np

PKG_DIR = Path(__file__).resolve().parents[1]
LIB_DIR = PKG_DIR / "lib"
REPO_DIR = PKG_DIR.parent
HEADER = REPO_DIR / "include" / "flare_snappy_gpu.h"
HEADERS = (HEADER, REPO_DIR / "include" / "flare_lz4_gpu.h")

FSG_OK, FSG_CORRUPT, FSG_BAD_HEADER, FSG_SLOT_TOO_SMALL, FSG_IOV_TOO_SMALL = 0, 1, 2, 3, 4
FSG_FLAG_VALIDATE_ONLY, FSG_FLAG_STRICT_HEADER = 1, 2

_c = ctypes
_vp, _sz, _u32, _u64, _i32 = _c.c_void_p, _c.c_size_t, _c.c_uint32, _c.c_uint64, _c.c_int32

_SIGS = {
    "fsg_version": (_c.c_char_p, []),
    "fsg_init": (_c.c_int, [_c.c_int]),
    "fsg_last_error": (_c.c_char_p, []),
    "fsg_select_kernels": (_c.c_int, [_c.c_int, _c.c_int]),
    "fsg_set_split_region_cap": (_c.c_int, [_u32]),
    "fsg_set_option": (_c.c_int, [_c.c_char_p, _c.c_int64]),
    "fsg_get_option": (_c.c_int, [_c.c_char_p, _c.POINTER(_c.c_int64)]),
    "fsg_default_option": (_c.c_int, [_c.c_char_p, _c.POINTER(_c.c_int64)]),
    "fsg_max_compressed_length": (_sz, [_sz]),
    "fsg_get_uncompressed_length": (_c.c_int, [_vp, _sz, _c.POINTER(_u32), _c.c_int]),
    "fsg_uncompressed_lengths_batch": (_c.c_int, [_vp, _vp, _vp, _u32, _vp, _c.c_int, _vp]),
    "fsg_compress_workspace_bytes": (_sz, [_u32, _u32]),
    "fsg_decompress_workspace_bytes": (_sz, [_u32, _u64]),
    "fsg_compress_batch": (_c.c_int, [_vp, _vp, _vp, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "fsg_decompress_batch": (_c.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _u32, _vp, _sz, _vp]),
    "fsg_decompress_batch_2s": (_c.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _u32, _vp, _sz, _vp,
                                           _vp]),
    "fsg_decompress_batch_partial": (_c.c_int, [_vp, _vp, _vp, _u32, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                                _sz, _vp]),
    "fsg_decompress_batch_iovec": (_c.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp,
                                              _sz, _vp]),
    "fsg_lz4_max_compressed_length": (_sz, [_sz]),
    "fsg_lz4_compress_workspace_bytes": (_sz, [_u32]),
    "fsg_lz4_compress_batch": (_c.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "fsg_lz4_decompress_batch": (_c.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp]),
    "fsg_lz4_decompress_workspace_bytes": (_sz, [_u32, _u64]),
    "fsg_lz4_decompress_batch_ws": (_c.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp]),
    "fsg_lz4_decompress_batch_2s": (_c.c_int, [_vp, _vp, _vp, _u32, _vp, _vp, _vp, _vp, _vp, _vp, _sz, _vp,
                                               _vp]),
}


def header_symbols(header: Path | None = None) -> list[str]:
    """Every fsg_* function declared in include/flare_snappy_gpu.h and
    include/flare_lz4_gpu.h (or in `header`)."""
    import re
    text = "".join(h.read_text() for h in ((header,) if header else HEADERS))
    return sorted(set(re.findall(r"\b(fsg_[a-z0-9_]+)\s*\(", text)))


# entry points an older library under A/B may lack
_OPTIONAL = {"fsg_decompress_batch_2s", "fsg_decompress_batch_partial", "fsg_decompress_batch_iovec", "fsg_lz4_decompress_batch_2s", "fsg_lz4_decompress_batch_ws",
             "fsg_lz4_decompress_workspace_bytes", "fsg_set_option", "fsg_get_option", "fsg_default_option"}


def load_gpu_lib(path: Path | None = None) -> ctypes.CDLL:
    path = Path(path or os.environ.get("FSG_LIB", LIB_DIR / "libflare_snappy_gpu.so"))
    if not path.exists():
        raise RuntimeError(f"HIP codec library missing: {path} (run __graft_entry__.build())")
    lib = ctypes.CDLL(str(path))
    for name, (res, args) in _SIGS.items():
        if name in _OPTIONAL and not hasattr(lib, name):
            continue  # an older build under A/B (FSG_LIB)
        fn = getattr(lib, name)
        fn.restype, fn.argtypes = res, args
    return lib


def get_option(name: str, lib: ctypes.CDLL | None = None) -> int:
    """fsg_get_option: a process-wide tuning/test option (include/flare_snappy_gpu.h)."""
    lib = lib or load_gpu_lib()
    v = _c.c_int64(0)
    if lib.fsg_get_option(name.encode(), _c.byref(v)) != 0:
        raise KeyError(name)
    return v.value


def set_option(name: str, value: int, lib: ctypes.CDLL | None = None) -> None:
    lib = lib or load_gpu_lib()
    if lib.fsg_set_option(name.encode(), int(value)) != 0:
        raise KeyError(name)


class options:
    """Context manager: set library options for a block, restore them after.

        with fsg.options(decode_fork=1, split_walk=3): ...
    """

    def __init__(self, **kv):
        self.kv = kv
        self.saved = {}

    def __enter__(self):
        lib = load_gpu_lib()
        for k, v in self.kv.items():
            self.saved[k] = get_option(k, lib)
            set_option(k, v, lib)
        return self

    def __exit__(self, *exc):
        lib = load_gpu_lib()
        for k, v in self.saved.items():
            set_option(k, v, lib)
        return False


def _ptr(t) -> int | None:
    if t is None:
        return None
    return t.data_ptr()


class SnappyGPU:
    """Batched device codec through the C ABI.  Tensors must be on one cuda device."""

    def __init__(self, device: int = 0, lib_path: Path | None = None):
        self.lib = load_gpu_lib(lib_path)
        rc = self.lib.fsg_init(device)
        if rc != 0:
            raise RuntimeError(f"fsg_init({device}) = {rc}: {self.lib.fsg_last_error().decode()}")
        self.device = device

    def select_kernels(self, decode: int = 0, encode: int = 0):
        self._check(self.lib.fsg_select_kernels(decode, encode), "fsg_select_kernels")

    def _check(self, rc: int, what: str):
        if rc != 0:
            raise RuntimeError(f"{what} failed rc={rc}: {self.lib.fsg_last_error().decode()}")

    @staticmethod
    def _stream(stream) -> int | None:
        if stream is None:
            import torch
            return torch.cuda.current_stream().cuda_stream
        return stream.cuda_stream if hasattr(stream, "cuda_stream") else int(stream)

    def decompress_workspace(self, n, total_in=0, device=None):
        import torch
        nbytes = self.lib.fsg_decompress_workspace_bytes(n, total_in)
        return torch.zeros(max(nbytes, 1), dtype=torch.uint8, device=device or f"cuda:{self.device}")

    def set_split_region_cap(self, nbytes: int):
        self._check(self.lib.fsg_set_split_region_cap(nbytes), "fsg_set_split_region_cap")

    def compress_workspace(self, n, max_in_len, device=None):
        """Allocate the device workspace fsg_compress_batch wants (torch uint8)."""
        import torch
        nbytes = self.lib.fsg_compress_workspace_bytes(n, max_in_len)
        return torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device or f"cuda:{self.device}")

    def compress(self, d_in, d_in_off, d_in_len, n, max_in_len, d_out, d_out_off, d_out_len,
                 d_status, stream=None, workspace=None):
        ws = 0 if workspace is None else workspace.numel() * workspace.element_size()
        self._check(self.lib.fsg_compress_batch(
            _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len), n, max_in_len, _ptr(d_out),
            _ptr(d_out_off), _ptr(d_out_len), _ptr(d_status), _ptr(workspace), ws,
            self._stream(stream)), "fsg_compress_batch")

    def decompress(self, d_in, d_in_off, d_in_len, n, d_out, d_out_off, d_out_cap, d_out_len,
                   d_status, flags=0, stream=None, workspace=None, pass1_stream=None):
        """fsg_decompress_batch; with `pass1_stream`, fsg_decompress_batch_2s
        (the tag walk on pass1_stream, the execution on `stream`)."""
        ws = 0 if workspace is None else workspace.numel() * workspace.element_size()
        args = (_ptr(d_in), _ptr(d_in_off), _ptr(d_in_len), n, _ptr(d_out), _ptr(d_out_off),
                _ptr(d_out_cap), _ptr(d_out_len), _ptr(d_status), flags, _ptr(workspace), ws,
                self._stream(stream))
        if pass1_stream is None:
            self._check(self.lib.fsg_decompress_batch(*args), "fsg_decompress_batch")
        else:
            self._check(self.lib.fsg_decompress_batch_2s(*args, self._stream(pass1_stream)),
                        "fsg_decompress_batch_2s")

    def decompress_partial(self, d_in, d_in_off, d_in_len, n, frag, d_out, d_out_off, d_out_cap, d_got,
                           d_produced, d_status, stream=None, workspace=None):
        """fsg_decompress_batch_partial: UncompressAsMuchAsPossible per message
        (d_produced int64 / uint64, d_got int32 / uint32)."""
        ws = 0 if workspace is None else workspace.numel() * workspace.element_size()
        self._check(self.lib.fsg_decompress_batch_partial(
            _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len), n, frag, _ptr(d_out), _ptr(d_out_off), _ptr(d_out_cap),
            _ptr(d_got), _ptr(d_produced), _ptr(d_status), _ptr(workspace), ws, self._stream(stream)),
            "fsg_decompress_batch_partial")

    def decompress_iovec(self, d_in, d_in_off, d_in_len, n, d_iov_base, d_iov_len, d_iov_first, d_stage,
                         d_stage_off, d_stage_cap, d_out_len, d_status, stream=None, workspace=None):
        """fsg_decompress_batch_iovec: RawUncompressToIOVec per message (d_iov_base:
        int64 device addresses, d_iov_len int64, d_iov_first int32 with n + 1 entries)."""
        ws = 0 if workspace is None else workspace.numel() * workspace.element_size()
        self._check(self.lib.fsg_decompress_batch_iovec(
            _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len), n, _ptr(d_iov_base), _ptr(d_iov_len), _ptr(d_iov_first),
            _ptr(d_stage), _ptr(d_stage_off), _ptr(d_stage_cap), _ptr(d_out_len), _ptr(d_status), _ptr(workspace),
            ws, self._stream(stream)), "fsg_decompress_batch_iovec")

    # ---- LZ4 (include/flare_lz4_gpu.h)
    def lz4_compress_workspace(self, n, device=None):
        import torch
        nbytes = self.lib.fsg_lz4_compress_workspace_bytes(n)
        return torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device or f"cuda:{self.device}")

    def lz4_compress(self, d_in, d_in_off, d_in_len, n, d_out, d_out_off, d_out_len, d_status, workspace,
                     stream=None):
        self._check(self.lib.fsg_lz4_compress_batch(
            _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len), n, _ptr(d_out), _ptr(d_out_off), _ptr(d_out_len),
            _ptr(d_status), _ptr(workspace), workspace.numel(), self._stream(stream)), "fsg_lz4_compress_batch")

    def lz4_decompress_workspace(self, n, total_in_bytes, device=None):
        import torch
        if not hasattr(self.lib, "fsg_lz4_decompress_workspace_bytes"):
            return None  # an older library under A/B: the one-pass kernel runs
        nbytes = self.lib.fsg_lz4_decompress_workspace_bytes(n, total_in_bytes)
        return torch.empty(max(nbytes, 1), dtype=torch.uint8, device=device or f"cuda:{self.device}")

    def lz4_decompress(self, d_in, d_in_off, d_in_len, n, d_out, d_out_off, d_out_cap, d_out_len, d_status,
                       stream=None, workspace=None, pass1_stream=None):
        """workspace=None: the one-pass lane kernel; else the two-pass
        decoder (fsg_lz4_decompress_batch_ws; with `pass1_stream`,
        fsg_lz4_decompress_batch_2s: the index pass there, the execution on
        `stream`)."""
        if workspace is None or not hasattr(self.lib, "fsg_lz4_decompress_batch_ws"):
            self._check(self.lib.fsg_lz4_decompress_batch(
                _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len), n, _ptr(d_out), _ptr(d_out_off), _ptr(d_out_cap),
                _ptr(d_out_len), _ptr(d_status), self._stream(stream)), "fsg_lz4_decompress_batch")
            return
        args = (_ptr(d_in), _ptr(d_in_off), _ptr(d_in_len), n, _ptr(d_out), _ptr(d_out_off), _ptr(d_out_cap),
                _ptr(d_out_len), _ptr(d_status), _ptr(workspace), workspace.numel(), self._stream(stream))
        if pass1_stream is None:
            self._check(self.lib.fsg_lz4_decompress_batch_ws(*args), "fsg_lz4_decompress_batch_ws")
        else:
            self._check(self.lib.fsg_lz4_decompress_batch_2s(*args, self._stream(pass1_stream)),
                        "fsg_lz4_decompress_batch_2s")

    def uncompressed_lengths(self, d_in, d_in_off, d_in_len, n, d_ulen, lenient=True, stream=None):
        self._check(self.lib.fsg_uncompressed_lengths_batch(
            _ptr(d_in), _ptr(d_in_off), _ptr(d_in_len), n, _ptr(d_ulen), int(lenient),
            self._stream(stream)), "fsg_uncompressed_lengths_batch")


# ---------------------------------------------------------------------------
# Batches (host side): one contiguous uint8 buffer + uint64 offsets + uint32 lengths.

class Batch:
    def __init__(self, data: np.ndarray, offsets: np.ndarray, lens: np.ndarray):
        self.data = np.ascontiguousarray(data, dtype=np.uint8)
        self.offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
        self.lens = np.ascontiguousarray(lens, dtype=np.uint32)

    def __len__(self):
        return len(self.lens)

    def item(self, i: int) -> bytes:
        o = int(self.offsets[i])
        return self.data[o:o + int(self.lens[i])].tobytes()

    @property
    def total(self) -> int:
        return int(self.lens.astype(np.uint64).sum())

    @staticmethod
    def from_list(items) -> "Batch":
        lens = np.array([len(x) for x in items], dtype=np.uint32)
        offs = np.zeros(len(items), dtype=np.uint64)
        if len(items) > 1:
            offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
        data = np.frombuffer(b"".join(items), dtype=np.uint8) if items else np.zeros(0, np.uint8)
        if data.size == 0:
            data = np.zeros(1, np.uint8)
        return Batch(data.copy(), offs, lens)


def slot_offsets(caps: np.ndarray, align: int = 16) -> tuple[np.ndarray, int]:
    """Exclusive prefix offsets of slots of the given capacities, `align`-aligned."""
    caps = caps.astype(np.uint64)
    sizes = (caps + np.uint64(align - 1)) // np.uint64(align) * np.uint64(align)
    offs = np.zeros(len(caps), dtype=np.uint64)
    if len(caps) > 1:
        offs[1:] = np.cumsum(sizes[:-1])
    total = int(sizes.sum()) if len(caps) else 0
    return offs, max(total, align)


def max_compressed_length(n):
    return 32 + n + n // 6


# ---------------------------------------------------------------------------
# Synthetic data (flare-cpp_amd/tools/datagen.c).

_DG = None


def datagen() -> ctypes.CDLL:
    global _DG
    if _DG is None:
        p = LIB_DIR / "libflare_datagen.so"
        if not p.exists():
            raise RuntimeError(f"datagen library missing: {p}")
        lib = ctypes.CDLL(str(p))
        lib.dg_text_body.argtypes = [_u64, _vp, _sz]
        lib.dg_random_body.argtypes = [_u64, _vp, _sz]
        lib.dg_mixed_sizes.argtypes = [_u64, _vp]
        lib.dg_snappy_message.argtypes = [_u64, _u32, _vp]
        lib.dg_snappy_message.restype = _sz
        lib.dg_fnv1a64.argtypes = [_vp, _sz]
        lib.dg_fnv1a64.restype = _u64
        lib.dg_fill_batch.argtypes = [_c.c_int, _u64, _u64, _vp, _vp, _vp, _vp, _c.c_int]
        lib.dg_digest_batch.argtypes = [_vp, _vp, _vp, _u64, _vp]
        _DG = lib
    return _DG


KIND_TEXT, KIND_RANDOM, KIND_MIXED, KIND_PROTO = 0, 1, 2, 3


def _threads() -> int:
    return max(1, min(16, os.cpu_count() or 1))


def make_batch(kind: int, sizes, first_index: int = 0, threads: int | None = None) -> Batch:
    """Generate message bodies first_index.. with the given sizes (for KIND_PROTO the
    sizes are text lengths and the returned lengths are serialized lengths)."""
    dg = datagen()
    sizes = np.ascontiguousarray(np.asarray(sizes, dtype=np.uint32))
    n = len(sizes)
    if kind == KIND_PROTO:
        lens = np.array([dg.dg_snappy_message(first_index + i, int(s), None) for i, s in enumerate(sizes)],
                        dtype=np.uint32)
    else:
        lens = sizes.copy()
    offs = np.zeros(n, dtype=np.uint64)
    if n > 1:
        offs[1:] = np.cumsum(lens[:-1].astype(np.uint64))
    total = int(lens.astype(np.uint64).sum())
    data = np.zeros(max(total, 1), dtype=np.uint8)
    out_lens = np.zeros(n, dtype=np.uint32)
    dg.dg_fill_batch(kind, first_index, n, sizes.ctypes.data, offs.ctypes.data, data.ctypes.data,
                     out_lens.ctypes.data, threads or _threads())
    return Batch(data, offs, lens)


def mixed_sizes(n: int) -> np.ndarray:
    s = np.zeros(n, dtype=np.uint32)
    datagen().dg_mixed_sizes(n, s.ctypes.data)
    return s


def fnv1a64(b: bytes) -> int:
    buf = np.frombuffer(b, dtype=np.uint8) if b else np.zeros(1, np.uint8)
    return int(datagen().dg_fnv1a64(buf.ctypes.data, len(b)))


def digests(data: np.ndarray, offsets: np.ndarray, lens: np.ndarray) -> np.ndarray:
    out = np.zeros(len(lens), dtype=np.uint64)
    datagen().dg_digest_batch(data.ctypes.data, np.ascontiguousarray(offsets, np.uint64).ctypes.data,
                              np.ascontiguousarray(lens, np.uint32).ctypes.data, len(lens),
                              out.ctypes.data)
    return out
