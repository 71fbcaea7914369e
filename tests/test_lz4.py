"""LZ4 oracle (oracle/lz4_oracle.c) against the pins: the liblz4 1.9.3
fixtures in tests/golden/lz4_vectors.json (make_lz4_golden.py) and, where the
image has it, the system liblz4 live.  The reference holds no LZ4 code, so
this is the LZ4 path's parity anchor."""
import json
from pathlib import Path

import numpy as np
import pytest

import fsg
from bind import Lz4Oracle
from gen_inputs import build_input
from lz4_walk import first_violation

GOLDEN = Path(__file__).resolve().parent / "golden"
VEC = json.loads((GOLDEN / "lz4_vectors.json").read_text())


@pytest.fixture(scope="module")
def o():
    return Lz4Oracle()


def test_oracle_blocks_equal_liblz4_fixtures(o):
    for v in VEC["compress"]:
        x = build_input(v)
        assert len(x) == v["input_len"] and "%016x" % fsg.fnv1a64(x) == v["input_fnv"], v["name"]
        b = o.compress_block(x)
        assert len(b) == v["block_len"] and "%016x" % fsg.fnv1a64(b) == v["block_fnv"], v["name"]
        if "block_hex" in v:
            assert b.hex() == v["block_hex"], v["name"]
        ok, y = o.decompress_block(b, len(x))
        assert ok and y == x, v["name"]


def test_oracle_decode_verdicts_equal_liblz4(o):
    n_ok = 0
    for d in VEC["decode"]:
        b = bytes.fromhex(d["hex"])
        ok, y = o.decompress_block(b, d["ulen"])
        if d["offset0"]:
            assert not ok  # liblz4 copies from the write position; rejected here
            continue
        assert ok == d["liblz4_ok"], d
        if ok:
            n_ok += 1
            assert "%016x" % fsg.fnv1a64(y) == d["output_fnv"]
        assert (first_violation(b, d["ulen"]) is None) == ok
    assert n_ok > 100


def test_body_framing(o):
    for x in (b"", b"a", b"hello hello hello hello", bytes(70000)):
        body = o.compress(x)
        st, ulen, y = o.uncompress(body)
        assert st == 1 and ulen == len(x) and y == x
    assert o.uncompress(b"")[0] == -1
    assert o.uncompress(b"\x80\x80\x80\x80\x80")[0] == -1   # 6th byte needed
    assert o.uncompress(b"\x80\x80\x80\x80\x10")[0] == -1   # > 32 bits
    assert o.uncompress(o.compress(b"abc"), cap=2)[0] == -2


def test_oracle_against_system_liblz4_live(o):
    from lz4_sys import SysLz4, load
    L = load()
    if L is None:
        pytest.skip("no system liblz4 in this image")
    z = SysLz4(L)
    rng = np.random.default_rng(12)
    for t in range(300):
        n = int(rng.choice([rng.integers(0, 40), rng.integers(0, 3000), rng.integers(60000, 70000),
                            rng.integers(0, 300000)]))
        alpha = int(rng.choice([1, 2, 4, 16, 256]))
        x = rng.integers(0, alpha, n, dtype=np.uint8).tobytes()
        b = o.compress_block(x)
        assert b == z.compress(x), (n, alpha)
        m, y = z.decompress(b, n)
        assert m == n and y == x


# ---- the product host codec (host/lz4_cpu.cc through include/flare_snappy_host.h)

@pytest.fixture(scope="module")
def host():
    import ctypes
    import subprocess
    repo = Path(__file__).resolve().parents[1]
    lib = repo / "flare-cpp_amd" / "lib" / "libflare_rpc_snappy.so"
    if not lib.exists():
        subprocess.run(["make", "-C", str(repo), "host"], check=True, capture_output=True)
    L = ctypes.CDLL(str(lib))
    L.fsh_lz4_max_compressed_length.argtypes = [ctypes.c_size_t]
    L.fsh_lz4_max_compressed_length.restype = ctypes.c_size_t
    L.fsh_cpu_lz4_compress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    L.fsh_cpu_lz4_compress.restype = ctypes.c_size_t
    L.fsh_cpu_lz4_uncompress.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                         ctypes.POINTER(ctypes.c_uint32)]
    return L


def _host_compress(L, x: bytes) -> bytes:
    import ctypes
    out = ctypes.create_string_buffer(L.fsh_lz4_max_compressed_length(len(x)) + 1)
    n = L.fsh_cpu_lz4_compress(ctypes.create_string_buffer(x, max(len(x), 1)), len(x), out)
    return out.raw[:n]


def _host_uncompress(L, body: bytes, cap: int):
    import ctypes
    out = ctypes.create_string_buffer(max(cap, 1))
    ulen = ctypes.c_uint32(0)
    r = L.fsh_cpu_lz4_uncompress(ctypes.create_string_buffer(body, max(len(body), 1)), len(body), out, cap,
                                 ctypes.byref(ulen))
    return r, ulen.value, (out.raw[:ulen.value] if r == 1 else None)


def test_host_codec_blocks_equal_fixtures_and_oracle(host, o):
    for v in VEC["compress"]:
        x = build_input(v)
        body = _host_compress(host, x)
        assert body == o.compress(x), v["name"]
        r, ulen, y = _host_uncompress(host, body, len(x))
        assert r == 1 and y == x, v["name"]


def test_host_codec_verdicts_equal_oracle(host, o):
    rng = np.random.default_rng(23)
    src = [fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0) for s in (30, 700, 9000)]
    src.append(rng.integers(0, 3, 4000, dtype=np.uint8).tobytes())
    for i in range(3000):
        b = bytearray(o.compress(src[i % len(src)]))
        for _ in range(int(rng.integers(1, 3))):
            b[int(rng.integers(len(b)))] = int(rng.integers(256))
        if rng.random() < 0.3:
            b = b[:int(rng.integers(1, len(b) + 1))]
        b = bytes(b)
        want = o.uncompress(b, cap=1 << 15)
        got = _host_uncompress(host, b, 1 << 15)
        assert got[0] == want[0] and (want[0] != 1 or got[2] == want[2]), i
