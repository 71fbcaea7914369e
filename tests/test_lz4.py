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


def test_host_codec_rejects_implausible_header(host):
    # a 2-byte block cannot decode to 4 GiB: the header is refused before
    # any output is sized from it (the drop-in's Lz4Decompress does the same)
    body = bytes([0xFF, 0xFF, 0xFF, 0xFF, 0x0F, 0x10, 0x61])
    r, _, _ = _host_uncompress(host, body, 1 << 20)
    assert r != 1
    r, ulen, _ = _host_uncompress(host, bytes([0xFF, 0xFF, 0x03, 0x10, 0x61]), 1 << 20)
    assert r == 0 and ulen == 0xFFFF  # fits the cap, exceeds 255 x 2 + 64: invalid


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


# ---- the GPU kernels' block codec on the CPU under AddressSanitizer
# (tests/cpp/lz4_host_check.hip includes csrc/lz4.hip; its block functions are
# __host__ __device__), so an out-of-bounds access shows up without a GPU.

@pytest.fixture(scope="module")
def host_check(tmp_path_factory):
    import shutil
    import subprocess
    repo = Path(__file__).resolve().parents[1]
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not Path(hipcc).exists():
        pytest.skip("hipcc not available")
    exe = tmp_path_factory.mktemp("lz4hc") / "lz4_host_check"
    r = subprocess.run([hipcc, "--offload-arch=gfx950", "-O1", "-g", "-Xarch_host", "-fsanitize=address",
                        "-I", str(repo / "flare-cpp_amd" / "csrc"), str(repo / "tests" / "cpp" / "lz4_host_check.hip"),
                        "-o", str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return exe


def _run_check(exe, mode, payload: bytes, tmp_path):
    import subprocess
    fin, fout = tmp_path / f"{mode}.in", tmp_path / f"{mode}.out"
    fin.write_bytes(payload)
    r = subprocess.run([str(exe), mode, str(fin), str(fout)], capture_output=True, text=True, timeout=300,
                       env={"ASAN_OPTIONS": "detect_leaks=0"})
    assert r.returncode == 0, r.stderr[-3000:]
    return fout.read_bytes()


def test_gpu_block_codec_on_host_asan(host_check, o, tmp_path):
    import struct
    rng = np.random.default_rng(29)
    xs = [build_input(v) for v in VEC["compress"] if v["input_len"] <= 300000]
    for t in range(150):
        n = int(rng.choice([rng.integers(0, 40), rng.integers(0, 5000), rng.integers(60000, 70000)]))
        xs.append(rng.integers(0, int(rng.choice([1, 2, 4, 256])), n, dtype=np.uint8).tobytes())
    out = _run_check(host_check, "c", b"".join(struct.pack("<I", len(x)) + x for x in xs), tmp_path)
    p = 0
    for x in xs:
        (n,) = struct.unpack_from("<I", out, p)
        p += 4
        assert out[p:p + n] == o.compress_block(x), len(x)
        p += n
    cases = [(d["ulen"], bytes.fromhex(d["hex"])) for d in VEC["decode"]]
    src = [fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0) for s in (40, 900, 20000)]
    for i in range(2000):
        b = bytearray(o.compress_block(src[i % 3]))
        for _ in range(int(rng.integers(1, 3))):
            b[int(rng.integers(len(b)))] = int(rng.integers(256))
        if rng.random() < 0.3:
            b = b[:int(rng.integers(1, len(b) + 1))]
        cases.append((len(src[i % 3]) if rng.random() < 0.8 else int(rng.integers(0, 30000)), bytes(b)))
    out = _run_check(host_check, "d", b"".join(struct.pack("<II", u, len(b)) + b for u, b in cases), tmp_path)
    p = 0
    for u, b in cases:
        (ok,) = struct.unpack_from("<i", out, p)
        p += 4
        want, y = o.decompress_block(b, u)
        assert bool(ok) == want
        if ok:
            assert out[p:p + u] == y
            p += u


def test_synthetic_blocks_valid_under_oracle(o):
    """tests/lz4_blocks.py (the two-pass GPU decoder's edge-case inputs):
    every block it builds is accepted by the oracle with the expected bytes."""
    from lz4_blocks import random_block
    rng = np.random.default_rng(5)
    for t in range(40):
        body, want = random_block(rng, int(rng.choice([100, 5000, 70000])))
        r, ulen, got = o.uncompress(body, cap=len(want))
        assert r == 1 and ulen == len(want) and got == want, t
