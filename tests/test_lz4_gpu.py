"""GPU parity of the LZ4 path (flare-cpp_amd/csrc/lz4.hip) through the C ABI
(include/flare_lz4_gpu.h): bodies byte-equal to the oracle and to the liblz4
fixtures, every decode verdict and byte equal to the oracle's."""
import json
from pathlib import Path

import numpy as np
import pytest

import fsg
from bind import Lz4Oracle
from gen_inputs import build_input

pytestmark = pytest.mark.gpu
GOLDEN = Path(__file__).resolve().parent / "golden"
VEC = json.loads((GOLDEN / "lz4_vectors.json").read_text())


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    from gpu_harness import GpuCodec
    return GpuCodec()


@pytest.fixture(scope="module")
def o():
    return Lz4Oracle()


def _header(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


def test_lz4_compress_matches_liblz4_fixtures(gpu, o):
    vecs = [v for v in VEC["compress"] if v["input_len"] <= 1 << 20]
    xs = [build_input(v) for v in vecs]
    bodies, st = gpu.lz4_compress(fsg.Batch.from_list(xs))
    assert (st == fsg.FSG_OK).all()
    for v, x, body in zip(vecs, xs, bodies):
        h = _header(len(x))
        assert body[:len(h)] == h, v["name"]
        blk = body[len(h):]
        assert len(blk) == v["block_len"] and "%016x" % fsg.fnv1a64(blk) == v["block_fnv"], v["name"]
        assert body == o.compress(x), v["name"]
    outs, ol, st = gpu.lz4_decompress(bodies, [len(x) for x in xs])
    assert (st == fsg.FSG_OK).all()
    assert all(y == x for y, x in zip(outs, xs))


def test_lz4_randomized_against_oracle(gpu, o):
    rng = np.random.default_rng(17)
    xs = []
    for t in range(600):
        n = int(rng.choice([rng.integers(0, 40), rng.integers(0, 5000), rng.integers(60000, 70000),
                            rng.integers(0, 200000)]))
        alpha = int(rng.choice([1, 2, 4, 40, 256]))
        xs.append(rng.integers(0, alpha, n, dtype=np.uint8).tobytes())
    xs += [fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0) for s in (13, 64, 4096, 65546, 65547, 100000)]
    bodies, st = gpu.lz4_compress(fsg.Batch.from_list(xs))
    assert (st == 0).all()
    for x, b in zip(xs, bodies):
        assert b == o.compress(x), len(x)
    outs, ol, st = gpu.lz4_decompress(bodies, [len(x) for x in xs])
    assert (st == 0).all() and all(y == x for y, x in zip(outs, xs))


def test_lz4_decode_verdicts_against_oracle(gpu, o):
    cases = VEC["decode"]
    bodies = [_header(d["ulen"]) + bytes.fromhex(d["hex"]) for d in cases]
    rng = np.random.default_rng(3)
    src = [fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0) for s in (40, 900, 20000)]
    for i in range(1500):  # mutated bodies, header included
        b = bytearray(o.compress(src[i % 3]))
        for _ in range(int(rng.integers(1, 3))):
            b[int(rng.integers(len(b)))] = int(rng.integers(256))
        if rng.random() < 0.3:
            b = b[:int(rng.integers(1, len(b) + 1))]
        bodies.append(bytes(b))
    cap = 1 << 16
    outs, ol, st = gpu.lz4_decompress(bodies, [cap] * len(bodies))
    for i, (b, y, l, s) in enumerate(zip(bodies, outs, ol, st)):
        r, ulen, ref = o.uncompress(b, cap=cap)
        want = {1: fsg.FSG_OK, 0: fsg.FSG_CORRUPT, -1: fsg.FSG_BAD_HEADER, -2: fsg.FSG_SLOT_TOO_SMALL}[r]
        assert s == want, (i, r, s)
        if r == 1:
            assert y == ref, i
    for d, s in zip(cases, st[:len(cases)]):
        if not d["offset0"]:
            assert (s == fsg.FSG_OK) == d["liblz4_ok"]


def test_lz4_empty_and_edges(gpu, o):
    xs = [b"", b"x", b"a" * 12, b"a" * 13, bytes(65547)]
    bodies, st = gpu.lz4_compress(fsg.Batch.from_list(xs))
    assert (st == 0).all() and bodies[0] == b"\x00\x00"
    outs, ol, st = gpu.lz4_decompress(bodies + [b"", b"\x05\x50hello"], [len(x) for x in xs] + [0, 4])
    assert list(st) == [0] * 5 + [fsg.FSG_BAD_HEADER, fsg.FSG_SLOT_TOO_SMALL]
    assert outs[:5] == xs
