"""GPU parity: the HIP path (through the C ABI) against the oracle and the
golden vectors generated from the reference.  Bit-exact: every compressed
byte, every decompressed byte, every status."""
import json
from pathlib import Path

import numpy as np
import pytest

import fsg
from bind import Oracle
from gen_inputs import build_input

GOLDEN = Path(__file__).resolve().parent / "golden"
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    from gpu_harness import GpuCodec
    return GpuCodec()


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def test_golden_vectors_compress_and_decompress(gpu):
    vecs = json.loads((GOLDEN / "vectors.json").read_text())
    datas = [build_input(v) for v in vecs]
    comps, st = gpu.compress(fsg.Batch.from_list(datas))
    assert (st == fsg.FSG_OK).all()
    for v, c in zip(vecs, comps):
        assert len(c) == v["compressed_len"], v["name"]
        assert "%016x" % fsg.fnv1a64(c) == v["compressed_fnv"], v["name"]
        if "compressed_hex" in v:
            assert c.hex() == v["compressed_hex"], v["name"]
    outs, ol, st = gpu.decompress(comps, [len(d) for d in datas])
    assert (st == fsg.FSG_OK).all()
    for v, d, o, l in zip(vecs, datas, outs, ol):
        assert l == len(d) and o == d, v["name"]


def test_golden_negative_verdicts(gpu):
    negs = [v for v in json.loads((GOLDEN / "negative.json").read_text()) if v["ok"] is not None]
    comps = [bytes.fromhex(v["hex"]) for v in negs]
    caps = [v["ulen"] if v["header_ok"] else 0 for v in negs]
    outs, ol, st = gpu.decompress(comps, caps)
    for v, o, l, s in zip(negs, outs, ol, st):
        if not v["header_ok"]:
            assert s == fsg.FSG_BAD_HEADER, v["name"]
            continue
        assert l == v["ulen"], v["name"]
        assert (s == fsg.FSG_OK) == v["ok"], (v["name"], s)
        if v["ok"]:
            assert "%016x" % fsg.fnv1a64(o) == v["output_fnv"], v["name"]
    # validate-only mode == IsValidCompressedBuffer
    allv = json.loads((GOLDEN / "negative.json").read_text())
    _, _, st = gpu.decompress([bytes.fromhex(v["hex"]) for v in allv], [0] * len(allv),
                              flags=fsg.FSG_FLAG_VALIDATE_ONLY)
    for v, s in zip(allv, st):
        assert (s == fsg.FSG_OK) == v["valid"], v["name"]


def test_strict_header_flag(gpu):
    negs = json.loads((GOLDEN / "negative.json").read_text())
    comps = [bytes.fromhex(v["hex"]) for v in negs]
    _, _, st = gpu.decompress(comps, [0] * len(comps),
                              flags=fsg.FSG_FLAG_STRICT_HEADER | fsg.FSG_FLAG_VALIDATE_ONLY)
    for v, s in zip(negs, st):
        if not v["strict_header_ok"]:
            assert s == fsg.FSG_BAD_HEADER, v["name"]


def test_slot_too_small(gpu, oracle):
    data = fsg.make_batch(fsg.KIND_TEXT, [5000]).item(0)
    c = oracle.compress(data)
    _, ol, st = gpu.decompress([c, c], [4999, 5000])
    assert st[0] == fsg.FSG_SLOT_TOO_SMALL and st[1] == fsg.FSG_OK and ol[0] == 5000


@pytest.mark.parametrize("name", ["C2", "C3", "CM", "C5"])
def test_config_digests(gpu, name):
    d = np.load(GOLDEN / f"digests_{name}.npz")
    n = len(d["input_len"])
    kind = {"C2": fsg.KIND_RANDOM, "C3": fsg.KIND_TEXT, "CM": fsg.KIND_MIXED, "C5": fsg.KIND_PROTO}[name]
    sizes = {"C2": np.full(n, 4096), "C3": np.full(n, 65536), "CM": fsg.mixed_sizes(n),
             "C5": fsg.mixed_sizes(n)}[name]
    b = fsg.make_batch(kind, sizes)
    comps, st = gpu.compress(b)
    assert (st == 0).all()
    clen = np.array([len(c) for c in comps], np.uint32)
    assert np.array_equal(clen, d["compressed_len"])
    assert np.array_equal(np.array([fsg.fnv1a64(c) for c in comps], np.uint64), d["compressed_fnv"])
    outs, ol, st = gpu.decompress(comps, list(b.lens))
    assert (st == 0).all()
    assert all(o == b.item(i) for i, o in enumerate(outs))


def test_randomized_against_oracle(gpu, oracle):
    rng = np.random.default_rng(3)
    items = []
    for t in range(400):
        n = int(rng.choice([rng.integers(0, 100), rng.integers(0, 5000), rng.integers(0, 140000)]))
        alpha = int(rng.choice([2, 3, 8, 40, 256]))
        items.append(rng.integers(0, alpha, n, dtype=np.uint8).tobytes())
    comps, st = gpu.compress(fsg.Batch.from_list(items))
    assert (st == 0).all()
    for x, c in zip(items, comps):
        assert c == oracle.compress(x)
    outs, ol, st = gpu.decompress(comps, [len(x) for x in items])
    assert (st == 0).all() and all(o == x for o, x in zip(outs, items))


def test_decode_fuzz_against_oracle(gpu, oracle):
    rng = np.random.default_rng(9)
    srcs = [fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0) for s in (64, 700, 9000, 70000)]
    comps, caps = [], []
    for _ in range(3000):
        c = bytearray(oracle.compress(srcs[int(rng.integers(len(srcs)))]))
        for _ in range(int(rng.integers(1, 4))):
            c[int(rng.integers(len(c)))] = int(rng.integers(256))
        if rng.random() < 0.3:
            c = c[: int(rng.integers(1, len(c) + 1))]
        comps.append(bytes(c))
        caps.append(1 << 17)
    outs, ol, st = gpu.decompress(comps, caps)
    for c, o, l, s in zip(comps, outs, ol, st):
        ok, ulen, ref = oracle.uncompress(c, cap=1 << 17)
        if ok is None:
            assert s == fsg.FSG_SLOT_TOO_SMALL
            continue
        if not ok:
            assert s in (fsg.FSG_CORRUPT, fsg.FSG_BAD_HEADER)
        else:
            assert s == fsg.FSG_OK and o[:ulen] == ref


@pytest.mark.parametrize("variant", [1, 2])
def test_kernel_variants_agree(gpu, oracle, variant):
    """Both generations of kernels give the oracle's bytes and statuses."""
    gpu.codec.select_kernels(variant, variant)
    try:
        vecs = json.loads((GOLDEN / "vectors.json").read_text())
        datas = [build_input(v) for v in vecs if v["input_len"] <= 200000]
        comps, st = gpu.compress(fsg.Batch.from_list(datas))
        assert (st == 0).all()
        assert all(c == oracle.compress(d) for c, d in zip(comps, datas))
        outs, ol, st = gpu.decompress(comps, [len(d) for d in datas])
        assert (st == 0).all() and all(o == d for o, d in zip(outs, datas))
        negs = [v for v in json.loads((GOLDEN / "negative.json").read_text()) if v["ok"] is not None]
        _, _, st = gpu.decompress([bytes.fromhex(v["hex"]) for v in negs],
                                  [v["ulen"] if v["header_ok"] else 0 for v in negs])
        for v, s in zip(negs, st):
            assert (s == 0) == bool(v["ok"]), v["name"]
    finally:
        gpu.codec.select_kernels(0, 0)


@pytest.mark.parametrize("lanes", [0, 64, 1000])
def test_persistent_decode_lane_counts(gpu, oracle, lanes):
    """Bounded-lane persistent decode (lanes pull messages from a device
    counter) gives the same bytes/statuses for any lane count."""
    gpu.codec.set_decode_lanes(lanes)
    try:
        rng = np.random.default_rng(lanes + 1)
        items = [fsg.make_batch(fsg.KIND_TEXT, [int(rng.integers(0, 70000))], first_index=i).item(0)
                 for i in range(300)]
        comps = [oracle.compress(x) for x in items]
        comps[7] = comps[7][:-3]                       # truncated -> CORRUPT
        comps[11] = b"\x80"                            # bad header
        outs, ol, st = gpu.decompress(comps, [len(x) for x in items])
        for i, (x, c, o, s) in enumerate(zip(items, comps, outs, st)):
            ok, ulen, ref = oracle.uncompress(c, cap=len(x))
            assert (s == fsg.FSG_OK) == bool(ok), i
            if ok:
                assert o == x
        assert st[11] == fsg.FSG_BAD_HEADER
    finally:
        gpu.codec.set_decode_lanes(16384)


def test_empty_batch_and_empty_messages(gpu):
    comps, st = gpu.compress(fsg.Batch.from_list([b"", b"", b"x"]))
    assert comps == [b"\x00", b"\x00", b"\x01\x00x"] and (st == 0).all()
    outs, ol, st = gpu.decompress([b"\x00"], [0])
    assert st[0] == 0 and ol[0] == 0
