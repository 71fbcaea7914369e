"""Oracle pinning (CPU only): the C restatement (oracle/snappy_oracle.c) against
the committed golden vectors generated from the reference's own snappy.cc, and
-- where oracle/_ref was built -- directly against the reference on
randomized inputs."""
import json
import random
from pathlib import Path

import numpy as np
import pytest

import fsg
from bind import Oracle, Reference
from gen_inputs import build_input

GOLDEN = Path(__file__).resolve().parent / "golden"


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def _vectors():
    return json.loads((GOLDEN / "vectors.json").read_text())


def _negatives():
    return json.loads((GOLDEN / "negative.json").read_text())


def test_max_compressed_length(oracle):
    for n in (0, 1, 5, 6, 4096, 65536, 1 << 20):
        assert oracle.max_compressed_length(n) == 32 + n + n // 6
    assert oracle.max_compressed_length(4096) == 4810
    assert oracle.max_compressed_length(65536) == 76490


@pytest.mark.parametrize("v", _vectors(), ids=lambda v: v["name"])
def test_oracle_compress_golden(oracle, v):
    data = build_input(v)
    assert len(data) == v["input_len"]
    assert "%016x" % fsg.fnv1a64(data) == v["input_fnv"]
    comp = oracle.compress(data)
    assert len(comp) == v["compressed_len"]
    assert "%016x" % fsg.fnv1a64(comp) == v["compressed_fnv"]
    if "compressed_hex" in v:
        assert comp.hex() == v["compressed_hex"]
    ok, ulen, out = oracle.uncompress(comp)
    assert ok and ulen == len(data) and out == data


def test_known_answer_200_pattern(oracle):
    # the 200-byte a..z0..9 pattern (rpc_snappy_compress_test.cc:139-166)
    data = build_input({"gen": "pattern", "size": 200, "digits": True})
    assert oracle.compress(data).hex() == (
        "c801" + "90" + data[:37].hex() + "fe2400" + "fe2400" + "8a2400")


def test_known_answer_random_4k_header(oracle):
    data = fsg.make_batch(fsg.KIND_RANDOM, [4096]).item(0)
    comp = oracle.compress(data)
    assert len(comp) == 4101 and comp[:5].hex() == "8020f4ff0f"


def test_known_answer_text_64k(oracle):
    data = fsg.make_batch(fsg.KIND_TEXT, [65536]).item(0)
    assert data.startswith(b"jkvd dcgbv\nzzv ugzoj ")
    assert len(oracle.compress(data)) == 32380


@pytest.mark.parametrize("v", _negatives(), ids=lambda v: v["name"])
def test_oracle_decode_verdicts_golden(oracle, v):
    comp = bytes.fromhex(v["hex"])
    h, ulen = oracle.header(comp, lenient=True)
    assert bool(h) == v["header_ok"]
    if h:
        assert ulen == v["ulen"]
    hs, _ = oracle.header(comp, lenient=False)
    assert bool(hs) == v["strict_header_ok"]
    assert oracle.is_valid(comp) == v["valid"]
    if v["ok"] is None:
        return
    ok, ulen2, out = oracle.uncompress(comp, cap=v["ulen"] if v["header_ok"] else 0)
    assert bool(ok) == v["ok"]
    if ok:
        assert "%016x" % fsg.fnv1a64(out) == v["output_fnv"]


@pytest.mark.parametrize("name", ["C2", "C3", "CM", "C5"])
def test_oracle_config_digests(oracle, name):
    d = np.load(GOLDEN / f"digests_{name}.npz")
    n = len(d["input_len"])
    kind = {"C2": fsg.KIND_RANDOM, "C3": fsg.KIND_TEXT, "CM": fsg.KIND_MIXED, "C5": fsg.KIND_PROTO}[name]
    sizes = {"C2": np.full(n, 4096), "C3": np.full(n, 65536), "CM": fsg.mixed_sizes(n),
             "C5": fsg.mixed_sizes(n)}[name]
    b = fsg.make_batch(kind, sizes)
    assert np.array_equal(b.lens, d["input_len"])
    assert np.array_equal(fsg.digests(b.data, b.offsets, b.lens), d["input_fnv"])
    # batched oracle (threads) must equal per-message digests
    caps = np.array([32 + x + x // 6 for x in b.lens], dtype=np.uint32)
    oo, tot = fsg.slot_offsets(caps)
    out = np.zeros(tot, np.uint8)
    olen = np.zeros(n, np.uint32)
    oracle.compress_batch(b.data, b.offsets, b.lens, out, oo, olen, threads=4)
    assert np.array_equal(olen, d["compressed_len"])
    assert np.array_equal(fsg.digests(out, oo, olen), d["compressed_fnv"])
    # batched decode round trip
    dout = np.zeros(max(b.total, 1), np.uint8)
    dlen = np.zeros(n, np.uint32)
    st = np.full(n, -1, np.int32)
    oracle.uncompress_batch(out, oo, olen, dout, b.offsets, b.lens.copy(), dlen, st, threads=4)
    assert (st == 0).all() and np.array_equal(dlen, b.lens)
    assert np.array_equal(dout[:b.total], b.data[:b.total])


@pytest.mark.skipif(not Reference.available(), reason="oracle/_ref not built here")
def test_oracle_matches_reference_randomized(oracle):
    ref = Reference()
    rng = random.Random(11)
    for t in range(200):
        n = rng.choice([rng.randint(0, 80), rng.randint(0, 3000), rng.randint(0, 150000)])
        alpha = rng.choice([2, 4, 16, 64, 256])
        data = np.random.default_rng(t).integers(0, alpha, n, dtype=np.uint8).tobytes()
        comp = oracle.compress(data)
        assert comp == ref.compress(data, rng.choice([1, 13, 8160, 65536]))
        ok, out = ref.uncompress(comp, len(data))
        assert ok and out == data


@pytest.mark.skipif(not Reference.available(), reason="oracle/_ref not built here")
def test_oracle_decode_fuzz_matches_reference(oracle):
    ref = Reference()
    rng = random.Random(5)
    srcs = [fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0) for s in (40, 900, 20000)]
    for _ in range(1500):
        c = bytearray(oracle.compress(rng.choice(srcs)))
        for _ in range(rng.randint(1, 3)):
            c[rng.randrange(len(c))] = rng.randrange(256)
        if rng.random() < 0.3:
            c = c[: rng.randrange(1, len(c) + 1)]
        c = bytes(c)
        ok, ulen, out = oracle.uncompress(c, cap=1 << 20)
        if ok is None:
            continue
        rok, rout = ref.uncompress(c, 1 << 20, rng.choice([1, 8160]))
        assert bool(ok) == rok
        if ok:
            assert out == rout[:ulen]


def _agg(col):
    return fsg.fnv1a64(np.ascontiguousarray(col, np.uint64).tobytes())


@pytest.mark.parametrize("name", ["C2", "C3", "CM", "C5"])
def test_full_size_fixtures(oracle, name):
    """The full-size reference digests (tests/golden/full_*.npz, SURVEY §8(c)
    item 4) agree with the committed prefix digests, their aggregates with
    their columns, and the C restatement reproduces a strided sample of the
    whole batch (every 2,048th message; CM every 32,768th, C5 every 8,192nd)."""
    f = np.load(GOLDEN / f"full_{name}.npz")
    d = np.load(GOLDEN / f"digests_{name}.npz")
    k = len(d["compressed_len"])
    assert np.array_equal(f["compressed_len"][:k], d["compressed_len"])
    n = len(f["compressed_len"])
    assert n == {"CM": 1 << 20, "C5": 262144}.get(name, 65536)
    if name in ("C2", "C3"):
        assert np.array_equal(f["compressed_fnv"][:k], d["compressed_fnv"])
        assert np.array_equal(f["input_fnv"][:k], d["input_fnv"])
        assert int(f["aggregate"][0]) == _agg(f["input_fnv"]) and int(f["aggregate"][1]) == _agg(f["compressed_fnv"])
        sizes = np.full(n, 4096 if name == "C2" else 65536, np.uint32)
        step = 2048
    elif name == "C5":
        assert np.array_equal(f["compressed_fnv"][:k], d["compressed_fnv"])
        assert int(f["aggregate"][1]) == _agg(f["compressed_fnv"])
        assert int(f["totals"][1]) == int(f["compressed_len"].astype(np.uint64).sum())
        sizes = fsg.mixed_sizes(n)
        step = 8192
    else:
        sizes = fsg.mixed_sizes(n)
        assert int(f["totals"][0]) == int(sizes.astype(np.uint64).sum())
        assert int(f["totals"][1]) == int(f["compressed_len"].astype(np.uint64).sum())
        step = 32768
    kind = {"C2": fsg.KIND_RANDOM, "C3": fsg.KIND_TEXT, "CM": fsg.KIND_MIXED, "C5": fsg.KIND_PROTO}[name]
    for i in range(7, n, step):
        x = fsg.make_batch(kind, sizes[i:i + 1], first_index=i).item(0)
        c = oracle.compress(x)
        assert len(c) == f["compressed_len"][i], i
        if name != "CM":
            assert fsg.fnv1a64(c) == f["compressed_fnv"][i], i
        if name in ("C2", "C3"):
            assert fsg.fnv1a64(x) == f["input_fnv"][i], i


# ---- UncompressAsMuchAsPossible and RawUncompressToIOVec restated
# (snappy.cc:1530-1535, :963-1132): pinned to the negative.json fixtures
# (made by the reference, 8160-byte source pieces) and to the reference build.

@pytest.mark.parametrize("v", _negatives(), ids=lambda v: v["name"])
def test_oracle_as_much_golden(oracle, v):
    if v["ok"] is None or not v["header_ok"]:
        return
    r, got = oracle.uncompress_as_much(bytes.fromhex(v["hex"]), v["ulen"], frag=8160)
    assert r == v["partial_ret"]
    assert len(got) == v["partial_len"]
    assert "%016x" % fsg.fnv1a64(got) == v["partial_fnv"]


def _partial_frag_cases():
    return json.loads((GOLDEN / "partial_frag.json").read_text())


def test_oracle_as_much_small_pieces_golden(oracle):
    """Long-literal tags straddling 1-, 3- and 7-byte source pieces (RefillTag
    stitching, snappy.cc:790-847), pinned to the reference's own results
    (tests/golden/partial_frag.json, make_golden.py)."""
    cases = _partial_frag_cases()
    assert len(cases) >= 200
    for v in cases:
        r, got = oracle.uncompress_as_much(bytes.fromhex(v["hex"]), v["ulen"], frag=v["frag"])
        key = (v["frag"], v["nbytes"], v["before"], v["kind"])
        assert r == v["ret"] and len(got) == v["got_len"], key
        assert "%016x" % fsg.fnv1a64(got) == v["got_fnv"], key


def _mutants(oracle, rng, count):
    srcs = [fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0) for s in (40, 900, 20000, 70000, 140000)]
    for _ in range(count):
        c = bytearray(oracle.compress(rng.choice(srcs)))
        for _ in range(rng.randint(0, 3)):
            c[rng.randrange(len(c))] = rng.randrange(256)
        if rng.random() < 0.3:
            c = c[: rng.randrange(1, len(c) + 1)]
        yield bytes(c)


@pytest.mark.skipif(not Reference.available(), reason="oracle/_ref not built here")
def test_oracle_as_much_matches_reference(oracle):
    ref = Reference()
    rng = random.Random(23)
    n_partial = 0
    for c in _mutants(oracle, rng, 600):
        h, ulen = oracle.header(c)
        if not h or ulen > 1 << 20:
            continue
        frag = rng.choice([0, 1, 7, 8160])
        r, got = oracle.uncompress_as_much(c, ulen, frag)
        rr, rgot = ref.uncompress_as_much(c, ulen, frag if frag else len(c))
        assert (r, got) == (rr, rgot), frag
        n_partial += r != ulen
    assert n_partial > 50


def _iov_split(rng, total):
    """Random iovec lengths: empty ones, exact, short and roomy lists."""
    k = rng.randint(1, 6)
    cuts = sorted(rng.randint(0, total) for _ in range(k - 1))
    lens = [b - a for a, b in zip([0] + cuts, cuts + [total])]
    mode = rng.random()
    if mode < 0.2 and lens:
        lens[-1] += rng.randint(1, 40)          # room to spare
    elif mode < 0.35 and total:
        lens[rng.randrange(len(lens))] = max(0, lens[-1] - rng.randint(1, 20))  # too short
    if rng.random() < 0.3:
        lens.insert(rng.randrange(len(lens) + 1), 0)
    return lens


@pytest.mark.skipif(not Reference.available(), reason="oracle/_ref not built here")
def test_oracle_iovec_matches_reference(oracle):
    ref = Reference()
    rng = random.Random(29)
    seen = {True: 0, False: 0}
    for c in _mutants(oracle, rng, 600):
        h, ulen = oracle.header(c)
        if not h or ulen > 1 << 20:
            continue
        lens = _iov_split(rng, ulen)
        ok, bufs = oracle.uncompress_iovec(c, lens)
        rok, rbufs = ref.uncompress_iovec(c, lens)
        assert ok == rok
        assert bufs == rbufs  # the prefix the reference leaves on failure too
        if ok:
            flat = oracle.uncompress(c)[2]
            assert b"".join(bufs)[:ulen] == flat
        seen[ok] += 1
    assert seen[True] > 50 and seen[False] > 50
