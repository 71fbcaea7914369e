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


@pytest.mark.parametrize("small_batch", [0, 64])
def test_small_batch_verdicts(gpu, oracle, small_batch, fsg_opts):
    """Batches of <= 64 messages index every body with a wave (pass 1b) by
    default (option small_batch); small_batch 0 keeps them on the lane walk.
    Both: the reference's verdicts and bytes on the negative vectors and on
    mutated text bodies, in batches of 1, 17 and 64."""
    fsg_opts(small_batch=small_batch)
    negs = [v for v in json.loads((GOLDEN / "negative.json").read_text()) if v["ok"] is not None]
    comps = [bytes.fromhex(v["hex"]) for v in negs]
    rng = np.random.default_rng(5)
    srcs = [fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0) for s in (100, 3000, 20000, 70000)]
    for k in range(120):
        c = bytearray(oracle.compress(srcs[k % len(srcs)]))
        if k % 3:
            c[int(rng.integers(len(c)))] = int(rng.integers(256))
        if k % 7 == 0:
            c = c[: int(rng.integers(1, len(c) + 1))]
        comps.append(bytes(c))
    for size in (1, 17, 64):
        for b0 in range(0, len(comps), size if size > 1 else 11):
            part = comps[b0:b0 + size]
            outs, ol, st = gpu.decompress(part, [1 << 17] * len(part))
            for c, o, s in zip(part, outs, st):
                ok, ulen, ref = oracle.uncompress(c, cap=1 << 17)
                if ok is None:
                    assert s == fsg.FSG_SLOT_TOO_SMALL
                elif not ok:
                    assert s in (fsg.FSG_CORRUPT, fsg.FSG_BAD_HEADER)
                else:
                    assert s == fsg.FSG_OK and o[:ulen] == ref


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


@pytest.mark.parametrize("encoder", [0, 1])
def test_randomized_against_oracle(gpu, oracle, encoder):
    """Random-alphabet inputs (0 B to 140 KB): the default encoder and the
    LDS-table wave encoder (v1, DPP row exchanges) byte-equal to the oracle."""
    gpu.codec.select_kernels(0, encoder)
    rng = np.random.default_rng(3 + encoder)
    items = []
    for t in range(400 if encoder == 0 else 150):
        n = int(rng.choice([rng.integers(0, 100), rng.integers(0, 5000), rng.integers(0, 140000)]))
        alpha = int(rng.choice([2, 3, 8, 40, 256]))
        items.append(rng.integers(0, alpha, n, dtype=np.uint8).tobytes())
    try:
        comps, st = gpu.compress(fsg.Batch.from_list(items))
    finally:
        gpu.codec.select_kernels(0, 0)
    assert (st == 0).all()
    for x, c in zip(items, comps):
        assert c == oracle.compress(x)
    outs, ol, st = gpu.decompress(comps, [len(x) for x in items])
    assert (st == 0).all() and all(o == x for o, x in zip(outs, items))


@pytest.mark.parametrize("variant,fork", [(0, "0"), (3, "0"), (4, "0"), (0, "1"), (0, "1p"), (0, "1k"), (0, "1s0"),
                                          (0, "1s1"), (0, "1s2")])
def test_decode_fuzz_against_oracle(gpu, oracle, variant, fork, fsg_opts):
    """Mutated and truncated streams (64 B to 70 KB bodies).  fork "1" runs
    the path of batches over 128K messages: plan pass, the large messages'
    passes on side streams, the small ones on a persistent grid; "1p" with the small
    messages' execution grid shrunk to 5 blocks, so each wave loops over
    ~150 messages (FSG_SMALL_PERSIST); "1sK" with FSG_SPLIT_WALK=K (0: the
    small bodies executed in message order; 1: walk and execution split by
    size on two streams; 2: one execution launch in walk order; default 3:
    two execution launches by size); "1k": the smaller bodies packed 32 to a
    wave (exec_pack 32) instead of one wave each."""
    fsg_opts(decode_fork=fork[0])
    fsg_opts(small_persist="5" if fork == "1p" else "1792")
    if fork == "1k":
        fsg_opts(exec_pack=32)
    fsg_opts(split_walk=fork[2] if fork.startswith("1s") else "3")
    gpu.codec.select_kernels(variant, 0)
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
    gpu.codec.select_kernels(0, 0)


@pytest.mark.parametrize("fork", ["0", "1", "1c"])
def test_large_message_index_fuzz(gpu, oracle, fork, fsg_opts):
    """Compressed bodies over 48 KiB take the wave-per-message index pass
    (index_big_kernel): intact, bit-flipped and truncated ones, mixed with
    small ones in one batch, against the oracle's verdicts and bytes.  With
    FSG_DECODE_FORK=1 pass 1b and the large-message exec blocks run on the
    library's side stream beside the small messages' exec launch (the
    default for batches of > 128K messages).  "1c": the huge bodies (> 256 KiB
    compressed) through the chunked pass 1b (FSG_CHUNKED_HUGE=1), corruption
    in every chunk position included."""
    fsg_opts(decode_fork=fork[0])
    fsg_opts(chunked_huge="1" if fork == "1c" else "0")
    rng = np.random.default_rng(21)
    srcs = [fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0) for s in (120000, 400000, 1 << 20)]
    if fork == "1c":  # more huge bodies: 3 MiB text, text with a long random run across chunks
        srcs.append(fsg.make_batch(fsg.KIND_TEXT, [3 << 20], first_index=77).item(0))
        t = fsg.make_batch(fsg.KIND_TEXT, [900000], first_index=78).item(0)
        srcs.append(t[:300000] + fsg.make_batch(fsg.KIND_RANDOM, [100000], first_index=79).item(0) + t[300000:])
    srcs.append(fsg.make_batch(fsg.KIND_RANDOM, [70000]).item(0))
    srcs.append(fsg.make_batch(fsg.KIND_TEXT, [3000]).item(0))  # small, lane path
    base = [oracle.compress(s) for s in srcs]
    assert all(len(c) > 48 * 1024 for c in base[:4])
    comps, caps = [], []
    for i in range(160 if fork != "1c" else 224):
        c = bytearray(base[i % len(base)])
        mode = i // len(base) % 4
        if mode == 1:
            for _ in range(int(rng.integers(1, 4))):
                c[int(rng.integers(len(c)))] = int(rng.integers(256))
        elif mode == 2:
            c = c[: int(rng.integers(1, len(c) + 1))]
        elif mode == 3:  # corrupt late in the stream
            c[len(c) - 1 - int(rng.integers(min(64, len(c) - 1)))] ^= 0x5A
        comps.append(bytes(c))
        caps.append(1 << 22)
    outs, ol, st = gpu.decompress(comps, caps)
    for i, (c, o, l, s) in enumerate(zip(comps, outs, ol, st)):
        ok, ulen, ref = oracle.uncompress(c, cap=1 << 22)
        if ok is None:
            assert s == fsg.FSG_SLOT_TOO_SMALL, i
        elif not ok:
            assert s in (fsg.FSG_CORRUPT, fsg.FSG_BAD_HEADER), i
        else:
            assert s == fsg.FSG_OK and o[:ulen] == ref, i


@pytest.mark.parametrize("variant", [1, 3, 4, 5])
def test_kernel_variants_agree(gpu, oracle, variant):
    """Every generation of kernels gives the oracle's bytes and statuses."""
    gpu.codec.select_kernels(variant, min(variant, 3))
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


def test_empty_batch_and_empty_messages(gpu):
    comps, st = gpu.compress(fsg.Batch.from_list([b"", b"", b"x"]))
    assert comps == [b"\x00", b"\x00", b"\x01\x00x"] and (st == 0).all()
    outs, ol, st = gpu.decompress([b"\x00"], [0])
    assert st[0] == 0 and ol[0] == 0


def _lit(b: bytes) -> bytes:
    n = len(b) - 1
    if n < 60:
        return bytes([n << 2]) + b
    k = (n.bit_length() + 7) // 8
    return bytes([(59 + k) << 2]) + n.to_bytes(k, "little") + b


def _copy(off: int, ln: int, wide: bool = False) -> bytes:
    if wide or off > 0xFFFF:                             # COPY_4
        return bytes([((ln - 1) << 2) | 3]) + off.to_bytes(4, "little")
    if 4 <= ln <= 11 and off < 2048:                     # COPY_1
        return bytes([((off >> 8) << 5) | ((ln - 4) << 2) | 1, off & 0xFF])
    return bytes([((ln - 1) << 2) | 2]) + off.to_bytes(2, "little")  # COPY_2


def _synthetic_stream(rng, target):
    """A valid-by-construction tag stream stressing what the encoder rarely
    emits: offsets 1..15 (pattern copies) at every length 1..64, COPY_4,
    long literals (which jump the decoder's input ring), back-to-back short
    copies, and output ends at every alignment."""
    body, out = [], bytearray()
    first = bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8))
    body.append(_lit(first)); out += first
    while len(out) < target:
        r = rng.random()
        if r < 0.45:
            off = int(rng.integers(1, min(16, len(out)) + 1))
        elif r < 0.75:
            off = int(rng.integers(1, min(300, len(out)) + 1))
        elif r < 0.85:
            off = int(rng.integers(1, len(out) + 1))
        else:
            n = int(rng.integers(1, 3000 if rng.random() < 0.1 else 30))
            lit = bytes(rng.integers(0, 256, n, dtype=np.uint8))
            body.append(_lit(lit)); out += lit
            continue
        ln = int(rng.integers(1, 65))
        body.append(_copy(off, ln, wide=rng.random() < 0.05))
        for _ in range(ln):
            out.append(out[-off])
    hdr = bytearray()
    n = len(out)
    while n >= 0x80:
        hdr.append((n & 0x7F) | 0x80); n >>= 7
    hdr.append(n)
    return bytes(hdr) + b"".join(body), bytes(out)


@pytest.mark.parametrize("variant", [0, 1, 3, 4])
def test_pattern_copies_and_ring_jumps(gpu, oracle, variant):
    """Hand-built streams: every small offset/length combination, COPY_4 and
    long literals, at output ends of every alignment; decoded bytes equal the
    oracle's (and the construction's)."""
    gpu.codec.select_kernels(variant, 0)
    try:
        rng = np.random.default_rng(2024 + variant)
        comps, raws = [], []
        for i in range(600):
            target = int(rng.integers(1, 9000)) if i % 5 else int(rng.integers(20000, 70000))
            c, raw = _synthetic_stream(rng, target)
            comps.append(c); raws.append(raw)
        outs, ol, st = gpu.decompress(comps, [len(r) for r in raws])
        for i, (c, raw, o, s) in enumerate(zip(comps, raws, outs, st)):
            ok, ulen, ref = oracle.uncompress(c, cap=len(raw))
            assert ok and ref == raw, i
            assert s == fsg.FSG_OK and o == raw, i
    finally:
        gpu.codec.select_kernels(0, 0)


@pytest.mark.parametrize("pack,skew", [(0, 0), (32, 0), (32, 7), (1, 3), (7, 5), (64, 0)])
def test_small_bodies_forked(gpu, oracle, pack, skew, fsg_opts):
    """Bodies under 512 compressed bytes on the forked path (the lane walk in
    size-class order + the small bodies' execution): text of every small
    size, hand-built streams (patterns of every offset, COPY_4, 4-byte
    literal lengths, literals over 64 bytes from global memory), random
    single literals, runs with a large output, the reference's negative
    vectors and mutated bodies, trailing zero-length literals -- bytes and
    statuses against the oracle.  (Round 5's one-lane-per-body pass for
    these, measured slower, was removed in round 6.)  pack: bodies per batch
    of the packed execution pass (exec_pack; 0 = a wave per body); skew:
    output slots of every alignment (gpu_harness slot_skew)."""
    fsg_opts(decode_fork=1, exec_pack=pack)
    rng = np.random.default_rng(77)
    comps = []
    for n in list(range(1, 200, 7)) + list(range(200, 800, 23)):
        comps.append(oracle.compress(fsg.make_batch(fsg.KIND_TEXT, [n], first_index=n).item(0)))
    for i in range(400):
        c, _ = _synthetic_stream(rng, int(rng.integers(1, 760)))
        comps.append(c)
    for n in (1, 15, 16, 17, 63, 64, 65, 100, 300, 490):
        comps.append(oracle.compress(rng.integers(0, 256, n, dtype=np.uint8).tobytes()))
    for n in (700, 768, 769, 2000, 5000, 20000):  # runs: small compressed, large output
        comps.append(oracle.compress(bytes([n % 251]) * n))
    comps.append(b"\x05" + _lit(b"abcde"))                          # 1-byte literal length field
    comps.append(b"\x46" + b"\xf0\x45" + bytes(range(70)))           # literal of 70 bytes, nb = 1
    comps.append(b"\x46" + b"\xfc\x45\x00\x00\x00" + bytes(range(70)))  # nb = 4
    comps.append(b"\x0a" + _lit(b"ab") + _copy(2, 8, wide=True))
    base = list(comps)
    for _ in range(600):
        c = bytearray(base[int(rng.integers(len(base)))])
        for _ in range(int(rng.integers(1, 3))):
            c[int(rng.integers(len(c)))] = int(rng.integers(256))
        if rng.random() < 0.2:
            c = c[: int(rng.integers(1, len(c) + 1))]
        comps.append(bytes(c))
    comps += [c + b"\xfc\xff\xff\xff\xff" for c in base[:40]]
    comps += [bytes.fromhex(v["hex"]) for v in json.loads((GOLDEN / "negative.json").read_text())
              if v["header_ok"] and v["ulen"] <= 1 << 16]
    # padded with larger text bodies so the batch has every path of the fork
    comps += [oracle.compress(fsg.make_batch(fsg.KIND_TEXT, [n], first_index=n).item(0))
              for n in (3000, 9000, 70000)]
    assert sum(len(c) < 512 for c in comps) > 1000
    caps = [1 << 17] * len(comps)
    outs, ol, st = gpu.decompress(comps, caps, slot_skew=skew)
    for i, (c, o, s) in enumerate(zip(comps, outs, st)):
        ok, ulen, ref = oracle.uncompress(c, cap=caps[i])
        if ok is None:
            assert s == fsg.FSG_SLOT_TOO_SMALL, i
        elif not ok:
            assert s in (fsg.FSG_CORRUPT, fsg.FSG_BAD_HEADER), (i, c[:16].hex(), s)
        else:
            assert s == fsg.FSG_OK and o[:ulen] == ref, (i, c[:16].hex(), s)


@pytest.mark.parametrize("total_in", [0, 1, 4096, 60000])
def test_two_pass_workspace_fallback(gpu, oracle, total_in):
    """v4 with a workspace sized for less input than the batch holds: the
    messages whose tag bitmap does not fit are finished by the v3 kernel
    (internal status kNeedFallback); every byte and status still matches."""
    gpu.codec.select_kernels(4, 0)
    try:
        rng = np.random.default_rng(77)
        items = [fsg.make_batch(fsg.KIND_TEXT if i % 3 else fsg.KIND_RANDOM,
                                [int(rng.integers(0, 70000))], first_index=i).item(0) for i in range(200)]
        comps = [oracle.compress(x) for x in items]
        comps[5] = comps[5][:-2]
        outs, ol, st = gpu.decompress(comps, [len(x) for x in items], ws_total_in=total_in)
        for i, (x, c, o, s) in enumerate(zip(items, comps, outs, st)):
            ok, ulen, ref = oracle.uncompress(c, cap=len(x))
            assert (s == fsg.FSG_OK) == bool(ok), (i, s)
            if ok:
                assert o == x, i
    finally:
        gpu.codec.select_kernels(0, 0)


@pytest.mark.parametrize("cap", [0, 4096, 40000])
def test_split_message_encode(gpu, oracle, cap):
    """Messages longer than 64 KiB are encoded one fragment per lane, staged
    per fragment and packed; capped staging regions force the whole-message
    fallback pass.  Bytes equal the oracle's either way."""
    gpu.codec.set_split_region_cap(cap)
    try:
        rng = np.random.default_rng(cap + 5)
        sizes = [65535, 65536, 65537, 131072, 131073, 200000, 1 << 20, 300001, 5, 70000]
        items = []
        for i, n in enumerate(sizes):
            kind = fsg.KIND_RANDOM if i % 3 == 1 else fsg.KIND_TEXT
            items.append(fsg.make_batch(kind, [n], first_index=100 + i).item(0))
        items.append(bytes(rng.integers(0, 4, 150000, dtype=np.uint8)))
        comps, st = gpu.compress(fsg.Batch.from_list(items))
        assert (st == 0).all()
        for x, c in zip(items, comps):
            assert c == oracle.compress(x), len(x)
        outs, ol, st = gpu.decompress(comps, [len(x) for x in items])
        assert (st == 0).all() and all(o == x for o, x in zip(outs, items))
    finally:
        gpu.codec.set_split_region_cap(0)


def _varint(n: int) -> bytes:
    out = bytearray()
    while True:
        b = n & 0x7F
        n >>= 7
        out.append(b | (0x80 if n else 0))
        if not n:
            return bytes(out)


def _literal(data: bytes, nbytes: int | None = None) -> bytes:
    """A LITERAL tag (snappy.cc:156-196 form) with `nbytes` length bytes (0 =
    length in the tag byte); non-minimal encodings are legal for the decoder."""
    n = len(data) - 1
    if nbytes is None:
        nbytes = 0 if n < 60 else (n.bit_length() + 7) // 8
    tag = (n << 2) if nbytes == 0 else ((59 + nbytes) << 2)
    return bytes([tag]) + (n.to_bytes(nbytes, "little") if nbytes else b"") + data


@pytest.mark.parametrize("variant", [0, 3, 4])
def test_single_literal_streams(gpu, oracle, variant):
    """Messages that are one literal take pass 2's straight-copy path (pass 1
    marks them); near misses (truncated, trailing bytes, a second tag, header
    disagreeing with the literal, non-minimal length bytes) must keep the
    reference's verdict and bytes."""
    import fsg as _f
    rng = np.random.default_rng(11)
    comps = []
    for n in [1, 2, 15, 16, 17, 59, 60, 61, 64, 65, 255, 256, 257, 1000, 4096, 4097, 8191, 40000]:
        d = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        for nb in sorted({None, 1, 2, 3, 4} if n <= 256 else {None, 3, 4}, key=lambda x: -1 if x is None else x):
            if nb is not None and n - 1 >= 1 << (8 * nb):
                continue
            s = _varint(n) + _literal(d, nb)
            comps += [s, s[:-1], s + b"\x00", _varint(n + 1) + s[len(_varint(n)):],
                      _varint(max(n - 1, 0)) + s[len(_varint(n)):]]
        comps.append(_varint(n + 4) + _literal(d) + bytes([0x01 | (0 << 2), 1]))  # + COPY_1 len 4 off 1
    # 4-byte length 0xffffffff wraps to a zero-length literal (uint32 arithmetic)
    comps.append(b"\x00" + bytes([63 << 2]) + b"\xff\xff\xff\xff")
    comps.append(b"\x05" + bytes([63 << 2]) + b"\xff\xff\xff\xff")
    # 5-byte lenient header in front of a literal
    comps.append(b"\x84\x80\x80\x80\x00" + _literal(b"abcd"))
    gpu.codec.select_kernels(variant, 0)
    try:
        outs, ol, st = gpu.decompress(comps, [1 << 17] * len(comps))
    finally:
        gpu.codec.select_kernels(0, 0)
    n_ok = 0
    for i, (c, o, s) in enumerate(zip(comps, outs, st)):
        ok, ulen, ref = oracle.uncompress(c, cap=1 << 17)
        if not ok:
            assert s in (_f.FSG_CORRUPT, _f.FSG_BAD_HEADER), (i, c[:8].hex(), s)
        else:
            n_ok += 1
            assert s == _f.FSG_OK and o[:ulen] == ref, (i, c[:8].hex(), s)
    assert n_ok > 40


def _copy2(length: int, offset: int) -> bytes:
    """COPY_2_BYTE_OFFSET tag (len 1..64, offset < 65536)."""
    return bytes([((length - 1) << 2) | 2]) + offset.to_bytes(2, "little")


def _copy4(length: int, offset: int) -> bytes:
    """COPY_4_BYTE_OFFSET tag (len 1..64)."""
    return bytes([((length - 1) << 2) | 3]) + offset.to_bytes(4, "little")


@pytest.mark.parametrize("fork", ["0", "1", "1c"])
def test_large_message_segments(gpu, oracle, fork, fsg_opts):
    """Large bodies run in pass 2 as 64 KiB output segments when no tag spans
    a segment boundary and no copy reaches below its segment (every stream the
    reference encoder writes); otherwise whole.  Raw sizes around the
    boundaries, a tail of < 4 bytes (joins the previous segment), and
    hand-built streams that must run whole; on one stream and forked ("1c":
    the huge bodies through the chunked pass 1b, huge hand-built streams that
    must run whole included)."""
    fsg_opts(decode_fork=fork[0])
    fsg_opts(chunked_huge="1" if fork == "1c" else "0")
    rng = np.random.default_rng(5)
    items = []
    for n in (65537, 131072, 131073, 131074, 131075, 131076, 196609, 300000, 1 << 20):
        items.append(fsg.make_batch(fsg.KIND_TEXT, [n], first_index=n).item(0))
    comps = [oracle.compress(x) for x in items]
    lit = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    # a copy at output 70000 reading 60000 (below its segment)
    comps.append(_varint(len(lit) + 64) + _literal(lit) + _copy2(64, 10000))
    # a copy spanning output 65536
    lit2 = lit[:65500]
    comps.append(_varint(65500 + 64 * 20) + _literal(lit2) + _copy2(64, 30000) * 20)
    # segmentable hand-built stream: literal to the boundary, then copies inside segment 1
    comps.append(_varint(65536 + 1000 + 640) + _literal(lit[:65536]) + _literal(lit[:1000])
                 + _copy2(64, 1000) * 10)
    comps += [oracle.compress(fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0))
              for s in (100, 5000, 20000)]
    if fork == "1c":
        big = rng.integers(0, 256, 400000, dtype=np.uint8).tobytes()
        # huge (> 256 KiB compressed): a copy at output 400000 reaching below its segment
        comps.append(_varint(len(big) + 64) + _literal(big) + _copy4(64, 70000))
        # huge, copies spanning 64 KiB boundaries after a long literal
        comps.append(_varint(300000 + 64 * 4000) + _literal(big[:300000]) + _copy2(64, 30000) * 4000)
        # huge text of 2 MiB and 3 MiB (segmentable)
        comps += [oracle.compress(fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0)) for s in (2 << 20, 3 << 20)]
    outs, ol, st = gpu.decompress(comps, [1 << 22] * len(comps))
    for i, (c, o, s) in enumerate(zip(comps, outs, st)):
        ok, ulen, ref = oracle.uncompress(c, cap=1 << 22)
        assert ok, i
        assert s == fsg.FSG_OK and o[:ulen] == ref, (i, s)


@pytest.mark.parametrize("variant,rule", [(5, "tags"), (4, "pieces")])
def test_far_copies_at_window_edge(gpu, oracle, variant, rule):
    """Copies whose sources lie a few bytes either side of pass 2's window base
    (tests/window_edge.py replays the kernel's group/window rules to place
    them, per execution pass: one tag per lane, or <= 16-byte pieces): far
    copies read back output stored to global memory in earlier groups,
    including 16-byte loads straddling the base, right after window slides
    and long-literal restarts.  Decoded bytes equal the construction's and
    the oracle's, messages side by side in 16-byte-aligned slots."""
    from window_edge import edge_stream
    rng = np.random.default_rng(31)
    comps, raws, n_edge = [], [], 0
    for i in range(800):
        c, raw, e = edge_stream(rng, int(rng.integers(2000, 40000)), rule=rule)
        comps.append(c); raws.append(raw); n_edge += e
    assert n_edge > 5000
    gpu.codec.select_kernels(variant, 0)
    try:
        outs, ol, st = gpu.decompress(comps, [len(r) for r in raws])
    finally:
        gpu.codec.select_kernels(0, 0)
    for i, (c, raw, o, s) in enumerate(zip(comps, raws, outs, st)):
        assert s == fsg.FSG_OK and o == raw, i
    for i in range(0, 800, 97):
        ok, ulen, ref = oracle.uncompress(comps[i], cap=len(raws[i]))
        assert ok and ref == raws[i], i


def test_mutations_and_trailing_tags(gpu, oracle):
    """Text bodies of 3-60 KB (compressed 1.5-30 KB, the lane index pass),
    with an incompressible block placed near the middle (a long literal),
    intact and with 1-3 mutated bytes anywhere, plus tags after the output is
    complete: a zero-length literal (fc ff ff ff ff) is accepted by the
    reference, any other tag rejected (writer space, snappy.cc:1166/:1400)."""
    rng = np.random.default_rng(17)
    comps = []
    for n in (3000, 4500, 8000, 20000, 60000):
        text = fsg.make_batch(fsg.KIND_TEXT, [n], first_index=n).item(0)
        base = oracle.compress(text)
        comps.append(base)
        for frac in (0.35, 0.45, 0.5, 0.55):
            blk = rng.integers(0, 256, int(rng.choice([100, 300, 1500])), dtype=np.uint8).tobytes()
            at = int(len(text) * frac)
            comps.append(oracle.compress(text[:at] + blk + text[at:]))
        for _ in range(60):
            c = bytearray(base)
            for _ in range(int(rng.integers(1, 4))):
                c[int(rng.integers(len(c)))] = int(rng.integers(256))
            comps.append(bytes(c))
        comps.append(base + b"\xfc\xff\xff\xff\xff")
        comps.append(base + b"\xfc\xff\xff\xff\xff" + b"\xfc\xff\xff\xff\xff")
        comps.append(base + b"\x00A")
        comps.append(base + b"\x05\x01")  # COPY_1 len 5 offset 1
        comps.append(base + b"\xfc\xff\xff\xff\xff\x00A")
    outs, ol, st = gpu.decompress(comps, [1 << 17] * len(comps))
    n_ok = n_bad = 0
    for i, (c, o, s) in enumerate(zip(comps, outs, st)):
        ok, ulen, ref = oracle.uncompress(c, cap=1 << 17)
        if ok is None:
            assert s == fsg.FSG_SLOT_TOO_SMALL, i
        elif not ok:
            n_bad += 1
            assert s in (fsg.FSG_CORRUPT, fsg.FSG_BAD_HEADER), (i, len(c), s)
        else:
            n_ok += 1
            assert s == fsg.FSG_OK and o[:ulen] == ref, (i, len(c), s)
    assert n_ok > 40 and n_bad > 40


@pytest.mark.parametrize("keep", ["512", "768", "1024", "2000"])
def test_window_slide_flush_rule(gpu, oracle, keep, fsg_opts):
    """A window slide must leave every byte a far piece can read in global
    memory: the piece's source lies below the new base but its 16-byte load
    reaches up to 15 bytes above it, so the slide flushes (and waits) when
    the flush lag leaves fewer than 16 stored bytes at the base.  1024 is the
    shipped default (FSG_KEEP, 3 KiB window) and 2000 the largest history the
    window allows (kMaxKeep); a smaller history (FSG_EXEC_KEEP) makes the
    short-lag slide frequent.  Before the rule covered the 16
    bytes, 512 B decoded a zero at offset 343,000 of the 1 MiB golden text.
    Golden vectors (up to 1 MiB, segmented and whole), window-edge streams
    and a C3-like batch, byte-equal to the inputs."""
    fsg_opts(exec_keep=keep)
    vecs = json.loads((GOLDEN / "vectors.json").read_text())
    datas = [build_input(v) for v in vecs]
    comps = [oracle.compress(d) for d in datas]
    from window_edge import edge_stream
    rng = np.random.default_rng(41)
    for _ in range(200):
        c, raw, _e = edge_stream(rng, int(rng.integers(2000, 40000)))
        comps.append(c)
        datas.append(raw)
    b = fsg.make_batch(fsg.KIND_TEXT, np.full(256, 65536, np.uint32), first_index=777)
    for i in range(256):
        datas.append(b.item(i))
        comps.append(oracle.compress(b.item(i)))
    outs, ol, st = gpu.decompress(comps, [len(d) for d in datas])
    for i, (d, o, s) in enumerate(zip(datas, outs, st)):
        assert s == fsg.FSG_OK and o == d, i


def test_two_stream_decode_stream_of_batches(gpu, oracle):
    """fsg_decompress_batch_2s: pass 1 on a second stream, pass 2 on the
    caller's, over a stream of distinct batches alternating two buffer sets
    (batch k+1's tag walk beside batch k's execution; a set is reused only
    after its previous execution, by an event).  Every batch's bytes and
    statuses equal the oracle's: small and large bodies (the segment path),
    random bodies and corrupt ones."""
    import torch
    from gpu_harness import dev
    rng = np.random.default_rng(77)
    batches = []
    for k in range(6):
        srcs = [fsg.make_batch(fsg.KIND_TEXT, [int(s)], first_index=1000 * k + j).item(0)
                for j, s in enumerate(rng.integers(1, 70000, 40))]
        srcs.append(fsg.make_batch(fsg.KIND_TEXT, [200000 + k], first_index=k).item(0))
        srcs.append(fsg.make_batch(fsg.KIND_RANDOM, [5000], first_index=k).item(0))
        comps = [oracle.compress(s) for s in srcs]
        bad = bytearray(comps[3])
        bad[len(bad) // 2] ^= 0x77
        comps.append(bytes(bad))
        batches.append(comps)
    codec = gpu.codec
    s_main = torch.cuda.current_stream()
    s1 = torch.cuda.Stream()
    sets = []
    for k, comps in enumerate(batches):
        b = fsg.Batch.from_list(comps)
        caps = np.full(len(b), 1 << 18, dtype=np.uint32)
        oo, tot = fsg.slot_offsets(caps.astype(np.uint64))
        sets.append(dict(n=len(b), d_in=dev(b.data), d_io=dev(b.offsets), d_il=dev(b.lens), oo=oo, d_oo=dev(oo),
                         d_cap=dev(caps), caps=caps))
    slot_bufs = []
    for _ in range(2):
        n = max(s["n"] for s in sets)
        slot_bufs.append(dict(out=torch.full((n << 18,), 0xA5, dtype=torch.uint8, device="cuda"),
                              ol=torch.zeros(n, dtype=torch.int32, device="cuda"),
                              st=torch.full((n,), -7, dtype=torch.int32, device="cuda"),
                              ws=codec.decompress_workspace(n, max(int(s["d_in"].numel()) for s in sets)),
                              done=None))
    torch.cuda.synchronize()
    results = []

    def collect(k):
        sl = slot_bufs[k % 2]
        s = sets[k]
        torch.cuda.synchronize()
        out = sl["out"].cpu().numpy()
        ol = sl["ol"].cpu().numpy()[:s["n"]].view(np.uint32)
        st = sl["st"].cpu().numpy()[:s["n"]]
        results.append((k, [out[int(s["oo"][i]):int(s["oo"][i]) + int(min(ol[i], s["caps"][i]))].tobytes()
                            for i in range(s["n"])], st.copy()))

    for k, s in enumerate(sets):
        sl = slot_bufs[k % 2]
        if sl["done"] is not None:
            collect(k - 2)  # (also orders: the set is free again)
            s1.wait_event(sl["done"])
        codec.decompress(s["d_in"], s["d_io"], s["d_il"], s["n"], sl["out"], s["d_oo"], s["d_cap"], sl["ol"],
                         sl["st"], stream=s_main, workspace=sl["ws"], pass1_stream=s1)
        ev = torch.cuda.Event()
        ev.record(s_main)
        sl["done"] = ev
    collect(len(sets) - 2)
    collect(len(sets) - 1)
    assert sorted(r[0] for r in results) == list(range(len(sets)))
    for k, outs, st in results:
        for i, c in enumerate(batches[k]):
            ok, ulen, ref = oracle.uncompress(c, cap=1 << 18)
            assert (st[i] == fsg.FSG_OK) == bool(ok), (k, i, st[i])
            if ok:
                assert outs[i][:ulen] == ref, (k, i)


@pytest.mark.parametrize("fork", ["0", "1", "1p", "1d"])
@pytest.mark.parametrize("fill", [0xFF, 0x5A])
def test_decode_with_garbage_workspace(gpu, oracle, fork, fill, fsg_opts):
    """The launch zeroes only the workspace's counters and lists: the index
    passes must store every bitmap word the execution pass reads (zero words,
    the words a long literal jumps over, the tail up to the allocation;
    pass 1b its whole message).  Decode with the workspace filled with
    garbage: text of many sizes, long literals inside text, single-literal
    and large (pass 1b) bodies, a 1 MiB text body (compressed > 256 KiB: the
    forked path's chunked huge-body walk, whose record region sits at the
    workspace's end and is never zeroed), intact and corrupted, against the
    oracle.  "1d": the forked path at the shipped small_persist default."""
    fsg_opts(decode_fork=fork[0])
    if fork != "1d":
        fsg_opts(small_persist="3" if fork == "1p" else "1792")
    rng = np.random.default_rng(fill)
    srcs = [fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0)
            for s in (1, 33, 200, 1000, 4096, 9000, 65536, 70000, 200000, 1 << 20)]
    srcs += [fsg.make_batch(fsg.KIND_RANDOM, [s], first_index=s).item(0) for s in (100, 5000, 65536, 600000)]
    # text with random runs inside: long literals between copies
    for k in range(4):
        t = bytearray(fsg.make_batch(fsg.KIND_TEXT, [30000], first_index=50 + k).item(0))
        r = fsg.make_batch(fsg.KIND_RANDOM, [2000 + 3000 * k], first_index=60 + k).item(0)
        pos = int(rng.integers(0, len(t)))
        srcs.append(bytes(t[:pos]) + r + bytes(t[pos:]))
    comps, caps = [], []
    for i in range(240):
        c = bytearray(oracle.compress(srcs[i % len(srcs)]))
        if i % 5 == 4:
            c[int(rng.integers(len(c)))] ^= 0x41
        comps.append(bytes(c))
        caps.append(max(1 << 19, len(srcs[i % len(srcs)])))
    assert max(len(c) for c in comps) > 256 * 1024
    outs, ol, st = gpu.decompress(comps, caps, ws_fill=fill)
    for i, (c, o, s) in enumerate(zip(comps, outs, st)):
        ok, ulen, ref = oracle.uncompress(c, cap=caps[i])
        if ok is None:
            assert s == fsg.FSG_SLOT_TOO_SMALL, i
        elif not ok:
            assert s in (fsg.FSG_CORRUPT, fsg.FSG_BAD_HEADER), i
        else:
            assert s == fsg.FSG_OK and o[:ulen] == ref, i


@pytest.mark.parametrize("wave_min,all_mb", [("1", "640"), ("16384", "640"), ("4096", "0")])
def test_wave_encoder_against_oracle(gpu, oracle, wave_min, all_mb, fsg_opts):
    """The wave encoder (hash table in LDS, one wave per fragment:
    csrc/snappy_encode_wave.hip) takes every fragment of a split message and
    the messages of >= FSG_ENCODE_WAVE_MIN bytes, the lane encoder the rest.
    Bytes equal the oracle's on the golden inputs, random alphabets (runs,
    long matches, incompressible stretches), text with random stretches,
    periodic data, split messages (incl. capped staging regions, which force
    the whole-message fallback) and messages of every size class.
    FSG_ENCODE_WAVE_ALL_MB=0 gives the lanes their share of the long units
    too (the split the encoder uses for batches of more than 640 MB of them)."""
    fsg_opts(encode_wave_min=wave_min)
    fsg_opts(encode_wave_all_mb=all_mb)
    vecs = json.loads((GOLDEN / "vectors.json").read_text())
    items = [build_input(v) for v in vecs]
    rng = np.random.default_rng(int(wave_min) + 11)
    for t in range(300):
        n = int(rng.choice([rng.integers(0, 100), rng.integers(0, 5000), rng.integers(0, 140000)]))
        alpha = int(rng.choice([2, 3, 8, 40, 256]))
        items.append(rng.integers(0, alpha, n, dtype=np.uint8).tobytes())
    for per in range(1, 70, 5):
        items.append(bytes(((np.arange(20000 + 37 * per) % per) * 7 + 1).astype(np.uint8)))
    for k in range(8):
        t = bytearray(fsg.make_batch(fsg.KIND_TEXT, [40000], first_index=900 + k).item(0))
        r = fsg.make_batch(fsg.KIND_RANDOM, [500 + 2000 * k], first_index=950 + k).item(0)
        pos = int(rng.integers(0, len(t)))
        items.append(bytes(t[:pos]) + r + bytes(t[pos:]))
    for i, n in enumerate([65535, 65536, 65537, 131073, 200000, 1 << 20, 70000]):
        kind = fsg.KIND_RANDOM if i % 3 == 1 else fsg.KIND_TEXT
        items.append(fsg.make_batch(kind, [n], first_index=300 + i).item(0))
    items.append(bytes(70000))  # one long run: matches far past the 20 preloaded bytes
    comps, st = gpu.compress(fsg.Batch.from_list(items))
    assert (st == 0).all()
    for i, (x, c) in enumerate(zip(items, comps)):
        assert c == oracle.compress(x), (i, len(x))
    for cap in (4096, 40000):  # split fragments overflowing their regions
        gpu.codec.set_split_region_cap(cap)
        try:
            big = [fsg.make_batch(fsg.KIND_RANDOM, [200000], first_index=7).item(0),
                   fsg.make_batch(fsg.KIND_TEXT, [300001], first_index=8).item(0)]
            comps, st = gpu.compress(fsg.Batch.from_list(big))
        finally:
            gpu.codec.set_split_region_cap(0)
        assert (st == 0).all()
        assert all(c == oracle.compress(x) for x, c in zip(big, comps))


def test_small_batch_wave_encoder(gpu, oracle):
    """Batches of <= 64 messages put every message of >= 15 bytes on the wave
    encoder (snappy_encode_v3.hip kSmallBatchEnc).  Batches of 1, 7 and 64
    messages over golden inputs, random alphabets, periodic data, long runs,
    split messages and the input-margin edge sizes: bytes equal the
    oracle's."""
    vecs = json.loads((GOLDEN / "vectors.json").read_text())
    items = [build_input(v) for v in vecs]
    rng = np.random.default_rng(77)
    for n in (14, 15, 16, 17, 31, 63, 64, 65, 127, 4095, 4096, 65535, 65536, 65537):
        items.append(fsg.make_batch(fsg.KIND_TEXT, [n], first_index=n).item(0))
    for t in range(60):
        n = int(rng.choice([rng.integers(0, 5000), rng.integers(0, 140000)]))
        alpha = int(rng.choice([2, 3, 8, 40, 256]))
        items.append(rng.integers(0, alpha, n, dtype=np.uint8).tobytes())
    for per in (1, 3, 17, 61):
        items.append(bytes(((np.arange(30000 + per) % per) * 7 + 1).astype(np.uint8)))
    items.append(bytes(70000))
    items.append(fsg.make_batch(fsg.KIND_TEXT, [200000], first_index=5).item(0))
    for size in (1, 7, 64):
        for b0 in range(0, len(items), size if size > 1 else 9):
            part = items[b0:b0 + size]
            comps, st = gpu.compress(fsg.Batch.from_list(part))
            assert (st == 0).all()
            for i, (x, c) in enumerate(zip(part, comps)):
                assert c == oracle.compress(x), (size, b0 + i, len(x))


@pytest.mark.parametrize("name", ["C3", "C5"])
def test_wave_encoder_config_digests(gpu, name, fsg_opts):
    """Config digests (reference-generated) with the wave encoder on every
    message of >= 16 KiB and every split fragment."""
    fsg_opts(encode_wave_min="16384")
    d = np.load(GOLDEN / f"digests_{name}.npz")
    n = len(d["input_len"])
    kind = {"C3": fsg.KIND_TEXT, "C5": fsg.KIND_PROTO}[name]
    sizes = {"C3": np.full(n, 65536), "C5": fsg.mixed_sizes(n)}[name]
    b = fsg.make_batch(kind, sizes)
    comps, st = gpu.compress(b)
    assert (st == 0).all()
    assert np.array_equal(np.array([len(c) for c in comps], np.uint32), d["compressed_len"])
    assert np.array_equal(np.array([fsg.fnv1a64(c) for c in comps], np.uint64), d["compressed_fnv"])
