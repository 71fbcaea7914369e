"""GPU parity of the LZ4 path (flare-cpp_amd/csrc/lz4.hip, lz4_decode2.hip)
through the C ABI (include/flare_lz4_gpu.h): bodies byte-equal to the oracle
and to the liblz4 fixtures, every decode verdict and byte equal to the
oracle's -- for the one-pass lane decoder (fsg_lz4_decompress_batch) and the
two-pass decoder (fsg_lz4_decompress_batch_ws)."""
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


# FSG_L4_BIG_MIN per index-pass variant: the lane walk for every block, the
# wave walk (lz4_index_big_kernel) for every block of more than 64 bytes
_WALK_MIN = {"lane_walk": "4294967295", "wave_walk": "64"}


@pytest.fixture(params=["one_pass", "two_pass", "two_pass_lane_walk", "two_pass_wave_walk"])
def two(request, fsg_opts):
    """one_pass: lz4.hip's lane kernel; two_pass: lz4_decode2.hip at its
    default thresholds (the wave walk for blocks over 64 KiB, over 2 KiB in
    batches of <= 256 messages); _lane_walk / _wave_walk force one index
    pass for every block."""
    for k, v in _WALK_MIN.items():
        if request.param.endswith(k):
            fsg_opts(lz4_big_min=v)
    return request.param != "one_pass"


@pytest.fixture(params=["lane_walk", "wave_walk"])
def walk(request, fsg_opts):
    """The index pass of the two-pass decoder forced for every block: the
    lane walk, or (blocks of more than 64 bytes) the wave walk."""
    fsg_opts(lz4_big_min=_WALK_MIN[request.param])
    return request.param


def test_lz4_compress_matches_liblz4_fixtures(gpu, o, two):
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
    outs, ol, st = gpu.lz4_decompress(bodies, [len(x) for x in xs], two_pass=two)
    assert (st == fsg.FSG_OK).all()
    assert all(y == x for y, x in zip(outs, xs))


def test_lz4_randomized_against_oracle(gpu, o, two):
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
    outs, ol, st = gpu.lz4_decompress(bodies, [len(x) for x in xs], two_pass=two)
    assert (st == 0).all() and all(y == x for y, x in zip(outs, xs))


def test_lz4_decode_verdicts_against_oracle(gpu, o, two):
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
    outs, ol, st = gpu.lz4_decompress(bodies, [cap] * len(bodies), two_pass=two)
    for i, (b, y, l, s) in enumerate(zip(bodies, outs, ol, st)):
        r, ulen, ref = o.uncompress(b, cap=cap)
        want = {1: fsg.FSG_OK, 0: fsg.FSG_CORRUPT, -1: fsg.FSG_BAD_HEADER, -2: fsg.FSG_SLOT_TOO_SMALL}[r]
        assert s == want, (i, r, s)
        if r == 1:
            assert y == ref, i
    for d, s in zip(cases, st[:len(cases)]):
        if not d["offset0"]:
            assert (s == fsg.FSG_OK) == d["liblz4_ok"]


def test_lz4_empty_and_edges(gpu, o, two):
    xs = [b"", b"x", b"a" * 12, b"a" * 13, bytes(65547)]
    bodies, st = gpu.lz4_compress(fsg.Batch.from_list(xs))
    assert (st == 0).all() and bodies[0] == b"\x00\x00"
    outs, ol, st = gpu.lz4_decompress(bodies + [b"", b"\x05\x50hello"], [len(x) for x in xs] + [0, 4],
                                      two_pass=two)
    assert list(st) == [0] * 5 + [fsg.FSG_BAD_HEADER, fsg.FSG_SLOT_TOO_SMALL]
    assert outs[:5] == xs


def _kinds(rng, n):
    """Bodies of every kind the bench and the RPC path see, 0 B .. 2 MiB."""
    out = []
    for i in range(n):
        k = i % 6
        size = int(rng.choice([0, 1, 13, 200, 4096, 65536, 65547, 100000, 300000, 1 << 21]))
        if k == 0:
            x = fsg.make_batch(fsg.KIND_TEXT, [size], first_index=i).item(0) if size else b""
        elif k == 1:
            x = rng.integers(0, 256, size, dtype=np.uint8).tobytes()
        elif k == 2:
            x = bytes(size)
        elif k == 3:
            x = (bytes(rng.integers(0, 256, int(rng.integers(1, 40)), dtype=np.uint8)) * (size // 2 + 1))[:size]
        elif k == 4:
            x = rng.integers(0, 3, size, dtype=np.uint8).tobytes()
        else:
            x = fsg.make_batch(fsg.KIND_PROTO, [size], first_index=i).item(0) if size else b""
        out.append(x)
    return out


def test_lz4_two_pass_kinds_against_oracle(gpu, o, walk):
    """Compressor output of every kind and size (long literals of random
    bodies, long runs of zeros, short periods, text, JSON) through the
    two-pass decoder: bytes equal to the inputs, statuses OK."""
    rng = np.random.default_rng(31)
    xs = _kinds(rng, 60)
    bodies = [o.compress(x) for x in xs]
    outs, ol, st = gpu.lz4_decompress(bodies, [len(x) for x in xs])
    assert (st == 0).all()
    for i, (y, x) in enumerate(zip(outs, xs)):
        assert y == x, (i, len(x))


def test_lz4_two_pass_synthetic_sequences(gpu, o, walk):
    """Blocks built sequence by sequence (tests/lz4_blocks.py): every
    extension-byte boundary of both lengths, 255 runs, empty literals,
    offsets 1..15 / 16..1536 / above, matches longer than their offset and
    tens of KiB long -- the whole-wave path of the execution pass."""
    from lz4_blocks import random_block
    rng = np.random.default_rng(41)
    bodies, wants = [], []
    for t in range(120):
        b, w = random_block(rng, int(rng.choice([50, 3000, 40000, 200000])))
        bodies.append(b)
        wants.append(w)
    outs, ol, st = gpu.lz4_decompress(bodies, [len(w) for w in wants])
    for i, (b, y, w, s) in enumerate(zip(bodies, outs, wants, st)):
        assert s == 0 and y == w, i


def test_lz4_two_pass_workspace_garbage_and_fallback(gpu, o, walk):
    """The workspace may hold anything (filled with 0xff first), and one
    sized for less input than the batch sends the messages whose bitmap does
    not fit to the one-pass kernel: the same bytes and statuses either way."""
    rng = np.random.default_rng(7)
    xs = _kinds(rng, 36)
    bodies = [o.compress(x) for x in xs]
    bodies[3] = bodies[3][:-1] if len(bodies[3]) > 2 else bodies[3]  # a truncated one among them
    caps = [len(x) for x in xs]
    ref = [o.uncompress(b, cap=c) for b, c in zip(bodies, caps)]
    want_st = [{1: 0, 0: fsg.FSG_CORRUPT, -1: fsg.FSG_BAD_HEADER, -2: fsg.FSG_SLOT_TOO_SMALL}[r] for r, _, _ in ref]
    for kw in ({"ws_fill": 0xFF}, {"ws_total_in": sum(map(len, bodies)) // 3, "ws_fill": 0x5A}):
        outs, ol, st = gpu.lz4_decompress(bodies, caps, **kw)
        assert list(st) == want_st, kw
        for (r, _, y0), y in zip(ref, outs):
            if r == 1:
                assert y == y0, kw


def test_lz4_two_pass_c3_like_batch(gpu, o):
    """A few hundred 64 KiB text bodies (the bench's C3 shape): the index
    pass's wave-wide bitmap allocation and the execution pass's one wave per
    message, bytes against the inputs."""
    b = fsg.make_batch(fsg.KIND_TEXT, np.full(300, 65536, np.uint32))
    xs = [b.item(i) for i in range(len(b))]
    bodies = [o.compress(x) for x in xs]
    outs, ol, st = gpu.lz4_decompress(bodies, [len(x) for x in xs])
    assert (st == 0).all() and all(y == x for y, x in zip(outs, xs))


def test_lz4_two_stream_form(gpu, o, walk):
    """fsg_lz4_decompress_batch_2s: two batches with their own buffers,
    decoded alternately four times, each batch's index pass on a second
    stream beside the other's execution (the slot's previous execution
    waited for by event, as bench.py's time_pipelined does): the verdicts and
    bytes of the oracle every time, a corrupt body and a slot too small among
    them."""
    import torch
    from gpu_harness import POISON
    rng = np.random.default_rng(57)
    dev = torch.device("cuda", 0)
    H = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    slots = []
    for t in range(2):
        xs = _kinds(rng, 30)
        bodies = [o.compress(x) for x in xs]
        bodies[5] = bodies[5][:-1] if len(bodies[5]) > 2 else bodies[5]
        caps = [len(x) for x in xs]
        caps[7] = max(caps[7] - 1, 0)
        ref = [o.uncompress(b, cap=c) for b, c in zip(bodies, caps)]
        b = fsg.Batch.from_list(bodies)
        n = len(b)
        capa = np.array(caps, dtype=np.uint32)
        oo, tot = fsg.slot_offsets(capa.astype(np.uint64))
        slots.append(dict(n=n, ref=ref, oo=oo, caps=capa, d_in=H(b.data), d_io=H(b.offsets), d_il=H(b.lens),
                          d_oo=H(oo), d_cap=H(capa),
                          d_out=torch.full((max(tot, 1),), POISON, dtype=torch.uint8, device=dev),
                          d_ol=torch.zeros(n, dtype=torch.int32, device=dev),
                          d_st=torch.full((n,), -7, dtype=torch.int32, device=dev),
                          ws=gpu.codec.lz4_decompress_workspace(n, int(b.data.size))))
    s = torch.cuda.current_stream(dev)
    s1 = torch.cuda.Stream(dev)
    done = [None, None]
    for k in range(8):
        sl = slots[k % 2]
        if done[k % 2] is not None:
            s1.wait_event(done[k % 2])
        gpu.codec.lz4_decompress(sl["d_in"], sl["d_io"], sl["d_il"], sl["n"], sl["d_out"], sl["d_oo"], sl["d_cap"],
                                 sl["d_ol"], sl["d_st"], stream=s, workspace=sl["ws"], pass1_stream=s1)
        ev = torch.cuda.Event()
        ev.record(s)
        done[k % 2] = ev
    torch.cuda.synchronize()
    code = {1: 0, 0: fsg.FSG_CORRUPT, -1: fsg.FSG_BAD_HEADER, -2: fsg.FSG_SLOT_TOO_SMALL}
    for sl in slots:
        st = sl["d_st"].cpu().numpy()
        out = sl["d_out"].cpu().numpy()
        for i, (r, _, y0) in enumerate(sl["ref"]):
            assert st[i] == code[r], i
            if r == 1:
                a = int(sl["oo"][i])
                assert out[a:a + len(y0)].tobytes() == y0, i
