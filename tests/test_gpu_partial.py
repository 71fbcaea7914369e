"""GPU parity for the two decode entry points beside Uncompress, through the C
ABI (csrc/snappy_decode_partial.hip):

* fsg_decompress_batch_partial = UncompressAsMuchAsPossible
  (snappy.cc:1530-1535): the return value and the bytes the sink receives,
  against the reference-made negative.json fixtures (8160-byte source pieces)
  and against the oracle's restatement (oracle/snappy_oracle.c, pinned to the
  reference build in tests/test_oracle.py) on mutated streams, for several
  source piece sizes;
* fsg_decompress_batch_iovec = RawUncompressToIOVec (snappy.cc:1122-1132):
  the verdict and the iovecs' bytes against the oracle, on mutated streams and
  random iovec lists (empty, exact, short and roomy ones).  The iovecs' bytes
  are compared after a `false` verdict too: the decoded prefix the reference
  leaves in place, a literal cut by the end of input, the spill of its last
  16-byte fast append (SnappyIOVecWriter, snappy.cc:963-1120)."""
import json
from pathlib import Path

import numpy as np
import pytest

import fsg
from bind import Oracle

GOLDEN = Path(__file__).resolve().parent / "golden"
POISON = 0xA5
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def codec():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test run without a visible GPU")
    return fsg.SnappyGPU(torch.cuda.current_device())


@pytest.fixture(scope="module")
def oracle():
    return Oracle()


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _partial(codec, comps, caps, frag):
    """(produced, got bytes per message, status) from the device."""
    import torch
    b = fsg.Batch.from_list(comps)
    n = len(b)
    caps = np.array(caps, dtype=np.uint32)
    oo, tot = fsg.slot_offsets(caps.astype(np.uint64))
    d_out = torch.full((max(tot, 1),), POISON, dtype=torch.uint8, device="cuda")
    d_got = torch.zeros(max(n, 1), dtype=torch.int32, device="cuda")
    d_prod = torch.zeros(max(n, 1), dtype=torch.int64, device="cuda")
    d_st = torch.full((max(n, 1),), -7, dtype=torch.int32, device="cuda")
    ws = codec.decompress_workspace(n, int(b.data.size))
    codec.decompress_partial(_dev(b.data), _dev(b.offsets), _dev(b.lens), n, frag, d_out, _dev(oo), _dev(caps),
                             d_got, d_prod, d_st, workspace=ws)
    torch.cuda.synchronize()
    out = d_out.cpu().numpy()
    got = d_got.cpu().numpy()[:n].view(np.uint32)
    prod = d_prod.cpu().numpy()[:n]
    st = d_st.cpu().numpy()[:n]
    return prod, [out[int(oo[i]):int(oo[i]) + int(min(got[i], caps[i]))].tobytes() for i in range(n)], st


def _mutants(oracle, rng, count, sizes=(40, 900, 9000, 70000, 140000)):
    srcs = [fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0) for s in sizes]
    out = []
    for _ in range(count):
        c = bytearray(oracle.compress(srcs[int(rng.integers(len(srcs)))]))
        for _ in range(int(rng.integers(0, 4))):
            c[int(rng.integers(len(c)))] = int(rng.integers(256))
        if rng.random() < 0.3:
            c = c[: int(rng.integers(1, len(c) + 1))]
        out.append(bytes(c))
    return out


def test_as_much_golden(codec):
    """negative.json: the reference's own UncompressAsMuchAsPossible results
    (8160-byte pieces), including its double-counted block."""
    negs = [v for v in json.loads((GOLDEN / "negative.json").read_text()) if v["ok"] is not None and v["header_ok"]]
    comps = [bytes.fromhex(v["hex"]) for v in negs]
    prod, got, st = _partial(codec, comps, [max(v["ulen"], 1) for v in negs], 8160)
    quirk = 0
    for v, p, g, s in zip(negs, prod, got, st):
        assert p == v["partial_ret"], v["name"]
        assert len(g) == v["partial_len"], v["name"]
        assert "%016x" % fsg.fnv1a64(g) == v["partial_fnv"], v["name"]
        assert (s == fsg.FSG_OK) == bool(v["ok"]), v["name"]
        quirk += p != len(g)
    assert quirk > 0


@pytest.mark.parametrize("frag", [1, 3, 7])
def test_as_much_small_pieces_golden(codec, oracle, frag):
    """The reference's own UncompressAsMuchAsPossible results at 1-, 3- and
    7-byte source pieces, long-literal tags straddling a piece boundary
    (tests/golden/partial_frag.json; snappy.cc:790-847)."""
    cases = [v for v in json.loads((GOLDEN / "partial_frag.json").read_text()) if v["frag"] == frag]
    comps = [bytes.fromhex(v["hex"]) for v in cases]
    prod, got, st = _partial(codec, comps, [max(v["ulen"], 1) for v in cases], frag)
    for i, v in enumerate(cases):
        key = (v["nbytes"], v["before"], v["kind"])
        assert prod[i] == v["ret"], key
        assert len(got[i]) == v["got_len"] and "%016x" % fsg.fnv1a64(got[i]) == v["got_fnv"], key
        assert (st[i] == fsg.FSG_OK) == bool(oracle.uncompress(comps[i], cap=1 << 19)[0]), key


@pytest.mark.parametrize("frag,fork", [(0, 0), (7, 0), (8160, 0), (8160, 1)])
def test_as_much_fuzz_against_oracle(codec, oracle, frag, fork, fsg_opts):
    """fork 1: the batch decoder under it takes the path of batches over 128K
    messages (plan pass, side streams), forced on this batch."""
    fsg_opts(decode_fork=fork)
    rng = np.random.default_rng(31 + frag)
    comps = _mutants(oracle, rng, 1500)
    comps += [oracle.compress(fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0)) for s in (0, 1, 20, 65536)]
    caps = []
    for c in comps:
        h, ulen = oracle.header(c)
        # slots for the header length; some a little short (the device must
        # then either match a run that stops early or say SLOT_TOO_SMALL)
        cap = min(ulen, 1 << 18) if h else 16
        if h and rng.random() < 0.1 and cap > 8:
            cap -= int(rng.integers(1, 8))
        caps.append(max(cap, 1))
    prod, got, st = _partial(codec, comps, caps, frag)
    n_partial = n_small = 0
    for i, c in enumerate(comps):
        h, ulen = oracle.header(c)
        r, rgot = oracle.uncompress_as_much(c, 1 << 19, frag)
        if not h:
            assert st[i] == fsg.FSG_BAD_HEADER and prod[i] == 0 and got[i] == b"", i
            continue
        if len(rgot) > caps[i]:
            assert st[i] == fsg.FSG_SLOT_TOO_SMALL, i
            n_small += 1
            continue
        assert prod[i] == r, i
        assert got[i] == rgot, i
        full = oracle.uncompress(c, cap=1 << 19)[0]
        assert (st[i] == fsg.FSG_OK) == bool(full), i
        n_partial += r != ulen
    assert n_partial > 100


def _iov_lists(rng, total):
    k = int(rng.integers(1, 7))
    cuts = sorted(int(rng.integers(0, total + 1)) for _ in range(k - 1))
    lens = [b - a for a, b in zip([0] + cuts, cuts + [total])]
    r = rng.random()
    if r < 0.25:
        lens[-1] += int(rng.integers(1, 40))                         # room to spare
    elif r < 0.4 and total:
        j = int(rng.integers(len(lens)))
        lens[j] = max(0, lens[j] - int(rng.integers(1, 20)))          # too short
    if rng.random() < 0.3:
        lens.insert(int(rng.integers(len(lens) + 1)), 0)              # an empty iovec
    return lens


def _iovec(codec, comps, iov_lens):
    import torch
    b = fsg.Batch.from_list(comps)
    n = len(b)
    o = Oracle()
    ulens = [u if h else 0 for h, u in (o.header(c) for c in comps)]
    caps = np.array([max(min(u, 1 << 18), 1) for u in ulens], np.uint32)
    so, stot = fsg.slot_offsets(caps.astype(np.uint64))
    d_stage = torch.full((max(stot, 1),), POISON, dtype=torch.uint8, device="cuda")
    flat = [x for lens in iov_lens for x in lens]
    first = np.zeros(n + 1, np.uint32)
    first[1:] = np.cumsum([len(lens) for lens in iov_lens])
    ioff = np.zeros(len(flat) + 1, np.uint64)
    ioff[1:] = np.cumsum(np.array(flat, np.uint64) + 8)  # 8 guard bytes between iovecs
    d_iov = torch.full((int(ioff[-1]) + 1,), POISON, dtype=torch.uint8, device="cuda")
    base = np.array([d_iov.data_ptr() + int(o) for o in ioff[:-1]], np.uint64).view(np.int64)
    d_ol = torch.zeros(max(n, 1), dtype=torch.int32, device="cuda")
    d_st = torch.full((max(n, 1),), -7, dtype=torch.int32, device="cuda")
    ws = codec.decompress_workspace(n, int(b.data.size))
    codec.decompress_iovec(_dev(b.data), _dev(b.offsets), _dev(b.lens), n, _dev(base),
                           _dev(np.array(flat, np.uint64).view(np.int64)), _dev(first), d_stage, _dev(so),
                           _dev(caps), d_ol, d_st, workspace=ws)
    torch.cuda.synchronize()
    mem = d_iov.cpu().numpy()
    st = d_st.cpu().numpy()[:n]
    bufs, k = [], 0
    for lens in iov_lens:
        bufs.append([mem[int(ioff[k + j]):int(ioff[k + j]) + lens[j]].tobytes() for j in range(len(lens))])
        k += len(lens)
    guards = np.concatenate([mem[int(ioff[j + 1]) - 8:int(ioff[j + 1])] for j in range(len(flat))]) if flat else []
    return st, bufs, guards, caps, ulens


@pytest.mark.parametrize("fork", [0, 1])
def test_iovec_fuzz_against_oracle(codec, oracle, fork, fsg_opts):
    fsg_opts(decode_fork=fork)
    rng = np.random.default_rng(41 + fork)
    comps = _mutants(oracle, rng, 1200)
    comps += [oracle.compress(fsg.make_batch(fsg.KIND_TEXT, [s], first_index=s).item(0)) for s in (0, 1, 20, 65536)]
    hdr = [oracle.header(c) for c in comps]
    iov_lens = [_iov_lists(rng, min(u, 1 << 18) if h else 4) for h, u in hdr]
    st, bufs, guards, caps, ulens = _iovec(codec, comps, iov_lens)
    assert (np.asarray(guards) == POISON).all()  # nothing written between iovecs
    seen = {True: 0, False: 0}
    too_small = prefix = 0
    for i, c in enumerate(comps):
        h, ulen = hdr[i]
        if h and ulen > caps[i]:
            assert st[i] == fsg.FSG_SLOT_TOO_SMALL, i
            continue
        ok, rbufs = oracle.uncompress_iovec(c, iov_lens[i], fill=POISON)
        assert (st[i] == fsg.FSG_OK) == ok, (i, st[i])
        assert bufs[i] == rbufs, (i, ok, st[i])  # the bytes the reference leaves, after a `false` too
        if not ok:
            assert st[i] in (fsg.FSG_CORRUPT, fsg.FSG_BAD_HEADER, fsg.FSG_IOV_TOO_SMALL), i
            if h and oracle.uncompress(c)[0]:
                assert st[i] == fsg.FSG_IOV_TOO_SMALL, i
                too_small += 1
            elif any(x != bytes([POISON]) * len(x) for x in rbufs):
                prefix += 1
        seen[ok] += 1
    assert seen[True] > 100 and seen[False] > 100
    assert too_small > 20 and prefix > 100, (too_small, prefix)


def test_iovec_large_valid_batch(codec, oracle):
    """512 x 64 KiB text bodies, each split over three iovecs (one empty):
    the wave-per-message copy over whole 16-byte chunks and ragged tails."""
    rng = np.random.default_rng(5)
    b = fsg.make_batch(fsg.KIND_TEXT, np.full(512, 65536, np.uint32))
    comps = [oracle.compress(b.item(i)) for i in range(len(b))]
    iov_lens = []
    for _ in comps:
        a = int(rng.integers(0, 65537))
        iov_lens.append([a, 0, 65536 - a])
    st, bufs, guards, _, _ = _iovec(codec, comps, iov_lens)
    assert (st == fsg.FSG_OK).all()
    assert (np.asarray(guards) == POISON).all()
    for i in range(len(b)):
        assert b"".join(bufs[i]) == b.item(i), i
