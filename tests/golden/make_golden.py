"""Generate the committed golden vectors from the REFERENCE's own Snappy build.

Run in the dev container (where /root/reference exists and `make -C oracle`
built oracle/_ref/libsnappy_ref.so):

    python tests/golden/make_golden.py

Every expected output below is produced by the reference code
(flare/io/snappy/snappy.cc compiled in place), driven through a cord_buf-like
fragmenting Source (8160-byte fragments, flare/io/cord_buf.h:67) and a
copying Sink -- the same Source/Sink path policy::SnappyCompress /
SnappyDecompress take (flare/rpc/policy/snappy_compress.cc:28-61).  The
reference ships no golden vectors of its own; its test inputs
(test/rpc/rpc_snappy_compress_test.cc) are reproduced here as data.

Outputs (all data, no code):
  vectors.json   positive vectors: input spec (or hex) -> compressed hex /
                 (length, fnv1a64)
  negative.json  decode vectors: compressed hex -> reference verdict, header
                 length, strict-header verdict, validator verdict
  digests_*.npz  per-message (compressed_len, fnv1a64) for the first N
                 messages of the C2/C3/CM/C5 synthetic batches
  partial_frag.json  UncompressAsMuchAsPossible (snappy.cc:1530-1535) at
                 source pieces of 1, 3 and 7 bytes: long-literal tags (1-4
                 length bytes) placed to straddle a piece boundary (RefillTag's
                 stitching, :790-847), exact and short header lengths, cut and
                 corrupted tails -- the reference's return value and the bytes
                 its sink received (`--partial-only` regenerates it)
  full_*.npz     the BASELINE configs at FULL size:
                 per-message (input_fnv, compressed_len, compressed_fnv) of all
                 65,536 C2 and C3 bodies, and for CM's 1,048,576 bodies the
                 aggregate digests (fnv1a64 over the per-message fnv column,
                 sums of lengths) plus the compressed-length column; for C5's
                 262,144 SnappyMessageProto bodies the per-message
                 (compressed_len, compressed_fnv) columns and the input
                 aggregate.
                 `python tests/golden/make_golden.py --full-only` regenerates
                 just these (`--c5-only`: just full_C5.npz).
"""
from __future__ import annotations

import json
import random
import sys
from pathlib import Path

import numpy as np

HERE = Path(__file__).resolve().parent
REPO = HERE.parents[1]
sys.path.insert(0, str(REPO / "oracle"))
sys.path.insert(0, str(REPO / "flare-cpp_amd" / "py"))

from bind import Reference  # noqa: E402
import fsg  # noqa: E402
from gen_inputs import build_input, positive_specs, negative_cases  # noqa: E402


def aggregate(col: np.ndarray) -> int:
    """The checksum of checksums: fnv1a64 over a u64 digest column's bytes."""
    a = np.ascontiguousarray(col, np.uint64)
    return fsg.fnv1a64(a.tobytes())


def full_digests(ref, kind, sizes, chunk=8192, threads=8):
    """Reference compress of the whole batch (oracle/_ref, the handler's
    Source/Sink path, `threads` host threads) in chunks of `chunk` bodies:
    per-message input fnv, compressed length and compressed fnv."""
    n = len(sizes)
    in_fnv = np.zeros(n, np.uint64)
    clen = np.zeros(n, np.uint32)
    cfnv = np.zeros(n, np.uint64)
    for a in range(0, n, chunk):
        b = fsg.make_batch(kind, sizes[a:a + chunk], first_index=a)
        caps = np.array([fsg.max_compressed_length(int(x)) for x in b.lens], np.uint64)
        oo, tot = fsg.slot_offsets(caps)
        out = np.zeros(tot, np.uint8)
        ol = np.zeros(len(b), np.uint32)
        ref.batch(0, b.data, b.offsets, b.lens, out, oo, None, ol, threads=threads)
        in_fnv[a:a + len(b)] = fsg.digests(b.data, b.offsets, b.lens)
        clen[a:a + len(b)] = ol
        cfnv[a:a + len(b)] = fsg.digests(out, oo, ol)
    return in_fnv, clen, cfnv


def make_full_c5(ref):
    """C5 at full size: 262,144 SnappyMessageProto bodies (bench.py's
    c5-compress batch), every body's compressed (length, fnv)."""
    n = 262144
    sizes = fsg.mixed_sizes(n)
    in_fnv, clen, cfnv = full_digests(ref, fsg.KIND_PROTO, sizes, chunk=32768)
    b_total = int(sum(len(fsg.make_batch(fsg.KIND_PROTO, sizes[a:a + 32768], first_index=a).data)
                      for a in range(0, n, 32768)))
    np.savez_compressed(HERE / "full_C5.npz", compressed_len=clen, compressed_fnv=cfnv,
                        aggregate=np.array([aggregate(in_fnv), aggregate(cfnv)], np.uint64),
                        totals=np.array([b_total, int(clen.astype(np.uint64).sum())], np.uint64))
    print("C5 full:", n, "bodies,", b_total, "bytes, ratio %.3f" % (b_total / clen.sum()))


def make_full(ref):
    n = 65536
    for name, kind, size in (("C2", fsg.KIND_RANDOM, 4096), ("C3", fsg.KIND_TEXT, 65536)):
        in_fnv, clen, cfnv = full_digests(ref, kind, np.full(n, size, np.uint32))
        np.savez_compressed(HERE / f"full_{name}.npz", input_fnv=in_fnv, compressed_len=clen, compressed_fnv=cfnv,
                            aggregate=np.array([aggregate(in_fnv), aggregate(cfnv)], np.uint64))
        print(name, "full:", n, "bodies, ratio %.3f" % (n * size / clen.sum()))
    n = 1 << 20
    sizes = fsg.mixed_sizes(n)
    in_fnv, clen, cfnv = full_digests(ref, fsg.KIND_MIXED, sizes, chunk=65536)
    np.savez_compressed(HERE / "full_CM.npz", compressed_len=clen,
                        aggregate=np.array([aggregate(in_fnv), aggregate(cfnv)], np.uint64),
                        totals=np.array([int(sizes.astype(np.uint64).sum()), int(clen.astype(np.uint64).sum())],
                                        np.uint64))
    print("CM full:", n, "bodies,", int(sizes.astype(np.uint64).sum()), "bytes")
    make_full_c5(ref)


def _long_literal(data: bytes, nbytes: int) -> bytes:
    """LITERAL tag with `nbytes` (1-4) little-endian length bytes."""
    n = len(data) - 1
    return bytes([(59 + nbytes) << 2]) + n.to_bytes(nbytes, "little") + data


def _varint(v: int) -> bytes:
    out = bytearray()
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def make_partial_frag(ref):
    """Streams whose long-literal tag straddles a source-piece boundary at
    pieces of 1, 3 and 7 bytes, decoded by the reference's
    UncompressAsMuchAsPossible."""
    rng = random.Random(1234)
    cases = []
    for frag in (1, 3, 7):
        for nbytes in (1, 2, 3, 4):
            for before in range(1, 5):  # the tag starts `before` bytes ahead of a piece end
                for kind in ("exact", "short", "cut", "badcopy", "overrun"):
                    lit_len = rng.choice([61, 64, 100, 200, 256] if nbytes == 1 else [61, 64, 100, 300, 1000])
                    data = bytes(rng.randrange(97, 123) for _ in range(lit_len))
                    # a prefix literal that puts the long tag `before` bytes ahead of a piece end
                    pre = b""
                    for plen in range(1, 40):
                        cand = _lit(bytes(rng.randrange(65, 91) for _ in range(plen)))
                        hdr_len = len(_varint(plen + lit_len + 8))
                        start = hdr_len + len(cand)
                        if (start + before) % frag == 0 or frag == 1:
                            pre = cand
                            break
                    body = pre + _long_literal(data, nbytes) + _copy(4, 8)
                    ulen = (len(pre) - 1) + lit_len + 8
                    if kind == "short":
                        ulen -= rng.randrange(1, lit_len // 2)
                    elif kind == "overrun":
                        ulen = (len(pre) - 1) + rng.randrange(1, lit_len)
                    elif kind == "cut":
                        body = body[: len(pre) + 1 + nbytes + rng.randrange(0, lit_len)]
                    elif kind == "badcopy":
                        body = body[:-2] + _copy(4000, 8)
                    comp = _varint(ulen) + body
                    r, got = ref.uncompress_as_much(comp, ulen, frag)
                    cases.append({"frag": frag, "nbytes": nbytes, "before": before, "kind": kind,
                                  "hex": comp.hex(), "ulen": ulen, "ret": r, "got_len": len(got),
                                  "got_fnv": "%016x" % fsg.fnv1a64(got)})
    (HERE / "partial_frag.json").write_text(json.dumps(cases, indent=1) + "\n")
    print(len(cases), "partial_frag cases")


def _lit(b: bytes) -> bytes:
    n = len(b) - 1
    if n < 60:
        return bytes([n << 2]) + b
    k = (n.bit_length() + 7) // 8
    return bytes([(59 + k) << 2]) + n.to_bytes(k, "little") + b


def _copy(off: int, ln: int) -> bytes:
    if 4 <= ln <= 11 and off < 2048:
        return bytes([((off >> 8) << 5) | ((ln - 4) << 2) | 1, off & 0xFF])
    return bytes([((ln - 1) << 2) | 2]) + off.to_bytes(2, "little")


def main():
    ref = Reference()
    if "--partial-only" in sys.argv:
        make_partial_frag(ref)
        return
    if "--c5-only" in sys.argv:
        make_full_c5(ref)
        return
    if "--full-only" in sys.argv:
        make_full(ref)
        return
    vectors = []
    for spec in positive_specs():
        data = build_input(spec)
        comp = ref.compress(data)
        # fragmentation independence: same bytes at other Peek sizes
        for frag in (1, 7, 65536, 1 << 30):
            assert ref.compress(data, frag) == comp, spec
        ok, out = ref.uncompress(comp, len(data))
        assert ok and out == data, spec
        entry = dict(spec)
        entry["input_len"] = len(data)
        entry["input_fnv"] = "%016x" % fsg.fnv1a64(data)
        entry["compressed_len"] = len(comp)
        entry["compressed_fnv"] = "%016x" % fsg.fnv1a64(comp)
        if len(comp) <= 2048:
            entry["compressed_hex"] = comp.hex()
        vectors.append(entry)
    (HERE / "vectors.json").write_text(json.dumps(vectors, indent=1) + "\n")

    neg = []
    for name, comp in negative_cases(ref):
        ok_src, ulen_src = ref.header_source(comp)
        ok_strict, ulen_strict = ref.header_strict(comp)
        cap = ulen_src if ok_src and ulen_src <= (1 << 22) else 0
        if ok_src and ulen_src > (1 << 22):
            verdict = None  # too large to materialise; only header verdicts recorded
            out = b""
        else:
            verdict, out = ref.uncompress(comp, cap)
            for frag in (1, 3, 8160):
                assert ref.uncompress(comp, cap, frag)[0] == verdict, name
        # what UncompressAsMuchAsPossible (snappy.cc:1530-1535) leaves behind
        pret, partial = ref.uncompress_as_much(comp, cap) if ok_src and verdict is not None else (0, b"")
        neg.append({
            "name": name,
            "hex": comp.hex(),
            "header_ok": ok_src,
            "ulen": ulen_src if ok_src else 0,
            "strict_header_ok": ok_strict,
            "ok": verdict,
            "valid": ref.is_valid(comp),
            "output_fnv": "%016x" % fsg.fnv1a64(out) if verdict else None,
            "partial_ret": pret,
            "partial_len": len(partial),
            "partial_fnv": "%016x" % fsg.fnv1a64(partial),
        })
    (HERE / "negative.json").write_text(json.dumps(neg, indent=1) + "\n")

    # Per-config digests (first N messages of each synthetic batch).
    cfgs = {
        "C2": (fsg.KIND_RANDOM, np.full(1024, 4096, np.uint32)),
        "C3": (fsg.KIND_TEXT, np.full(256, 65536, np.uint32)),
        "CM": (fsg.KIND_MIXED, fsg.mixed_sizes(4096)),
        "C5": (fsg.KIND_PROTO, fsg.mixed_sizes(1024)),
    }
    for name, (kind, sizes) in cfgs.items():
        b = fsg.make_batch(kind, sizes)
        clen = np.zeros(len(b), np.uint32)
        cfnv = np.zeros(len(b), np.uint64)
        for i in range(len(b)):
            c = ref.compress(b.item(i))
            clen[i] = len(c)
            cfnv[i] = fsg.fnv1a64(c)
        np.savez(HERE / f"digests_{name}.npz", input_len=b.lens, input_fnv=fsg.digests(b.data, b.offsets, b.lens),
                 compressed_len=clen, compressed_fnv=cfnv)
        print(name, len(b), "bodies, ratio %.3f" % (b.total / max(1, int(clen.sum()))))
    print(len(vectors), "positive vectors,", len(neg), "negative vectors")
    make_partial_frag(ref)
    make_full(ref)


if __name__ == "__main__":
    main()
