"""TEST INFRASTRUCTURE ONLY: LZ4 blocks built sequence by sequence, valid by
construction under oracle/lz4_oracle.c's rules (lz4o_decompress_block), to
reach what the compressor rarely emits: literal and match lengths at every
extension-byte boundary (14/15/269/270/..., 18/19/273/274/...), long 255
runs, zero-length literals, offsets 1..15 (periodic copies), 16..1536 and
above, matches longer than their offset, and matches of tens of KiB.

A block is a list of (literal bytes, offset, match length) sequences and a
final literal run of >= 12 bytes, which makes every earlier sequence a
non-last one (op + lit + 12 <= ulen, ip + lit + 8 <= n, ml + 5 <= ulen - op)
and the final run a valid last sequence."""
import numpy as np


def _length(out: bytearray, v: int):
    while v >= 255:
        out.append(255)
        v -= 255
    out.append(v)


def encode_block(seqs, final: bytes) -> bytes:
    blk = bytearray()
    for lit, off, ml in seqs:
        ll, mm = len(lit), ml - 4
        blk.append((min(ll, 15) << 4) | min(mm, 15))
        if ll >= 15:
            _length(blk, ll - 15)
        blk += lit
        blk += bytes([off & 0xFF, off >> 8])
        if mm >= 15:
            _length(blk, mm - 15)
    ll = len(final)
    blk.append(min(ll, 15) << 4)
    if ll >= 15:
        _length(blk, ll - 15)
    blk += final
    return bytes(blk)


def header(n: int) -> bytes:
    out = bytearray()
    while n >= 0x80:
        out.append((n & 0x7F) | 0x80)
        n >>= 7
    out.append(n)
    return bytes(out)


_LITS = [0, 0, 0, 1, 2, 5, 13, 14, 15, 16, 17, 30, 63, 64, 65, 100, 269, 270, 271, 524, 525, 1000, 4000]
_MLS = [4, 5, 8, 15, 16, 17, 18, 19, 20, 31, 63, 64, 65, 66, 100, 273, 274, 275, 528, 529, 1500, 5000, 40000]
_OFFS_SMALL = list(range(1, 16))


def random_block(rng, target: int):
    """(body, expected output) for a random valid block of about `target`
    output bytes.  The output is assembled here by the same rules the
    decoder follows (byte by byte for overlapping matches)."""
    out = bytearray()
    seqs = []
    # a first literal run gives the matches something to copy
    first = rng.integers(0, 256, int(rng.integers(1, 64)), dtype=np.uint8).tobytes()
    while len(out) < target:
        r = rng.random()
        if r < 0.6:
            ll = int(rng.choice(_LITS))
        else:
            ll = int(rng.integers(0, 40))
        lit = rng.integers(0, int(rng.choice([4, 256])), ll, dtype=np.uint8).tobytes()
        if not seqs and not out:
            lit = first + lit
        op = len(out) + len(lit)
        r = rng.random()
        if r < 0.3:
            off = int(rng.choice(_OFFS_SMALL))
        elif r < 0.55:
            off = int(rng.integers(16, 1537))
        elif r < 0.75:
            off = int(rng.integers(1537, 65536))
        else:
            off = int(rng.integers(1, 64))
        off = max(1, min(off, op, 65535))
        ml = int(rng.choice(_MLS)) if rng.random() < 0.6 else int(rng.integers(4, 40))
        out += lit
        for _ in range(ml):
            out.append(out[-off])
        seqs.append((lit, off, ml))
    final = rng.integers(0, 256, int(rng.integers(12, 80)), dtype=np.uint8).tobytes()
    out += final
    return header(len(out)) + encode_block(seqs, final), bytes(out)
