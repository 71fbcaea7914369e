"""Streams whose copy sources sit exactly at the edge of pass 2's LDS window.

exec_message (flare-cpp_amd/csrc/snappy_decode_v4.hip, pass 2) assembles a
message's output in a per-wave window holding output positions
[sbase, sbase + 3072).  A copy whose source starts below sbase is a "far" copy:
round A loads it from the output already stored to global memory; any other
copy reads the window (rounds B).  `window_model` replays the kernel's group
and window rules on a tag list:

  * a group is the next <= 64 tags, cut before a literal longer than 64 bytes
    and, for the default execution pass (decode variant 5, one tag per lane,
    rule "tags"), where the group's output would pass 1,024 bytes; for the
    piece-per-lane pass (variant 4, rule "pieces") where the group's pieces
    (ceil(len / 16), or the pattern piece count for offsets < 16) would pass
    64;
  * a literal longer than 64 bytes runs alone, and the window restarts one
    block below the block holding the new write position:
    sbase = (op & ~15) - 16;
  * before a group whose output would overrun the window, the window slides to
    sbase = (op - 1024) & ~15.

(Slots 16-byte aligned, as the test harness allocates them.)  The generator
lays down the tag lengths first, runs the model, then gives each copy an
offset that puts its source a few bytes either side of its group's sbase, so
far/near classification, the straddling 16-byte loads and the window restart
after long literals are all hit at the exact boundary.
"""
from __future__ import annotations

import numpy as np

WINDOW, KEEP, MAX_PIECES, GROUP_BYTES = 3072, 1024, 64, 1024


def _pieces(ln: int, off: int) -> int:
    if off and off < 16:  # pattern copy: pieces of (16 // off) * off bytes
        step = (16 // off) * off
        return -(-ln // step)
    return -(-ln // 16)


def window_model(tags, rule: str = "tags"):
    """tags: list of (is_literal, length, offset).  Returns, per tag, the
    window base (sbase) in force when its group runs and its output position.
    rule: "tags" (decode variant 5) or "pieces" (variant 4)."""
    sb = [0] * len(tags)
    pos = [0] * len(tags)
    op, sbase, i = 0, 0, 0
    while i < len(tags):
        lit, ln, off = tags[i]
        if lit and ln > 64:
            sb[i], pos[i] = sbase, op
            op += ln
            sbase = (op & ~15) - 16
            i += 1
            continue
        j, pc, tot = i, 0, 0
        while j < len(tags) and j - i < 64:
            l2, n2, o2 = tags[j]
            if l2 and n2 > 64:
                break
            p = _pieces(n2, 0 if l2 else o2) if rule == "pieces" else 0
            if pc + p > MAX_PIECES or (rule == "tags" and tot + n2 > GROUP_BYTES):
                break
            pc += p
            tot += n2
            j += 1
        if op + tot - sbase > WINDOW:
            sbase = (op - KEEP) & ~15
        t = op
        for k in range(i, j):
            sb[k], pos[k] = sbase, t
            t += tags[k][1]
        op, i = t, j
    return sb, pos


def _emit_literal(data: bytes) -> bytes:
    n = len(data) - 1
    if n < 60:
        return bytes([n << 2]) + data
    k = (n.bit_length() + 7) // 8
    return bytes([(59 + k) << 2]) + n.to_bytes(k, "little") + data


def _emit_copy(off: int, ln: int) -> bytes:
    if 4 <= ln <= 11 and off < 2048:
        return bytes([((off >> 8) << 5) | ((ln - 4) << 2) | 1, off & 0xFF])
    return bytes([((ln - 1) << 2) | 2]) + off.to_bytes(2, "little")


def edge_stream(rng, target: int, spread: int = 24, rule: str = "tags"):
    """(compressed, raw, n_edge): a valid stream of ~target output bytes whose
    copies read from sbase - spread .. sbase + spread of their group (when the
    output so far allows), plus the count of copies whose 16-byte source load
    straddles sbase."""
    tags = []
    n = 0
    while n < target:
        r = rng.random()
        if r < 0.08 and n > 0:
            ln = int(rng.integers(65, 400))       # long literal: window restart
            tags.append((True, ln, 0))
        elif r < 0.35 or n < 32:
            ln = int(rng.integers(1, 17))
            tags.append((True, ln, 0))
        else:
            ln = int(rng.integers(4, 65))
            tags.append((False, ln, 16))          # offset fixed below (>= 16)
        n += ln
    sb, pos = window_model(tags, rule)
    out = bytearray()
    body = []
    n_edge = 0
    for (lit, ln, _), s, p in zip(tags, sb, pos):
        assert p == len(out)
        if lit:
            data = bytes(rng.integers(0, 256, ln, dtype=np.uint8))
            body.append(_emit_literal(data))
            out += data
            continue
        src = s + int(rng.integers(-spread, spread + 1))
        off = p - src
        if off < 16 or off > p or off > 0xFFFF:
            off = int(rng.integers(16, p + 1)) if p >= 16 else p
        if off < 16:  # too little output yet for a non-pattern copy: a literal instead
            data = bytes(rng.integers(0, 256, ln, dtype=np.uint8))
            body.append(_emit_literal(data))
            out += data
            continue
        src = p - off
        n_edge += src < s < src + 16
        body.append(_emit_copy(off, ln))
        for _ in range(ln):
            out.append(out[-off])
    hdr = bytearray()
    v = len(out)
    while v >= 0x80:
        hdr.append((v & 0x7F) | 0x80)
        v >>= 7
    hdr.append(v)
    return bytes(hdr) + b"".join(body), bytes(out), n_edge
