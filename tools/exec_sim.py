"""Exec-pass model (design tool, not product): replays the v5 exec pass's group,
window and chunk rules over C3 messages and counts dependency rounds per group
under several readiness / forwarding policies, so a restructuring can be priced
before it is built.

usage: python tools/exec_sim.py [n_msgs] [kind]     (kind 0 = C3 text)
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "flare-cpp_amd" / "py"))
sys.path.insert(0, str(ROOT))
import fsg  # noqa: E402
from oracle.bind import Oracle  # noqa: E402  (test infrastructure: compresses the samples)

WINDOW, KEEP, GROUP_BYTES = 3072, 1024, 1024


def pat_step(off):
    return (16 // off) * off


def parse(comp: bytes):
    """[(is_lit, len, src_or_off)] ; literals carry their input offset."""
    ip, r, sh = 0, 0, 0
    while True:
        c = comp[ip]
        r |= (c & 0x7F) << sh
        sh += 7
        ip += 1
        if c < 128:
            break
    tags = []
    n = len(comp)
    while ip < n:
        c = comp[ip]
        t = c & 3
        if t == 0:
            l0 = (c >> 2) + 1
            if l0 <= 60:
                tags.append((True, l0, ip + 1))
                ip += 1 + l0
            else:
                nb = l0 - 60
                ln = int.from_bytes(comp[ip + 1:ip + 1 + nb], "little") + 1
                tags.append((True, ln, ip + 1 + nb))
                ip += 1 + nb + ln
        elif t == 1:
            tags.append((False, 4 + ((c >> 2) & 7), ((c >> 5) << 8) | comp[ip + 1]))
            ip += 2
        elif t == 2:
            tags.append((False, (c >> 2) + 1, comp[ip + 1] | comp[ip + 2] << 8))
            ip += 3
        else:
            tags.append((False, (c >> 2) + 1, int.from_bytes(comp[ip + 1:ip + 5], "little")))
            ip += 5
    return tags


def groups(tags):
    """Yield (op, sbase, [(is_lit, len, src, t_op)]) per group as v5 forms them."""
    op, sbase = 0, -16 if False else 0
    i, n = 0, len(tags)
    while i < n:
        take0 = min(64, n - i)
        big = [k for k in range(take0) if tags[i + k][0] and tags[i + k][1] > 64]
        if big and big[0] == 0:
            op += tags[i][1]
            sbase = (op & ~15) - 16
            i += 1
            continue
        take = big[0] if big else take0
        g, tot = [], 0
        for k in range(take):
            lit, ln, x = tags[i + k]
            if tot + ln > GROUP_BYTES:
                break
            t_op = op + tot
            src = x if lit else t_op - x
            g.append((lit, ln, src, t_op))
            tot += ln
        if op + tot - sbase > WINDOW:
            sbase = (op - KEEP) & ~15
        yield op, sbase, g
        op += tot
        i += len(g)


def chunks(op, sbase, g):
    """Per tag: list of chunks (dst, n, src, kind) kind: 'A' round A, 'B' rounds B
    (src in output coordinates), 'P' first chunk of a pattern."""
    out = []
    for lit, ln, src, t_op in g:
        nch = (ln + 15) >> 4
        if lit:
            out.append([(t_op + 16 * k, min(16, ln - 16 * k), None, "L") for k in range(nch)])
            continue
        off = t_op - src
        pat = off < 16 and off < ln
        below = sbase - src
        kfar = ((below - 1) >> 4) + 1 if below > 0 else 0
        kc = 0 if pat else min(kfar, nch)
        cl = [(t_op + 16 * k, min(16, ln - 16 * k), src + 16 * k, "F") for k in range(kc)]
        stp = pat_step(off) if pat else 16
        cw, sw, rem, first = t_op + 16 * kc, src + 16 * kc, ln - 16 * kc, True
        while rem > 0:
            nn = min(rem, stp)
            cl.append((cw, nn, sw, "P" if (pat and first) else "B"))
            rem -= nn
            cw += nn
            sw = cw - stp if pat else sw + nn
            first = False
        out.append(cl)
    return out


def rounds_watermark(op, tc):
    """v5 rule: per lane a sequence of B chunks; the lane's current chunk runs when
    its needed end ne <= W = the lowest pending lane's current destination."""
    lanes = [[c for c in cl if c[3] in "BP"] for cl in tc]
    pos = [0] * len(lanes)
    rounds = 0
    act = 0
    while True:
        pend = [j for j in range(len(lanes)) if pos[j] < len(lanes[j])]
        if not pend:
            return rounds, act
        W = lanes[pend[0]][pos[pend[0]]][0]
        ready = []
        for j in pend:
            dst, n, src, kind = lanes[j][pos[j]]
            ne = dst if kind == "P" else src + n
            if ne <= W:
                ready.append(j)
        for j in ready:
            pos[j] += 1
        rounds += 1
        act += len(ready)


def rounds_exact(op, tc, forward=False, sbase=0):
    """Exact byte readiness: a chunk runs once every byte it reads is final.
    forward: a B chunk whose source lies inside one round-A chunk of this group
    (a literal or a far chunk) reads that chunk's source instead (round A)."""
    final = {}
    allc = [c for cl in tc for c in cl]
    pend = []
    for c in allc:
        if c[3] in "LF":
            for b in range(c[0], c[0] + c[1]):
                final[b] = True
        else:
            pend.append(c)
    if forward:
        # byte -> (kind, source byte) of round-A chunks
        amap = {}
        for c in allc:
            if c[3] in "LF":
                for k in range(c[1]):
                    amap[c[0] + k] = c
        changed = True
        fw = []
        for c in pend:
            dst, n, src, kind = c
            if kind == "B" and src >= op:
                a = amap.get(src)
                if a is not None and src + n <= a[0] + a[1]:
                    for b in range(dst, dst + n):
                        final[b] = True
                    continue
            fw.append(c)
        pend = fw
    rounds = 0
    while pend:
        ready, rest = [], []
        for c in pend:
            dst, n, src, kind = c
            lo = dst - (pat_src_span(c)) if kind == "P" else src
            hi = dst if kind == "P" else src + n
            if all(b < op or final.get(b) for b in range(lo, hi)):
                ready.append(c)
            else:
                rest.append(c)
        # chunks of one lane run in order: only the first pending of a tag may run
        for c in ready:
            for b in range(c[0], c[0] + c[1]):
                final[b] = True
        pend = rest
        rounds += 1
        if rounds > 200:
            raise RuntimeError("no progress")
    return rounds


def pat_src_span(c):
    return c[0] - c[2] if c[2] is not None else 0


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    kind = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    b = fsg.make_batch(kind, np.full(n, 65536, np.uint32))
    orc = Oracle()
    st = dict(groups=0, tags=0, bytes=0, rw=0, act=0, rex=0, rfw=0, chunksA=0, chunksB=0, far=0)
    for i in range(n):
        comp = orc.compress(b.item(i))
        tags = parse(comp)
        for op, sbase, g in groups(tags):
            tc = chunks(op, sbase, g)
            st["groups"] += 1
            st["tags"] += len(g)
            st["bytes"] += sum(t[1] for t in g)
            r, a = rounds_watermark(op, tc)
            st["rw"] += r
            st["act"] += a
            st["rex"] += rounds_exact(op, tc)
            st["rfw"] += rounds_exact(op, tc, forward=True)
            for cl in tc:
                for c in cl:
                    st["chunksA" if c[3] in "LF" else "chunksB"] += 1
                    st["far"] += c[3] == "F"
    G = st["groups"]
    print(f"msgs {n} groups {G} tags/group {st['tags']/G:.1f} bytes/group {st['bytes']/G:.0f}")
    print(f"chunks per group: round A {st['chunksA']/G:.1f} (far {st['far']/G:.1f}), rounds B {st['chunksB']/G:.1f}")
    print(f"rounds B per group: watermark {st['rw']/G:.2f} (lanes per round {st['act']/max(1,st['rw']):.1f}),"
          f" exact {st['rex']/G:.2f}, exact+forward-from-round-A {st['rfw']/G:.2f}")


if __name__ == "__main__":
    main()
