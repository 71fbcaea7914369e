"""Copy-dependency depth model (design tool, not product).

Prices a segment-resident execution pass before it is built: the whole 64 KiB
output of a segment lives in LDS, every literal lands in round 0, and in round
r every copy whose source bytes all landed in rounds < r lands.  Reports the
rounds each message needs and how many copies are still pending per round.

usage: python tools/depth_sim.py [n_msgs] [kind]     (kind 0 = C3 text)
"""
from __future__ import annotations

import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "flare-cpp_amd" / "py"))
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tools"))
import fsg  # noqa: E402
from oracle.bind import Oracle  # noqa: E402  (test infrastructure: compresses the samples)
from exec_sim import parse  # noqa: E402


def rounds_of(tags):
    """Per-tag landing round under Jacobi execution at byte granularity."""
    total = sum(t[1] for t in tags)
    rnd = np.zeros(total, np.int32)
    out = []
    op = 0
    for is_lit, ln, x in tags:
        if is_lit:
            r = 0
        else:
            src = op - x
            if x >= ln:
                r = 1 + int(rnd[src:src + ln].max())
            else:                       # pattern copy: needs [src, op)
                r = 1 + int(rnd[src:op].max())
        rnd[op:op + ln] = r
        out.append((is_lit, ln, x, r))
        op += ln
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    kind = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    b = fsg.make_batch(kind, np.full(n, 65536, np.uint32))
    o = Oracle()
    maxes, ntags, ncopies = [], [], []
    hist = np.zeros(512, np.int64)
    pend = np.zeros(512, np.int64)
    for i in range(n):
        comp = o.compress(b.item(i))
        tags = parse(comp)
        rt = rounds_of(tags)
        rs = np.array([t[3] for t in rt])
        maxes.append(rs.max())
        ntags.append(len(rt))
        ncopies.append(sum(1 for t in rt if not t[0]))
        h = np.bincount(rs, minlength=512)[:512]
        hist += h
        pend += np.cumsum(h[::-1])[::-1]
    print(f"msgs {n}: tags/msg {np.mean(ntags):.0f}, copies/msg {np.mean(ncopies):.0f}")
    print(f"max round per msg: mean {np.mean(maxes):.1f} p50 {np.median(maxes):.0f} max {np.max(maxes)}")
    print("round: tags landing (per msg) / tags pending at round start (per msg)")
    for r in range(int(np.max(maxes)) + 1):
        print(f"  {r:3d}: {hist[r] / n:8.1f}  {pend[r] / n:8.1f}")


if __name__ == "__main__":
    main()
