"""The packed execution pass's virtual layout (csrc/snappy_decode_v4.hip,
exec5_packed), restated on the host: the bodies of a batch end to end, body
j at V_j congruent to its slot address modulo 16, so that every 16-byte
virtual block belongs to one body and maps to one 16-byte-aligned slot
block; the gap before a body's first tag is < 32 bytes (it rides in 5 bits
of the body's word).  Pure arithmetic, no GPU."""
import numpy as np


def layout(slot_addr, lens):
    """(V, VE, gap) as the kernel computes them: sz = round_up16((addr & 15)
    + E), V = exclusive prefix of sz + (addr & 15), gap = V - VE(previous)."""
    sz = ((slot_addr & 15) + lens + 15) & ~np.uint64(15)
    V = np.cumsum(sz) - sz + (slot_addr & 15)
    VE = V + lens
    gap = np.zeros_like(V)
    gap[1:] = V[1:] - VE[:-1]
    return V, VE, gap


def test_layout_invariants():
    rng = np.random.default_rng(11)
    for _ in range(200):
        n = int(rng.integers(1, 65))
        lens = rng.integers(1, 20000, n).astype(np.uint64)
        addr = rng.integers(0, 1 << 40, n).astype(np.uint64)
        V, VE, gap = layout(addr, lens)
        assert (V % 16 == addr % 16).all()          # window blocks = slot blocks
        assert (gap < 32).all() and gap[0] == 0     # fits the 5-bit gap field
        assert (V[1:] >= VE[:-1]).all()             # bodies in order, disjoint
        # no 16-byte block holds bytes of two bodies
        assert (((VE[:-1] - 1) >> np.uint64(4)) < (V[1:] >> np.uint64(4))).all()
        # slot offset of virtual position v in body j: v + (addr_j - V_j), 16-aligned shift
        assert ((addr - V) % 16 == 0).all()
