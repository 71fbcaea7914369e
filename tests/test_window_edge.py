"""CPU side of the window-edge streams (tests/window_edge.py): every stream is
valid (the oracle decodes it to the generator's bytes) and the set straddles
the window base often.  The GPU decode of the same streams is
test_gpu_parity.py::test_far_copies_at_window_edge."""
import numpy as np

from bind import Oracle
from window_edge import edge_stream, window_model


def test_window_model_rules():
    # 64 16-byte literals per group; the window slides once output passes 3072
    tags = [(True, 16, 0)] * 400
    sb, pos = window_model(tags)
    assert pos[64] == 64 * 16 and sb[0] == 0
    first_slide = next(i for i, s in enumerate(sb) if s)
    assert pos[first_slide] + 64 * 16 > 3072 >= pos[first_slide]
    assert sb[first_slide] == (pos[first_slide] - 1024) & ~15
    # a long literal runs alone and restarts the window below its end
    sb, pos = window_model([(True, 10, 0), (True, 100, 0), (False, 8, 20)])
    assert sb[2] == ((110 & ~15) - 16)
    # the first slide comes before the group that would pass 3072: one tag per
    # lane cuts groups at 1,024 output bytes (51 x 20-byte literals), pieces
    # at 64 pieces (32 x two-piece literals)
    tags = [(True, 20, 0)] * 400
    for rule, per_group in (("tags", 51), ("pieces", 32)):
        sb, pos = window_model(tags, rule)
        first_slide = next(i for i, s in enumerate(sb) if s)
        assert first_slide % per_group == 0, rule
        assert pos[first_slide] + 20 * per_group > 3072 >= pos[first_slide], rule


def test_edge_streams_valid():
    o = Oracle()
    rng = np.random.default_rng(8)
    n_edge = 0
    for i in range(60):
        c, raw, e = edge_stream(rng, int(rng.integers(3000, 30000)), rule="tags" if i % 2 else "pieces")
        ok, ulen, ref = o.uncompress(c, cap=len(raw))
        assert ok and ref == raw, i
        n_edge += e
    assert n_edge > 500
