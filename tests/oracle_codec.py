"""TEST INFRASTRUCTURE ONLY: the oracle behind fsg.SnappyGPU's method surface,
on CPU tensors.  Used by the CPU runs of bench.py's multi-rank launcher
(tests/bench_cpu_rank.py) so the sharding, timing and collectives can be
exercised with gloo where there is no GPU.  Never imported by the product
path or by bench.py itself."""
from __future__ import annotations

import numpy as np

from bind import Oracle


def _np(t):
    return t.numpy()


class OracleCodec:
    def __init__(self):
        self.o = Oracle()

    def select_kernels(self, decode=0, encode=0):
        pass

    def compress_workspace(self, n, max_in_len, device=None):
        import torch
        return torch.zeros(1, dtype=torch.uint8)

    def decompress_workspace(self, n, total_in=0, device=None):
        import torch
        return torch.zeros(1, dtype=torch.uint8)

    def compress(self, d_in, d_in_off, d_in_len, n, max_in_len, d_out, d_out_off, d_out_len, d_status,
                 stream=None, workspace=None):
        if n == 0:
            return
        self.o.compress_batch(_np(d_in), _np(d_in_off)[:n], _np(d_in_len)[:n], _np(d_out), _np(d_out_off)[:n],
                              _np(d_out_len)[:n], threads=2)
        d_status[:n] = 0

    def decompress(self, d_in, d_in_off, d_in_len, n, d_out, d_out_off, d_out_cap, d_out_len, d_status,
                   flags=0, stream=None, workspace=None):
        if n == 0:
            return
        st = np.zeros(n, np.int32)
        self.o.uncompress_batch(_np(d_in), _np(d_in_off)[:n], _np(d_in_len)[:n], _np(d_out),
                                _np(d_out_off)[:n], _np(d_out_cap)[:n], _np(d_out_len)[:n], st, threads=2)
        d_status[:n] = __import__("torch").from_numpy(st)
