"""Shared GPU-test plumbing: move host batches to the device, run the C ABI,
bring results back.  torch is used only for device allocations/streams.

Output slots are filled with POISON (0xA5) before every call, never zeros: an
output byte a kernel fails to write then shows up as 0xA5 instead of passing
whenever its true value happens to be 0."""
from __future__ import annotations

import numpy as np

import fsg

POISON = 0xA5


def dev(a: np.ndarray, device="cuda"):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(device)


def empty(n: int, dtype, device="cuda"):
    import torch
    return torch.empty(max(n, 1), dtype=dtype, device=device)


class GpuCodec:
    def __init__(self, use_workspace: bool = True):
        import torch
        self.use_workspace = use_workspace
        self.torch = torch
        self.codec = fsg.SnappyGPU(torch.cuda.current_device())

    def compress(self, batch: fsg.Batch):
        torch = self.torch
        n = len(batch)
        caps = np.array([fsg.max_compressed_length(int(x)) for x in batch.lens], dtype=np.uint64)
        oo, tot = fsg.slot_offsets(caps)
        d_in = dev(batch.data)
        d_io, d_il = dev(batch.offsets), dev(batch.lens)
        d_out = torch.full((max(tot, 1),), POISON, dtype=torch.uint8, device="cuda")
        d_oo = dev(oo)
        d_ol = empty(n, torch.int32)
        d_st = torch.full((max(n, 1),), -7, dtype=torch.int32, device="cuda")
        mx = int(batch.lens.max()) if n else 0
        ws = self.codec.compress_workspace(n, mx) if self.use_workspace else None
        self.codec.compress(d_in, d_io, d_il, n, mx, d_out, d_oo, d_ol, d_st, workspace=ws)
        torch.cuda.synchronize()
        out = d_out.cpu().numpy()
        ol = d_ol.cpu().numpy()[:n].view(np.uint32)
        st = d_st.cpu().numpy()[:n]
        return [out[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() for i in range(n)], st

    def decompress(self, comps: list[bytes], caps: list[int], flags: int = 0,
                   ws_total_in: int | None = None, ws_fill: int | None = None, slot_skew: int = 0):
        """ws_total_in: input size the workspace is sized for (default: the
        real packed size; smaller values force the v4 fallback path).
        ws_fill: byte the workspace is filled with before the call (the
        decoder must not rely on a zeroed workspace).
        slot_skew: output slot i starts (i * slot_skew) % 16 bytes past its
        16-byte-aligned place (slots of every alignment)."""
        torch = self.torch
        b = fsg.Batch.from_list(comps)
        n = len(b)
        caps = np.array(caps, dtype=np.uint32)
        oo, tot = fsg.slot_offsets(caps.astype(np.uint64) + (16 if slot_skew else 0))
        if slot_skew:
            oo = oo + (np.arange(n, dtype=np.uint64) * slot_skew) % 16
        d_out = torch.full((max(tot, 1),), POISON, dtype=torch.uint8, device="cuda")
        d_ol = empty(n, torch.int32)
        d_st = torch.full((max(n, 1),), -7, dtype=torch.int32, device="cuda")
        total_in = int(b.data.size) if ws_total_in is None else ws_total_in
        ws = self.codec.decompress_workspace(n, total_in) if self.use_workspace else None
        if ws is not None and ws_fill is not None:
            ws.fill_(ws_fill)
        self.codec.decompress(dev(b.data), dev(b.offsets), dev(b.lens), n, d_out, dev(oo), dev(caps),
                              d_ol, d_st, flags=flags, workspace=ws)
        torch.cuda.synchronize()
        out = d_out.cpu().numpy()
        ol = d_ol.cpu().numpy()[:n].view(np.uint32)
        st = d_st.cpu().numpy()[:n]
        outs = [out[int(oo[i]):int(oo[i]) + int(min(ol[i], caps[i]))].tobytes() for i in range(n)]
        return outs, ol, st

    # ---- LZ4 bodies (include/flare_lz4_gpu.h)
    def lz4_compress(self, batch: fsg.Batch):
        torch = self.torch
        n = len(batch)
        caps = np.array([self.codec.lib.fsg_lz4_max_compressed_length(int(x)) for x in batch.lens], dtype=np.uint64)
        oo, tot = fsg.slot_offsets(caps)
        d_out = torch.full((max(tot, 1),), POISON, dtype=torch.uint8, device="cuda")
        d_ol = empty(n, torch.int32)
        d_st = torch.full((max(n, 1),), -7, dtype=torch.int32, device="cuda")
        ws = self.codec.lz4_compress_workspace(n)
        self.codec.lz4_compress(dev(batch.data), dev(batch.offsets), dev(batch.lens), n, d_out, dev(oo), d_ol, d_st,
                                ws)
        torch.cuda.synchronize()
        out = d_out.cpu().numpy()
        ol = d_ol.cpu().numpy()[:n].view(np.uint32)
        st = d_st.cpu().numpy()[:n]
        return [out[int(oo[i]):int(oo[i]) + int(ol[i])].tobytes() for i in range(n)], st

    def lz4_decompress(self, bodies: list[bytes], caps: list[int], two_pass: bool = True,
                       ws_total_in: int | None = None, ws_fill: int | None = None):
        """two_pass: fsg_lz4_decompress_batch_ws with a workspace sized for
        ws_total_in input bytes (default: the real size; smaller values send
        messages to the one-pass fallback), filled with ws_fill first."""
        torch = self.torch
        b = fsg.Batch.from_list(bodies)
        n = len(b)
        caps = np.array(caps, dtype=np.uint32)
        oo, tot = fsg.slot_offsets(caps.astype(np.uint64))
        d_out = torch.full((max(tot, 1),), POISON, dtype=torch.uint8, device="cuda")
        d_ol = empty(n, torch.int32)
        d_st = torch.full((max(n, 1),), -7, dtype=torch.int32, device="cuda")
        ws = None
        if two_pass:
            ws = self.codec.lz4_decompress_workspace(n, int(b.data.size) if ws_total_in is None else ws_total_in)
            if ws_fill is not None:
                ws.fill_(ws_fill)
        self.codec.lz4_decompress(dev(b.data), dev(b.offsets), dev(b.lens), n, d_out, dev(oo), dev(caps), d_ol, d_st,
                                  workspace=ws)
        torch.cuda.synchronize()
        out = d_out.cpu().numpy()
        ol = d_ol.cpu().numpy()[:n].view(np.uint32)
        st = d_st.cpu().numpy()[:n]
        outs = [out[int(oo[i]):int(oo[i]) + int(min(ol[i], caps[i]))].tobytes() for i in range(n)]
        return outs, ol, st
