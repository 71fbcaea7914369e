"""LZ4 leg: device-resident batched LZ4 encode
and decode of the C3 bodies (65,536 x 64 KiB text), timed with HIP events on
the launch stream, round trip and an oracle sample checked untimed.  CPU
lines beside it: the oracle (single thread) and the system liblz4 1.9.3 on a
sample (checkers only, never the product path).

    python tools/lz4_bench.py [--n 65536] [--size 65536] [--steps 5]
"""
import argparse
import json
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parents[1]
for p in (REPO / "flare-cpp_amd" / "py", REPO / "oracle", REPO / "tests"):
    sys.path.insert(0, str(p))
import fsg  # noqa: E402

GIB = float(1 << 30)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=65536)
    ap.add_argument("--size", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--two-pass-only", action="store_true", help="skip the one-pass decode timing")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU lines")
    ap.add_argument("--no-pipelined", action="store_true",
                    help="skip the stream of two alternating batches (fsg_lz4_decompress_batch_2s)")
    a = ap.parse_args()
    import torch
    dev = torch.device("cuda", 0)
    codec = fsg.SnappyGPU(0)
    lib = codec.lib
    batch = fsg.make_batch(fsg.KIND_TEXT, np.full(a.n, a.size, np.uint32))
    n, raw = len(batch), batch.total
    H = lambda x: torch.from_numpy(np.ascontiguousarray(x)).to(dev)  # noqa: E731
    d_raw, d_ro, d_rl = H(batch.data), H(batch.offsets), H(batch.lens)
    caps = np.array([lib.fsg_lz4_max_compressed_length(int(x)) for x in batch.lens], np.uint64)
    c_off, c_tot = fsg.slot_offsets(caps)
    d_c, d_co = torch.zeros(c_tot, dtype=torch.uint8, device=dev), H(c_off)
    d_cl = torch.zeros(n, dtype=torch.int32, device=dev)
    d_st = torch.zeros(n, dtype=torch.int32, device=dev)
    ws = codec.lz4_compress_workspace(n)
    d_out = torch.zeros(raw, dtype=torch.uint8, device=dev)
    d_ol = torch.zeros(n, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()

    def enc():
        codec.lz4_compress(d_raw, d_ro, d_rl, n, d_c, d_co, d_cl, d_st, ws, stream=s)

    def dec():
        codec.lz4_decompress(d_c, d_co, d_cl, n, d_out, d_ro, d_rl, d_ol, d_st, stream=s)

    dws = None

    def dec2():  # the two-pass decoder (fsg_lz4_decompress_batch_ws)
        codec.lz4_decompress(d_c, d_co, d_cl, n, d_out, d_ro, d_rl, d_ol, d_st, stream=s, workspace=dws)

    def timed(fn, steps=None):
        steps = a.steps if steps is None else steps
        fn()
        torch.cuda.synchronize()
        if steps == 0:
            return float("nan")
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(steps):
            fn()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps

    enc_ms = timed(enc, 0 if a.two_pass_only else None)
    comp_len = d_cl.cpu().numpy().view(np.uint32)
    comp = int(comp_len.astype(np.uint64).sum())
    enc_ok = int((d_st != 0).sum().item()) == 0
    dec_ms = timed(dec) if not a.two_pass_only else float("nan")
    dec_ok = a.two_pass_only or (int((d_st != 0).sum().item()) == 0 and bool(torch.equal(d_out, d_raw)))
    dws = codec.lz4_decompress_workspace(n, int(c_tot))
    d_out.fill_(0xA5)
    dec2_ms = timed(dec2)
    dec2_ok = int((d_st != 0).sum().item()) == 0 and bool(torch.equal(d_out, d_raw))
    # A stream of two alternating batches (the second one distinct), batch
    # k+1's index pass on a second stream beside batch k's execution
    # (fsg_lz4_decompress_batch_2s; bench.py's time_pipelined)
    pipe = None
    if not a.no_pipelined:
        sys.path.insert(0, str(REPO))
        from bench import time_pipelined
        batch2 = fsg.make_batch(fsg.KIND_TEXT, np.full(a.n, a.size, np.uint32), first_index=a.n)
        d_raw2, d_ro2, d_rl2 = H(batch2.data), H(batch2.offsets), H(batch2.lens)
        d_c2 = torch.zeros(c_tot, dtype=torch.uint8, device=dev)
        d_cl2 = torch.zeros(n, dtype=torch.int32, device=dev)
        d_st2 = torch.zeros(n, dtype=torch.int32, device=dev)
        codec.lz4_compress(d_raw2, d_ro2, d_rl2, n, d_c2, d_co, d_cl2, d_st2, ws, stream=s)
        d_out2 = torch.full((raw,), 0xA5, dtype=torch.uint8, device=dev)
        d_ol2 = torch.zeros(n, dtype=torch.int32, device=dev)
        dws2 = codec.lz4_decompress_workspace(n, int(c_tot))
        d_out.fill_(0xA5)
        slots = [(d_c, d_cl, d_out, d_ro, d_rl, d_ol, d_st, dws), (d_c2, d_cl2, d_out2, d_ro2, d_rl2, d_ol2, d_st2, dws2)]

        def issue(k, s1):
            c, cl, o, ro, rl, ol, st, w = slots[k % 2]
            codec.lz4_decompress(c, d_co, cl, n, o, ro, rl, ol, st, stream=s, workspace=w, pass1_stream=s1)

        steps = max(2, a.steps - a.steps % 2)
        _, t_ev, lat = time_pipelined(torch, dev, s, slots, issue, steps, 2, 1, None)
        ok = (int((d_st != 0).sum().item()) == 0 and int((d_st2 != 0).sum().item()) == 0
              and bool(torch.equal(d_out, d_raw)) and bool(torch.equal(d_out2, d_raw2)))
        raw2 = (raw + int(batch2.total)) / 2
        pipe = {"ms": round(t_ev * 1e3, 3), "gib_s": round(raw2 / t_ev / GIB, 3), "roundtrip_ok": ok,
                "latency_ms": round(lat * 1e3, 3), "steps": steps,
                "roofline_frac": round((raw2 + comp) / t_ev / 8e12, 4),
                "mode": "two alternating batches; batch k+1's index pass on a second stream beside batch k's "
                        "execution (fsg_lz4_decompress_batch_2s)"}
        del d_raw2, d_c2, d_out2, dws2
    from bind import Lz4Oracle
    o = Lz4Oracle()
    host_c = d_c.cpu().numpy()
    idx = np.linspace(0, n - 1, 32).astype(np.int64)
    sample_ok = all(host_c[int(c_off[i]):int(c_off[i]) + int(comp_len[i])].tobytes() == o.compress(batch.item(int(i)))
                    for i in idx)
    # CPU lines on a sample (checkers): oracle and system liblz4, one thread
    k = min(n, 1024 if not a.no_cpu else 1)
    items = [batch.item(i) for i in range(k)]
    t = time.perf_counter()
    blocks = [o.compress_block(x) for x in items]
    t_oc = time.perf_counter() - t
    t = time.perf_counter()
    for x, b in zip(items, blocks):
        o.decompress_block(b, len(x))
    t_od = time.perf_counter() - t
    sysl = None
    try:
        from lz4_sys import SysLz4, load
        L = load()
        if L is not None:
            z = SysLz4(L)
            t = time.perf_counter()
            for x in items:
                z.compress(x)
            t_sc = time.perf_counter() - t
            t = time.perf_counter()
            for x, b in zip(items, blocks):
                z.decompress(b, len(x))
            t_sd = time.perf_counter() - t
            kb = sum(map(len, items))
            sysl = {"compress_gib_s": round(kb / t_sc / GIB, 3), "decompress_gib_s": round(kb / t_sd / GIB, 3),
                    "cores": 1, "version": z.version}
    except Exception as e:  # pragma: no cover - diagnostic only
        sysl = {"error": str(e)}
    kb = sum(map(len, items))
    out = {
        "workload": f"C3 bodies through LZ4: {n} x {a.size} B text, device-resident",
        "raw_bytes": raw, "compressed_bytes": comp, "ratio": round(raw / comp, 4),
        "encode": {"ms": round(enc_ms, 3), "gib_s": round(raw / (enc_ms / 1e3) / GIB, 3), "status_ok": enc_ok,
                   "roofline_frac": round((raw + comp) / (enc_ms / 1e3) / 8e12, 4)},
        "decode": {"ms": round(dec_ms, 3), "gib_s": round(raw / (dec_ms / 1e3) / GIB, 3), "roundtrip_ok": dec_ok,
                   "roofline_frac": round((raw + comp) / (dec_ms / 1e3) / 8e12, 4)},
        "decode_two_pass": {"ms": round(dec2_ms, 3), "gib_s": round(raw / (dec2_ms / 1e3) / GIB, 3),
                            "roundtrip_ok": dec2_ok, "roofline_frac": round((raw + comp) / (dec2_ms / 1e3) / 8e12, 4)},
        "decode_two_pass_pipelined": pipe,
        "oracle_sample_ok": sample_ok,
        "cpu_oracle_1thread": {"compress_gib_s": round(kb / t_oc / GIB, 3), "decompress_gib_s": round(kb / t_od / GIB, 3),
                               "sample": f"first {k} bodies"},
        "cpu_system_liblz4_1thread": sysl,
    }
    print(json.dumps(out))


if __name__ == "__main__":
    main()
