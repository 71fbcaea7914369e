#!/usr/bin/env python3
"""Device-resident batched Snappy benchmark (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload c3-decompress]

One "step" = one pass of the hot path over one batch resident in HBM.
Default workload (the north-star target config): decompress
65,536 x 64 KiB Zipf-text bodies.  Other workloads: c2-decompress (65,536 x
4 KiB random), c3-compress, cm-decompress (power-law 256 B..1 MiB), c5-compress.

For N > 1 launch with torch.distributed.run; each rank owns its own shard of
messages (weak scaling, no data-path collective: messages are independent).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time
from pathlib import Path

import numpy as np

REPO = Path(__file__).resolve().parent
sys.path.insert(0, str(REPO / "flare-cpp_amd" / "py"))

import fsg  # noqa: E402
import shard  # noqa: E402

GIB = float(1 << 30)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak, /opt/skills/guides/MI355X_MICROARCH.md

WORKLOADS = {
    # name: (op, kind, n_msgs, size spec, description)
    "c3-decompress": ("decompress", fsg.KIND_TEXT, 65536, 65536,
                      "C3 decompress: 65,536 x 64 KiB Zipf-text bodies (~2.0x), device-resident"),
    "c2-decompress": ("decompress", fsg.KIND_RANDOM, 65536, 4096,
                      "C2 decompress: 65,536 x 4 KiB random bodies, device-resident"),
    "c3-compress": ("compress", fsg.KIND_TEXT, 65536, 65536,
                    "C3 compress: 65,536 x 64 KiB Zipf-text bodies, device-resident"),
    "cm-decompress": ("decompress", fsg.KIND_MIXED, 1 << 20, "mixed",
                      "CM decompress: 1,048,576 power-law bodies 256 B..1 MiB, 1 in 4 random"),
    "c5-compress": ("compress", fsg.KIND_PROTO, 262144, "mixed",
                    "C5 compress: 262,144 synthetic SnappyMessageProto responses"),
}


def kernel_source_hash() -> str:
    h = hashlib.sha256()
    for p in sorted((REPO / "flare-cpp_amd" / "csrc").glob("*")):
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="c3-decompress", choices=sorted(WORKLOADS))
    ap.add_argument("--n-msgs", type=int, default=0, help="override messages per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--verify-sample", type=int, default=64)
    ap.add_argument("--decode-lanes", type=int, default=-1,
                    help="lanes in flight for the persistent decoder (-1 = library default)")
    ap.add_argument("--decode-kernel", type=int, default=0,
                    help="decoder variant (0 = library default, 1-4 = force; A/B runs)")
    ap.add_argument("--encode-kernel", type=int, default=0,
                    help="encoder variant (0 = library default, 1-3 = force; A/B runs)")
    ap.add_argument("--scaling", choices=["weak", "strong"], default="weak",
                    help="weak: every GPU owns a full batch; strong: one batch split by bytes")
    return ap.parse_args()


def batch_sizes(size_spec, first_index, n):
    if size_spec == "mixed":
        # shard of the CM/C5 size stream: regenerate the stream prefix and slice
        return fsg.mixed_sizes(first_index + n)[first_index:]
    return np.full(n, size_spec, dtype=np.uint32)


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    codec = fsg.SnappyGPU(local)
    codec.select_kernels(args.decode_kernel, args.encode_kernel)

    op, kind, n_default, size_spec, desc = WORKLOADS[args.workload]
    n_cfg = args.n_msgs or n_default
    t_gen = time.time()
    if args.scaling == "weak":
        first, last = shard.weak_range(n_cfg, rank)  # rank owns [rank*n, (rank+1)*n)
    else:
        first, last = shard.byte_balanced_ranges(batch_sizes(size_spec, 0, n_cfg), world)[rank]
    n = last - first
    batch = fsg.make_batch(kind, batch_sizes(size_spec, first, n), first_index=first)
    raw_total = batch.total

    def H(a):
        return torch.from_numpy(np.ascontiguousarray(a)).to(dev)

    d_raw = H(batch.data)
    d_raw_off, d_raw_len = H(batch.offsets), H(batch.lens)
    caps = np.array([fsg.max_compressed_length(int(x)) for x in batch.lens], dtype=np.uint64)
    c_off, c_tot = fsg.slot_offsets(caps)
    d_comp = torch.zeros(c_tot, dtype=torch.uint8, device=dev)
    d_comp_off = H(c_off)
    d_comp_len = torch.zeros(n, dtype=torch.int32, device=dev)
    d_status = torch.zeros(n, dtype=torch.int32, device=dev)
    max_len = int(batch.lens.max())
    d_ws = codec.compress_workspace(n, max_len)
    # Compressed inputs come from the GPU encoder (checked against the oracle below).
    codec.compress(d_raw, d_raw_off, d_raw_len, n, max_len, d_comp, d_comp_off, d_comp_len, d_status,
                   workspace=d_ws)
    torch.cuda.synchronize()
    comp_len = d_comp_len.cpu().numpy().view(np.uint32).copy()
    comp_total = int(comp_len.astype(np.uint64).sum())
    errors = int((d_status != 0).sum().item())

    # Oracle spot check of the compressed bytes (checker only, never timed).
    sample_ok = None
    if args.verify_sample > 0:
        sys.path.insert(0, str(REPO / "oracle"))
        from bind import Oracle
        orc = Oracle()
        idx = np.linspace(0, n - 1, min(n, args.verify_sample)).astype(np.int64)
        host_comp = d_comp.cpu().numpy()
        sample_ok = all(
            host_comp[int(c_off[i]):int(c_off[i]) + int(comp_len[i])].tobytes() == orc.compress(batch.item(int(i)))
            for i in idx)

    # Decode output slots (exact uncompressed sizes) -- laid out like the raw batch.
    d_out = torch.zeros(max(raw_total, 1), dtype=torch.uint8, device=dev)
    d_out_len = torch.zeros(n, dtype=torch.int32, device=dev)
    d_cap = d_raw_len
    d_comp_len_u = d_comp_len  # int32 view is fine: lengths < 2^31
    stream = torch.cuda.current_stream()
    d_dws = codec.decompress_workspace(n, c_tot)

    if op == "decompress":
        def step():
            codec.decompress(d_comp, d_comp_off, d_comp_len_u, n, d_out, d_raw_off, d_cap, d_out_len,
                             d_status, stream=stream, workspace=d_dws)
        algo_bytes = raw_total + comp_total  # each input byte read once, each output byte written once
    else:
        def step():
            codec.compress(d_raw, d_raw_off, d_raw_len, n, max_len, d_comp, d_comp_off, d_comp_len,
                           d_status, stream=stream, workspace=d_ws)
        algo_bytes = raw_total + comp_total
    gen_s = time.time() - t_gen

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    evs = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps + 1)]
    t0 = time.perf_counter()
    evs[0].record(stream)
    for k in range(args.steps):
        step()
        evs[k + 1].record(stream)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    kern_ms = [evs[k].elapsed_time(evs[k + 1]) for k in range(args.steps)]
    avg_kernel_s = float(np.mean(kern_ms)) / 1e3

    # Correctness of the timed output (device-side, untimed).
    if op == "decompress":
        errors += int((d_status != 0).sum().item())
        roundtrip_ok = bool(torch.equal(d_out[:raw_total], d_raw[:raw_total]))
    else:
        errors += int((d_status != 0).sum().item())
        roundtrip_ok = bool((d_comp_len.cpu().numpy().view(np.uint32) == comp_len).all())

    t_step = wall / args.steps
    if world > 1:
        t_step, avg_kernel_s, (raw_all, comp_all, errors, bad) = shard.reduce_measurements(
            dist, dev, t_step, avg_kernel_s, raw_total, comp_total, errors, int(not roundtrip_ok))
        roundtrip_ok = bad == 0
    else:
        raw_all, comp_all = raw_total, comp_total

    # End-to-end (host pinned -> device -> kernel -> host pinned), untimed in `value`.
    e2e = None
    if not args.no_e2e and rank == 0:
        e2e = end_to_end(torch, codec, op, batch, d_comp, c_off, comp_len, raw_total, comp_total, n,
                         max_len, dev, d_ws)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(op, batch, d_comp, c_off, comp_len, args.cpu_threads)

    if rank == 0:
        value = raw_all / t_step / GIB
        achieved = algo_bytes / avg_kernel_s / 1e9
        pmc = load_traffic(args.workload)
        line = {
            "metric": "GiB/s device-resident Snappy decode+encode, batched RPC bodies, 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "GiB/s (uncompressed bytes)",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_step * 1e3, 4),
            "higher_is_better": True,
            "scaling": args.scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64-seeded bodies, SURVEY.md §8(d)); compressed by the GPU "
                    "encoder, byte-checked against the oracle",
            "config": {
                "workload": desc,
                "op": op,
                "messages_per_gpu": n,
                "global_batch": n * world if args.scaling == "weak" else n_cfg,
                "raw_bytes_per_gpu": raw_total,
                "compressed_bytes_per_gpu": comp_total,
                "ratio": round(raw_total / max(1, comp_total), 4),
                "parallelism": f"shard{world} ({args.scaling}: messages by index"
                               f"{', byte-balanced' if args.scaling == 'strong' else ''}; no data-path collective)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": pmc.get("traffic_bytes_per_launch") if pmc else None,
                "algorithmic_bytes_per_launch": algo_bytes,
                "avg_kernel_ms": round(avg_kernel_s * 1e3, 4),
                "read_frac": round((comp_total if op == "decompress" else raw_total) / avg_kernel_s / 1e9
                                   / HBM_PEAK_GBS, 4),
            },
            "cpu_baseline": cpu,
            "end_to_end": e2e,
            "correct": {"status_errors": errors, "roundtrip_ok": roundtrip_ok, "oracle_sample_ok": sample_ok},
            "kernel_src": kernel_source_hash(),
            "decode_lanes": args.decode_lanes,
            "kernels": {"decode": args.decode_kernel, "encode": args.encode_kernel},
            "setup_s": round(gen_s, 2),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


def load_traffic(workload: str):
    p = REPO / "profiles" / f"pmc_{workload}.json"
    if not p.exists():
        return None
    d = json.loads(p.read_text())
    return d if d.get("kernel_src") == kernel_source_hash() else None


def end_to_end(torch, codec, op, batch, d_comp, c_off, comp_len, raw_total, comp_total, n, max_len, dev,
               d_ws):
    """Pinned host -> HBM -> kernel -> pinned host, one pass (reported in DESIGN.md)."""
    stream = torch.cuda.current_stream()
    d_dws = codec.decompress_workspace(n, d_comp.numel())
    if op == "decompress":
        h_in = torch.empty(d_comp.numel(), dtype=torch.uint8, pin_memory=True)
        h_in.copy_(d_comp.cpu())
        h_out = torch.empty(raw_total, dtype=torch.uint8, pin_memory=True)
        d_in = torch.empty_like(d_comp)
        d_out = torch.empty(raw_total, dtype=torch.uint8, device=dev)
        in_bytes, out_bytes = comp_total, raw_total
    else:
        h_in = torch.from_numpy(batch.data).pin_memory()
        h_out = torch.empty(d_comp.numel(), dtype=torch.uint8, pin_memory=True)
        d_in = torch.empty(h_in.numel(), dtype=torch.uint8, device=dev)
        d_out = torch.empty_like(d_comp)
        in_bytes, out_bytes = raw_total, comp_total
    d_off_in = torch.from_numpy(c_off if op == "decompress" else batch.offsets).to(dev)
    d_len_in = torch.from_numpy((comp_len if op == "decompress" else batch.lens).view(np.int32)).to(dev)
    d_off_out = torch.from_numpy(batch.offsets if op == "decompress" else c_off).to(dev)
    d_cap = torch.from_numpy(batch.lens.view(np.int32)).to(dev)
    d_ol = torch.empty(n, dtype=torch.int32, device=dev)
    d_st = torch.empty(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    best = None
    for _ in range(2):
        e = [torch.cuda.Event(enable_timing=True) for _ in range(4)]
        e[0].record(stream)
        d_in.copy_(h_in, non_blocking=True)
        e[1].record(stream)
        if op == "decompress":
            codec.decompress(d_in, d_off_in, d_len_in, n, d_out, d_off_out, d_cap, d_ol, d_st, stream=stream,
                             workspace=d_dws)
        else:
            codec.compress(d_in, d_off_in, d_len_in, n, max_len, d_out, d_off_out, d_ol, d_st, stream=stream,
                           workspace=d_ws)
        e[2].record(stream)
        h_out.copy_(d_out[:h_out.numel()], non_blocking=True)
        e[3].record(stream)
        torch.cuda.synchronize()
        ms = [e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2]), e[2].elapsed_time(e[3])]
        if best is None or sum(ms) < sum(best):
            best = ms
    tot = sum(best) / 1e3
    out = {
        "gib_s_uncompressed": round(raw_total / tot / GIB, 3),
        "h2d_ms": round(best[0], 3), "kernel_ms": round(best[1], 3), "d2h_ms": round(best[2], 3),
        "h2d_gb_s": round(in_bytes / (best[0] / 1e3) / 1e9, 2),
        "d2h_gb_s": round(out_bytes / (best[2] / 1e3) / 1e9, 2),
        "note": "serial pinned hipMemcpyAsync H2D + kernel + D2H on one stream, no overlap",
    }
    if op == "decompress":
        out["pipelined"] = [end_to_end_pipelined(torch, codec, h_in, h_out, d_in, d_out, c_off, comp_len,
                                                 batch, raw_total, n, dev, chunks=c) for c in (4, 16)]
    return out


def end_to_end_pipelined(torch, codec, h_in, h_out, d_in, d_out, c_off, comp_len, batch, raw_total,
                         n, dev, chunks=16):
    """The same pass cut into message-range chunks: chunk k's H2D, decode and
    D2H go to three streams with event dependencies, so chunk k+1's upload and
    chunk k-1's download overlap chunk k's kernels."""
    bounds = [n * k // chunks for k in range(chunks + 1)]
    s_up, s_k, s_down = (torch.cuda.Stream(device=dev) for _ in range(3))
    d_off_in = torch.from_numpy(c_off).to(dev)
    d_len_in = torch.from_numpy(comp_len.view(np.int32)).to(dev)
    d_off_out = torch.from_numpy(batch.offsets).to(dev)
    d_cap = torch.from_numpy(batch.lens.view(np.int32)).to(dev)
    d_ol = torch.empty(n, dtype=torch.int32, device=dev)
    d_st = torch.empty(n, dtype=torch.int32, device=dev)
    c_end = np.append(c_off[1:], np.uint64(d_in.numel())).astype(np.uint64)
    r_end = (batch.offsets.astype(np.uint64) + batch.lens.astype(np.uint64))
    wss = []
    for k in range(chunks):
        a, b = bounds[k], bounds[k + 1]
        wss.append(codec.decompress_workspace(b - a, int(c_end[b - 1] - c_off[a])) if b > a else None)
    torch.cuda.synchronize()
    best = None
    for _ in range(2):
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        t0.record(s_up)
        s_k.wait_event(t0)
        s_down.wait_event(t0)
        for k in range(chunks):
            a, b = bounds[k], bounds[k + 1]
            if b == a:
                continue
            ca, cb = int(c_off[a]), int(c_end[b - 1])
            ra, rb = int(batch.offsets[a]), int(r_end[b - 1])
            with torch.cuda.stream(s_up):
                d_in[ca:cb].copy_(h_in[ca:cb], non_blocking=True)
                up = torch.cuda.Event()
                up.record(s_up)
            s_k.wait_event(up)
            codec.decompress(d_in, d_off_in[a:b], d_len_in[a:b], b - a, d_out, d_off_out[a:b], d_cap[a:b],
                             d_ol[a:b], d_st[a:b], stream=s_k, workspace=wss[k])
            kd = torch.cuda.Event()
            kd.record(s_k)
            s_down.wait_event(kd)
            with torch.cuda.stream(s_down):
                h_out[ra:rb].copy_(d_out[ra:rb], non_blocking=True)
        t1.record(s_down)
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1)
        best = ms if best is None else min(best, ms)
    ok = bool((d_st == 0).all().item())
    return {"gib_s_uncompressed": round(raw_total / (best / 1e3) / GIB, 3), "ms": round(best, 3),
            "chunks": chunks, "status_ok": ok,
            "note": f"{chunks} message-range chunks; H2D / decode / D2H on three streams with event "
                    "dependencies"}


def cpu_baseline(op, batch, d_comp, c_off, comp_len, threads):
    """The reference's own CPU Snappy (oracle/_ref, per-message Source/Sink path with
    8160-byte cord_buf fragments) on a bounded sample of the same workload, timed on
    this host's cores.  Falls back to the C restatement ("port") if _ref is absent."""
    sys.path.insert(0, str(REPO / "oracle"))
    from bind import Oracle, Reference
    nthreads = threads or max(1, min(16, len(os.sched_getaffinity(0))))
    n = len(batch)
    per_msg = batch.total / max(1, n)
    # bounded sample: ~1 GiB of decode work or ~0.25 GiB of encode work per pass
    target = (1 << 30) if op == "decompress" else (1 << 28)
    m = int(max(1, min(n, target // max(1, per_msg))))
    lens = batch.lens[:m].copy()
    offs = batch.offsets[:m].copy()
    host_comp = d_comp[: int(c_off[m - 1] + comp_len[m - 1]) + 1].cpu().numpy()
    clen = comp_len[:m].copy()
    coff = c_off[:m].copy()
    kind = "reference" if Reference.available() else "port"
    eng = Reference() if kind == "reference" else Oracle()
    out_len = np.zeros(m, np.uint32)
    # repeated passes over the sample until ~1 s of wall time (~16 s of CPU
    # work at 16 threads), at most 20 passes
    passes, dt = 0, 0.0
    while passes < 20 and (passes == 0 or dt < 1.0):
        if op == "decompress":
            out = np.zeros(max(1, int(lens.astype(np.uint64).sum())), np.uint8)
            if kind == "reference":
                dt += eng.batch(1, host_comp, coff, clen, out, offs, lens, out_len, nthreads)
            else:
                st = np.zeros(m, np.int32)
                dt += eng.uncompress_batch(host_comp, coff, clen, out, offs, lens, out_len, st, nthreads)
            nraw = int(lens.astype(np.uint64).sum())
            ok = bool(np.array_equal(out[:nraw], batch.data[:nraw]))
        else:
            caps = np.array([fsg.max_compressed_length(int(x)) for x in lens], np.uint64)
            oo, tot = fsg.slot_offsets(caps)
            out = np.zeros(tot, np.uint8)
            if kind == "reference":
                dt += eng.batch(0, batch.data, offs, lens, out, oo, None, out_len, nthreads)
            else:
                dt += eng.compress_batch(batch.data, offs, lens, out, oo, out_len, nthreads)
            ok = bool(np.array_equal(out_len, clen))
        passes += 1
    raw = int(lens.astype(np.uint64).sum()) * passes
    return {
        "value": round(raw / dt / GIB, 3),
        "unit": "GiB/s (uncompressed bytes)",
        "cores": nthreads,
        "kind": kind,
        "sample": f"first {m} messages of the same batch ({raw / passes / GIB:.3f} GiB raw) x {passes} "
                  f"passes, {op}, {nthreads} threads x strided messages, 8160-B fragments; wall {dt:.3f} s "
                  f"(~{dt * nthreads:.0f} s of CPU work); output equal to GPU's: {ok}",
    }


if __name__ == "__main__":
    main()
