"""Multi-GPU path on CPU: world_size-2 `gloo` runs of the sharding and the
measurement collectives bench.py uses (the GPU runs use RCCL with the same
code).  Each rank encodes/decodes its shard with the ORACLE standing in for the
device (this test checks the distribution logic, not the codec), and the
ranks' results must reassemble the single-process answer exactly."""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import fsg
import shard


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_byte_balanced_ranges_cover_and_balance():
    sizes = fsg.mixed_sizes(20000)
    for world in (1, 2, 4, 8):
        rs = shard.byte_balanced_ranges(sizes, world)
        assert rs[0][0] == 0 and rs[-1][1] == len(sizes)
        assert all(rs[i][1] == rs[i + 1][0] for i in range(world - 1))
        per = [int(sizes[lo:hi].astype(np.uint64).sum()) for lo, hi in rs]
        assert max(per) - min(per) <= int(sizes.max())  # within one body of perfect
    assert shard.weak_range(65536, 3) == (3 * 65536, 4 * 65536)


def _worker(rank, world, port, sizes, out_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from bind import Oracle
    o = Oracle()
    lo, hi = shard.byte_balanced_ranges(sizes, world)[rank]
    b = fsg.make_batch(fsg.KIND_MIXED, sizes[lo:hi], first_index=lo)
    comp = [o.compress(b.item(i)) for i in range(len(b))]
    ok = all(o.uncompress(c)[2] == b.item(i) for i, c in enumerate(comp))
    t_step, t_kern, (raw, cb, errs, bad) = shard.reduce_measurements(
        dist, "cpu", 0.1 * (rank + 1), 0.05 * (rank + 1), b.total, sum(map(len, comp)), 0, int(not ok))
    digest = [fsg.fnv1a64(c) for c in comp]
    gathered = [None] * world
    dist.all_gather_object(gathered, (lo, digest))
    if rank == 0:
        out_q.put((t_step, t_kern, raw, cb, errs, bad, gathered))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_shards_reassemble():
    sizes = fsg.mixed_sizes(3000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, sizes, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    t_step, t_kern, raw, cb, errs, bad, gathered = res
    assert t_step == pytest.approx(0.2) and t_kern == pytest.approx(0.1)  # MAX over ranks
    assert raw == int(sizes.astype(np.uint64).sum()) and bad == 0 and errs == 0
    # concatenated per-rank digests == single-process digests
    from bind import Oracle
    o = Oracle()
    b = fsg.make_batch(fsg.KIND_MIXED, sizes)
    whole = [fsg.fnv1a64(o.compress(b.item(i))) for i in range(len(b))]
    merged = [d for lo, ds in sorted(gathered) for d in ds]
    assert merged == whole
    assert cb == sum(len(o.compress(b.item(i))) for i in range(len(b)))


def _run_bench_launcher(nprocs, extra):
    """bench.py's own launcher (bench.launch) starting CPU ranks whose codec is
    the oracle (tests/bench_cpu_rank.py); returns rank 0's JSON line."""
    import json
    import subprocess
    import sys
    from pathlib import Path
    repo = Path(__file__).resolve().parents[1]
    argv = ["--device", "cpu", "--gpus", str(nprocs), "--steps", "2", "--warmup", "1", "--no-e2e",
            "--no-cpu-baseline", "--verify-sample", "4", *extra]
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch(%d, %r, entry=%r, timeout_s=240))"
            % (str(repo), nprocs, argv, str(repo / "tests" / "bench_cpu_rank.py")))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300, cwd=repo)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints ONE line
    return json.loads(lines[0])


def test_bench_launcher_two_ranks_weak():
    d = _run_bench_launcher(2, ["--workload", "c3-decompress", "--n-msgs", "48"])
    assert d["n_gpus"] == 2 and d["config"]["world_size_seen_by_collectives"] == 2
    assert d["scaling"] == "weak" and d["config"]["global_batch"] == 96
    assert d["config"]["raw_bytes_all_ranks"] == 96 * 65536
    assert d["correct"]["status_errors"] == 0 and d["correct"]["roundtrip_ok"]
    assert d["correct"]["oracle_sample_ok"]
    ag = d["multi_gpu"]["allgather"]
    assert ag["messages"] == 96 and ag["mismatches"] == 0
    rs = d["multi_gpu"]["root_scatter"]
    assert rs["mismatches"] == 0 and rs["scatter_plus_decode_ms"] > 0


def test_bench_launcher_two_ranks_strong_mixed():
    d = _run_bench_launcher(2, ["--workload", "cm-decompress", "--n-msgs", "600"])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    assert d["config"]["global_batch"] == 600
    sizes = fsg.mixed_sizes(600)
    assert d["config"]["raw_bytes_all_ranks"] == int(sizes.astype(np.uint64).sum())
    assert d["correct"]["status_errors"] == 0 and d["correct"]["roundtrip_ok"]
    assert d["multi_gpu"]["allgather"]["messages"] == 600
    assert d["multi_gpu"]["allgather"]["mismatches"] == 0
    assert d["multi_gpu"]["root_scatter"]["mismatches"] == 0
