"""The N-rank path with the HIP codec on a one-GPU box: bench.py's own
launcher starts two ranks that both run the device codec on cuda:0
(FSG_BENCH_SHARED_DEVICE=0; their collectives go over gloo, since RCCL
refuses two ranks on one device).  Covers the shard split, each rank's
device encode + decode of its shard, the all-gather of per-message
(length, status) and the reassembly checks, with the device path that the
CPU tests (tests/test_distributed.py) replace by the oracle."""
import json
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "flare-cpp_amd" / "py"))
import fsg  # noqa: E402


def _launch(extra):
    argv = ["--gpus", "2", "--steps", "2", "--warmup", "1", "--no-e2e", "--no-cpu-baseline",
            "--no-encode", "--pipeline", "0", "--verify-sample", "8", *extra]
    code = ("import sys; sys.path.insert(0, %r); import bench; "
            "sys.exit(bench.launch(2, %r, env_extra={'FSG_BENCH_SHARED_DEVICE': '0'}, timeout_s=150))"
            % (str(REPO), argv))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=180, cwd=REPO)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints ONE line
    return json.loads(lines[0])


@pytest.mark.gpu
def test_two_ranks_device_codec_weak_c3():
    d = _launch(["--workload", "c3-decompress", "--n-msgs", "512"])
    assert d["n_gpus"] == 2 and d["config"]["world_size_seen_by_collectives"] == 2
    assert d["scaling"] == "weak" and d["config"]["global_batch"] == 1024
    assert d["config"]["raw_bytes_all_ranks"] == 1024 * 65536
    assert d["correct"]["status_errors"] == 0 and d["correct"]["roundtrip_ok"]
    assert d["correct"]["oracle_sample_ok"]
    ag = d["multi_gpu"]["allgather"]
    assert ag["messages"] == 1024 and ag["mismatches"] == 0
    rs = d["multi_gpu"]["root_scatter"]
    assert rs["mismatches"] == 0 and rs["scatter_plus_decode_ms"] > 0


@pytest.mark.gpu
def test_two_ranks_device_codec_strong_mixed():
    d = _launch(["--workload", "cm-decompress", "--n-msgs", "3000", "--no-root-scatter"])
    assert d["n_gpus"] == 2 and d["scaling"] == "strong"
    sizes = fsg.mixed_sizes(3000)
    assert d["config"]["global_batch"] == 3000
    assert d["config"]["raw_bytes_all_ranks"] == int(sizes.astype(np.uint64).sum())
    assert d["correct"]["status_errors"] == 0 and d["correct"]["roundtrip_ok"]
    assert d["multi_gpu"]["allgather"]["messages"] == 3000
    assert d["multi_gpu"]["allgather"]["mismatches"] == 0
