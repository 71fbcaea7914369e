"""The host C++ drop-in (cord_buf, CompressHandler registry, GPU-backed
policy::SnappyCompress/SnappyDecompress, flat flare::snappy API, cross-call
batcher), exercised by tests/cpp/test_rpc_snappy_compress.cc -- the reference's
rpc_snappy_compress_test.cc cases re-run against the GPU handler."""
import os
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
BIN = REPO / "build" / "test_rpc_snappy_compress"


def _binary():
    if not BIN.exists():
        subprocess.run(["make", "-C", str(REPO), "cpptests"], check=True, capture_output=True)
    return BIN


def test_host_layer_cpu_cases():
    r = subprocess.run([str(_binary()), "--cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("chunk_bytes", [None, "4096"])
def test_host_layer_gpu_cases(chunk_bytes):
    """chunk_bytes 4096 cuts every batch into many chunks, so the host runtime's
    pipeline (gather / H2D / kernels / D2H / scatter over three streams) runs."""
    env = dict(os.environ)
    if chunk_bytes:
        env["FLARE_SNAPPY_GPU_CHUNK_BYTES"] = chunk_bytes
    r = subprocess.run([str(_binary()), "--gpu"], capture_output=True, text=True, timeout=600, env=env)
    print(r.stdout)
    print(r.stderr[-3000:])
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 failures" in r.stdout


ECHO = REPO / "build" / "echo_bench"


@pytest.mark.parametrize("codec", ["runtime", "none"])
def test_echo_loopback_cpu(codec):
    """Config 1's harness (tools/echo_bench.cc): baidu_std echo over loopback,
    SNAPPY request and response, a 4,096-byte body; every echo comes back intact."""
    if not ECHO.exists():
        subprocess.run(["make", "-C", str(REPO), "echobench"], check=True, capture_output=True)
    r = subprocess.run([str(ECHO), "--codec", codec, "--calls", "300", "--warmup", "20"], capture_output=True,
                       text=True, timeout=120, cwd=str(REPO))
    assert r.returncode == 0, r.stdout + r.stderr
    import json
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["errors"] == 0 and d["server_ok"] and d["body_bytes"] == 4096 and d["qps"] > 0


@pytest.mark.gpu
def test_echo_loopback_gpu():
    """The same echo with every body sent through the GPU (threshold 0)."""
    if not ECHO.exists():
        subprocess.run(["make", "-C", str(REPO), "echobench"], check=True, capture_output=True)
    r = subprocess.run([str(ECHO), "--codec", "gpu", "--calls", "300", "--warmup", "20"], capture_output=True,
                       text=True, timeout=120, cwd=str(REPO))
    assert r.returncode == 0, r.stdout + r.stderr
    import json
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["errors"] == 0 and d["server_ok"] and d["gpu_messages"] == 4 * 320
