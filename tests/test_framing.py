"""baidu_std framing and rpc_dump capture.

The host layer serializes RpcMeta / RpcDumpMeta by hand (flare-cpp_amd/host/
pb_wire.h, baidu_rpc_meta.cc).  These tests pin that wire format against an
independent proto2 implementation -- the pure-Python protobuf runtime, with
the messages declared from the reference's .proto field tables
(flare/rpc/policy/baidu_rpc_meta.proto:26-50, flare/rpc/options.proto:38-80,
flare/rpc/streaming_rpc_meta.proto:24-28, flare/rpc/rpc_dump.proto:23-45) --
in both directions:
  * the C++ binary writes its fixtures (--emit); Python parses them and
    re-serializes: fields and bytes must match;
  * Python writes messages (incl. unknown fields, reordered and repeated
    fields, closed-enum out-of-range values); the C++ binary parses them
    (--parse-meta / --parse-dump-meta) and must report the same fields.
The C++ binary's own --cpu cases (header bytes, parse errors, attachment
split, dump files) run here too; --gpu cases run on the MI355X.
"""
import json
import os
import struct
import subprocess
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
BIN = REPO / "build" / "test_baidu_std"

pb = pytest.importorskip("google.protobuf")
from google.protobuf import descriptor_pb2, descriptor_pool, message_factory  # noqa: E402

F = descriptor_pb2.FieldDescriptorProto


def _binary():
    if not BIN.exists():
        subprocess.run(["make", "-C", str(REPO), "cpptests"], check=True, capture_output=True)
    return BIN


def _pool():
    fd = descriptor_pb2.FileDescriptorProto(name="framing_test.proto", package="t", syntax="proto2")
    enum = fd.enum_type.add(name="CompressType")
    for i, n in enumerate(["NONE", "SNAPPY", "GZIP", "ZLIB", "LZ4"]):
        enum.value.add(name="COMPRESS_TYPE_" + n, number=i)
    penum = fd.enum_type.add(name="ProtocolType")
    for i in range(27):
        penum.value.add(name="PROTOCOL_%d" % i, number=i)

    def msg(name, fields):
        m = fd.message_type.add(name=name)
        for num, fname, ftype, label, tname in fields:
            f = m.field.add(name=fname, number=num, type=ftype, label=label)
            if tname:
                f.type_name = ".t." + tname
        return m

    O, R = F.LABEL_OPTIONAL, F.LABEL_REQUIRED
    msg("ChunkInfo", [(1, "stream_id", F.TYPE_INT64, R, None), (2, "chunk_id", F.TYPE_INT64, R, None)])
    msg("StreamSettings", [(1, "stream_id", F.TYPE_INT64, R, None),
                           (2, "need_feedback", F.TYPE_BOOL, O, None),
                           (3, "writable", F.TYPE_BOOL, O, None)])
    msg("RpcRequestMeta", [(1, "service_name", F.TYPE_STRING, R, None),
                           (2, "method_name", F.TYPE_STRING, R, None),
                           (3, "log_id", F.TYPE_INT64, O, None),
                           (4, "trace_id", F.TYPE_INT64, O, None),
                           (5, "span_id", F.TYPE_INT64, O, None),
                           (6, "parent_span_id", F.TYPE_INT64, O, None),
                           (7, "request_id", F.TYPE_STRING, O, None)])
    msg("RpcResponseMeta", [(1, "error_code", F.TYPE_INT32, O, None),
                            (2, "error_text", F.TYPE_STRING, O, None)])
    msg("RpcMeta", [(1, "request", F.TYPE_MESSAGE, O, "RpcRequestMeta"),
                    (2, "response", F.TYPE_MESSAGE, O, "RpcResponseMeta"),
                    (3, "compress_type", F.TYPE_INT32, O, None),
                    (4, "correlation_id", F.TYPE_INT64, O, None),
                    (5, "attachment_size", F.TYPE_INT32, O, None),
                    (6, "chunk_info", F.TYPE_MESSAGE, O, "ChunkInfo"),
                    (7, "authentication_data", F.TYPE_BYTES, O, None),
                    (8, "stream_settings", F.TYPE_MESSAGE, O, "StreamSettings")])
    dm = msg("RpcDumpMeta", [(1, "service_name", F.TYPE_STRING, O, None),
                             (2, "method_name", F.TYPE_STRING, O, None),
                             (3, "method_index", F.TYPE_INT32, O, None),
                             (6, "attachment_size", F.TYPE_INT32, O, None),
                             (7, "authentication_data", F.TYPE_BYTES, O, None),
                             (8, "user_data", F.TYPE_BYTES, O, None)])
    dm.field.add(name="compress_type", number=4, type=F.TYPE_ENUM, label=O, type_name=".t.CompressType")
    dm.field.add(name="protocol_type", number=5, type=F.TYPE_ENUM, label=O, type_name=".t.ProtocolType")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(fd)
    return pool


POOL = _pool()
RpcMeta = message_factory.GetMessageClass(POOL.FindMessageTypeByName("t.RpcMeta"))
RpcDumpMeta = message_factory.GetMessageClass(POOL.FindMessageTypeByName("t.RpcDumpMeta"))

BYTES_FIELDS = {"service_name", "method_name", "request_id", "error_text", "authentication_data",
                "user_data"}


def _as_json(m):
    """The C++ binary's JSON rendering: set fields only, strings as hex."""
    out = {}
    for fd, v in m.ListFields():
        if fd.type == F.TYPE_MESSAGE:
            out[fd.name] = _as_json(v)
        elif fd.name in BYTES_FIELDS:
            out[fd.name] = (v.encode() if isinstance(v, str) else v).hex()
        else:
            out[fd.name] = v
    return out


# The C++ meta_cases() / dump_meta_cases(), restated.
def _meta_cases():
    a = RpcMeta()
    a.request.service_name = "example.EchoService"
    a.request.method_name = "Echo"
    a.request.log_id = 123456789012345
    a.compress_type = 1
    a.correlation_id = 42
    a.attachment_size = 5
    b = RpcMeta()
    b.response.error_code = 1003
    b.response.error_text = "Fail to parse request message, CompressType=snappy"
    b.correlation_id = -7
    b.compress_type = 1
    c = RpcMeta()
    c.request.service_name = ""
    c.request.method_name = "M"
    c.request.log_id = -1
    c.request.trace_id = 1 << 62
    c.request.span_id = 0
    c.request.parent_span_id = -(1 << 40)
    c.request.request_id = "x-request-id"
    c.response.error_code = -1
    c.compress_type = -2
    c.correlation_id = 9223372036854775807
    c.attachment_size = 0
    c.chunk_info.stream_id = 3
    c.chunk_info.chunk_id = 4
    c.authentication_data = b"\x00\xff\x80token"
    c.stream_settings.stream_id = 77
    c.stream_settings.need_feedback = True
    c.stream_settings.writable = False
    return [a, b, c, RpcMeta()]


def _dump_meta_cases():
    a = RpcDumpMeta(service_name="example.EchoService", method_name="Echo", compress_type=1,
                    protocol_type=1, attachment_size=3, authentication_data=b"auth")
    b = RpcDumpMeta(method_index=-3, compress_type=0, protocol_type=3, user_data=b"\x01\x00\x02")
    return [a, b]


@pytest.fixture(scope="module")
def emitted(tmp_path_factory):
    d = tmp_path_factory.mktemp("emit")
    r = subprocess.run([str(_binary()), "--emit", str(d)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    return d


def test_cpp_meta_bytes_equal_protobuf(emitted):
    for i, want in enumerate(_meta_cases()):
        raw = (emitted / f"meta_{i}.bin").read_bytes()
        assert raw == want.SerializeToString(), i  # byte-identical serialization
        got = RpcMeta()
        got.ParseFromString(raw)
        assert got == want and got.IsInitialized()


def test_cpp_dump_meta_bytes_equal_protobuf(emitted):
    for i, want in enumerate(_dump_meta_cases()):
        raw = (emitted / f"dump_meta_{i}.bin").read_bytes()
        assert raw == want.SerializeToString(), i
        got = RpcDumpMeta()
        got.ParseFromString(raw)
        assert got == want


def test_cpp_request_frame_layout(emitted):
    raw = (emitted / "request_frame.bin").read_bytes()
    assert raw[:4] == b"PRPC"
    body_size, meta_size = struct.unpack(">II", raw[4:12])
    assert len(raw) == 12 + body_size
    meta = RpcMeta()
    meta.ParseFromString(raw[12:12 + meta_size])
    assert meta.request.service_name == "example.EchoService"
    assert meta.request.method_name == "Echo"
    assert meta.correlation_id == 5 and meta.compress_type == 0
    assert meta.attachment_size == 3
    assert raw[12 + meta_size:] == b"payload-bytes" + b"ATT"


def _cpp_parse(tmp_path, raw, dump=False):
    f = tmp_path / "in.bin"
    f.write_bytes(raw)
    r = subprocess.run([str(_binary()), "--parse-dump-meta" if dump else "--parse-meta", str(f)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    out = r.stdout.strip()
    return None if out == "PARSE_FAIL" else json.loads(out)


def test_protobuf_bytes_parse_in_cpp(tmp_path):
    for m in _meta_cases():
        assert _cpp_parse(tmp_path, m.SerializeToString()) == _as_json(m)
    for m in _dump_meta_cases():
        assert _cpp_parse(tmp_path, m.SerializeToString(), dump=True) == _as_json(m)


def test_unknown_reordered_repeated_fields(tmp_path):
    m = _meta_cases()[0]
    # unknown fields of every wire type, fields in reverse order, a repeated
    # scalar (last wins) and a sub-message split in two (merged)
    unknown = bytes([0x48, 0x05, 0x52, 0x02]) + b"hi" + bytes([0x5D, 1, 2, 3, 4, 0x61]) + bytes(8)
    req = m.request.SerializeToString()
    cut = 2 + len(m.request.service_name)  # after field 1
    parts = [b"\x28\x05", b"\x20\x2a", b"\x18\x07", b"\x18\x01",
             b"\x0a" + bytes([cut]) + req[:cut],
             b"\x0a" + bytes([len(req) - cut]) + req[cut:]]
    raw = unknown + b"".join(parts)
    want = RpcMeta()
    want.ParseFromString(raw)
    assert want.compress_type == 1 and want.request.log_id == m.request.log_id
    assert _cpp_parse(tmp_path, raw) == _as_json(want)


def test_required_fields_and_malformed(tmp_path):
    m = RpcMeta()
    m.request.service_name = "S"  # method_name missing
    raw = m.SerializePartialToString()
    partial = RpcMeta()
    partial.ParseFromString(raw)
    assert not partial.IsInitialized()  # ParsePbFromCordBuf would fail it
    assert _cpp_parse(tmp_path, raw) is None
    good = _meta_cases()[0].SerializeToString()
    assert _cpp_parse(tmp_path, good[:-1]) is None  # truncated


def test_closed_enum_out_of_range(tmp_path):
    # compress_type 7 is not a CompressType: protobuf keeps it out of the field
    raw = b"\x20\x07\x28\x01"
    want = RpcDumpMeta()
    want.ParseFromString(raw)
    assert not want.HasField("compress_type") and want.protocol_type == 1
    assert _cpp_parse(tmp_path, raw, dump=True) == _as_json(want)


def test_framing_cpu_cases():
    r = subprocess.run([str(_binary()), "--cpu"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failures" in r.stdout


@pytest.mark.gpu
@pytest.mark.parametrize("chunk_bytes", [None, "4096"])
def test_framing_gpu_cases(chunk_bytes):
    env = dict(os.environ)
    if chunk_bytes:  # many chunks: the host runtime's multi-stream pipeline
        env["FLARE_SNAPPY_GPU_CHUNK_BYTES"] = chunk_bytes
    r = subprocess.run([str(_binary()), "--gpu"], capture_output=True, text=True, timeout=600, env=env)
    print(r.stdout)
    assert r.returncode == 0, r.stdout + r.stderr
    assert " 0 failures" in r.stdout
