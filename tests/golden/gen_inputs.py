"""Deterministic inputs behind the golden vectors (shared by make_golden.py and
the tests, so fixtures store only specs + expected outputs)."""
from __future__ import annotations

import random
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parents[1] / "flare-cpp_amd" / "py"))
import fsg  # noqa: E402


def _pattern(n: int, digits: bool) -> bytes:
    """test/rpc/rpc_snappy_compress_test.cc text loops: a..z then 0..9."""
    out = bytearray()
    while len(out) < n:
        for i in range(26):
            if len(out) < n:
                out.append(97 + i)
        if digits:
            for i in range(10):
                if len(out) < n:
                    out.append(48 + i)
    return bytes(out)


def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while v >= 128:
        out.append((v & 127) | 128)
        v >>= 7
    out.append(v)
    return bytes(out)


def snappy_message_proto(text: bytes, numbers) -> bytes:
    """SnappyMessageProto (test/snappy_message.proto:21-24) in proto2 wire format:
    field 1 string (LEN), field 2 repeated int32 (unpacked varints)."""
    out = b"\x0a" + _varint(len(text)) + text
    for x in numbers:
        out += b"\x10" + _varint(x if x >= 0 else x + (1 << 64))
    return out


def _rand_bytes(seed: int, n: int) -> bytes:
    r = random.Random(seed)
    return bytes(r.getrandbits(8) for _ in range(n))


def build_input(spec: dict) -> bytes:
    g = spec["gen"]
    n = spec.get("size", 0)
    if g == "literal":
        return bytes.fromhex(spec["hex"])
    if g == "text":
        return fsg.make_batch(fsg.KIND_TEXT, [n], first_index=spec["seed"]).item(0)
    if g == "random":
        return fsg.make_batch(fsg.KIND_RANDOM, [n], first_index=spec["seed"]).item(0)
    if g == "run":
        return bytes([spec.get("byte", 0x61)]) * n
    if g == "period":
        unit = _rand_bytes(spec["seed"], spec["period"])
        return (unit * (n // spec["period"] + 1))[:n]
    if g == "pattern":
        return _pattern(n, spec.get("digits", True))
    if g == "proto_pattern":
        return snappy_message_proto(_pattern(n, True), spec["numbers"])
    if g == "proto_text":
        return snappy_message_proto(spec["text"].encode(), spec["numbers"])
    if g == "far_match":
        # chunk C, `gap` random bytes, C again: one copy at offset len(C)+gap
        c = _rand_bytes(spec["seed"], spec["chunk"])
        gap = _rand_bytes(spec["seed"] + 1, spec["gap"])
        return c + gap + c + _rand_bytes(spec["seed"] + 2, spec.get("tail", 20))
    raise ValueError(g)


def positive_specs() -> list[dict]:
    specs = [
        # reference test inputs (rpc_snappy_compress_test.cc)
        {"name": "ref_snappy_hello", "gen": "proto_text", "text": "Hello World!", "numbers": [2, 7, 45]},
        {"name": "ref_snappy_iobuf", "gen": "literal", "hex": b"this is a test".hex()},
        {"name": "ref_mass_snappy", "gen": "proto_pattern", "size": 12435, "numbers": [2, 7, 45]},
        {"name": "ref_snappy_test_200", "gen": "pattern", "size": 200, "digits": True},
        {"name": "ref_snappy_test_123456", "gen": "literal", "hex": b"123456".hex()},
        {"name": "ref_mass_snappy_iobuf_782", "gen": "pattern", "size": 782, "digits": False},
    ]
    for s in (128, 1024, 16 * 1024, 32 * 1024, 512 * 1024):  # throughput_compare sizes
        specs.append({"name": f"ref_throughput_pattern_{s}", "gen": "proto_pattern", "size": s, "numbers": []})
    sizes = [0, 1, 2, 3, 4, 5, 14, 15, 16, 17, 31, 32, 33, 63, 64, 65, 255, 256, 257, 1023, 1024, 1025,
             4095, 4096, 4097, 8191, 8192, 8193, 16383, 16384, 16385, 32768, 65535, 65536, 65537,
             131071, 131072, 131073, 1 << 20]
    for s in sizes:
        specs.append({"name": f"text_{s}", "gen": "text", "seed": s, "size": s})
        specs.append({"name": f"random_{s}", "gen": "random", "seed": s, "size": s})
        if s <= 65537 or s == 1 << 20:
            specs.append({"name": f"run_{s}", "gen": "run", "size": s, "byte": 0x61})
    for p in range(2, 9):
        for s in (17, 100, 1000, 70000):
            specs.append({"name": f"period{p}_{s}", "gen": "period", "seed": p, "period": p, "size": s})
    for chunk in (64, 65, 66, 67, 68, 69, 127, 128, 200, 1000):
        specs.append({"name": f"long_match_{chunk}", "gen": "far_match", "seed": chunk, "chunk": chunk, "gap": 50})
    for gap in (1990, 2047, 2048, 2100, 30000, 65000, 65400, 65470):
        specs.append({"name": f"far_match_gap{gap}", "gen": "far_match", "seed": gap, "chunk": 40, "gap": gap})
    return specs


def negative_cases(ref) -> list[tuple[str, bytes]]:
    """Hand-made and fuzzed decode inputs; verdicts come from the reference."""
    cases = [
        ("empty", b""),
        ("header_only_zero", b"\x00"),
        ("header_truncated", b"\x80"),
        ("header_truncated2", b"\xff\xff"),
        ("header_lenient_5th_byte", b"\xff\xff\xff\xff\x1f"),
        ("header_5th_cont", b"\xff\xff\xff\xff\x8f\x01"),
        ("header_max_strict_ok", b"\xff\xff\xff\xff\x0f"),
        ("ulen_mismatch_short", b"\x05\x08abc"),
        ("ulen_mismatch_long", b"\x02\x08abc"),
        ("trailing_literal", b"\x03\x08abc\x00z"),
        ("truncated_literal", b"\x05\x10ab"),
        ("offset_zero", b"\x08\x0cabcd\x01\x00"),
        ("offset_beyond", b"\x08\x0cabcd\x01\x05"),
        ("offset_equal_produced", b"\x08\x0cabcd\x01\x04"),
        ("copy_overrun", b"\x06\x0cabcd\x05\x04"),
        ("copy_overlap_rle_bad_len", b"\x0c\x00a\x19\x01"),
        ("copy_overlap_rle", b"\x0b\x00a\x19\x01"),
        ("copy_overlap_period3", b"\x13\x08abc\x3e\x03\x00"),
        ("copy2_truncated", b"\x08\x0cabcd\x0e\x04"),
        ("copy4_truncated", b"\x08\x0cabcd\x0f\x04\x00\x00"),
        ("copy4_ok", b"\x08\x0cabcd\x0f\x04\x00\x00\x00"),
        ("literal_len1_trunc", b"\x40\xf0"),
        ("literal_len4_trunc", b"\x40\xfc\x01\x02"),
        ("literal_len_wrap_zero", b"\x01\xfc\xff\xff\xff\xff\x00a"),
        ("literal_huge", b"\x01\xfc\x00\x00\x00\x80\x00a"),
        ("literal_61", b"\x3d" + b"\xf0\x3c" + bytes(range(61))),
    ]
    # 4-byte literal lengths 0xfffffffa..0xfffffffe: tag position + 5 + length
    # wraps back to 0..4 bytes past the tag, so a u32 walk lands on its own
    # length bytes (0xff = a COPY_4 of 64) and the wrapped op can look sane.
    for val in range(0xFFFFFFFA, 0xFFFFFFFF):
        body = b"\x24" + b"0123456789" + b"\xfc" + val.to_bytes(4, "little") + b"\x01\x00\x00\x00"
        for ulen in (73, 74, 10):
            cases.append((f"literal_len_wrap_{val:08x}_u{ulen}", _varint(ulen) + body))
    # COPY_4 crossing a 64 KiB block (accepted by the reference decoder): a
    # 70000-byte literal then a COPY_4 with offset 69000 of length 64.
    lit = _rand_bytes(99, 70000)
    body = bytes([0xf8]) + (70000 - 1).to_bytes(3, "little") + lit
    body += bytes([3 | ((64 - 1) << 2)]) + (69000).to_bytes(4, "little")
    cases.append(("copy4_cross_block", _varint(70064) + body))
    # COPY_2 reaching back across a block boundary (offset 65535)
    lit2 = _rand_bytes(98, 66000)
    body2 = bytes([0xf8]) + (66000 - 1).to_bytes(3, "little") + lit2
    body2 += bytes([2 | ((20 - 1) << 2)]) + (65535).to_bytes(2, "little")
    cases.append(("copy2_cross_block_65535", _varint(66020) + body2))
    # fuzz: mutate valid streams
    rng = random.Random(2024)
    srcs = [build_input({"gen": "text", "seed": s, "size": s}) for s in (30, 300, 3000)]
    srcs.append(build_input({"gen": "period", "seed": 3, "period": 3, "size": 500}))
    for i in range(160):
        c = bytearray(ref.compress(rng.choice(srcs)))
        op = i % 4
        if op == 0:
            c = c[: rng.randrange(len(c))]
        elif op == 1:
            for _ in range(rng.randint(1, 3)):
                c[rng.randrange(len(c))] = rng.randrange(256)
        elif op == 2:
            c += bytes(rng.randrange(256) for _ in range(rng.randint(1, 5)))
        else:
            c[rng.randrange(1, len(c))] = rng.choice([0xfc, 0xf8, 0xf4, 0xf0, 0x03, 0x02, 0x01, 0xff, 0x00])
        cases.append((f"fuzz_{i}", bytes(c)))
    return cases
