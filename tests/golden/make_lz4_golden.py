"""Generates tests/golden/lz4_vectors.json from the image's system liblz4
(1.9.3, LZ4_compress_default / LZ4_decompress_safe) -- the pin of the LZ4
path, since the reference ships no LZ4 code (parity vs the reference:
unpinned; vs liblz4: pinned here).

  python tests/golden/make_lz4_golden.py

Inputs: the Snappy golden vectors' input recipes (gen_inputs.build_input,
171 specs: texts, random bytes, patterns, protos, 0 B .. 1 MiB) plus inputs at
the 64 KiB table-switch boundary and runs long enough for multi-byte length
extensions.  Decode cases: blocks of those inputs with bytes flipped or cut,
and lengths off by a few, with liblz4's verdict (an offset-0 match, which
liblz4 accepts and this repo rejects, is flagged and excluded from the
comparison).
"""
import json
import random
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE))
sys.path.insert(0, str(HERE.parent))
sys.path.insert(0, str(HERE.parents[1] / "flare-cpp_amd" / "py"))
import fsg  # noqa: E402
from gen_inputs import build_input  # noqa: E402
from lz4_sys import SysLz4, load  # noqa: E402
from lz4_walk import first_violation  # noqa: E402


def main():
    L = load()
    if L is None:
        raise SystemExit("liblz4 not found")
    z = SysLz4(L)
    keys = ("name", "gen", "seed", "size", "hex", "text", "numbers", "digits", "byte", "period", "chunk", "gap",
            "tail")
    specs = [{k: v[k] for k in v if k in keys} for v in json.loads((HERE / "vectors.json").read_text())]
    extra = [
        {"name": "lz4_text_65546", "gen": "text", "seed": 7, "size": 65546},
        {"name": "lz4_text_65547", "gen": "text", "seed": 7, "size": 65547},
        {"name": "lz4_text_200000", "gen": "text", "seed": 8, "size": 200000},
        {"name": "lz4_random_65547", "gen": "random", "seed": 9, "size": 65547},
        {"name": "lz4_zeros_70000", "gen": "literal", "hex": "00" * 70000},
        {"name": "lz4_zeros_300", "gen": "literal", "hex": "00" * 300},
        {"name": "lz4_ab_20000", "gen": "literal", "hex": "6162" * 10000},
    ]
    vecs, rng = [], random.Random(44)
    for spec in specs + extra:
        try:
            x = build_input(spec)
        except Exception as e:  # a recipe this generator does not know
            raise SystemExit(f"{spec['name']}: {e}")
        blk = z.compress(x)
        n, y = z.decompress(blk, len(x))
        assert n == len(x) and y == x
        v = dict(spec, input_len=len(x), input_fnv="%016x" % fsg.fnv1a64(x), block_len=len(blk),
                 block_fnv="%016x" % fsg.fnv1a64(blk))
        if len(blk) <= 256:
            v["block_hex"] = blk.hex()
        vecs.append(v)
    decode = []
    small = [build_input(s) for s in specs if 20 <= (s.get("size") or 0) <= 3000][:40]
    for i in range(600):
        x = small[i % len(small)]
        b = bytearray(z.compress(x))
        for _ in range(rng.randint(1, 2)):
            b[rng.randrange(len(b))] = rng.randrange(256)
        if rng.random() < 0.3:
            b = b[:rng.randint(1, len(b))]
        ulen = len(x) if rng.random() < 0.8 else max(0, len(x) + rng.randint(-20, 20))
        b = bytes(b)
        n, y = z.decompress(b, ulen)
        decode.append({"hex": b.hex(), "ulen": ulen, "liblz4_ok": n == ulen,
                       "output_fnv": "%016x" % fsg.fnv1a64(y) if n == ulen else None,
                       "offset0": first_violation(b, ulen) == "offset 0"})
    out = {"liblz4_version": z.version, "compress": vecs, "decode": decode}
    (HERE / "lz4_vectors.json").write_text(json.dumps(out, indent=0) + "\n")
    print(len(vecs), "compress vectors,", len(decode), "decode cases,",
          sum(d["liblz4_ok"] for d in decode), "accepted by liblz4")


if __name__ == "__main__":
    main()
