"""TEST INFRASTRUCTURE ONLY: one rank of bench.py on the CPU (gloo), with the
oracle standing in for the HIP codec.  Started by bench.launch() from
tests/test_distributed.py, exactly as bench.py --gpus N starts its ranks."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
for p in (REPO, REPO / "flare-cpp_amd" / "py", REPO / "oracle", REPO / "tests"):
    sys.path.insert(0, str(p))

import bench  # noqa: E402
from oracle_codec import OracleCodec  # noqa: E402

if __name__ == "__main__":
    args = bench.parse(sys.argv[1:])
    assert args.device == "cpu", "the oracle stand-in runs on CPU tensors only"
    bench.rank_main(args, codec_factory=lambda local: OracleCodec())
