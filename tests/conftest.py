import sys
from pathlib import Path

import pytest

REPO = Path(__file__).resolve().parents[1]
for p in (REPO / "flare-cpp_amd" / "py", REPO / "oracle", REPO / "tests" / "golden", REPO):
    if str(p) not in sys.path:
        sys.path.insert(0, str(p))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


@pytest.fixture
def fsg_opts():
    """Setter for the codec library's process-wide options (fsg_set_option,
    include/flare_snappy_gpu.h); every option it touched is restored after the
    test.  Usage: fsg_opts(decode_fork=1, small_persist=1792)."""
    import fsg
    saved = {}

    def setopt(**kv):
        for k, v in kv.items():
            if k not in saved:
                saved[k] = fsg.get_option(k)
            fsg.set_option(k, int(v))

    yield setopt
    for k, v in saved.items():
        fsg.set_option(k, v)
