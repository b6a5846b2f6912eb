import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs on the GPU box via gpurun)")
    # A/B builds (tools/build_variant.sh -> abv/libgcow_NAME.so) are checked with the same tests before they are timed
    lib = os.environ.get("GCOW_TEST_LIB")
    if lib:
        from gcow_amd import _ffi
        _ffi.LIB_PATH = os.path.abspath(lib)
    config.addinivalue_line("markers", "slow: large-size property tests")


@pytest.fixture(scope="session")
def orc():
    from oracle import oracle as O
    O.build()
    return O
