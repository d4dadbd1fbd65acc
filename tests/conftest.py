import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C ABI)")
    config.addinivalue_line("markers", "slow: full-size (GiB) configurations")
    # build the native pieces once if a fresh checkout lacks them (hipcc cross-compiles without a GPU)
    need = [os.path.join(ROOT, "tools", "libfcxgen.so"), os.path.join(ROOT, "oracle", "liboracle.so"),
            os.path.join(ROOT, "my_compress_amd", "lib", "libfcx.so")]
    if not all(os.path.exists(p) for p in need):
        import __graft_entry__

        __graft_entry__.build()


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(ROOT, "tests", "golden", "golden.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def cuda():
    import torch

    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")
