import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblsp_hip.so on the device)")
    config.addinivalue_line("markers", "slow: larger sizes")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import cref
    cref.build()
    return cref


@pytest.fixture(scope="session")
def product_lib():
    from linea_stark_prover_amd import build as B
    if not os.path.exists(B.LIB):
        B.build()
    from linea_stark_prover_amd import _lib
    return _lib.lib()


@pytest.fixture(scope="session")
def gpu_ctx(product_lib):
    from linea_stark_prover_amd.prover import Context, StarkConfig
    ctx = Context(StarkConfig())
    yield ctx
    ctx.close()
