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


@pytest.fixture
def heartbeat(request):
    """heartbeat(label): a context manager for a long silent stretch (an oracle
    proof of minutes): every 30 s it prints a progress line past pytest's
    capture and appends it to gpurun_out/heartbeat.log (on the GPU box), so a
    runner that kills silent commands does not take it for a hang."""
    import contextlib
    import threading
    import time

    cap = request.config.pluginmanager.getplugin("capturemanager")
    out_dir = os.path.join(ROOT, "gpurun_out") if os.environ.get("GRAFT_REPO_ROOT") else None

    @contextlib.contextmanager
    def run(label):
        stop = threading.Event()
        t0 = time.time()

        def beat():
            while not stop.wait(30):
                line = f"[heartbeat] {request.node.name}: {label}, {time.time() - t0:.0f} s"
                if cap is not None:
                    with cap.global_and_fixture_disabled():
                        print(line, file=sys.stderr, flush=True)
                if out_dir:
                    os.makedirs(out_dir, exist_ok=True)
                    with open(os.path.join(out_dir, "heartbeat.log"), "a") as f:
                        f.write(line + "\n")

        th = threading.Thread(target=beat, daemon=True)
        th.start()
        try:
            yield
        finally:
            stop.set()
            th.join()
    return run


@pytest.fixture(scope="session")
def gpu_ctx(product_lib):
    from linea_stark_prover_amd.prover import Context, StarkConfig
    ctx = Context(StarkConfig())
    yield ctx
    ctx.close()
