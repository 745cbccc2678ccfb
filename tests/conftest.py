import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through liblsp_hip.so on the device)")
    config.addinivalue_line("markers", "slow: larger sizes")


# Long oracle proofs started in the background as soon as their tests are
# selected (tests/oracle_job.py: one process, the jobs in this order), so they
# overlap the rest of the suite: test name -> (log_n, ncols).
# LSP_ORACLE_PRESTART=0 computes them inline instead.
ORACLE_JOBS = {"test_benchlog_shape_whole_proof_2e19_vs_oracle": (19, 6),
               "test_configs1_whole_proof_2e22_vs_oracle": (22, 3)}
ORACLE_THREADS = min(16, os.cpu_count() or 1)  # the GPU box's CPU share (os.cpu_count() shows the whole machine)
_job = {}  # "proc", "err" (stderr file), "out": test name -> proof path


@pytest.hookimpl(trylast=True)  # after -m / -k deselection: only tests that will run
def pytest_collection_modifyitems(session, config, items):
    if os.environ.get("LSP_ORACLE_PRESTART", "1") == "0" or config.getoption("collectonly") or _job:
        return
    import subprocess
    import tempfile
    # the tests that wait for the background oracle proofs run last, so the rest
    # of the suite runs while the oracle computes (its 2^22 proof is ~5 min of
    # the box's 16 threads); in collection order they waited ~95 s
    waiting = [it for it in items if it.name in ORACLE_JOBS]
    if waiting:
        items[:] = [it for it in items if it.name not in ORACLE_JOBS] + waiting
    names = {item.name for item in items}
    sel = [(n, j) for n, j in ORACLE_JOBS.items() if n in names]
    if not sel:
        return
    tmp = tempfile.mkdtemp(prefix="lsp_oracle_")
    out = {n: os.path.join(tmp, f"{n}.bin") for n, _ in sel}
    err = open(os.path.join(tmp, "stderr.txt"), "w+b")
    env = dict(os.environ, OMP_NUM_THREADS=str(ORACLE_THREADS))
    cmd = [sys.executable, os.path.join(ROOT, "tests", "oracle_job.py"), str(ORACLE_THREADS)]
    cmd += [f"{out[n]}:{log_n}:{ncols}" for n, (log_n, ncols) in sel]
    _job.update(proc=subprocess.Popen(cmd, env=env, stdout=subprocess.DEVNULL, stderr=err), err=err, out=out)


def pytest_sessionfinish(session, exitstatus):
    proc = _job.get("proc")
    if proc is not None and proc.poll() is None:
        proc.kill()
        proc.wait()


def oracle_job_result(name, timeout=1800):
    """The background job's proof bytes for test `name` (waits for them), or
    None when no job was started for it (LSP_ORACLE_PRESTART=0, or the test
    was run some other way)."""
    import time
    if name not in _job.get("out", {}):
        return None
    proc, out = _job["proc"], _job["out"][name]
    t0 = time.time()
    while not os.path.exists(out):
        if proc.poll() is not None and not os.path.exists(out):
            _job["err"].seek(0)
            tail = _job["err"].read().decode(errors="replace")[-2000:]
            raise RuntimeError(f"oracle job for {name} ended without it (rc {proc.returncode}): {tail}")
        if time.time() - t0 > timeout:
            proc.kill()
            raise TimeoutError(f"oracle job for {name}: no proof after {timeout} s")
        time.sleep(0.2)
    with open(out, "rb") as f:
        return f.read()


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
