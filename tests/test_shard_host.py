"""Host side of the process-per-GPU sharded prove (no GPU): the gloo
transport behind lsp_comm_ops on a world_size-2 group, and the C-ABI's
argument / state checks."""
import os
import socket
import subprocess
import sys
import textwrap

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import ctypes, json, os, sys
    sys.path.insert(0, {root!r})
    from linea_stark_prover_amd.replicas import init_from_env
    d = init_from_env()
    import numpy as np
    from linea_stark_prover_amd.shard import GlooComm
    c = GlooComm()
    n = 37
    mine = (np.arange(n, dtype=np.uint8) * 3 + 11 * (c.rank + 1)).astype(np.uint8)
    recv = np.zeros(n * c.size, np.uint8)
    # through the ctypes callback objects, as the C side calls them
    rc1 = c.ops.allgather(None, mine.ctypes.data, recv.ctypes.data, n)
    buf = mine.copy() if c.rank == 1 else np.zeros(n, np.uint8)
    rc2 = c.ops.bcast(None, buf.ctypes.data, n, 1)
    print(json.dumps({{"rank": c.rank, "rc": [rc1, rc2], "recv": recv.tolist(), "bcast": buf.tolist(),
                      "schedule": c.schedule}}), flush=True)
    d.close()
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_gloo_comm_ops_two_ranks(tmp_path, product_lib):
    import json
    script = tmp_path / "w.py"
    script.write_text(WORKER.format(root=ROOT))
    port = _free_port()
    procs = []
    for r in range(2):
        env = dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(script)], env=env, stdout=subprocess.PIPE,
                                      stderr=subprocess.PIPE, text=True))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e
        outs.append(json.loads(o.strip().splitlines()[-1]))
    outs.sort(key=lambda x: x["rank"])
    n = 37
    exp = np.concatenate([(np.arange(n) * 3 + 11 * (r + 1)) % 256 for r in range(2)]).tolist()
    for o in outs:
        assert o["rc"] == [0, 0]
        assert o["recv"] == exp
        assert o["bcast"] == exp[n:]  # rank 1's pattern on every rank
        # the communicator records what it carried, in order (the 8-process GPU
        # test compares these schedules across ranks)
        assert o["schedule"] == [["allgather", n, None], ["bcast", n, 1]]


@pytest.fixture
def host_ctx(product_lib):
    from linea_stark_prover_amd.prover import Context, StarkConfig
    return Context(StarkConfig(), device=-1)


def test_prove_sharded_needs_a_communicator(host_ctx):
    from linea_stark_prover_amd import _lib
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.shard import prove_sharded
    tr = np.zeros((8, 8, 4), np.uint64)
    with pytest.raises(_lib.LspError, match="no communicator"):
        prove_sharded(host_ctx, tr, permutation_air(3), np.zeros((2, 4), np.uint64))


def test_comm_ops_argument_checks(host_ctx):
    import ctypes
    from linea_stark_prover_amd import _lib as L
    ag = L.ALLGATHER_FN(lambda *a: 0)
    bc = L.BCAST_FN(lambda *a: 0)
    bad = L.LspCommOps(2, 2, None, ag, bc)  # rank outside [0, size)
    assert L.lib().lsp_ctx_attach_comm_ops(host_ctx.h, ctypes.byref(bad)) == L.LSP_E_ARG
    ok = L.LspCommOps(0, 1, None, ag, bc)
    assert L.lib().lsp_ctx_attach_comm_ops(host_ctx.h, ctypes.byref(ok)) == L.LSP_OK
    # the self-test needs the GPU the host-only context does not have
    assert L.lib().lsp_comm_selftest(host_ctx.h) == L.LSP_E_STATE
    assert L.lib().lsp_ctx_detach_comm(host_ctx.h) == L.LSP_OK


def test_group_needs_gpu_contexts(host_ctx):
    from linea_stark_prover_amd import _lib
    from linea_stark_prover_amd.prover import ProverGroup
    with pytest.raises(_lib.LspError, match="GPU context"):
        ProverGroup([host_ctx, host_ctx])


def test_loopback_attach_and_mem_stats_checks(host_ctx):
    """the rehearsal transport (lsp_ctx_attach_loopback) takes any rank of any
    size without a peer; memory stats need the GPU a host-only context lacks"""
    import ctypes
    from linea_stark_prover_amd import _lib as L
    assert L.lib().lsp_ctx_attach_loopback(host_ctx.h, 8, 8) == L.LSP_E_ARG
    assert L.lib().lsp_ctx_attach_loopback(host_ctx.h, 7, 8) == L.LSP_OK
    r, n = ctypes.c_int(), ctypes.c_int()
    assert L.lib().lsp_comm_info(host_ctx.h, ctypes.byref(r), ctypes.byref(n)) == L.LSP_OK
    assert (r.value, n.value) == (7, 8)
    a, b, c = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
    assert L.lib().lsp_ctx_mem_stats(host_ctx.h, ctypes.byref(a), ctypes.byref(b), ctypes.byref(c)) == L.LSP_E_STATE
    assert L.lib().lsp_ctx_detach_comm(host_ctx.h) == L.LSP_OK


def test_exchange_plan_uncalibrated_and_forced(host_ctx, monkeypatch):
    """lsp_comm_exchange_plan: a communicator never self-tested (here the
    loopback rehearsal transport, which calibration skips) plans the split
    inverse; LSP_SHARD_SPLIT_INTT forces either exchange, read per proof"""
    from linea_stark_prover_amd import _lib
    _lib.check(_lib.lib().lsp_ctx_attach_loopback(host_ctx.h, 0, 8), host_ctx.h)
    p = host_ctx.exchange_plan(1 << 26, 8)
    assert p["split_intt"] is True and p["allgather_gbs"] == 0 and p["model_allgather_ms"] == 0
    monkeypatch.setenv("LSP_SHARD_SPLIT_INTT", "0")
    assert host_ctx.exchange_plan(1 << 26, 8)["split_intt"] is False
    monkeypatch.setenv("LSP_SHARD_SPLIT_INTT", "1")
    assert host_ctx.exchange_plan(1 << 26, 8)["split_intt"] is True
    _lib.check(_lib.lib().lsp_ctx_detach_comm(host_ctx.h), host_ctx.h)
    with pytest.raises(_lib.LspError):
        host_ctx.exchange_plan(1 << 20, 8)  # no communicator


_POOL_CHILD = """
import os, sys
sys.path.insert(0, {root!r})
cpus = {cpus!r}
if cpus:
    os.sched_setaffinity(0, set(sorted(os.sched_getaffinity(0))[:cpus]))
from linea_stark_prover_amd.prover import Context, StarkConfig
print(Context(StarkConfig(), device=-1).host_threads())
"""


@pytest.mark.parametrize("env,cpus,expect", [
    ({"LSP_HOST_THREADS": "3"}, 0, lambda n: 3),
    ({"LOCAL_WORLD_SIZE": "1"}, 0, lambda n: min(16, n)),
    # the process's set is divided among the local ranks
    ({"LOCAL_WORLD_SIZE": "4"}, 0, lambda n: max(1, min(16, n // 4))),
    # a small set several ranks may share (8 ranks on a 2-CPU cpuset) is divided too:
    # never ranks x pool threads on a few CPUs; a launcher that pinned this slice for one rank
    # says so with LSP_HOST_THREADS (replicas.init_from_env does)
    ({"LOCAL_WORLD_SIZE": "8"}, 2, lambda n: 1),
    ({"LOCAL_WORLD_SIZE": "8", "LSP_HOST_THREADS": "2"}, 2, lambda n: 2),
])
def test_host_pool_size(product_lib, env, cpus, expect):
    """the host pool divides the process's CPU set among the
    LOCAL_WORLD_SIZE ranks (the library cannot tell a shared set from a pinned
    slice, and dividing is the safe mistake); LSP_HOST_THREADS overrides"""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    machine = len(os.sched_getaffinity(0))
    if cpus and cpus >= machine:
        pytest.skip("needs more CPUs than the slice")
    e = {k: v for k, v in os.environ.items() if k not in ("LSP_HOST_THREADS", "LOCAL_WORLD_SIZE")}
    e.update(env)
    out = subprocess.run([sys.executable, "-c", _POOL_CHILD.format(root=root, cpus=cpus)], env=e,
                         capture_output=True, text=True, timeout=120)
    assert out.returncode == 0, out.stderr[-2000:]
    assert int(out.stdout.strip().splitlines()[-1]) == expect(machine)
