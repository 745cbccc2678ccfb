"""The N > 1 control plane of bench.py on CPU: world_size-2 gloo, barrier +
max-over-ranks timing, distinct per-rank traces (no GPU needed)."""
import os
import socket
import subprocess
import sys
import textwrap

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

WORKER = textwrap.dedent("""
    import os, sys, time, json
    sys.path.insert(0, {root!r})
    from linea_stark_prover_amd.replicas import init_from_env, rank_seed, timed_steps
    d = init_from_env()
    import numpy as np
    from linea_stark_prover_amd.prover import StarkConfig, gen_permutation_trace
    cfg = StarkConfig()
    a, dl, _ = cfg.seeded()
    tr = gen_permutation_trace(6, 3, a, dl, seed=rank_seed(cfg.seed, d.rank))
    # rank r sleeps (r+1)*20 ms per step: the reported time must be the slowest rank's
    el, _ = timed_steps(lambda: time.sleep(0.02 * (d.rank + 1)), 3, 1, d)
    print(json.dumps({{"rank": d.rank, "world": d.world, "elapsed": el,
                       "trace_head": [int(x) for x in tr[0, 0]]}}), flush=True)
    d.close()
""")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_gloo_replicas(tmp_path, product_lib):
    script = tmp_path / "worker.py"
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
        import json
        outs.append(json.loads(o.strip().splitlines()[-1]))
    outs.sort(key=lambda x: x["rank"])
    assert [o["world"] for o in outs] == [2, 2]
    # max over ranks: both report the same elapsed, at least the slow rank's 3 x 40 ms
    assert abs(outs[0]["elapsed"] - outs[1]["elapsed"]) < 1e-9
    assert outs[0]["elapsed"] >= 0.12
    # independent replicas: distinct traces per rank
    assert outs[0]["trace_head"] != outs[1]["trace_head"]


def test_single_process_default(product_lib):
    sys.path.insert(0, ROOT)
    from linea_stark_prover_amd.replicas import Dist, timed_steps
    el, out = timed_steps(lambda: 7, 2, 1, Dist())
    assert out == 7 and el >= 0
