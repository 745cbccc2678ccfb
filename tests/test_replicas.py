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
                       "trace_head": [int(x) for x in tr[0, 0]],
                       "host_threads": os.environ.get("LSP_HOST_THREADS"),
                       "cpus": len(os.sched_getaffinity(0))}}), flush=True)
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
    # both ranks share this process's affinity set: each takes half of it (init_from_env)
    assert [int(o["host_threads"]) for o in outs] == [max(1, min(16, o["cpus"] // 2)) for o in outs]
    assert outs[0]["elapsed"] >= 0.12
    # independent replicas: distinct traces per rank
    assert outs[0]["trace_head"] != outs[1]["trace_head"]


def test_single_process_default(product_lib):
    sys.path.insert(0, ROOT)
    from linea_stark_prover_amd.replicas import Dist, timed_steps
    el, out = timed_steps(lambda: 7, 2, 1, Dist())
    assert out == 7 and el >= 0


def _bench(args, env_extra=None, timeout=240):
    env = dict(os.environ, **(env_extra or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        if not env_extra or k not in env_extra:
            env.pop(k, None)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                          text=True, timeout=timeout, cwd=ROOT)


def test_gpus_2_without_launcher_spawns_two_ranks():
    """bench.py --gpus 2 started bare runs torch.distributed.run with two ranks
    (never one rank reported as two GPUs); --dry-run stops before any GPU work"""
    import json
    r = _bench(["--gpus", "2", "--dry-run"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    assert lines[0]["n_gpus"] == 2 and lines[0]["n_ranks_seen"] == 2
    assert lines[0]["launcher"] == "torch.distributed.run"


def test_world_size_mismatch_is_an_error():
    import json
    r = _bench(["--gpus", "4", "--dry-run"], {"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode == 2
    assert "refusing" in json.loads(r.stdout.strip().splitlines()[-1])["error"]


def test_hung_sharded_leg_exits_nonzero():
    """bench.py's sharded-leg watchdog: a leg that never returns (a hung
    collective) still gets the main line printed, with the error noted, and the
    process exits with a non-zero status -- a driver reading the exit code sees
    the hang (round-2 review item 6)."""
    import json
    code = textwrap.dedent(f"""
        import sys, time, types
        sys.path.insert(0, {ROOT!r})
        sys.argv = ["bench.py"]
        import bench
        args = types.SimpleNamespace(shard_timeout=1.0)
        dist = types.SimpleNamespace(rank=0)
        out = {{"metric": "m", "value": 1.0}}
        bench.guarded_shard_leg(args, dist, None, [24], out, leg=lambda *a: time.sleep(60))
        print("not reached")
    """)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=120, cwd=ROOT)
    sys.path.insert(0, ROOT)
    import bench
    assert r.returncode == bench.WATCHDOG_EXIT != 0, (r.returncode, r.stderr[-2000:])
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert "exceeded" in line["sharded"]["error"] and line["value"] == 1.0
    assert "not reached" not in r.stdout


def test_bench_helpers():
    """frmul count of the trace LDE and the stamp check of PMC profiles"""
    sys.path.insert(0, ROOT)
    import bench
    # 2^19 x 8 into 8 cosets: (2^18 * 19 + 8 * 2^19 + 8 * 2^18 * 19) * 8 products (~0.39 G)
    assert bench.lde_products(1 << 19, 8, 8) == 8 * ((1 << 18) * 19 + 8 * (1 << 19) + 8 * (1 << 18) * 19)
    assert abs(bench.FRMUL_PEAK_GPS - 307.2) < 1e-9
    assert len(bench.LIB_SRC) == 16
    # a profile from another build is never used: null plus the reason
    bench.lde_traffic(5, 3)
    assert bench.TRAFFIC_SRC[(5, 3)].startswith("null")


def test_host_pool_split_follows_affinity(tmp_path, product_lib):
    """init_from_env sizes each rank's host pool from the ranks that share its
    CPU set: ranks pinned to disjoint sets keep their own (no division), ranks
    on one set split it"""
    import json
    cpus = sorted(os.sched_getaffinity(0))
    if len(cpus) < 4:
        pytest.skip("needs 4 CPUs")
    half = len(cpus) // 2
    worker = textwrap.dedent(f"""
        import os, sys, json
        sys.path.insert(0, {ROOT!r})
        r = int(os.environ["RANK"])
        cpus = {cpus!r}
        os.sched_setaffinity(0, cpus[:{half}] if r == 0 else cpus[{half}:])
        from linea_stark_prover_amd.replicas import init_from_env
        d = init_from_env()
        print(json.dumps({{"rank": d.rank, "threads": int(os.environ["LSP_HOST_THREADS"]),
                           "cpus": len(os.sched_getaffinity(0))}}), flush=True)
        d.close()
    """)
    script = tmp_path / "pin.py"
    script.write_text(worker)
    port = _free_port()
    procs = [subprocess.Popen([sys.executable, str(script)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                              env=dict(os.environ, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE="2",
                                       MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port)))
             for r in range(2)]
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e
        outs.append(json.loads(o.strip().splitlines()[-1]))
    for o in outs:  # disjoint sets: each rank's own, undivided
        assert o["threads"] == min(16, o["cpus"]), o


def test_host_pool_mixed_override_does_not_hang(tmp_path, product_lib):
    """a rank with its own LSP_HOST_THREADS still joins the control
    group's all_gather, so ranks without it do not block; its override wins"""
    import json
    worker = textwrap.dedent(f"""
        import os, sys, json
        sys.path.insert(0, {ROOT!r})
        from linea_stark_prover_amd.replicas import init_from_env
        d = init_from_env()
        print(json.dumps({{"rank": d.rank, "threads": int(os.environ["LSP_HOST_THREADS"])}}), flush=True)
        d.close()
    """)
    script = tmp_path / "mixed.py"
    script.write_text(worker)
    port = _free_port()
    base = {k: v for k, v in os.environ.items() if k != "LSP_HOST_THREADS"}
    procs = []
    for r in range(2):
        env = dict(base, WORLD_SIZE="2", RANK=str(r), LOCAL_RANK=str(r), LOCAL_WORLD_SIZE="2",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if r == 1:
            env["LSP_HOST_THREADS"] = "3"
        procs.append(subprocess.Popen([sys.executable, str(script)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                                      text=True, env=env))
    outs = []
    for p in procs:
        o, e = p.communicate(timeout=240)
        assert p.returncode == 0, e
        outs.append(json.loads(o.strip().splitlines()[-1]))
    outs.sort(key=lambda o: o["rank"])
    assert outs[1]["threads"] == 3
    assert 1 <= outs[0]["threads"] <= 16


def test_clock_sampler_without_a_gpu(product_lib):
    """bench.py's box-speed stamp never fails the bench: with no GPU (or no
    amdsmi device) the sampler says why and reports None, and start/stop are
    harmless; the summary of given samples is their mean / min / max"""
    sys.path.insert(0, ROOT)
    import bench
    s = bench.ClockSampler(0, period=0.001)
    assert s.handle is None and s.status != "ok"
    assert s.start().stop() is None
    s.samples = [(2100.0, 2000.0, 900.0), (2300.0, None, 1100.0), (None, None, None)]
    got = s.summary()
    assert got["sclk_mhz_mean"] == 2200.0 and got["sclk_mhz_min"] == 2100.0 and got["sclk_mhz_max"] == 2300.0
    assert got["avg_gfxclk_mhz_mean"] == 2000.0 and got["socket_power_w_mean"] == 1000.0 and got["samples"] == 2


def test_host_compress_rate(product_lib):
    """the host half of the box-speed stamp runs on a host-only context"""
    sys.path.insert(0, ROOT)
    import bench
    from linea_stark_prover_amd.prover import Context, StarkConfig
    with Context(StarkConfig(), device=-1) as ctx:
        assert bench.host_compress_rate(ctx, n=64, reps=2) > 0
