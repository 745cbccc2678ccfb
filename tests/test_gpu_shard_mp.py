"""Process-per-GPU sharded prove: bench.py --shard under torch.distributed.run.

Two ranks share the box's one GPU through the gloo transport (lsp_comm_ops,
host-staged), so this runs the multi-process code path end to end; RCCL
cannot put two ranks on one GPU, so its transport is exercised with a single
rank.  Both proofs must equal the single-GPU proof byte for byte."""
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, nproc, comm, port, log_n=10, schedules=None, env_extra=None, plans=None):
    out = tmp_path / f"proof_{comm}_{nproc}_{log_n}_{port}.bin"
    sched = tmp_path / f"sched_{nproc}_{log_n}_{port}"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", LSP_FRI_SHARD_MIN="16", **(env_extra or {}))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--shard", "--comm", comm, "--device", "0", "--log-n", str(log_n), "--steps", "1",
           "--warmup", "0", "--no-cpu-baseline", "--dump-proof", str(out), "--dump-comm-schedule", str(sched)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    if nproc > 1:  # the per-collective table of the JSON line (lsp_comm_log on every rank)
        import json
        o = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
        assert o["schedule_identical"] is True and len(o["comm_init_ms_by_rank"]) == nproc
        rows = o["collectives"]
        assert rows and all(len(x["ms_by_rank"]) == nproc and x["op"] in ("allgather", "bcast") for x in rows)
        assert "query openings" in {x["tag"] for x in rows}
        if schedules is not None and comm == "gloo":  # the library's log = the transport's own record
            lib_sched = [(x["op"], x["bytes"], x["root"]) for x in rows]
            assert len(lib_sched) >= 5
        # the attach-time calibration and the inverse-NTT exchange it chose (lsp_comm_exchange_plan)
        ex = o["exchange"]
        assert ex["allgather_gbs"] > 0 and ex["intt_gelem_per_s"] > 0 and ex["probe_bytes"] > 0, ex
        assert isinstance(ex["split_intt"], bool)
        assert ("trace coefficients" in {x["tag"] for x in rows}) == ex["split_intt"]
        # every rank's raw probes (the minimum of which the plan used), and the
        # quotient-chunk broadcasts the model prices beside the trace exchange
        assert len(ex["per_rank"]) == nproc and all(r["intt_gelem_per_s"] > 0 and r["allgather_4mib_gbs"] > 0
                                                      for r in ex["per_rank"]), ex
        assert min(r["intt_gelem_per_s"] for r in ex["per_rank"]) == pytest.approx(ex["intt_gelem_per_s"])
        qrows = [x for x in rows if x["tag"] in ("quotient chunk coefficients", "quotient values")]
        assert len(qrows) == ex["quotient_bcasts"] and all(x["bytes"] == ex["quotient_bcast_bytes_each"]
                                                            for x in qrows), (qrows, ex)
        assert ex["model_quotient_bcast_ms"] > 0
        if plans is not None:
            plans.append(ex)
    if schedules is not None and comm == "gloo":
        import json
        for rk in range(nproc):
            schedules.append(json.load(open(f"{sched}.{rk}.json")))
    return out.read_bytes()


def _single(gpu_ctx, log_n=10):
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import gen_permutation_trace
    a, d, _ = gpu_ctx.config.seeded()
    tr = gen_permutation_trace(log_n, 3, a, d)
    return gpu_ctx.prove(tr, permutation_air(3), np.concatenate([a, d]))


def test_two_processes_gloo(gpu_ctx, tmp_path):
    assert _run(tmp_path, 2, "gloo", 29611) == _single(gpu_ctx)


@pytest.mark.parametrize("nproc", [2, 8])
def test_exchange_choice_logged_and_both_paths_identical(gpu_ctx, tmp_path, nproc):
    """every run logs the calibrated allgather bandwidth, the
    inverse-NTT rate and the exchange chosen on them; forcing either exchange
    (LSP_SHARD_SPLIT_INTT=1: split inverse + coefficient allgather, 0:
    redundant inverse) gives the single-GPU proof byte for byte"""
    single = _single(gpu_ctx, 11)
    plans = []
    for k, forced in enumerate(("1", "0")):
        got = _run(tmp_path, nproc, "gloo", 29650 + 10 * nproc + k, 11, env_extra={"LSP_SHARD_SPLIT_INTT": forced},
                   plans=plans)
        assert got == single
    assert [p["split_intt"] for p in plans] == [True, False]
    auto = []
    assert _run(tmp_path, nproc, "gloo", 29680 + nproc, 11, plans=auto) == single
    # over gloo (host-staged, a few GB/s) the model prefers the redundant inverse
    assert auto[0]["model_allgather_ms"] > 0 and auto[0]["model_redundant_intt_ms"] > 0
    assert auto[0]["split_intt"] == (auto[0]["model_allgather_ms"] < auto[0]["model_redundant_intt_ms"])


def test_four_processes_gloo(gpu_ctx, tmp_path):
    assert _run(tmp_path, 4, "gloo", 29612) == _single(gpu_ctx)


@pytest.mark.parametrize("log_n", [10, 12])
def test_eight_processes_gloo(gpu_ctx, tmp_path, log_n):
    """BASELINE configs[3]'s rank count (8 processes, here all on the box's one
    GPU over gloo): the proof equals the single-GPU proof byte for byte, and
    every rank issued the same collectives in the same order with the same
    sizes and roots -- what a collective transport (RCCL) needs not to hang."""
    scheds = []
    assert _run(tmp_path, 8, "gloo", 29614 + log_n, log_n, scheds) == _single(gpu_ctx, log_n)
    assert [s["rank"] for s in scheds] == list(range(8)) and all(s["world"] == 8 for s in scheds)
    ref = scheds[0]["schedule"]
    assert len(ref) >= 5 and {op for op, _, _ in ref} == {"allgather", "bcast"}
    for s in scheds[1:]:
        assert s["schedule"] == ref, f"rank {s['rank']} issued a different collective schedule"


def test_rccl_transport_single_rank(gpu_ctx, tmp_path):
    """RCCL loads (dlopen), initialises and carries the sharded prove's
    collectives; one rank because RCCL needs a GPU per rank"""
    assert _run(tmp_path, 1, "rccl", 29613) == _single(gpu_ctx)


def _bench_json(args, timeout=420):
    import json
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    return lines[0]


def test_bench_gpus2_shard_spawns_ranks():
    """bench.py --gpus 2 started without a launcher runs two
    ranks (here both on the box's one GPU over gloo) and reports n_gpus 2"""
    o = _bench_json(["--gpus", "2", "--shard", "--comm", "gloo", "--log-n", "12", "--steps", "1", "--warmup", "1",
                     "--no-cpu-baseline", "--shard-leg", "none", "--batch-leg", "none"])
    assert o["n_gpus"] == 2 and o["n_ranks_seen"] == 2 and o["verified"] is True
    assert o["scaling"] == "strong"


def test_bench_sharded_leg_two_ranks():
    """the C4 'sharded' field: one device-generated trace proved by two ranks
    (gloo, sharing one GPU) verifies; the replicas value beside it is weak scaling"""
    o = _bench_json(["--gpus", "2", "--log-n", "10", "--steps", "1", "--warmup", "1", "--no-cpu-baseline",
                     "--shard-leg", "12,13", "--shard-leg-steps", "1", "--shard-leg-warmup", "0",
                     "--batch-leg", "11", "--batch-leg-steps", "1", "--shape-pow-bits", "0"])
    assert o["n_gpus"] == 2 and o["scaling"] == "weak" and o["verified"] is True
    b = o["batch"]["runs"][0]  # configs[4]'s shape: one independent proof per rank
    assert b["log_n"] == 11 and b["verified"] is True and b["scaling"] == "weak"
    sh = o["sharded"]
    assert sh["comm"] == "gloo" and sh["n_ranks_seen"] == 2, sh
    assert [r["log_n"] for r in sh["runs"]] == [12, 13]
    assert all(r["verified"] for r in sh["runs"])
    for r in sh["runs"]:  # every collective, per rank, with its device time
        assert r["schedule_identical"] is True and len(r["comm_init_ms_by_rank"]) == 2
        assert r["collectives"] and all(len(x["ms_by_rank"]) == 2 for x in r["collectives"])
        assert ("trace coefficients" in r["collectives_by_tag"]) == r["exchange"]["split_intt"]


def test_bench_sharded_leg_single_gpu_equals_prove():
    """N = 1: the sharded field is lsp_prove itself (prove_shard over SoloComm),
    and the device-generated trace proves and verifies"""
    o = _bench_json(["--log-n", "10", "--steps", "1", "--warmup", "1", "--no-cpu-baseline", "--inflight", "0",
                     "--shape-pow-bits", "0",
                     "--shard-leg", "14", "--shard-leg-steps", "2", "--batch-leg", "none"])
    sh = o["sharded"]
    assert sh["comm"] == "solo" and sh["n_ranks_seen"] == 1
    assert sh["runs"][0]["verified"] is True
    assert o["prove_time_host_trace_s"]["median"] > 0
