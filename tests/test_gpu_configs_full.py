"""BASELINE configs[3] and configs[4] at their full per-rank sizes on the
box's one GPU (VERDICT r3 "Next round" item 1).

configs[3] -- the 3x3 permutation AIR at 2^26 rows over 8 MI355X.  Ranks 0,
5 and 7 each run in a fresh child process (tools/rank_rehearsal.py) as rank
g of an 8-rank lsp_prove_sharded under the loopback transport
(lsp_ctx_attach_loopback: the peers' parts of each exchange fabricated
locally).  Each rank must fit the 288 GB of an MI355X, produce a proof whose
wire size is the real 2^26 proof's (proof.wire_size), refuse to hand the
rehearsal proof out as bytes, and -- what RCCL needs not to hang on the
first real 8-GPU run -- issue exactly the same collective schedule (op,
bytes, root, in order) as every other rank: the 2 GiB trace-coefficient
allgather, the 1 GiB quotient broadcasts, the FRI-slice switch and the query
allgather included.

configs[4] -- 8 independent 2^22 proofs, one per GPU.  Two replica ranks run
bench.py's batch leg at 2^22 under torch.distributed.run, both on the box's
one GPU; each rank's proof verifies and equals a single-context proof of its
rank seed.
"""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

LOG_N, G = 26, 8
_REHEARSALS = {}


def _rehearse(rank):
    """rank `rank` of configs[3], once per session (a child process each)"""
    if rank not in _REHEARSALS:
        cmd = [sys.executable, os.path.join(ROOT, "tools", "rank_rehearsal.py"), "--log-n", str(LOG_N), "--size",
               str(G), "--ranks", str(rank), "--steps", "1"]
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=280, cwd=ROOT,
                           env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        out = json.loads(r.stdout.strip().splitlines()[-1])
        print(json.dumps({k: v for k, v in out.items() if k != "comm_log"}))
        _REHEARSALS[rank] = out
    return _REHEARSALS[rank]


def _schedule(out):
    return [(e["op"], e["bytes"], e["root"]) for e in out["comm_log"]]


@pytest.mark.parametrize("rank", [0, 7])
def test_configs3_rank_fits_and_has_the_real_proof_shape(rank):
    from linea_stark_prover_amd.proof import wire_size
    out = _rehearse(rank)
    assert out["log_n"] == LOG_N and out["size"] == G and out["rank"] == rank
    assert out["fits_288gb"] and out["device_used_bytes"] < 288e9, out["device_used_gib"]
    assert out["proof_wire_bytes"] == wire_size(LOG_N, 8, 2), out["proof_wire_bytes"]
    assert out["rehearsal_bytes_refused"], "a loopback (rehearsal) proof must not serialize"
    tags = {e["tag"] for e in out["comm_log"]}
    assert {"trace coefficients", "trace subtree roots", "quotient chunk coefficients", "quotient subtree roots",
            "opened values", "FRI subtree roots", "FRI vector", "query openings"} <= tags, tags
    big = [e for e in out["comm_log"] if e["tag"] == "trace coefficients"]
    assert len(big) == 1 and big[0]["op"] == "allgather" and big[0]["bytes"] == (1 << LOG_N) * 1 * 32  # 8 cols / 8 ranks
    assert all(e["ms"] >= 0 for e in out["comm_log"])


def test_configs3_collective_schedule_is_rank_invariant():
    ref = _schedule(_rehearse(0))
    assert len(ref) > 20
    for rank in (5, 7):
        assert _schedule(_rehearse(rank)) == ref, f"rank {rank} issues a different collective schedule"


def test_wire_size_matches_real_proofs(gpu_ctx):
    """the size the rehearsal is checked against, on real proofs (3x3 and 6x6 AIRs)"""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.proof import wire_size
    from linea_stark_prover_amd.prover import gen_permutation_trace
    a, d, _ = gpu_ctx.config.seeded()
    for log_n, ncols, log_q in ((9, 3, 2), (12, 3, 2), (10, 6, 3)):
        proof = gpu_ctx.prove(gen_permutation_trace(log_n, ncols, a, d), permutation_air(ncols), np.concatenate([a, d]))
        assert len(proof) == wire_size(log_n, 2 * ncols + 2, log_q)


def test_configs4_two_replica_ranks_at_2e22(gpu_ctx, tmp_path):
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.replicas import rank_seed
    prefix = tmp_path / "batch"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", "29631", os.path.join(ROOT, "bench.py"), "--gpus", "2", "--device", "0",
           "--log-n", "10", "--steps", "1", "--warmup", "0", "--no-cpu-baseline", "--shard-leg", "none",
           "--batch-leg", "22", "--batch-leg-steps", "1", "--dump-batch-proofs", str(prefix)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=280, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    o = json.loads([x for x in r.stdout.splitlines() if x.startswith("{")][-1])
    run = o["batch"]["runs"][0]
    assert run["log_n"] == 22 and run["scaling"] == "weak" and run["verified_ranks"] == 2
    cfg = gpu_ctx.config
    a, d, _ = cfg.seeded()
    pub = np.concatenate([a, d])
    air = permutation_air(3)
    h, w = 1 << 22, 8
    for rank in range(2):
        got = (tmp_path / f"batch.{rank}.22.bin").read_bytes()
        dtrace = gpu_ctx.gen_permutation_trace_device(22, 3, a, d, seed=rank_seed(cfg.seed, rank))
        try:
            expect = gpu_ctx.prove(dtrace, air, pub, h, w)
        finally:
            gpu_ctx.dev_free(dtrace)
        assert got == expect, f"rank {rank}'s replica proof differs from a single-context proof of its seed"
        assert gpu_ctx.verify(got, air, pub)
