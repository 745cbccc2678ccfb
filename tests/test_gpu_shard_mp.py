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


def _run(tmp_path, nproc, comm, port, log_n=10):
    out = tmp_path / f"proof_{comm}_{nproc}.bin"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", LSP_FRI_SHARD_MIN="16")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "bench.py"),
           "--shard", "--comm", comm, "--device", "0", "--log-n", str(log_n), "--steps", "1", "--warmup", "0",
           "--no-cpu-baseline", "--dump-proof", str(out)]
    r = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return out.read_bytes()


def _single(gpu_ctx, log_n=10):
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import gen_permutation_trace
    a, d, _ = gpu_ctx.config.seeded()
    tr = gen_permutation_trace(log_n, 3, a, d)
    return gpu_ctx.prove(tr, permutation_air(3), np.concatenate([a, d]))


def test_two_processes_gloo(gpu_ctx, tmp_path):
    assert _run(tmp_path, 2, "gloo", 29611) == _single(gpu_ctx)


def test_four_processes_gloo(gpu_ctx, tmp_path):
    assert _run(tmp_path, 4, "gloo", 29612) == _single(gpu_ctx)


def test_rccl_transport_single_rank(gpu_ctx, tmp_path):
    """RCCL loads (dlopen), initialises and carries the sharded prove's
    collectives; one rank because RCCL needs a GPU per rank"""
    assert _run(tmp_path, 1, "rccl", 29613) == _single(gpu_ctx)
