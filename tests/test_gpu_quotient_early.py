"""Constraints before alpha (csrc/prove.cpp, round 4): the constraint values
are evaluated on a side stream beside the trace tree's narrow levels and
folded with alpha afterwards (k_quotient<true> + k_quotient_fold).  Both
paths must give the oracle's proof byte for byte: LSP_QUOTIENT_EARLY=1 forces
the early path (also on shapes the default leaves on one kernel), =0 the one
kernel after alpha."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _oracle_perm(oracle_lib, logn, ncols):
    p = oracle_lib.setup()
    tb, w = oracle_lib.gen_perm_trace(p, logn, ncols)
    trace = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << logn, w, 4).copy()
    pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
    return p, trace, w, pub


@pytest.mark.parametrize("mode", ["1", "0"])
@pytest.mark.parametrize("logn,ncols", [(1, 3), (4, 3), (9, 6), (12, 3), (16, 3)])
def test_perm_air_both_paths_match_oracle(gpu_ctx, oracle_lib, monkeypatch, mode, logn, ncols):
    from linea_stark_prover_amd.air import permutation_air
    monkeypatch.setenv("LSP_QUOTIENT_EARLY", mode)
    p, trace, w, pub = _oracle_perm(oracle_lib, logn, ncols)
    got = gpu_ctx.prove(trace, permutation_air(ncols), pub)
    assert got == oracle_lib.prove(p, trace.ctypes.data, 1 << logn, w, oracle_lib.perm_air(ncols))


def test_default_path_repeated_proofs(gpu_ctx, oracle_lib, monkeypatch):
    """the default (early at this size) several times on one context: the side
    stream's buffers are reused proof after proof"""
    from linea_stark_prover_amd.air import permutation_air
    monkeypatch.delenv("LSP_QUOTIENT_EARLY", raising=False)
    p, trace, w, pub = _oracle_perm(oracle_lib, 14, 3)
    exp = oracle_lib.prove(p, trace.ctypes.data, 1 << 14, w, oracle_lib.perm_air(3))
    for _ in range(3):
        assert gpu_ctx.prove(trace, permutation_air(3), pub) == exp


@pytest.mark.parametrize("log_n,shape", [(5, (4, 3, 2, 8, 6)), (9, (2, 3, 2, 3, 6))])
def test_wide_air_forced_early_matches_oracle(gpu_ctx, oracle_lib, monkeypatch, log_n, shape):
    """lookup + permutation configs: every constraint of the interpreter written and folded"""
    from linea_stark_prover_amd.prover import gen_wide_trace
    monkeypatch.setenv("LSP_QUOTIENT_EARLY", "1")
    a, d, _ = gpu_ctx.config.seeded()
    tr, air = gen_wide_trace(log_n, a, d, *shape)
    pub = np.concatenate([a, d])
    got = gpu_ctx.prove(tr, air, pub)
    p = oracle_lib.setup()
    assert got == oracle_lib.prove(p, tr.ctypes.data, 1 << log_n, tr.shape[1], air.descriptor())


@pytest.mark.parametrize("G", [2, 8])
def test_sharded_forced_early_equals_single(gpu_ctx, monkeypatch, G):
    """virtual ranks: the quotient-point holders each run the early path on their slot"""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, ProverGroup, gen_permutation_trace
    a, d, _ = gpu_ctx.config.seeded()
    tr = gen_permutation_trace(10, 3, a, d)
    pub = np.concatenate([a, d])
    air = permutation_air(3)
    monkeypatch.setenv("LSP_QUOTIENT_EARLY", "0")
    single = gpu_ctx.prove(tr, air, pub)
    monkeypatch.setenv("LSP_QUOTIENT_EARLY", "1")
    grp = ProverGroup([Context(gpu_ctx.config) for _ in range(G)])
    assert grp.prove(tr, air, pub) == single
