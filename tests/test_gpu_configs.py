"""Bit-exact parity vs the C oracle across the configuration switches the
boundary exposes (lsp_params): S-box degree (U1), round counts, the
public-value degree rule (U6) and the FRI parameters (bin/src/main.rs:58-64)."""
import numpy as np
import pytest

from oracle import pyoracle as O

pytestmark = pytest.mark.gpu

CASES = [
    dict(sbox_degree=17),
    dict(rounds_f=4, rounds_p=10),
    dict(rounds_f=6, rounds_p=7),  # odd: the partial rounds run in pairs plus a last single one
    dict(public_degree=0),
    dict(log_blowup=2, log_final_poly_len=1, num_queries=7),
    dict(log_blowup=4, log_final_poly_len=2, num_queries=50),
    dict(log_blowup=3, num_queries=1, proof_of_work_bits=4),
]


@pytest.mark.parametrize("kw", CASES, ids=lambda k: ",".join(f"{a}={b}" for a, b in k.items()))
@pytest.mark.parametrize("log_n,ncols", [(6, 3), (9, 6)])
def test_config_matches_oracle(oracle_lib, kw, log_n, ncols):
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, StarkConfig
    perm = {k: kw[k] for k in ("sbox_degree", "rounds_f", "rounds_p") if k in kw}
    fri = {k: kw[k] for k in ("log_blowup", "log_final_poly_len", "num_queries", "proof_of_work_bits") if k in kw}
    pdeg = kw.get("public_degree", 1)
    p = oracle_lib.setup(**perm)
    tb, w = oracle_lib.gen_perm_trace(p, log_n, ncols)
    trace = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << log_n, w, 4).copy()
    pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
    cfg = StarkConfig(public_degree=pdeg, **perm, **fri)
    log_q = (3 if ncols == 6 else 2) if pdeg == 1 else (2 if ncols == 6 else 1)
    if log_q > cfg.log_blowup:  # more quotient chunks than cosets: rejected, as Plonky3 cannot prove it
        from linea_stark_prover_amd import _lib
        with Context(cfg) as ctx, pytest.raises(_lib.LspError, match="exceeds the blowup"):
            ctx.prove(trace, permutation_air(ncols), pub)
        return
    with Context(cfg) as ctx:
        got = ctx.prove(trace, permutation_air(ncols), pub)
        assert ctx.verify(got, permutation_air(ncols), pub)
    f = oracle_lib.fri_params(O.FriParams(**fri))
    exp = oracle_lib.prove(p, trace.ctypes.data, 1 << log_n, w, oracle_lib.perm_air(ncols), fri=f,
                           public_degree=pdeg)
    assert got == exp
    if fri.get("log_final_poly_len", 0) == 0:  # the C oracle's verifier reads a 1-coefficient final poly only
        assert oracle_lib.verify(p, got, oracle_lib.perm_air(ncols), fri=f, public_degree=pdeg) == 0
    else:
        # the product verifier evaluates the whole final polynomial: a changed coefficient must fail
        with Context(cfg) as ctx:
            bad = bytearray(got)
            nr = log_n - fri.get("log_final_poly_len", 0)      # FRI rounds
            q = 1 << log_q
            off = 8 + 24 + 64 + 32 * (2 * (2 * ncols + 2) + q) + 32 * nr + 32  # second final coefficient
            bad[off] ^= 1
            assert not ctx.verify(bytes(bad), permutation_air(ncols), pub)


def test_odd_partial_rounds_every_lane_width(oracle_lib):
    """rounds_p odd at 2^13 rows: the LDE's 2^16 leaves take the one-state-per-lane
    kernels, the 32K level the lane-pair one and the narrower levels the quad one,
    each with the pairwise partial rounds and their single last round."""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, StarkConfig
    perm = dict(rounds_f=8, rounds_p=23)
    p = oracle_lib.setup(**perm)
    log_n, ncols = 13, 3
    tb, w = oracle_lib.gen_perm_trace(p, log_n, ncols)
    trace = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << log_n, w, 4).copy()
    pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
    with Context(StarkConfig(**perm)) as ctx:
        got = ctx.prove(trace, permutation_air(ncols), pub)
    assert got == oracle_lib.prove(p, trace.ctypes.data, 1 << log_n, w, oracle_lib.perm_air(ncols))


def test_sharded_with_small_blowup(gpu_ctx):
    """log_blowup 2 allows at most 4 ranks; the group proof equals the single one"""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, ProverGroup, StarkConfig, gen_permutation_trace
    cfg = StarkConfig(log_blowup=2, num_queries=9)
    a, d, _ = cfg.seeded()
    tr = gen_permutation_trace(10, 3, a, d)
    pub = np.concatenate([a, d])
    with Context(cfg) as ctx:
        single = ctx.prove(tr, permutation_air(3), pub)
    ctxs = [Context(cfg) for _ in range(4)]
    assert ProverGroup(ctxs).prove(tr, permutation_air(3), pub) == single
