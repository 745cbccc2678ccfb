"""GPU parity on the wide AIR (LogUp lookups + permutation groups): the
quotient interpreter over many configs, wide rows in the leaf hash."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("log_n,shape", [(4, (4, 3, 2, 8, 6)), (7, (2, 3, 2, 3, 6)), (9, (1, 3, 2, 1, 3))])
def test_wide_prove_matches_oracle(gpu_ctx, oracle_lib, log_n, shape):
    from linea_stark_prover_amd.prover import gen_wide_trace
    a, d, _ = gpu_ctx.config.seeded()
    tr, air = gen_wide_trace(log_n, a, d, *shape)
    pub = np.concatenate([a, d])
    got = gpu_ctx.prove(tr, air, pub)
    assert gpu_ctx.verify(got, air, pub)
    p = oracle_lib.setup()
    exp = oracle_lib.prove(p, tr.ctypes.data, 1 << log_n, tr.shape[1], air.descriptor())
    assert got == exp


def test_wide_prove_matches_oracle_2e12(gpu_ctx, oracle_lib):
    from linea_stark_prover_amd.prover import gen_wide_trace
    a, d, _ = gpu_ctx.config.seeded()
    tr, air = gen_wide_trace(12, a, d)  # the C3 shape: 4 lookups + 8 groups of 6+6, W = 184
    pub = np.concatenate([a, d])
    got = gpu_ctx.prove(tr, air, pub)
    p = oracle_lib.setup()
    assert got == oracle_lib.prove(p, tr.ctypes.data, 1 << 12, tr.shape[1], air.descriptor())


@pytest.mark.parametrize("ncols", [1023, 2300])
def test_very_wide_trace_matches_oracle(product_lib, oracle_lib, ncols):
    """w = 2048 and w = 4602: the reduce-rows constants beyond 64 KiB of LDS
    (in LDS up to gfx950's 160 KiB, in global memory beyond), which round 2's
    kernel refused (review: any width the reference handles must prove).
    Public degree 0 keeps q = 2 at this width."""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, StarkConfig
    log_n = 4
    p = oracle_lib.setup()
    tb, w = oracle_lib.gen_perm_trace(p, log_n, ncols)
    exp = oracle_lib.prove(p, tb, 1 << log_n, w, oracle_lib.perm_air(ncols), public_degree=0)
    trace = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << log_n, w, 4).copy()
    pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
    with Context(StarkConfig(public_degree=0)) as ctx:
        got = ctx.prove(trace, permutation_air(ncols), pub)
        assert got == exp
        assert ctx.verify(got, permutation_air(ncols), pub)
