"""The wide-AIR workload: the product's host witness
generator (RawLookupTrace / RawPermutationTrace semantics) against the Python
oracle, and the C oracle proving it (CPU)."""
import pytest

from oracle import pyoracle as O


@pytest.mark.parametrize("log_n,shape", [(3, (1, 2, 2, 1, 2)), (4, (2, 3, 2, 2, 3)), (5, (1, 3, 3, 0, 1))])
def test_wide_trace_matches_pyoracle(product_lib, log_n, shape):
    from linea_stark_prover_amd.field import from_mont
    from linea_stark_prover_amd.prover import StarkConfig, gen_wide_trace
    nlookup, na, ntab, nperm, pcols = shape
    a, d, _ = StarkConfig().seeded()
    tr, air = gen_wide_trace(log_n, a, d, nlookup, na, ntab, nperm, pcols)
    s = O.setup_from_seed()
    cfgs, cols = O.synthetic_wide_trace(log_n, s.alpha, s.delta, O.DEFAULT_SEED, nlookup, na, ntab, nperm, pcols)
    rows = O.columns_to_rows(cols)
    assert tr.shape[1] == len(rows[0]) == air.width
    assert from_mont(tr.reshape(-1, 4)) == [x for r in rows for x in r]
    from oracle import cref
    assert air.descriptor() == cref.air_desc(cfgs)


def test_wide_trace_default_width(product_lib):
    from linea_stark_prover_amd.prover import StarkConfig, gen_wide_trace
    a, d, _ = StarkConfig().seeded()
    tr, air = gen_wide_trace(3, a, d)
    assert tr.shape[1] == 184 == air.width  # 8*14 + 4*(3 + 2*6 + 3)


def test_wide_proof_python_vs_c(oracle_lib):
    s = O.setup_from_seed()
    p = oracle_lib.setup()
    cfgs, cols = O.synthetic_wide_trace(3, s.alpha, s.delta, O.DEFAULT_SEED, 1, 2, 2, 1, 2)
    rows = O.columns_to_rows(cols)
    pf = O.prove(cfgs, rows, [s.alpha, s.delta], s.perm)
    assert O.verify(cfgs, pf, [s.alpha, s.delta], s.perm)
    cb = oracle_lib.prove(p, oracle_lib.fr_buf([x for r in rows for x in r]), 8, len(rows[0]),
                          oracle_lib.air_desc(cfgs))
    assert cb == O.serialize_proof(pf)


def test_push_traces_rejects_extra_b_filters(product_lib):
    """more b_filter columns than tables would overrun the raw-column
    scratch on the device; push_traces refuses them before allocating anything"""
    import numpy as np
    import pytest
    from linea_stark_prover_amd.prover import Context, StarkConfig
    from linea_stark_prover_amd.trace import RawLookupTrace, RawTrace
    one = np.ones((4, 4), np.uint64)
    lt = RawLookupTrace([one], [[one]], None, [one, one])  # 1 table, 2 filters
    with Context(StarkConfig(), device=-1) as ctx:
        rt = RawTrace(ctx, [np.zeros(4, np.uint64), np.zeros(4, np.uint64)])
        with pytest.raises(ValueError, match="b_filter"):
            rt.push_traces([], [lt])
