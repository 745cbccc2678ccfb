"""The proof's structure pinned to the reference's own record of one proof:
bench.log:19-67 (6+6 permutation AIR, w = 14, 2^19 rows), extracted as data
into tests/golden/benchlog_shape.json by tests/golden/make_benchlog_shape.py.

What bench.log pins (and these tests check):
  * trace LDE: one coset_lde_batch of 14 x 2^19, added_bits 3 (log_blowup);
  * quotient: 8 chunk LDEs of 1 x 2^19 (degree rule U6 -> q = 8 for 6+6);
  * opening order: the trace matrix (14 x 2^22) reduced at two points (zeta,
    zeta * w_h), then the 8 chunks (1 x 2^22) at one point each;
  * FRI: the final vector has 8 values (divide_by_height 1x8: the final
    polynomial's IDFT over 2^(log_blowup + log_final_poly_len) points).
CPU tests: the fixture, and the oracle's proof layout at the same shape
(smaller n).  GPU test: the product prover's own span log at 2^19 equals the
fixture line for line.
"""
import json
import os

import numpy as np
import pytest

from oracle import pyoracle as O

FIX = os.path.join(os.path.dirname(__file__), "golden", "benchlog_shape.json")


def _spans():
    return [s["span"] for s in json.load(open(FIX))["spans"]]


def expected(log_n, w, q, log_blowup=3, log_final_poly_len=0):
    """bench.log's span sequence for a proof of this shape"""
    h, N = 1 << log_n, 1 << (log_n + log_blowup)
    s = [f"coset_lde_batch dims: {w}x{h} | added_bits: {log_blowup}"]
    s += [f"coset_lde_batch dims: 1x{h} | added_bits: {log_blowup}"] * q
    s += [f"reduce matrix quotient dims: {w}x{N}"] * 2
    s += [f"reduce matrix quotient dims: 1x{N}"] * q
    s += [f"divide_by_height dims: 1x{1 << (log_blowup + log_final_poly_len)}"]
    return s


def test_fixture_is_the_benchlog_proof():
    sp = _spans()
    assert len(sp) == 20
    assert sp == expected(19, 14, 8)


def test_oracle_proof_layout_at_benchlog_shape(oracle_lib):
    """6+6 (w = 14) proof from the C oracle: opened values in bench.log's
    opening order and counts, FRI rounds down to the 8-value final vector."""
    log_n, ncols = 8, 6
    p = oracle_lib.setup()
    tb, w = oracle_lib.gen_perm_trace(p, log_n, ncols)
    assert w == 14
    proof = O.deserialize_proof(oracle_lib.prove(p, tb, 1 << log_n, w, oracle_lib.perm_air(ncols)))
    assert proof.degree_bits == log_n and proof.width == 14
    assert proof.log_q == 3                        # 8 chunk LDEs
    assert len(proof.trace_local) == len(proof.trace_next) == 14   # trace at two points
    assert len(proof.quotient_chunks) == 8         # each chunk at one point
    assert len(proof.fri_roots) == log_n + 3 - 3   # folds N -> 8 (divide_by_height 1x8)
    for (t_row, t_path, q_row, q_path, steps) in proof.queries:
        assert len(t_row) == 14 and len(q_row) == 8
        assert len(t_path) == len(q_path) == log_n + 3
        assert [len(pth) for _, pth in steps] == [log_n + 3 - 1 - r for r in range(len(steps))]


@pytest.mark.gpu
def test_product_spans_match_benchlog(oracle_lib):
    """the GPU prover at the bench.log shape (6+6, 2^19) logs exactly the
    reference's data-shaped spans, in order"""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, StarkConfig
    log_n, ncols = 19, 6
    p = oracle_lib.setup()
    tb, w = oracle_lib.gen_perm_trace(p, log_n, ncols)
    trace = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << log_n, w, 4)
    pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
    with Context(StarkConfig()) as ctx:
        proof = ctx.prove(trace, permutation_air(ncols), pub)
        assert ctx.last_spans() == _spans()
        assert ctx.verify(proof, permutation_air(ncols), pub)
    # a different shape follows the same rule
    with Context(StarkConfig()) as ctx:
        tb, w = oracle_lib.gen_perm_trace(p, 10, 3)
        t = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << 10, w, 4)
        ctx.prove(t, permutation_air(3), pub)
        assert ctx.last_spans() == expected(10, 8, 4)
