"""U7 / U8 / U12 transcript switches on the GPU (include/lsp.h lsp_params):
under every non-default variant the GPU proof is byte-identical to the C
oracle set up the same way (tests/test_transcript.py pins the C oracle to
the Python one), verifies under its own setting and is rejected under the
default; the device grinder honours U8's Montgomery source; and a sharded
proof (2 and 4 virtual ranks) follows the switches too."""
import numpy as np
import pytest

from oracle import pyoracle as O
from test_transcript import VARIANTS, stark_switches

pytestmark = pytest.mark.gpu


def _case(oracle_lib, log_n, ncols):
    p = oracle_lib.setup()
    tb, w = oracle_lib.gen_perm_trace(p, log_n, ncols)
    trace = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << log_n, w, 4).copy()
    pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
    return p, trace, w, pub


@pytest.mark.parametrize("name", sorted(VARIANTS))
@pytest.mark.parametrize("log_n,ncols,pow_bits", [(6, 3, 4), (11, 6, 12)])
def test_variant_matches_oracle(oracle_lib, name, log_n, ncols, pow_bits):
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, StarkConfig
    p, trace, w, pub = _case(oracle_lib, log_n, ncols)
    air = permutation_air(ncols)
    with Context(StarkConfig(proof_of_work_bits=pow_bits, **stark_switches(name))) as ctx:
        got = ctx.prove(trace, air, pub)
        assert ctx.verify(got, air, pub)
    fp = O.FriParams(proof_of_work_bits=pow_bits, **VARIANTS[name])
    exp = oracle_lib.prove(p, trace.ctypes.data, 1 << log_n, w, oracle_lib.perm_air(ncols),
                           fri=oracle_lib.fri_params(fp))
    assert got == exp
    with Context(StarkConfig(proof_of_work_bits=pow_bits), device=-1) as v:
        assert not v.verify(got, air, pub)


@pytest.mark.parametrize("G", [2, 4])
def test_sharded_proof_follows_the_switches(oracle_lib, G):
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, ProverGroup, StarkConfig
    log_n, ncols = 10, 3
    p, trace, w, pub = _case(oracle_lib, log_n, ncols)
    cfg = StarkConfig(proof_of_work_bits=6, **stark_switches("all"))
    ctxs = [Context(cfg) for _ in range(G)]
    try:
        grp = ProverGroup(ctxs)
        got = grp.prove(trace, permutation_air(ncols), pub)
        grp.close()
        assert got == ctxs[0].prove(trace, permutation_air(ncols), pub)
    finally:
        for c in ctxs:
            c.close()
    fp = O.FriParams(proof_of_work_bits=6, **VARIANTS["all"])
    assert got == oracle_lib.prove(p, trace.ctypes.data, 1 << log_n, w, oracle_lib.perm_air(ncols),
                                   fri=oracle_lib.fri_params(fp))
