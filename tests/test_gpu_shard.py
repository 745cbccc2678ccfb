"""Sharded prove (lsp_prove_group): G = 2 .. 32 ranks as virtual
ranks on one GPU (one context and one host thread each, exchanges through
device copies).  The proof must be byte-identical to the single-rank proof,
which the parity tests pin to the oracle."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _group(ctx, G):
    from linea_stark_prover_amd.prover import Context, ProverGroup
    ctxs = [Context(ctx.config) for _ in range(G)]
    return ProverGroup(ctxs), ctxs


@pytest.mark.parametrize("G", [2, 4, 8])
@pytest.mark.parametrize("log_n,ncols", [(3, 3), (9, 3), (10, 6)])
@pytest.mark.parametrize("fri_min", [None, "2"])
def test_group_proof_equals_single(gpu_ctx, monkeypatch, G, log_n, ncols, fri_min):
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import gen_permutation_trace
    if fri_min:
        monkeypatch.setenv("LSP_FRI_SHARD_MIN", fri_min)  # shard the FRI rounds down to 4-element slices
    a, d, _ = gpu_ctx.config.seeded()
    tr = gen_permutation_trace(log_n, ncols, a, d)
    pub = np.concatenate([a, d])
    air = permutation_air(ncols)
    single = gpu_ctx.prove(tr, air, pub)
    grp, _ = _group(gpu_ctx, G)
    got = grp.prove(tr, air, pub)
    assert got == single
    assert gpu_ctx.verify(got, air, pub)


def test_group_matches_oracle(gpu_ctx, oracle_lib, monkeypatch):
    from linea_stark_prover_amd.air import permutation_air
    monkeypatch.setenv("LSP_FRI_SHARD_MIN", "8")
    p = oracle_lib.setup()
    tb, w = oracle_lib.gen_perm_trace(p, 8, 3)
    tr = np.frombuffer(tb.raw, dtype=np.uint64).reshape(1 << 8, w, 4).copy()
    pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
    grp, _ = _group(gpu_ctx, 4)
    got = grp.prove(tr, permutation_air(3), pub)
    exp = oracle_lib.prove(p, tr.ctypes.data, 1 << 8, w, oracle_lib.perm_air(3))
    assert got == exp


@pytest.mark.parametrize("G", [2, 8])
def test_group_wide_air(gpu_ctx, monkeypatch, G):
    """lookup + permutation configs, q = 8 for the 6+6 groups: with G = 8 every
    rank owns one quotient chunk"""
    from linea_stark_prover_amd.prover import gen_wide_trace
    monkeypatch.setenv("LSP_FRI_SHARD_MIN", "4")
    a, d, _ = gpu_ctx.config.seeded()
    tr, air = gen_wide_trace(7, a, d, 2, 3, 2, 3, 6)
    pub = np.concatenate([a, d])
    single = gpu_ctx.prove(tr, air, pub)
    grp, _ = _group(gpu_ctx, G)
    assert grp.prove(tr, air, pub) == single


def test_group_device_resident_traces(gpu_ctx):
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import gen_permutation_trace
    a, d, _ = gpu_ctx.config.seeded()
    tr = gen_permutation_trace(12, 3, a, d)
    pub = np.concatenate([a, d])
    grp, ctxs = _group(gpu_ctx, 2)
    ptrs = []
    for c in ctxs:
        p = c.dev_alloc(tr.nbytes)
        c.h2d(p, tr)
        ptrs.append(p)
    got = grp.prove(ptrs, permutation_air(3), pub, tr.shape[0], tr.shape[1])
    assert got == gpu_ctx.prove(tr, permutation_air(3), pub)


@pytest.mark.parametrize("G", [16, 32])
@pytest.mark.parametrize("log_n,ncols", [(5, 3), (9, 3), (10, 6)])
@pytest.mark.parametrize("split", ["1", "0"])
def test_more_ranks_than_cosets(gpu_ctx, monkeypatch, G, log_n, ncols, split):
    """G > blowup: each rank owns a sub-coset of N/G < h
    rows, folded from the coefficients; the quotient's next rows come from
    the partner sub-coset, the chunk values are broadcast and inverted on
    every rank, the low coset's partial sums are added across its ranks.
    Byte-identical to the single-GPU proof, with the split inverse and
    without it (LSP_SHARD_SPLIT_INTT=0)"""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import gen_permutation_trace
    monkeypatch.setenv("LSP_SHARD_SPLIT_INTT", split)
    monkeypatch.setenv("LSP_FRI_SHARD_MIN", "2")
    a, d, _ = gpu_ctx.config.seeded()
    tr = gen_permutation_trace(log_n, ncols, a, d)
    pub = np.concatenate([a, d])
    air = permutation_air(ncols)
    single = gpu_ctx.prove(tr, air, pub)
    grp, _ = _group(gpu_ctx, G)
    assert grp.prove(tr, air, pub) == single


def test_more_ranks_than_cosets_wide_air(gpu_ctx, monkeypatch):
    """lookup + permutation configs (q = 8) over 16 ranks: every rank holds
    quotient points, half a chunk each"""
    from linea_stark_prover_amd.prover import gen_wide_trace
    monkeypatch.setenv("LSP_FRI_SHARD_MIN", "4")
    a, d, _ = gpu_ctx.config.seeded()
    tr, air = gen_wide_trace(7, a, d, 2, 3, 2, 3, 6)
    pub = np.concatenate([a, d])
    single = gpu_ctx.prove(tr, air, pub)
    grp, _ = _group(gpu_ctx, 16)
    assert grp.prove(tr, air, pub) == single


def test_group_rejects_too_many_ranks(gpu_ctx):
    """fewer than 2 LDE rows per rank (2^2 rows, N = 32, G = 32): a clean error on every rank"""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import gen_permutation_trace
    a, d, _ = gpu_ctx.config.seeded()
    tr = gen_permutation_trace(2, 3, a, d)
    grp, _ = _group(gpu_ctx, 32)
    with pytest.raises(RuntimeError, match="more ranks than LDE rows"):
        grp.prove(tr, permutation_air(3), np.concatenate([a, d]))


@pytest.mark.parametrize("log_n,split", [(20, "1"), (22, "1"), (22, "0")])
def test_group_large_equals_single(gpu_ctx, monkeypatch, log_n, split):
    """2^20 and 2^22 (BASELINE configs[1]'s size) rows over 8 virtual ranks
    (default FRI slice threshold: sharded rounds down to 8K-element slices,
    then replicated), with the split inverse + coefficient allgather and with
    the redundant inverse -- the two exchanges a calibrated communicator
    chooses between (lsp_comm_exchange_plan)"""
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import gen_permutation_trace
    monkeypatch.setenv("LSP_SHARD_SPLIT_INTT", split)
    a, d, _ = gpu_ctx.config.seeded()
    tr = gen_permutation_trace(log_n, 3, a, d)
    pub = np.concatenate([a, d])
    single = gpu_ctx.prove(tr, permutation_air(3), pub)
    grp, ctxs = _group(gpu_ctx, 8)
    try:
        assert grp.prove(tr, permutation_air(3), pub) == single
    finally:
        grp.close()
        for c in ctxs:
            c.close()


@pytest.mark.parametrize("rank", [0, 7])
def test_loopback_rank_rehearsal(product_lib, rank):
    """tools/rank_rehearsal.py's transport: rank g of 8 proves its share at a
    small size on its own (peers fabricated), returns a proof of the real
    proof's shape -- answered only as its size: the library refuses to hand the
    rehearsal proof out as bytes or as a view -- and reports its
    pool; the memory grows with the size"""
    import ctypes
    from linea_stark_prover_amd import _lib as L
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.prover import Context, StarkConfig, _take_proof
    cfg = StarkConfig()
    a, d, _ = cfg.seeded()
    pub = np.concatenate([a, d])
    pools = []
    for log_n in (12, 14):
        with Context(cfg) as ctx:
            L.check(L.lib().lsp_ctx_attach_loopback(ctx.h, rank, 8), ctx.h)
            dt = ctx.gen_permutation_trace_device(log_n, 3, a, d)
            desc = (ctypes.c_int32 * len(permutation_air(3).descriptor()))(*permutation_air(3).descriptor())
            h = ctypes.c_void_p()
            ctx._chk(L.lib().lsp_prove_sharded(ctx.h, dt, 1 << log_n, 8, desc, len(desc), pub.ctypes.data, 2,
                                               L.LSP_MEM_DEVICE, ctypes.byref(h)))
            n = ctypes.c_size_t()
            assert L.lib().lsp_proof_serialize(h, None, 0, ctypes.byref(n)) == L.LSP_OK  # the size query
            buf = ctypes.create_string_buffer(n.value)
            assert L.lib().lsp_proof_serialize(h, buf, n.value, ctypes.byref(n)) == L.LSP_E_STATE
            view = ctypes.create_string_buffer(4096)
            assert L.lib().lsp_proof_get_view(h, view) == L.LSP_E_STATE
            proof_len = _take_proof(h, size_only=True)
            ctx.dev_free(dt)
            pool, used, tot = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
            ctx._chk(L.lib().lsp_ctx_mem_stats(ctx.h, ctypes.byref(pool), ctypes.byref(used), ctypes.byref(tot)))
            assert 0 < pool.value <= used.value <= tot.value
            pools.append(pool.value)
            with Context(cfg) as ref:
                real = ref.prove(ref_trace(ref, log_n, a, d), permutation_air(3), pub)
            assert proof_len == len(real)  # same shape, fabricated peer data
    assert pools[1] > pools[0]


def ref_trace(ctx, log_n, a, d):
    h, w = 1 << log_n, 8
    p = ctx.gen_permutation_trace_device(log_n, 3, a, d)
    out = np.zeros((h, w, 4), np.uint64)
    ctx.d2h(out, p)
    ctx.dev_free(p)
    return out
