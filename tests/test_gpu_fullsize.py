"""Parity at the bench workload's full size (3x3 permutation AIR, 2^19 rows;
configs[1] at 2^22 is compared as a whole proof in test_gpu_fullsize_oracle.py).
These tests check the trace commitment in full and the rest through
properties that hold at any size:

* the trace LDE: every value against the C oracle's NTT LDE (bit-exact), and
  sampled rows against barycentric evaluation of the trace columns
  (`lo_eval_points`, no NTT, independent of either LDE);
* the trace Merkle tree from the fine-grained entry points
  (`lsp_coset_lde_batch` + `lsp_merkle_commit`): at 2^19 the oracle's whole
  tree (root and leaves); sampled leaves against the oracle's
  sponge, sampled nodes of every level against the oracle's compression, and
  the root against the trace root inside the fused `lsp_prove` proof;
* the proof: deterministic, accepted by the verifier, rejected once tampered;
* at 2^19 the whole proof byte for byte against the oracle's proof (36 s).
"""
import ctypes

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


def _oracle_compress(L, p, l, r):
    s = np.zeros((3, 4), np.uint64)
    s[0], s[1] = l, r
    L.lo_poseidon2_permute(ctypes.byref(p), _p(s))
    return s[0]


def _oracle_leaf(L, p, row):
    row = np.ascontiguousarray(row)
    out = np.zeros(4, np.uint64)
    L.lo_hash_iter(ctypes.byref(p), _p(row), ctypes.c_size_t(row.shape[0]), _p(out))
    return out


# 2^19 (the bench size).  2^22 ran here until round 5 (52 s); configs[1]'s
# evidence at 2^22 is now the whole proof byte-identical to the C oracle's
# (test_gpu_fullsize_oracle.py::test_configs1_whole_proof_2e22_vs_oracle),
# whose trace root already commits to every LDE value
@pytest.mark.parametrize("log_n", [19])
def test_full_size_lde_tree_and_proof(gpu_ctx, oracle_lib, log_n):
    from linea_stark_prover_amd.air import permutation_air
    from linea_stark_prover_amd.field import from_mont, to_mont
    from linea_stark_prover_amd.prover import MerkleTreeMmcs, Radix2DitParallel
    L = oracle_lib.lib()
    p = oracle_lib.setup()
    h, added = 1 << log_n, 3
    N = h << added
    tb, w = oracle_lib.gen_perm_trace(p, log_n, 3)
    trace = np.frombuffer(tb, dtype=np.uint64).reshape(h, w, 4).copy()
    del tb
    pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
    air = permutation_air(3)

    # ---- the proof (fused path)
    proof = gpu_ctx.prove(trace, air, pub)
    assert gpu_ctx.prove(trace, air, pub) == proof
    assert gpu_ctx.verify(proof, air, pub)
    bad = bytearray(proof)
    bad[40] ^= 1  # inside the trace root
    assert not gpu_ctx.verify(bytes(bad), air, pub)

    # ---- the LDE (fine-grained path)
    gen = to_mont([22])
    lde = Radix2DitParallel(gpu_ctx).coset_lde_batch(trace, added, gen)
    assert lde.shape == (N, w, 4)
    # the oracle's own NTT LDE, every value (one thread per column)
    exp = np.zeros_like(lde)
    shifts = np.repeat(gen.reshape(1, 4), w, axis=0).copy()
    L.lo_coset_lde_batch(_p(trace), ctypes.c_size_t(h), ctypes.c_size_t(w), added, _p(shifts), _p(exp), w)
    assert np.array_equal(lde, exp)
    del exp
    rng = np.random.default_rng(log_n)
    rows = np.concatenate([[0, 1, h - 1, h, N - 1], rng.integers(0, N, size=3)]).astype(np.uint64)
    xs = np.zeros((len(rows), 4), np.uint64)
    for k, j in enumerate(rows):
        L.lo_lde_point(ctypes.c_size_t(h), added, _p(gen), ctypes.c_uint64(int(j)), _p(xs[k]))
    vals = np.zeros((len(rows), w, 4), np.uint64)
    L.lo_eval_points(_p(trace), ctypes.c_size_t(h), ctypes.c_size_t(w), _p(xs), ctypes.c_size_t(len(rows)),
                     _p(vals), 16)
    assert np.array_equal(lde[rows.astype(np.int64)], vals)

    # ---- the trace tree (fine-grained path) against the oracle and the proof
    root, tree = MerkleTreeMmcs(gpu_ctx).commit([lde])
    assert from_mont(root)[0] == int.from_bytes(proof[32:64], "little")  # after "LSPPRF02" and 6 u32 fields
    if log_n <= 19:  # the oracle's whole tree (21 M permutations on 16 threads)
        lay = np.zeros((2 * N - 1, 4), np.uint64)
        L.lo_merkle_commit(ctypes.byref(p), _p(lde), ctypes.c_size_t(N), ctypes.c_size_t(w), _p(lay), 16)
        assert np.array_equal(lay[-1], root.reshape(4))
        assert np.array_equal(lay[:N], tree.layer(0))
        del lay
    leaves = tree.layer(0)
    for i in np.concatenate([[0, N - 1], rng.integers(0, N, size=14)]):
        assert np.array_equal(leaves[i], _oracle_leaf(L, p, lde[i]))
    del leaves, lde
    below = tree.layer(0)
    for lev in range(1, log_n + added + 1):
        cur = tree.layer(lev)
        for j in np.concatenate([[0, cur.shape[0] - 1], rng.integers(0, cur.shape[0], size=4)]):
            assert np.array_equal(cur[j], _oracle_compress(L, p, below[2 * j], below[2 * j + 1])), (lev, j)
        below = cur
    assert np.array_equal(below[0], root.reshape(4))


def test_full_proof_bench_size_vs_oracle(gpu_ctx, oracle_lib):
    """The whole 2^19-row proof (the bench workload) byte for byte against the C
    oracle's proof of the same trace (~36 s of oracle time on 16 host threads;
    2^22 was run the same way, `tools/full_oracle_proof.py`,
    `profiles/r01q_full_oracle_proofs.txt`)."""
    import os

    from linea_stark_prover_amd.air import permutation_air
    log_n = 19
    p = oracle_lib.setup()
    tb, w = oracle_lib.gen_perm_trace(p, log_n, 3)
    trace = np.frombuffer(tb, dtype=np.uint64).reshape(1 << log_n, w, 4).copy()
    pub = np.concatenate([np.array(p.alpha, np.uint64).reshape(1, 4), np.array(p.delta, np.uint64).reshape(1, 4)])
    proof = gpu_ctx.prove(trace, permutation_air(3), pub)
    threads = min(16, os.cpu_count() or 1)  # the GPU box's CPU share (os.cpu_count() shows the whole machine)
    expect = oracle_lib.prove(p, tb, 1 << log_n, w, oracle_lib.perm_air(3), nthreads=threads)
    assert proof == expect
