"""Python mirror of the reference's plug point (bin/src/config.rs:9-25) over
the C-ABI of liblsp_hip.so.

Reference item                                   -> here
  StarkConfig / FriConfig / Perm::new_from_rng    -> StarkConfig (+ seeded U4/U5 setup)
  Radix2DitParallel::coset_lde_batch (Dft)        -> Radix2DitParallel.coset_lde_batch
  MerkleTreeMmcs commit/open_batch/verify_batch   -> MerkleTreeMmcs
  TwoAdicFriGenericConfig::fold_matrix/fold_row   -> TwoAdicFriGenericConfig
  p3_uni_stark::quotient_values                   -> Context.quotient_values
  p3_interpolation::interpolate_coset             -> Context.interpolate_coset
  TwoAdicFriPcs::open compute_inverse_denominators -> Context.inverse_denominators
  TwoAdicFriPcs::open reduce rows                 -> Context.open_reduce
  p3_uni_stark::prove / verify (main.rs:80-96)    -> prove / verify

Arrays are numpy uint64 with a trailing axis of 4 limbs (Montgomery form).
Everything runs through the HIP library; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .air import LineaAIR
from .field import to_mont

DEFAULT_SEED = 0x4C494E4541  # "LINEA"


def _ptr(a: np.ndarray) -> int:
    return a.ctypes.data


def _fr_arr(a) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.uint64)
    assert a.shape[-1] == 4, "element arrays need a trailing axis of 4 limbs"
    return a


@dataclass
class StarkConfig:
    """bin/src/config.rs:9-25 + bin/src/main.rs:49-64 (+ the U1/U6 switches)."""
    sbox_degree: int = 11           # U1
    rounds_f: int = 8               # Perm::new_from_rng(8, 22)
    rounds_p: int = 22
    log_blowup: int = 3             # FriConfig
    log_final_poly_len: int = 0
    num_queries: int = 33
    proof_of_work_bits: int = 0
    public_degree: int = 1          # U6
    seed: int = DEFAULT_SEED        # U4/U5
    # U2/U3, the Poseidon2 linear layers (include/lsp.h): canonical ints,
    # None = the default layer (internal diag (1, 1, 2); external circ(2, 1, 1))
    internal_diag: Optional[Tuple[int, int, int]] = None
    external_mds: Optional[Tuple[int, ...]] = None   # 9 entries, row-major
    # U7/U8/U12 transcript conventions (include/lsp.h lsp_params), 0/False = default
    skip_log_degree: bool = False         # U7: log2(h) not observed
    skip_public_values: bool = False      # U7: [alpha, delta] not observed before the quotient challenge
    observe_opened_values: bool = False   # U7: opened values observed before alpha_fri
    sample_bits_montgomery: bool = False  # U8: sample_bits from the Montgomery form
    skip_final_poly: bool = False         # U12: final polynomial not observed

    def seeded(self) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
        """(alpha, delta, round_constants) from the documented seeded generator."""
        n = 3 * self.rounds_f + self.rounds_p
        a, d, rc = np.zeros((1, 4), np.uint64), np.zeros((1, 4), np.uint64), np.zeros((n, 4), np.uint64)
        L.check(L.lib().lsp_seeded_setup(self.seed, self.rounds_f, self.rounds_p, _ptr(a), _ptr(d), _ptr(rc)))
        return a, d, rc


def _take_proof(proof: ctypes.c_void_p, size_only: bool = False):
    """serialize and free an lsp_proof handle (size_only: its wire size, the
    one thing a rehearsal proof answers).  The library writes into a bytearray
    the caller's bytes are then copied from (one 324 KB copy per 2^19 proof,
    tens of microseconds; round 4 wrote into an immutable bytes object instead)"""
    try:
        n = ctypes.c_size_t()
        L.check(L.lib().lsp_proof_serialize(proof, None, 0, ctypes.byref(n)))
        if size_only:
            return n.value
        size = n.value
        buf = bytearray(max(size, 1))
        dst = (ctypes.c_char * len(buf)).from_buffer(buf)
        L.check(L.lib().lsp_proof_serialize(proof, dst, size, ctypes.byref(n)))
        if n.value != size:
            raise RuntimeError(f"lsp_proof_serialize wrote {n.value} of {size} bytes")
        del dst  # release the export before the copy
        return bytes(buf[:size]) if size != len(buf) else bytes(buf)
    finally:
        L.lib().lsp_proof_free(proof)


class Context:
    """One lsp_ctx: a GPU, a stream, the Poseidon2 constants and a buffer pool."""

    def __init__(self, config: StarkConfig = StarkConfig(), device: int = 0,
                 round_constants: Optional[np.ndarray] = None):
        self.config = config
        self.device = device
        if round_constants is None:
            _, _, round_constants = config.seeded()
        self._rc = _fr_arr(round_constants)
        self._diag = None if config.internal_diag is None else to_mont(config.internal_diag)
        self._mds = None if config.external_mds is None else to_mont(config.external_mds)
        assert self._diag is None or self._diag.shape[0] == 3, "internal_diag needs 3 entries"
        assert self._mds is None or self._mds.shape[0] == 9, "external_mds needs 9 entries"
        p = L.LspParams(sbox_degree=config.sbox_degree, rounds_f=config.rounds_f, rounds_p=config.rounds_p,
                        round_constants=_ptr(self._rc), log_blowup=config.log_blowup,
                        log_final_poly_len=config.log_final_poly_len, num_queries=config.num_queries,
                        proof_of_work_bits=config.proof_of_work_bits, public_degree=config.public_degree,
                        internal_diag=None if self._diag is None else _ptr(self._diag),
                        external_mds=None if self._mds is None else _ptr(self._mds),
                        **{k: int(getattr(config, k)) for k in L.TRANSCRIPT_SWITCHES})
        h = ctypes.c_void_p()
        L.check(L.lib().lsp_ctx_create(device, ctypes.byref(p), ctypes.byref(h)))
        self.h = h

    def close(self):
        if self.h:
            L.lib().lsp_ctx_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _chk(self, rc):
        L.check(rc, self.h)

    def synchronize(self):
        self._chk(L.lib().lsp_synchronize(self.h))

    def comm_log(self):
        """the attached communicator's collectives of the last sharded proof
        (lsp_comm_log): (entries, init_ms), each entry a dict with op
        ("allgather" / "bcast"), bytes, root, tag and device ms"""
        n, init = ctypes.c_size_t(), ctypes.c_double()
        self._chk(L.lib().lsp_comm_log(self.h, None, None, None, None, None, 0, ctypes.byref(n),
                                       ctypes.byref(init)))
        k = n.value
        ops = ctypes.create_string_buffer(max(k, 1))
        nb, roots = (ctypes.c_size_t * max(k, 1))(), (ctypes.c_int * max(k, 1))()
        ms, tags = (ctypes.c_double * max(k, 1))(), (ctypes.c_char_p * max(k, 1))()
        self._chk(L.lib().lsp_comm_log(self.h, ops, nb, roots, ms, tags, k, ctypes.byref(n), ctypes.byref(init)))
        out = [{"op": "allgather" if ops.raw[i:i + 1] == b"A" else "bcast", "bytes": int(nb[i]),
                "root": None if roots[i] < 0 else int(roots[i]), "tag": tags[i].decode(), "ms": float(ms[i])}
               for i in range(min(k, n.value))]
        return out, float(init.value)

    # ---------------------------------------------------------- device buffers
    def dev_alloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        self._chk(L.lib().lsp_dev_alloc(self.h, nbytes, ctypes.byref(p)))
        return p.value

    def dev_free(self, p: int):
        self._chk(L.lib().lsp_dev_free(self.h, p))

    def h2d(self, dst: int, a: np.ndarray):
        a = np.ascontiguousarray(a)
        self._chk(L.lib().lsp_memcpy_h2d(self.h, dst, _ptr(a), a.nbytes))

    def d2h(self, a: np.ndarray, src: int):
        self._chk(L.lib().lsp_memcpy_d2h(self.h, _ptr(a), src, a.nbytes))

    # ------------------------------------------------------------------- Dft
    def coset_lde_batch(self, mat: np.ndarray, added_bits: int, shift) -> np.ndarray:
        mat = _fr_arr(mat)
        h, w = mat.shape[0], mat.shape[1]
        out = np.zeros((h << added_bits, w, 4), np.uint64)
        sh = _fr_arr(shift).reshape(-1, 4)
        if sh.shape[0] == 1:
            self._chk(L.lib().lsp_coset_lde_batch(self.h, _ptr(mat), h, w, added_bits, _ptr(sh), _ptr(out),
                                                  L.LSP_MEM_HOST))
        else:
            assert sh.shape[0] == w
            self._chk(L.lib().lsp_coset_lde_batch_shifts(self.h, _ptr(mat), h, w, added_bits, _ptr(sh), _ptr(out),
                                                         L.LSP_MEM_HOST))
        return out

    def coset_dft_batch(self, coeffs: np.ndarray, shift=None) -> np.ndarray:
        """TwoAdicSubgroupDft::coset_dft_batch (dft_batch: shift None): h x w
        coefficients -> evaluations on shift*H_h, rows bit-reversed"""
        coeffs = _fr_arr(coeffs)
        h, w = coeffs.shape[0], coeffs.shape[1]
        out = np.zeros((h, w, 4), np.uint64)
        sh = None if shift is None else _fr_arr(shift).reshape(4)
        self._chk(L.lib().lsp_coset_dft_batch(self.h, _ptr(coeffs), h, w, None if sh is None else _ptr(sh), _ptr(out),
                                              L.LSP_MEM_HOST))
        return out

    def coset_idft_batch(self, evals: np.ndarray, shift=None) -> np.ndarray:
        """TwoAdicSubgroupDft::coset_idft_batch (idft_batch: shift None): h x w
        evaluations on shift*H_h in natural order -> coefficients"""
        evals = _fr_arr(evals)
        h, w = evals.shape[0], evals.shape[1]
        out = np.zeros((h, w, 4), np.uint64)
        sh = None if shift is None else _fr_arr(shift).reshape(4)
        self._chk(L.lib().lsp_coset_idft_batch(self.h, _ptr(evals), h, w, None if sh is None else _ptr(sh), _ptr(out),
                                               L.LSP_MEM_HOST))
        return out

    # -------------------------------------------------------------- symmetric
    def poseidon2_permute(self, states: np.ndarray) -> np.ndarray:
        s = _fr_arr(states).copy()
        self._chk(L.lib().lsp_poseidon2_permute_batch(self.h, _ptr(s), s.shape[0], L.LSP_MEM_HOST))
        return s

    def hash_rows(self, rows: np.ndarray) -> np.ndarray:
        rows = _fr_arr(rows)
        out = np.zeros((rows.shape[0], 4), np.uint64)
        self._chk(L.lib().lsp_hash_rows(self.h, _ptr(rows), rows.shape[0], rows.shape[1], _ptr(out),
                                        L.LSP_MEM_HOST))
        return out

    # -------------------------------------------------------------- quotient
    def quotient_values(self, lde: np.ndarray, h: int, air: LineaAIR, public_values: np.ndarray,
                        alpha: np.ndarray) -> np.ndarray:
        lde = _fr_arr(lde)
        desc = (ctypes.c_int32 * len(air.descriptor()))(*air.descriptor())
        lq = ctypes.c_uint32()
        L.check(L.lib().lsp_log_quotient_degree(desc, len(desc), self.config.public_degree, ctypes.byref(lq)))
        out = np.zeros((h << lq.value, 4), np.uint64)
        pub = _fr_arr(public_values).reshape(-1, 4)
        al = _fr_arr(alpha).reshape(-1, 4)
        self._chk(L.lib().lsp_quotient_values(self.h, _ptr(lde), h, lde.shape[1], desc, len(desc), _ptr(pub),
                                              pub.shape[0], _ptr(al), _ptr(out), L.LSP_MEM_HOST))
        return out

    def interpolate_coset(self, lde_bitrev: np.ndarray, h: int, shift, z) -> np.ndarray:
        m = _fr_arr(lde_bitrev)
        w = m.shape[1]
        out = np.zeros((w, 4), np.uint64)
        sh, zz = _fr_arr(shift).reshape(-1, 4), _fr_arr(z).reshape(-1, 4)
        self._chk(L.lib().lsp_interpolate_coset(self.h, _ptr(m), h, w, _ptr(sh), _ptr(zz), _ptr(out),
                                                L.LSP_MEM_HOST))
        return out

    def inverse_denominators(self, points, log_n: int, shift) -> np.ndarray:
        """compute_inverse_denominators: (len(points), 2^log_n, 4) array of
        1/(z - shift w_N^bitrev(i))."""
        pts = _fr_arr(points).reshape(-1, 4)
        sh = _fr_arr(shift).reshape(-1, 4)
        out = np.zeros((pts.shape[0], 1 << log_n, 4), np.uint64)
        self._chk(L.lib().lsp_inverse_denominators(self.h, _ptr(pts), pts.shape[0], log_n, _ptr(sh), _ptr(out),
                                                   L.LSP_MEM_HOST))
        return out

    def open_reduce(self, mat: np.ndarray, inv_denoms: np.ndarray, ys: np.ndarray, alpha, alpha_pow_offset,
                    ro: np.ndarray) -> np.ndarray:
        """Reduce rows of one opened matrix (n x w) at len(ys) points into ro
        (updated in place); returns the advanced alpha-power offset."""
        m = _fr_arr(mat)
        n, w = m.shape[0], m.shape[1]
        inv = _fr_arr(inv_denoms).reshape(-1, n, 4)
        y = _fr_arr(ys).reshape(inv.shape[0], w, 4)
        al = _fr_arr(alpha).reshape(-1, 4)
        off = _fr_arr(alpha_pow_offset).reshape(-1, 4).copy()
        assert ro.dtype == np.uint64 and ro.shape == (n, 4) and ro.flags["C_CONTIGUOUS"]
        self._chk(L.lib().lsp_open_reduce(self.h, _ptr(m), n, w, _ptr(inv), _ptr(y), inv.shape[0], _ptr(al),
                                          _ptr(off), _ptr(ro), L.LSP_MEM_HOST))
        return off[0]

    def batch_inverse(self, x: np.ndarray) -> np.ndarray:
        x = _fr_arr(x).reshape(-1, 4)
        out = np.zeros_like(x)
        self._chk(L.lib().lsp_batch_inverse(self.h, _ptr(x), x.shape[0], _ptr(out), L.LSP_MEM_HOST))
        return out

    # ----------------------------------------------------------------- prove
    def prove(self, trace, air: LineaAIR, public_values: np.ndarray, h: Optional[int] = None,
              w: Optional[int] = None) -> bytes:
        """p3_uni_stark::prove.  `trace` is an (h, w, 4) host array, or a device
        pointer (int) to an h x w matrix with h and w given."""
        desc = (ctypes.c_int32 * len(air.descriptor()))(*air.descriptor())
        pub = _fr_arr(public_values).reshape(-1, 4)
        proof = ctypes.c_void_p()
        if isinstance(trace, int):
            self._chk(L.lib().lsp_prove(self.h, trace, h, w, desc, len(desc), _ptr(pub), pub.shape[0],
                                        L.LSP_MEM_DEVICE, ctypes.byref(proof)))
        else:
            t = _fr_arr(trace)
            self._chk(L.lib().lsp_prove(self.h, _ptr(t), t.shape[0], t.shape[1], desc, len(desc), _ptr(pub),
                                        pub.shape[0], L.LSP_MEM_HOST, ctypes.byref(proof)))
        return _take_proof(proof)

    def verify(self, proof: bytes, air: LineaAIR, public_values: np.ndarray) -> bool:
        desc = (ctypes.c_int32 * len(air.descriptor()))(*air.descriptor())
        pub = _fr_arr(public_values).reshape(-1, 4)
        rc = L.lib().lsp_verify(self.h, desc, len(desc), _ptr(pub), pub.shape[0], proof, len(proof))
        if rc == L.LSP_E_VERIFY:
            return False
        L.check(rc)
        return True

    def set_phase_timing(self, on: bool = True, only: Optional[Sequence[str]] = None):
        """lsp_ctx_set_phase_timing: which phases the next proofs time (all by
        default; off saves ~0.3 ms of host time per 2^19 proof).  `only`: just
        these phases (names as last_timings() reports them)."""
        names = [n.encode() for n in (only or [])]
        arr = (ctypes.c_char_p * len(names))(*names) if names else None
        self._chk(L.lib().lsp_ctx_set_phase_timing(self.h, int(bool(on)), arr, len(names)))

    def calibrate_fr_mul(self) -> float:
        """G Fr-mul/s of the device multiplier (register-resident chains)."""
        v = ctypes.c_double()
        self._chk(L.lib().lsp_calibrate_fr_mul(self.h, ctypes.byref(v)))
        return v.value

    def gen_permutation_trace_device(self, log_n: int, ncols: int, alpha: np.ndarray, delta: np.ndarray,
                                     seed: int = DEFAULT_SEED) -> int:
        """The C1 workload shape generated on the device (lsp_gen_permutation_trace_device):
        returns a device pointer to the (2^log_n, 2*ncols+2) row-major trace; free it with
        dev_free.  Values differ from gen_permutation_trace's (see include/lsp.h)."""
        w = 2 * ncols + 2
        p = self.dev_alloc((1 << log_n) * w * 32)
        try:
            self._chk(L.lib().lsp_gen_permutation_trace_device(self.h, seed, log_n, ncols, _ptr(_fr_arr(alpha)),
                                                               _ptr(_fr_arr(delta)), p))
        except BaseException:
            self.dev_free(p)
            raise
        return p

    def exchange_plan(self, h: int, w: int, q: int = 0) -> dict:
        """lsp_comm_exchange_plan: the calibrated allgather bandwidth and inverse-NTT
        rate of the attached communicator and the inverse-NTT exchange a sharded
        proof of h x w with q quotient chunks takes on them (q = 0: the trace's
        share of the model only)"""
        gbs, rate, ms_ag, ms_red = ctypes.c_double(), ctypes.c_double(), ctypes.c_double(), ctypes.c_double()
        probe, split = ctypes.c_size_t(), ctypes.c_int()
        self._chk(L.lib().lsp_comm_exchange_plan(self.h, h, w, q, ctypes.byref(gbs), ctypes.byref(rate),
                                                 ctypes.byref(probe), ctypes.byref(split), ctypes.byref(ms_ag),
                                                 ctypes.byref(ms_red)))
        out = {"allgather_gbs": gbs.value, "intt_gelem_per_s": rate.value, "probe_bytes": probe.value,
               "split_intt": bool(split.value), "model_allgather_ms": ms_ag.value,
               "model_redundant_intt_ms": ms_red.value, "per_rank": self.comm_calibration()}
        if q:
            # the quotient-chunk broadcasts (the same bytes under either choice)
            nb, each, qms = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_double()
            self._chk(L.lib().lsp_comm_quotient_exchange(self.h, h, q, ctypes.byref(nb), ctypes.byref(each),
                                                         ctypes.byref(qms)))
            out.update({"quotient_bcasts": nb.value, "quotient_bcast_bytes_each": each.value,
                        "model_quotient_bcast_ms": qms.value,
                        "model_exchange_ms": qms.value + (ms_ag.value if split.value else 0.0)})
        return out

    def comm_calibration(self) -> list:
        """lsp_comm_calibration: every rank's own probes, rank order --
        {"allgather_4mib_gbs", "allgather_256mib_gbs" (0: not run), "intt_gelem_per_s"}"""
        n = ctypes.c_size_t()
        self._chk(L.lib().lsp_comm_calibration(self.h, None, 0, ctypes.byref(n)))
        if not n.value:
            return []
        buf = (ctypes.c_double * n.value)()
        self._chk(L.lib().lsp_comm_calibration(self.h, buf, n.value, ctypes.byref(n)))
        v = list(buf)
        return [{"allgather_4mib_gbs": v[i], "allgather_256mib_gbs": v[i + 1], "intt_gelem_per_s": v[i + 2]}
                for i in range(0, len(v), 3)]

    def calibrate_intt(self, log_h: int = 20, w: int = 8) -> float:
        """lsp_calibrate_intt: this GPU's inverse-NTT rate on random data, G elements/s"""
        v = ctypes.c_double()
        self._chk(L.lib().lsp_calibrate_intt(self.h, log_h, w, ctypes.byref(v)))
        return v.value

    def host_threads(self) -> int:
        """lsp_ctx_host_threads: the size of this context's host pool"""
        n = ctypes.c_int()
        self._chk(L.lib().lsp_ctx_host_threads(self.h, ctypes.byref(n)))
        return n.value

    def comm_info(self) -> Tuple[int, int]:
        """(rank, size) of the attached communicator"""
        r, n = ctypes.c_int(), ctypes.c_int()
        self._chk(L.lib().lsp_comm_info(self.h, ctypes.byref(r), ctypes.byref(n)))
        return r.value, n.value

    def calibrate_poseidon2(self) -> float:
        """M Poseidon2 permutations/s (register-resident chained states)."""
        v = ctypes.c_double()
        self._chk(L.lib().lsp_calibrate_poseidon2(self.h, ctypes.byref(v)))
        return v.value

    def last_timings(self) -> List[Tuple[str, float]]:
        n = ctypes.c_size_t()
        L.lib().lsp_last_timings(self.h, None, None, 0, ctypes.byref(n))
        ms = (ctypes.c_double * n.value)()
        names = (ctypes.c_char_p * n.value)()
        L.lib().lsp_last_timings(self.h, ms, names, n.value, ctypes.byref(n))
        return [(names[i].decode(), ms[i]) for i in range(n.value)]

    def last_spans(self) -> List[str]:
        """the last proof's operations with dims, in the reference's bench.log wording"""
        n = ctypes.c_size_t()
        self._chk(L.lib().lsp_last_spans(self.h, None, 0, ctypes.byref(n)))
        lines = (ctypes.c_char_p * n.value)()
        self._chk(L.lib().lsp_last_spans(self.h, lines, n.value, ctypes.byref(n)))
        return [lines[i].decode() for i in range(n.value)]


class Radix2DitParallel:
    """TwoAdicSubgroupDft (bin/src/config.rs:22) on the GPU; returns the
    bit-reversed rows TwoAdicFriPcs::commit consumes."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def coset_lde_batch(self, mat: np.ndarray, added_bits: int, shift) -> np.ndarray:
        return self.ctx.coset_lde_batch(mat, added_bits, shift)

    def lde_batch(self, mat: np.ndarray, added_bits: int) -> np.ndarray:
        from .field import to_mont
        return self.ctx.coset_lde_batch(mat, added_bits, to_mont([1])[0])

    def dft_batch(self, coeffs: np.ndarray) -> np.ndarray:
        return self.ctx.coset_dft_batch(coeffs)

    def coset_dft_batch(self, coeffs: np.ndarray, shift) -> np.ndarray:
        return self.ctx.coset_dft_batch(coeffs, shift)

    def idft_batch(self, evals: np.ndarray) -> np.ndarray:
        return self.ctx.coset_idft_batch(evals)

    def coset_idft_batch(self, evals: np.ndarray, shift) -> np.ndarray:
        return self.ctx.coset_idft_batch(evals, shift)


class MerkleTree:
    def __init__(self, ctx: Context, handle, height: int, widths: Sequence[int]):
        self.ctx, self.handle, self.height, self.widths = ctx, handle, height, list(widths)

    def __del__(self):
        if getattr(self, "handle", None):
            L.lib().lsp_tree_free(self.handle)
            self.handle = None

    def layer(self, level: int) -> np.ndarray:
        out = np.zeros((self.height >> level, 4), np.uint64)
        self.ctx._chk(L.lib().lsp_merkle_layer(self.handle, level, _ptr(out)))
        return out


class MerkleTreeMmcs:
    """MerkleTreeMmcs<Val, Val, Hash, Compress, 1> (bin/src/config.rs:19-20)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def commit(self, mats: Sequence[np.ndarray]) -> Tuple[np.ndarray, MerkleTree]:
        mats = [_fr_arr(m) for m in mats]
        hgt = mats[0].shape[0]
        assert all(m.shape[0] == hgt for m in mats), "equal heights only"
        ptrs = (ctypes.c_void_p * len(mats))(*[_ptr(m) for m in mats])
        widths = (ctypes.c_size_t * len(mats))(*[m.shape[1] for m in mats])
        root = np.zeros((1, 4), np.uint64)
        t = ctypes.c_void_p()
        self.ctx._chk(L.lib().lsp_merkle_commit(self.ctx.h, ptrs, widths, len(mats), hgt, L.LSP_MEM_HOST,
                                                _ptr(root), ctypes.byref(t)))
        return root, MerkleTree(self.ctx, t, hgt, [m.shape[1] for m in mats])

    def open_batch(self, index: int, tree: MerkleTree) -> Tuple[List[np.ndarray], np.ndarray]:
        rows = np.zeros((sum(tree.widths), 4), np.uint64)
        path = np.zeros((max(tree.height.bit_length() - 1, 1), 4), np.uint64)
        self.ctx._chk(L.lib().lsp_merkle_open(tree.handle, index, _ptr(rows), _ptr(path)))
        out, o = [], 0
        for w in tree.widths:
            out.append(rows[o:o + w])
            o += w
        return out, path[:tree.height.bit_length() - 1]

    def verify_batch(self, root: np.ndarray, widths: Sequence[int], log_height: int, index: int,
                     rows: Sequence[np.ndarray], path: np.ndarray) -> bool:
        flat = _fr_arr(np.concatenate([_fr_arr(r).reshape(-1, 4) for r in rows]))
        ws = (ctypes.c_size_t * len(widths))(*widths)
        p = _fr_arr(path).reshape(-1, 4) if log_height else np.zeros((1, 4), np.uint64)
        rc = L.lib().lsp_merkle_verify(self.ctx.h, _ptr(_fr_arr(root)), ws, len(widths), log_height, index,
                                       _ptr(flat), _ptr(p))
        return rc == L.LSP_OK


class TwoAdicFriGenericConfig:
    """The north_star's 'FriFolder' ([EXT p3-fri] FriGenericConfig)."""

    def __init__(self, ctx: Context):
        self.ctx = ctx

    def fold_matrix(self, beta: np.ndarray, v: np.ndarray) -> np.ndarray:
        v = _fr_arr(v).reshape(-1, 4)
        out = np.zeros((v.shape[0] // 2, 4), np.uint64)
        b = _fr_arr(beta).reshape(-1, 4)
        self.ctx._chk(L.lib().lsp_fri_fold(self.ctx.h, _ptr(v), v.shape[0], _ptr(b), _ptr(out), L.LSP_MEM_HOST))
        return out

    @staticmethod
    def fold_row(index: int, log_height: int, beta: np.ndarray, e0: np.ndarray, e1: np.ndarray) -> np.ndarray:
        out = np.zeros((1, 4), np.uint64)
        L.lib().lsp_fri_fold_row(index, log_height, _ptr(_fr_arr(beta)), _ptr(_fr_arr(e0)), _ptr(_fr_arr(e1)),
                                 _ptr(out))
        return out


def gen_permutation_trace(log_n: int, ncols: int, alpha: np.ndarray, delta: np.ndarray,
                          seed: int = DEFAULT_SEED, small_values: bool = False) -> np.ndarray:
    """Synthetic trace of SURVEY 8(d) C1 with RawPermutationTrace's witness
    columns (trace/src/permutation.rs:24-93): (2^log_n, 2*ncols+2, 4)."""
    out = np.zeros((1 << log_n, 2 * ncols + 2, 4), np.uint64)
    L.check(L.lib().lsp_gen_permutation_trace(seed, log_n, ncols, _ptr(_fr_arr(alpha)), _ptr(_fr_arr(delta)),
                                              int(small_values), _ptr(out)))
    return out


def gen_wide_trace(log_n: int, alpha: np.ndarray, delta: np.ndarray, nlookup: int = 4, na: int = 3, ntab: int = 2,
                   nperm: int = 8, pcols: int = 6, seed: int = DEFAULT_SEED) -> Tuple[np.ndarray, LineaAIR]:
    """SURVEY 8(d) C3 wide AIR (default: 4 LogUp lookups with 3-column A and two
    3-column tables, 8 permutation groups of 6+6; width 184).  Returns the
    (2^log_n, W, 4) trace and its LineaAIR."""
    w, dl = ctypes.c_size_t(), ctypes.c_size_t()
    args = (seed, log_n, nlookup, na, ntab, nperm, pcols, _ptr(_fr_arr(alpha)), _ptr(_fr_arr(delta)))
    L.check(L.lib().lsp_gen_wide_trace(*args, None, 0, None, 0, ctypes.byref(w), ctypes.byref(dl)))
    rows = np.zeros((1 << log_n, w.value, 4), np.uint64)
    desc = (ctypes.c_int32 * dl.value)()
    L.check(L.lib().lsp_gen_wide_trace(*args, _ptr(rows), rows.shape[0] * w.value, desc, dl.value, ctypes.byref(w),
                                       ctypes.byref(dl)))
    return rows, LineaAIR.from_descriptor(list(desc))


class ProverGroup:
    """G = 2^b contexts proving one proof together (lsp_prove_group, SURVEY
    8(e)): distinct devices of one host, or one device repeated as virtual
    ranks.  The proof is byte-identical to Context.prove's."""

    def __init__(self, contexts: Sequence[Context]):
        self.contexts = list(contexts)
        arr = (ctypes.c_void_p * len(self.contexts))(*[c.h.value for c in self.contexts])
        g = ctypes.c_void_p()
        L.check(L.lib().lsp_group_create(arr, len(self.contexts), ctypes.byref(g)))
        self.h = g

    def close(self):
        if self.h:
            L.lib().lsp_group_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def prove(self, traces, air: LineaAIR, public_values: np.ndarray, h: Optional[int] = None,
              w: Optional[int] = None) -> bytes:
        """`traces`: one (h, w, 4) host array (every rank copies it), or a list of
        per-rank device pointers (ints) with h and w given."""
        desc = (ctypes.c_int32 * len(air.descriptor()))(*air.descriptor())
        pub = _fr_arr(public_values).reshape(-1, 4)
        G = len(self.contexts)
        proof = ctypes.c_void_p()
        if isinstance(traces, (list, tuple)):
            ptrs = (ctypes.c_void_p * G)(*traces)
            mem = L.LSP_MEM_DEVICE
        else:
            t = _fr_arr(traces)
            h, w = t.shape[0], t.shape[1]
            ptrs = (ctypes.c_void_p * G)(*([t.ctypes.data] * G))
            mem = L.LSP_MEM_HOST
        L.check(L.lib().lsp_prove_group(self.h, ptrs, h, w, desc, len(desc), _ptr(pub), pub.shape[0], mem,
                                        ctypes.byref(proof)), self.contexts[0].h)
        return _take_proof(proof)


def prove(config: StarkConfig, air: LineaAIR, trace: np.ndarray, public_values: np.ndarray,
          ctx: Optional[Context] = None) -> bytes:
    """p3_uni_stark::prove(&config, &air, &mut challenger, trace, &public_values)."""
    own = ctx is None
    ctx = ctx or Context(config)
    try:
        return ctx.prove(trace, air, public_values)
    finally:
        if own:
            ctx.close()


def verify(config: StarkConfig, air: LineaAIR, proof: bytes, public_values: np.ndarray,
           ctx: Optional[Context] = None) -> bool:
    own = ctx is None
    ctx = ctx or Context(config)
    try:
        return ctx.verify(proof, air, public_values)
    finally:
        if own:
            ctx.close()


__all__ = ["StarkConfig", "Context", "Radix2DitParallel", "MerkleTreeMmcs", "MerkleTree",
           "TwoAdicFriGenericConfig", "gen_permutation_trace", "gen_wide_trace", "prove", "verify", "to_mont"]
