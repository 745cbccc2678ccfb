"""ctypes binding of liblsp_hip.so (include/lsp.h).

The library is the product: there is no CPU fallback.  If it is missing or
cannot be loaded this module raises; if no GPU is present, calls that need
one return LSP_E_STATE and raise LspError.
"""
from __future__ import annotations

import ctypes
import os

_PKG = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LSP_LIB", os.path.join(_PKG, "_lib", "liblsp_hip.so"))

LSP_OK, LSP_E_ARG, LSP_E_OOM, LSP_E_HIP, LSP_E_SIZE, LSP_E_VERIFY, LSP_E_STATE = range(7)
LSP_MEM_HOST, LSP_MEM_DEVICE = 0, 1
LSP_AIR_PERMUTATION, LSP_AIR_LOOKUP = 1, 2

c_fr_p = ctypes.c_void_p  # lsp_fr* (32-byte elements)


class LspParams(ctypes.Structure):
    """include/lsp.h lsp_params; keyword construction, struct_size filled in.
    The U7/U8/U12 transcript switches default to 0 (SURVEY 8(c)'s choices)."""
    _fields_ = [("struct_size", ctypes.c_uint32),
                ("sbox_degree", ctypes.c_uint32), ("rounds_f", ctypes.c_uint32), ("rounds_p", ctypes.c_uint32),
                ("round_constants", ctypes.c_void_p), ("log_blowup", ctypes.c_uint32),
                ("log_final_poly_len", ctypes.c_uint32), ("num_queries", ctypes.c_uint32),
                ("proof_of_work_bits", ctypes.c_uint32), ("public_degree", ctypes.c_int32),
                ("internal_diag", ctypes.c_void_p), ("external_mds", ctypes.c_void_p),
                ("skip_log_degree", ctypes.c_uint32), ("skip_public_values", ctypes.c_uint32),
                ("observe_opened_values", ctypes.c_uint32), ("sample_bits_montgomery", ctypes.c_uint32),
                ("skip_final_poly", ctypes.c_uint32)]

    def __init__(self, **kw):
        super().__init__(struct_size=ctypes.sizeof(LspParams), **kw)


TRANSCRIPT_SWITCHES = ("skip_log_degree", "skip_public_values", "observe_opened_values", "sample_bits_montgomery",
                       "skip_final_poly")


ALLGATHER_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t)
BCAST_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int)


class LspCommOps(ctypes.Structure):
    _fields_ = [("rank", ctypes.c_int), ("size", ctypes.c_int), ("user", ctypes.c_void_p),
                ("allgather", ALLGATHER_FN), ("bcast", BCAST_FN)]


class LspError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"lsp error {code}: {msg}")
        self.code = code


# name -> (restype, argtypes)
_SIGS = {
    "lsp_version": (ctypes.c_char_p, []),
    "lsp_debug_bounds_probe": (ctypes.c_int, [ctypes.c_void_p]),
    "lsp_device_count": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int)]),
    "lsp_last_error": (ctypes.c_char_p, [ctypes.c_void_p]),
    "lsp_seeded_setup": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, c_fr_p, c_fr_p, c_fr_p]),
    "lsp_fr_from_canonical": (None, [ctypes.c_void_p, c_fr_p]),
    "lsp_fr_to_canonical": (None, [c_fr_p, ctypes.c_void_p]),
    "lsp_fr_from_be_bytes_mod_order": (None, [ctypes.c_char_p, ctypes.c_size_t, c_fr_p]),
    "lsp_fr_mul": (None, [c_fr_p, c_fr_p, c_fr_p]),
    "lsp_fr_inv": (None, [c_fr_p, c_fr_p]),
    "lsp_two_adic_generator": (None, [ctypes.c_uint32, c_fr_p]),
    "lsp_ctx_create": (ctypes.c_int, [ctypes.c_int, ctypes.POINTER(LspParams), ctypes.POINTER(ctypes.c_void_p)]),
    "lsp_ctx_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "lsp_synchronize": (ctypes.c_int, [ctypes.c_void_p]),
    "lsp_dev_alloc": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    "lsp_dev_free": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "lsp_memcpy_h2d": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "lsp_memcpy_d2h": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t]),
    "lsp_coset_lde_batch": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_size_t,
                                           ctypes.c_uint32, c_fr_p, c_fr_p, ctypes.c_int]),
    "lsp_coset_lde_batch_shifts": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_size_t,
                                                  ctypes.c_uint32, c_fr_p, c_fr_p, ctypes.c_int]),
    "lsp_coset_dft_batch": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_size_t, c_fr_p, c_fr_p,
                                           ctypes.c_int]),
    "lsp_coset_idft_batch": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_size_t, c_fr_p, c_fr_p,
                                            ctypes.c_int]),
    "lsp_poseidon2_permute_batch": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_int]),
    "lsp_hash_rows": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_size_t, c_fr_p,
                                     ctypes.c_int]),
    "lsp_merkle_commit": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                         ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_size_t,
                                         ctypes.c_int, c_fr_p, ctypes.POINTER(ctypes.c_void_p)]),
    "lsp_merkle_open": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, c_fr_p, c_fr_p]),
    "lsp_merkle_layer": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, c_fr_p]),
    "lsp_merkle_verify": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t,
                                         ctypes.c_uint32, ctypes.c_size_t, c_fr_p, c_fr_p]),
    "lsp_tree_free": (ctypes.c_int, [ctypes.c_void_p]),
    "lsp_fri_fold": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, c_fr_p, c_fr_p, ctypes.c_int]),
    "lsp_fri_fold_row": (None, [ctypes.c_size_t, ctypes.c_uint32, c_fr_p, c_fr_p, c_fr_p, c_fr_p]),
    "lsp_log_quotient_degree": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32,
                                               ctypes.POINTER(ctypes.c_uint32)]),
    "lsp_quotient_values": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_size_t,
                                           ctypes.c_void_p, ctypes.c_size_t, c_fr_p, ctypes.c_size_t, c_fr_p,
                                           c_fr_p, ctypes.c_int]),
    "lsp_interpolate_coset": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_size_t, c_fr_p,
                                             c_fr_p, c_fr_p, ctypes.c_int]),
    "lsp_inverse_denominators": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_uint32, c_fr_p,
                                                c_fr_p, ctypes.c_int]),
    "lsp_open_reduce": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_size_t, c_fr_p, c_fr_p,
                                       ctypes.c_size_t, c_fr_p, c_fr_p, c_fr_p, ctypes.c_int]),
    "lsp_host_compress_batch": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, c_fr_p]),
    "lsp_host_hash_rows": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_size_t, c_fr_p]),
    "lsp_batch_inverse": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, c_fr_p, ctypes.c_int]),
    "lsp_prove": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                                 ctypes.c_size_t, c_fr_p, ctypes.c_size_t, ctypes.c_int,
                                 ctypes.POINTER(ctypes.c_void_p)]),
    "lsp_proof_serialize": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                                           ctypes.POINTER(ctypes.c_size_t)]),
    "lsp_proof_free": (ctypes.c_int, [ctypes.c_void_p]),
    "lsp_proof_deserialize": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    "lsp_proof_get_view": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),  # lsp_proof_view* (proof.py)
    "lsp_proof_from_view": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)]),
    "lsp_ctx_attach_comm_ops": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(LspCommOps)]),
    "lsp_comm_rccl_unique_id": (ctypes.c_int, [ctypes.c_void_p]),
    "lsp_ctx_attach_rccl": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "lsp_ctx_detach_comm": (ctypes.c_int, [ctypes.c_void_p]),
    "lsp_ctx_attach_loopback": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.c_int]),
    "lsp_ctx_mem_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_size_t),
                                         ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]),
    "lsp_ctx_set_phase_timing": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                                ctypes.c_size_t]),
    "lsp_comm_selftest": (ctypes.c_int, [ctypes.c_void_p]),
    "lsp_comm_calibration": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.c_size_t,
                                            ctypes.POINTER(ctypes.c_size_t)]),
    "lsp_comm_quotient_exchange": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t,
                                                  ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t),
                                                  ctypes.POINTER(ctypes.c_double)]),
    "lsp_comm_exchange_plan": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_size_t,
                                              ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double),
                                              ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_int),
                                              ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_double)]),
    "lsp_ctx_host_threads": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]),
    "lsp_comm_info": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_int)]),
    "lsp_comm_log": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_size_t),
                                    ctypes.POINTER(ctypes.c_int), ctypes.POINTER(ctypes.c_double),
                                    ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_double)]),
    "lsp_prove_sharded": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p,
                                         ctypes.c_size_t, c_fr_p, ctypes.c_size_t, ctypes.c_int,
                                         ctypes.POINTER(ctypes.c_void_p)]),
    "lsp_group_create": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int,
                                        ctypes.POINTER(ctypes.c_void_p)]),
    "lsp_group_destroy": (ctypes.c_int, [ctypes.c_void_p]),
    "lsp_prove_group": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t,
                                       ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, c_fr_p, ctypes.c_size_t,
                                       ctypes.c_int, ctypes.POINTER(ctypes.c_void_p)]),
    "lsp_verify": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, c_fr_p, ctypes.c_size_t,
                                  ctypes.c_char_p, ctypes.c_size_t]),
    "lsp_last_timings": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double),
                                        ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t,
                                        ctypes.POINTER(ctypes.c_size_t)]),
    "lsp_last_spans": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_char_p), ctypes.c_size_t,
                                      ctypes.POINTER(ctypes.c_size_t)]),
    "lsp_gen_wide_trace": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                          ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32, c_fr_p, c_fr_p, c_fr_p,
                                          ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_size_t), ctypes.POINTER(ctypes.c_size_t)]),
    "lsp_calibrate_fr_mul": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]),
    "lsp_witness_permutation": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_uint32, c_fr_p, ctypes.c_uint32,
                                               ctypes.c_size_t, c_fr_p, c_fr_p, c_fr_p, ctypes.c_size_t,
                                               ctypes.c_size_t, ctypes.c_int]),
    "lsp_witness_lookup": (ctypes.c_int, [ctypes.c_void_p, c_fr_p, ctypes.c_uint32, c_fr_p, ctypes.c_uint32,
                                          ctypes.c_uint32, c_fr_p, c_fr_p, ctypes.c_size_t, c_fr_p, c_fr_p, c_fr_p,
                                          ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]),
    "lsp_raw_trace_parse": (ctypes.c_int, [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p)]),
    "lsp_raw_trace_shape": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_int),
                                           ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                           ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_size_t),
                                           ctypes.POINTER(ctypes.c_size_t)]),
    "lsp_raw_trace_columns": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t, c_fr_p, ctypes.c_size_t,
                                             ctypes.POINTER(ctypes.c_size_t)]),
    "lsp_raw_trace_push": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, c_fr_p, c_fr_p, c_fr_p,
                                          ctypes.c_size_t, ctypes.c_size_t, ctypes.c_int]),
    "lsp_raw_trace_free": (ctypes.c_int, [ctypes.c_void_p]),
    "lsp_calibrate_poseidon2": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_double)]),
    "lsp_calibrate_intt": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_size_t,
                                          ctypes.POINTER(ctypes.c_double)]),
    "lsp_gen_permutation_trace": (ctypes.c_int, [ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, c_fr_p, c_fr_p,
                                                 ctypes.c_int, c_fr_p]),
    "lsp_gen_permutation_trace_device": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint32,
                                                        ctypes.c_uint32, c_fr_p, c_fr_p, c_fr_p]),
}

EXPORTED = sorted(_SIGS)

_lib = None


def lib() -> ctypes.CDLL:
    """Load liblsp_hip.so (raises if the HIP extension was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"liblsp_hip.so not found at {LIB_PATH}; run "
                              "`python -m linea_stark_prover_amd.build` (no CPU fallback exists)")
        L = ctypes.CDLL(LIB_PATH)
        # an older build chosen for an A/B (LSP_LIB_OLDER=1 beside LSP_LIB) may
        # lack later entry points; the product library must export them all
        older = os.environ.get("LSP_LIB_OLDER") == "1"
        for name, (res, args) in _SIGS.items():
            f = getattr(L, name, None) if older else getattr(L, name)
            if f is None:
                continue
            f.restype = res
            f.argtypes = args
        _lib = L
    return _lib


def check(rc: int, ctx=None):
    if rc != LSP_OK:
        msg = lib().lsp_last_error(ctx)
        raise LspError(rc, msg.decode() if msg else "")
