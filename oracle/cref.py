"""ctypes wrapper around the C restatement ``oracle/_build/liblsp_oracle.so``.

TEST INFRASTRUCTURE ONLY (checker and timed CPU baseline) -- see lsp_oracle.h.
Elements cross this boundary as 32-byte little-endian Montgomery limbs
(ark-ff in-memory form), the same encoding as the product C-ABI.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

from . import pyoracle as O

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "_build", "liblsp_oracle.so")


class Params(ctypes.Structure):
    _fields_ = [("sbox_degree", ctypes.c_uint32), ("rounds_f", ctypes.c_uint32),
                ("rounds_p", ctypes.c_uint32),
                ("ext_initial", ctypes.c_uint64 * (8 * 3 * 4)),
                ("ext_terminal", ctypes.c_uint64 * (8 * 3 * 4)),
                ("internal", ctypes.c_uint64 * (64 * 4)),
                ("alpha", ctypes.c_uint64 * 4), ("delta", ctypes.c_uint64 * 4),
                ("generic_lin", ctypes.c_uint32),
                ("ext_mds", ctypes.c_uint64 * (9 * 4)), ("int_diag", ctypes.c_uint64 * (3 * 4))]


class Fri(ctypes.Structure):
    _fields_ = [("log_blowup", ctypes.c_uint32), ("log_final_poly_len", ctypes.c_uint32),
                ("num_queries", ctypes.c_uint32), ("pow_bits", ctypes.c_uint32),
                ("transcript", ctypes.c_uint32)]  # LO_T_* mask (U7/U8/U12), 0 = defaults


class Debug(ctypes.Structure):
    _fields_ = [("trace_lde", ctypes.c_void_p), ("trace_layers", ctypes.c_void_p),
                ("quotient", ctypes.c_void_p), ("quotient_lde", ctypes.c_void_p),
                ("quotient_layers", ctypes.c_void_p), ("fri_input", ctypes.c_void_p),
                ("challenges", ctypes.c_uint64 * 16)]


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            build()
        L = ctypes.CDLL(LIB_PATH)
        L.lo_prove.restype = ctypes.c_int
        L.lo_verify.restype = ctypes.c_int
        L.lo_log_quotient_degree.restype = ctypes.c_int
        L.lo_gen_perm_trace.restype = ctypes.c_int
        _lib = L
    return _lib


# ---------------------------------------------------------------- encoding
def fr_buf(values) -> ctypes.Array:
    """python ints -> ctypes buffer of Montgomery limbs."""
    b = b"".join(O.to_mont_bytes(v) for v in values)
    return ctypes.create_string_buffer(b, len(b))


def buf_to_ints(buf, n: int, offset: int = 0):
    raw = ctypes.string_at(ctypes.addressof(buf) + offset * 32, n * 32)
    return [O.from_mont_bytes(raw[i * 32:(i + 1) * 32]) for i in range(n)]


def air_desc(cfgs) -> list:
    """Encode pyoracle configs into the int32 AIR descriptor of include/lsp.h."""
    out = [len(cfgs)]
    for c in cfgs:
        if isinstance(c, O.PermCfg):
            out += [1, len(c.a_cols), len(c.b_cols)] + list(c.a_cols) + list(c.b_cols) + [c.b_inv, c.check]
        else:
            out += [2, len(c.a_cols)] + list(c.a_cols) + [len(c.b_cols), len(c.b_cols[0])]
            for t in c.b_cols:
                out += list(t)
            out += [c.a_filter] + list(c.b_filter) + [c.a_inv] + list(c.b_inv) + list(c.occ) + [c.check]
    return out


def params_from_setup(s: O.Setup) -> Params:
    p = Params()
    p.sbox_degree, p.rounds_f, p.rounds_p = s.perm.sbox_degree, s.perm.rounds_f, s.perm.rounds_p

    def put(arr, idx, v):
        raw = O.to_mont_bytes(v)
        for k in range(4):
            arr[idx * 4 + k] = int.from_bytes(raw[8 * k:8 * k + 8], "little")
    for r, rc in enumerate(s.perm.ext_initial):
        for j in range(3):
            put(p.ext_initial, r * 3 + j, rc[j])
    for r, rc in enumerate(s.perm.ext_terminal):
        for j in range(3):
            put(p.ext_terminal, r * 3 + j, rc[j])
    for r, rc in enumerate(s.perm.internal):
        put(p.internal, r, rc)
    put(p.alpha, 0, s.alpha)
    put(p.delta, 0, s.delta)
    set_linear_layers(p, s.perm.int_diag, s.perm.ext_mds)
    return p


def _put(arr, idx, v):
    raw = O.to_mont_bytes(v)
    for k in range(4):
        arr[idx * 4 + k] = int.from_bytes(raw[8 * k:8 * k + 8], "little")


def set_linear_layers(p: Params, int_diag=None, ext_mds=None) -> Params:
    """U2/U3: internal diag d (3 ints) and external M_E (9 ints, row-major);
    None = the default layer.  Both None -> generic_lin = 0 (default path)."""
    if int_diag is None and ext_mds is None:
        p.generic_lin = 0
        return p
    d = O.DEFAULT_INT_DIAG if int_diag is None else int_diag
    m = O.DEFAULT_EXT_MDS if ext_mds is None else ext_mds
    assert len(d) == 3 and len(m) == 9
    for i, v in enumerate(m):
        _put(p.ext_mds, i, v % O.P)
    for i, v in enumerate(d):
        _put(p.int_diag, i, v % O.P)
    p.generic_lin = 1
    return p


def setup(seed: int = O.DEFAULT_SEED, sbox_degree=11, rounds_f=8, rounds_p=22, int_diag=None,
          ext_mds=None) -> Params:
    p = Params()
    lib().lo_setup(ctypes.c_uint64(seed), sbox_degree, rounds_f, rounds_p, ctypes.byref(p))
    return set_linear_layers(p, int_diag, ext_mds)


def fri_params(fp: O.FriParams = O.FriParams()) -> Fri:
    return Fri(fp.log_blowup, fp.log_final_poly_len, fp.num_queries, fp.proof_of_work_bits, fp.transcript_bits())


def gen_perm_trace(p: Params, log_n: int, ncols: int, seed: int = O.DEFAULT_SEED, small=False):
    n, w = 1 << log_n, 2 * ncols + 2
    buf = ctypes.create_string_buffer(n * w * 32)
    rc = lib().lo_gen_perm_trace(log_n, ncols, ctypes.byref(p.alpha), ctypes.byref(p.delta),
                                 ctypes.c_uint64(seed), int(small), buf)
    assert rc == 0
    return buf, w


def perm_air(ncols: int) -> list:
    w = ncols
    return [1, 1, w, w] + list(range(w)) + list(range(w, 2 * w)) + [2 * w, 2 * w + 1]


def prove(p: Params, trace_buf, h: int, w: int, air: list, fri: Fri = None, public_degree=1,
          nthreads=None, debug: bool = False):
    fri = fri or fri_params()
    nthreads = nthreads or (os.cpu_count() or 1)
    arr = (ctypes.c_int32 * len(air))(*air)
    out = ctypes.POINTER(ctypes.c_uint8)()
    ln = ctypes.c_size_t()
    dbg = None
    bufs = {}
    if debug:
        N = h << fri.log_blowup
        lq = lib().lo_log_quotient_degree(arr, len(air), public_degree)
        q = 1 << lq
        bufs = dict(trace_lde=N * w, trace_layers=2 * N - 1, quotient=h * q, quotient_lde=N * q,
                    quotient_layers=2 * N - 1, fri_input=N)
        bufs = {k: ctypes.create_string_buffer(v * 32) for k, v in bufs.items()}
        dbg = Debug()
        for k, b in bufs.items():
            setattr(dbg, k, ctypes.addressof(b))
    if isinstance(trace_buf, int):
        trace_buf = ctypes.c_void_p(trace_buf)
    rc = lib().lo_prove(ctypes.byref(p), ctypes.byref(fri), trace_buf, ctypes.c_size_t(h), ctypes.c_size_t(w),
                        arr, ctypes.c_size_t(len(air)), public_degree, nthreads, ctypes.byref(out),
                        ctypes.byref(ln), ctypes.byref(dbg) if dbg is not None else None)
    if rc != 0:
        raise RuntimeError(f"lo_prove failed: {rc}")
    proof = ctypes.string_at(out, ln.value)
    lib().lo_free(out)
    if debug:
        bufs["challenges"] = dbg.challenges
        return proof, bufs
    return proof


def verify(p: Params, proof: bytes, air: list, fri: Fri = None, public_degree=1) -> int:
    fri = fri or fri_params()
    arr = (ctypes.c_int32 * len(air))(*air)
    return lib().lo_verify(ctypes.byref(p), ctypes.byref(fri), arr, ctypes.c_size_t(len(air)), public_degree,
                           proof, ctypes.c_size_t(len(proof)))
