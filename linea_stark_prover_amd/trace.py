"""The reference's ``trace`` crate on the device.

``RawPermutationTrace`` / ``RawLookupTrace`` hold raw columns (trace/src/
permutation.rs:9-14, trace/src/lookup.rs:10-17) as Montgomery-form Fr arrays
of shape (n, 4) uint64; ``RawTrace.push_traces`` (trace/src/lib.rs:62-92)
pads every block to the common height, then generates each block's witness
columns on the GPU (lsp_witness_lookup / lsp_witness_permutation: row
combinations, batch inversion, prefix products / sums, LogUp
multiplicities) directly into one row-major device trace in push order
(lookups first), returning the shifted AirConfigs.  ``get_trace`` returns the
device pointer (what ``Context.prove`` takes) or a host copy.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass, field
from typing import List, Optional, Sequence, Tuple

import numpy as np

from . import _lib as L
from .air import AirLookupConfig, AirPermutationConfig, LineaAIR
from .field import to_mont
from .prover import Context, _fr_arr, _ptr


def _parse_cbor(data: bytes):
    """lsp_raw_trace_parse -> (kind, na, ntables, nbc, height, columns (k, height, 4))"""
    h = ctypes.c_void_p()
    L.check(L.lib().lsp_raw_trace_parse(data, len(data), ctypes.byref(h)))
    try:
        kind, na, nt, nbc = ctypes.c_int(), ctypes.c_uint32(), ctypes.c_uint32(), ctypes.c_uint32()
        mh, w = ctypes.c_size_t(), ctypes.c_size_t()
        L.check(L.lib().lsp_raw_trace_shape(h, ctypes.byref(kind), ctypes.byref(na), ctypes.byref(nt),
                                            ctypes.byref(nbc), ctypes.byref(mh), ctypes.byref(w)))
        n = ctypes.c_size_t()
        L.check(L.lib().lsp_raw_trace_columns(h, mh.value, None, 0, ctypes.byref(n)))
        cols = np.zeros((n.value, 4), np.uint64)
        L.check(L.lib().lsp_raw_trace_columns(h, mh.value, _ptr(cols), n.value, ctypes.byref(n)))
        height = mh.value
        return kind.value, na.value, nt.value, nbc.value, height, cols.reshape(-1, height, 4) if height else cols
    finally:
        L.lib().lsp_raw_trace_free(h)


def _read(path_or_bytes) -> bytes:
    if isinstance(path_or_bytes, (bytes, bytearray)):
        return bytes(path_or_bytes)
    with open(path_or_bytes, "rb") as f:
        return f.read()


def _col(c) -> np.ndarray:
    return _fr_arr(c).reshape(-1, 4)


@dataclass
class RawPermutationTrace:
    a: List[np.ndarray]
    b: List[np.ndarray]
    name: str = ""

    @staticmethod
    def read_file(path_or_bytes) -> "RawPermutationTrace":
        """trace/src/permutation.rs:17-22 (CBOR via the library's parser)"""
        kind, na, nb, _, h, cols = _parse_cbor(_read(path_or_bytes))
        if kind != L.LSP_AIR_PERMUTATION:
            raise ValueError("not a RawPermutationTrace")
        return RawPermutationTrace([cols[k] for k in range(na)], [cols[na + k] for k in range(nb)])

    def get_max_height(self) -> int:  # trace/src/permutation.rs:120-132
        return max(len(c) for c in list(self.a) + list(self.b))

    def width(self) -> int:
        return len(self.a) + len(self.b) + 2


@dataclass
class RawLookupTrace:
    a: List[np.ndarray]
    b: List[List[np.ndarray]]
    a_filter: Optional[np.ndarray] = None
    b_filter: List[np.ndarray] = field(default_factory=list)
    name: str = ""

    @staticmethod
    def read_file(path_or_bytes) -> "RawLookupTrace":
        """trace/src/lookup.rs:20-44 (CBOR via the library's parser; filter defaults applied)"""
        kind, na, nt, nbc, h, cols = _parse_cbor(_read(path_or_bytes))
        if kind != L.LSP_AIR_LOOKUP:
            raise ValueError("not a RawLookupTrace")
        a = [cols[k] for k in range(na)]
        b = [[cols[na + t * nbc + c] for c in range(nbc)] for t in range(nt)]
        af = cols[na + nt * nbc]
        bf = [cols[na + nt * nbc + 1 + t] for t in range(nt)]
        return RawLookupTrace(a, b, af, bf)

    def fill_filters(self) -> None:
        """RawLookupTrace::read_file's defaults (trace/src/lookup.rs:25-41): a
        missing filter entry is 1 (enabled)."""
        one = to_mont([1])[0]
        n = len(self.a[0])
        af = np.zeros((0, 4), np.uint64) if self.a_filter is None else _col(self.a_filter)
        if len(af) < n:
            af = np.concatenate([af, np.tile(one, (n - len(af), 1))])
        self.a_filter = af
        bfs = [_col(f) for f in self.b_filter]
        while len(bfs) < len(self.b):
            bfs.append(np.zeros((0, 4), np.uint64))
        for t, f in enumerate(bfs):
            m = len(self.b[t][0])
            if len(f) < m:
                bfs[t] = np.concatenate([f, np.tile(one, (m - len(f), 1))])
        self.b_filter = bfs

    def get_max_height(self) -> int:  # trace/src/lookup.rs:216-229
        return max([len(c) for c in self.a] + [len(c) for t in self.b for c in t])

    def width(self) -> int:
        return len(self.a) + len(self.b) * (len(self.b[0]) + 3) + 3


class RawTrace:
    """trace/src/lib.rs:17-107: the blocks of one trace, generated on `ctx`'s GPU."""

    def __init__(self, ctx: Context, challenges: Sequence[np.ndarray]):
        assert len(challenges) == 2, "Two challenges should be provided"
        self.ctx = ctx
        self.alpha = _col(challenges[0])[0].copy()
        self.delta = _col(challenges[1])[0].copy()
        self.height = 0
        self.width = 0
        self.ptr: Optional[int] = None

    def push_traces(self, permutation_traces: Sequence[RawPermutationTrace],
                    lookup_traces: Sequence[RawLookupTrace]) -> List:
        for lt in lookup_traces:  # one filter per table: the scratch below holds that many
            if len(lt.b_filter) > len(lt.b):
                raise ValueError(f"RawLookupTrace has {len(lt.b_filter)} b_filter columns for {len(lt.b)} tables")
        h = 0
        for t in list(lookup_traces) + list(permutation_traces):
            h = max(h, t.get_max_height())
        self.height = h
        self.width = sum(t.width() for t in lookup_traces) + sum(t.width() for t in permutation_traces)
        if self.ptr is not None:
            self.ctx.dev_free(self.ptr)
        self.ptr = self.ctx.dev_alloc(h * self.width * 32)
        # one device buffer for the raw columns of every block in turn (the
        # largest block's), instead of an allocation and a synchronizing free per block
        raw = [len(t.a) + sum(len(x) for x in t.b) + 1 + len(t.b) for t in lookup_traces] + \
              [len(t.a) + len(t.b) for t in permutation_traces]
        self._scratch_bytes = max(max(raw, default=1) * h * 32, 32)
        self._scratch = self.ctx.dev_alloc(self._scratch_bytes)
        try:
            cfgs, col = [], 0
            for lt in lookup_traces:  # lookups first (trace/src/lib.rs:81-89)
                cfg = self._push_lookup(lt, col)
                cfgs.append(cfg)
                col += lt.width()
            for pt in permutation_traces:
                cfgs.append(self._push_permutation(pt, col))
                col += pt.width()
        finally:
            self.ctx.dev_free(self._scratch)
            self._scratch = None
        return cfgs

    def air(self, cfgs) -> LineaAIR:
        return LineaAIR(list(cfgs))

    def _push_permutation(self, pt: RawPermutationTrace, col0: int) -> AirPermutationConfig:
        n = self.height
        na, nb = len(pt.a), len(pt.b)
        da = self._scratch
        db = self._upload_cols(pt.a, n, da)
        assert self._upload_cols(pt.b, n, db) - da <= self._scratch_bytes, "raw columns overran the scratch buffer"
        self.ctx._chk(L.lib().lsp_witness_permutation(
            self.ctx.h, da, na, db, nb, n, _ptr(self.alpha), _ptr(self.delta), self.ptr, self.width, col0,
            L.LSP_MEM_DEVICE))
        cfg = AirPermutationConfig(list(range(na)), list(range(na, na + nb)), na + nb, na + nb + 1)
        cfg.shift(col0)
        return cfg

    def _push_lookup(self, lt: RawLookupTrace, col0: int) -> AirLookupConfig:
        n = self.height
        lt.fill_filters()
        nt, nbc, na = len(lt.b), len(lt.b[0]), len(lt.a)
        ptrs = [self._scratch]
        for cols in (lt.a, [c for t in lt.b for c in t], [lt.a_filter], list(lt.b_filter)):
            ptrs.append(self._upload_cols(cols, n, ptrs[-1]))
        # the scratch was sized in push_traces for exactly these columns
        assert ptrs[-1] - self._scratch <= self._scratch_bytes, "raw columns overran the scratch buffer"
        self.ctx._chk(L.lib().lsp_witness_lookup(
            self.ctx.h, ptrs[0], na, ptrs[1], nt, nbc, ptrs[2], ptrs[3], n, _ptr(self.alpha),
            _ptr(self.delta), self.ptr, self.width, col0, L.LSP_MEM_DEVICE))
        # column ids (trace/src/lookup.rs:178-214)
        a_ids = list(range(na))
        b_ids = [[na + t * nbc + c for c in range(nbc)] for t in range(nt)]
        af_id = na + nt * nbc
        bf_ids = [af_id + 1 + t for t in range(nt)]
        ai_id = af_id + 1 + nt
        bi_ids = [ai_id + 1 + t for t in range(nt)]
        oc_ids = [ai_id + 1 + nt + t for t in range(nt)]
        cfg = AirLookupConfig(a_ids, b_ids, af_id, bf_ids, ai_id, bi_ids, oc_ids, ai_id + 1 + 2 * nt)
        cfg.shift(col0)
        return cfg

    def _upload_cols(self, cols, n: int, p: int) -> int:
        """len(cols) columns of n elements each, column-major at device address
        p, each column straight from its own array (no stacked host copy); a
        short column's tail is zeros (Vec::resize(n, [0u8; 32]):
        trace/src/permutation.rs:134-140, trace/src/lookup.rs:231-245).
        Returns the address after the last column."""
        zeros = None
        for k, c in enumerate(cols):
            c = _col(c)
            m = min(c.shape[0], n)
            if m:
                self.ctx.h2d(p + k * n * 32, c[:m])
            if m < n:
                if zeros is None or zeros.shape[0] < n - m:
                    zeros = np.zeros((n - m, 4), np.uint64)
                self.ctx.h2d(p + (k * n + m) * 32, zeros[:n - m])
        return p + len(cols) * n * 32

    def get_trace(self, host: bool = False):
        """(device pointer, height, width), or the (height, width, 4) host matrix"""
        if not host:
            return self.ptr, self.height, self.width
        out = np.zeros((self.height, self.width, 4), np.uint64)
        self.ctx.d2h(out, self.ptr)
        return out

    def close(self):
        if self.ptr is not None:
            self.ctx.dev_free(self.ptr)
            self.ptr = None
