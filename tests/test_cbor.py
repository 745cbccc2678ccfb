"""F4: CBOR RawPermutationTrace / RawLookupTrace input through the library's
native parser (lsp_raw_trace_parse) -- host only, no GPU."""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import cbor_enc as C  # noqa: E402

R = 0x12AB655E9A2CA55660B44D1E5C37B00159AA76FED00000010A11800000000001


def _vals(col):
    from linea_stark_prover_amd.field import from_mont
    return from_mont(np.asarray(col))


def test_fixture_permutation(product_lib):
    from linea_stark_prover_amd.trace import RawPermutationTrace
    t = RawPermutationTrace.read_file(os.path.join(HERE, "golden", "perm_small.cbor"))
    top = ((1 << 256) - 1) % R  # from_be_bytes_mod_order
    assert [_vals(c) for c in t.a] == [[5, 7, 9, top]]
    assert [_vals(c) for c in t.b] == [[top, 9, 7, 5]]


def test_fixture_lookup(product_lib):
    from linea_stark_prover_amd.trace import RawLookupTrace
    t = RawLookupTrace.read_file(os.path.join(HERE, "golden", "lookup_small.cbor"))
    assert _vals(t.a[0]) == [2, 2, 3, 1, 1, 8, 8, 8]      # r + 1 -> 1
    assert _vals(t.b[0][0]) == [1, 2, 3, 4, 1, 6, 7, 8]
    assert _vals(t.a_filter) == [1] * 8 and _vals(t.b_filter[0]) == [1] * 8


@pytest.mark.parametrize("words_as_bytes,indefinite", [(False, False), (True, False), (False, True)])
def test_random_lookup_round_trip(product_lib, words_as_bytes, indefinite):
    from linea_stark_prover_amd.trace import RawLookupTrace
    g = np.random.default_rng(3)
    n, nt, nbc = 37, 2, 3
    rnd = lambda: int.from_bytes(g.bytes(32), "big")  # noqa: E731  (any 256-bit word, reduced mod r)
    a = [[rnd() for _ in range(n)] for _ in range(nbc)]
    b = [[[rnd() for _ in range(n + 5)] for _ in range(nbc)] for _ in range(nt)]
    af = [int(g.integers(0, 2)) for _ in range(n)]
    bf = [[int(g.integers(0, 2)) for _ in range(n + 5)] for _ in range(nt)]
    data = C.enc(C.lookup_trace(a, b, af, bf), words_as_bytes, indefinite)
    t = RawLookupTrace.read_file(data)
    h = n + 5  # every column comes back resized to the max height with zero words
    pad = lambda c: [v % R for v in c] + [0] * (h - len(c))  # noqa: E731
    assert [_vals(c) for c in t.a] == [pad(c) for c in a]
    assert [[_vals(c) for c in tab] for tab in t.b] == [[pad(c) for c in tab] for tab in b]
    assert _vals(t.a_filter) == pad(af)
    assert [_vals(f) for f in t.b_filter] == [pad(f) for f in bf]


def test_missing_filters_default_to_one(product_lib):
    from linea_stark_prover_amd.trace import RawLookupTrace
    d = C.lookup_trace([[1, 2, 3]], [[[1, 2, 3, 4]]], [1], [])
    t = RawLookupTrace.read_file(C.enc(d))
    # read_file pads a_filter to len(a[0]) with 1, b_filter to len(b[t][0]) with 1; then the
    # RawTrace resize pads every column to the max height (4) with zero words
    assert _vals(t.a_filter) == [1, 1, 1, 0]
    assert _vals(t.b_filter[0]) == [1, 1, 1, 1]


def test_unknown_keys_are_skipped(product_lib):
    from linea_stark_prover_amd.trace import RawPermutationTrace
    d = C.permutation_trace([[1, 2]], [[2, 1]])
    d["extra"] = [{"x": b"\x00" * 5}, "text", 7]
    t = RawPermutationTrace.read_file(C.enc(d))
    assert [_vals(c) for c in t.a] == [[1, 2]]


@pytest.mark.parametrize("data,msg", [
    (C.enc([1, 2]), "map"),
    (C.enc({"a": [[b"\x01" * 31]], "b": [[C.word(1)]]}, words_as_bytes=True), "32"),
    (C.enc({"a": [[[300] + [0] * 31]], "b": [[C.word(1)]]}), "exceeds 255"),
    (C.enc(C.permutation_trace([[1]], [[1]]))[:-3], "truncated"),
    (C.enc(C.permutation_trace([[1]], [[1]])) + b"\x00", "trailing"),
    (C.enc({"name": "no columns"}), "non-empty"),
])
def test_malformed_input_is_rejected(product_lib, data, msg):
    from linea_stark_prover_amd import _lib
    from linea_stark_prover_amd.trace import RawPermutationTrace
    with pytest.raises(_lib.LspError, match=msg) as e:
        RawPermutationTrace.read_file(data)
    assert e.value.code == _lib.LSP_E_ARG


def test_kind_mismatch(product_lib):
    from linea_stark_prover_amd.trace import RawLookupTrace, RawPermutationTrace
    with pytest.raises(ValueError):
        RawLookupTrace.read_file(os.path.join(HERE, "golden", "perm_small.cbor"))
    with pytest.raises(ValueError):
        RawPermutationTrace.read_file(os.path.join(HERE, "golden", "lookup_small.cbor"))
