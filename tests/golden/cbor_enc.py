"""Minimal CBOR encoder shaped like serde + ciborium output for the trace
crate's structs (a map of field names; Vec -> array; [u8; 32] -> array of 32
uints, or a byte string with words_as_bytes) -- test infrastructure for the
F4 input path.  `python tests/golden/cbor_enc.py` rewrites the fixtures."""
import os
import struct


def _head(major: int, n: int) -> bytes:
    if n < 24:
        return bytes([major << 5 | n])
    if n < 1 << 8:
        return bytes([major << 5 | 24, n])
    if n < 1 << 16:
        return bytes([major << 5 | 25]) + struct.pack(">H", n)
    if n < 1 << 32:
        return bytes([major << 5 | 26]) + struct.pack(">I", n)
    return bytes([major << 5 | 27]) + struct.pack(">Q", n)


def enc(x, words_as_bytes=False, indefinite=False) -> bytes:
    if isinstance(x, bool) or x is None:
        raise TypeError("unsupported")
    if isinstance(x, int):
        return _head(0, x)
    if isinstance(x, str):
        b = x.encode()
        return _head(3, len(b)) + b
    if isinstance(x, (bytes, bytearray)):
        if len(x) == 32 and not words_as_bytes:  # [u8; 32] as serde's tuple
            return _head(4, 32) + b"".join(_head(0, v) for v in x)
        return _head(2, len(x)) + bytes(x)
    if isinstance(x, dict):
        out = _head(5, len(x))
        for k, v in x.items():
            out += enc(k) + enc(v, words_as_bytes, indefinite)
        return out
    if isinstance(x, (list, tuple)):
        body = b"".join(enc(v, words_as_bytes, indefinite) for v in x)
        return (bytes([0x9f]) + body + b"\xff") if indefinite else _head(4, len(x)) + body
    raise TypeError(type(x))


def word(v: int) -> bytes:
    return v.to_bytes(32, "big")


def permutation_trace(a, b, name="perm") -> dict:
    return {"a": [[word(v) for v in c] for c in a], "b": [[word(v) for v in c] for c in b], "name": name}


def lookup_trace(a, b, a_filter, b_filter, name="lookup") -> dict:
    return {"a": [[word(v) for v in c] for c in a], "b": [[[word(v) for v in c] for c in t] for t in b],
            "name": name, "a_filter": [word(v) for v in a_filter],
            "b_filter": [[word(v) for v in f] for f in b_filter]}


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    # a 4-row 1+1 permutation (b = a reversed) and an 8-row lookup with a value >= r
    r = 0x12AB655E9A2CA55660B44D1E5C37B00159AA76FED00000010A11800000000001
    a = [[5, 7, 9, (1 << 256) - 1]]
    with open(os.path.join(here, "perm_small.cbor"), "wb") as f:
        f.write(enc(permutation_trace(a, [list(reversed(a[0]))])))
    tab = [[1, 2, 3, 4, r + 1, 6, 7, 8]]
    la = [[2, 2, 3, r + 1, 1, 8, 8, 8]]
    with open(os.path.join(here, "lookup_small.cbor"), "wb") as f:
        f.write(enc(lookup_trace(la, [tab], [1] * 8, [[1] * 8])))
