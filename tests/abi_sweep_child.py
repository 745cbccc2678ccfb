"""Child process of tests/test_abi_sweep.py: calls C-ABI entry points of
liblsp_hip.so with NULL pointers and prints one JSON line per call (the case
line goes out before the call, so a crash names the call that faulted).

    python tests/abi_sweep_child.py all-null     # every pointer NULL, every size 1
    python tests/abi_sweep_child.py one-null     # one pointer NULL at a time, the
                                                 # others 1 MiB zeroed host buffers

A host-only context (LSP_HOST_ONLY) stands in for lsp_ctx* in one-null mode:
no GPU is touched, so device entry points stop at their state check and the
host ones (verify, Merkle verify, the AIR parser, proofs, CBOR traces, field
helpers) run their argument checks for real.  Opaque handles (lsp_tree*,
lsp_proof*, lsp_raw_trace*, lsp_group*) are always NULL: a dummy buffer is
not an object.
"""
import ctypes
import json
import os
import re
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from linea_stark_prover_amd import _lib  # noqa: E402

HANDLE = re.compile(r"\s*(const\s+)?(lsp_tree|lsp_proof|lsp_raw_trace|lsp_group)\s*\*\s*\w+$")
CTX = re.compile(r"\s*(const\s+)?lsp_ctx\s*\*\s*\w+$")
# the first argument is the object they release: a host context there would be freed twice
RELEASERS = {"lsp_ctx_destroy"}


def header_params():
    h = open(os.path.join(ROOT, "include", "lsp.h")).read()
    return {n: [p.strip() for p in a.split(",")]
            for n, a in re.findall(r"\n\s*[\w\s\*]+?\b(lsp_\w+)\s*\(([^;]*?)\)\s*;", h)}


def is_ptr(p):
    return "*" in p or "[" in p


def main():
    mode = sys.argv[1]
    L = _lib.lib()
    params = header_params()
    ctx = None
    if mode == "one-null":
        from linea_stark_prover_amd.prover import Context, StarkConfig
        ctx = Context(StarkConfig(), device=-1)  # LSP_HOST_ONLY
    keep = []
    for name, (res, argtypes) in _lib._SIGS.items():
        ps = params[name]
        assert len(ps) == len(argtypes) or (ps == ["void"] and not argtypes), name
        if mode == "all-null":
            cases = [None]
        else:
            cases = [i for i, p in enumerate(ps) if is_ptr(p) and not (name in RELEASERS and i == 0)]
        for which in cases:
            vals = []
            for i, (a, p) in enumerate(zip(argtypes, ps)):
                if not is_ptr(p):
                    vals.append(1)
                elif which is None or i == which or HANDLE.match(p):
                    vals.append(None)
                elif CTX.match(p):
                    vals.append(ctx.h)
                else:
                    b = ctypes.create_string_buffer(1 << 20)
                    keep.append(b)
                    vals.append(ctypes.cast(b, a) if a is not ctypes.c_void_p else ctypes.cast(b, ctypes.c_void_p).value)
            null_param = ps[which] if which is not None else "all"
            print(json.dumps({"fn": name, "null": null_param, "phase": "call"}), flush=True)
            r = getattr(L, name)(*vals)
            ret = r if isinstance(r, int) or r is None else "ptr"
            print(json.dumps({"fn": name, "null": null_param, "phase": "ret", "ret": ret,
                              "ctx_null": bool(CTX.match(ps[which])) if which is not None else True}), flush=True)
            keep.clear()
    print(json.dumps({"phase": "done"}), flush=True)


if __name__ == "__main__":
    main()
