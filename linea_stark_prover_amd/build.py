"""Build liblsp_hip.so (HIP kernels + host orchestration) for gfx950, in-tree.

    python -m linea_stark_prover_amd.build [--force] [-j N] [--debug-bounds]

Objects go to ``linea_stark_prover_amd/_build/``, the library to
``linea_stark_prover_amd/_lib/liblsp_hip.so`` (git-ignored, travels to the GPU
box with the snapshot).  Rebuilds only what changed (any header change
rebuilds everything).

``--debug-bounds``: the bounds-checked debug build (csrc/dbg_bounds.hpp)
-- ``-DLSP_DEBUG_BOUNDS``, objects in ``_build_dbg/``, library
``_lib/liblsp_hip_dbg.so``; select it with ``LSP_LIB=<path>`` (linea_stark_prover_amd/_lib.py).
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import os
import subprocess
import sys

PKG = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(PKG)
CSRC = os.path.join(PKG, "csrc")
BUILD = os.path.join(PKG, "_build")
LIBDIR = os.path.join(PKG, "_lib")
LIB = os.path.join(LIBDIR, "liblsp_hip.so")
STAMP = LIB + ".src"  # source_hash() of the sources the library was linked from
ARCH = os.environ.get("LSP_OFFLOAD_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

SOURCES = ["k_ntt.hip", "k_hash.hip", "k_field.hip", "k_quotient.hip", "k_open.hip", "k_witness.hip",
           "host.cpp", "host_ifma.cpp", "prove.cpp", "verify.cpp", "proof.cpp", "witness.cpp", "cbor.cpp", "comm_ext.cpp", "capi.cpp"]
CFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-result",
          # host code: mulx/adcx/adox for the 4 x 64-bit host multiplier (x86-64 with BMI2 + ADX:
          # the build container and the MI355X hosts)
          "-Xarch_host", "-mbmi2", "-Xarch_host", "-madx",
          "-Wno-unused-variable", "-I", os.path.join(ROOT, "include")]


def source_hash() -> str:
    """sha256 (16 hex digits) of everything the library is built from: the
    csrc/ sources, include/lsp.h and the compile flags.  Profiles measured on
    one build (PMC traffic, VALU issue) carry it, and bench.py uses a profile
    only when it matches the library being benched."""
    import hashlib
    hsh = hashlib.sha256()
    files = sorted(f for f in os.listdir(CSRC) if f.endswith((".hip", ".cpp", ".hpp", ".inc")))
    for f in files:
        hsh.update(f.encode())
        with open(os.path.join(CSRC, f), "rb") as fh:
            hsh.update(fh.read())
    with open(os.path.join(ROOT, "include", "lsp.h"), "rb") as fh:
        hsh.update(fh.read())
    hsh.update(" ".join(CFLAGS[:-1] + [ARCH]).encode())
    return hsh.hexdigest()[:16]


def library_hash() -> str | None:
    """source_hash() of the sources liblsp_hip.so was linked from (written next
    to the library at link time), or None when the library has no stamp.  The
    stamp travels with the library, so a profile taken on a GPU box names the
    build that ran there even when the working tree has moved on."""
    return _read_stamp(LIB)


def _headers():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".inc"))] + \
        [os.path.join(ROOT, "include", "lsp.h")]


DBG_BUILD = os.path.join(PKG, "_build_dbg")
DBG_LIB = os.path.join(LIBDIR, "liblsp_hip_dbg.so")


def _stamp_path(lib):
    return lib + ".src"


def _read_stamp(lib):
    try:
        with open(_stamp_path(lib)) as fh:
            return fh.read().strip() or None
    except OSError:
        return None


def _compile(src, build_dir=BUILD, extra=()):
    obj = os.path.join(build_dir, os.path.splitext(src)[0] + ".o")
    flags = CFLAGS + list(extra)
    cmd = [HIPCC] + flags + ["-c", os.path.join(CSRC, src), "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC] + flags + ["-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def _file_hash(path, seed=b""):
    import hashlib
    h = hashlib.sha256(seed)
    with open(path, "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def build(force: bool = False, jobs: int = None, verbose: bool = True, debug_bounds: bool = False) -> str:
    """Compile what changed and relink.  "Changed" is decided by content, not
    mtimes: every object carries the hash of its source, the headers and the
    flags it was compiled from (``x.o.src``), and the library the hash of
    everything it was linked from (``liblsp_hip.so.src``, the stamp bench.py
    ties profiles to).  A checkout or an ``rsync -t`` can change a source
    without making it newer than its object; that object is recompiled and the
    library relinked, never relabelled."""
    import hashlib
    build_dir, lib = (DBG_BUILD, DBG_LIB) if debug_bounds else (BUILD, LIB)
    extra = ["-DLSP_DEBUG_BOUNDS"] if debug_bounds else []
    os.makedirs(build_dir, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    want = source_hash()
    common = hashlib.sha256(" ".join(CFLAGS + extra + [ARCH]).encode())
    for hdr in sorted(_headers()):
        common.update(os.path.basename(hdr).encode())
        with open(hdr, "rb") as fh:
            common.update(fh.read())
    seed = common.digest()
    todo, objs, hashes = [], [], {}
    for s in SOURCES:
        obj = os.path.join(build_dir, os.path.splitext(s)[0] + ".o")
        objs.append(obj)
        hashes[s] = _file_hash(os.path.join(CSRC, s), seed)
        if force or not os.path.exists(obj) or _read_stamp(obj) != hashes[s]:
            todo.append(s)
    jobs = jobs or min(len(todo) or 1, os.cpu_count() or 4, 16)
    if todo:
        if verbose:
            print(f"[lsp build] compiling {len(todo)} file(s) for {ARCH}{' (debug-bounds)' if debug_bounds else ''}: "
                  f"{' '.join(todo)}", flush=True)

        def one(src):
            obj = _compile(src, build_dir, extra)
            with open(_stamp_path(obj), "w") as fh:
                fh.write(hashes[src] + "\n")

        with cf.ThreadPoolExecutor(jobs) as ex:
            list(ex.map(one, todo))
    if todo or not os.path.exists(lib) or _read_stamp(lib) != want:
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", lib] + objs + ["-lpthread", "-ldl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[lsp build] linked {lib}", flush=True)
        # the stamp is written only here, after a link from objects whose own
        # stamps name the sources they were compiled from
        with open(_stamp_path(lib), "w") as fh:
            fh.write(want + "\n")
    return lib


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    ap.add_argument("--debug-bounds", action="store_true", help="the bounds-checked debug library (liblsp_hip_dbg.so)")
    a = ap.parse_args(argv)
    build(a.force, a.j, debug_bounds=a.debug_bounds)


if __name__ == "__main__":
    sys.exit(main())
