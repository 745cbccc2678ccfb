"""Build liblsp_hip.so (HIP kernels + host orchestration) for gfx950, in-tree.

    python -m linea_stark_prover_amd.build [--force] [-j N]

Objects go to ``linea_stark_prover_amd/_build/``, the library to
``linea_stark_prover_amd/_lib/liblsp_hip.so`` (git-ignored, travels to the GPU
box with the snapshot).  Rebuilds only what changed (any header change
rebuilds everything).
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
    try:
        with open(STAMP) as fh:
            return fh.read().strip() or None
    except OSError:
        return None


def _headers():
    return [os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hpp", ".inc"))] + \
        [os.path.join(ROOT, "include", "lsp.h")]


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


def _compile(src):
    obj = os.path.join(BUILD, os.path.splitext(src)[0] + ".o")
    cmd = [HIPCC] + CFLAGS + ["-c", os.path.join(CSRC, src), "-o", obj]
    if src.endswith(".cpp"):
        cmd = [HIPCC] + CFLAGS + ["-x", "hip", "-c", os.path.join(CSRC, src), "-o", obj]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"compile failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
    return obj


def build(force: bool = False, jobs: int = None, verbose: bool = True) -> str:
    os.makedirs(BUILD, exist_ok=True)
    os.makedirs(LIBDIR, exist_ok=True)
    hdrs = _headers()
    todo = []
    objs = []
    for s in SOURCES:
        obj = os.path.join(BUILD, os.path.splitext(s)[0] + ".o")
        objs.append(obj)
        if force or _stale(obj, [os.path.join(CSRC, s)] + hdrs):
            todo.append(s)
    jobs = jobs or min(len(todo) or 1, os.cpu_count() or 4, 16)
    if todo:
        if verbose:
            print(f"[lsp build] compiling {len(todo)} file(s) for {ARCH}: {' '.join(todo)}", flush=True)
        with cf.ThreadPoolExecutor(jobs) as ex:
            list(ex.map(_compile, todo))
    if todo or _stale(LIB, objs):
        cmd = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", LIB] + objs + ["-lpthread", "-ldl"]
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{r.stdout}\n{r.stderr}")
        if verbose:
            print(f"[lsp build] linked {LIB}", flush=True)
    if library_hash() != source_hash():
        with open(STAMP, "w") as fh:
            fh.write(source_hash() + "\n")
    return LIB


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--force", action="store_true")
    ap.add_argument("-j", type=int, default=None)
    a = ap.parse_args(argv)
    build(a.force, a.j)


if __name__ == "__main__":
    sys.exit(main())
