"""ASan + UBSan over the host code that reads untrusted bytes (VERDICT r01
weak 10): tools/sanitize/run.sh builds liblsp_hip.so's host side with
-fsanitize=address,undefined (device code unchanged) and fuzzes the CBOR trace
parser (cbor.cpp), the proof parser and view (proof.cpp), the host verifier
(verify.cpp) and the big-endian word reader with truncations and random
mutations of a real proof and of the CBOR fixtures.  CPU only."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="needs hipcc")
@pytest.mark.parametrize("log_n,ncols,seed", [(6, 3, 1), (5, 6, 2)])
def test_parsers_under_asan_ubsan(oracle_lib, tmp_path, log_n, ncols, seed):
    p = oracle_lib.setup()
    tb, w = oracle_lib.gen_perm_trace(p, log_n, ncols)
    proof = tmp_path / "proof.bin"
    proof.write_bytes(oracle_lib.prove(p, tb, 1 << log_n, w, oracle_lib.perm_air(ncols)))
    env = dict(os.environ, LSP_SAN_NCOLS=str(ncols))
    r = subprocess.run(["bash", os.path.join(ROOT, "tools", "sanitize", "run.sh"), str(proof), "400", str(seed)],
                       capture_output=True, text=True, timeout=900, env=env)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "sanitize ok" in r.stdout


@pytest.mark.skipif(shutil.which("/opt/rocm/bin/hipcc") is None, reason="needs hipcc")
def test_debug_bounds_build(product_lib):
    """SURVEY 5's bounds-checked debug kernels: build.py --debug-bounds
    compiles every kernel with LSP_DEBUG_BOUNDS (csrc/dbg_bounds.hpp) into
    liblsp_hip_dbg.so, which exports the product's symbols and names itself;
    tests/test_gpu_debug_bounds.py runs it on the GPU"""
    import ctypes
    from linea_stark_prover_amd import _lib
    from linea_stark_prover_amd import build as B
    lib_path = B.build(verbose=False, debug_bounds=True)
    assert os.path.basename(lib_path) == "liblsp_hip_dbg.so"
    code = ("import ctypes, sys; L = ctypes.CDLL(sys.argv[1]); L.lsp_version.restype = ctypes.c_char_p; "
            "print(L.lsp_version().decode()); "
            "[getattr(L, n) for n in sys.argv[2:]]")
    r = subprocess.run([os.sys.executable, "-c", code, lib_path] + list(_lib.EXPORTED), capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    assert "debug-bounds" in r.stdout
    product_lib.lsp_version.restype = ctypes.c_char_p
    assert b"debug-bounds" not in product_lib.lsp_version()
