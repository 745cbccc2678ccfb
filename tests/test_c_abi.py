"""The C-ABI from plain C (examples/prove_c.c): compiled by gcc against
include/lsp.h only and linked to liblsp_hip.so -- the binding a Rust -sys
crate or any FFI makes."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "linea_stark_prover_amd", "_lib")


def _build(tmp_path):
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    exe = str(tmp_path / "prove_c")
    r = subprocess.run(["gcc", "-std=c99", "-O2", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "include"),
                        os.path.join(ROOT, "examples", "prove_c.c"), "-o", exe, "-L", LIBDIR, "-llsp_hip",
                        f"-Wl,-rpath,{LIBDIR}"], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    return exe


def test_c_program_host_only(product_lib, tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe, "6", "--host-only"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "host-only ok" in r.stdout


@pytest.mark.gpu
def test_c_program_proves_and_verifies(product_lib, tmp_path):
    exe = _build(tmp_path)
    r = subprocess.run([exe, "12"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "verify ok, tampered rejected" in r.stdout and "rebuilt bytes identical" in r.stdout
