"""Every C-ABI entry point with NULL pointers: a status code, never a fault.

The calls run in a child process (tests/abi_sweep_child.py) so that a
segmentation fault fails the test with the call that caused it instead of
ending the test run.  CPU only: with a GPU context the dummy buffers would be
read as device pointers.
"""
import json
import os
import subprocess
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
# entry points that return nothing, a string, or LSP_OK for NULL (release functions,
# size queries with optional outputs)
NO_STATUS = {"lsp_version", "lsp_last_error", "lsp_fr_from_canonical", "lsp_fr_to_canonical",
             "lsp_fr_from_be_bytes_mod_order", "lsp_fr_mul", "lsp_fr_inv", "lsp_two_adic_generator",
             "lsp_fri_fold_row", "lsp_ctx_destroy", "lsp_tree_free", "lsp_proof_free", "lsp_group_destroy",
             "lsp_raw_trace_free"}


def _sweep(product_lib, mode):
    r = subprocess.run([sys.executable, os.path.join(HERE, "abi_sweep_child.py"), mode],
                       capture_output=True, text=True, timeout=300)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    last = lines[-1] if lines else None
    assert r.returncode == 0 and last and last["phase"] == "done", (
        f"child ended with status {r.returncode} during {last}: {r.stderr[-2000:]}")
    return [x for x in lines if x["phase"] == "ret"]


def test_all_null_arguments_return_errors(product_lib):
    rets = _sweep(product_lib, "all-null")
    assert len(rets) == len({x["fn"] for x in rets}) >= 60
    bad = [x for x in rets if x["fn"] not in NO_STATUS and x["ret"] == 0]
    assert not bad, f"accepted all-NULL arguments: {bad}"


def test_one_null_argument_never_faults(product_lib):
    rets = _sweep(product_lib, "one-null")
    assert len(rets) > 150
    # a NULL context is always an error for the entry points that report one
    bad = [x for x in rets if x["ctx_null"] and x["fn"] not in NO_STATUS and x["ret"] == 0]
    assert not bad, f"accepted a NULL context: {bad}"
