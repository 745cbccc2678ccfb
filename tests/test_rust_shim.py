"""rust/p3-hip (the Plonky3-side shim; source only -- the image has no cargo):
its -sys layer is generated from include/lsp.h and must match it, and every
C entry point the safe layer calls must exist in the header and the library."""
import ctypes
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CRATE = os.path.join(ROOT, "rust", "p3-hip")


def test_sys_rs_matches_header():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_rust_sys.py"), "--check"])
    assert r.returncode == 0, "rust/p3-hip/src/sys.rs is stale: run python tools/gen_rust_sys.py"


def test_shim_calls_only_exported_functions(product_lib):
    declared = set(re.findall(r"pub fn (lsp_\w+)\(", open(os.path.join(CRATE, "src", "sys.rs")).read()))
    hdr = set(re.findall(r"\b(lsp_\w+)\s*\(", re.sub(r"/\*.*?\*/", "", open(os.path.join(ROOT, "include", "lsp.h")).read(), flags=re.S)))
    assert declared <= hdr
    used = set()
    for d in ("src", "tests"):
        for f in os.listdir(os.path.join(CRATE, d)):
            used |= set(re.findall(r"sys::(lsp_\w+)\(", open(os.path.join(CRATE, d, f)).read()))
    assert used and used <= declared, used - declared
    for name in used:  # and the built library exports them
        getattr(product_lib, name)


def test_shim_implements_the_plug_point_traits():
    src = {f: open(os.path.join(CRATE, "src", f)).read() for f in os.listdir(os.path.join(CRATE, "src"))}
    allsrc = "\n".join(src.values())
    # bin/src/config.rs:19-22 aliases and bin/src/main.rs:80-86 prove
    assert "impl TwoAdicSubgroupDft<Val> for HipDft" in src["dft.rs"]
    assert "fn coset_lde_batch(" in src["dft.rs"] and "lsp_coset_lde_batch" in src["dft.rs"]
    assert "impl Mmcs<Val> for HipMmcs" in src["mmcs.rs"]
    for m in ("fn commit<", "fn open_batch<", "fn get_matrices<", "fn verify_batch("):
        assert m in src["mmcs.rs"], m
    assert "FriGenericConfig<Val> for HipFriFolder" in src["fri.rs"]
    assert "pub fn prove<SC>" in src["proof.rs"] and "Proof<SC>" in src["proof.rs"]
    # the serde mirror must name every field of p3-uni-stark / p3-fri's proof structs
    for field in ("commitments", "opened_values", "opening_proof", "degree_bits", "trace", "quotient_chunks",
                  "trace_local", "trace_next", "commit_phase_commits", "query_proofs", "final_poly", "pow_witness",
                  "input_proof", "commit_phase_openings", "sibling_value"):
        assert re.search(rf"\b{field}:", allsrc), field
