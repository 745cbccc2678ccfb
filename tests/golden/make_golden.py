"""Regenerate tests/golden/golden.json from the Python mini oracle.

These are regression vectors for the build's documented conventions
 -- the reference ships no fixtures, so they pin the
oracle against itself across rounds, not against the reference.

    python tests/golden/make_golden.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import pyoracle as O  # noqa: E402


def main():
    s = O.setup_from_seed()
    g = {}
    g["field"] = {"modulus": hex(O.P), "two_adicity": O.TWO_ADICITY, "generator": O.GENERATOR,
                  "root_2_47": hex(O.ROOT_2_47), "mont_r": hex(O.MONT_R)}
    g["setup"] = {"seed": hex(O.DEFAULT_SEED), "alpha": hex(s.alpha), "delta": hex(s.delta),
                  "ext_initial": [[hex(x) for x in r] for r in s.perm.ext_initial],
                  "ext_terminal": [[hex(x) for x in r] for r in s.perm.ext_terminal],
                  "internal": [hex(x) for x in s.perm.internal]}
    g["poseidon2_012"] = [hex(x) for x in O.permute([0, 1, 2], s.perm)]
    g["hash_iter_range"] = {str(w): hex(O.hash_iter(list(range(w)), s.perm)) for w in range(0, 6)}
    g["compress_1_2"] = hex(O.compress(1, 2, s.perm))
    # U2/U3 as parameters (lsp_params.internal_diag / external_mds): one
    # non-default internal diagonal and external matrix
    diag, mds = (3, 5, O.P - 7), (5, 7, 1, 3, 2, 9, 4, 4, O.P - 1)
    s.perm.int_diag, s.perm.ext_mds = diag, mds
    g["poseidon2_012_layers"] = {"int_diag": [hex(x) for x in diag], "ext_mds": [hex(x) for x in mds],
                                 "out": [hex(x) for x in O.permute([0, 1, 2], s.perm)]}
    s.perm.int_diag = s.perm.ext_mds = None
    col = [pow(3, i, O.P) for i in range(4)]
    g["lde_col_3pow_h4_b3"] = [hex(x) for x in O.coset_lde_column(col, 3, O.GENERATOR)]
    g["proofs"] = {}
    for logn, ncols in ((3, 3), (3, 6), (4, 3)):
        cfgs, cols = O.synthetic_perm_trace(logn, ncols, s.alpha, s.delta, O.DEFAULT_SEED)
        pf = O.prove(cfgs, O.columns_to_rows(cols), [s.alpha, s.delta], s.perm)
        b = O.serialize_proof(pf)
        ent = {"sha256": hashlib.sha256(b).hexdigest(), "len": len(b),
               "trace_root": hex(pf.trace_root), "quotient_root": hex(pf.quotient_root),
               "final_poly": hex(pf.final_poly)}
        if (logn, ncols) == (3, 3):
            ent["hex"] = b.hex()
        g["proofs"][f"perm_{ncols}x{ncols}_n{logn}"] = ent
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(g, f, indent=1)
    print("wrote golden.json")


if __name__ == "__main__":
    main()
