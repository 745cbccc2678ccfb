"""p3_uni_stark::Proof<SC> as Python objects over the C-ABI proof view
(include/lsp.h lsp_proof_view; csrc/proof.cpp).

The classes mirror the Plonky3 structs field for field, for the reference's
Config (bin/src/config.rs:19-25: Val = Challenge = Bls12_377Fr,
MerkleTreeMmcs<Val, Val, Hash, Compress, 1>, TwoAdicFriPcs), so a proof from
lsp_prove reads as the Proof<SC> that bin/src/main.rs:80-86 returns and
hands to p3_uni_stark::verify (bin/src/main.rs:88-96):

  Proof { commitments: Commitments { trace, quotient_chunks },
          opened_values: OpenedValues { trace_local, trace_next, quotient_chunks },
          opening_proof: FriProof { commit_phase_commits, query_proofs: [QueryProof {
              input_proof: [BatchOpening { opened_values, opening_proof }; 2],
              commit_phase_openings: [CommitPhaseProofStep { sibling_value, opening_proof }] }],
            final_poly, pow_witness },
          degree_bits }

Elements are numpy uint64 arrays with a trailing axis of 4 limbs (Montgomery
form, the lsp_fr convention).  Proof.from_bytes / to_bytes go through
lsp_proof_deserialize + lsp_proof_get_view and lsp_proof_from_view +
lsp_proof_serialize; the library does every parse and layout step.
"""
from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import List

import numpy as np

from . import _lib as L


def wire_size(log_h: int, w: int, log_q: int, log_blowup: int = 3, log_final_poly_len: int = 0,
              num_queries: int = 33) -> int:
    """Bytes of a serialized proof (csrc/proof.cpp serialize) of an h x w
    trace with 2^log_q quotient chunks: header, commitments, opened values,
    FRI roots and final polynomial, pow witness, then per query the trace and
    quotient rows with their paths and, per FRI round r, the sibling and a
    path of log N - 1 - r digests (each path prefixed by its u32 length)."""
    logN = log_h + log_blowup
    nr = logN - log_blowup - log_final_poly_len
    q = 1 << log_q
    per_query_fr = w + logN + q + logN + nr + sum(logN - 1 - r for r in range(nr))
    nfr = 3 + 2 * w + q + nr + (1 << log_final_poly_len) + num_queries * per_query_fr
    nu32 = 6 + num_queries * (2 + nr)
    return 8 + 4 * nu32 + 32 * nfr


class LspProofView(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in ("degree_bits", "log_quotient_chunks", "width", "num_queries",
                                                "num_fri_rounds", "final_poly_len", "input_path_len")] + \
               [("fri_path_lens", ctypes.POINTER(ctypes.c_uint32))] + \
               [(n, ctypes.c_void_p) for n in ("trace_commit", "quotient_commit", "pow_witness", "trace_local",
                                              "trace_next", "quotient_chunks", "fri_commits", "final_poly",
                                              "trace_rows", "trace_paths", "quotient_rows", "quotient_paths",
                                              "fri_siblings", "fri_paths")]


@dataclass
class Commitments:
    trace: np.ndarray            # Hash<Val, Val, 1>: (1, 4)
    quotient_chunks: np.ndarray  # (1, 4)


@dataclass
class OpenedValues:
    trace_local: np.ndarray            # (w, 4)
    trace_next: np.ndarray             # (w, 4)
    quotient_chunks: List[np.ndarray]  # q x (1, 4): Vec<Vec<Challenge>>, one value per chunk


@dataclass
class BatchOpening:
    opened_values: List[np.ndarray]  # one row per matrix of the committed round
    opening_proof: np.ndarray        # Vec<[Val; 1]>: siblings leaf -> root, (path_len, 4)


@dataclass
class CommitPhaseProofStep:
    sibling_value: np.ndarray  # (4,)
    opening_proof: np.ndarray  # (path_len, 4)


@dataclass
class QueryProof:
    input_proof: List[BatchOpening]  # [trace round, quotient round]
    commit_phase_openings: List[CommitPhaseProofStep]


@dataclass
class FriProof:
    commit_phase_commits: np.ndarray  # (rounds, 4)
    query_proofs: List[QueryProof]
    final_poly: np.ndarray            # (final_poly_len, 4)
    pow_witness: np.ndarray           # (4,)


@dataclass
class Proof:
    commitments: Commitments
    opened_values: OpenedValues
    opening_proof: FriProof
    degree_bits: int

    # ------------------------------------------------------------ from bytes
    @staticmethod
    def from_handle(h: ctypes.c_void_p) -> "Proof":
        v = LspProofView()
        L.check(L.lib().lsp_proof_get_view(h, ctypes.byref(v)))

        def arr(ptr, n):
            if n == 0:
                return np.zeros((0, 4), np.uint64)
            return np.ctypeslib.as_array(ctypes.cast(ptr, ctypes.POINTER(ctypes.c_uint64)), (n * 4,)) \
                .reshape(n, 4).copy()
        w, q, nq, nr = v.width, 1 << v.log_quotient_chunks, v.num_queries, v.num_fri_rounds
        pl = v.input_path_len
        fpl = [v.fri_path_lens[k] for k in range(nr)]
        trows, tpaths = arr(v.trace_rows, nq * w), arr(v.trace_paths, nq * pl)
        qrows, qpaths = arr(v.quotient_rows, nq * q), arr(v.quotient_paths, nq * pl)
        sibs, fpaths = arr(v.fri_siblings, nq * nr), arr(v.fri_paths, nq * sum(fpl))
        qps = []
        for i in range(nq):
            o, steps = i * sum(fpl), []
            for k in range(nr):
                steps.append(CommitPhaseProofStep(sibs[i * nr + k], fpaths[o:o + fpl[k]]))
                o += fpl[k]
            qrow = qrows[i * q:(i + 1) * q]
            qps.append(QueryProof(
                [BatchOpening([trows[i * w:(i + 1) * w]], tpaths[i * pl:(i + 1) * pl]),
                 BatchOpening([qrow[j:j + 1] for j in range(q)], qpaths[i * pl:(i + 1) * pl])], steps))
        qc = arr(v.quotient_chunks, q)
        return Proof(Commitments(arr(v.trace_commit, 1), arr(v.quotient_commit, 1)),
                     OpenedValues(arr(v.trace_local, w), arr(v.trace_next, w), [qc[j:j + 1] for j in range(q)]),
                     FriProof(arr(v.fri_commits, nr), qps, arr(v.final_poly, v.final_poly_len),
                              arr(v.pow_witness, 1)[0]),
                     v.degree_bits)

    @staticmethod
    def from_bytes(b: bytes) -> "Proof":
        h = ctypes.c_void_p()
        L.check(L.lib().lsp_proof_deserialize(b, len(b), ctypes.byref(h)))
        try:
            return Proof.from_handle(h)
        finally:
            L.lib().lsp_proof_free(h)

    # -------------------------------------------------------------- to bytes
    def to_bytes(self) -> bytes:
        from .prover import _take_proof
        ov, fp = self.opened_values, self.opening_proof
        w, q, nr = len(ov.trace_local), len(ov.quotient_chunks), len(fp.commit_phase_commits)
        qps = fp.query_proofs
        pl = len(qps[0].input_proof[0].opening_proof) if qps else 0
        fpl = [len(s.opening_proof) for s in qps[0].commit_phase_openings] if qps else [0] * nr

        def cat(parts):
            parts = [np.asarray(p, np.uint64).reshape(-1, 4) for p in parts]
            return np.ascontiguousarray(np.concatenate(parts) if parts else np.zeros((0, 4), np.uint64))
        keep = {
            "trace_commit": cat([self.commitments.trace]), "quotient_commit": cat([self.commitments.quotient_chunks]),
            "pow_witness": cat([fp.pow_witness]), "trace_local": cat([ov.trace_local]),
            "trace_next": cat([ov.trace_next]), "quotient_chunks": cat(ov.quotient_chunks),
            "fri_commits": cat([fp.commit_phase_commits]), "final_poly": cat([fp.final_poly]),
            "trace_rows": cat([qp.input_proof[0].opened_values[0] for qp in qps]),
            "trace_paths": cat([qp.input_proof[0].opening_proof for qp in qps]),
            "quotient_rows": cat([r for qp in qps for r in qp.input_proof[1].opened_values]),
            "quotient_paths": cat([qp.input_proof[1].opening_proof for qp in qps]),
            "fri_siblings": cat([s.sibling_value for qp in qps for s in qp.commit_phase_openings]),
            "fri_paths": cat([s.opening_proof for qp in qps for s in qp.commit_phase_openings]),
        }
        lens = (ctypes.c_uint32 * max(1, nr))(*fpl)
        v = LspProofView(degree_bits=self.degree_bits, log_quotient_chunks=q.bit_length() - 1, width=w,
                         num_queries=len(qps), num_fri_rounds=nr, final_poly_len=len(fp.final_poly),
                         input_path_len=pl, fri_path_lens=lens,
                         **{k: a.ctypes.data for k, a in keep.items()})
        h = ctypes.c_void_p()
        L.check(L.lib().lsp_proof_from_view(ctypes.byref(v), ctypes.byref(h)))
        return _take_proof(h)
