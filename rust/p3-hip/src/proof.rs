//! `p3_uni_stark::Proof<SC>` across the C-ABI (include/lsp.h lsp_proof_view).
//!
//! `Proof`'s fields are `pub(crate)` in p3-uni-stark, so the proof is built
//! the way serde sees it: a mirror of the struct tree with the same field
//! names and the real leaf types (`Val`, `Hash<Val, Val, 1>`, `[Val; 1]`) is
//! written as CBOR and read back as `Proof<SC>` (and the reverse).  Any `SC`
//! whose proof has this shape -- the reference's `Config`
//! (`bin/src/config.rs:24-25`) with `MerkleTreeMmcs` or [`crate::HipMmcs`] --
//! works; a mismatching `SC` fails loudly at the conversion.
use serde::de::DeserializeOwned;
use serde::{Deserialize, Serialize};

use p3_symmetric::Hash;
use p3_uni_stark::{Proof, StarkGenericConfig};

use crate::{check_global, fr_ptr, sys, vals, Ctx, Val};

type Com = Hash<Val, Val, 1>;

#[derive(Serialize, Deserialize)]
struct Commitments {
    trace: Com,
    quotient_chunks: Com,
}

#[derive(Serialize, Deserialize)]
struct OpenedValues {
    trace_local: Vec<Val>,
    trace_next: Vec<Val>,
    quotient_chunks: Vec<Vec<Val>>,
}

#[derive(Serialize, Deserialize)]
struct BatchOpening {
    opened_values: Vec<Vec<Val>>,
    opening_proof: Vec<[Val; 1]>,
}

#[derive(Serialize, Deserialize)]
struct CommitPhaseProofStep {
    sibling_value: Val,
    opening_proof: Vec<[Val; 1]>,
}

#[derive(Serialize, Deserialize)]
struct QueryProof {
    input_proof: Vec<BatchOpening>,
    commit_phase_openings: Vec<CommitPhaseProofStep>,
}

#[derive(Serialize, Deserialize)]
struct FriProof {
    commit_phase_commits: Vec<Com>,
    query_proofs: Vec<QueryProof>,
    final_poly: Vec<Val>,
    pow_witness: Val,
}

#[derive(Serialize, Deserialize)]
struct ProofMirror {
    commitments: Commitments,
    opened_values: OpenedValues,
    opening_proof: FriProof,
    degree_bits: usize,
}

fn recast<A: Serialize, B: DeserializeOwned>(a: &A, what: &str) -> B {
    let mut buf = Vec::new();
    ciborium::into_writer(a, &mut buf).expect("CBOR encode");
    ciborium::from_reader(buf.as_slice()).unwrap_or_else(|e| panic!("{what}: proof shape mismatch: {e}"))
}

fn paths(p: *const sys::lsp_fr, n: usize) -> Vec<[Val; 1]> {
    unsafe { vals(p, n) }.into_iter().map(|x| [x]).collect()
}

/// lsp_proof handle -> Proof<SC> (the handle is not freed)
pub fn to_proof<SC>(h: *const sys::lsp_proof) -> Proof<SC>
where
    SC: StarkGenericConfig,
    Proof<SC>: DeserializeOwned,
{
    let mut v = std::mem::MaybeUninit::<sys::lsp_proof_view>::zeroed();
    check_global(unsafe { sys::lsp_proof_get_view(h, v.as_mut_ptr()) }, "lsp_proof_get_view");
    let v = unsafe { v.assume_init() };
    let (w, q) = (v.width as usize, 1usize << v.log_quotient_chunks);
    let (nq, nr, pl) = (v.num_queries as usize, v.num_fri_rounds as usize, v.input_path_len as usize);
    let fpl: Vec<usize> = (0..nr).map(|k| unsafe { *v.fri_path_lens.add(k) } as usize).collect();
    let fsum: usize = fpl.iter().sum();
    let one = |p: *const sys::lsp_fr| unsafe { vals(p, 1) }[0];
    let mut query_proofs = Vec::with_capacity(nq);
    for i in 0..nq {
        let qrow = unsafe { vals(v.quotient_rows.add(i * q), q) };
        let mut steps = Vec::with_capacity(nr);
        let mut off = i * fsum;
        for (k, &len) in fpl.iter().enumerate() {
            steps.push(CommitPhaseProofStep {
                sibling_value: one(unsafe { v.fri_siblings.add(i * nr + k) }),
                opening_proof: paths(unsafe { v.fri_paths.add(off) }, len),
            });
            off += len;
        }
        query_proofs.push(QueryProof {
            input_proof: vec![
                BatchOpening {
                    opened_values: vec![unsafe { vals(v.trace_rows.add(i * w), w) }],
                    opening_proof: paths(unsafe { v.trace_paths.add(i * pl) }, pl),
                },
                BatchOpening {
                    opened_values: qrow.into_iter().map(|x| vec![x]).collect(),
                    opening_proof: paths(unsafe { v.quotient_paths.add(i * pl) }, pl),
                },
            ],
            commit_phase_openings: steps,
        });
    }
    let m = ProofMirror {
        commitments: Commitments {
            trace: Hash::from([one(v.trace_commit)]),
            quotient_chunks: Hash::from([one(v.quotient_commit)]),
        },
        opened_values: OpenedValues {
            trace_local: unsafe { vals(v.trace_local, w) },
            trace_next: unsafe { vals(v.trace_next, w) },
            quotient_chunks: unsafe { vals(v.quotient_chunks, q) }.into_iter().map(|x| vec![x]).collect(),
        },
        opening_proof: FriProof {
            commit_phase_commits: unsafe { vals(v.fri_commits, nr) }.into_iter().map(|x| Hash::from([x])).collect(),
            query_proofs,
            final_poly: unsafe { vals(v.final_poly, v.final_poly_len as usize) },
            pow_witness: one(v.pow_witness),
        },
        degree_bits: v.degree_bits as usize,
    };
    recast(&m, "lsp_proof -> Proof<SC>")
}

/// The flat view (include/lsp.h lsp_proof_view) gives every query the shape
/// of query 0, and lsp_proof_from_view reads that many elements per query out
/// of the Vecs built below.  A deserialized (untrusted) Proof<SC> with ragged
/// queries must therefore be rejected here, before any pointer is handed out.
fn check_shape(m: &ProofMirror) -> Result<(), String> {
    let (ov, fp) = (&m.opened_values, &m.opening_proof);
    let w = ov.trace_local.len();
    if ov.trace_next.len() != w {
        return Err(format!("trace_next has {} values, trace_local {w}", ov.trace_next.len()));
    }
    let q = ov.quotient_chunks.len();
    if !q.is_power_of_two() || ov.quotient_chunks.iter().any(|c| c.len() != 1) {
        return Err("quotient_chunks: need 2^k chunks of one value each".into());
    }
    if !fp.final_poly.len().is_power_of_two() {
        return Err(format!("final_poly length {} is not a power of two", fp.final_poly.len()));
    }
    let nr = fp.commit_phase_commits.len();
    let first = fp.query_proofs.first();
    let pl = first.and_then(|qp| qp.input_proof.first()).map_or(0, |b| b.opening_proof.len());
    let fpl: Vec<usize> = first.map_or_else(
        || vec![0; nr],
        |qp| qp.commit_phase_openings.iter().map(|s| s.opening_proof.len()).collect(),
    );
    for (i, qp) in fp.query_proofs.iter().enumerate() {
        let bad = |what: &str| Err(format!("query {i}: {what}"));
        if qp.input_proof.len() != 2 {
            return bad("needs two batch openings (trace, quotient chunks)");
        }
        let (t, qb) = (&qp.input_proof[0], &qp.input_proof[1]);
        if t.opened_values.len() != 1 || t.opened_values[0].len() != w {
            return bad("trace row width differs from trace_local");
        }
        if qb.opened_values.len() != q || qb.opened_values.iter().any(|r| r.len() != 1) {
            return bad("quotient row shape differs from quotient_chunks");
        }
        if t.opening_proof.len() != pl || qb.opening_proof.len() != pl {
            return bad("input Merkle path length differs from query 0");
        }
        if qp.commit_phase_openings.len() != nr {
            return bad("commit-phase openings differ from commit_phase_commits");
        }
        if qp.commit_phase_openings.iter().zip(&fpl).any(|(s, &l)| s.opening_proof.len() != l) {
            return bad("FRI path length differs from query 0");
        }
    }
    Ok(())
}

/// Proof<SC> -> a new lsp_proof handle (free with sys::lsp_proof_free);
/// Err on a proof whose queries do not share one shape
pub fn try_from_proof<SC>(proof: &Proof<SC>) -> Result<*mut sys::lsp_proof, String>
where
    SC: StarkGenericConfig,
    Proof<SC>: Serialize,
{
    let m: ProofMirror = recast(proof, "Proof<SC> -> lsp_proof");
    check_shape(&m)?;
    Ok(view_to_handle(&m))
}

/// Proof<SC> -> a new lsp_proof handle (free with sys::lsp_proof_free);
/// panics on a malformed proof (see [`try_from_proof`])
pub fn from_proof<SC>(proof: &Proof<SC>) -> *mut sys::lsp_proof
where
    SC: StarkGenericConfig,
    Proof<SC>: Serialize,
{
    try_from_proof(proof).unwrap_or_else(|e| panic!("from_proof: malformed Proof<SC>: {e}"))
}

fn view_to_handle(m: &ProofMirror) -> *mut sys::lsp_proof {
    let fp = &m.opening_proof;
    let flat = |xs: &[[Val; 1]]| xs.iter().map(|d| d[0]).collect::<Vec<Val>>();
    let (mut trows, mut tpaths, mut qrows, mut qpaths, mut sibs, mut fpaths) =
        (Vec::new(), Vec::new(), Vec::new(), Vec::new(), Vec::new(), Vec::new());
    for qp in &fp.query_proofs {
        assert_eq!(qp.input_proof.len(), 2, "two committed rounds: trace, quotient chunks");
        trows.extend(qp.input_proof[0].opened_values.concat());
        tpaths.extend(flat(&qp.input_proof[0].opening_proof));
        qrows.extend(qp.input_proof[1].opened_values.concat());
        qpaths.extend(flat(&qp.input_proof[1].opening_proof));
        for s in &qp.commit_phase_openings {
            sibs.push(s.sibling_value);
            fpaths.extend(flat(&s.opening_proof));
        }
    }
    let fpl: Vec<u32> = fp
        .query_proofs
        .first()
        .map(|qp| qp.commit_phase_openings.iter().map(|s| s.opening_proof.len() as u32).collect())
        .unwrap_or_else(|| vec![0; fp.commit_phase_commits.len()]);
    let roots: Vec<Val> = fp.commit_phase_commits.iter().map(|c| <[Val; 1]>::from(*c)[0]).collect();
    let qc: Vec<Val> = m.opened_values.quotient_chunks.concat();
    let single = [
        <[Val; 1]>::from(m.commitments.trace)[0],
        <[Val; 1]>::from(m.commitments.quotient_chunks)[0],
        fp.pow_witness,
    ];
    let v = sys::lsp_proof_view {
        degree_bits: m.degree_bits as u32,
        log_quotient_chunks: qc.len().trailing_zeros(),
        width: m.opened_values.trace_local.len() as u32,
        num_queries: fp.query_proofs.len() as u32,
        num_fri_rounds: roots.len() as u32,
        final_poly_len: fp.final_poly.len() as u32,
        input_path_len: fp.query_proofs.first().map_or(0, |qp| qp.input_proof[0].opening_proof.len() as u32),
        fri_path_lens: fpl.as_ptr(),
        trace_commit: fr_ptr(&single[0..1]),
        quotient_commit: fr_ptr(&single[1..2]),
        pow_witness: fr_ptr(&single[2..3]),
        trace_local: fr_ptr(&m.opened_values.trace_local),
        trace_next: fr_ptr(&m.opened_values.trace_next),
        quotient_chunks: fr_ptr(&qc),
        fri_commits: fr_ptr(&roots),
        final_poly: fr_ptr(&fp.final_poly),
        trace_rows: fr_ptr(&trows),
        trace_paths: fr_ptr(&tpaths),
        quotient_rows: fr_ptr(&qrows),
        quotient_paths: fr_ptr(&qpaths),
        fri_siblings: fr_ptr(&sibs),
        fri_paths: fr_ptr(&fpaths),
    };
    let mut out: *mut sys::lsp_proof = std::ptr::null_mut();
    check_global(unsafe { sys::lsp_proof_from_view(&v, &mut out) }, "lsp_proof_from_view");
    out
}

fn take_bytes(h: *mut sys::lsp_proof) -> Vec<u8> {
    let mut n = 0usize;
    check_global(unsafe { sys::lsp_proof_serialize(h, std::ptr::null_mut(), 0, &mut n) }, "lsp_proof_serialize");
    let mut b = vec![0u8; n];
    check_global(unsafe { sys::lsp_proof_serialize(h, b.as_mut_ptr(), n, &mut n) }, "lsp_proof_serialize");
    unsafe { sys::lsp_proof_free(h) };
    b
}

/// the library's wire bytes of a Proof<SC>
pub fn proof_to_bytes<SC>(proof: &Proof<SC>) -> Vec<u8>
where
    SC: StarkGenericConfig,
    Proof<SC>: Serialize,
{
    take_bytes(from_proof(proof))
}

/// Proof<SC> from the library's wire bytes
pub fn proof_from_bytes<SC>(b: &[u8]) -> Proof<SC>
where
    SC: StarkGenericConfig,
    Proof<SC>: DeserializeOwned,
{
    let mut h: *mut sys::lsp_proof = std::ptr::null_mut();
    check_global(unsafe { sys::lsp_proof_deserialize(b.as_ptr(), b.len(), &mut h) }, "lsp_proof_deserialize");
    let p = to_proof::<SC>(h);
    unsafe { sys::lsp_proof_free(h) };
    p
}

/// `p3_uni_stark::prove(config, air, challenger, trace, public_values)`
/// (`bin/src/main.rs:80-86`) on the GPU.  `air` is the AIR descriptor
/// (INTEGRATION.md `air_descriptor`), `public_values` = `[alpha, delta]`.
/// The result goes to `p3_uni_stark::verify` unchanged (`bin/src/main.rs:88-96`).
pub fn prove<SC>(
    ctx: &Ctx,
    trace: &p3_matrix::dense::RowMajorMatrix<Val>,
    air: &[i32],
    public_values: &[Val],
) -> Proof<SC>
where
    SC: StarkGenericConfig,
    Proof<SC>: DeserializeOwned,
{
    use p3_matrix::Matrix;
    let mut out: *mut sys::lsp_proof = std::ptr::null_mut();
    let rc = unsafe {
        sys::lsp_prove(
            ctx.raw(),
            fr_ptr(&trace.values),
            trace.height(),
            trace.width(),
            air.as_ptr(),
            air.len(),
            fr_ptr(public_values),
            public_values.len(),
            sys::LSP_MEM_HOST,
            &mut out,
        )
    };
    ctx.check(rc, "lsp_prove");
    let p = to_proof::<SC>(out);
    unsafe { sys::lsp_proof_free(out) };
    p
}
