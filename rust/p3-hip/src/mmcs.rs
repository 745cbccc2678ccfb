//! `Mmcs<Val>` on the GPU: the `ValMmcs` / `ChallengeMmcs` aliases of
//! `bin/src/config.rs:19-20` (`MerkleTreeMmcs<Val, Val, Hash, Compress, 1>`).
//! Same commitment and proof types as MerkleTreeMmcs (`Hash<Val, Val, 1>`,
//! `Vec<[Val; 1]>`), so proofs and verifiers are interchangeable.  The tree
//! layers stay in HBM (`lsp_tree`); the committed matrices stay on the host
//! because `TwoAdicFriPcs` reads them back through `get_matrices`.
use std::sync::Arc;

use p3_commit::Mmcs;
use p3_field::FieldAlgebra;
use p3_matrix::{Dimensions, Matrix};
use p3_symmetric::Hash;

use crate::{fr1, fr_ptr, fr_ptr_mut, sys, Ctx, Val};

#[derive(Clone)]
pub struct HipMmcs {
    ctx: Arc<Ctx>,
}

impl HipMmcs {
    pub fn new(ctx: Arc<Ctx>) -> Self {
        HipMmcs { ctx }
    }
}

impl Default for HipMmcs {
    fn default() -> Self {
        HipMmcs { ctx: crate::global() }
    }
}

/// `ProverData<M>`: the device tree plus the committed host matrices
pub struct HipTree<M> {
    tree: *mut sys::lsp_tree,
    leaves: Vec<M>,
    height: usize,
    widths: Vec<usize>,
}

// lsp_tree is only read after commit, under the owning context's mutex
unsafe impl<M: Send> Send for HipTree<M> {}
unsafe impl<M: Sync> Sync for HipTree<M> {}

impl<M> Drop for HipTree<M> {
    fn drop(&mut self) {
        unsafe { sys::lsp_tree_free(self.tree) };
    }
}

#[derive(Debug)]
pub enum HipMmcsError {
    WrongBatchSize,
    UnequalHeights,
    WrongProofLength,
    RootMismatch,
}

impl Mmcs<Val> for HipMmcs {
    type ProverData<M> = HipTree<M>;
    type Commitment = Hash<Val, Val, 1>;
    type Proof = Vec<[Val; 1]>;
    type Error = HipMmcsError;

    /// lsp_merkle_commit: leaf i = hash_iter(row i of every matrix, in order),
    /// nodes = compress(left, right).  Every caller in this prover commits
    /// matrices of one height (trace; quotient chunks; one FRI round).
    fn commit<M: Matrix<Val>>(&self, inputs: Vec<M>) -> (Self::Commitment, Self::ProverData<M>) {
        assert!(!inputs.is_empty(), "HipMmcs::commit of no matrices");
        let height = inputs[0].height();
        assert!(inputs.iter().all(|m| m.height() == height), "HipMmcs commits matrices of one height");
        // any M: Matrix -> one contiguous host copy per matrix for the upload
        // (host memory holds the matrices twice while this runs)
        let staged: Vec<Vec<Val>> = inputs.iter().map(|m| m.rows().flatten().collect()).collect();
        let ptrs: Vec<*const sys::lsp_fr> = staged.iter().map(|v| fr_ptr(v)).collect();
        let widths: Vec<usize> = inputs.iter().map(|m| m.width()).collect();
        let mut root = [Val::ZERO];
        let mut tree: *mut sys::lsp_tree = std::ptr::null_mut();
        let rc = unsafe {
            sys::lsp_merkle_commit(
                self.ctx.raw(),
                ptrs.as_ptr(),
                widths.as_ptr(),
                ptrs.len(),
                height,
                sys::LSP_MEM_HOST,
                fr_ptr_mut(&mut root),
                &mut tree,
            )
        };
        self.ctx.check(rc, "lsp_merkle_commit");
        (Hash::from(root), HipTree { tree, leaves: inputs, height, widths })
    }

    fn open_batch<M: Matrix<Val>>(&self, index: usize, d: &HipTree<M>) -> (Vec<Vec<Val>>, Self::Proof) {
        let mut rows = vec![Val::ZERO; d.widths.iter().sum()];
        let mut path = vec![Val::ZERO; d.height.trailing_zeros() as usize];
        let rc = unsafe { sys::lsp_merkle_open(d.tree, index, fr_ptr_mut(&mut rows), fr_ptr_mut(&mut path)) };
        self.ctx.check(rc, "lsp_merkle_open");
        let mut opened = Vec::with_capacity(d.widths.len());
        let mut off = 0;
        for &w in &d.widths {
            opened.push(rows[off..off + w].to_vec());
            off += w;
        }
        (opened, path.into_iter().map(|x| [x]).collect())
    }

    fn get_matrices<'a, M: Matrix<Val>>(&self, d: &'a HipTree<M>) -> Vec<&'a M> {
        d.leaves.iter().collect()
    }

    /// lsp_merkle_verify on the host (the verifier never needs a GPU)
    fn verify_batch(
        &self,
        commit: &Self::Commitment,
        dimensions: &[Dimensions],
        index: usize,
        opened_values: &[Vec<Val>],
        proof: &Self::Proof,
    ) -> Result<(), Self::Error> {
        if dimensions.is_empty() || dimensions.len() != opened_values.len() {
            return Err(HipMmcsError::WrongBatchSize);
        }
        let height = dimensions[0].height;
        if !height.is_power_of_two() || dimensions.iter().any(|d| d.height != height) {
            return Err(HipMmcsError::UnequalHeights);
        }
        let log_height = height.trailing_zeros();
        if proof.len() != log_height as usize {
            return Err(HipMmcsError::WrongProofLength);
        }
        let widths: Vec<usize> = opened_values.iter().map(|r| r.len()).collect();
        let rows: Vec<Val> = opened_values.iter().flatten().copied().collect();
        let path: Vec<Val> = proof.iter().map(|d| d[0]).collect();
        let root: [Val; 1] = (*commit).into();
        let rc = unsafe {
            sys::lsp_merkle_verify(
                self.ctx.raw(),
                fr1(&root[0]),
                widths.as_ptr(),
                widths.len(),
                log_height,
                index,
                fr_ptr(&rows),
                fr_ptr(&path),
            )
        };
        match rc {
            sys::LSP_OK => Ok(()),
            sys::LSP_E_VERIFY => Err(HipMmcsError::RootMismatch),
            _ => {
                self.ctx.check(rc, "lsp_merkle_verify");
                unreachable!()
            }
        }
    }
}
