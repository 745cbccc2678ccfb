//! `FriGenericConfig<Val>` with the fold on the GPU (the north_star's
//! "FriFolder"): `TwoAdicFriGenericConfig::fold_matrix` / `fold_row`
//! ([EXT p3-fri]).  `TwoAdicFriPcs::open` instantiates its own
//! `TwoAdicFriGenericConfig`, so in the fine-grained plug-in (Dft + Mmcs
//! swapped) FRI folds stay on the CPU; they run on the GPU (fused into the next
//! round's leaf hashing) in the coarse path, [`crate::prove`].  This type
//! serves a caller that drives `p3_fri::prover::prove` itself.
use std::marker::PhantomData;
use std::sync::Arc;

use p3_field::FieldAlgebra;
use p3_fri::FriGenericConfig;
use p3_matrix::Matrix;

use crate::{fr1, fr_ptr, fr_ptr_mut, sys, Ctx, Val};

pub struct HipFriFolder<InputProof, InputError> {
    ctx: Arc<Ctx>,
    _marker: PhantomData<(InputProof, InputError)>,
}

impl<InputProof, InputError> HipFriFolder<InputProof, InputError> {
    pub fn new(ctx: Arc<Ctx>) -> Self {
        HipFriFolder { ctx, _marker: PhantomData }
    }
}

impl<InputProof, InputError: std::fmt::Debug> FriGenericConfig<Val> for HipFriFolder<InputProof, InputError> {
    type InputProof = InputProof;
    type InputError = InputError;

    fn extra_query_index_bits(&self) -> usize {
        0
    }

    /// lsp_fri_fold_row (host): the verifier-side fold of one pair
    fn fold_row(&self, index: usize, log_height: usize, beta: Val, evals: impl Iterator<Item = Val>) -> Val {
        let e: Vec<Val> = evals.collect();
        assert_eq!(e.len(), 2, "arity-2 FRI");
        let mut out = Val::ZERO;
        unsafe {
            sys::lsp_fri_fold_row(index, log_height as u32, fr1(&beta), fr1(&e[0]), fr1(&e[1]), fr_ptr_mut(std::slice::from_mut(&mut out)))
        };
        out
    }

    /// lsp_fri_fold: out[i] = (1/2 + beta/2 g^-bitrev(i)) m[i][0] + (1/2 - beta/2 g^-bitrev(i)) m[i][1]
    fn fold_matrix<M: Matrix<Val>>(&self, beta: Val, m: M) -> Vec<Val> {
        assert_eq!(m.width(), 2, "arity-2 FRI");
        let v: Vec<Val> = m.rows().flatten().collect();
        let mut out = vec![Val::ZERO; v.len() / 2];
        let rc = unsafe {
            sys::lsp_fri_fold(self.ctx.raw(), fr_ptr(&v), v.len(), fr1(&beta), fr_ptr_mut(&mut out), sys::LSP_MEM_HOST)
        };
        self.ctx.check(rc, "lsp_fri_fold");
        out
    }
}
