//! `TwoAdicSubgroupDft` on the GPU: the `Dft` alias of `bin/src/config.rs:22`
//! (`Radix2DitParallel<Val>`), called by `TwoAdicFriPcs::commit` for the trace
//! (`coset_lde_batch(evals, log_blowup, GENERATOR)`) and the quotient chunks.
use std::sync::Arc;

use p3_dft::{Radix2DitParallel, TwoAdicSubgroupDft};
use p3_field::FieldAlgebra;
use p3_matrix::bitrev::BitReversedMatrixView;
use p3_matrix::dense::RowMajorMatrix;
use p3_matrix::Matrix;

use crate::{fr1, fr_ptr, fr_ptr_mut, sys, Ctx, Val};

#[derive(Clone)]
pub struct HipDft {
    ctx: Arc<Ctx>,
}

impl HipDft {
    pub fn new(ctx: Arc<Ctx>) -> Self {
        HipDft { ctx }
    }
}

impl Default for HipDft {
    fn default() -> Self {
        HipDft { ctx: crate::global() }
    }
}

impl TwoAdicSubgroupDft<Val> for HipDft {
    // as Radix2DitParallel: the LDE is stored bit-reversed and viewed in
    // natural order, so `.bit_reverse_rows().to_row_major_matrix()` in
    // TwoAdicFriPcs::commit is the stored matrix itself (no copy)
    type Evaluations = BitReversedMatrixView<RowMajorMatrix<Val>>;

    fn dft_batch(&self, mat: RowMajorMatrix<Val>) -> Self::Evaluations {
        // a plain coefficient DFT is not on the prover's path (only
        // coset_lde_batch is) and the library exports no coefficient-input
        // transform: this runs the CPU radix-2 DIT (identical, unique result)
        // and costs CPU time for a caller that does use it
        Radix2DitParallel::<Val>::default().dft_batch(mat)
    }

    /// `out[bitrev(i)] = p(shift * w_N^i)` for every column -- lsp_coset_lde_batch
    fn coset_lde_batch(&self, mat: RowMajorMatrix<Val>, added_bits: usize, shift: Val) -> Self::Evaluations {
        let (h, w) = (mat.height(), mat.width());
        let mut out = vec![Val::ZERO; (h << added_bits) * w];
        let rc = unsafe {
            sys::lsp_coset_lde_batch(
                self.ctx.raw(),
                fr_ptr(&mat.values),
                h,
                w,
                added_bits as u32,
                fr1(&shift),
                fr_ptr_mut(&mut out),
                sys::LSP_MEM_HOST,
            )
        };
        self.ctx.check(rc, "lsp_coset_lde_batch");
        BitReversedMatrixView::new(RowMajorMatrix::new(out, w))
    }
}
