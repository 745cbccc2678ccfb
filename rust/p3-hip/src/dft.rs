//! `TwoAdicSubgroupDft` on the GPU: the `Dft` alias of `bin/src/config.rs:22`
//! (`Radix2DitParallel<Val>`), called by `TwoAdicFriPcs::commit` for the trace
//! (`coset_lde_batch(evals, log_blowup, GENERATOR)`) and the quotient chunks.
use std::sync::Arc;

use p3_dft::TwoAdicSubgroupDft;
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

impl HipDft {
    fn forward(&self, mat: RowMajorMatrix<Val>, shift: Option<Val>) -> BitReversedMatrixView<RowMajorMatrix<Val>> {
        let (h, w) = (mat.height(), mat.width());
        let mut out = vec![Val::ZERO; h * w];
        let rc = unsafe {
            sys::lsp_coset_dft_batch(
                self.ctx.raw(),
                fr_ptr(&mat.values),
                h,
                w,
                shift.as_ref().map_or(std::ptr::null(), fr1),
                fr_ptr_mut(&mut out),
                sys::LSP_MEM_HOST,
            )
        };
        self.ctx.check(rc, "lsp_coset_dft_batch");
        BitReversedMatrixView::new(RowMajorMatrix::new(out, w))
    }

    fn inverse(&self, mat: RowMajorMatrix<Val>, shift: Option<Val>) -> RowMajorMatrix<Val> {
        let (h, w) = (mat.height(), mat.width());
        let mut out = vec![Val::ZERO; h * w];
        let rc = unsafe {
            sys::lsp_coset_idft_batch(
                self.ctx.raw(),
                fr_ptr(&mat.values),
                h,
                w,
                shift.as_ref().map_or(std::ptr::null(), fr1),
                fr_ptr_mut(&mut out),
                sys::LSP_MEM_HOST,
            )
        };
        self.ctx.check(rc, "lsp_coset_idft_batch");
        RowMajorMatrix::new(out, w)
    }
}

impl TwoAdicSubgroupDft<Val> for HipDft {
    // as Radix2DitParallel: the LDE is stored bit-reversed and viewed in
    // natural order, so `.bit_reverse_rows().to_row_major_matrix()` in
    // TwoAdicFriPcs::commit is the stored matrix itself (no copy)
    type Evaluations = BitReversedMatrixView<RowMajorMatrix<Val>>;

    /// `out[bitrev(j)] = p(w_h^j)` for every column -- lsp_coset_dft_batch, shift 1
    fn dft_batch(&self, mat: RowMajorMatrix<Val>) -> Self::Evaluations {
        self.forward(mat, None)
    }

    /// `out[bitrev(j)] = p(shift * w_h^j)` -- lsp_coset_dft_batch
    fn coset_dft_batch(&self, mat: RowMajorMatrix<Val>, shift: Val) -> Self::Evaluations {
        self.forward(mat, Some(shift))
    }

    /// natural-order evaluations on H_h -> coefficients -- lsp_coset_idft_batch, shift 1
    fn idft_batch(&self, mat: RowMajorMatrix<Val>) -> RowMajorMatrix<Val> {
        self.inverse(mat, None)
    }

    /// natural-order evaluations on shift * H_h -> coefficients -- lsp_coset_idft_batch
    fn coset_idft_batch(&self, mat: RowMajorMatrix<Val>, shift: Val) -> RowMajorMatrix<Val> {
        self.inverse(mat, Some(shift))
    }

    /// `lde_batch` = `coset_lde_batch` with shift 1 (the trait default would
    /// go through idft_batch + dft_batch)
    fn lde_batch(&self, mat: RowMajorMatrix<Val>, added_bits: usize) -> Self::Evaluations {
        self.coset_lde_batch(mat, added_bits, Val::ONE)
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
