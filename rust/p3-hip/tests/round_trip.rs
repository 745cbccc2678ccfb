//! Proof<Config> of the reference's exact Config type (bin/src/config.rs:9-25)
//! from a GPU proof, and back to identical library bytes.  Needs a GPU and
//! LSP_LIB_DIR (see build.rs); mirrors tests/test_proof_view.py.
use p3_bls12_377_fr::Poseidon2Bls12337;
use p3_challenger::HashChallenger;
use p3_dft::Radix2DitParallel;
use p3_fri::TwoAdicFriPcs;
use p3_matrix::dense::RowMajorMatrix;
use p3_merkle_tree::MerkleTreeMmcs;
use p3_symmetric::{CompressionFunctionFromHasher, PaddingFreeSponge};
use p3_uni_stark::{Proof, StarkConfig};

use p3_hip::{sys, Ctx, Params, Val};

type Perm = Poseidon2Bls12337<3>;
type Hash = PaddingFreeSponge<Perm, 3, 2, 1>;
type Compress = CompressionFunctionFromHasher<Hash, 2, 1>;
type ValMmcs = MerkleTreeMmcs<Val, Val, Hash, Compress, 1>;
type Config = StarkConfig<TwoAdicFriPcs<Val, Radix2DitParallel<Val>, ValMmcs, ValMmcs>, Val, HashChallenger<Val, Hash, 1>>;

#[test]
fn gpu_proof_is_a_plonky3_proof() {
    let params = Params::default();
    let ctx = Ctx::new(0, &params);
    let (log_n, ncols) = (10u32, 3u32);
    let (mut alpha, mut delta) = (sys::lsp_fr::default(), sys::lsp_fr::default());
    let mut rc = vec![sys::lsp_fr::default(); 3 * 8 + 22];
    assert_eq!(unsafe { sys::lsp_seeded_setup(0x4C494E4541, 8, 22, &mut alpha, &mut delta, rc.as_mut_ptr()) }, 0);
    let w = (2 * ncols + 2) as usize;
    let mut rows = vec![sys::lsp_fr::default(); (1usize << log_n) * w];
    assert_eq!(unsafe { sys::lsp_gen_permutation_trace(0x4C494E4541, log_n, ncols, &alpha, &delta, 0, rows.as_mut_ptr()) }, 0);
    let values: Vec<Val> = unsafe { std::slice::from_raw_parts(rows.as_ptr() as *const Val, rows.len()) }.to_vec();
    let trace = RowMajorMatrix::new(values, w);
    let n = ncols as i32;
    let mut air = vec![1, 1, n, n];
    air.extend(0..2 * n);
    air.extend([2 * n, 2 * n + 1]);
    let pv: Vec<Val> = unsafe { std::slice::from_raw_parts([alpha, delta].as_ptr() as *const Val, 2) }.to_vec();

    let proof: Proof<Config> = p3_hip::prove(&ctx, &trace, &air, &pv);
    let bytes = p3_hip::proof_to_bytes(&proof);
    let again: Proof<Config> = p3_hip::proof_from_bytes(&bytes);
    assert_eq!(p3_hip::proof_to_bytes(&again), bytes);
    let air_len = air.len();
    let ok = unsafe { sys::lsp_verify(ctx.raw(), air.as_ptr(), air_len, [alpha, delta].as_ptr(), 2, bytes.as_ptr(), bytes.len()) };
    assert_eq!(ok, 0);
}
