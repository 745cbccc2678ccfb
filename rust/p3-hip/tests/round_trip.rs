//! A GPU proof checked by the reference's own verifier, unchanged.
//!
//! The config is built exactly as `bin/src/main.rs:49-78` builds it, with the
//! one change INTEGRATION.md section 3 describes at `main.rs:49`: the
//! Poseidon2 constants come from `p3_hip::Params::from_rng` (the draws
//! `Perm::new_from_rng(8, 22, &mut rng)` would make) and `perm` is
//! `p3_hip::perm(&params)`, so the Mmcs and the challenger hash with the
//! constants the library proves with.  The AIR is the reference's `air`
//! crate; the proof goes through `p3_uni_stark::verify` (`main.rs:88-96`).
//! Needs a GPU and LSP_LIB_DIR (see build.rs); the Python twins are
//! tests/test_proof_view.py and tests/test_linear_layers.py (its GPU cases).
use air::air_permutation::AirPermutationConfig;
use air::{AirConfig, LineaAIR};
use p3_bls12_377_fr::Poseidon2Bls12337;
use p3_challenger::HashChallenger;
use p3_dft::Radix2DitParallel;
use p3_fri::{FriConfig, TwoAdicFriPcs};
use p3_matrix::dense::RowMajorMatrix;
use p3_merkle_tree::MerkleTreeMmcs;
use p3_symmetric::{CompressionFunctionFromHasher, PaddingFreeSponge};
use p3_uni_stark::{verify, Proof, StarkConfig};
use rand::distributions::Standard;
use rand::rngs::StdRng;
use rand::{Rng, SeedableRng};

use p3_hip::{sys, Ctx, Params, Val};

type Perm = Poseidon2Bls12337<3>;
type Hash = PaddingFreeSponge<Perm, 3, 2, 1>;
type Compress = CompressionFunctionFromHasher<Hash, 2, 1>;
type ValMmcs = MerkleTreeMmcs<Val, Val, Hash, Compress, 1>;
type Challenger = HashChallenger<Val, Hash, 1>;
type Config = StarkConfig<TwoAdicFriPcs<Val, Radix2DitParallel<Val>, ValMmcs, ValMmcs>, Val, Challenger>;

fn config(perm: &Perm) -> (Config, Hash) {
    let hash = Hash::new(perm.clone());
    let compress = Compress::new(hash.clone());
    let mmcs = ValMmcs::new(hash.clone(), compress.clone());
    let fri = FriConfig { log_blowup: 3, log_final_poly_len: 0, num_queries: 33, proof_of_work_bits: 0, mmcs: mmcs.clone() };
    (Config::new(TwoAdicFriPcs::new(Radix2DitParallel::default(), mmcs, fri)), hash)
}

#[test]
fn gpu_proof_passes_p3_uni_stark_verify() {
    // bin/src/main.rs:29-31,49 with a seeded rng in place of thread_rng
    let mut rng = StdRng::seed_from_u64(0x4C494E4541);
    let alpha: Val = rng.sample(Standard);
    let delta: Val = rng.sample(Standard);
    let params = Params::from_rng(8, 22, &mut rng);
    let perm = p3_hip::perm(&params);
    let ctx = Ctx::new(0, &params);

    // a 3x3 permutation trace with its witness columns (trace/src/permutation.rs:24-93)
    let (log_n, ncols) = (10u32, 3u32);
    let w = (2 * ncols + 2) as usize;
    let mut rows = vec![sys::lsp_fr::default(); (1usize << log_n) * w];
    let (a, d) = (&alpha as *const Val as *const sys::lsp_fr, &delta as *const Val as *const sys::lsp_fr);
    assert_eq!(unsafe { sys::lsp_gen_permutation_trace(7, log_n, ncols, a, d, 0, rows.as_mut_ptr()) }, 0);
    let values: Vec<Val> = unsafe { std::slice::from_raw_parts(rows.as_ptr() as *const Val, rows.len()) }.to_vec();
    let trace = RowMajorMatrix::new(values, w);
    let n = ncols as usize;
    let cfg = AirPermutationConfig {
        a_columns_ids: (0..n).collect(),
        b_columns_ids: (n..2 * n).collect(),
        b_inverse_id: 2 * n,
        check_id: 2 * n + 1,
    };
    let mut desc = vec![1, 1, n as i32, n as i32];
    desc.extend((0..2 * n as i32).collect::<Vec<_>>());
    desc.extend([2 * n as i32, 2 * n as i32 + 1]);
    let air = LineaAIR::new(vec![AirConfig::Permutation(cfg)]);
    let pv = vec![alpha, delta];

    let proof: Proof<Config> = p3_hip::prove(&ctx, &trace, &desc, &pv);

    // bin/src/main.rs:88-96, unchanged
    let (config, hash) = config(&perm);
    let mut challenger = Challenger::new(vec![], hash);
    verify(&config, &air, &mut challenger, &proof, &pv).expect("p3_uni_stark::verify rejected the GPU proof");

    // and the library's own verifier and wire bytes agree
    let bytes = p3_hip::proof_to_bytes(&proof);
    let again: Proof<Config> = p3_hip::proof_from_bytes(&bytes);
    assert_eq!(p3_hip::proof_to_bytes(&again), bytes);
    let st = unsafe { sys::lsp_verify(ctx.raw(), desc.as_ptr(), desc.len(), pv.as_ptr().cast(), 2, bytes.as_ptr(), bytes.len()) };
    assert_eq!(st, 0);
}
