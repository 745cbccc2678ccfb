//! p3-hip: liblsp_hip.so (MI355X / gfx950 HIP kernels) behind the Plonky3
//! traits the reference plugs together in `bin/src/config.rs:9-25`.
//!
//! Two ways in, as in INTEGRATION.md:
//! * fine-grained -- swap the type aliases of `bin/src/config.rs:19-22`:
//!   `type ValMmcs = p3_hip::HipMmcs; type ChallengeMmcs = p3_hip::HipMmcs;
//!   type Dft = p3_hip::HipDft;` -- `TwoAdicFriPcs` then runs its coset LDEs
//!   and Merkle commitments on the GPU, everything else unchanged;
//! * coarse -- replace the `p3_uni_stark::prove` call of `bin/src/main.rs:80-86`
//!   by [`prove`], which runs the whole proof on the GPU and returns a real
//!   `p3_uni_stark::Proof<Config>`; the `p3_uni_stark::verify` call of
//!   `bin/src/main.rs:88-96` stays as it is.
//!
//! Elements cross the ABI in ark-ff's in-memory form (4 x u64 Montgomery,
//! `lsp_fr`), so `&[Bls12_377Fr]` is passed without conversion.
//! Every library error panics, as Plonky3 does on bad input (lsp.h
//! "Errors"); `verify_batch` returns `Err` instead.

pub mod sys;

mod dft;
mod fri;
mod mmcs;
mod proof;

pub use dft::HipDft;
pub use fri::HipFriFolder;
pub use mmcs::{HipMmcs, HipMmcsError, HipTree};
pub use proof::{from_proof, prove, proof_from_bytes, proof_to_bytes, to_proof, try_from_proof};

use std::ffi::CStr;
use std::ptr::NonNull;
use std::sync::{Arc, OnceLock};

pub type Val = p3_bls12_377_fr::Bls12_377Fr;

// the ABI passes Val slices as lsp_fr: same size, same bytes (ark-ff Fp256)
const _: () = assert!(std::mem::size_of::<Val>() == std::mem::size_of::<sys::lsp_fr>());

#[inline]
pub(crate) fn fr_ptr(v: &[Val]) -> *const sys::lsp_fr {
    v.as_ptr() as *const sys::lsp_fr
}

#[inline]
pub(crate) fn fr_ptr_mut(v: &mut [Val]) -> *mut sys::lsp_fr {
    v.as_mut_ptr() as *mut sys::lsp_fr
}

#[inline]
pub(crate) fn fr1(v: &Val) -> *const sys::lsp_fr {
    v as *const Val as *const sys::lsp_fr
}

/// a copy of `n` lsp_fr at `p` as Vals (p may be dangling when n == 0)
pub(crate) unsafe fn vals(p: *const sys::lsp_fr, n: usize) -> Vec<Val> {
    if n == 0 {
        return Vec::new();
    }
    std::slice::from_raw_parts(p as *const Val, n).to_vec()
}

/// `StarkConfig` / `FriConfig` / `Perm::new_from_rng` parameters
/// (`bin/src/main.rs:49-64`; conventions U1-U12 of DESIGN.md).
#[derive(Clone, Debug)]
pub struct Params {
    pub sbox_degree: u32,
    pub rounds_f: u32,
    pub rounds_p: u32,
    /// 3 * rounds_f + rounds_p constants in new_from_rng order; empty = the
    /// library's documented seeded set (U4)
    pub round_constants: Vec<Val>,
    pub log_blowup: u32,
    pub log_final_poly_len: u32,
    pub num_queries: u32,
    pub proof_of_work_bits: u32,
    pub public_degree: i32,
    /// U7: `challenger.observe(log_degree)` before the trace root (default true)
    pub observe_log_degree: bool,
    /// U7: `challenger.observe_slice(public_values)` before alpha (default true)
    pub observe_public_values: bool,
    /// U7: `TwoAdicFriPcs::open` observes the opened values before alpha_fri
    /// (default false; later upstream Plonky3 does)
    pub observe_opened_values: bool,
    /// U8: `sample_bits` from the Montgomery form's low bits (default false:
    /// the canonical value's)
    pub sample_bits_montgomery: bool,
    /// U12: the final polynomial is observed before grinding (default true)
    pub observe_final_poly: bool,
    /// U2: the internal layer's diagonal d (s_i <- sum + d_i s_i); None =
    /// (1, 1, 2).  Must be the diagonal of the fork's
    /// `Poseidon2InternalLayerBls12337<3>`, which [`perm`] instantiates.
    pub internal_diag: Option<[Val; 3]>,
    /// U3: the external layer M_E, row-major; None = circ(2, 1, 1).  Must be
    /// the fork's `Poseidon2ExternalLayerBls12337<3>` matrix.
    pub external_mds: Option<[Val; 9]>,
}

impl Params {
    /// The Poseidon2 constants `Perm::new_from_rng(rounds_f, rounds_p, rng)`
    /// (`bin/src/main.rs:49`) draws, drawn from `rng` in the same order and
    /// by the fork's own samplers: `ExternalLayerConstants::new_from_rng`
    /// (the rounds_f/2 initial, then the rounds_f/2 terminal `[Val; 3]`),
    /// then rounds_p internal constants.  So
    /// `perm(&Params::from_rng(8, 22, &mut rng))` is the permutation
    /// `Perm::new_from_rng(8, 22, &mut rng)` builds from the same rng state,
    /// and the library proves with exactly those constants.  The one-line
    /// change at `bin/src/main.rs:49`:
    /// `let params = p3_hip::Params::from_rng(8, 22, &mut rng); let perm = p3_hip::perm(&params);`
    pub fn from_rng<R: rand::Rng>(rounds_f: usize, rounds_p: usize, rng: &mut R) -> Params
    where
        rand::distributions::Standard: rand::distributions::Distribution<Val> + rand::distributions::Distribution<[Val; 3]>,
    {
        use rand::distributions::Standard;
        let ext = p3_poseidon2::ExternalLayerConstants::<Val, 3>::new_from_rng(rounds_f, rng);
        let internal: Vec<Val> = (&mut *rng).sample_iter(Standard).take(rounds_p).collect();
        let mut rc = Vec::with_capacity(3 * rounds_f + rounds_p);
        for r in ext.get_initial_constants().iter().chain(ext.get_terminal_constants()) {
            rc.extend_from_slice(r);
        }
        rc.extend(internal);
        Params { rounds_f: rounds_f as u32, rounds_p: rounds_p as u32, round_constants: rc, ..Params::default() }
    }

    /// `round_constants`, or the library's seeded set (lsp_seeded_setup, U4) when empty
    pub fn resolved_round_constants(&self) -> Vec<Val> {
        if !self.round_constants.is_empty() {
            return self.round_constants.clone();
        }
        let n = (3 * self.rounds_f + self.rounds_p) as usize;
        let (mut a, mut d) = (sys::lsp_fr::default(), sys::lsp_fr::default());
        let mut rc = vec![sys::lsp_fr::default(); n];
        let st = unsafe {
            sys::lsp_seeded_setup(DEFAULT_SEED, self.rounds_f, self.rounds_p, &mut a, &mut d, rc.as_mut_ptr())
        };
        check_global(st, "lsp_seeded_setup");
        unsafe { vals(rc.as_ptr(), n) }
    }
}

/// the library's documented seed (U4/U5, "LINEA")
pub const DEFAULT_SEED: u64 = 0x4C494E4541;

/// `Poseidon2Bls12337<3>` built from exactly `p`'s round constants: the
/// `Perm` of `bin/src/main.rs:49`, which the Hash, both Mmcs and the
/// challenger share (`main.rs:50-57,78,88`), so the reference's unchanged
/// `p3_uni_stark::verify` hashes with the constants the library proved with.
pub fn perm(p: &Params) -> p3_bls12_377_fr::Poseidon2Bls12337<3> {
    let rc = p.resolved_round_constants();
    let half = (p.rounds_f / 2) as usize;
    let row = |k: usize| -> [Val; 3] { [rc[3 * k], rc[3 * k + 1], rc[3 * k + 2]] };
    let initial: Vec<[Val; 3]> = (0..half).map(row).collect();
    let terminal: Vec<[Val; 3]> = (half..2 * half).map(row).collect();
    let internal = rc[6 * half..].to_vec();
    p3_bls12_377_fr::Poseidon2Bls12337::<3>::new(
        p3_poseidon2::ExternalLayerConstants::new(initial, terminal),
        internal,
    )
}

impl Default for Params {
    fn default() -> Self {
        Params {
            sbox_degree: 11,
            rounds_f: 8,
            rounds_p: 22,
            round_constants: Vec::new(),
            log_blowup: 3,
            log_final_poly_len: 0,
            num_queries: 33,
            proof_of_work_bits: 0,
            public_degree: 1,
            observe_log_degree: true,
            observe_public_values: true,
            observe_opened_values: false,
            sample_bits_montgomery: false,
            observe_final_poly: true,
            internal_diag: None,
            external_mds: None,
        }
    }
}

/// One `lsp_ctx`: a GPU (or none: [`Ctx::host_only`]), one HIP stream and a
/// buffer pool.  The library serialises calls on a context with a mutex, so
/// `&Ctx` may be used from any rayon thread (the traits require `Sync`).
pub struct Ctx {
    raw: NonNull<sys::lsp_ctx>,
}

unsafe impl Send for Ctx {}
unsafe impl Sync for Ctx {}

impl Ctx {
    pub fn new(device: i32, p: &Params) -> Ctx {
        // lsp_ctx_create needs the constants: the seeded set when none are given
        let rc = p.resolved_round_constants();
        let rc_ptr = fr_ptr(&rc);
        let raw_params = sys::lsp_params {
            struct_size: std::mem::size_of::<sys::lsp_params>() as u32,
            sbox_degree: p.sbox_degree,
            rounds_f: p.rounds_f,
            rounds_p: p.rounds_p,
            round_constants: rc_ptr,
            log_blowup: p.log_blowup,
            log_final_poly_len: p.log_final_poly_len,
            num_queries: p.num_queries,
            proof_of_work_bits: p.proof_of_work_bits,
            public_degree: p.public_degree,
            internal_diag: p.internal_diag.as_ref().map_or(std::ptr::null(), |d| fr_ptr(d)),
            external_mds: p.external_mds.as_ref().map_or(std::ptr::null(), |m| fr_ptr(m)),
            skip_log_degree: (!p.observe_log_degree) as u32,
            skip_public_values: (!p.observe_public_values) as u32,
            observe_opened_values: p.observe_opened_values as u32,
            sample_bits_montgomery: p.sample_bits_montgomery as u32,
            skip_final_poly: (!p.observe_final_poly) as u32,
        };
        let mut out: *mut sys::lsp_ctx = std::ptr::null_mut();
        let rc = unsafe { sys::lsp_ctx_create(device, &raw_params, &mut out) };
        check_global(rc, "lsp_ctx_create");
        Ctx { raw: NonNull::new(out).expect("lsp_ctx_create returned null") }
    }

    /// verifier-only context: never touches a GPU
    pub fn host_only(p: &Params) -> Ctx {
        Ctx::new(sys::LSP_HOST_ONLY, p)
    }

    pub fn raw(&self) -> *mut sys::lsp_ctx {
        self.raw.as_ptr()
    }

    /// the library's message for a failed call on this context
    pub fn last_error(&self) -> String {
        unsafe { cstr(sys::lsp_last_error(self.raw.as_ptr())) }
    }

    /// panic on a non-zero status, with the library's message
    pub fn check(&self, rc: i32, what: &str) {
        if rc != sys::LSP_OK {
            panic!("{what} failed ({rc}): {}", self.last_error());
        }
    }

    /// `(span, ms)` of the last proof, named as the reference's bench.log spans
    pub fn last_timings(&self) -> Vec<(String, f64)> {
        let mut n = 0usize;
        unsafe { sys::lsp_last_timings(self.raw(), std::ptr::null_mut(), std::ptr::null_mut(), 0, &mut n) };
        let mut ms = vec![0f64; n];
        let mut names = vec![std::ptr::null(); n];
        unsafe { sys::lsp_last_timings(self.raw(), ms.as_mut_ptr(), names.as_mut_ptr(), n, &mut n) };
        names.into_iter().zip(ms).map(|(p, t)| (unsafe { cstr(p) }, t)).collect()
    }
}

impl Drop for Ctx {
    fn drop(&mut self) {
        unsafe { sys::lsp_ctx_destroy(self.raw.as_ptr()) };
    }
}

pub(crate) unsafe fn cstr(p: *const std::os::raw::c_char) -> String {
    if p.is_null() {
        String::new()
    } else {
        CStr::from_ptr(p).to_string_lossy().into_owned()
    }
}

pub(crate) fn check_global(rc: i32, what: &str) {
    if rc != sys::LSP_OK {
        panic!("{what} failed ({rc}): {}", unsafe { cstr(sys::lsp_last_error(std::ptr::null())) });
    }
}

static GLOBAL: OnceLock<Arc<Ctx>> = OnceLock::new();

/// The process-wide context behind `HipDft::default()` / `HipMmcs::default()`
/// (`TwoAdicSubgroupDft` requires `Default`).  Call once before building the
/// config; later calls return the first context.
pub fn init(device: i32, p: &Params) -> Arc<Ctx> {
    GLOBAL.get_or_init(|| Arc::new(Ctx::new(device, p))).clone()
}

pub(crate) fn global() -> Arc<Ctx> {
    GLOBAL.get().cloned().expect("p3_hip::init(device, &params) must run before the Dft / Mmcs are built")
}
