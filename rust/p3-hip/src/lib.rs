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
pub use proof::{from_proof, prove, proof_from_bytes, proof_to_bytes, to_proof};

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
        let rc_ptr = if p.round_constants.is_empty() { std::ptr::null() } else { fr_ptr(&p.round_constants) };
        let raw_params = sys::lsp_params {
            sbox_degree: p.sbox_degree,
            rounds_f: p.rounds_f,
            rounds_p: p.rounds_p,
            round_constants: rc_ptr,
            log_blowup: p.log_blowup,
            log_final_poly_len: p.log_final_poly_len,
            num_queries: p.num_queries,
            proof_of_work_bits: p.proof_of_work_bits,
            public_degree: p.public_degree,
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
