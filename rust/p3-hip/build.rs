//! Link liblsp_hip.so: LSP_LIB_DIR = the directory holding it
//! (linea_stark_prover_amd/_lib after `python -m linea_stark_prover_amd.build`).
fn main() {
    println!("cargo:rerun-if-env-changed=LSP_LIB_DIR");
    if let Ok(dir) = std::env::var("LSP_LIB_DIR") {
        println!("cargo:rustc-link-search=native={dir}");
        println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    }
    println!("cargo:rustc-link-lib=dylib=lsp_hip");
}
