//! Links the prebuilt librrte_hip.so (rrte_amd/csrc/Makefile builds it for gfx950 with hipcc).
//! RRTE_HIP_LIB_DIR points at the directory holding it; the rpath lets the example binaries run
//! without LD_LIBRARY_PATH.
fn main() {
    let dir = std::env::var("RRTE_HIP_LIB_DIR").unwrap_or_else(|_| "../../rrte_amd/lib".into());
    println!("cargo:rustc-link-search=native={dir}");
    println!("cargo:rustc-link-lib=dylib=rrte_hip");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{dir}");
    println!("cargo:rerun-if-env-changed=RRTE_HIP_LIB_DIR");
}
