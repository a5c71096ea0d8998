//! Builds libhbgpu.so with hipcc for gfx950 from this repository's sources
//! (hydrabadger_amd/csrc/*.hip + include/hbgpu.h), or links a prebuilt one.
//!
//!   HBGPU_SRC      repository root (default: two levels above this crate)
//!   HIPCC          hipcc to use (default /opt/rocm/bin/hipcc)
//!   HBGPU_LIB_DIR  with --features prebuilt: directory holding libhbgpu.so
use std::{env, fs, path::PathBuf, process::Command};

fn main() {
    if env::var_os("CARGO_FEATURE_PREBUILT").is_some() {
        let dir = env::var("HBGPU_LIB_DIR").expect("--features prebuilt needs HBGPU_LIB_DIR");
        println!("cargo:rustc-link-search=native={}", dir);
        println!("cargo:rustc-link-lib=dylib=hbgpu");
        return;
    }
    let manifest = PathBuf::from(env::var("CARGO_MANIFEST_DIR").unwrap());
    let root = env::var("HBGPU_SRC").map(PathBuf::from).unwrap_or_else(|_| manifest.join("../.."));
    let csrc = root.join("hydrabadger_amd").join("csrc");
    let out = PathBuf::from(env::var("OUT_DIR").unwrap());
    let hipcc = env::var("HIPCC").unwrap_or_else(|_| "/opt/rocm/bin/hipcc".into());
    let mut objs = Vec::new();
    for entry in fs::read_dir(&csrc).expect("hydrabadger_amd/csrc") {
        let path = entry.unwrap().path();
        let ext = path.extension().and_then(|e| e.to_str()).unwrap_or("");
        if ext == "h" {
            println!("cargo:rerun-if-changed={}", path.display());
        }
        if ext != "hip" {
            continue;
        }
        println!("cargo:rerun-if-changed={}", path.display());
        let obj = out.join(format!("{}.o", path.file_name().unwrap().to_str().unwrap()));
        let ok = Command::new(&hipcc)
            .args(&["-O3", "-std=c++20", "-fPIC", "--offload-arch=gfx950", "-fconstexpr-steps=100000000", "-c"])
            .arg(&path)
            .arg("-o")
            .arg(&obj)
            .status()
            .expect("run hipcc")
            .success();
        assert!(ok, "hipcc failed on {}", path.display());
        objs.push(obj);
    }
    println!("cargo:rerun-if-changed={}", root.join("include").join("hbgpu.h").display());
    let lib = out.join("libhbgpu.so");
    let ok = Command::new(&hipcc)
        .args(&["--offload-arch=gfx950", "-shared", "-fPIC", "-o"])
        .arg(&lib)
        .args(&objs)
        .status()
        .expect("link with hipcc")
        .success();
    assert!(ok, "linking libhbgpu.so failed");
    println!("cargo:rustc-link-search=native={}", out.display());
    println!("cargo:rustc-link-lib=dylib=hbgpu");
}
