//! Links libfantoch_hip.so, built by `python -m fantoch_amd.build`
//! (hipcc --offload-arch=gfx950) from this repository's fantoch_amd/csrc.
use std::path::PathBuf;
use std::process::Command;

fn main() {
    println!("cargo:rerun-if-env-changed=FANTOCH_HIP_LIB_DIR");
    println!("cargo:rerun-if-env-changed=FANTOCH_AMD_ROOT");
    let dir = match std::env::var("FANTOCH_HIP_LIB_DIR") {
        Ok(d) => PathBuf::from(d),
        Err(_) => {
            // build it from a checkout of the engine repository
            let root = PathBuf::from(
                std::env::var("FANTOCH_AMD_ROOT")
                    .expect("set FANTOCH_HIP_LIB_DIR (dir of libfantoch_hip.so) or FANTOCH_AMD_ROOT"),
            );
            let ok = Command::new("python3")
                .args(&["-m", "fantoch_amd.build"])
                .current_dir(&root)
                .status()
                .expect("python3 -m fantoch_amd.build")
                .success();
            assert!(ok, "building libfantoch_hip.so failed");
            root.join("fantoch_amd")
        }
    };
    println!("cargo:rustc-link-search=native={}", dir.display());
    println!("cargo:rustc-link-lib=dylib=fantoch_hip");
    println!("cargo:rustc-link-arg=-Wl,-rpath,{}", dir.display());
}
