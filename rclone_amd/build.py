"""Build the native library in-tree: rclone_amd/librclone_crypt.so (hipcc, gfx950).

The .so holds the HIP kernels (csrc/xs_kernels.hip), the device C ABI (csrc/xs_api.cpp) and
the host mirror of backend/crypt/cipher.go (csrc/cipher.cpp, csrc/scrypt.cpp).  It is
git-ignored but travels to the GPU box with the repo snapshot.
"""
import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "librclone_crypt.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RCLONE_AMD_ARCH", "gfx950")

SOURCES = ["xs_kernels.hip", "xs_md5.hip", "xs_eme.hip", "xs_probe.hip", "xs_api.cpp", "xs_topo.cpp", "cipher.cpp", "names.cpp",
           "names_gpu.cpp", "scrypt.cpp"]


# what the crypt kernels (xs_seal / xs_open / keygen) are compiled from: PMC counters committed under
# profiles/ (tools/make_traffic.py) are valid only for this exact set of bytes
KERNEL_SOURCES = ["rclone_amd/csrc/xs_kernels.hip", "rclone_amd/csrc/xs_salsa_lazy.h",
                  "rclone_amd/csrc/xs_internal.h"]


def kernel_sources_sha256(root=None):
    import hashlib
    root = root or os.path.dirname(HERE)
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        p = os.path.join(root, rel)
        h.update(rel.encode() + b"\0")
        if os.path.exists(p):
            with open(p, "rb") as f:
                h.update(f.read())
    return h.hexdigest()


def sources():
    return [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def needs_build():
    if not os.path.exists(LIB):
        return True
    t = os.path.getmtime(LIB)
    deps = sources() + [os.path.join(CSRC, h) for h in ("xs_internal.h", "xs_aes.h", "rc_internal.h", "xs_host_md5.h", "md5_workers.h", "md5_x16.h", "xs_topo.h")] + [
                        os.path.join(os.path.dirname(HERE), "include", "rclone_crypt_gpu.h")]
    return any(os.path.getmtime(d) > t for d in deps if os.path.exists(d))


def build(force=False, verbose=False):
    if not force and not needs_build():
        return LIB
    cmd = [HIPCC, f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared", "-Wall",
           "-Wno-unused-result", "-o", LIB] + sources() + ["-lpthread"]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.check_call(cmd)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB)
