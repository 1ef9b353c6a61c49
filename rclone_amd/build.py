"""Build the native library in-tree: rclone_amd/librclone_crypt.so (hipcc, gfx950).

The .so holds the HIP kernels (csrc/xs_kernels.hip), the device C ABI (csrc/xs_api.cpp) and
the host mirror of backend/crypt/cipher.go (csrc/cipher.cpp, csrc/scrypt.cpp).  It is
git-ignored but travels to the GPU box with the repo snapshot.

Provenance: every build embeds `build_sources_sha256()` -- the sha256 of every file under
csrc/, the public header and the compile command -- as the library's build id
(`xs_build_id()`, and a tagged string the loader reads from the file without loading it).
`needs_build()` compares that id with the tree's, not file times, so a library built from other
sources is never taken for this tree's (rclone_amd/_lib.py rebuilds or refuses it).  The compiler
is stamped beside it (`compiler_id()`: a digest of the installed hipcc / clang / ROCm release,
tag "xs-build-compiler:"): where
hipcc is installed, a library built by another hipcc / ROCm counts as stale too.  It is kept out of
the build id so a box without a compiler can still load the library it was given.
"""
import fcntl
import hashlib
import os
import re
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
CSRC = os.path.join(HERE, "csrc")
LIB = os.path.join(HERE, "librclone_crypt.so")
# TEST-ONLY twin of LIB: the same objects with csrc/xs_api.cpp compiled under -DXS_TEST_HOOKS (failure
# injection into the engine's combined batches, tests/test_engine_failure_gpu.py).  Nothing in the
# product loads it; rclone_amd/_lib.py hooks_lib() is its only loader.
HOOKS_LIB = os.path.join(HERE, "librclone_crypt_testhooks.so")
HOOKS_SOURCE = "xs_api.cpp"
HEADER = os.path.join(ROOT, "include", "rclone_crypt_gpu.h")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
ARCH = os.environ.get("RCLONE_AMD_ARCH", "gfx950")

SOURCES = ["xs_kernels.hip", "xs_md5.hip", "xs_eme.hip", "xs_probe.hip", "xs_api.cpp", "xs_topo.cpp", "cipher.cpp", "names.cpp",
           "names_gpu.cpp", "scrypt.cpp"]
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-Wall", "-Wno-unused-result"]
BUILD_ID_TAG = b"xs-build-id:"
COMPILER_TAG = b"xs-build-compiler:"
_compiler_id = None


# what the crypt kernels (xs_seal / xs_open / keygen) are compiled from: PMC counters committed under
# profiles/ (tools/make_traffic.py) are valid only for this exact set of bytes
KERNEL_SOURCES = ["rclone_amd/csrc/xs_kernels.hip", "rclone_amd/csrc/xs_salsa_lazy.h",
                  "rclone_amd/csrc/xs_internal.h"]


def kernel_sources_sha256(root=None):
    root = root or ROOT
    h = hashlib.sha256()
    for rel in KERNEL_SOURCES:
        p = os.path.join(root, rel)
        h.update(rel.encode() + b"\0")
        if os.path.exists(p):
            with open(p, "rb") as f:
                h.update(f.read())
    return h.hexdigest()


def hipcc_available():
    import shutil
    return os.path.exists(HIPCC) or shutil.which(HIPCC) is not None


def sources():
    return [os.path.join(CSRC, s) for s in SOURCES if os.path.exists(os.path.join(CSRC, s))]


def build_inputs():
    """Every file the library is compiled from: all of csrc/ (sources and headers) + the C header."""
    files = sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC)
                   if f.endswith((".hip", ".cpp", ".h")))
    return files + [HEADER]


def build_sources_sha256():
    h = hashlib.sha256()
    h.update(" ".join([ARCH] + FLAGS + SOURCES).encode() + b"\0")
    for p in build_inputs():
        h.update(os.path.relpath(p, ROOT).encode() + b"\0")
        with open(p, "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


def library_build_id(path=LIB):
    """The build id embedded in a built library file (None if absent or unstamped)."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    m = re.search(re.escape(BUILD_ID_TAG) + rb"([0-9a-f]{64})\0", data)
    return m.group(1).decode() if m else None


def compiler_id():
    """First 16 hex digits of a sha256 over what identifies the installed compiler -- the resolved
    hipcc and clang paths, the clang binary's size and the ROCm release files -- or None without a
    usable hipcc.  Read from the file system, never by running hipcc: the loader runs in processes
    that have initialised the GPU, where no child program should be started."""
    global _compiler_id
    if _compiler_id is None:
        import shutil
        hipcc = shutil.which(HIPCC) or HIPCC
        if not os.path.exists(hipcc):
            return None
        real = os.path.realpath(hipcc)
        rocm = os.path.dirname(os.path.dirname(real))
        h = hashlib.sha256(real.encode() + b"\0")
        clang = os.path.realpath(os.path.join(rocm, "lib", "llvm", "bin", "clang"))
        if os.path.exists(clang):
            h.update(clang.encode() + b"\0" + str(os.path.getsize(clang)).encode() + b"\0")
        info = os.path.join(rocm, ".info")
        try:
            entries = sorted(os.listdir(info)) if os.path.isdir(info) else []
        except OSError:
            entries = []
        for f in entries:  # regular, readable files only: anything else never blocks a load
            p = os.path.join(info, f)
            try:
                if not os.path.isfile(p):
                    continue
                with open(p, "rb") as fh:
                    h.update(f.encode() + b"\0" + fh.read() + b"\0")
            except OSError:
                continue
        _compiler_id = h.hexdigest()[:16]
    return _compiler_id


def library_compiler_id(path=LIB):
    """The compiler digest stamped into a built library file (None if absent or unstamped)."""
    try:
        with open(path, "rb") as f:
            data = f.read()
    except OSError:
        return None
    m = re.search(re.escape(COMPILER_TAG) + rb"([0-9a-f]{16})\0", data)
    return m.group(1).decode() if m else None


def stale_reason(path=LIB):
    """Why the library at `path` is not this tree's build (None when it is): its build id differs
    from the tree's sources, or -- where hipcc is installed -- another compiler built it."""
    have, want = library_build_id(path), build_sources_sha256()
    if have != want:
        return f"built from sources {have or 'unknown/missing'}, this tree is {want}"
    cc = compiler_id() if hipcc_available() else None
    if cc is not None and library_compiler_id(path) != cc:
        return f"built by compiler {library_compiler_id(path) or 'unstamped'}, installed hipcc is {cc}"
    return None


def needs_build():
    return stale_reason(LIB) is not None or stale_reason(HOOKS_LIB) is not None


def build(force=False, verbose=False):
    """Compile into a temporary file and rename it over LIB, under a lock: ranks of one job that
    find the library stale at the same time build it once, and no process ever maps a
    half-written file."""
    with open(LIB + ".lock", "a") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        if not force and not needs_build():
            return LIB
        bid = build_sources_sha256()
        cc = compiler_id() or "unstamped"
        tmp = f"{LIB}.tmp{os.getpid()}"
        tmp_hooks = f"{HOOKS_LIB}.tmp{os.getpid()}"
        # one object per source, compiled in parallel (xs_kernels.hip alone is most of the time),
        # then one link
        import tempfile
        from concurrent.futures import ThreadPoolExecutor
        with tempfile.TemporaryDirectory(prefix="rclone_amd_build_") as od:
            def compile_one(src, hooks=False):
                obj = os.path.join(od, os.path.basename(src) + (".hooks.o" if hooks else ".o"))
                cmd = ([HIPCC, f"--offload-arch={ARCH}"] + [f for f in FLAGS if f != "-shared"] +
                       [f'-DXS_BUILD_ID="{bid}"', f'-DXS_BUILD_COMPILER="{cc}"'] + (["-DXS_TEST_HOOKS"] if hooks else []) +
                       ["-c", "-o", obj, src])
                if verbose:
                    print(" ".join(cmd), file=sys.stderr)
                subprocess.check_call(cmd)
                return obj
            jobs = max(1, min(len(SOURCES), int(os.environ.get("MAX_JOBS", os.cpu_count() or 4)), 16))
            srcs = sources()
            hooks_src = os.path.join(CSRC, HOOKS_SOURCE)
            with ThreadPoolExecutor(jobs) as ex:
                hooks_fut = ex.submit(compile_one, hooks_src, True)
                objs = list(ex.map(compile_one, srcs))
                hooks_obj = hooks_fut.result()
            hooks_objs = [hooks_obj if src == hooks_src else o for src, o in zip(srcs, objs)]
            try:
                for out, tmpf, ob in ((HOOKS_LIB, tmp_hooks, hooks_objs), (LIB, tmp, objs)):
                    cmd = [HIPCC, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", tmpf] + ob + ["-lpthread"]
                    if verbose:
                        print(" ".join(cmd), file=sys.stderr)
                    subprocess.check_call(cmd)
                    os.replace(tmpf, out)
            finally:
                for tmpf in (tmp, tmp_hooks):
                    if os.path.exists(tmpf):
                        os.unlink(tmpf)
    return LIB


if __name__ == "__main__":
    build(force="--force" in sys.argv, verbose=True)
    print(LIB, build_sources_sha256())
