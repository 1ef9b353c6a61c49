"""CPU-only checks of the native library (no GPU compute): the C ABI exports every symbol
include/rclone_crypt_gpu.h declares, and the host logic of the cipher.go mirror (sizes,
calculateUnderlying, nonce arithmetic, scrypt key derivation, error strings) against the
reference's own tables (tests/golden/reference_kat.json, from backend/crypt/cipher_test.go).
"""
import os
import re

import pytest

from rclone_amd import _lib, crypt

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    src = open(os.path.join(ROOT, "include", "rclone_crypt_gpu.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    names = set(re.findall(r"\b((?:xs|rc)_[a-z0-9_]+)\s*\(", src))
    return sorted(n for n in names if not n.endswith("_fn"))


def test_library_exports_every_header_symbol():
    lib = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 40
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    assert set(syms) <= set(_lib.SYMBOLS) | {"xs_engine_create"}


def test_failure_hooks_only_in_the_test_library():
    # xs_api.cpp's failure injection (-DXS_TEST_HOOKS) is compiled into the test-only twin alone:
    # the product library has no such entry points, the twin has them and the same build id
    import ctypes
    from rclone_amd import build
    assert not hasattr(_lib.lib(), "xs_test_fail_batch")
    h = ctypes.CDLL(build.HOOKS_LIB)
    assert hasattr(h, "xs_test_fail_batch") and hasattr(h, "xs_test_failed_requests")
    assert build.library_build_id(build.HOOKS_LIB) == build.library_build_id(build.LIB)


def test_version_and_devices():
    lib = _lib.lib()
    assert b"gfx950" in lib.xs_version()
    assert lib.xs_device_count() >= 0


def test_build_id_ties_library_to_tree():
    from rclone_amd import build
    want = build.build_sources_sha256()
    assert _lib.build_id() == want == build.library_build_id()
    assert not build.needs_build()


_STALE_PROBE = r"""
import sys
sys.path.insert(0, {root!r})
from rclone_amd import _lib, build
build.LIB = {path!r}
try:
    _lib.lib()
except _lib.StaleLibraryError as e:
    print("REFUSED", e)
else:
    print("LOADED")
"""


def _probe(tmp_path, data, extra_env=None, patch_check=False):
    import subprocess
    import sys
    p = tmp_path / "librclone_crypt.so"
    p.write_bytes(data)
    code = _STALE_PROBE.format(root=ROOT, path=str(p))
    if patch_check:  # the file check passes: only the loaded library's own xs_build_id() can refuse
        code = code.replace("build.LIB =", "build.library_build_id = lambda path=None: build.build_sources_sha256()\nbuild.LIB =")
    env = dict(os.environ, RCLONE_AMD_REBUILD="0", **(extra_env or {}))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=env, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout


def test_stale_library_is_refused(tmp_path):
    """A library whose embedded build id is not this tree's (built from other sources) is
    refused, both by the file check before loading and by the loaded library's xs_build_id()."""
    from rclone_amd import build
    data = open(build.LIB, "rb").read()
    want = build.build_sources_sha256().encode()
    i = data.index(build.BUILD_ID_TAG + want)
    stale = bytearray(data)
    j = i + len(build.BUILD_ID_TAG)
    stale[j:j + 8] = b"00000000" if want[:8] != b"00000000" else b"11111111"
    assert "LOADED" in _probe(tmp_path, bytes(data))
    out = _probe(tmp_path, bytes(stale))
    assert "REFUSED" in out and "built from sources" in out
    out = _probe(tmp_path, bytes(stale), patch_check=True)
    assert "REFUSED" in out and "loaded library reports build" in out


def test_library_from_another_compiler_is_refused(tmp_path):
    """The compiler is stamped beside the build id: where hipcc is installed, a library another
    hipcc / ROCm built counts as stale (rebuilt, or refused with RCLONE_AMD_REBUILD=0)."""
    from rclone_amd import build
    if not build.hipcc_available():
        pytest.skip("no hipcc: the compiler stamp is not checked")
    data = open(build.LIB, "rb").read()
    cc = build.compiler_id().encode()
    i = data.index(build.COMPILER_TAG + cc) + len(build.COMPILER_TAG)
    other = bytearray(data)
    other[i:i + 16] = b"0123456789abcdef" if cc != b"0123456789abcdef" else b"fedcba9876543210"
    out = _probe(tmp_path, bytes(other))
    assert "REFUSED" in out and "built by compiler" in out


_FAKE_HIPCC = r"""#!{py}
# TEST INFRASTRUCTURE: stands in for hipcc -- '-c' writes an empty object slowly (widens the race),
# the link copies a current library (the real one, stamped with this stand-in's compiler id) and
# is logged
import os, shutil, sys, time
args = sys.argv[1:]
out = args[args.index("-o") + 1]
if "-c" in args:
    time.sleep(0.5)
    open(out, "wb").close()
else:
    with open({log!r}, "a") as f:
        f.write("link %d %s\n" % (os.getpid(), os.path.basename(out).split(".so")[0]))
    shutil.copyfile({lib!r}, out)
"""


def test_concurrent_loaders_rebuild_once(tmp_path):
    """Four processes (ranks of one job) find a stale library at once: exactly one rebuilds it,
    under the build lock, and all four load the same, current build id.  The package is copied
    into a scratch tree (same relative paths, hence the same build id), with a stand-in hipcc whose
    link step hands back this tree's real library."""
    import shutil
    import subprocess
    import sys

    from rclone_amd import build
    if not build.hipcc_available():
        pytest.skip("no hipcc")
    tree = tmp_path / "tree"
    pkg = tree / "rclone_amd"
    shutil.copytree(os.path.join(ROOT, "rclone_amd"), pkg,
                    ignore=shutil.ignore_patterns("__pycache__", "*.so", "*.lock", "*.tmp*"))
    shutil.copytree(os.path.join(ROOT, "include"), tree / "include")
    data = bytearray(open(build.LIB, "rb").read())
    want = build.build_sources_sha256()
    j = data.index(build.BUILD_ID_TAG + want.encode()) + len(build.BUILD_ID_TAG)
    data[j:j + 8] = b"00000000" if want[:8] != "00000000" else b"11111111"
    (pkg / "librclone_crypt.so").write_bytes(bytes(data))  # stale: another build id
    log = tmp_path / "hipcc.log"
    fake = tmp_path / "hipcc"
    good = tmp_path / "good.so"
    fake.write_text(_FAKE_HIPCC.format(py=sys.executable, log=str(log), lib=str(good)))
    fake.chmod(0o755)
    env = dict(os.environ, HIPCC=str(fake), RCLONE_AMD_REBUILD="1")
    # the library the stand-in's link hands back: this tree's build, stamped with the compiler id
    # the scratch tree computes for the stand-in
    cc = subprocess.check_output([sys.executable, "-c", "import sys; sys.path.insert(0, %r)\n"
                                  "from rclone_amd import build; print(build.compiler_id())" % str(tree)],
                                 env=env, text=True).strip()
    real = bytearray(open(build.LIB, "rb").read())
    k = real.index(build.COMPILER_TAG) + len(build.COMPILER_TAG)
    real[k:k + 16] = cc.encode()
    good.write_bytes(bytes(real))
    code = ("import sys; sys.path.insert(0, %r)\nfrom rclone_amd import _lib\nprint('ID', _lib.build_id())" % str(tree))
    procs = [subprocess.Popen([sys.executable, "-c", code], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                              env=env, cwd=str(tmp_path)) for _ in range(4)]
    outs = [p.communicate(timeout=180) for p in procs]
    for p, (o, e) in zip(procs, outs):
        assert p.returncode == 0, e[-2000:]
    ids = {o.split("ID", 1)[1].strip() for o, _ in outs}
    assert ids == {want}
    # one build: the library and its test-only twin linked once each (a second build would link
    # both again)
    links = [ln.split() for ln in log.read_text().splitlines()]
    assert sorted(x[2] for x in links) == ["librclone_crypt", "librclone_crypt_testhooks"], links
    assert build.library_build_id(str(pkg / "librclone_crypt.so")) == want


def test_encrypted_decrypted_size(ref_kat):
    for n, e in ref_kat["encrypted_size"]:
        assert crypt.encrypted_size(n) == e
        assert crypt.decrypted_size(e) == n
    for n, name in ref_kat["decrypted_size_errors"]:
        with pytest.raises(getattr(crypt, name)):
            crypt.decrypted_size(n)


def test_calculate_underlying(ref_kat):
    for off, lim, woff, wlim, wdisc, wblocks in ref_kat["calculate_underlying"]:
        assert crypt.calculate_underlying(off, lim) == (woff, wlim, wdisc, wblocks)


def test_nonce_increment_add(ref_kat):
    for row in ref_kat["nonce_increment"]:
        assert crypt.nonce_increment(bytes.fromhex(row["in"])).hex() == row["out"]
    for row in ref_kat["nonce_add"]:
        assert crypt.nonce_add(bytes.fromhex(row["in"]), row["add"]).hex() == row["out"]


def test_key(ref_kat):
    # TestKey cipher_test.go:1609-1642
    c = crypt.Cipher()
    assert c.data_key == bytes(32) and c.name_key == bytes(32) and c.name_tweak == bytes(16)
    for kat in ref_kat["key_kat"]:
        c.key(kat["password"], kat["salt"])
        assert c.data_key.hex() == kat["dataKey"]
        assert c.name_key.hex() == kat["nameKey"]
        assert c.name_tweak.hex() == kat["nameTweak"]
    c.key("", "")
    assert c.data_key == bytes(32)


def test_error_strings():
    lib = _lib.lib()
    assert lib.rc_error_string(-104) == b"failed to authenticate decrypted block - bad password?"
    assert lib.rc_error_string(-101) == b"file is too short to be encrypted"
    assert lib.rc_error_string(-106) == b"Seek beyond end of file"
    assert str(crypt.ErrorEncryptedBadMagic(crypt.ErrorEncryptedBadMagic.message)) == \
        "not an encrypted file - bad magic string"


def test_nonce_plus_matches_nonce_add():
    # shard.nonce_plus (vectorised nonce0 + i for descriptor tables) == nonce.add (cipher.go:665)
    import numpy as np

    from oracle import pyoracle as orc
    from rclone_amd.shard import nonce_plus
    idx = np.array([0, 1, 2, 255, 256, 65535, 2**32, 2**63, 2**64 - 1], dtype=np.uint64)
    for n0 in (bytes(24), b"\xff" * 24, b"\xfe" + b"\xff" * 7 + bytes(range(16)), bytes(range(24)),
               b"\xff" * 23 + b"\x00"):
        got = nonce_plus(n0, idx)
        for j, i in enumerate(idx.tolist()):
            assert got[j].tobytes() == orc.nonce_add(n0, i), (n0.hex(), i)


def test_splitmix_block_stream():
    from rclone_amd.testdata import splitmix64_block, splitmix64_bytes
    whole = splitmix64_bytes(7, 5 * 65536)
    for g in range(5):
        assert splitmix64_block(7, g) == whole[g * 65536:(g + 1) * 65536]


def test_random_source():
    # TestRandomSource (cipher_test.go:1054-1067): the test infrastructure first.  The reference
    # copies 1e8 bytes; 1e6 here (every byte crosses Python).  The vectorised form the parity
    # tests use (testdata.random_source) is the same sequence.
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from go_readers import EOF, RandomSource

    from rclone_amd.testdata import random_source
    n = 10**6
    source, sink = RandomSource(n), RandomSource(n)
    copied = 0
    while True:
        p, err = source.read_go(32768)
        copied += sink.write(p)
        if err is EOF:
            break
    assert copied == n
    assert RandomSource(70000).read_go(70001) == (random_source(70000), EOF)
    source = RandomSource(n)
    source.read_go(16)
    with pytest.raises(AssertionError, match="Error in stream at 1$"):
        RandomSource(n).write(source.read_go(32768)[0])


def test_device_entry_points_reject_bad_arguments():
    # argument checks run before any HIP call, so they hold on a machine without a GPU
    import ctypes
    lib = _lib.lib()
    XS_ERR_INVALID = -1  # include/rclone_crypt_gpu.h
    word = ctypes.c_uint64(0)
    buf = ctypes.create_string_buffer(65536 + 16)
    aligned = (ctypes.addressof(buf) + 15) & ~15
    assert lib.xs_verify_blocks_dev(None, 1, 0, 1, 7, ctypes.byref(word), None) == XS_ERR_INVALID
    assert "xs_verify_blocks_dev" in _lib.last_error()
    assert lib.xs_verify_blocks_dev(aligned, 1, 0, 1, 7, None, None) == XS_ERR_INVALID
    assert lib.xs_verify_blocks_dev(aligned + 4, 1, 0, 1, 7, ctypes.byref(word), None) == XS_ERR_INVALID
    assert lib.xs_verify_blocks_dev(aligned, 1, 0, 0, 7, ctypes.byref(word), None) == XS_ERR_INVALID
    assert lib.xs_fill_blocks_dev(aligned, 1, 0, 0, 7, None) == XS_ERR_INVALID


def test_reopen_error_keeps_the_openers_error():
    # DecryptDataSeek at an offset: the header opens, the re-open at the block fails; the error is
    # "couldn't reopen file with offset and limit: %w" around the opener's own error
    # (cipher.go:1011) -- host-only, no GPU involved (rc_decrypt_data_seek_ex)
    from tests.go_readers import Buffer

    class Gone(Exception):
        pass

    c = crypt.Cipher("potato", "")
    calls = []

    def open_fn(off, lim):
        calls.append((off, lim))
        if len(calls) == 1:
            return Buffer(b"RCLONE\x00\x00" + bytes(range(24)))
        raise Gone("object not found")

    with pytest.raises(crypt.CryptError) as ei:
        c.decrypt_data_seek(open_fn, 70000, -1)
    assert "couldn't reopen file with offset and limit: object not found" in str(ei.value)
    assert isinstance(ei.value.__cause__, Gone)
    assert calls == [(0, 32), (32 + 65552, -1)]


def test_ablation_patches_still_apply():
    """tools/archive/ablate_variant.py keeps the diagnostic (wrong-output) kernel variants out of the
    product file as text patches; their anchors must follow the product kernel or they rot."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("ablate_variant", os.path.join(ROOT, "tools", "archive", "ablate_variant.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    src = open(mod.SRC).read()
    for name in mod.PATCHES:
        patched = mod.variant_source(name)  # raises SystemExit when an anchor is missing
        assert patched != src, name
