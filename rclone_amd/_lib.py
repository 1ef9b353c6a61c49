"""ctypes binding of rclone_amd/librclone_crypt.so (include/rclone_crypt_gpu.h).

There is no fallback: if the native library is missing or has no GPU, calls fail loudly.
"""
import ctypes
import os

from . import build as _build

_lib = None

c_u8p = ctypes.POINTER(ctypes.c_uint8)
vp = ctypes.c_void_p
u64 = ctypes.c_uint64
i64 = ctypes.c_int64
i32 = ctypes.c_int32


class XsBlockDesc(ctypes.Structure):
    _fields_ = [("src_off", ctypes.c_uint64), ("dst_off", ctypes.c_uint64), ("len", ctypes.c_uint32),
                ("reserved", ctypes.c_uint32), ("nonce", ctypes.c_uint8 * 24)]


assert ctypes.sizeof(XsBlockDesc) == 48


class XsNameDesc(ctypes.Structure):
    _fields_ = [("off", ctypes.c_uint64), ("nblk", ctypes.c_uint32), ("reserved", ctypes.c_uint32)]


assert ctypes.sizeof(XsNameDesc) == 16

READ_FN = ctypes.CFUNCTYPE(i64, vp, c_u8p, i64, ctypes.POINTER(i32))
CLOSE_FN = ctypes.CFUNCTYPE(i32, vp)
RANGE_SEEK_FN = ctypes.CFUNCTYPE(i32, vp, i64, i32, i64)


class RcReader(ctypes.Structure):
    _fields_ = [("read", READ_FN), ("close", CLOSE_FN), ("range_seek", RANGE_SEEK_FN), ("user", vp)]


OPEN_FN = ctypes.CFUNCTYPE(i32, vp, i64, i64, ctypes.POINTER(RcReader))

# (name, restype, argtypes)
_SIGS = [
    ("xs_version", ctypes.c_char_p, []),
    ("xs_build_id", ctypes.c_char_p, []),
    ("xs_last_error", ctypes.c_char_p, []),
    ("xs_device_count", ctypes.c_int, []),
    ("xs_workspace_bytes", ctypes.c_size_t, [u64]),
    ("xs_seal_object_dev", ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, u64, vp, u64, vp, vp, vp]),
    ("xs_open_object_dev", ctypes.c_int, [ctypes.c_char_p, ctypes.c_char_p, u64, vp, u64, vp, vp, vp, vp]),
    ("xs_seal_batch_dev", ctypes.c_int, [ctypes.c_char_p, vp, u64, vp, u64, vp, u64, vp, vp]),
    ("xs_open_batch_dev", ctypes.c_int, [ctypes.c_char_p, vp, u64, vp, u64, vp, u64, vp, vp, vp]),
    ("xs_keygen_object_dev", ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, u64, u64, vp, vp]),
    ("xs_crypt_dev", ctypes.c_int, [ctypes.c_int, vp, u64, vp, vp, vp, vp]),
    ("xs_keygen_batch_dev", ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, vp, u64, vp, u64, vp, u64, vp, vp]),
    ("xs_fill_random_dev", ctypes.c_int, [vp, u64, u64, vp]),
    ("xs_fill_blocks_dev", ctypes.c_int, [vp, u64, u64, u64, u64, vp]),
    ("xs_verify_blocks_dev", ctypes.c_int, [vp, u64, u64, u64, u64, vp, vp]),
    ("xs_md5_batch_dev", ctypes.c_int, [vp, u64, vp, u64, vp, vp, vp]),
    ("xs_clock_probe_dev", ctypes.c_int, [vp, vp, ctypes.c_double, vp]),
    ("xs_engine_create", vp, [ctypes.c_int, ctypes.c_uint32, ctypes.c_int]),
    ("xs_engine_destroy", None, [vp]),
    ("xs_engine_seal", ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_char_p, u64, vp, u64, vp]),
    ("xs_engine_open", ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_char_p, u64, vp, u64, vp, vp]),
    ("xs_engine_open_range", ctypes.c_int, [vp, ctypes.c_char_p, ctypes.c_char_p, u64, vp, u64, vp, vp, u64, u64]),
    ("xs_engine_seal_md5", ctypes.c_int, [vp, ctypes.c_char_p, u64, vp, vp, vp, vp, vp]),
    ("xs_engine_put_batch", ctypes.c_int, [vp, ctypes.c_char_p, u64, vp, vp, vp, vp, vp, vp]),
    ("xs_put_body_bytes", u64, [u64, vp]),
    ("xs_engine_set_coalesce", None, [vp, ctypes.c_int]),
    ("xs_engine_stats", None, [vp, vp]),
    ("xs_engine_set_host_md5", None, [vp, ctypes.c_int]),
    ("xs_engine_md5_stats", None, [vp, vp]),
    ("xs_pool_create", vp, [vp, ctypes.c_int, ctypes.c_uint32, ctypes.c_int]),
    ("xs_pool_destroy", None, [vp]),
    ("xs_pool_size", ctypes.c_int, [vp]),
    ("xs_pool_engine", vp, [vp, ctypes.c_int]),
    ("xs_pool_next", vp, [vp]),
    ("xs_pool_seal_md5", ctypes.c_int, [vp, ctypes.c_char_p, u64, vp, vp, vp, vp, vp]),
    ("xs_pool_put_batch", ctypes.c_int, [vp, ctypes.c_char_p, u64, vp, vp, vp, vp, vp, vp]),
    ("xs_host_alloc", vp, [ctypes.c_size_t]),
    ("xs_host_alloc_node", vp, [ctypes.c_size_t, ctypes.c_int]),
    ("xs_device_numa_node", ctypes.c_int, [ctypes.c_int]),
    ("xs_engine_numa_node", ctypes.c_int, [vp]),
    ("xs_engine_device", ctypes.c_int, [vp]),
    ("xs_pci_numa_node", ctypes.c_int, [ctypes.c_char_p]),
    ("xs_numa_node_cpus", ctypes.c_int, [ctypes.c_int, vp, ctypes.c_int]),
    ("xs_parse_device_list", ctypes.c_int, [ctypes.c_char_p, vp, ctypes.c_int]),
    ("xs_effective_cpus", ctypes.c_int, []),
    ("xs_host_free", None, [vp]),
    # cipher.go mirror
    ("rc_cipher_new", vp, [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(i32)]),
    ("rc_cipher_key", i32, [vp, ctypes.c_char_p, ctypes.c_char_p]),
    ("rc_cipher_keys", None, [vp, vp, vp, vp]),
    ("rc_cipher_set_keys", None, [vp, ctypes.c_char_p, ctypes.c_char_p, ctypes.c_char_p]),
    ("rc_cipher_set_pass_bad_blocks", None, [vp, i32]),
    ("rc_cipher_set_rand", None, [vp, RcReader]),
    ("rc_cipher_set_batch_blocks", None, [vp, ctypes.c_uint32]),
    ("rc_cipher_set_readahead", None, [vp, ctypes.c_uint32]),
    ("rc_cipher_set_readahead_growth", None, [vp, ctypes.c_uint32]),
    ("rc_cipher_set_pool", None, [vp, vp]),
    ("rc_default_pool", vp, []),
    ("rc_cipher_free", None, [vp]),
    ("rc_encrypted_size", i64, [i64]),
    ("rc_decrypted_size", i64, [i64, ctypes.POINTER(i32)]),
    ("rc_calculate_underlying", None, [i64, i64, ctypes.POINTER(i64)]),
    ("rc_nonce_increment", None, [vp]),
    ("rc_nonce_add", None, [vp, u64]),
    ("rc_encrypt_data", vp, [vp, RcReader, ctypes.c_char_p, ctypes.POINTER(i32)]),
    ("rc_encrypter_read", i64, [vp, vp, i64, ctypes.POINTER(i32)]),
    ("rc_encrypter_nonce", None, [vp, vp]),
    ("rc_encrypter_free", None, [vp]),
    ("rc_encrypter_set_md5", i32, [vp, i32]),
    ("rc_encrypter_md5", i32, [vp, vp]),
    ("rc_decrypt_data", vp, [vp, RcReader, ctypes.POINTER(i32)]),
    ("rc_decrypt_data_seek", vp, [vp, OPEN_FN, vp, i64, i64, ctypes.POINTER(i32)]),
    ("rc_decrypt_data_seek_ex", vp, [vp, OPEN_FN, vp, i64, i64, ctypes.POINTER(i32), ctypes.POINTER(i32)]),
    ("rc_decrypter_read", i64, [vp, vp, i64, ctypes.POINTER(i32)]),
    ("rc_decrypter_range_seek", i64, [vp, i64, i32, i64, ctypes.POINTER(i32)]),
    ("rc_decrypter_close", i32, [vp]),
    ("rc_decrypter_nonce", None, [vp, vp]),
    ("rc_decrypter_wrapped_error", i32, [vp]),
    ("rc_decrypter_free", None, [vp]),
    ("rc_hash_batch_with_nonce", i32, [vp, u64, vp, vp, vp, vp]),
    ("rc_compute_hash_with_nonce", i32, [vp, RcReader, vp, vp]),
    ("rc_error_string", ctypes.c_char_p, [i32]),
    # file names (cipher.go:120-618)
    ("xs_eme_batch_dev", ctypes.c_int, [ctypes.c_int, ctypes.c_char_p, ctypes.c_char_p, vp, u64, vp, vp, u64, vp]),
    ("rc_new_name_encryption_mode", i32, [ctypes.c_char_p, ctypes.POINTER(i32)]),
    ("rc_new_name_encoding", i32, [ctypes.c_char_p, ctypes.POINTER(i32)]),
    ("rc_cipher_set_name_encryption", None, [vp, i32, i32, i32]),
    ("rc_cipher_set_encrypted_suffix", None, [vp, ctypes.c_char_p]),
    ("rc_name_encode", i64, [i32, ctypes.c_char_p, u64, vp, u64]),
    ("rc_name_decode", i32, [i32, ctypes.c_char_p, u64, vp, u64, ctypes.POINTER(u64), ctypes.POINTER(i64)]),
    ("rc_names_run", i32, [vp, i32, u64, vp, vp, ctypes.POINTER(vp)]),
    ("rc_names_get", None, [vp, u64, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(u64), ctypes.POINTER(i32),
                            ctypes.POINTER(i64)]),
    ("rc_names_kernel_ms", ctypes.c_double, [vp]),
    ("rc_names_free", None, [vp]),
]

SYMBOLS = [s[0] for s in _SIGS]


class StaleLibraryError(RuntimeError):
    """The library on disk was not built from this tree's sources (build id mismatch)."""


def lib():
    """Load the native library built from this tree's sources.  A library whose embedded build id
    differs from the tree's (rclone_amd/build.py build_sources_sha256), or that another installed
    hipcc built (build.stale_reason), is rebuilt, or refused with StaleLibraryError when
    RCLONE_AMD_REBUILD=0 or no hipcc is present; a library missing
    any declared entry point is refused too.  Never a fallback."""
    global _lib
    if _lib is None:
        path = _build.LIB
        want = _build.build_sources_sha256()
        why = _build.stale_reason(path)
        if why is not None:
            if os.environ.get("RCLONE_AMD_REBUILD", "1") == "0" or not _build.hipcc_available():
                raise StaleLibraryError(f"{path}: {why} (rebuild: python -m rclone_amd.build)")
            _build.build()  # under the build lock: concurrent callers build once
        if not os.path.exists(path):
            raise RuntimeError(f"rclone_amd native library missing: {path}")
        L = ctypes.CDLL(path)
        missing = [name for name, _, _ in _SIGS if not hasattr(L, name)]
        if missing:
            raise StaleLibraryError(f"{path} lacks entry points {missing}")
        for name, res, args in _SIGS:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        got = L.xs_build_id().decode()
        if got != want:
            raise StaleLibraryError(f"{path}: loaded library reports build {got}, this tree is {want}")
        _lib = L
    return _lib


_hooks = None


def hooks_lib():
    """TEST ONLY: the failure-injection twin of the library (build.HOOKS_LIB, xs_api.cpp under
    -DXS_TEST_HOOKS), with the same entry points plus xs_test_fail_batch / xs_test_failed_requests.
    Load it in a process of its own (tests/test_engine_failure_gpu.py), never beside lib()."""
    global _hooks
    if _hooks is None:
        lib()  # builds both when stale
        why = _build.stale_reason(_build.HOOKS_LIB)
        if why is not None:
            raise StaleLibraryError(f"{_build.HOOKS_LIB}: {why}")
        L = ctypes.CDLL(_build.HOOKS_LIB)
        for name, res, args in _SIGS + [("xs_test_fail_batch", None, [ctypes.c_int]),
                                        ("xs_test_failed_requests", ctypes.c_int, [])]:
            f = getattr(L, name)
            f.restype = res
            f.argtypes = args
        _hooks = L
    return _hooks


def build_id():
    return lib().xs_build_id().decode()


def last_error():
    return lib().xs_last_error().decode(errors="replace")


def check(rc, what="xs call"):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc}): {last_error()}")
