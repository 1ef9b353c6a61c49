"""TEST INFRASTRUCTURE ONLY -- ctypes front-end for oracle/build/liboracle.so.

The checker for the HIP path (never the thing measured as the product, never shipped).
Built from oracle/xsalsa_oracle.c and oracle/eme_oracle.c by oracle/Makefile (see that file's header for the
reference file:line each function restates).
"""
import ctypes
import os
import subprocess

HERE = os.path.dirname(os.path.abspath(__file__))
LIBPATH = os.path.join(HERE, "build", "liboracle.so")

BLOCK_DATA = 65536
BLOCK_SIZE = 65552
FILE_HDR = 32


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def _load():
    if not os.path.exists(LIBPATH):
        build()
    lib = ctypes.CDLL(LIBPATH)
    c_p = ctypes.c_char_p
    vp = ctypes.c_void_p
    lib.orc_secretbox_seal.argtypes = [vp, vp, ctypes.c_size_t, c_p, c_p]
    lib.orc_secretbox_open.argtypes = [vp, vp, ctypes.c_size_t, c_p, c_p]
    lib.orc_secretbox_open.restype = ctypes.c_int
    lib.orc_hsalsa20.argtypes = [vp, c_p, c_p]
    lib.orc_salsa20_block.argtypes = [vp, c_p, c_p, ctypes.c_uint64]
    lib.orc_poly1305.argtypes = [vp, vp, ctypes.c_size_t, c_p]
    lib.orc_nonce_increment.argtypes = [vp]
    lib.orc_nonce_add.argtypes = [vp, ctypes.c_uint64]
    lib.orc_encrypted_size.argtypes = [ctypes.c_int64]
    lib.orc_encrypted_size.restype = ctypes.c_int64
    lib.orc_decrypted_size.argtypes = [ctypes.c_int64]
    lib.orc_decrypted_size.restype = ctypes.c_int64
    lib.orc_calculate_underlying.argtypes = [ctypes.c_int64, ctypes.c_int64, vp]
    lib.orc_encrypt_file.argtypes = [vp, vp, ctypes.c_int64, c_p, c_p]
    lib.orc_decrypt_file.argtypes = [vp, vp, ctypes.c_int64, c_p, ctypes.c_int, vp]
    lib.orc_decrypt_file.restype = ctypes.c_int64
    lib.orc_seal_blocks.argtypes = [vp, vp, ctypes.c_int64, c_p, c_p]
    lib.orc_seal_blocks.restype = ctypes.c_int
    lib.orc_open_blocks.argtypes = [vp, vp, vp, ctypes.c_int64, c_p, c_p]
    lib.orc_open_blocks.restype = ctypes.c_int
    # vectorised CPU baseline (oracle/xsalsa_simd.c): same secretbox, AVX-512 / AVX2 Salsa20
    lib.orc_simd_level.restype = ctypes.c_int
    lib.orc_simd_force.argtypes = [ctypes.c_int]
    lib.orc_simd_secretbox_seal.argtypes = [vp, vp, ctypes.c_size_t, c_p, c_p]
    lib.orc_simd_secretbox_open.argtypes = [vp, vp, ctypes.c_size_t, c_p, c_p]
    lib.orc_simd_secretbox_open.restype = ctypes.c_int
    lib.orc_simd_seal_blocks.argtypes = [vp, vp, ctypes.c_int64, c_p, c_p]
    lib.orc_simd_seal_blocks.restype = ctypes.c_int
    lib.orc_simd_open_blocks.argtypes = [vp, vp, vp, ctypes.c_int64, c_p, c_p]
    lib.orc_simd_open_blocks.restype = ctypes.c_int
    lib.orc_simd_open_window.argtypes = [vp, vp, ctypes.c_size_t, c_p, c_p, ctypes.c_size_t, ctypes.c_size_t]
    lib.orc_simd_open_window.restype = ctypes.c_int
    lib.orc_simd_encrypt_gen_file.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64, c_p, c_p]
    lib.orc_simd_encrypt_gen_file.restype = ctypes.c_int
    lib.orc_gen_block.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint64]
    lib.orc_simd_seal_gen.argtypes = [vp, ctypes.c_int64, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64, c_p, vp,
                                      c_p, vp]
    lib.orc_simd_seal_gen.restype = ctypes.c_int
    lib.orc_seal_desc.argtypes = [vp, vp, vp, ctypes.c_int64, c_p]
    lib.orc_seal_desc.restype = ctypes.c_int
    lib.orc_open_desc.argtypes = [vp, vp, vp, vp, ctypes.c_int64, c_p]
    lib.orc_open_desc.restype = ctypes.c_int
    # eme_oracle.c (file names)
    lib.orc_aes256_expand.argtypes = [c_p, vp]
    lib.orc_aes256_encrypt.argtypes = [vp, c_p, vp]
    lib.orc_aes256_decrypt.argtypes = [vp, c_p, vp]
    lib.orc_eme_transform.argtypes = [c_p, c_p, c_p, vp, ctypes.c_int, ctypes.c_int]
    lib.orc_eme_transform.restype = ctypes.c_int
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _buf(b):
    return ctypes.create_string_buffer(bytes(b), len(b)) if len(b) else ctypes.create_string_buffer(1)


def seal(msg: bytes, nonce: bytes, key: bytes) -> bytes:
    out = ctypes.create_string_buffer(len(msg) + 16)
    lib().orc_secretbox_seal(out, _buf(msg), len(msg), nonce, key)
    return out.raw


def open_box(box: bytes, nonce: bytes, key: bytes):
    out = ctypes.create_string_buffer(max(len(box) - 16, 1))
    rc = lib().orc_secretbox_open(out, _buf(box), len(box), nonce, key)
    return out.raw[: len(box) - 16] if rc == 0 else None


def nonce_increment(n: bytes) -> bytes:
    b = ctypes.create_string_buffer(bytes(n), 24)
    lib().orc_nonce_increment(b)
    return b.raw


def nonce_add(n: bytes, x: int) -> bytes:
    b = ctypes.create_string_buffer(bytes(n), 24)
    lib().orc_nonce_add(b, x)
    return b.raw


def encrypted_size(n: int) -> int:
    return lib().orc_encrypted_size(n)


def decrypted_size(n: int) -> int:
    return lib().orc_decrypted_size(n)


def calculate_underlying(offset: int, limit: int):
    out = (ctypes.c_int64 * 4)()
    lib().orc_calculate_underlying(offset, limit, out)
    return tuple(out)


def encrypt_file(plain: bytes, nonce0: bytes, key: bytes) -> bytes:
    out = ctypes.create_string_buffer(encrypted_size(len(plain)))
    lib().orc_encrypt_file(out, _buf(plain), len(plain), nonce0, key)
    return out.raw


def decrypt_file(ct: bytes, key: bytes, pass_bad_blocks=False):
    """Returns (plaintext or None, code) with code 0 ok, -1 too short, -2 bad magic,
    -3 truncated block header, -4 bad block (first bad block index in the tuple)."""
    out = ctypes.create_string_buffer(max(len(ct), 1))
    bad = ctypes.c_int64(-1)
    rc = lib().orc_decrypt_file(out, _buf(ct), len(ct), key, int(pass_bad_blocks), ctypes.byref(bad))
    if rc < 0:
        return None, rc, bad.value
    return out.raw[:rc], 0, -1


def seal_desc(dst, src, desc, key: bytes) -> int:
    """Seal every descriptor (numpy structured array, xs_block_desc layout) from the numpy
    u8 array src into dst (both host arrays).  Returns the OpenMP thread count."""
    assert desc.dtype.itemsize == 48
    return lib().orc_seal_desc(dst.ctypes.data, src.ctypes.data, desc.ctypes.data, len(desc), bytes(key))


def open_desc(dst, ok, src, desc, key: bytes) -> int:
    assert desc.dtype.itemsize == 48
    return lib().orc_open_desc(dst.ctypes.data, ok.ctypes.data, src.ctypes.data, desc.ctypes.data, len(desc),
                               bytes(key))


# ------------------------------------------------------------------ file names (eme_oracle.c)
def aes256_encrypt(key: bytes, block: bytes) -> bytes:
    rk = ctypes.create_string_buffer(240)
    lib().orc_aes256_expand(bytes(key), rk)
    out = ctypes.create_string_buffer(16)
    lib().orc_aes256_encrypt(rk, bytes(block), out)
    return out.raw


def aes256_decrypt(key: bytes, block: bytes) -> bytes:
    rk = ctypes.create_string_buffer(240)
    lib().orc_aes256_expand(bytes(key), rk)
    out = ctypes.create_string_buffer(16)
    lib().orc_aes256_decrypt(rk, bytes(block), out)
    return out.raw


def eme_transform(key: bytes, tweak: bytes, data: bytes, encrypt: bool) -> bytes:
    """eme.Transform(aes(key), tweak, data, direction) (rfjakob/eme v1.2.0)."""
    data = bytes(data)
    assert len(data) % 16 == 0
    out = ctypes.create_string_buffer(max(len(data), 1))
    rc = lib().orc_eme_transform(bytes(key), bytes(tweak), data, out, len(data) // 16, 0 if encrypt else 1)
    if rc != 0:
        raise ValueError("EME operates on 1 to 128 block-cipher blocks")
    return out.raw[:len(data)]


def pkcs7_pad(b: bytes) -> bytes:
    p = 16 - len(b) % 16
    return bytes(b) + bytes([p]) * p


def pkcs7_unpad(b: bytes):
    """Returns the unpadded bytes or the pkcs7.go error name."""
    if not b:
        return "ErrorPaddingNotFound"
    if len(b) % 16:
        return "ErrorPaddingNotAMultiple"
    p = b[-1]
    if p > 16:
        return "ErrorPaddingTooLong"
    if p == 0:
        return "ErrorPaddingTooShort"
    if any(x != p for x in b[-p:]):
        return "ErrorPaddingNotAllTheSame"
    return b[:-p]


# ------------------------------------------------------------------ generated object sets (xsalsa_simd.c)
def gen_block(seed: int, g: int) -> bytes:
    """Global 64 KiB block g of the SplitMix64 stream (what xs_fill_blocks_dev writes)."""
    out = ctypes.create_string_buffer(BLOCK_DATA)
    lib().orc_gen_block(out, seed, g)
    return out.raw


def seal_gen(nblocks: int, first: int, stride: int, seed: int, nonce0: bytes, key: bytes, out=None, nonces=None):
    """Seal generated blocks g = first + j*stride (j < nblocks), block g with nonce0 + g, or with
    nonces[j] (a C-contiguous u8 array of nblocks x 24) when given.
    out: None (digest only) or a writable u8 numpy array of nblocks*65552 bytes for the wire blocks.
    Returns ((tag sum lo, tag sum hi) mod 2^64, OpenMP threads)."""
    if out is not None:
        assert out.nbytes >= nblocks * BLOCK_SIZE
    if nonces is not None:
        assert nonces.dtype.itemsize == 1 and nonces.size == nblocks * 24 and nonces.flags.c_contiguous
    s = (ctypes.c_uint64 * 2)()
    threads = lib().orc_simd_seal_gen(None if out is None else out.ctypes.data, nblocks, first, stride, seed,
                                      bytes(nonce0), None if nonces is None else nonces.ctypes.data, bytes(key), s)
    if threads == 0:
        raise RuntimeError("orc_simd_seal_gen needs AVX2")
    return (int(s[0]), int(s[1])), threads


def encrypt_gen_file_into(buf, seed: int, size: int, nonce: bytes, key: bytes) -> int:
    """The crypt file of the SplitMix64(seed) object of `size` bytes into buf (a writable numpy u8
    array of at least encrypted_size(size) bytes); returns that size.  Releases the GIL (ctypes)."""
    n = encrypted_size(size)
    assert buf.nbytes >= n
    if lib().orc_simd_encrypt_gen_file(buf.ctypes.data, seed, size, bytes(nonce), bytes(key)) != 0:
        raise RuntimeError("orc_simd_encrypt_gen_file needs AVX2")
    return n
