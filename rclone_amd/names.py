"""File-name half of rclone's crypt cipher (backend/crypt/cipher.go:86-618) over the rc_* C ABI.

Strings are Go strings, i.e. byte strings: ``str`` arguments are UTF-8 encoded with
``surrogateescape`` (so invalid UTF-8 round-trips) and results decoded the same way; ``bytes``
are accepted as well.  The EME-AES-256 segment cipher runs on the GPU (xs_eme.hip), one
kernel launch per batch; there is no CPU fallback.

    Go (cipher.go)                                 here
    NameEncryptionOff / Standard / Obfuscated      NAME_ENCRYPTION_OFF / _STANDARD / _OBFUSCATED
    NewNameEncryptionMode / mode.String()          new_name_encryption_mode / name_encryption_mode_string
    NewNameEncoding -> fileNameEncoding            new_name_encoding -> NameEncoding
    c.encryptSegment / decryptSegment              Cipher.encrypt_segment / decrypt_segment
    c.obfuscateSegment / deobfuscateSegment        Cipher.obfuscate_segment / deobfuscate_segment
    EncryptFileName / DecryptFileName              Cipher.encrypt_file_name / decrypt_file_name
    EncryptDirName / DecryptDirName                Cipher.encrypt_dir_name / decrypt_dir_name
    (batched listing)                              Cipher.encrypt_file_names / decrypt_file_names ...
    c.setEncryptedSuffix                           Cipher.set_encrypted_suffix
"""
import ctypes

from . import _lib

NAME_ENCRYPTION_OFF, NAME_ENCRYPTION_STANDARD, NAME_ENCRYPTION_OBFUSCATED = 0, 1, 2
ENC_BASE32, ENC_BASE64, ENC_BASE32768 = 0, 1, 2
_ENC_NAMES = {ENC_BASE32: "base32", ENC_BASE64: "base64", ENC_BASE32768: "base32768"}

OP_ENCRYPT_FILE_NAME, OP_DECRYPT_FILE_NAME, OP_ENCRYPT_DIR_NAME, OP_DECRYPT_DIR_NAME = 0, 1, 2, 3
OP_ENCRYPT_SEGMENT, OP_DECRYPT_SEGMENT, OP_OBFUSCATE_SEGMENT, OP_DEOBFUSCATE_SEGMENT = 4, 5, 6, 7


class NameError_(Exception):
    """Base of the file-name errors."""

    message = ""

    def __init__(self, *a):
        super().__init__(*(a or (self.message,)))

    def __eq__(self, other):
        return type(self) is type(other) and self.args == other.args

    def __hash__(self):
        return hash((type(self), self.args))


def _sentinel(name, msg):
    return type(name, (NameError_,), {"message": msg})


# cipher.go:44-58
ErrorNotAMultipleOfBlocksize = _sentinel("ErrorNotAMultipleOfBlocksize", "not a multiple of blocksize")
ErrorTooShortAfterDecode = _sentinel("ErrorTooShortAfterDecode", "too short after base32 decode")
ErrorTooLongAfterDecode = _sentinel("ErrorTooLongAfterDecode", "too long after base32 decode")
ErrorBadBase32Encoding = _sentinel("ErrorBadBase32Encoding", "bad base32 filename encoding")
ErrorNotAnEncryptedFile = _sentinel("ErrorNotAnEncryptedFile", "not an encrypted file - does not match suffix")
# backend/crypt/pkcs7/pkcs7.go:9-15
ErrorPaddingNotFound = _sentinel("ErrorPaddingNotFound", "bad PKCS#7 padding - not padded")
ErrorPaddingNotAMultiple = _sentinel("ErrorPaddingNotAMultiple", "bad PKCS#7 padding - not a multiple of blocksize")
ErrorPaddingTooLong = _sentinel("ErrorPaddingTooLong", "bad PKCS#7 padding - too long")
ErrorPaddingTooShort = _sentinel("ErrorPaddingTooShort", "bad PKCS#7 padding - too short")
ErrorPaddingNotAllTheSame = _sentinel("ErrorPaddingNotAllTheSame", "bad PKCS#7 padding - not all the same")
ErrorNameTooLong = _sentinel("ErrorNameTooLong", "EME operates on 1 to 128 block-cipher blocks")


class _CorruptInputError(NameError_):
    codec = ""

    def __init__(self, offset):
        super().__init__(int(offset))
        self.offset = int(offset)

    def __str__(self):
        return f"illegal {self.codec} data at input byte {self.offset}"


class Base32CorruptInputError(_CorruptInputError):
    """encoding/base32.CorruptInputError"""
    codec = "base32"


class Base64CorruptInputError(_CorruptInputError):
    """encoding/base64.CorruptInputError"""
    codec = "base64"


class Base32768CorruptInputError(_CorruptInputError):
    """base32768.CorruptInputError"""
    codec = "base32768"


_CODES = {
    -130: ErrorNotAMultipleOfBlocksize, -131: ErrorTooShortAfterDecode, -132: ErrorTooLongAfterDecode,
    -133: ErrorBadBase32Encoding, -134: ErrorNotAnEncryptedFile, -140: ErrorPaddingNotFound,
    -141: ErrorPaddingNotAMultiple, -142: ErrorPaddingTooLong, -143: ErrorPaddingTooShort,
    -144: ErrorPaddingNotAllTheSame, -155: ErrorNameTooLong,
}
_CORRUPT = {-150: Base32CorruptInputError, -151: Base64CorruptInputError, -152: Base32768CorruptInputError}


def _exc(code, arg):
    if code in _CORRUPT:
        return _CORRUPT[code](arg)
    if code in _CODES:
        return _CODES[code]()
    return RuntimeError(f"name cipher error {code}: {_lib.lib().rc_error_string(code).decode()}")


def _b(s):
    return s if isinstance(s, (bytes, bytearray)) else s.encode("utf-8", "surrogateescape")


def _s(b):
    return b.decode("utf-8", "surrogateescape")


# ------------------------------------------------------------------ modes and encodings
def new_name_encryption_mode(s: str) -> int:
    """NewNameEncryptionMode (cipher.go:92)."""
    m = ctypes.c_int32(0)
    if _lib.lib().rc_new_name_encryption_mode(_b(s), ctypes.byref(m)) != 0:
        raise ValueError(f"unknown file name encryption mode {s.lower()!r}".replace("'", '"'))
    return m.value


def name_encryption_mode_string(mode: int) -> str:
    """NameEncryptionMode.String (cipher.go:107)."""
    return {0: "off", 1: "standard", 2: "obfuscate"}.get(mode, f"Unknown mode #{mode}")


class NameEncoding:
    """fileNameEncoding (cipher.go:121): EncodeToString / DecodeString."""

    def __init__(self, enc: int):
        self.enc = enc

    def __repr__(self):
        return f"NameEncoding({_ENC_NAMES.get(self.enc)})"

    def encode_to_string(self, src: bytes) -> str:
        src = bytes(src)
        n = _lib.lib().rc_name_encode(self.enc, src, len(src), None, 0)
        buf = ctypes.create_string_buffer(max(n, 1))
        _lib.lib().rc_name_encode(self.enc, src, len(src), buf, n)
        return _s(buf.raw[:n])

    def decode_string(self, s) -> bytes:
        b = _b(s)
        cap = len(b) + 8
        buf = ctypes.create_string_buffer(cap)
        n, arg = ctypes.c_uint64(0), ctypes.c_int64(0)
        code = _lib.lib().rc_name_decode(self.enc, b, len(b), buf, cap, ctypes.byref(n), ctypes.byref(arg))
        if code != 0:
            raise _exc(code, arg.value)
        return buf.raw[:n.value]


def new_name_encoding(s: str) -> NameEncoding:
    """NewNameEncoding (cipher.go:155)."""
    e = ctypes.c_int32(0)
    if _lib.lib().rc_new_name_encoding(_b(s), ctypes.byref(e)) != 0:
        raise ValueError(f"unknown file name encoding mode {s.lower()!r}".replace("'", '"'))
    return NameEncoding(e.value)


# ------------------------------------------------------------------ batched runner
class NamesResult:
    """Per-name results of one batched call: values (str) or exceptions, plus the EME kernel time."""

    def __init__(self, values, kernel_ms):
        self.values = values
        self.kernel_ms = kernel_ms


def run(handle, op: int, names, as_bytes=False) -> NamesResult:
    """Apply one cipher.go name function to every name with one GPU EME launch (rc_names_run)."""
    L = _lib.lib()
    bs = [_b(x) for x in names]
    n = len(bs)
    arr = (ctypes.c_char_p * max(n, 1))(*bs)
    lens = (ctypes.c_uint64 * max(n, 1))(*[len(x) for x in bs])
    out = ctypes.c_void_p()
    rc = L.rc_names_run(handle, op, n, arr, lens, ctypes.byref(out))
    if rc != 0:
        raise RuntimeError(f"rc_names_run failed ({rc}): {_lib.last_error()}")
    try:
        vals = []
        p, ln, err, arg = ctypes.c_void_p(), ctypes.c_uint64(), ctypes.c_int32(), ctypes.c_int64()
        for i in range(n):
            L.rc_names_get(out, i, ctypes.byref(p), ctypes.byref(ln), ctypes.byref(err), ctypes.byref(arg))
            if err.value != 0:
                vals.append(_exc(err.value, arg.value))
            else:
                raw = ctypes.string_at(p.value, ln.value) if ln.value else b""
                vals.append(raw if as_bytes else _s(raw))
        return NamesResult(vals, L.rc_names_kernel_ms(out))
    finally:
        L.rc_names_free(out)


def one(handle, op, name):
    v = run(handle, op, [name]).values[0]
    if isinstance(v, BaseException):
        raise v
    return v


class NameCipherMixin:
    """Name methods of crypt.Cipher (cipher.go:264-618); self._h is the rc_cipher handle."""

    def set_name_encryption(self, mode: int = NAME_ENCRYPTION_STANDARD, dir_name_encrypt: bool = True, enc=None):
        """newCipher's mode / dirNameEncrypt / enc arguments (cipher.go:187)."""
        if enc is None:
            enc = NameEncoding(ENC_BASE32)
        self._name_mode, self._dir_name_encrypt, self._name_enc = mode, bool(dir_name_encrypt), enc
        _lib.lib().rc_cipher_set_name_encryption(self._h, mode, int(bool(dir_name_encrypt)), enc.enc)

    def name_encryption_mode(self) -> int:
        return self._name_mode

    def set_encrypted_suffix(self, suffix: str):
        """setEncryptedSuffix (cipher.go:207)."""
        _lib.lib().rc_cipher_set_encrypted_suffix(self._h, _b(suffix))

    def encrypt_segment(self, s):
        return one(self._h, OP_ENCRYPT_SEGMENT, s)

    def decrypt_segment(self, s):
        return one(self._h, OP_DECRYPT_SEGMENT, s)

    def obfuscate_segment(self, s):
        return one(self._h, OP_OBFUSCATE_SEGMENT, s)

    def deobfuscate_segment(self, s):
        return one(self._h, OP_DEOBFUSCATE_SEGMENT, s)

    def encrypt_file_name(self, s):
        return one(self._h, OP_ENCRYPT_FILE_NAME, s)

    def decrypt_file_name(self, s):
        return one(self._h, OP_DECRYPT_FILE_NAME, s)

    def encrypt_dir_name(self, s):
        return one(self._h, OP_ENCRYPT_DIR_NAME, s)

    def decrypt_dir_name(self, s):
        return one(self._h, OP_DECRYPT_DIR_NAME, s)

    # batched (a listing's worth of names per GPU launch)
    def encrypt_file_names(self, names):
        return run(self._h, OP_ENCRYPT_FILE_NAME, names).values

    def decrypt_file_names(self, names):
        return run(self._h, OP_DECRYPT_FILE_NAME, names).values

    def encrypt_dir_names(self, names):
        return run(self._h, OP_ENCRYPT_DIR_NAME, names).values

    def decrypt_dir_names(self, names):
        return run(self._h, OP_DECRYPT_DIR_NAME, names).values

    def names_run(self, op, names, as_bytes=False) -> NamesResult:
        return run(self._h, op, names, as_bytes)
