"""Python front-end of rclone's backend/crypt data cipher, running on the MI355X.

Mirrors backend/crypt/cipher.go (rclone v1.76.0) -- names, argument meaning and error
behaviour -- over the rc_* C ABI of librclone_crypt.so (include/rclone_crypt_gpu.h), whose
encrypter/decrypter seal and open 64 KiB blocks with the HIP kernels.  There is no CPU
fallback: without the native library or a HIP device, encryption raises.

    Go (cipher.go)                         here
    newCipher(mode, password, salt, ...)   Cipher(password, salt)
    (*Cipher).Key                          Cipher.key
    c.cryptoRand                           Cipher.crypto_rand  (any reader; None = OS random)
    c.passBadBlocks / setPassBadBlocks     Cipher.pass_bad_blocks
    EncryptData / newEncrypter(in, nonce)  Cipher.encrypt_data(reader, nonce=None)
    DecryptData / newDecrypter             Cipher.decrypt_data(reader)
    DecryptDataSeek(ctx, open, off, lim)   Cipher.decrypt_data_seek(open, offset, limit)
    EncryptedSize / DecryptedSize          Cipher.encrypted_size / decrypted_size
    calculateUnderlying                    calculate_underlying
    nonce.increment / nonce.add            nonce_increment / nonce_add
    ErrorEncrypted* sentinels              exception classes of the same names

Readers follow Python's protocol: ``read(n)`` returns bytes, ``b""`` at EOF, and raises to
report an error.  A reader may instead implement ``read_go(n) -> (bytes, err)`` to return
data and an error from one call exactly like a Go io.Reader (``err`` None, ``EOF`` or an
exception).  Exceptions raised by readers/openers are passed through unchanged wherever the
reference passes the underlying error through.
"""
import ctypes
import threading

from . import _lib
from .names import NAME_ENCRYPTION_STANDARD, NameCipherMixin

BLOCK_DATA_SIZE = 65536  # blockDataSize cipher.go:39
BLOCK_HEADER_SIZE = 16   # blockHeaderSize cipher.go:38
BLOCK_SIZE = 65552       # blockSize cipher.go:40
FILE_HEADER_SIZE = 32    # fileHeaderSize cipher.go:37
FILE_MAGIC = b"RCLONE\x00\x00"

RC_NIL, RC_EOF, RC_UNEXPECTED_EOF, RC_USER_BASE = 0, 1, 2, 16


class _EOF:
    """io.EOF marker for read_go() readers."""

    def __repr__(self):
        return "EOF"


EOF = _EOF()


class CryptError(Exception):
    """Base class of the crypt sentinel errors (cipher.go:44-58)."""


def _sentinel(name, msg):
    cls = type(name, (CryptError,), {})
    cls.message = msg
    return cls


ErrorEncryptedFileTooShort = _sentinel("ErrorEncryptedFileTooShort", "file is too short to be encrypted")
ErrorEncryptedFileBadHeader = _sentinel("ErrorEncryptedFileBadHeader", "file has truncated block header")
ErrorEncryptedBadMagic = _sentinel("ErrorEncryptedBadMagic", "not an encrypted file - bad magic string")
ErrorEncryptedBadBlock = _sentinel("ErrorEncryptedBadBlock", "failed to authenticate decrypted block - bad password?")
ErrorFileClosed = _sentinel("ErrorFileClosed", "file already closed")
ErrorBadSeek = _sentinel("ErrorBadSeek", "Seek beyond end of file")
ErrUnexpectedEOF = _sentinel("ErrUnexpectedEOF", "unexpected EOF")
GPUError = _sentinel("GPUError", "GPU crypt engine failure")
# io.EOF where the reference returns it as a call's only error (RangeSeek at the end of a
# whole-block file, DecryptDataSeek opened there: cipher.go:1019-1022, :848-853), not a Read's
ErrEOF = _sentinel("ErrEOF", "EOF")

_CODE_TO_CLASS = {
    -101: ErrorEncryptedFileTooShort,
    -102: ErrorEncryptedFileBadHeader,
    -103: ErrorEncryptedBadMagic,
    -104: ErrorEncryptedBadBlock,
    -105: ErrorFileClosed,
    -106: ErrorBadSeek,
    -120: GPUError,
    RC_EOF: ErrEOF,
    RC_UNEXPECTED_EOF: ErrUnexpectedEOF,
}


class _ErrTable:
    """Maps Python exceptions raised in callbacks to pass-through int codes and back."""

    def __init__(self):
        self._lock = threading.Lock()
        self._by_code = {}
        self._next = RC_USER_BASE

    def code(self, exc):
        if isinstance(exc, ErrUnexpectedEOF):
            return RC_UNEXPECTED_EOF
        with self._lock:
            c = self._next
            self._next += 1
            if self._next > 2**30:
                self._next = RC_USER_BASE
            self._by_code[c] = exc
            return c

    def exc(self, code, wrapped=None):
        if code >= RC_USER_BASE:
            with self._lock:
                return self._by_code.get(code, CryptError(f"reader error {code}"))
        if code == -107:
            return CryptError("short read of nonce: " + _msg(wrapped if wrapped is not None else RC_EOF))
        if code == -108:
            return CryptError("can't seek - not initialised with newDecrypterSeek")
        if code == -109:
            return CryptError("can only seek from the start")
        if code == -110:  # fmt.Errorf("couldn't reopen file with offset and limit: %w", err)
            inner = self.exc(wrapped) if wrapped not in (None, RC_NIL) else CryptError("?")
            e = CryptError(f"couldn't reopen file with offset and limit: {inner}")
            e.__cause__ = inner
            return e
        cls = _CODE_TO_CLASS.get(code)
        if cls is not None:
            return cls(cls.message)
        return CryptError(_lib.lib().rc_error_string(code).decode())


_ERRS = _ErrTable()


def _msg(code):
    return "EOF" if code == RC_EOF else str(_ERRS.exc(code))


def _raise(code, wrapped=None):
    if code in (RC_NIL, RC_EOF):
        return
    raise _ERRS.exc(code, wrapped)


def new_cipher(mode, password, salt, dir_name_encrypt, enc):
    """newCipher (cipher.go:187) with the reference's argument order."""
    return Cipher(password, salt, mode=mode, dir_name_encrypt=dir_name_encrypt, enc=enc)


# ------------------------------------------------------------------ reader adaptation
class _ReaderBridge:
    """Wraps a Python reader as an rc_reader (io.Reader [+ io.Closer] [+ fs.RangeSeeker])."""

    def __init__(self, reader, closer=True):
        self.reader = reader

        def _read(user, p, n, errp):
            try:
                if hasattr(reader, "read_go"):
                    data, err = reader.read_go(n)
                    data = bytes(data or b"")[:n]
                    if err is None:
                        errp[0] = RC_NIL
                    elif err is EOF:
                        errp[0] = RC_EOF
                    else:
                        errp[0] = _ERRS.code(err)
                else:
                    data = reader.read(n)
                    data = bytes(data or b"")[:n]
                    errp[0] = RC_NIL if data else RC_EOF
                if data:
                    ctypes.memmove(p, data, len(data))
                return len(data)
            except Exception as e:  # the reader's error, passed through
                errp[0] = _ERRS.code(e)
                return 0

        def _close(user):
            try:
                c = getattr(reader, "close", None)
                if c is not None:
                    c()
                return RC_NIL
            except Exception as e:
                return _ERRS.code(e)

        def _range_seek(user, offset, whence, limit):
            try:
                reader.range_seek(offset, whence, limit)
                return RC_NIL
            except Exception as e:
                return _ERRS.code(e)

        self._read = _lib.READ_FN(_read)
        self._close = _lib.CLOSE_FN(_close) if closer else _lib.CLOSE_FN()
        self._rs = _lib.RANGE_SEEK_FN(_range_seek) if hasattr(reader, "range_seek") else _lib.RANGE_SEEK_FN()
        self.c = _lib.RcReader(self._read, self._close, self._rs, None)


def calculate_underlying(offset, limit):
    """calculateUnderlying (cipher.go:935): (underlyingOffset, underlyingLimit, discard, blocks)."""
    out = (ctypes.c_int64 * 4)()
    _lib.lib().rc_calculate_underlying(offset, limit, out)
    return tuple(out)


def nonce_increment(nonce: bytes) -> bytes:
    b = ctypes.create_string_buffer(bytes(nonce), 24)
    _lib.lib().rc_nonce_increment(b)
    return b.raw


def nonce_add(nonce: bytes, x: int) -> bytes:
    b = ctypes.create_string_buffer(bytes(nonce), 24)
    _lib.lib().rc_nonce_add(b, x)
    return b.raw


def encrypted_size(size: int) -> int:
    return _lib.lib().rc_encrypted_size(size)


def decrypted_size(size: int) -> int:
    e = ctypes.c_int32(0)
    v = _lib.lib().rc_decrypted_size(size, ctypes.byref(e))
    _raise(e.value)
    return v


class Cipher(NameCipherMixin):
    """The crypt cipher (cipher.go:172 Cipher, :187 newCipher, :231 Key): data path here, the
    file-name methods from names.NameCipherMixin."""

    def __init__(self, password: str = "", salt: str = "", pass_bad_blocks: bool = False, batch_blocks: int = 64,
                 mode: int = NAME_ENCRYPTION_STANDARD, dir_name_encrypt: bool = True, enc=None):
        e = ctypes.c_int32(0)
        self._free = _lib.lib().rc_cipher_free
        self._h = _lib.lib().rc_cipher_new(password.encode(), salt.encode(), ctypes.byref(e))
        _raise(e.value)
        self.set_name_encryption(mode, dir_name_encrypt, enc)
        self._rand = None
        self._rand_bridge = None
        self.pass_bad_blocks = pass_bad_blocks
        self.batch_blocks = batch_blocks

    def __del__(self):
        # at interpreter exit the module globals may already be gone: bound function only
        h, free = getattr(self, "_h", None), getattr(self, "_free", None)
        if h and free is not None:
            free(h)
            self._h = None

    def key(self, password: str, salt: str = ""):
        _raise(_lib.lib().rc_cipher_key(self._h, password.encode(), salt.encode()))

    def _keys(self):
        d, n, t = (ctypes.c_uint8 * 32)(), (ctypes.c_uint8 * 32)(), (ctypes.c_uint8 * 16)()
        _lib.lib().rc_cipher_keys(self._h, d, n, t)
        return bytes(d), bytes(n), bytes(t)

    @property
    def data_key(self):
        return self._keys()[0]

    @property
    def name_key(self):
        return self._keys()[1]

    @property
    def name_tweak(self):
        return self._keys()[2]

    @property
    def pass_bad_blocks(self):
        return self._pbb

    @pass_bad_blocks.setter
    def pass_bad_blocks(self, v):
        self._pbb = bool(v)
        _lib.lib().rc_cipher_set_pass_bad_blocks(self._h, int(bool(v)))

    @property
    def batch_blocks(self):
        return self._batch

    @batch_blocks.setter
    def batch_blocks(self, v):
        self._batch = int(v)
        _lib.lib().rc_cipher_set_batch_blocks(self._h, int(v))

    @property
    def readahead(self):
        """Blocks read by the first refill of a stream / after a seek (rc_cipher_set_readahead;
        1 = the reference's one block, doubling up to batch_blocks after that; 0 = full batches)."""
        return getattr(self, "_ra", 1)

    @readahead.setter
    def readahead(self, v):
        self._ra = int(v)
        _lib.lib().rc_cipher_set_readahead(self._h, int(v))

    @property
    def readahead_growth(self):
        """Refill growth factor (rc_cipher_set_readahead_growth; 0 = adaptive to the source rate)."""
        return getattr(self, "_rag", 0)

    @readahead_growth.setter
    def readahead_growth(self, v):
        self._rag = int(v)
        _lib.lib().rc_cipher_set_readahead_growth(self._h, int(v))

    @property
    def pool(self):
        return getattr(self, "_pool", None)

    @pool.setter
    def pool(self, p):
        """Bind this cipher's handles and batches to an EnginePool (None: the process pool)."""
        self._pool = p
        _lib.lib().rc_cipher_set_pool(self._h, p.handle if p is not None else None)

    @property
    def crypto_rand(self):
        return self._rand

    @crypto_rand.setter
    def crypto_rand(self, reader):
        self._rand = reader
        if reader is None:
            self._rand_bridge = None
            _lib.lib().rc_cipher_set_rand(self._h, _lib.RcReader())
        else:
            self._rand_bridge = _ReaderBridge(reader, closer=False)
            _lib.lib().rc_cipher_set_rand(self._h, self._rand_bridge.c)

    def encrypted_size(self, size):
        return encrypted_size(size)

    def decrypted_size(self, size):
        return decrypted_size(size)

    def encrypt_data(self, reader, nonce: bytes = None):
        """EncryptData (cipher.go:771) / newEncrypter(in, nonce) (:694)."""
        return Encrypter(self, reader, nonce)

    def decrypt_data(self, reader):
        """DecryptData (cipher.go:1099)."""
        return Decrypter(self, reader)

    def decrypt_data_seek(self, open_fn, offset: int, limit: int):
        """DecryptDataSeek (cipher.go:1112); open_fn(offset, limit) -> reader."""
        return Decrypter(self, None, open_fn=open_fn, offset=offset, limit=limit)

    # ---------------------------------------------------------------- hashes (crypt.go:784-852)
    def hash_batch_with_nonce(self, items):
        """Fs.computeHashWithNonce (crypt.go:784) for MD5, batched: items = [(nonce, src)], src a
        Go-style reader (closed after reading, fs.CheckClose).  Sealing and MD5 both run on the
        GPU (rc_hash_batch_with_nonce); returns per item the 16-byte digest, or the exception
        the source raised (the reference wraps it: "failed to hash data: %w")."""
        n = len(items)
        if n == 0:
            return []
        nonces = b"".join(bytes(nc) for nc, _ in items)
        if len(nonces) != 24 * n:
            raise ValueError("nonces must be 24 bytes")
        bridges = [_ReaderBridge(src, closer=True) for _, src in items]
        arr = (_lib.RcReader * n)(*[b.c for b in bridges])
        md5 = ctypes.create_string_buffer(16 * n)
        errs = (ctypes.c_int32 * n)()
        _raise(_lib.lib().rc_hash_batch_with_nonce(self._h, n, arr, nonces, md5, errs))
        out = []
        for i in range(n):
            out.append(md5.raw[16 * i:16 * i + 16] if errs[i] == RC_NIL else _ERRS.exc(errs[i]))
        return out

    def compute_hash_with_nonce(self, nonce: bytes, src) -> str:
        """computeHashWithNonce (crypt.go:784): MD5 hex of src encrypted with nonce, one object per
        call (rc_compute_hash_with_nonce: GPU seal, group-committed with concurrent callers; MD5
        on host cores).  src is closed if it has close() (fs.CheckClose); its error is raised."""
        nb = bytes(nonce)
        if len(nb) != 24:
            raise ValueError("nonce must be 24 bytes")
        bridge = _ReaderBridge(src, closer=True)
        md5 = ctypes.create_string_buffer(16)
        _raise(_lib.lib().rc_compute_hash_with_nonce(self._h, bridge.c, nb, md5))
        return md5.raw.hex()

    def compute_hash(self, obj, src) -> str:
        """ComputeHash (crypt.go:816): the nonce comes from the encrypted object's header (read
        with newDecrypter, then closed), then computeHashWithNonce over src."""
        d = self.decrypt_data(obj)
        nonce = d.nonce
        d.close()
        return self.compute_hash_with_nonce(nonce, src)


class EnginePool:
    """xs_pool: GPU engines over a device list (repeats allowed: several engines on one device);
    None -> RCLONE_AMD_DEVICES / RCLONE_AMD_DEVICE / every device."""

    def __init__(self, devices=None, batch_blocks: int = 256, slots: int = 3):
        L = _lib.lib()
        if devices:
            arr = (ctypes.c_int * len(devices))(*devices)
            self.handle = L.xs_pool_create(arr, len(devices), batch_blocks, slots)
        else:
            self.handle = L.xs_pool_create(None, 0, batch_blocks, slots)
        if not self.handle:
            raise RuntimeError("xs_pool_create: " + _lib.last_error())

    def __len__(self):
        return _lib.lib().xs_pool_size(self.handle)

    def engine(self, i):
        return _lib.lib().xs_pool_engine(self.handle, i)

    def stats(self):
        """Per engine: (combined batches, requests, blocks) of its coalescing queue."""
        out = []
        for i in range(len(self)):
            a = (ctypes.c_uint64 * 3)()
            _lib.lib().xs_engine_stats(self.engine(i), a)
            out.append(tuple(a))
        return out

    def close(self):
        if getattr(self, "handle", None):
            _lib.lib().xs_pool_destroy(self.handle)
            self.handle = None


class Encrypter:
    """encrypter (cipher.go:681): an io.Reader of the encrypted stream."""

    def __init__(self, cipher: Cipher, reader, nonce=None):
        self._cipher = cipher
        self._bridge = _ReaderBridge(reader, closer=False)
        e = ctypes.c_int32(0)
        nb = bytes(nonce) if nonce is not None else None
        if nb is not None and len(nb) != 24:
            raise ValueError("nonce must be 24 bytes")
        self._free = _lib.lib().rc_encrypter_free
        self._h = _lib.lib().rc_encrypt_data(cipher._h, self._bridge.c, nb, ctypes.byref(e))
        if not self._h:
            _raise(e.value, wrapped=RC_EOF)
            raise GPUError(GPUError.message)

    def __del__(self):
        # at interpreter exit the module globals may already be gone: bound function only
        h, free = getattr(self, "_h", None), getattr(self, "_free", None)
        if h and free is not None:
            free(h)
            self._h = None

    @property
    def nonce(self) -> bytes:
        b = (ctypes.c_uint8 * 24)()
        _lib.lib().rc_encrypter_nonce(self._h, b)
        return bytes(b)

    def set_md5(self, on: bool = True):
        """crypt.put's ciphertext tee hash taken by the encrypter (rc_encrypter_set_md5); before
        the first read only."""
        _raise(_lib.lib().rc_encrypter_set_md5(self._h, int(bool(on))))

    def md5(self) -> bytes:
        """MD5 of exactly the bytes read so far (hasher.Sums() of the reference's TeeReader)."""
        d = ctypes.create_string_buffer(16)
        _raise(_lib.lib().rc_encrypter_md5(self._h, d))
        return d.raw

    def read_go(self, n):
        """Go-style Read: returns (data, err) with err None, EOF or an exception."""
        buf = ctypes.create_string_buffer(max(n, 1))
        e = ctypes.c_int32(0)
        got = _lib.lib().rc_encrypter_read(self._h, buf, n, ctypes.byref(e))
        err = None if e.value == RC_NIL else (EOF if e.value == RC_EOF else _ERRS.exc(e.value))
        return buf.raw[:got], err

    def read(self, n=-1):
        if n is None or n < 0:
            return self.readall()
        while True:
            data, err = self.read_go(n)
            if err is not None and err is not EOF:
                raise err
            if data or err is EOF or n == 0:
                return data

    def readall(self):
        out = []
        while True:
            data = self.read(1 << 20)
            if not data:
                return b"".join(out)
            out.append(data)


class Decrypter:
    """decrypter (cipher.go:776): io.ReadCloser + io.Seeker + fs.RangeSeeker of plaintext."""

    def __init__(self, cipher: Cipher, reader, open_fn=None, offset=0, limit=-1):
        self._cipher = cipher
        self._bridges = []
        self._free = _lib.lib().rc_decrypter_free
        e = ctypes.c_int32(0)
        if open_fn is None:
            b = _ReaderBridge(reader)
            self._bridges.append(b)
            self._h = _lib.lib().rc_decrypt_data(cipher._h, b.c, ctypes.byref(e))
        else:
            def _open(user, off, lim, out):
                try:
                    r = open_fn(off, lim)
                    br = _ReaderBridge(r)
                    self._bridges.append(br)
                    out[0] = br.c
                    return RC_NIL
                except Exception as ex:
                    return _ERRS.code(ex)
            self._open_cb = _lib.OPEN_FN(_open)
            w = ctypes.c_int32(0)
            self._h = _lib.lib().rc_decrypt_data_seek_ex(cipher._h, self._open_cb, None, offset, limit, ctypes.byref(e),
                                                         ctypes.byref(w))
            if not self._h and e.value != RC_NIL:  # RC_ERR_REOPEN: the opener's own error as the cause
                raise _ERRS.exc(e.value, w.value)  # (RC_EOF too: newDecrypterSeek's RangeSeek hit the end)
        if not self._h:
            _raise(e.value)
            raise GPUError(GPUError.message)

    def __del__(self):
        # at interpreter exit the module globals may already be gone: bound function only
        h, free = getattr(self, "_h", None), getattr(self, "_free", None)
        if h and free is not None:
            free(h)
            self._h = None

    @property
    def nonce(self) -> bytes:
        b = (ctypes.c_uint8 * 24)()
        _lib.lib().rc_decrypter_nonce(self._h, b)
        return bytes(b)

    def read_go(self, n):
        buf = ctypes.create_string_buffer(max(n, 1))
        e = ctypes.c_int32(0)
        got = _lib.lib().rc_decrypter_read(self._h, buf, n, ctypes.byref(e))
        if e.value in (RC_NIL,):
            err = None
        elif e.value == RC_EOF:
            err = EOF
        else:
            err = _ERRS.exc(e.value, _lib.lib().rc_decrypter_wrapped_error(self._h))
        return buf.raw[:got], err

    def read(self, n=-1):
        if n is None or n < 0:
            return self.readall()
        while True:
            data, err = self.read_go(n)
            if err is not None and err is not EOF:
                if data:
                    return data  # the error is sticky: the next read raises it
                raise err
            if data or err is EOF or n == 0:
                return data

    def readall(self):
        out = []
        while True:
            data, err = self.read_go(1 << 20)
            if data:
                out.append(data)
            if err is EOF:
                return b"".join(out)
            if err is not None:
                raise err

    def range_seek(self, offset: int, whence: int = 0, limit: int = -1) -> int:
        """RangeSeek (cipher.go:972)."""
        e = ctypes.c_int32(0)
        off = _lib.lib().rc_decrypter_range_seek(self._h, offset, whence, limit, ctypes.byref(e))
        if e.value != RC_NIL:
            raise _ERRS.exc(e.value, _lib.lib().rc_decrypter_wrapped_error(self._h))
        return off

    def seek(self, offset: int, whence: int = 0) -> int:
        return self.range_seek(offset, whence, -1)

    def close(self):
        """Close (cipher.go:1069): ErrorFileClosed on a second close."""
        rc = _lib.lib().rc_decrypter_close(self._h)
        _raise(rc)
