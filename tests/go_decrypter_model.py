"""TEST INFRASTRUCTURE: step-by-step Python restatements of the reference's decrypter and
encrypter state machines (backend/crypt/cipher.go:681-1087), used as the checkers for randomised
operation sequences on the GPU decrypter and encrypter (tests/test_decrypter_fuzz_gpu.py).  Blocks
are sealed and opened with the CPU oracle (oracle/pyoracle.py, secretbox.Seal / Open); nothing
here is part of the product path.

Followed line by line:
  newEncrypter       cipher.go:694-716  (header = magic + nonce, served first)
  encrypter.Read     cipher.go:719-745  (ReadFill of one block; n == 0 -> finish(err); Seal; increment)
  encrypter.finish   cipher.go:748-758
  newDecrypterSeek   cipher.go:821-859  (open the header only, the header + limit, or the whole file)
  newDecrypter       cipher.go:793-818  (ReadFill of the 32-byte header, magic, nonce)
  fillBuffer         cipher.go:862-898  (ReadFill of one block, header check, Open, nonce.increment)
  Read               cipher.go:901-927  (sticky error, limit, finish(io.EOF) when the limit runs out)
  RangeSeek          cipher.go:972-1034 (whence, unFinish after EOF, reopen, fill, discard, limit)
  finish / unFinish  cipher.go:1042-1066
  Close              cipher.go:1069-1087
The opener hands out bytes.Buffer-like readers (tests/go_readers.Buffer) over the requested
underlying range, which is what every reader in these tests is; lib/readers.ReadFill is
restated in _read_fill.
"""
from oracle import pyoracle as orc
from rclone_amd import crypt
from rclone_amd.crypt import EOF

FILE_HEADER = 32
BLOCK_HEADER = 16
BLOCK_DATA = 65536
BLOCK_SIZE = BLOCK_HEADER + BLOCK_DATA
MAGIC = b"RCLONE\x00\x00"


def _read_fill(r, n):
    """lib/readers.ReadFill: read until n bytes or an error; (data, err)."""
    out = bytearray()
    err = None
    while len(out) < n and err is None:
        d, err = r.read_go(n - len(out))
        out += d
    return bytes(out), err


class SeekStartError(crypt.CryptError):
    pass


class ModelEncrypter:
    """newEncrypter(in, nonce) + Read (cipher.go:694-758)."""

    def __init__(self, key, src, nonce):
        self.key, self.src, self.nonce = bytes(key), src, bytes(nonce)
        self.buf = MAGIC + self.nonce  # bufSize = fileHeaderSize, bufIndex 0
        self.idx = 0
        self.err = None

    def read_go(self, n):
        if self.err is not None:
            return b"", self.err
        if self.idx >= len(self.buf):
            data, err = _read_fill(self.src, BLOCK_DATA)
            if not data:
                if self.err is None:  # finish (cipher.go:748-758)
                    self.err = err
                return b"", self.err
            self.buf = orc.seal(data, self.nonce, self.key)  # possibly err != nil: the next fill returns it
            self.idx = 0
            self.nonce = orc.nonce_increment(self.nonce)
        out = self.buf[self.idx:self.idx + n]
        self.idx += len(out)
        return out, None


class ModelDecrypter:
    def __init__(self, key, opener, offset, limit, pass_bad_blocks=False):
        """newDecrypterSeek (cipher.go:821); raises the error the reference returns."""
        self.key, self.open, self.pass_bad_blocks = bytes(key), opener, pass_bad_blocks
        self.err = None
        self.limit = -1
        self.buf, self.idx = b"", 0
        do_range_seek = set_limit = False
        if offset == 0 and limit < 0:
            rc = opener(0, -1)
        elif offset == 0:
            _, ulimit, _, _ = orc.calculate_underlying(offset, limit)
            rc = opener(0, FILE_HEADER + ulimit)
            set_limit = True
        else:
            rc = opener(0, FILE_HEADER)
            do_range_seek = True
        self.rc = rc
        # newDecrypter (cipher.go:793-818)
        hdr, err = _read_fill(rc, FILE_HEADER)
        if len(hdr) < FILE_HEADER and err is EOF:
            raise crypt.ErrorEncryptedFileTooShort(crypt.ErrorEncryptedFileTooShort.message)
        if err is not None and err is not EOF:
            raise err
        if hdr[:8] != MAGIC:
            raise crypt.ErrorEncryptedBadMagic(crypt.ErrorEncryptedBadMagic.message)
        self.nonce = self.initial = hdr[8:32]
        if do_range_seek:
            _, e = self.range_seek(offset, 0, limit)
            if e is not None:
                raise e if e is not EOF else crypt.ErrEOF(crypt.ErrEOF.message)
        if set_limit:
            self.limit = limit

    def _finish(self, err):
        if self.err is not None:
            return self.err
        self.err = err
        return err

    def _fill(self):
        """fillBuffer (cipher.go:862-898): None or the error."""
        data, err = _read_fill(self.rc, BLOCK_SIZE)
        if not data:
            return err
        if len(data) <= BLOCK_HEADER:
            if err is not None and err is not EOF:
                return err
            return crypt.ErrorEncryptedFileBadHeader(crypt.ErrorEncryptedFileBadHeader.message)
        pt = orc.open_box(data, self.nonce, self.key)
        if pt is None:
            if err is not None and err is not EOF:
                return err
            if not self.pass_bad_blocks:
                return crypt.ErrorEncryptedBadBlock(crypt.ErrorEncryptedBadBlock.message)
            pt = bytes(len(data) - BLOCK_HEADER)
        self.buf, self.idx = pt, 0
        self.nonce = orc.nonce_increment(self.nonce)
        return None

    def read_go(self, n):
        """Read (cipher.go:901-927)."""
        if self.err is not None:
            return b"", self.err
        if self.idx >= len(self.buf):
            e = self._fill()
            if e is not None:
                return b"", self._finish(e)
        to_copy = len(self.buf) - self.idx
        if 0 <= self.limit < to_copy:
            to_copy = self.limit
        out = self.buf[self.idx:self.idx + min(n, to_copy)]
        self.idx += len(out)
        if self.limit >= 0:
            self.limit -= len(out)
            if self.limit == 0:
                return out, self._finish(EOF)
        return out, None

    def range_seek(self, offset, whence, limit):
        """RangeSeek (cipher.go:972-1034): (offset, None) or (0, err)."""
        if whence != 0:
            return 0, self._finish(SeekStartError("can only seek from the start"))
        if self.err is EOF:
            self.err = None  # unFinish (cipher.go:1055-1066)
            self.buf, self.idx = b"", 0
        elif self.err is not None:
            return 0, self.err
        uoff, ulimit, discard, blocks = orc.calculate_underlying(offset, limit)
        self.nonce = orc.nonce_add(self.initial, blocks)
        # the readers here are not fs.RangeSeekers: close and reopen (cipher.go:1003-1015)
        self.rc = self.open(uoff, ulimit)
        e = self._fill()
        if e is not None:
            return 0, self._finish(e)
        if discard > len(self.buf):
            return 0, self._finish(crypt.ErrorBadSeek(crypt.ErrorBadSeek.message))
        self.idx = discard
        self.limit = limit
        return offset, None

    def close(self):
        """Close (cipher.go:1069-1087): None, or ErrorFileClosed the second time."""
        if isinstance(self.err, crypt.ErrorFileClosed):
            return self.err
        if self.err is None:
            self._finish(EOF)
        self.err = crypt.ErrorFileClosed(crypt.ErrorFileClosed.message)
        return None


def kind(err):
    """A comparable name for an error from either side: None, "EOF", the sentinel class, or the
    message of a plain error."""
    if err is None:
        return None
    if err is EOF or isinstance(err, crypt.ErrEOF):
        return "EOF"
    if isinstance(err, SeekStartError) or str(err) == "can only seek from the start":
        return "can only seek from the start"
    return type(err).__name__
