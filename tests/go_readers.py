"""Test doubles with Go io.Reader semantics (read_go -> (data, err)), as used by
backend/crypt/cipher_test.go and lib/readers."""
from rclone_amd.crypt import EOF


class RandomSource:
    """randomSource (cipher_test.go:1007-1045): byte = counter % 257 for counter 1..size."""

    def __init__(self, size):
        self.counter = 0
        self.size = size

    def read_go(self, n):
        out = bytearray()
        err = None
        while len(out) < n:
            if self.counter >= self.size:
                err = EOF
                break
            self.counter += 1
            out.append(self.counter % 257 & 0xFF)
        return bytes(out), err

    def write(self, p):
        """randomSource.Write: check p continues the sequence."""
        for b in p:
            self.counter += 1
            if b != (self.counter % 257) & 0xFF:
                raise AssertionError(f"Error in stream at {self.counter}")
        return len(p)


class Zeroes:
    def read_go(self, n):
        return bytes(n), None


class Buffer:
    """bytes.Buffer reader: (n, nil) while data remains, then (0, EOF)."""

    def __init__(self, data):
        self.data = bytes(data)
        self.pos = 0

    def read_go(self, n):
        if self.pos >= len(self.data):
            return b"", EOF
        chunk = self.data[self.pos:self.pos + n]
        self.pos += len(chunk)
        return chunk, None


class ErrorReader:
    """lib/readers ErrorReader: always (0, err)."""

    def __init__(self, err):
        self.err = err

    def read_go(self, n):
        return b"", self.err


class MultiReader:
    """io.MultiReader."""

    def __init__(self, *readers):
        self.readers = list(readers)

    def read_go(self, n):
        while self.readers:
            data, err = self.readers[0].read_go(n)
            if err is EOF:
                self.readers.pop(0)
                if data:
                    return data, (EOF if not self.readers else None)
                continue
            return data, err
        return b"", EOF


class CloseDetector:
    """closeDetector (cipher_test.go:1207-1221)."""

    def __init__(self, r):
        self.r = r
        self.closed = 0

    def read_go(self, n):
        return self.r.read_go(n)

    def close(self):
        self.closed += 1


class Potato(Exception):
    def __str__(self):
        return "potato"


def read_all(r, bufsize=1 << 20):
    """io.ReadAll over a Go-style reader; returns (data, err) with err None on EOF."""
    out = []
    while True:
        data, err = r.read_go(bufsize)
        if data:
            out.append(data)
        if err is EOF:
            return b"".join(out), None
        if err is not None:
            return b"".join(out), err


def copy_buffer(dst_write, r, bufsize):
    """io.CopyBuffer(dst, r, buf): returns (n, err)."""
    n = 0
    while True:
        data, err = r.read_go(bufsize)
        if data:
            dst_write(data)
            n += len(data)
        if err is EOF:
            return n, None
        if err is not None:
            return n, err
