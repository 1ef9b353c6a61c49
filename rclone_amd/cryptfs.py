"""The crypt overlay's data-path wrapper surface over a wrapped remote (SURVEY §8(a) rows
a13-a16), on top of the GPU cipher (rclone_amd.crypt -> librclone_crypt.so):

* ``CryptFs.put``          Fs.put / Put / Update (crypt.go:497-563, :1091-1097): encrypt the
                           stream into the wrapped remote's put, tee the ciphertext into the
                           destination's hash, compare, remove the object on mismatch.
* ``CryptFs.open``         Object.Open (crypt.go:1050-1088): Seek/Range options -> (offset,
                           limit) -> DecryptDataSeek with the underlying range-open closure.
* ``CryptFs.size``         Object.Size (crypt.go:1026-1036) / ObjectInfo.Size (:1168-1177).
* ``CryptFs.compute_hash`` Fs.ComputeHash (crypt.go:816-852).
* ``CryptFs.cryptcheck``   cmd/cryptcheck cryptCheck (cryptcheck.go:67-117): underlying hash
                           vs ComputeHash for every pair, batched across objects so the
                           re-encryption and the MD5 both run on the GPU.

``MemoryRemote`` is the minimal backend/memory the tests and tools wrap (memory.go:580-646:
MD5 hash computed on demand, Open honouring Range/Seek).  File names use crypt's "off" name
mode (cipher.go:529: remote + ".bin"); name encryption itself is out of scope.
"""
import hashlib

from . import crypt
from .crypt import EOF, CryptError

SUFFIX = ".bin"  # encryptedSuffix, cipher.go:193


class SeekOption:
    """fs.SeekOption (fs/open_options.go)."""

    def __init__(self, offset: int):
        self.offset = offset


class RangeOption:
    """fs.RangeOption; start/end inclusive, -1 = unset (fs/open_options.go:118 Decode)."""

    def __init__(self, start: int, end: int):
        self.start, self.end = start, end

    def decode(self, size: int):
        if self.start >= 0:
            return self.start, (self.end - self.start + 1) if self.end >= 0 else -1
        if self.end >= 0:
            return max(size - self.end, 0), -1
        return 0, -1


class _BytesReader:
    """io.NopCloser(bytes.NewBuffer(data)) with Go read semantics."""

    def __init__(self, data: bytes):
        self.data, self.pos = data, 0

    def read_go(self, n):
        if self.pos >= len(self.data):
            return b"", EOF
        out = self.data[self.pos:self.pos + n]
        self.pos += len(out)
        return out, None

    def close(self):
        pass


class MemoryRemote:
    """Minimal backend/memory: objects are byte strings, MD5 is the supported hash."""

    def __init__(self):
        self.objects = {}
        self._hash = {}
        self.opens = []  # (remote, offset, limit) of every Open, for tests

    def put(self, remote: str, reader, size: int = -1):
        chunks = []
        while True:
            data, err = reader.read_go(1 << 20)
            if data:
                chunks.append(bytes(data))
            if err is EOF:
                break
            if err is not None:
                raise err
        self.objects[remote] = b"".join(chunks)
        self._hash.pop(remote, None)

    def open(self, remote: str, *options):
        data = self.objects[remote]
        offset, limit = 0, -1
        for o in options:
            if isinstance(o, RangeOption):
                offset, limit = o.decode(len(data))
            elif isinstance(o, SeekOption):
                offset = o.offset
        self.opens.append((remote, offset, limit))
        offset = min(offset, len(data))
        data = data[offset:]
        if limit >= 0:
            data = data[:limit]
        return _BytesReader(data)

    def hash(self, remote: str) -> str:
        if remote not in self._hash:
            self._hash[remote] = hashlib.md5(self.objects[remote]).hexdigest()
        return self._hash[remote]

    def size(self, remote: str) -> int:
        return len(self.objects[remote])

    def remove(self, remote: str):
        self.objects.pop(remote, None)
        self._hash.pop(remote, None)

    def list(self):
        return sorted(self.objects)


class _TeeReader:
    """io.TeeReader(r, hasher)."""

    def __init__(self, r, h):
        self.r, self.h = r, h

    def read_go(self, n):
        data, err = self.r.read_go(n)
        if data:
            self.h.update(data)
        return data, err


class CryptFs:
    """crypt.Fs data path over a wrapped remote (MemoryRemote or anything with the same
    put/open/hash/size/remove)."""

    def __init__(self, wrapped, cipher: crypt.Cipher, ignore_checksum: bool = False, encrypter_md5: bool = True):
        """encrypter_md5: put's tee hash is taken by the encrypter (rc_encrypter_set_md5, hashed on
        host workers while the wrapped put reads) instead of a TeeReader around it."""
        self.wrapped, self.cipher, self.ignore_checksum = wrapped, cipher, ignore_checksum
        self.encrypter_md5 = encrypter_md5

    @staticmethod
    def enc_name(remote: str) -> str:
        return remote + SUFFIX

    # -------------------------------------------------------------- Fs.put (crypt.go:497)
    def put(self, remote: str, reader, size: int = -1):
        enc = self.cipher.encrypt_data(reader)
        hasher = None if self.ignore_checksum or self.encrypter_md5 else hashlib.md5()
        src = enc if hasher is None else _TeeReader(enc, hasher)
        if not self.ignore_checksum and self.encrypter_md5:
            enc.set_md5(True)
        esize = crypt.encrypted_size(size) if size >= 0 else size  # ObjectInfo.Size (:1168)
        name = self.enc_name(remote)
        nonce = enc.nonce  # newObjectInfo(src, encrypter.nonce) is built before the transfer (:536)
        self.wrapped.put(name, src, esize)
        if not self.ignore_checksum:
            src_hash = hasher.hexdigest() if hasher is not None else enc.md5().hex()
            dst_hash = self.wrapped.hash(name)
            if src_hash and dst_hash and src_hash != dst_hash:
                self.wrapped.remove(name)
                raise CryptError(f"corrupted on transfer: md5 encrypted hashes differ src {src_hash!r} "
                                 f"vs dst {dst_hash!r}")
        return nonce

    # -------------------------------------------------------------- Object.Size (:1026)
    def size(self, remote: str) -> int:
        return crypt.decrypted_size(self.wrapped.size(self.enc_name(remote)))

    # -------------------------------------------------------------- Object.Open (:1050)
    def open(self, remote: str, *options):
        offset, limit = 0, -1
        passed = []
        for o in options:
            if isinstance(o, SeekOption):
                offset = o.offset
            elif isinstance(o, RangeOption):
                offset, limit = o.decode(self.size(remote))
            else:
                passed.append(o)
        name = self.enc_name(remote)
        usize = self.wrapped.size(name)

        def open_fn(u_off, u_lim):
            if u_off == 0 and u_lim < 0:
                return self.wrapped.open(name, *passed)
            end = -1
            if u_lim >= 0:
                end = u_off + u_lim - 1
                if end >= usize:
                    end = -1
            return self.wrapped.open(name, *passed, RangeOption(u_off, end))

        return self.cipher.decrypt_data_seek(open_fn, offset, limit)

    # -------------------------------------------------------------- Fs.ComputeHash (:816)
    def _nonce(self, remote: str) -> bytes:
        # "opening the file is sufficient to read the nonce": header range only
        d = self.cipher.decrypt_data(self.wrapped.open(self.enc_name(remote), RangeOption(0, crypt.FILE_HEADER_SIZE - 1)))
        nonce = d.nonce
        d.close()
        return nonce

    def compute_hash(self, remote: str, src) -> str:
        return self.cipher.compute_hash_with_nonce(self._nonce(remote), src)

    # -------------------------------------------------------------- cryptcheck (cryptcheck.go:67)
    def cryptcheck(self, sources: dict, batch: int = 4096, checkers: int = 0):
        """sources: remote -> zero-arg callable returning a reader of the plaintext source.
        checkers > 0: the unchanged cryptcheck's shape -- that many threads, each running the
        per-object ComputeHash (cryptcheck.go:91-114, --checkers); else batches of `batch` objects
        through hash_batch_with_nonce.
        Returns {"differ": [...], "no_hash": [...], "errors": {remote: exc}, "ok": n}."""
        res = {"differ": [], "no_hash": [], "errors": {}, "ok": 0}
        names = sorted(sources)
        if checkers > 0:
            import threading
            lock, it = threading.Lock(), iter(names)

            def check_one(r):
                try:
                    under = self.wrapped.hash(self.enc_name(r))
                except Exception as e:  # "error reading hash from underlying"
                    return "errors", e
                if not under:
                    return "no_hash", None
                try:
                    h = self.compute_hash(r, sources[r]())
                except Exception as e:  # "error computing hash"
                    return "errors", e
                return ("differ", None) if h != under else ("ok", None)

            def worker():
                while True:
                    with lock:
                        r = next(it, None)
                    if r is None:
                        return
                    kind, e = check_one(r)
                    with lock:
                        if kind == "errors":
                            res["errors"][r] = e
                        elif kind == "ok":
                            res["ok"] += 1
                        else:
                            res[kind].append(r)

            th = [threading.Thread(target=worker) for _ in range(checkers)]
            for t in th:
                t.start()
            for t in th:
                t.join()
            res["differ"].sort()
            res["no_hash"].sort()
            return res
        for i in range(0, len(names), batch):
            part = names[i:i + batch]
            under, items, keep = {}, [], []
            for r in part:
                try:
                    under[r] = self.wrapped.hash(self.enc_name(r))
                except Exception as e:  # "error reading hash from underlying"
                    res["errors"][r] = e
                    continue
                if not under[r]:
                    res["no_hash"].append(r)
                    continue
                try:
                    items.append((self._nonce(r), sources[r]()))
                    keep.append(r)
                except Exception as e:  # "error computing hash"
                    res["errors"][r] = e
            for r, h in zip(keep, self.cipher.hash_batch_with_nonce(items)):
                if isinstance(h, BaseException):
                    res["errors"][r] = h
                elif h.hex() != under[r]:
                    res["differ"].append(r)
                else:
                    res["ok"] += 1
        return res
