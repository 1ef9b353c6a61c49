#!/usr/bin/env python3
"""Generate the committed golden fixtures under tests/golden/ (run in the build container only).

Sources of truth, in order:
  1. The reference's own known-answer tables, extracted as DATA from
     /root/reference/backend/crypt/cipher_test.go (file0/file1/file16 :1123-1140,
     TestNonceIncrement :757-867, TestNonceAdd :869-1005, TestEncryptedSize :685-706,
     TestDecryptedSize :708-727, TestDecrypterCalculateUnderlying :1433-1483,
     TestKey :1609-1642).
  2. libsodium 1.0.18 (/opt/conda/lib/libsodium.so, ISC), an independent implementation
     of the NaCl secretbox spec that x/crypto v0.54.0 nacl/secretbox implements; it is
     used to produce vectors the reference does not pin (full 64 KiB blocks, every
     boundary length, nonce-carry edges, multi-block crypt files, per-file MD5s for the
     cryptcheck invariant).  libsodium does not exist on the GPU box, so only its
     outputs travel, as the JSON written here.
  3. hashlib.scrypt for key derivation (cipher.go:241), pinned by TestKey.

Plaintexts for large vectors come from generators that tests re-create bit-exactly
(rclone_amd.testdata): the reference's randomSource (cipher_test.go:1007-1045),
lib/readers PatternReader (pattern_reader.go:11-15) and SplitMix64.
"""
import ctypes
import hashlib
import json
import os
import re
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from rclone_amd.testdata import random_source, pattern_bytes, splitmix64_bytes  # noqa: E402

REF_TEST = "/root/reference/backend/crypt/cipher_test.go"
SODIUM = "/opt/conda/lib/libsodium.so"

BLOCK_DATA = 65536
BLOCK_SIZE = BLOCK_DATA + 16
MAGIC = b"RCLONE\x00\x00"


def sodium():
    lib = ctypes.CDLL(SODIUM)
    assert lib.sodium_init() >= 0
    lib.crypto_secretbox_easy.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.c_ulonglong,
                                          ctypes.c_char_p, ctypes.c_char_p]
    lib.crypto_secretbox_open_easy.argtypes = lib.crypto_secretbox_easy.argtypes
    return lib


LIB = sodium()


def seal(msg, nonce, key):
    out = ctypes.create_string_buffer(len(msg) + 16)
    assert LIB.crypto_secretbox_easy(out, msg, len(msg), nonce, key) == 0
    return out.raw


def open_box(box, nonce, key):
    out = ctypes.create_string_buffer(max(len(box) - 16, 1))
    rc = LIB.crypto_secretbox_open_easy(out, box, len(box), nonce, key)
    return out.raw[: len(box) - 16] if rc == 0 else None


def nonce_add(n, x):
    v = int.from_bytes(n, "little") + x
    return (v % (1 << 192)).to_bytes(24, "little")


def encrypt_file(plain, nonce0, key):
    out = [MAGIC, nonce0]
    nblocks = (len(plain) + BLOCK_DATA - 1) // BLOCK_DATA
    for b in range(nblocks):
        out.append(seal(plain[b * BLOCK_DATA:(b + 1) * BLOCK_DATA], nonce_add(nonce0, b), key))
    return b"".join(out)


# ---------------------------------------------------------------- reference tables (data)
def _bytes_list(s):
    return [int(x, 16) for x in re.findall(r"0[xX][0-9a-fA-F]+", s)]


def ref_tables():
    src = open(REF_TEST).read()
    lines = src.splitlines()

    def block(start, end):
        return "\n".join(lines[start - 1:end])

    out = {}
    # file0/file1/file16 cipher_test.go:1122-1140
    seg = block(1122, 1140)
    for name in ("file0", "file1", "file16"):
        m = re.search(name + r" = \[\]byte\{(.*?)\n\t\}", seg, re.S)
        out[name] = bytes(_bytes_list(m.group(1))).hex()
    # TestNonceIncrement :757-867 -> pairs of nonce{...}
    seg = block(757, 867)
    nonces = [bytes(_bytes_list(m) + [0] * (24 - len(_bytes_list(m)))).hex()
              for m in re.findall(r"nonce\{([^}]*)\}", seg)]
    out["nonce_increment"] = [{"in": nonces[i], "out": nonces[i + 1]} for i in range(0, len(nonces), 2)]
    # TestNonceAdd :869-1005 -> (add, in, out)
    seg = block(869, 1005)
    entries = re.findall(r"\{\s*(0x[0-9A-Fa-f]+),\s*nonce\{([^}]*)\},\s*nonce\{([^}]*)\},\s*\}", seg, re.S)
    out["nonce_add"] = [{"add": int(a, 16),
                         "in": bytes(_bytes_list(i) + [0] * (24 - len(_bytes_list(i)))).hex(),
                         "out": bytes(_bytes_list(o) + [0] * (24 - len(_bytes_list(o)))).hex()}
                        for a, i, o in entries]
    # TestEncryptedSize :685-706 evaluated (constant expressions only)
    seg = block(685, 706)
    out["encrypted_size"] = [[eval(a.replace("<<", "<<")), eval(b)] for a, b in
                             re.findall(r"\{([^,{}]+),\s*([^{}]+)\},", seg)]
    # TestDecryptedSize errors :708-727
    seg = block(708, 727)
    out["decrypted_size_errors"] = [[eval(a), e] for a, e in re.findall(r"\{([^,{}]+),\s*(Error\w+)\},", seg)]
    # calculateUnderlying :1433-1483
    seg = block(1433, 1476)
    env = {"fileHeaderSize": 32, "blockDataSize": BLOCK_DATA, "blockSize": BLOCK_SIZE,
           "int64": lambda x: x}
    rows = []
    for m in re.findall(r"\{([^{}]*)\},", seg):
        parts = [p.strip() for p in m.split(",")]
        if len(parts) == 6:
            rows.append([eval(p, env) for p in parts])
    out["calculate_underlying"] = rows
    # open-callback table of TestNewDecrypterSeekLimit :1367-1404
    seg = block(1367, 1409)
    rows = []
    for m in re.findall(r"\{([^{}]*)\},", seg):
        parts = [p.strip() for p in m.split(",")]
        if len(parts) == 4:
            rows.append([eval(p, env) for p in parts])
    out["seek_open_callback"] = rows
    # TestKey :1609-1642
    seg = block(1609, 1642)
    keys = []
    for call in re.finditer(r'c\.Key\("([^"]*)", "([^"]*)"\)\)\n(.*?)(?=\n\n|\n\trequire|\n\})', seg, re.S):
        pw, salt, body = call.group(1), call.group(2), call.group(3)
        arrays = re.findall(r"\]u?int8?\w*\{([^}]*)\}|\]byte\{([^}]*)\}", body)
        vals = [bytes(_bytes_list(a or b)).hex() for a, b in arrays]
        if len(vals) == 3 and vals[0]:
            keys.append({"password": pw, "salt": salt, "dataKey": vals[0], "nameKey": vals[1], "nameTweak": vals[2]})
    out["key_kat"] = keys
    return out


def main():
    ref = ref_tables()
    assert len(ref["nonce_increment"]) == 25, len(ref["nonce_increment"])
    assert len(ref["nonce_add"]) == 25, len(ref["nonce_add"])
    assert len(ref["encrypted_size"]) == 8, ref["encrypted_size"]
    assert len(ref["calculate_underlying"]) == 30, len(ref["calculate_underlying"])
    assert len(ref["seek_open_callback"]) == 30, len(ref["seek_open_callback"])
    assert len(ref["key_kat"]) == 4, ref["key_kat"]
    # scrypt pins (cipher.go:241 N=16384 r=8 p=1, 80 bytes; defaultSalt cipher.go:59)
    default_salt = bytes([0xA8, 0x0D, 0xF4, 0x3A, 0x8F, 0xBD, 0x03, 0x08, 0xA7, 0xCA, 0xB8, 0x3E, 0x58, 0x1F, 0x86, 0xB1])
    for kat in ref["key_kat"]:
        salt = kat["salt"].encode() if kat["salt"] else default_salt
        k = hashlib.scrypt(kat["password"].encode(), salt=salt, n=16384, r=8, p=1, maxmem=64 << 20, dklen=80)
        assert k[:32].hex() == kat["dataKey"], kat
        assert k[32:64].hex() == kat["nameKey"], kat
        assert k[64:80].hex() == kat["nameTweak"], kat
    # libsodium must reproduce the reference's own golden files (zero key, nonce 01..18)
    zkey = bytes(32)
    n0 = bytes(range(1, 25))
    assert encrypt_file(b"", n0, zkey).hex() == ref["file0"]
    assert encrypt_file(b"\x01", n0, zkey).hex() == ref["file1"]
    assert encrypt_file(bytes(range(1, 17)), n0, zkey).hex() == ref["file16"]
    with open(os.path.join(HERE, "reference_kat.json"), "w") as f:
        json.dump(ref, f, indent=1)

    # ----------------------------------------------------------- single secretbox vectors
    key = splitmix64_bytes(0xC0FFEE, 32)
    nonce = splitmix64_bytes(0xBADC0DE, 24)
    lengths = [1, 2, 15, 16, 17, 31, 32, 33, 47, 48, 63, 64, 65, 95, 96, 127, 128, 129, 255, 256, 257,
               1000, 1023, 1024, 1025, 4095, 4096, 4097, 16383, 16384, 16385, 65471, 65472, 65473,
               65503, 65504, 65505, 65519, 65520, 65521, 65535, 65536]
    single = []
    for i, n in enumerate(lengths):
        msg = splitmix64_bytes(1000 + i, n)
        box = seal(msg, nonce, key)
        assert open_box(box, nonce, key) == msg
        entry = {"len": n, "msg_seed": 1000 + i, "tag": box[:16].hex(), "sha256": hashlib.sha256(box).hexdigest()}
        if n <= 1025:
            entry["box"] = box.hex()
        else:
            entry["head"] = box[:80].hex()
            entry["tail"] = box[-64:].hex()
        single.append(entry)
    # nonces that exercise every carry path of the per-block nonce increment (cipher.go:647-678)
    carry_nonces = [
        bytes([0xFF] * 8) + bytes(16),                    # carry out of byte 7 into byte 8
        bytes([0xFE] + [0xFF] * 15) + bytes(8),          # carry through bytes 0..15 (HSalsa20 input) into 16
        bytes([0xFF] * 24),                              # full 192-bit wrap
        bytes([0xFD] + [0xFF] * 23),                     # wrap on block 2
        bytes([0xFF] * 16) + bytes([0x12] * 8),          # carry into the Salsa20 nonce words
    ]
    files = []
    sizes = [0, 1, 16, 17, 32, 33, 64, 1000, 65535, 65536, 65537, 65552, 131072, 131073, 200000, 3 * 65536 + 7]
    for i, sz in enumerate(sizes):
        for kind in ("random_source", "splitmix64", "pattern"):
            if kind == "random_source":
                plain = random_source(sz)
            elif kind == "splitmix64":
                plain = splitmix64_bytes(5000 + i, sz)
            else:
                plain = pattern_bytes(sz)
            n0i = splitmix64_bytes(7000 + i, 24)
            ct = encrypt_file(plain, n0i, key)
            files.append({"size": sz, "plain": kind, "plain_seed": 5000 + i, "nonce0": n0i.hex(),
                          "enc_size": len(ct), "sha256": hashlib.sha256(ct).hexdigest(),
                          "md5": hashlib.md5(ct).hexdigest(),
                          "tags": [ct[32 + b * BLOCK_SIZE: 48 + b * BLOCK_SIZE].hex()
                                   for b in range((len(ct) - 32 + BLOCK_SIZE - 1) // BLOCK_SIZE)]})
    for j, cn in enumerate(carry_nonces):
        plain = splitmix64_bytes(9000 + j, 4 * BLOCK_DATA + 123)
        ct = encrypt_file(plain, cn, key)
        files.append({"size": len(plain), "plain": "splitmix64", "plain_seed": 9000 + j, "nonce0": cn.hex(),
                      "enc_size": len(ct), "sha256": hashlib.sha256(ct).hexdigest(),
                      "md5": hashlib.md5(ct).hexdigest(),
                      "tags": [ct[32 + b * BLOCK_SIZE: 48 + b * BLOCK_SIZE].hex() for b in range(5)]})
    # config-1 shape: 1000 x 64 KiB random files (crypt over memory, then cryptcheck): the
    # cryptcheck invariant is MD5(ciphertext) == MD5 stored by the wrapped remote
    # (cmd/cryptcheck/cryptcheck.go:91-114, crypt.go:784-809).
    config1 = []
    ckey = hashlib.scrypt(b"potato", salt=default_salt, n=16384, r=8, p=1, maxmem=64 << 20, dklen=80)[:32]
    for i in range(1000):
        plain = splitmix64_bytes(100000 + i, BLOCK_DATA)
        n0i = splitmix64_bytes(200000 + i, 24)
        ct = encrypt_file(plain, n0i, ckey)
        config1.append(hashlib.md5(ct).hexdigest())
    out = {"key": key.hex(), "nonce": nonce.hex(), "single": single, "files": files,
           "config1": {"password": "potato", "salt": "", "plain_seed_base": 100000,
                       "nonce_seed_base": 200000, "n": 1000, "size": BLOCK_DATA, "md5": config1}}
    with open(os.path.join(HERE, "sodium_vectors.json"), "w") as f:
        json.dump(out, f, indent=0)
    print("wrote reference_kat.json and sodium_vectors.json")


if __name__ == "__main__":
    main()
