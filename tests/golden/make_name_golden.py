#!/usr/bin/env python3
"""Generate tests/golden/name_vectors.json (run in the build container only).

Sources:
  1. The reference's own file-name tables, extracted as DATA from
     /root/reference/backend/crypt/cipher_test.go: TestEncodeFileNameBase32/64/32768 (:72-136),
     TestEncryptSegmentBase32/64/32768 (:207-271; zero nameKey / nameTweak, i.e. password "").
  2. OpenSSL libcrypto AES-256-ECB (an independent AES implementation) for block-cipher
     known answers under random keys, pinning the oracle's AES beyond the EME vectors.
Only the resulting JSON travels; neither the reference nor libcrypto is needed at test time.
"""
import ctypes
import json
import os
import random
import re

HERE = os.path.dirname(os.path.abspath(__file__))
REF_TEST = "/root/reference/backend/crypt/cipher_test.go"
LIBCRYPTO = "/usr/lib/x86_64-linux-gnu/libcrypto.so.3"

PAIR = re.compile(r'\{"((?:[^"\\]|\\.)*)", "((?:[^"\\]|\\.)*)"\}')


def go_str(s):
    return json.loads('"' + s + '"')


def table(src, func):
    start = src.index(f"func {func}(")
    end = src.index("\n}\n", start)
    return [[go_str(a), go_str(b)] for a, b in PAIR.findall(src[start:end])]


def aes_vectors(n_keys=8, n_blocks=4, seed=0xAE5):
    L = ctypes.CDLL(LIBCRYPTO)
    L.EVP_CIPHER_CTX_new.restype = ctypes.c_void_p
    L.EVP_aes_256_ecb.restype = ctypes.c_void_p
    L.EVP_EncryptInit_ex.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_char_p,
                                     ctypes.c_char_p]
    L.EVP_CIPHER_CTX_set_padding.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.EVP_EncryptUpdate.argtypes = [ctypes.c_void_p, ctypes.c_char_p, ctypes.POINTER(ctypes.c_int), ctypes.c_char_p,
                                    ctypes.c_int]
    L.EVP_CIPHER_CTX_free.argtypes = [ctypes.c_void_p]
    rng = random.Random(seed)
    out = []
    for _ in range(n_keys):
        key = bytes(rng.randrange(256) for _ in range(32))
        pt = bytes(rng.randrange(256) for _ in range(16 * n_blocks))
        ctx = L.EVP_CIPHER_CTX_new()
        assert L.EVP_EncryptInit_ex(ctx, L.EVP_aes_256_ecb(), None, key, None) == 1
        L.EVP_CIPHER_CTX_set_padding(ctx, 0)
        buf = ctypes.create_string_buffer(len(pt) + 16)
        ol = ctypes.c_int(0)
        assert L.EVP_EncryptUpdate(ctx, buf, ctypes.byref(ol), pt, len(pt)) == 1
        L.EVP_CIPHER_CTX_free(ctx)
        out.append({"key": key.hex(), "pt": pt.hex(), "ct": buf.raw[:ol.value].hex()})
    return out


def main():
    src = open(REF_TEST, encoding="utf-8").read()
    data = {"source": "backend/crypt/cipher_test.go tables + OpenSSL AES-256-ECB"}
    for enc in ("Base32", "Base64", "Base32768"):
        data["encode_" + enc.lower()] = table(src, "TestEncodeFileName" + enc)
        data["segment_" + enc.lower()] = table(src, "TestEncryptSegment" + enc)
    data["aes256"] = aes_vectors()
    # FIPS-197 Appendix C.3
    data["fips197_c3"] = {"key": bytes(range(32)).hex(), "pt": "00112233445566778899aabbccddeeff",
                          "ct": "8ea2b7ca516745bfeafc49904b496089"}
    with open(os.path.join(HERE, "name_vectors.json"), "w", encoding="utf-8") as f:
        json.dump(data, f, indent=1, ensure_ascii=False)
    print({k: len(v) for k, v in data.items() if isinstance(v, list)})


if __name__ == "__main__":
    main()
