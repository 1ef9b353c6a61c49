"""Check e2e_sync --anchor records against the CPU oracle (test infrastructure, like
tests/test_e2e_anchor_gpu.py): every sampled stored crypt file's SHA-256 and put's tee MD5.
usage: python tools/check_anchor.py anchor.jsonl"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import pyoracle as orc  # noqa: E402
from rclone_amd.testdata import splitmix64_bytes  # noqa: E402


def main():
    key = hashlib.scrypt(b"potato", salt=bytes.fromhex("a80df43a8fbd0308a7cab83e581f86b1"), n=16384, r=8, p=1,
                         maxmem=2**26, dklen=80)[:32]
    rows = [json.loads(x) for x in open(sys.argv[1])]
    bad = 0
    for row in rows:
        ct = orc.encrypt_file(splitmix64_bytes(row["seed"], row["size"]), bytes.fromhex(row["nonce"]), key)
        bad += hashlib.sha256(ct).hexdigest() != row["sha256"] or hashlib.md5(ct).hexdigest() != row["tee_md5"]
    print(json.dumps({"anchored": len(rows), "mismatches": bad, "max_size": max(r["size"] for r in rows)}))
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
