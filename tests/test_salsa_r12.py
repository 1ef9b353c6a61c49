"""The generated uniform-aware Salsa20 double rounds 1-2 (rclone_amd/csrc/xs_salsa_r12.h, made by
tools/gen_salsa_r12.py) compute exactly two Salsa20 double rounds of the NaCl spec (SURVEY.md
8(a)) and leave the words in xs_salsa_lazy.h's lazy set: the header's statements are interpreted
on random input words and counters and compared with the plain rounds."""
import os
import random
import re

from test_salsa_lazy import M, plain_dr

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "rclone_amd", "csrc", "xs_salsa_r12.h")
LAZY_HDR = os.path.join(ROOT, "rclone_amd", "csrc", "xs_salsa_lazy.h")


def compile_r12(src):
    body = src[src.index("void xs_salsa_r12("):]
    body = body[body.index("{") + 1:]
    body = body[:body.index("\n}")]
    py = re.sub(r"//.*", "", body)
    py = py.replace("uint32_t s, r;", "").replace("uint32_t ub[16], tu[16];", "")
    py = re.sub(r"#pragma unroll\s*for \(int i = 0; i < 16; i\+\+\) ub\[i\] = w\[i\];", "ub[:] = w[:];", py)
    py = re.sub(r"xs_xad_[vs]{3}\(", "xad(", py)
    py = py.replace("xs_xor3(", "xor3(").replace("xs_r12_rotl_s(", "rotl(")
    py = re.sub(r"__builtin_amdgcn_alignbit\(s, s, (\d+)\)", r"rotr(s, \1)", py)
    py = re.sub(r"(\w+\[\d+\]) \^= (.*?);", r"\1 = (\1 ^ (\2)) & M;", py)
    py = re.sub(r"(\w+) = (\w+\[\d+\]) \+ (\w+\[\d+\]);", r"\1 = (\2 + \3) & M;", py)
    py = re.sub(r"rotl\((\w+\[\d+\]) \+ (\w+\[\d+\]), (\d+)\)", r"rotl((\1 + \2) & M, \3)", py)
    py = py.replace("0u", "0")
    lines = []
    for stmt in py.replace("\n", " ").split(";"):
        stmt = stmt.strip()
        if stmt:
            lines.append(stmt)
    return compile("\n".join(lines), "xs_salsa_r12", "exec")


def test_r12_matches_two_double_rounds():
    src = open(HDR).read()
    mask = int(re.search(r"XS_LAZY_MASK 0x([0-9a-f]+)u", open(LAZY_HDR).read()).group(1), 16)
    code = compile_r12(src)
    rnd = random.Random(11)
    for _ in range(200):
        w = [rnd.getrandbits(32) for _ in range(16)]
        w[8] = rnd.getrandbits(11)  # the counter (K < 1025)
        w[9] = 0
        b, t, ub, tu = [0] * 16, [rnd.getrandbits(32) for _ in range(16)], [0] * 16, [0] * 16
        env = {"w": w, "b": b, "t": t, "ub": ub, "tu": tu, "M": M,
               "rotr": lambda x, k: ((x >> k) | (x << (32 - k))) & M,
               "rotl": lambda x, k: ((x << k) | (x >> (32 - k))) & M,
               "xad": lambda a, b_, c: ((a ^ b_) + c) & M, "xor3": lambda a, b_, c: a ^ b_ ^ c}
        exec(code, env)
        want = plain_dr(plain_dr(w))
        got = [b[i] ^ t[i] if (mask >> i) & 1 else b[i] for i in range(16)]
        assert got == want


def test_r12_generator_is_reproducible():
    import subprocess
    import sys
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_salsa_r12.py")],
                         capture_output=True, text=True, check=True, timeout=600).stdout
    assert out == open(HDR).read()
