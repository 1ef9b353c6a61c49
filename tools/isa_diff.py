#!/usr/bin/env python3
"""Compare the gfx950 machine code of two versions of the crypt kernel file, kernel by kernel.

Compiles each version device-only to assembly (hipcc -S, the product flags) and compares every
kernel's instruction stream (comments, directives and basic-block label numbers stripped).
Used to show that a source-only change -- e.g. removing rejected #if variants -- leaves every
shipped kernel instruction-for-instruction identical, so its performance is unchanged by
construction.

usage: tools/isa_diff.py <old.hip> <new.hip>   (either may be a git rev:path, e.g. HEAD~1:rclone_amd/csrc/xs_kernels.hip)
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "rclone_amd", "csrc")


def source(spec, d, tag):
    if os.path.exists(spec):
        return spec
    text = subprocess.check_output(["git", "-C", ROOT, "show", spec])
    p = os.path.join(d, tag + ".hip")
    open(p, "wb").write(text)
    return p


def kernels(hip, d, tag):
    s_path = os.path.join(d, tag + ".s")
    subprocess.check_call(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", f"-I{CSRC}",
                           f"-I{os.path.join(ROOT, 'include')}", "--cuda-device-only", "-S", "-o", s_path, hip],
                          stderr=subprocess.DEVNULL)
    s = open(s_path).read()
    out = {}
    for m in re.finditer(r"^(_Z\w+):[^\n]*\n(.*?)^\.Lfunc_end", s, re.S | re.M):
        body = []
        for line in m.group(2).splitlines():
            t = line.split(";")[0].strip()
            if t and not t.startswith("."):
                body.append(re.sub(r"\.LBB\d+_\d+", "L", t))
        out[m.group(1)] = body
    return out


def main():
    with tempfile.TemporaryDirectory() as d:
        a = kernels(source(sys.argv[1], d, "old"), d, "old")
        b = kernels(source(sys.argv[2], d, "new"), d, "new")
    same = True
    for k in sorted(set(a) | set(b)):
        if k not in b:
            print(f"removed    {k}  ({len(a[k])} instructions)")
        elif k not in a:
            print(f"added      {k}  ({len(b[k])} instructions)")
            same = False
        else:
            eq = a[k] == b[k]
            same &= eq
            print(f"{'identical' if eq else 'DIFFERENT'}  {k}  ({len(a[k])} / {len(b[k])} instructions)")
    print("every kept kernel identical" if same else "kernels differ")
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
