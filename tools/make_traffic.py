#!/usr/bin/env python3
"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (tools/pmc.sh) into HBM bytes per
xs_crypt launch: profiles/pmc_traffic.json (read by bench.py as roofline.traffic).

Correction (MI355X_MICROARCH.md, HBM section): on gfx950 FETCH_SIZE counts exactly half the
bytes of a wide (16 B/lane) streaming read -- global_load and LDS-DMA alike -- so reads =
2 x FETCH_SIZE; WRITE_SIZE is exact for 16 B/lane stores.  Both are in KiB.
Also records SQ_INSTS_VALU (wave-instructions) and SQ_INSTS_VALU_MFMA_I8 per launch for the VALU
issue bound (MFMAs run on the matrix pipe: the bound counts SQ_INSTS_VALU - SQ_INSTS_VALU_MFMA_I8)."""
import json
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from rclone_amd.build import KERNEL_SOURCES, build_sources_sha256, kernel_sources_sha256  # noqa: E402


def git_head(root=ROOT):
    """(commit, kernel sources unchanged from it?): run here, in the build container, on the PMC
    passes copied back under profiles/ -- the GPU box has no .git (RCLONE_AMD_GIT_HEAD then)."""
    try:
        head = subprocess.check_output(["git", "-C", root, "rev-parse", "HEAD"], text=True).strip()
        clean = subprocess.run(["git", "-C", root, "diff", "--quiet", "HEAD", "--"] + KERNEL_SOURCES).returncode == 0
        return head, clean
    except Exception:  # noqa: BLE001
        return os.environ.get("RCLONE_AMD_GIT_HEAD", "unknown"), None


def main():
    d, out = sys.argv[1], sys.argv[2]
    acc = load(d)
    head, clean = git_head()
    rel = os.path.relpath(os.path.abspath(d), ROOT)
    res = {"source": f"rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE / SQ_INSTS_VALU / SQ_INSTS_VALU_MFMA_I8 ({rel}), one pass per counter group, "
                     "reads x2 (gfx950 FETCH_SIZE halving, MI355X_MICROARCH.md HBM section)",
           "blocks_per_launch": int(sys.argv[3]) if len(sys.argv) > 3 else 100_000,
           "kernel_sources_sha256": kernel_sources_sha256(),
           "kernel_sources": KERNEL_SOURCES,
           "git_head": head,
           "kernel_sources_clean_at_git_head": clean,
           "library_build_id": build_sources_sha256()}
    for k, cs in acc.items():
        for name, key in (("xs_seal", "seal"), ("xs_open", "open")):
            if name in k and "FETCH_SIZE" in cs and "WRITE_SIZE" in cs:
                fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 * 2
                write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
                res[f"{key}_read_bytes_per_launch"] = round(fetch)
                res[f"{key}_write_bytes_per_launch"] = round(write)
                res[f"{key}_bytes_per_launch"] = round(fetch + write)
            if name in k and "SQ_INSTS_VALU" in cs:
                res[f"{key}_valu_wave_insts_per_launch"] = round(sum(cs["SQ_INSTS_VALU"]) / len(cs["SQ_INSTS_VALU"]))
                if "SQ_WAVES" in cs:
                    res[f"{key}_waves_per_launch"] = round(sum(cs["SQ_WAVES"]) / len(cs["SQ_WAVES"]))
            # the matrix-core Poly1305 (v_mfma_i32_16x16x64_i8): SQ_INSTS_VALU counts these too, but
            # they execute on the SIMD's matrix pipe, so the VALU issue bound uses the difference
            for cname, rkey in (("SQ_INSTS_VALU_MFMA_I8", "mfma_wave_insts"), ("SQ_VALU_MFMA_BUSY_CYCLES", "mfma_busy_cycles"),
                                ("SQ_VALU_MFMA_COEXEC_CYCLES", "mfma_coexec_cycles"), ("GRBM_GUI_ACTIVE", "gui_active_cycles")):
                if name in k and cname in cs:
                    res[f"{key}_{rkey}_per_launch"] = round(sum(cs[cname]) / len(cs[cname]))
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
