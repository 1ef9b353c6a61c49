"""Median phase marks (us from entry) of the open's key wave and finalisation, per build and run
(tools/r04_kgrows.sh output)."""
import glob
import json
import sys

d = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/kgrows"
for kind in ("w0006", "full"):
    for v in (0, 1):
        rows = []
        for f in sorted(glob.glob(f"{d}/probe_{kind}_kg{v}_*.json")):
            m = json.load(open(f))["us_from_entry_median"]
            kg = [b[0] for b in m["open_w9"].values()]
            rows.append({"ks0": kg[2], "levels": kg[3:7], "corr": kg[-1], "Z": m["open_w8"]["ks0|Z"][0],
                         "B2": m["open_w0"]["B2"][0], "final": m["open_w0"]["final|loads"][0]})
        for r in rows:
            print(kind, f"kg{v}", json.dumps(r))
