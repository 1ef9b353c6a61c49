#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc CSVs (tools/pmc.sh output) per kernel: mean counter value per
dispatch.  usage: tools/pmc_summary.py gpurun_out/pmc1 [kernel-substring ...]"""
import collections
import csv
import glob
import json
import sys


def load(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True):
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
    # counters are reported per dispatch (summed over dimensions by rocprofv3 in csv rows)
    return acc


def main():
    d = sys.argv[1]
    subs = sys.argv[2:] or ["xs_seal", "xs_open", "xs_keygen"]
    acc = load(d)
    out = {}
    for k, cs in acc.items():
        if not any(s in k for s in subs):
            continue
        short = k.split("(")[0].replace("void ", "")
        out[short] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[short]["_dispatch_rows"] = {c: len(v) for c, v in cs.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
