#!/usr/bin/env python3
"""Compare rocprofv3 kernel-trace durations with bench.py's HIP-event averages for the same
profiled command (tools/gpu_round.sh writes both).  The timed region is the last --steps
launches of each kernel; the warmup launches before it are excluded, like bench.py does.
usage: tools/prof_agree.py <prof_dir> <prof.log> <out.json> [steps (default: the bench line's)]"""
import csv
import glob
import json
import sys


def main():
    d, log, out = sys.argv[1], sys.argv[2], sys.argv[3]
    rows = []
    for f in glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    bench = None
    for line in open(log):
        if line.startswith("{"):
            bench = json.loads(line)
    steps = int(sys.argv[4]) if len(sys.argv) > 4 else bench["steps"]  # the bench's own timed launches
    # the configs[3] leg (bench.py objectset_leg) runs after the headline timing: its launches
    # (warm-up + timed passes x rounds per pass) come last in the trace and are skipped
    tail = 0
    os_ = bench.get("objectset")
    if os_:
        per_rank = -(-os_["counters"]["blocks"] // os_["steps"] // bench["n_gpus"])
        rounds = -(-per_rank // 100_000)
        tail = (os_["steps"] + os_["warmup"]) * rounds
    res = {"steps": steps, "objectset_launches_skipped": tail}
    ev = {"xs_seal": bench["roofline"]["kernel_ms_avg"], "xs_open": bench["roofline"]["open"]["kernel_ms_avg"]}
    for name in ("xs_seal", "xs_open"):
        dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in rows if name in r["Kernel_Name"]
               and "split" not in r["Kernel_Name"]]
        dur_sorted = dur  # trace rows are in dispatch order per file
        if tail:
            dur_sorted = dur_sorted[:-tail]
        timed = dur_sorted[-steps:]
        avg = sum(timed) / len(timed)
        res[name] = {"rocprof_timed_avg_ms": round(avg, 4), "rocprof_all_avg_ms": round(sum(dur) / len(dur), 4),
                     "launches": len(dur), "hip_events_avg_ms": ev[name],
                     "rel_diff": round(abs(avg - ev[name]) / ev[name], 4)}
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
