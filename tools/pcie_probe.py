#!/usr/bin/env python3
"""PCIe ceiling for the host path: pinned host <-> HBM copy rates with
hipMemcpyAsync (torch non_blocking copies), H2D alone, D2H alone and both at once on two
streams, for a few chunk sizes.  Diagnostic only."""
import json
import time

import torch


def rate(fn, nbytes, reps=5):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return round(nbytes / 2**30 / best, 2)


def main():
    total = 4 << 30
    h_src = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    h_dst = torch.empty(total, dtype=torch.uint8, pin_memory=True)
    d_a = torch.empty(total, dtype=torch.uint8, device="cuda")
    d_b = torch.empty(total, dtype=torch.uint8, device="cuda")
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    out = {}
    for chunk in (4 << 20, 16 << 20, 64 << 20, 256 << 20):
        n = total // chunk

        def h2d():
            with torch.cuda.stream(s1):
                for i in range(n):
                    d_a[i * chunk:(i + 1) * chunk].copy_(h_src[i * chunk:(i + 1) * chunk], non_blocking=True)

        def d2h():
            with torch.cuda.stream(s2):
                for i in range(n):
                    h_dst[i * chunk:(i + 1) * chunk].copy_(d_b[i * chunk:(i + 1) * chunk], non_blocking=True)

        def both():
            h2d()
            d2h()
        out[f"{chunk >> 20}MiB"] = {"h2d_GiB_s": rate(h2d, total), "d2h_GiB_s": rate(d2h, total),
                                    "duplex_each_GiB_s": rate(both, total)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
