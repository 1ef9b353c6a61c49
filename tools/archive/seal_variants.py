"""Diagnostic: time xs_seal / xs_open on torch-allocated buffers under different launch
contexts, to explain differences between bench.py's kernel times and tools/abtest's.

  object      keygen (object mode) once, then K seal launches back to back
  desc        keygen (descriptor mode) once, then K seal launches back to back
  desc+kg     keygen before every seal launch (bench.py's step order)
  desc+open   bench.py's full step: keygen, seal, keygen, open
Prints one JSON line per variant with the median kernel milliseconds.
"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))  # tools/archive -> repo
sys.path.insert(0, ROOT)


def main():
    import numpy as np
    import torch

    from rclone_amd import _lib, device, shard
    L = _lib.lib()
    dev = torch.device("cuda", 0)
    nb = 100000
    K = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    key = bytes(range(32))
    nonce0 = bytes([0xF0]) + bytes([0xFF] * 7) + bytes(16)
    plain = torch.empty(nb * 65536, dtype=torch.uint8, device=dev)
    device.fill_blocks(plain, 0, 1, 0x5EED)
    body = torch.empty(nb * 65552, dtype=torch.uint8, device=dev)
    out = torch.empty(nb * 65536, dtype=torch.uint8, device=dev)
    ok = torch.empty(nb, dtype=torch.uint8, device=dev)
    ws = device.workspace(nb, dev)
    ws2 = device.workspace(nb, dev)
    gidx = shard.owned_blocks(nb, 1, 0)
    d_seal = torch.from_numpy(shard.seal_descriptors(nonce0, gidx).view(np.uint8).copy()).to(dev)
    d_open = torch.from_numpy(shard.seal_descriptors(nonce0, gidx, open_mode=True).view(np.uint8).copy()).to(dev)
    s = torch.cuda.current_stream(dev)
    sp = ctypes.c_void_p(s.cuda_stream)

    def kg_obj():
        _lib.check(L.xs_keygen_object_dev(1, key, nonce0, 0, nb * 65536, ws.data_ptr(), sp))

    def kg_desc():
        _lib.check(L.xs_keygen_batch_dev(1, key, d_seal.data_ptr(), nb, plain.data_ptr(), nb * 65536,
                                         body.data_ptr(), nb * 65552, ws.data_ptr(), sp))

    def kg_open():
        _lib.check(L.xs_keygen_batch_dev(0, key, d_open.data_ptr(), nb, body.data_ptr(), nb * 65552,
                                         out.data_ptr(), nb * 65536, ws2.data_ptr(), sp))

    def seal():
        _lib.check(L.xs_crypt_dev(1, ws.data_ptr(), nb, plain.data_ptr(), body.data_ptr(), None, sp))

    def opn():
        _lib.check(L.xs_crypt_dev(0, ws2.data_ptr(), nb, body.data_ptr(), out.data_ptr(), ok.data_ptr(), sp))

    def timed(fn, pre=None, warm=3):
        ts = []
        for i in range(warm + K):
            if pre:
                pre()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(s)
            fn()
            b.record(s)
            b.synchronize()
            if i >= warm:
                ts.append(a.elapsed_time(b))
        ts.sort()
        return round(ts[len(ts) // 2], 4)

    res = {}
    kg_obj()
    res["object_seal"] = timed(seal)
    kg_desc()
    res["desc_seal"] = timed(seal)
    res["desc+kg_seal"] = timed(seal, kg_desc)
    kg_open()
    res["desc_open"] = timed(opn)
    res["desc+kg_open"] = timed(opn, kg_open)

    def full_seal():
        seal()

    def pre_full():
        kg_desc()

    # bench order: keygen, seal, keygen, open -> time seal and open within it
    ts, to = [], []
    for i in range(3 + K):
        kg_desc()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s); seal(); b.record(s)
        kg_open()
        c, d = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c.record(s); opn(); d.record(s)
        d.synchronize()
        if i >= 3:
            ts.append(a.elapsed_time(b)); to.append(c.elapsed_time(d))
    ts.sort(); to.sort()
    res["bench_order_seal"] = round(ts[len(ts) // 2], 4)
    res["bench_order_open"] = round(to[len(to) // 2], 4)
    # the same, but without host sync between steps (bench.py launches all steps async)
    ev = []
    for i in range(3 + K):
        kg_desc()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s); seal(); b.record(s)
        kg_open()
        c, d = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        c.record(s); opn(); d.record(s)
        if i >= 3:
            ev.append((a, b, c, d))
    torch.cuda.synchronize()
    ts = sorted(a.elapsed_time(b) for a, b, c, d in ev)
    to = sorted(c.elapsed_time(d) for a, b, c, d in ev)
    res["async_seal"] = round(ts[len(ts) // 2], 4)
    res["async_open"] = round(to[len(to) // 2], 4)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
