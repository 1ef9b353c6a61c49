#!/usr/bin/env python3
"""Lower bound on VALU ops per Salsa20 double round under gfx950's instruction set.

tools/gen_salsa_lazy.py picks one cheapest *cycle* of lazy sets for the rolled double-round loop
(82 ops).  This script asks the wider question: over any number of double rounds, from the
all-materialised state, with every schedule the op model allows (v_xad_u32 absorbing one pending
XOR into an add, v_bitop3 folding a pending XOR into an update, materialising either operand of a
doubly-lazy add, and -- beyond gen_salsa_lazy -- re-deferring an update of a lazy word), what is
the least total cost?  The dynamic program runs over all 2^16 lazy sets after every step.  The
per-double-round increment of the minimum converges to the steady-state bound.

    python tools/salsa_lazy_bound.py [double_rounds]
"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_salsa_lazy import DR  # noqa: E402  (the 32 steps of one double round)


def layer(cur):
    for (x, p, q, _) in DR:
        nxt = {}
        for m, c in cur.items():
            lp, lq = (m >> p) & 1, (m >> q) & 1
            adds = [(m & ~(1 << p), 2), (m & ~(1 << q), 2)] if (lp and lq) else [(m, 1)]
            for m2, ca in adds:
                ca += 1  # v_alignbit rotate
                if (m2 >> x) & 1:
                    outs = [(m2 & ~(1 << x), 1), (m2, 1)]  # bitop3 -> materialised, or re-deferred
                else:
                    outs = [(m2 | (1 << x), 0), (m2, 1)]  # defer (0 ops) or xor now
                for m3, cu in outs:
                    t = c + ca + cu
                    if nxt.get(m3, 1 << 30) > t:
                        nxt[m3] = t
        cur = nxt
    return cur


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    cur, prev, rows = {0: 0}, 0, []
    for k in range(1, n + 1):
        cur = layer(cur)
        mn = min(cur.values())  # leaving the loop costs nothing: the feed-forward absorbs a lazy word
        rows.append({"double_rounds": k, "min_total_ops": mn, "increment": mn - prev, "states": len(cur)})
        prev = mn
    print(json.dumps({"plain_ops_per_double_round": 96, "rows": rows}, indent=1))


if __name__ == "__main__":
    main()
