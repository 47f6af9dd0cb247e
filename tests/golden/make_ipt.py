#!/usr/bin/env python3
"""Generate tests/golden/ipt.npz -- Intel-PT path keys and set novelty computed by the
REFERENCE's own feeders (oracle/_ref ref_ipt_keys: linux_ipt_instrumentation.c
add_tnt_to_hash / add_tip_to_hash / finish_tnt_hash over its xxhash.c streaming XXH64) for
seeded synthetic event streams of TNT packets and TIP addresses (no IPT hardware here: the
packet parse stays on the host and is out of scope).  Covers short (<= 6 bits) and long (<= 47)
TNT packets, partial 8-bit words, execs without TIP / TNT, TIPs inside coverage libraries,
inside the target and elsewhere, and repeated execs (the set novelty: HASH_FIND / HASH_ADD,
:418-424, expected in exec order).

Run from the repository root (needs /root/reference):  python tests/golden/make_ipt.py
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
import oracle  # noqa: E402

LIBS = np.array([[0x7F0000000000, 0x7F0000080000, 0xDEADBEEF],
                 [0x7F1000000000, 0x7F1000200000, 0x1234]], np.uint64)
TARGET = (0x400000, 0x480000)


def events(rng, n_exec):
    ev, kinds = [], []
    for e in range(n_exec):
        if e > 3 and rng.random() < 0.25:  # repeat an earlier exec exactly
            src = kinds[int(rng.integers(0, len(kinds)))]
            ev.extend(src)
            kinds.append(src)
            continue
        cur = []
        for _ in range(int(rng.integers(0, 60))):
            r = rng.random()
            if r < 0.45:
                cur.append((0, int(rng.integers(0, 2**63)), int(rng.integers(1, 7))))
            elif r < 0.6:
                cur.append((0, int(rng.integers(0, 2**47)), int(rng.integers(1, 48))))
            else:
                where = rng.random()
                if where < 0.4:
                    tip = int(rng.integers(LIBS[0, 0], LIBS[0, 1]))
                elif where < 0.6:
                    tip = int(rng.integers(LIBS[1, 0], LIBS[1, 1]))
                elif where < 0.9:
                    tip = int(rng.integers(*TARGET))
                else:
                    tip = int(rng.integers(0, 2**63))
                cur.append((1, tip, 0))
        cur.append((2, 0, 0))
        ev.extend(cur)
        kinds.append(cur)
    return np.array(ev, np.uint64)


def main():
    oracle.build()
    rng = np.random.default_rng(0x1B7)
    out = {"libs": LIBS, "target": np.array(TARGET, np.uint64)}
    for tag, libs in (("libs", LIBS), ("nolibs", LIBS[:0])):
        ev = events(rng, 400)
        keys = oracle.ipt_keys(ev, libs[:, 0], libs[:, 1], libs[:, 2].astype(np.uint32),
                               *TARGET, use_ref=True)
        seen, isnew = set(), np.zeros(keys.shape[0], np.uint8)
        for j, k in enumerate(map(tuple, keys.tolist())):
            if k not in seen:
                seen.add(k)
                isnew[j] = 1
        out[f"{tag}_events"], out[f"{tag}_keys"], out[f"{tag}_isnew"] = ev, keys, isnew
        print(tag, keys.shape[0], "execs,", int(isnew.sum()), "new")
    np.savez_compressed(os.path.join(HERE, "ipt.npz"), **out)


if __name__ == "__main__":
    main()
