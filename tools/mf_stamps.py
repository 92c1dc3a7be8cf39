#!/usr/bin/env python3
"""Per-level phase times of the multifrontal factorization from a BOS_MF_STAMPS dump (diagnostics).
Phases per front: start -> assembled -> folded landmarks eliminated -> children extend-added ->
factored -> panel / update written and forward step done. Times in us (100 MHz clock)."""
import sys

import numpy as np

raw = open(sys.argv[1], "rb").read()
n = int(np.frombuffer(raw[:8], dtype=np.int64)[0])
meta = np.frombuffer(raw[8:8 + 16 * n], dtype=np.int32).reshape(n, 4)
st = np.frombuffer(raw[8 + 16 * n:], dtype=np.uint64).reshape(n, 8).astype(np.int64)
ok = (st[:, 0] > 0) & (st[:, 5] > 0)
t0 = st[ok, 0].min()
print(f"supernodes {n}, stamped {ok.sum()}, factorization span {(st[ok, 5].max() - t0) / 100:.1f} us")
names = ["assemble", "fold", "extend", "factor", "write+fwd"]
print(f"{'lvl':>3} {'fronts':>6} {'k':>4} {'r':>4} {'fold':>4} {'start':>7} {'end':>7} " + " ".join(f"{x:>9}" for x in names))
for lev in range(meta[:, 0].max() + 1):
    sel = ok & (meta[:, 0] == lev)
    if not sel.any():
        continue
    S = st[sel]
    d = np.diff(S[:, :6], axis=1) / 100.0
    med = np.median(d, axis=0)
    print(f"{lev:3d} {sel.sum():6d} {np.median(meta[sel, 1]):4.0f} {np.median(meta[sel, 2]):4.0f} "
          f"{np.median(meta[sel, 3]):4.0f} {(S[:, 0].min() - t0) / 100:7.1f} {(S[:, 5].max() - t0) / 100:7.1f} "
          + " ".join(f"{v:9.2f}" for v in med))

fold = ok & (meta[:, 3] > 0)
if fold.any():
    print(f"folded fronts {fold.sum()}: median per front: row phase {np.median(st[fold, 6]) / 100:.2f} us, "
          f"extend-add phase {np.median(st[fold, 7]) / 100:.2f} us, landmarks {np.median(meta[fold, 3]):.0f}")
