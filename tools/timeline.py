"""Analyses a wave timeline saved by `bench.py --timeline PATH` (option
"timeline", ssa_amd_get_timeline): when the DP waves of one search ran, where,
and what the launch's tail is made of.

usage: python tools/timeline.py PATH.npy
Rows: (group | 0x80000000 + lane for long_kernel, start, end, place), ticks of
the 100 MHz s_memrealtime clock; place = XCC << 16 | HW_ID[15:0].  With strip
parts (option "pair_parts", auto for queries of >= 4 strips) a pair group's row
is its LAST part's workgroup: start is when that part began (after the group's
earlier parts), so pair "starts" late in the span -- use option pair_parts=1 to
see whole groups."""
import sys

import numpy as np


def main(path):
    t = np.load(path).astype(np.int64)
    t = t[(t[:, 1] != 0) | (t[:, 2] != 0)]
    is_long = (t[:, 0] & 0x80000000) != 0
    t0 = t[:, 1].min()
    st = (t[:, 1] - t0) / 100.0          # microseconds
    en = (t[:, 2] - t0) / 100.0
    du = en - st
    span = en.max()
    print(f"rows {len(t)}: pair waves {int((~is_long).sum())}, long entries {int(is_long.sum())}; span {span:.0f} us")
    for name, sel in (("pair", ~is_long), ("long", is_long)):
        if sel.any():
            print(f"  {name}: start {st[sel].min():.0f}-{st[sel].max():.0f} us, end {en[sel].min():.0f}-"
                  f"{en[sel].max():.0f} us, duration median {np.median(du[sel]):.0f} max {du[sel].max():.0f} us")
    place = t[:, 3]
    simd = ((place >> 16) << 12) | (((place >> 13) & 7) << 9) | (((place >> 12) & 1) << 8) \
        | (((place >> 8) & 15) << 4) | ((place >> 4) & 3)
    u, inv = np.unique(simd, return_inverse=True)
    last = np.zeros(len(u))
    busy = np.zeros(len(u))
    np.maximum.at(last, inv, en)
    np.add.at(busy, inv, du)
    print(f"SIMDs seen {len(u)}; last wave end per SIMD: min {last.min():.0f} median {np.median(last):.0f} "
          f"max {last.max():.0f} us")
    # resident pair waves per CU: the maximum over the launch of waves that
    # overlap in time on one CU (4 per workgroup: the occupancy the LDS and
    # registers actually allowed)
    cu = simd >> 4
    pr0 = ~is_long
    ucu, cinv = np.unique(cu[pr0], return_inverse=True)
    peak = np.zeros(len(ucu), dtype=np.int64)
    ev_t = np.concatenate([st[pr0], en[pr0]])
    ev_d = np.concatenate([np.ones(pr0.sum(), np.int64), -np.ones(pr0.sum(), np.int64)])
    ev_c = np.concatenate([cinv, cinv])
    o = np.lexsort((ev_d, ev_t))            # ends before starts at equal times
    cur = np.zeros(len(ucu), dtype=np.int64)
    for c, d in zip(ev_c[o], ev_d[o]):
        cur[c] += d
        if cur[c] > peak[c]:
            peak[c] = cur[c]
    vals, cnts = np.unique(peak, return_counts=True)
    print("peak resident pair waves per CU (waves: CUs):", dict(zip(vals.tolist(), cnts.tolist())))
    # active pair waves over time (1 % bins of the span)
    edges = np.linspace(0, span, 101)
    act = [int(((st < b) & (en > a) & ~is_long).sum()) for a, b in zip(edges[:-1], edges[1:])]
    actl = [int(((st < b) & (en > a) & is_long).sum()) for a, b in zip(edges[:-1], edges[1:])]
    print("active pair waves per 10 % of the span:", [max(act[i:i + 10]) for i in range(0, 100, 10)])
    print("active long entries per 10 % of the span:", [max(actl[i:i + 10]) for i in range(0, 100, 10)])
    order = np.argsort(-en)[:12]
    print("last to finish: kind group/lane start end duration (us)")
    for i in order:
        kind = "long" if is_long[i] else "pair"
        print(f"  {kind} {int(t[i, 0] & 0x7fffffff):7d} {st[i]:8.0f} {en[i]:8.0f} {du[i]:8.0f}")
    pr = ~is_long
    if pr.any():
        g = t[pr, 0]
        k = np.argsort(g)
        gd = du[pr][k]
        print("pair wave duration by group rank (longest groups first):")
        for q in (0, 64, 256, 1024, 2048, 4096, len(gd) - 1):
            if q < len(gd):
                print(f"  group #{q}: {gd[q]:.0f} us (start {st[pr][k][q]:.0f})")


if __name__ == "__main__":
    main(sys.argv[1])
