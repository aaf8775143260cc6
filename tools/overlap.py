"""Concurrency of a rocprofv3 kernel trace: for every kernel name matching a
filter, its summed duration and how much of it ran while some OTHER kernel
(any stream) was also running; plus the trace's busy union and span.

usage: python tools/overlap.py <kernel_trace.csv> [name filter ...]
"""
import csv
import sys
from collections import defaultdict


def main() -> None:
    path = sys.argv[1]
    filters = sys.argv[2:] or [""]
    iv = []
    for r in csv.DictReader(open(path)):
        iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    iv.sort()
    # sweep: coverage count over time
    ev = []
    for s, e, _ in iv:
        ev.append((s, 1))
        ev.append((e, -1))
    ev.sort()
    cover = []   # (t0, t1, active)
    act, last = 0, None
    for t, d in ev:
        if last is not None and t > last:
            cover.append((last, t, act))
        act += d
        last = t
    busy = sum(t1 - t0 for t0, t1, a in cover if a > 0)
    multi = sum(t1 - t0 for t0, t1, a in cover if a > 1)
    span = iv[-1][1] - iv[0][0] if iv else 0
    print(f"kernels {len(iv)}  span {span / 1e6:.1f} ms  busy {busy / 1e6:.1f} ms  "
          f">=2 kernels {multi / 1e6:.1f} ms  summed {sum(e - s for s, e, _ in iv) / 1e6:.1f} ms")
    import bisect
    starts = [c[0] for c in cover]
    for f in filters:
        tot, ovl, n = 0, 0, 0
        by = defaultdict(int)
        for s, e, name in iv:
            if f not in name:
                continue
            n += 1
            tot += e - s
            i = max(bisect.bisect_right(starts, s) - 1, 0)
            while i < len(cover) and cover[i][0] < e:
                t0, t1, a = cover[i]
                lo, hi = max(t0, s), min(t1, e)
                if hi > lo and a > 1:
                    ovl += hi - lo
                i += 1
            by[name.split("(")[0][-40:]] += e - s
        print(f"[{f or '*'}] calls {n}  total {tot / 1e6:.1f} ms  overlapped {ovl / 1e6:.1f} ms "
              f"({100 * ovl / max(tot, 1):.0f} %)")


if __name__ == "__main__":
    main()
