"""GPU busy time of a rocprofv3 kernel trace: the union of kernel intervals
(overlapping kernels on several streams counted once), optionally for kernels
whose name contains a filter, plus their summed durations.

usage: python tools/busy_union.py <kernel_trace.csv> [name filter]
"""
import csv
import sys


def main() -> None:
    path = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    iv = []
    for r in csv.DictReader(open(path)):
        if filt in r["Kernel_Name"]:
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    iv.sort()
    busy, cur_s, cur_e, total = 0, None, None, 0
    for s, e in iv:
        total += e - s
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        busy += cur_e - cur_s
    span = (iv[-1][1] - iv[0][0]) if iv else 0
    print(f"kernels={len(iv)} filter={filt!r} busy_s={busy / 1e9:.4f} summed_s={total / 1e9:.4f} span_s={span / 1e9:.4f}")


if __name__ == "__main__":
    main()
