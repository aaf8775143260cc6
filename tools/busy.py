"""GPU busy fraction from a rocprofv3 kernel trace: union of kernel intervals
vs the span from the first kernel start to the last kernel end, overall and
over the last ``--tail`` seconds of the trace (the timed steps of a bench run).
usage: python tools/busy.py <kernel_trace.csv> [--tail SECONDS]"""
import csv
import sys


def main() -> None:
    path = sys.argv[1]
    tail = float(sys.argv[sys.argv.index("--tail") + 1]) if "--tail" in sys.argv else None
    iv = []
    with open(path) as f:
        for r in csv.DictReader(f):
            iv.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    iv.sort()
    t_end = max(e for _, e in iv)
    lo = t_end - int(tail * 1e9) if tail else iv[0][0]
    busy, cur_s, cur_e, gaps = 0, None, None, []
    for s, e in iv:
        if e <= lo:
            continue
        s = max(s, lo)
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    span = t_end - lo
    gaps.sort(reverse=True)
    print(f"span {span / 1e9:.3f} s, kernels busy {busy / 1e9:.3f} s ({100 * busy / span:.1f} %), "
          f"{len(gaps)} gaps, largest {[round(g / 1e6, 2) for g in gaps[:8]]} ms, "
          f"gaps > 1 ms total {sum(g for g in gaps if g > 1e6) / 1e9:.3f} s")


if __name__ == "__main__":
    main()
