"""Kernels around the k-th dispatch of a kernel in a rocprofv3 kernel trace: start / end
(ms, relative), queue, stream, short name -- to see what a side-stream kernel ran beside.
usage: python tools/r6/timeline_window.py <kernel_trace.csv> <name> [k] [ms before] [ms after]"""
import csv
import sys


def main() -> None:
    path, name = sys.argv[1], sys.argv[2]
    k = int(sys.argv[3]) if len(sys.argv) > 3 else 10
    before = float(sys.argv[4]) if len(sys.argv) > 4 else 15.0
    after = float(sys.argv[5]) if len(sys.argv) > 5 else 15.0
    rows = []
    for r in csv.DictReader(open(path)):
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r.get("Queue_Id", "?"),
                     r.get("Stream_Id", "?"), r["Kernel_Name"]))
    rows.sort()
    hits = [x for x in rows if name in x[4]]
    if len(hits) <= k:
        print("not enough dispatches", len(hits))
        return
    t0 = hits[k][0]
    lo, hi = t0 - before * 1e6, hits[k][1] + after * 1e6
    for s, e, q, st, n in rows:
        if e >= lo and s <= hi:
            short = n.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][:60]
            print(f"{(s - t0) / 1e6:9.3f} {(e - t0) / 1e6:9.3f} q{q} s{st} {short}")


if __name__ == "__main__":
    main()
