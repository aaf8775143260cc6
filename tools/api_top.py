"""Summarise a rocprofv3 HIP API trace (``--hip-runtime-trace --output-format csv``):
total and maximum time per API function, and the longest individual calls.

usage: python tools/api_top.py <hip_api_trace.csv> [n]
"""
import collections
import csv
import sys


def main() -> None:
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 12
    tot = collections.defaultdict(float)
    cnt = collections.Counter()
    mx = collections.defaultdict(float)
    longest = []
    for r in csv.DictReader(open(sys.argv[1])):
        name = r.get("Function") or r.get("Operation") or r.get("Name")
        d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
        tot[name] += d
        cnt[name] += 1
        mx[name] = max(mx[name], d)
        longest.append((d, name, r.get("Thread_Id", "")))
    print(f"{'api':40s} {'calls':>7s} {'total ms':>10s} {'max ms':>9s}")
    for name, t in sorted(tot.items(), key=lambda x: -x[1])[:n]:
        print(f"{name[:40]:40s} {cnt[name]:7d} {t:10.2f} {mx[name]:9.2f}")
    print("longest calls:")
    for d, name, tid in sorted(longest, reverse=True)[:n]:
        print(f"  {d:9.2f} ms  {name}  thread {tid}")


if __name__ == "__main__":
    main()
