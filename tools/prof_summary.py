"""Condense a rocprofv3 ``*_kernel_stats.csv`` into a markdown table.

usage: python tools/prof_summary.py <kernel_stats.csv> <out.md> [title]
"""
import csv
import sys


def main() -> None:
    src, dst = sys.argv[1], sys.argv[2]
    title = sys.argv[3] if len(sys.argv) > 3 else src
    rows = list(csv.DictReader(open(src)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [f"# {title}", "", f"source: `{src}` (rocprofv3 --kernel-trace --stats)", "",
           f"total GPU kernel time: {tot / 1e6:.2f} ms", "",
           "| % | calls | total ms | avg us | kernel |", "|---:|---:|---:|---:|---|"]
    for r in rows[:25]:
        name = r["Name"].replace("|", "/")
        if len(name) > 110:
            name = name[:107] + "..."
        out.append(f"| {float(r['Percentage']):.2f} | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.3f} | "
                   f"{float(r['AverageNs']) / 1e3:.1f} | `{name}` |")
    with open(dst, "w") as f:
        f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
