"""Aggregate a rocprofv3 ``*_counter_collection.csv`` per kernel.

usage: python tools/pmc_summary.py <counter_collection.csv> [kernel-substring] [--md out.md]
Sums each counter over all dispatches of a kernel (kernels grouped by name);
prints one block per kernel with derived per-wave figures when SQ_WAVES is
present.
"""
import csv
import sys
from collections import defaultdict


def main() -> None:
    args = [a for a in sys.argv[1:]]
    md = None
    if "--md" in args:
        i = args.index("--md")
        md = args[i + 1]
        del args[i:i + 2]
    src = args[0]
    filt = args[1] if len(args) > 1 else ""
    agg = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    dur = defaultdict(dict)
    for r in csv.DictReader(open(src)):
        k = r["Kernel_Name"]
        if filt not in k:
            continue
        short = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0][-90:]
        agg[short][r["Counter_Name"]] += float(r["Counter_Value"])
        calls[short].add(r["Dispatch_Id"])
        dur[short][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    out = []
    for k, cs in sorted(agg.items(), key=lambda kv: -sum(dur[kv[0]].values())):
        ms = sum(dur[k].values()) / 1e6
        out.append(f"## `{k}`  ({len(calls[k])} dispatches, {ms:.2f} ms)")
        waves = cs.get("SQ_WAVES", 0)
        for name, v in sorted(cs.items()):
            extra = f"   ({v / waves:.1f} / wave)" if waves and name != "SQ_WAVES" else ""
            out.append(f"- {name}: {v:.4g}{extra}")
        out.append("")
    text = "\n".join(out)
    print(text)
    if md:
        with open(md, "w") as f:
            f.write(f"# PMC counters: `{src}`\n\n" + text + "\n")


if __name__ == "__main__":
    main()
