"""Split a rocprofv3 kernel-stats CSV of `bench.py --steps S --warmup W` into the kernels every
step launches (call count >= S + W: the graph-replayed step) and the set-up-only ones, with
each step kernel's time per step.  Flags rocPRIM / torch kernels in the step.

usage: python tools/step_kernels.py <kernel_stats.csv> <steps + warmup> <out.md> [title]
"""
import csv
import sys


def main() -> None:
    src, n, dst = sys.argv[1], int(sys.argv[2]), sys.argv[3]
    title = sys.argv[4] if len(sys.argv) > 4 else src
    rows = list(csv.DictReader(open(src)))
    step, setup = [], []
    for r in rows:
        calls = int(r["Calls"])
        avg_us = float(r["AverageNs"]) / 1e3
        name = r["Name"].replace("|", "/")
        name = name if len(name) <= 110 else name[:107] + "..."
        (step if calls >= n else setup).append((calls, avg_us, name))
    out = [f"# {title}", "", f"source: `{src}`; {n} timed + warm-up steps; a kernel launched >= {n} times is a "
           "step kernel", "", "## Step kernels", "", "| calls | per step | us per step | kernel |", "|---:|---:|---:|---|"]
    tot = 0.0
    for calls, avg, name in sorted(step, key=lambda x: -x[0] * x[1]):
        k = calls // n
        tot += k * avg
        out.append(f"| {calls} | {k} | {k * avg:.1f} | `{name}` |")
    lib = [nm for _, _, nm in step if "rocprim" in nm or "at::native" in nm or "at::cuda" in nm]
    out += ["", f"Step kernel time: {tot / 1e3:.3f} ms per step.  rocPRIM / PyTorch kernels in the step: "
            f"{len(lib)}" + (": " + ", ".join(f"`{x}`" for x in lib) if lib else " (none)"), "",
            "## Set-up only (operand generation, row plan of the eager reference product, graph warm-up)", "",
            "| calls | avg us | kernel |", "|---:|---:|---|"]
    for calls, avg, name in sorted(setup, key=lambda x: -x[0] * x[1])[:30]:
        out.append(f"| {calls} | {avg:.1f} | `{name}` |")
    with open(dst, "w") as f:
        f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
