"""Print the top kernels of a rocprofv3 run database (``-d DIR -o run`` -> run_results.db).

usage: python tools/prof_top.py <run_results.db> [tag] [n]
"""
import sqlite3
import sys


def main() -> None:
    db, tag = sys.argv[1], (sys.argv[2] if len(sys.argv) > 2 else "")
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    c = sqlite3.connect(db)
    for name, calls, tot in c.execute(f"select name, total_calls, total_duration from top_kernels limit {n}"):
        short = name.split("(")[0]
        short = short.split("::")[-1] if "::" in short else short
        print(f"{tag} {tot / 1e6 / calls:9.3f} ms x{calls:<4d} {tot / 1e6:9.2f} ms total  {short[:90]}")


if __name__ == "__main__":
    main()
