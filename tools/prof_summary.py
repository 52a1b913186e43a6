"""Summarise a rocprofv3 --kernel-trace run (rocpd SQLite db or kernel_stats.csv) as markdown.

Usage: python tools/prof_summary.py <run_results.db | kernel_stats.csv> [title] > profiles/<name>.md
"""
import csv
import sqlite3
import sys


def rows_from_db(path):
    c = sqlite3.connect(path)
    q = ("select name, count(*), sum(end-start), avg(end-start), min(end-start), max(end-start) "
         "from kernels group by name order by 3 desc")
    return [(r[0], r[1], r[2], r[3], r[4], r[5]) for r in c.execute(q)]


def rows_from_csv(path):
    out = []
    with open(path) as f:
        for r in csv.DictReader(f):
            out.append((r["Name"], int(r["Calls"]), float(r["TotalDurationNs"]), float(r["AverageNs"]),
                        float(r["MinNs"]), float(r["MaxNs"])))
    return sorted(out, key=lambda r: -r[2])


def main():
    path = sys.argv[1]
    title = sys.argv[2] if len(sys.argv) > 2 else path
    rows = rows_from_db(path) if path.endswith(".db") else rows_from_csv(path)
    tot = sum(r[2] for r in rows)
    print(f"# {title}\n")
    print("| kernel | calls | total ms | % | avg us | min us | max us |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for name, n, s, a, mn, mx in rows:
        short = name.replace("(anonymous namespace)::", "")
        if short.startswith("void "):
            short = short[5:]
        short = short.split("(")[0]
        print(f"| `{short}` | {n} | {s / 1e6:.3f} | {100 * s / tot:.1f} | {a / 1e3:.2f} | {mn / 1e3:.2f} | {mx / 1e3:.2f} |")


if __name__ == "__main__":
    main()
