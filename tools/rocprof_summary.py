#!/usr/bin/env python
"""Summarise a rocprofv3 ``--stats`` kernel table as markdown (top kernels by total time).

    python tools/rocprof_summary.py gpurun_out/prof/<host>/<pid>_kernel_stats.csv "title" > profiles/x.md
"""
import csv
import sys


def main():
    path, title = sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "rocprofv3 kernel stats"
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"# {title}\n")
    print("| kernel | calls | total ms | avg us | % |\n|---|---|---|---|---|")
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:top]:
        name = r["Name"].replace("|", "/")
        name = name if len(name) < 110 else name[:107] + "..."
        print(f"| `{name}` | {r['Calls']} | {float(r['TotalDurationNs']) / 1e6:.2f} | "
              f"{float(r['AverageNs']) / 1e3:.2f} | {100 * float(r['TotalDurationNs']) / tot:.2f} |")
    print(f"\nAll kernels: {tot / 1e6:.2f} ms device time.")


if __name__ == "__main__":
    main()
