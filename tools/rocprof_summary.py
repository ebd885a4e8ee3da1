#!/usr/bin/env python
"""Summarise a rocprofv3 ``--stats`` kernel table as markdown (top kernels by total time).

    python tools/rocprof_summary.py gpurun_out/prof/<host>/<pid>_kernel_stats.csv "title" > profiles/x.md
    python tools/rocprof_summary.py gpurun_out/prof/<name>_results.db "title" > profiles/x.md

Accepts the CSV stats table (``--output-format csv``) or the rocpd SQLite database that
rocprofv3 (ROCm 7) writes by default; ``--csv out.csv`` also dumps the full per-kernel table.
"""
import csv
import sqlite3
import sys


def _rows_db(path):
    c = sqlite3.connect(path)
    q = ("select name, count(*), sum(duration), avg(duration), max(grid_x), max(workgroup_x), max(vgpr_count), "
         "max(accum_vgpr_count), max(lds_size) from kernels group by name")
    out = []
    for name, calls, tot, avg, gx, wx, vg, ag, lds in c.execute(q):
        out.append({"Name": name, "Calls": calls, "TotalDurationNs": tot, "AverageNs": avg,
                    "Grid": gx, "WG": wx, "VGPR": vg, "AGPR": ag, "LDS": lds})
    return out


def main():
    args = [a for a in sys.argv[1:]]
    dump = None
    if "--csv" in args:
        i = args.index("--csv")
        dump = args[i + 1]
        del args[i:i + 2]
    path, title = args[0], args[1] if len(args) > 1 else "rocprofv3 kernel stats"
    top = int(args[2]) if len(args) > 2 else 25
    rows = _rows_db(path) if path.endswith(".db") else list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    if dump:
        with open(dump, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
                w.writerow(r)
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
