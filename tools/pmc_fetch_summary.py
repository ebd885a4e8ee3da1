#!/usr/bin/env python
"""Per-kernel FETCH_SIZE (HBM read traffic from rocprofv3 --pmc FETCH_SIZE) for the decode kernels
of a bench run: mean per dispatch, x2 for the gfx950 half-count of wide streaming reads
(MI355X_MICROARCH.md: FETCH_SIZE reports exactly 1/2 of a wide coalesced read), and per decode
step (dispatches per step = layers).  Markdown to stdout.

    python tools/pmc_fetch_summary.py run_counter_collection.csv "title" [layers=32] [min_calls=64]
"""
import csv
import sys
from collections import defaultdict


def main():
    path, title = sys.argv[1], sys.argv[2]
    layers = int(sys.argv[3]) if len(sys.argv) > 3 else 32
    min_calls = int(sys.argv[4]) if len(sys.argv) > 4 else 64
    acc = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != "FETCH_SIZE":
            continue
        acc[(r["Kernel_Name"], int(r["Grid_Size"]), int(r["Workgroup_Size"]))].append(float(r["Counter_Value"]))
    print(f"# {title}\n")
    print("| kernel | grid | WG | calls | FETCH_SIZE MB / call | x2 (wide-read half count) MB | per step (x{}) GB |".format(layers))
    print("|---|---|---|---|---|---|---|")
    tot = 0.0
    rows = []
    for (name, grid, wg), v in acc.items():
        if len(v) < min_calls:
            continue
        mb = sum(v) / len(v) / 1024.0            # FETCH_SIZE is in KB
        rows.append((mb * layers, name, grid, wg, len(v), mb))
    for step_mb, name, grid, wg, n, mb in sorted(rows, reverse=True):
        short = name.replace("|", "/")
        short = short if len(short) < 100 else short[:97] + "..."
        print(f"| `{short}` | {grid} | {wg} | {n} | {mb:.1f} | {2 * mb:.1f} | {2 * step_mb / 1024:.2f} |")
        if "ring2" in name or "gemv" in name or "gemm" in name:
            tot += 2 * step_mb / 1024
    print(f"\nDecode GEMM kernels: {tot:.2f} GB per step (x2-corrected FETCH_SIZE, {layers} dispatches per step each).")


if __name__ == "__main__":
    main()
