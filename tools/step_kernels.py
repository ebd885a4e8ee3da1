#!/usr/bin/env python
"""The kernel sequence of the last decode step in a rocprofv3 kernel trace, as markdown: one row
per dispatch (duration, grid, name) from the step's first kernel to the end of the trace, and the
per-step total.  A step is cut at the last occurrence of ``--first`` (a substring of the name of
the step's first kernel) that still has ``--min-kernels`` dispatches after it.

    python tools/step_kernels.py gpurun_out/r4sb/prof/run_kernel_trace.csv --first w8a8_gemv_kernel<1, 3 \
        --min-kernels 150 "title" > profiles/x.md
"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("title")
    ap.add_argument("--first", required=True, help="substring of the step's first kernel name")
    ap.add_argument("--min-kernels", type=int, default=1)
    ap.add_argument("--steps-back", type=int, default=0, help="take the step this many steps before the last")
    a = ap.parse_args()
    rows = sorted(csv.DictReader(open(a.trace)), key=lambda r: int(r["Start_Timestamp"]))
    starts = [i for i, r in enumerate(rows) if a.first in r["Kernel_Name"]]
    # step boundaries: a start whose previous dispatch is not of the same step (layer 0 only)
    cand = [i for i in starts if len(rows) - i >= a.min_kernels]
    assert cand, "no step start found"
    i0 = cand[-1 - a.steps_back]
    step = rows[i0:]
    print(f"# {a.title}\n")
    print("| # | us | grid | kernel |\n|---|---|---|---|")
    tot = 0.0
    for n, r in enumerate(step):
        us = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000.0
        tot += us
        name = r["Kernel_Name"].replace("|", "\\|")[:100]
        print(f"| {n} | {us:.2f} | {r.get('Grid_Size_X', '')} | `{name}` |")
    wall = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1000.0
    print(f"\n{len(step)} dispatches; sum of durations {tot:.1f} us; first start to last end {wall:.1f} us.")


if __name__ == "__main__":
    main()
