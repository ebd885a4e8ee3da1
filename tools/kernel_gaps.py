#!/usr/bin/env python
"""Busy vs idle time of the GPU in a rocprofv3 kernel trace: over the last ``--window`` ms of the
trace (the steady decode), the union of kernel intervals against the wall span, the idle gaps
between consecutive kernels (histogram), and per-kernel-name time.  Shows whether a decode step
is bound by kernel durations or by the gaps between them (launch / dependency latency).

    python tools/kernel_gaps.py gpurun_out/.../kernel_trace.csv --window 50
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--window", type=float, default=50.0, help="ms at the end of the trace")
    ap.add_argument("--top", type=int, default=15)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    t_end = max(e for _, e, _ in ks)
    t0 = t_end - a.window * 1e6
    ks = [k for k in ks if k[0] >= t0]
    span = t_end - ks[0][0]
    busy, cur_s, cur_e = 0, None, None
    gaps = []
    for s, e, _ in ks:
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                gaps.append(s - cur_e)
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    busy += cur_e - cur_s
    per = collections.defaultdict(lambda: [0, 0])
    for s, e, n in ks:
        per[n][0] += 1
        per[n][1] += e - s
    print(f"kernels {len(ks)}  span {span / 1e6:.3f} ms  busy {busy / 1e6:.3f} ms ({100 * busy / span:.1f} %)  "
          f"idle {100 * (span - busy) / span:.1f} % in {len(gaps)} gaps")
    if gaps:
        gs = sorted(gaps)
        print("gap us: p10 %.2f p50 %.2f p90 %.2f max %.2f mean %.2f" % tuple(
            x / 1e3 for x in (gs[len(gs) // 10], gs[len(gs) // 2], gs[int(len(gs) * 0.9)], gs[-1], sum(gs) / len(gs))))
    for n, (c, t) in sorted(per.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f"{c:6d} {t / 1e6:8.3f} ms {t / c / 1e3:8.2f} us  {n[:100]}")


if __name__ == "__main__":
    main()
