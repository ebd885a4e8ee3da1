#!/usr/bin/env python
"""Per-kernel mean of every PMC counter in one or more rocprofv3 counter_collection.csv files
(one pass each), plus derived ratios when their inputs are present.  Markdown to stdout.

    python tools/pmc_summary.py "title" pass1/run_counter_collection.csv pass2/... [--min-calls 8]

Derived (per dispatch, SQ_* counters are summed over the chip; WAVE/WAIT counters in quad-cycles):
  wait_frac = SQ_WAIT_ANY / SQ_WAVE_CYCLES         (waves parked on s_waitcnt / s_barrier)
  issue_stall_frac = SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  mfma_util = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024)   (1024 SIMDs, GUI summed over 8 XCDs)
  lds_conflict = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
"""
import csv
import sys
from collections import defaultdict


def main():
    args = [a for a in sys.argv[1:]]
    min_calls = 8
    if "--min-calls" in args:
        i = args.index("--min-calls")
        min_calls = int(args[i + 1])
        del args[i:i + 2]
    title, paths = args[0], args[1:]
    acc = defaultdict(lambda: defaultdict(list))
    for p in paths:
        for r in csv.DictReader(open(p)):
            key = r["Kernel_Name"]
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f"# {title}\n")
    for name, cs in acc.items():
        n = max(len(v) for v in cs.values())
        if n < min_calls:
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        short = name if len(name) < 140 else name[:137] + "..."
        print(f"## `{short}` ({n} dispatches)\n")
        print("| counter | mean per dispatch |")
        print("|---|---|")
        for c in sorted(m):
            print(f"| {c} | {m[c]:.4g} |")
        d = {}
        if "SQ_WAIT_ANY" in m and m.get("SQ_WAVE_CYCLES"):
            d["wait_frac"] = m["SQ_WAIT_ANY"] / m["SQ_WAVE_CYCLES"]
        if "SQ_WAIT_INST_ANY" in m and m.get("SQ_WAVE_CYCLES"):
            d["issue_stall_frac"] = m["SQ_WAIT_INST_ANY"] / m["SQ_WAVE_CYCLES"]
        if "SQ_ACTIVE_INST_ANY" in m and m.get("SQ_WAVE_CYCLES"):
            d["active_frac"] = m["SQ_ACTIVE_INST_ANY"] / m["SQ_WAVE_CYCLES"]
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and m.get("GRBM_GUI_ACTIVE"):
            d["mfma_util"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["GRBM_GUI_ACTIVE"] / 8 * 1024)
        if "SQ_LDS_BANK_CONFLICT" in m and m.get("SQ_LDS_IDX_ACTIVE"):
            d["lds_conflict"] = m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"]
        if m.get("GRBM_GUI_ACTIVE"):
            d["gui_cycles_per_xcd"] = m["GRBM_GUI_ACTIVE"] / 8
        if "TA_BUSY_avr" in m and m.get("GRBM_GUI_ACTIVE"):
            # the average TA (one per CU) busy over the dispatch's GUI-active cycles
            d["ta_busy_frac"] = m["TA_BUSY_avr"] / (m["GRBM_GUI_ACTIVE"] / 8)
        if "FETCH_SIZE" in m:
            # FETCH_SIZE (KB) counts half the bytes of wide streaming reads on gfx950: x2
            d["fetch_MB_x2"] = 2 * m["FETCH_SIZE"] / 1024
        if d:
            print("\n" + ", ".join(f"{k} = {v:.3g}" for k, v in d.items()))
        print()


if __name__ == "__main__":
    main()
