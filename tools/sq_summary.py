#!/usr/bin/env python
"""Per-dispatch SQ counter summary of one kernel from rocprofv3 --pmc CSV directories.

    python tools/sq_summary.py <kernel substring> <pmc dir or counter csv> [...]

Prints each counter's mean over the kernel's dispatches (SQ cycle counters are in quad-cycles on
gfx950: x4 for cycles) and a few ratios: VALU / MFMA issue share of the waves' cycles, wait share."""
import csv, glob, os, sys
from collections import defaultdict

k = sys.argv[1]
tot, cnt = defaultdict(float), defaultdict(set)
for d in sys.argv[2:]:
    files = [d] if d.endswith(".csv") else glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            if k in r["Kernel_Name"]:
                tot[r["Counter_Name"]] += float(r["Counter_Value"])
                cnt[r["Counter_Name"]].add(r["Dispatch_Id"])
mean = {c: tot[c] / len(cnt[c]) for c in tot}
for c in sorted(mean):
    print(f"{c:28s} {mean[c]:.4g}")
g = mean.get
if g("SQ_WAVE_CYCLES") and g("SQ_WAVES"):
    wc = g("SQ_WAVE_CYCLES")
    for c in ("SQ_ACTIVE_INST_ANY", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_VALU", "SQ_WAIT_INST_LDS"):
        if g(c):
            print(f"{c} / SQ_WAVE_CYCLES = {g(c) / wc:.3f}")
if g("SQ_INSTS_VALU") and g("SQ_WAVES"):
    print(f"VALU instructions per wave {g('SQ_INSTS_VALU') / g('SQ_WAVES'):.0f}")
if g("SQ_INSTS_MFMA") and g("SQ_WAVES"):
    print(f"MFMA instructions per wave {g('SQ_INSTS_MFMA') / g('SQ_WAVES'):.0f}")
if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
    # GRBM_GUI_ACTIVE is summed over the 8 XCDs; the MFMA busy cycles are per-SIMD cycles summed
    # over the 1024 SIMDs (MI355X_MICROARCH.md): busy / (GRBM / 8 x 1024)
    print(f"MFMA pipe busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs) = "
          f"{g('SQ_VALU_MFMA_BUSY_CYCLES') / (g('GRBM_GUI_ACTIVE') / 8 * 1024):.3f}")
