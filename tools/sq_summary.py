"""Per-kernel averages of SQ/GRBM counters from rocprofv3 --pmc runs (one or more counter_collection
CSVs), plus derived ratios: VALU / LDS instructions per wave-cycle, LDS busy share, issue stalls.
usage: python tools/sq_summary.py <csv> [<csv> ...] [--kernels ib_cn_fast,ib_vn_fast]"""
import csv
import sys
from collections import defaultdict

args = [a for a in sys.argv[1:] if not a.startswith("--")]
filt = None
for a in sys.argv[1:]:
    if a.startswith("--kernels="):
        filt = a.split("=", 1)[1].split(",")
vals = defaultdict(lambda: defaultdict(list))
for p in args:
    for r in csv.DictReader(open(p)):
        k = r["Kernel_Name"]
        if filt and not any(f in k for f in filt):
            continue
        k = k.replace("void ", "").split("(")[0]
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, c in vals.items():
    avg = {n: sum(v) / len(v) for n, v in c.items()}
    print(k, f"launches={max(len(v) for v in c.values())}")
    for n in sorted(avg):
        print(f"   {n:28s} {avg[n]:.4g}")
    g = lambda n: avg.get(n)
    if g("SQ_WAVE_CYCLES"):
        for n in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS", "SQ_WAIT_INST_LDS", "SQ_WAIT_ANY",
                  "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
            if g(n) is not None:
                print(f"   {n + '/WAVE_CYCLES':40s} {g(n) / g('SQ_WAVE_CYCLES'):.3f}")
    if g("SQ_BUSY_CYCLES") and g("SQ_INSTS_VALU"):
        print(f"   VALU insts per busy cycle per CU (x256 CUs)     {g('SQ_INSTS_VALU') / g('SQ_BUSY_CYCLES') / 256:.3f}")
    if g("SQ_LDS_IDX_ACTIVE") and g("GRBM_GUI_ACTIVE"):
        print(f"   LDS_IDX_ACTIVE / (GUI_ACTIVE*256)               {g('SQ_LDS_IDX_ACTIVE') / g('GRBM_GUI_ACTIVE') / 256:.3f}")
