"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes per kernel (per-launch HBM bytes).

FETCH_SIZE / WRITE_SIZE are in KiB. Per MI355X_MICROARCH.md §HBM, gfx950's FETCH_SIZE counts
128-B requests at 64 B (half the bytes of a wide streaming read); this tool reports the raw value
and the x2-corrected one, and the ratio of each to the algorithmic bytes, so the correction can be
checked against the known byte count of the pass (calibration).
usage: python tools/pmc_summary.py <dir with pmc_FETCH_SIZE, pmc_WRITE_SIZE> [batch] [out.json] [u4|u8]
(u4 = the fast path's 4-bit messages, two codewords per byte; u8 = byte messages)
"""
import csv, json, os, sys
from collections import defaultdict

d = sys.argv[1]
B = int(sys.argv[2]) if len(sys.argv) > 2 else 8192
vals = defaultdict(lambda: defaultdict(list))
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    p = os.path.join(d, f"pmc_{c}", "run_counter_collection.csv")
    for r in csv.DictReader(open(p)):
        vals[r["Kernel_Name"].replace("void ", "").split("(")[0].split("<")[0]][c].append(float(r["Counter_Value"]) * 1024)
# DVB-S2 structured code: E and N for the algorithmic bytes
E, N = 226799, 64800
fmt = sys.argv[4] if len(sys.argv) > 4 else "u4"
bpm = 0.5 if fmt == "u4" else 1.0   # stored bytes per message
alg = {"ibl::ib_cn_fast": (E * B * bpm, E * B * bpm), "ibl::ib_vn_fast": ((E + N) * B * bpm, E * B * bpm)}
out = {}
for k, v in vals.items():
    if not k.startswith("ibl::"):
        continue
    f = sum(v["FETCH_SIZE"]) / max(len(v["FETCH_SIZE"]), 1)
    w = sum(v["WRITE_SIZE"]) / max(len(v["WRITE_SIZE"]), 1)
    row = {"format": fmt, "launches": len(v["FETCH_SIZE"]), "fetch_bytes_raw": f, "fetch_bytes_x2": 2 * f, "write_bytes": w}
    if k in alg:
        ar, aw = alg[k]
        row.update(alg_read=ar, alg_write=aw, fetch_raw_over_alg=f / ar, fetch_x2_over_alg=2 * f / ar,
                   write_over_alg=w / aw)
    out[k] = row
    print(k, json.dumps({a: (round(b, 3) if isinstance(b, float) else b) for a, b in row.items()}))
if len(sys.argv) > 3:
    json.dump(out, open(sys.argv[3], "w"), indent=1)
