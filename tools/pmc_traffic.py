"""Write profiles/pmc_traffic.json (the per-launch HBM bytes bench.py reports as roofline.traffic) from a
tools/pmc_summary.py output: python tools/pmc_traffic.py <pmc_summary.json> <batch> <source note> [out]"""
import json
import sys

src, batch, note = sys.argv[1], int(sys.argv[2]), sys.argv[3]
out = sys.argv[4] if len(sys.argv) > 4 else "profiles/pmc_traffic.json"
s = json.load(open(src))
ib = {}
for k in ("ib_cn_fast", "ib_vn_fast"):
    e = s["ibl::" + k]
    ib[k] = {"batch": batch, "hbm_bytes_per_launch": int(round(e["fetch_bytes_x2"] + e["write_bytes"])),
             "fetch_bytes": int(round(e["fetch_bytes_x2"])), "write_bytes": int(round(e["write_bytes"])),
             "format": e["format"], "algorithmic_read": int(e["alg_read"]), "algorithmic_write": int(e["alg_write"])}
doc = {"_note": "per-launch HBM bytes from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes), FETCH_SIZE x2 "
                "(gfx950: a 128-B request is tallied at 64 B, MI355X_MICROARCH.md §HBM; checked on ib_stage4's known "
                "byte count), KiB->bytes; DVB-S2 N=64800, B=%d, i_max=50, 4-bit fast path (format u4: 2 codewords "
                "per byte); source %s" % (batch, note),
       "ib": ib}
json.dump(doc, open(out, "w"), indent=1)
print(json.dumps(ib, indent=1))
