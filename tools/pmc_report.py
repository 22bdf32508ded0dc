"""Summaries of rocprofv3 --pmc passes (counter_collection CSVs) for profiles/.

  python tools/pmc_report.py sq  <out.json> <config> <csv> [<csv> ...]
      per-kernel averages of SQ_* / GRBM_* counters and derived shares (one JSON per config)
  python tools/pmc_report.py hbm <out.json> <config> <fetch.csv> <write.csv> [--merge]
      per-launch HBM bytes (FETCH_SIZE x2, WRITE_SIZE) against the stored algorithmic bytes; with
      --merge the result is merged into out.json (profiles/pmc_traffic.json, the file bench.py reads)

Units (MI355X_MICROARCH.md): GRBM_GUI_ACTIVE is summed over the 8 XCDs (per-XCD cycles = value / 8);
SQ_INSTS_* and SQ_LDS_* are chip totals (wave-instructions, LDS-array cycles); SQ_WAVE_CYCLES,
SQ_WAIT_* and SQ_ACTIVE_INST_* count quad-cycles summed over waves; a wave64 VALU instruction takes
2 issue cycles of its SIMD. FETCH_SIZE / WRITE_SIZE are KiB; gfx950's FETCH_SIZE tallies a 128-B
request at 64 B, so it is doubled (checked on ib_stage4's known byte count, round 2).
"""
import csv
import json
import sys
from collections import defaultdict

CUS, SIMDS, XCDS = 256, 1024, 8
# code sizes of the BASELINE configs: (E, N, batch, stored bytes per message, kind)
CONFIGS = {"C4": (226799, 64800, 8192, 0.5, "ib"), "C5": (226799, 64800, 8192, 4, "bp"),
           "C2": (24000, 8000, 65536, 0.5, "ib"), "C3": (6804, 1944, 262144, 4, "minsum")}


def _short(name):
    return name.replace("void ", "").split("(")[0]


def _read(paths):
    vals = defaultdict(lambda: defaultdict(list))
    for p in paths:
        with open(p) as fh:
            for r in csv.DictReader(fh):
                vals[_short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def sq(out, config, paths):
    doc = {"_note": "rocprofv3 --pmc SQ/GRBM counters, per-launch averages, bench.py --config %s --steps 1 "
                    "--warmup 0; derived: lds_busy = SQ_LDS_IDX_ACTIVE / CUs / (GRBM_GUI_ACTIVE / 8), "
                    "conflict_share = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE, valu_issue = 2 * SQ_INSTS_VALU / "
                    "SIMDs / (GRBM_GUI_ACTIVE / 8) (share of each SIMD's VALU issue cycles), valu_per_lds = "
                    "SQ_INSTS_VALU / SQ_INSTS_LDS; wait shares are of SQ_WAVE_CYCLES" % config, "kernels": {}}
    for k, c in _read(paths).items():
        if not k.startswith("ibl::"):
            continue
        avg = {n: sum(v) / len(v) for n, v in c.items()}
        row = {"launches": max(len(v) for v in c.values()), "counters": avg}
        g = avg.get
        cyc = g("GRBM_GUI_ACTIVE", 0) / XCDS
        d = {}
        if cyc and g("SQ_LDS_IDX_ACTIVE") is not None:
            d["lds_busy"] = g("SQ_LDS_IDX_ACTIVE") / CUS / cyc
        if g("SQ_LDS_IDX_ACTIVE"):
            d["conflict_share"] = g("SQ_LDS_BANK_CONFLICT", 0) / g("SQ_LDS_IDX_ACTIVE")
        if cyc and g("SQ_INSTS_VALU") is not None:
            d["valu_issue"] = 2 * g("SQ_INSTS_VALU") / SIMDS / cyc
        if g("SQ_INSTS_LDS"):
            d["valu_per_lds"] = g("SQ_INSTS_VALU", 0) / g("SQ_INSTS_LDS")
        if g("SQ_WAVE_CYCLES"):
            for n in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_WAIT_INST_LDS", "SQ_ACTIVE_INST_ANY",
                      "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS"):
                if g(n) is not None:
                    d[n.lower() + "_share"] = g(n) / g("SQ_WAVE_CYCLES")
        d["cycles_per_xcd"] = cyc
        row["derived"] = {a: round(b, 4) for a, b in d.items()}
        doc["kernels"][k] = row
        print(k, json.dumps(row["derived"]))
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)


# float per-pass degree-2 fold (round 5): folded variables and check passes per decode (imax - 1; all but
# the last fold) of the configs that run it
FOLD = {"C5": (32399, 99)}


def _alg(config, kname):
    """Stored algorithmic (read, write) bytes per launch of a per-pass kernel (averaged over the decode's
    launches: with the fold, all check passes but the last also read 2 channel rows per folded variable)."""
    E, N, B, w, _ = CONFIGS[config]
    nf, ncn = FOLD.get(config, (0, 1))
    base = kname.split("::")[-1].split("<")[0]
    if base in ("ib_cn_fast", "fl_cn", "ib_cn_gen"):
        return (E + 2 * nf * (ncn - 1) / ncn) * B * w, E * B * w
    if base in ("ib_vn_fast", "fl_vn", "ib_vn_gen"):
        return (E - 2 * nf + N - nf) * B * w, (E - 2 * nf) * B * w
    return None


def hbm(out, config, fetch, write, merge):
    E, N, B, w, kind = CONFIGS[config]
    f, wr = _read([fetch]), _read([write])
    res = {}
    for k in sorted(set(f) | set(wr)):
        if not k.startswith("ibl::"):
            continue
        fb = [x * 1024 for x in f.get(k, {}).get("FETCH_SIZE", [])]
        wb = [x * 1024 for x in wr.get(k, {}).get("WRITE_SIZE", [])]
        if not fb or not wb:
            continue
        fa, wa = 2 * sum(fb) / len(fb), sum(wb) / len(wb)
        row = {"batch": B, "format": {0.5: "u4", 1: "u8", 4: "f32", 8: "f64"}[w], "launches": len(fb),
               "fetch_bytes": int(round(fa)), "write_bytes": int(round(wa)), "hbm_bytes_per_launch": int(round(fa + wa))}
        a = _alg(config, k)
        if a:
            row.update(algorithmic_read=int(a[0]), algorithmic_write=int(a[1]),
                       fetch_over_alg=round(fa / a[0], 4), write_over_alg=round(wa / a[1], 4))
        key = k.split("::")[-1].split("<")[0]
        if key not in res or row["launches"] > res[key]["launches"]:   # the loop's instantiation, not pass 0's
            res[key] = row
        print(k, json.dumps(row))
    if merge:
        try:
            with open(out) as fh:
                doc = json.load(fh)
        except FileNotFoundError:
            doc = {}
    else:
        doc = {}
    doc.setdefault("_notes", {})[kind] = (
        "per-launch HBM bytes from rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes, bench.py --config %s "
        "--steps 1 --warmup 0), FETCH_SIZE x2 (gfx950 tallies a 128-B request at 64 B, MI355X_MICROARCH.md "
        "§HBM), KiB -> bytes; algorithmic = stored bytes of the pass (E, N rows x batch x bytes per message)" % config)
    doc[kind] = {**doc.get(kind, {}), **{k: v for k, v in res.items() if _alg(config, k)}}
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)


if __name__ == "__main__":
    mode, out, config = sys.argv[1], sys.argv[2], sys.argv[3]
    rest = [a for a in sys.argv[4:] if not a.startswith("--")]
    if mode == "sq":
        sq(out, config, rest)
    else:
        hbm(out, config, rest[0], rest[1], "--merge" in sys.argv)
