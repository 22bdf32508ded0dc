"""Per-kernel duration summary (count, median, p10, p90 in us, grid, block) of a rocprofv3 --kernel-trace CSV.

  python tools/trace_summary.py run_kernel_trace.csv > summary.csv
"""
import collections
import csv
import statistics
import sys


def main(path):
    rows = list(csv.DictReader(open(path)))
    by = collections.OrderedDict()
    for r in sorted(rows, key=lambda r: int(r["Start_Timestamp"])):
        by.setdefault(r["Kernel_Name"], []).append(r)
    w = csv.writer(sys.stdout)
    w.writerow(["kernel", "count", "median_us", "p10_us", "p90_us", "grid", "block"])
    for k, rs in by.items():
        d = sorted((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3 for r in rs)
        w.writerow([k, len(d), round(statistics.median(d), 2), round(d[len(d) // 10], 2), round(d[9 * len(d) // 10], 2),
                    rs[0]["Grid_Size_X"], rs[0]["Workgroup_Size_X"]])


if __name__ == "__main__":
    main(sys.argv[1])
