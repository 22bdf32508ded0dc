"""Phase timeline of the fused float kernel (IBL_TRACE_FUSED dump, block 0's first group, diagnostic
build `tools/variants.py ftrace`): python tools/fused_trace_fl.py <file> [phase ...]
Per phase: duration to the barrier, and per wave (done clock - phase start, tasks taken); for the listed
phases also each wave's first task: body start (ticket + record taken) and body end, from the phase start.
Words per phase: kFlTraceWords (csrc/common.h)."""
import sys

import numpy as np

W = 65
t = np.fromfile(sys.argv[1], dtype=np.uint64).astype(np.int64).reshape(-1, W)
show = [int(x) for x in sys.argv[2:]]
ph = 0
while ph + 1 < len(t) and t[ph + 1, 0] > 0:
    start, end = t[ph, 0], t[ph + 1, 0]
    done = t[ph, 1:17] - start
    tasks = t[ph, 17:33]
    line = f"phase {ph:3d}: {end - start:7d} cycles; waves done min/med/max {done.min()}/{int(np.median(done))}/{done.max()}"
    if ph in show:
        b0 = np.where(tasks > 0, t[ph, 33:49] - start, -1)
        b1 = np.where(tasks > 0, t[ph, 49:65] - start, -1)
        line += "\n   done:tasks " + " ".join(f"{d}:{k}" for d, k in zip(done, tasks))
        line += "\n   first body start-end " + " ".join(f"{x}-{y}" for x, y in zip(b0, b1))
    print(line)
    ph += 1
