"""Phase timeline of the fused IB kernel (IBL_TRACE_FUSED dump of block 0's first group):
python tools/fused_trace.py <file> — prints per phase: work cycles, barrier+staging cycles."""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).astype(np.int64).reshape(-1, 3)
t0 = t[0, 0]
tot = {"work": 0, "drain": 0, "stage": 0}
for ph, (start, done, staged) in enumerate(t):
    if start == 0 and ph > 0:
        break
    nxt = t[ph + 1, 0] if ph + 1 < len(t) else 0
    work = done - start if done else 0
    stage = staged - done if staged else 0
    print(f"phase {ph:3d}: start {start - t0:9d}  tasks+drain {work:7d}  staging {stage:6d}")
    tot["work"] += max(work, 0)
    tot["stage"] += max(stage, 0)
print(tot)
