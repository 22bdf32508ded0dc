"""Phase timeline of the fused float kernel (IBL_TRACE_FUSED dump, block 0's first group):
python tools/fused_trace_fl.py <file>: per phase, thread 0's wave done and all waves done (cycles)."""
import sys

import numpy as np

t = np.fromfile(sys.argv[1], dtype=np.uint64).astype(np.int64)
t0 = t[0]
ph = 0
while 2 * ph + 2 < len(t) and t[2 * ph + 2] > 0:
    start = t[2 * ph]
    print(f"phase {ph:3d}: start {start - t0:9d} wave0 {t[2 * ph + 1] - start:7d} all {t[2 * ph + 2] - start:7d}")
    ph += 1
