"""Inter-CU balance of one traced fast-path launch (IBL_TRACE_WAVES=<prefix> -> <prefix>_{vn,cn}.bin).

Each wave wrote {start clock, end clock, items | hw_id << 32} (uint64 triples, s_memtime ticks). Waves
are grouped by their block (waves_per_block consecutive triples); the block's span is its first start to
its last end. Clocks are compared only within one XCD (blocks are dealt to XCDs round-robin: block b
runs on XCD b % 8), since each XCD has its own counter.
usage: python tools/wave_balance.py <prefix> [waves_per_block=16]
"""
import sys

import numpy as np


def report(path, wpb):
    t = np.fromfile(path, dtype=np.uint64).reshape(-1, 3)
    st, en = t[:, 0].astype(np.int64), t[:, 1].astype(np.int64)
    items = (t[:, 2] & 0xffffffff).astype(np.int64)
    nb = len(t) // wpb
    st, en, items = st[:nb * wpb].reshape(nb, wpb), en[:nb * wpb].reshape(nb, wpb), items[:nb * wpb].reshape(nb, wpb)
    bst, ben = st.min(1), en.max(1)
    print(f"{path}: {nb} blocks x {wpb} waves, items per block {items.sum(1).min()}..{items.sum(1).max()}")
    idle = []
    for x in range(8):
        sel = np.arange(x, nb, 8)
        t0 = bst[sel].min()
        span = ben[sel].max() - t0
        ends = ben[sel] - t0
        starts = bst[sel] - t0
        # fraction of the XCD's launch span a block sits idle after it finished (tail) or before it started
        idle.append(((span - ends) + starts).mean() / span)
        print(f"  xcd {x}: span {span} ticks, block end min/med/max {ends.min()}/{int(np.median(ends))}/{ends.max()},"
              f" start max {starts.max()}, mean idle {idle[-1]:.3f}")
    wend = en - st.min(1, keepdims=True)
    print(f"  in-block: last wave end / first wave end (median over blocks) "
          f"{np.median(wend.max(1) / np.maximum(wend.min(1), 1)):.3f}; mean idle fraction over XCDs {np.mean(idle):.3f}")


if __name__ == "__main__":
    pre = sys.argv[1]
    wpb = int(sys.argv[2]) if len(sys.argv) > 2 else 16
    for k in ("cn", "vn"):
        report(f"{pre}_{k}.bin", wpb)
