"""Test-only code constructions shared by the GPU parity tests."""
import numpy as np


def mixed_code(cdegs, vdegs, n, seed):
    """Random irregular code whose check / variable degrees cover the given sets (every fast-path
    body, incl. the column-fetched inputs of degrees 5..8, and the MAXD=16 bodies). Socket matching;
    double edges are merged, a draw that leaves a check of degree < 2 is redrawn."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    for _ in range(100):
        vd = np.concatenate([vdegs, rng.choice(vdegs, n - len(vdegs))])
        E = int(vd.sum())
        m = max(int(round(E / np.mean(cdegs))), len(cdegs))   # check total reachable within the degree range
        cd = np.concatenate([cdegs, rng.choice(cdegs, m - len(cdegs))])
        while cd.sum() != E:   # move the check total onto E within [min, max] of cdegs
            i = int(rng.integers(len(cdegs), m))
            step = 1 if cd.sum() < E else -1
            if min(cdegs) <= cd[i] + step <= max(cdegs):
                cd[i] += step
        rows = rng.permutation(np.repeat(np.arange(m), cd))
        cols = np.repeat(np.arange(n), vd)
        H = sp.csr_matrix((np.ones(E, dtype=np.int64), (rows, cols)), shape=(m, n))
        H.data[:] = 1
        c = np.diff(H.indptr)
        v = np.bincount(H.indices, minlength=n)
        if c.min() >= 2 and v.min() >= 1 and c.max() <= 16 and v.max() <= 16:
            return H
    raise RuntimeError("no simple mixed code drawn")
