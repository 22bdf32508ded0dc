import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); runs the HIP kernels")


@pytest.fixture(scope="session")
def golden():
    return np.load(os.path.join(GOLDEN, "reference_host.npz"), allow_pickle=False)


@pytest.fixture(scope="session")
def wlan_H():
    import scipy.sparse as sp
    z = np.load(os.path.join(GOLDEN, "wlan_H.npz"), allow_pickle=False)
    return sp.csr_matrix((np.ones(z["indices"].size, dtype=np.int64), z["indices"], z["indptr"]),
                         shape=tuple(z["shape"]))


@pytest.fixture(scope="session")
def reg_H(golden):
    import scipy.sparse as sp
    z = golden
    return sp.csr_matrix((np.ones(z["reg_H_indices"].size, dtype=np.int64), z["reg_H_indices"], z["reg_H_indptr"]),
                         shape=tuple(z["reg_H_shape"]))


@pytest.fixture(scope="session")
def dvb_H():
    from informationbottleneckdecodingldpc_amd import codes
    return codes.dvbs2_structured(seed=0)
