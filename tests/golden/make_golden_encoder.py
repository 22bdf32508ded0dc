"""Golden vectors for the LDPC encoder, from the REFERENCE (build container only).

Usage:  python tests/golden/make_golden_encoder.py [/root/reference]

Imports the reference's Discrete_LDPC_decoding/LDPC_encoder.py (np.int restored, GPU-only imports
stubbed as in make_golden.py, the uncompiled Cython helper stubbed — `encode` does not use it), builds its LDPCEncoder from each test code saved as a sparse .npz in a
temp directory, and runs its `encode` (:86-123) on seeded random information words (with the
numpy-1 integer promotion its substitution loop relies on, see below). Stores the info
bits, the reference codewords and the encoding algorithm the reference picked
(getLDPCEncoderParamters :197-269). No reference source is copied.
Output: tests/golden/reference_encoder.npz
"""
from __future__ import annotations

import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True

import make_golden  # noqa: E402

from informationbottleneckdecodingldpc_amd import codes  # noqa: E402


def main():
    make_golden._stub_reference_imports()
    import types
    # the Cython helper (GF2MatrixMul_c.pyx) is not compiled here; only encode_c uses it, encode
    # (the method this script runs) uses the pure-Python GF2MatrixMul
    import Discrete_LDPC_decoding
    stub = types.ModuleType("Discrete_LDPC_decoding.GF2MatrixMul_c")
    sys.modules["Discrete_LDPC_decoding.GF2MatrixMul_c"] = stub
    Discrete_LDPC_decoding.GF2MatrixMul_c = stub
    from Discrete_LDPC_decoding.LDPC_encoder import LDPCEncoder
    # (the seeded (3,6) test code is left out: its last N-K columns are singular in GF(2), which the
    # reference reports as "Not invertible Matrix" and then emits non-codewords)
    cases = {"wlan": (codes.wlan_80211n(54), 3), "dvb": (codes.dvbs2_structured(seed=0), 2)}
    out = {}
    with tempfile.TemporaryDirectory() as td:
        for name, (H, nvec) in cases.items():
            path = os.path.join(td, f"{name}.npz")
            codes.save_sparse_csr(path, codes.canonical_csr(H))
            enc = LDPCEncoder(path)
            # NEP 50: under numpy 2 `columnindex += direction` (GF2MatrixMul :180) stays np.int8 when
            # direction is the np.int8 EncodingMethod and wraps at 127; numpy 1.x, which the reference
            # was written for, promoted it to int64. Run it with that promotion:
            enc.EncodingMethod = np.int64(enc.EncodingMethod)
            rng = np.random.default_rng(7)
            X = rng.integers(0, 2, (enc.NumInfoBits, nvec))
            Y = np.stack([np.asarray(enc.encode(X[:, i].copy()), dtype=np.int64) for i in range(nvec)], axis=1)
            out[f"{name}_X"] = X.astype(np.uint8)
            out[f"{name}_Y"] = Y.astype(np.uint8)
            out[f"{name}_algo"] = np.array(enc.EncodingAlgorithm)
            out[f"{name}_roworder"] = np.asarray(enc.RowOrder, dtype=np.int32)
            print(name, enc.EncodingAlgorithm, "K", enc.NumInfoBits, "N", enc.BlockLength)
    np.savez_compressed(os.path.join(HERE, "reference_encoder.npz"), **out)


if __name__ == "__main__":
    main()
