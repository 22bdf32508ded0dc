"""Golden vectors for the channel generator's inversion rule, from the REFERENCE (build container only).

Usage:  python tests/golden/make_golden_channel.py [/root/reference]

Imports the reference's AWGN_Channel_Transmission/AWGN_Quantizer_BPSK.py (its information-bottleneck
design package is absent: stubbed; the quantiser is built with dont_calc=True and given a CDF), then
runs its host `quantize_direct(input_bits)` (:126-143) on uniforms drawn by np.random.seed(s) —
both the B > 1 branch (:132-134) and the B = 1 branch (:136-140), all-zero and random codeword bits.
Stores seeds, CDFs, bits and the reference's cluster ids; tests regenerate the uniforms with
np.random.RandomState(s).rand and check the oracle's inversion rule against them.
No reference source is copied. Output: tests/golden/reference_channel.npz
"""
from __future__ import annotations

import os
import sys
import types

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, HERE)
sys.path.insert(0, ROOT)
sys.dont_write_bytecode = True

import make_golden  # noqa: E402  (stubs for pyopencl / mako / np.int)

from informationbottleneckdecodingldpc_amd.channel import UniformQuantizer, sigma2_from_ebn0  # noqa: E402


def main():
    make_golden._stub_reference_imports()
    for name in ["information_bottleneck", "information_bottleneck.information_bottleneck_algorithms",
                 "information_bottleneck.information_bottleneck_algorithms.symmetric_sIB", "pyopencl.clrandom"]:
        sys.modules.setdefault(name, types.ModuleType(name))
    sys.modules["information_bottleneck.information_bottleneck_algorithms.symmetric_sIB"].symmetric_sIB = object
    sys.modules["pyopencl.clrandom"].rand = None
    from AWGN_Channel_Transmission.AWGN_Quantizer_BPSK import AWGN_Channel_Quantizer

    out = {}
    cases = [(16, 0.6, 64, 40, 0), (16, 2.0, 50, 1, 1), (8, 1.0, 33, 17, 2), (32, 0.0, 20, 9, 3)]
    for k, (T, ebn0, n, B, seed) in enumerate(cases):
        q = UniformQuantizer(sigma2_from_ebn0(ebn0, 0.5), T=T)
        ref = AWGN_Channel_Quantizer(q.sigma_n2, 3.0, T, 2000, dont_calc=True)
        ref.cardinality_T = T
        ref.cdf_t_given_x_equals_zero = q.cdf_t_given_x_equals_zero
        for kind in ("zero", "bits"):
            bits = np.zeros((n, B), np.int64) if kind == "zero" else \
                np.random.default_rng(100 + k).integers(0, 2, (n, B))
            np.random.seed(seed)
            t = ref.quantize_direct(bits)
            out[f"c{k}_{kind}_T"] = np.int32(T)
            out[f"c{k}_{kind}_seed"] = np.int64(seed)
            out[f"c{k}_{kind}_cdf"] = q.cdf_t_given_x_equals_zero
            out[f"c{k}_{kind}_bits"] = bits.astype(np.uint8)
            out[f"c{k}_{kind}_t"] = np.asarray(t, np.int32)
    out["ncases"] = np.int32(len(cases))
    np.savez_compressed(os.path.join(HERE, "reference_channel.npz"), **out)
    print("wrote", os.path.join(HERE, "reference_channel.npz"), len(out), "arrays")


if __name__ == "__main__":
    main()
