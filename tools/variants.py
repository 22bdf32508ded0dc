"""Build kernel variants of libibldpc.so side by side (in-tree, so they travel to the GPU box) for A/B
timing: `python tools/variants.py` then `IBLDPC_LIB=<path> python bench.py ...`."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from informationbottleneckdecodingldpc_amd import _build  # noqa: E402

VARIANTS = {
    "w1": ["IBL_W=1"],
    "w1u": ["IBL_W=1", "IBL_CN_UNROLL=1"],
    "w2": ["IBL_W=2"],
    "w2u": ["IBL_W=2", "IBL_CN_UNROLL=1", "IBL_LB8=512"],
    "w4": ["IBL_W=4", "IBL_LB8=512"],
    "w2b": ["IBL_W=2", "IBL_LB8=512"],
    "wpe5": ["IBL_WPE8=5"],
    "wpe6": ["IBL_WPE8=6"],
}

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    outdir = os.path.join(_build.PKG, "variants")
    os.makedirs(outdir, exist_ok=True)
    for n in names:
        lib = os.path.join(outdir, f"libibldpc_{n}.so")
        _build.build(defines=VARIANTS[n], lib=lib, tag=n, force="--force" in os.environ.get("VARIANT_FLAGS", ""))
        print(lib)
