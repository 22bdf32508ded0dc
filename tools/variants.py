"""Build kernel variants of libibldpc.so side by side (in-tree, so they travel to the GPU box) for A/B
timing: `python tools/variants.py` then `IBLDPC_LIB=<path> python bench.py ...`."""
import os
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from informationbottleneckdecodingldpc_amd import _build  # noqa: E402

VARIANTS = {
    "w1": ["IBL_W=1"],
    # one dword per lane everywhere (rows padded to 512 codewords): the Infinity-Cache sub-batch experiment
    "w1l1": ["IBL_W=1", "IBL_LIGHT_W=1"],
    "w1u": ["IBL_W=1", "IBL_CN_UNROLL=1"],
    "w2": ["IBL_W=2"],
    "w2u": ["IBL_W=2", "IBL_CN_UNROLL=1", "IBL_LB8=512"],
    "w4": ["IBL_W=4", "IBL_LB8=512"],
    "w2b": ["IBL_W=2", "IBL_LB8=512"],
    "wpe5": ["IBL_WPE8=5"],
    "wpe6": ["IBL_WPE8=6"],
    # spill experiment (DESIGN.md "Private segment"): MAXD=16 kernels at 1024-thread launch bounds
    # (128 VGPRs) spill their item buffers to scratch; run with IBL_ALLOW_SCRATCH=1
    "spill16": ["IBL_LB16=1024"],
    # variable pass co-scheduling: waves with (threadIdx.x >> 8) < IBL_MIX take the light (degree <= 4,
    # HBM-bound) items first, the others the heavy (LDS-bound) ones
    "mix1": ["IBL_MIX16=4"],
    # round 6: every wave interleaves one heavy and two light variable items (ib_phase_mix3)
    "vmix3": ["IBL_VN_MIX3=1"],
    "chloop": ["IBL_CH_BINNED=0"],
    "ntcn0": ["IBL_NT_CN=0"],   # check pass rows with the default cache policy (round 5 adopted nontemporal)
    "mix0": ["IBL_MIX16=0"],
    "mixw5": ["IBL_MIX16=5"],
    "mixw10": ["IBL_MIX16=10"],    # no light-first waves in the variable pass (round 5 adopted 4 of 16)   # channel sampler: T compares per sample (before round 6's binned inversion)
    "mix2": ["IBL_MIX16=8"],
    "mix3": ["IBL_MIX16=12"],
    "mixw2": ["IBL_MIX16=2"],
    "mixw3": ["IBL_MIX16=3"],
    "mixw6": ["IBL_MIX16=6"],
    # three light variable items in flight per wave instead of two; round-2 light rows (W=2, depth 3)
    "ld3": ["IBL_LIGHT_DEPTH=3"],
    "lw2": ["IBL_LIGHT_W=2", "IBL_LIGHT_DEPTH=3"],
    # variable pass light items with 1-KiB row segments per wave (4 dwords per lane), 3 / 2 in flight
    "lw4": ["IBL_LIGHT_W=4"],
    "lw4d2": ["IBL_LIGHT_W=4", "IBL_LIGHT_DEPTH=2"],
    # plain (cached) variable-pass row accesses instead of the default nontemporal ones
    "nt0": ["IBL_NT=0"],
    # check schedule of 2 codewords x 4 chains (half the column-term registers of 4 x 2)
    "s2n": ['IBL_SCHED_FILE="ib_sched_s2n.inc"'],
    # one dword per lane (8 codewords) and all 8 in one check-schedule group: 16 check chains in flight
    "w1s8": ["IBL_W=1", 'IBL_SCHED_FILE="ib_sched_w1s8.inc"'],
    "w1l4": ["IBL_W=1", 'IBL_SCHED_FILE="ib_sched_w1l4.inc"'],
    "w2l4": ['IBL_SCHED_FILE="ib_sched_w2l4.inc"'],
    "cl3": ['IBL_SCHED_FILE="ib_sched_cl3.inc"'],
    "v4l2": ['IBL_SCHED_FILE="ib_sched_v4l2.inc"'],
    "v2l3": ['IBL_SCHED_FILE="ib_sched_v2l3.inc"'],
    # table staging as 16-byte units, four per thread and global round trip (the loop before the shuffle staging)
    "stageu": ["IBL_STAGE_UNITS=1"],
    # small-batch kernels loading every lane's node record (no contiguous task records)
    "contig0": ["IBL_SMALL_CONTIG=0"],
    # fused IB kernel phase trace (IBL_TRACE_FUSED=<file>)
    "ftrace": ["IBL_FUSED_TRACE=1", "IBL_DIAG=1"],
    # timing-only host hooks (IBL_VN_PART, IBL_TRACE_WAVES, IBL_DEBUG_SYNC): not in the product build
    "diag": ["IBL_DIAG=1"],
    # column fetches (tools/gen_sched.py "Column fetches"; the schedule file is generated on demand).
    # Measured on DVB-S2 (B=8192, i_max=50): nc00 170.9k cw/s (CN 0.464 / VN 0.478 ms), nc23 140.9k
    # (0.622 / 0.526), nc22 142.0k, nc33 132.3k, s2 156.5k -> the default build keeps NC = 0.
    "nc23": ["IBL_NC_CN=2", "IBL_NC_VN=3", 'IBL_SCHED_FILE="ib_sched_nc23.inc"'],
    "nc22": ["IBL_NC_CN=2", "IBL_NC_VN=2", 'IBL_SCHED_FILE="ib_sched_nc22.inc"'],
    "nc33": ["IBL_NC_CN=3", "IBL_NC_VN=3", 'IBL_SCHED_FILE="ib_sched_nc33.inc"'],
    "s2": ["IBL_NC_CN=2", "IBL_NC_VN=3", 'IBL_SCHED_FILE="ib_sched_s2.inc"'],
    # float per-pass rows as plain loads / stores (the default is nontemporal since round 5)
    "flplain": ["IBL_FL_NT=0"],
    # nontemporal check-pass rows (the variable pass's are nontemporal by default)
    "ntcn": ["IBL_NT_CN=1"],
    "ntcn0": ["IBL_NT_CN=0"],
    # float variable items over 2-KiB row segments (two 16-byte pieces per lane)
    "flvn2": ["IBL_FL_VN2=1"],
    # float kernels built with NaNs not honoured but the IEEE mode bit on
    "ieeeon": [],
    # min-sum check node with the (min, second min) pair for every degree (the round-3 form)
    "msps0": ["IBL_MS_PS=0"],
    # fused float check tasks without the constant-stride body for full tasks
    "cn64off": ["IBL_FL_CN64=0"],
}
# per-source flag overrides (replace _build.SRC_FLAGS)
SRC_FLAGS = {"ieeeon": {"float_kernels.hip": ["-fno-honor-nans"]}}
# gen_sched.py arguments of the variants that need their own schedule file
SCHED_ARGS = {"nc23": "4 2 2 4 2 3", "nc22": "4 2 2 4 2 2", "nc33": "4 2 2 4 3 3", "s2": "2 4 2 4 2 3",
              "s2n": "2 4 2 4 0 0", "w1s8": "8 2 2 4 0 0", "w1l4": "4 4 2 4 0 0", "w2l4": "4 4 2 4 0 0", "cl3": "4 3 2 4 0 0", "v4l2": "4 2 4 2 0 0", "v2l3": "4 2 2 3 0 0"}

if __name__ == "__main__":
    names = sys.argv[1:] or list(VARIANTS)
    outdir = os.path.join(_build.PKG, "variants")
    os.makedirs(outdir, exist_ok=True)
    for n in names:
        if n in SCHED_ARGS:
            inc = os.path.join(_build.CSRC, f"ib_sched_{n}.inc")
            with open(inc, "w") as f:
                subprocess.run([sys.executable, os.path.join(os.path.dirname(__file__), "gen_sched.py"),
                                *SCHED_ARGS[n].split()], stdout=f, check=True)
        lib = os.path.join(outdir, f"libibldpc_{n}.so")
        _build.build(defines=VARIANTS[n], lib=lib, tag=n, src_flags=SRC_FLAGS.get(n), force="--force" in os.environ.get("VARIANT_FLAGS", ""))
        print(lib)
