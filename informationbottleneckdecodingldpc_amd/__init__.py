"""MI355X-native batched LDPC decoding (information-bottleneck LUT, min-sum, belief propagation).

Drop-in for the decoder classes of mx-strk/InformationBottleneckDecodingLDPC:

    from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder_irreg import \
        Discrete_LDPC_Decoder_class_irregular
    from informationbottleneckdecodingldpc_amd.discrete_LDPC_decoder import Discrete_LDPC_Decoder_class
    from informationbottleneckdecodingldpc_amd.min_sum_decoder_irreg import Min_Sum_Decoder_class_irregular
    from informationbottleneckdecodingldpc_amd.bp_decoder_irreg import BeliefPropagationDecoderClassIrregular

and for the channel side / drivers:

    from informationbottleneckdecodingldpc_amd.awgn_quantizer import AWGN_Channel_Quantizer  # device sampling
    from informationbottleneckdecodingldpc_amd.ber import BERConfig, run_ber                 # Eb/N0 sweeps
    from informationbottleneckdecodingldpc_amd.tables_io import load_decoder_config          # .npz/.json/.pkl

Decoding runs only in the hand-written HIP kernels of ``libibldpc.so`` (gfx950); see DESIGN.md.
"""
from . import codes, graph, tables, tables_io  # noqa: F401  (host-side set-up, importable without a GPU)

__version__ = "0.2.0"


def library_path() -> str:
    from ._lib import LIB_PATH
    return LIB_PATH
