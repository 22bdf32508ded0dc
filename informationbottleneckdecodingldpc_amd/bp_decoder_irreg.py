"""Float belief-propagation LDPC decoder — drop-in for the reference's
``Continous_LDPC_Decoding/bp_decoder_irreg.py`` (class ``BeliefPropagationDecoderClassIrregular``,
:19-432), running on MI355X HIP kernels (``ibl_float_*`` with ``IBL_BP``).
"""
from __future__ import annotations

from . import _lib
from .min_sum_decoder_irreg import Min_Sum_Decoder_class_irregular


class BeliefPropagationDecoderClassIrregular(Min_Sum_Decoder_class_irregular):
    """Reference ``__init__`` (bp_decoder_irreg.py:23-69); box-plus check nodes
    (kernels_min_and_BP.cl:5-71)."""

    _kind = _lib.IBL_BP

    def decode_OpenCL_belief_propagation(self, received_blocks, buffer_in=False, return_buffer=False):
        """Reference :221-286."""
        return self._decode(received_blocks, buffer_in, return_buffer)

    def decode_OpenCL_min_sum(self, *a, **k):  # pragma: no cover - not part of the BP class
        raise AttributeError("BeliefPropagationDecoderClassIrregular has no decode_OpenCL_min_sum")
