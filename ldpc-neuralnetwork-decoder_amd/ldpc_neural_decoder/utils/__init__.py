"""Utilities (drop-in for the reference's ldpc_neural_decoder.utils, utils/__init__.py:5-17)."""
from ldpc_neural_decoder.utils.ldpc_utils import (
    create_LLR_mapping, edge_list, expand_base_matrix, get_LLR_indexes, load_base_matrix)
from ldpc_neural_decoder.utils.channel import (
    qpsk_modulate, qpsk_demodulate, awgn_channel, compute_ber_fer, AWGNChannel, awgn_llr,
    count_errors)

__all__ = [
    "get_LLR_indexes", "create_LLR_mapping", "expand_base_matrix", "load_base_matrix", "edge_list",
    "qpsk_modulate", "qpsk_demodulate", "awgn_channel", "compute_ber_fer", "AWGNChannel",
    "awgn_llr", "count_errors",
]
