"""Utilities (drop-in for the reference's ldpc_neural_decoder.utils, utils/__init__.py:5-17)."""
from ldpc_neural_decoder.utils.ldpc_utils import expand_base_matrix, load_base_matrix, edge_list
from ldpc_neural_decoder.utils.channel import (
    qpsk_modulate, qpsk_demodulate, awgn_channel, compute_ber_fer, AWGNChannel, awgn_llr,
    count_errors)

__all__ = [
    "expand_base_matrix", "load_base_matrix", "edge_list",
    "qpsk_modulate", "qpsk_demodulate", "awgn_channel", "compute_ber_fer", "AWGNChannel",
    "awgn_llr", "count_errors",
]
