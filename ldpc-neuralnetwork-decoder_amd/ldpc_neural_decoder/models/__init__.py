"""Decoders (drop-in for the reference's models/__init__.py:7-30, hot-path subset)."""
from ldpc_neural_decoder.models.layers import CheckLayer, VariableLayer, ResidualLayer, OutputLayer
from ldpc_neural_decoder.models.decoder import LDPCNeuralDecoder
from ldpc_neural_decoder.models.traditional_decoders import (
    BeliefPropagationDecoder, MinSumScaledDecoder)
from ldpc_neural_decoder.models.message_gnn_decoder import (
    MessageGNNLayer, MessageGNNDecoder, TannerToMessageGraph, create_message_gnn_decoder)
from ldpc_neural_decoder.models.custom_decoders import (
    CustomCheckMessageGNNLayer, CustomMinSumMessageGNNDecoder, CustomVariableMessageGNNDecoder,
    CustomVariableMessageGNNLayer, create_custom_minsum_message_gnn_decoder,
    create_custom_variable_message_gnn_decoder)

__all__ = [
    "CheckLayer", "VariableLayer", "ResidualLayer", "OutputLayer", "LDPCNeuralDecoder",
    "BeliefPropagationDecoder", "MinSumScaledDecoder",
    "MessageGNNLayer", "MessageGNNDecoder", "TannerToMessageGraph", "create_message_gnn_decoder",
    "CustomCheckMessageGNNLayer", "CustomMinSumMessageGNNDecoder", "CustomVariableMessageGNNLayer",
    "create_custom_minsum_message_gnn_decoder", "CustomVariableMessageGNNDecoder",
    "create_custom_variable_message_gnn_decoder",
]
