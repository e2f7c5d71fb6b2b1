"""Training and evaluation harness (drop-in for the reference's training/__init__.py)."""
from ldpc_neural_decoder.training.trainer import LDPCDecoderTrainer
from ldpc_neural_decoder.training.comparative_evaluation import ComparativeEvaluator

__all__ = ["LDPCDecoderTrainer", "ComparativeEvaluator"]
