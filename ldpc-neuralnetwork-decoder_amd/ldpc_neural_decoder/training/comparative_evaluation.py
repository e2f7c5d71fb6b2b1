"""training/comparative_evaluation.py of the reference: the evaluator lives in sweep.py (the
on-device SNR sweep); this module keeps the reference's import path."""
from ldpc_neural_decoder.sweep import ComparativeEvaluator

__all__ = ["ComparativeEvaluator"]
