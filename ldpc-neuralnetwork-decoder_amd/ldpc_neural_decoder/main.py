"""Command-line front end (drop-in for the reference's ldpc_neural_decoder/main.py).

Same flags, defaults and modes (main.py:11-60, 324-337) and the same output files:
  train     -> trainer.save_model(--model_path) (TR:337-350 dict) + training_loss.png / error_rates.png
  evaluate  -> evaluation_results.pt {'snr_range', 'ber_results', 'fer_results'} + ber/fer_vs_snr.png
  compare   -> comparison_results.pt (ComparativeEvaluator dict, comparative_evaluation.py:86-104)
               + ber/fer/iterations_comparison.png
  visualize -> performance.png from evaluation_results.pt
so visualization/plot_comparison.py and the reference's loaders read the outputs unchanged.
Every decode runs on the HIP device: ``--device cpu`` keeps tensors on the host between calls,
it does not select a CPU implementation (there is none).

``--model_type``: 'standard' is models.decoder.LDPCNeuralDecoder (num_nodes = E, main.py:62-71);
'message_gnn' (an addition) trains/evaluates MessageGNNDecoder through the same trainer;
'tied' (TiedNeuralLDPCDecoder, notebook cell 15) is not built -- it raises.
"""
import argparse
import os

import torch

from ldpc_neural_decoder.utils.ldpc_utils import create_LLR_mapping, expand_base_matrix, load_base_matrix

_EXAMPLE_H = [[1, 1, 0, 0], [0, 1, 1, 1], [1, 0, 0, 1]]  # main.py:93-98


def _default_device():
    return "cuda" if torch.cuda.is_available() else "cpu"


def parse_args(argv=None):
    p = argparse.ArgumentParser(description="Train and evaluate LDPC neural decoder")
    p.add_argument("--mode", type=str, default="train", choices=["train", "evaluate", "visualize", "compare"])
    p.add_argument("--device", type=str, default=_default_device())
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--model_type", type=str, default="standard", choices=["standard", "tied", "message_gnn"])
    p.add_argument("--num_iterations", type=int, default=5)
    p.add_argument("--depth_L", type=int, default=2)
    p.add_argument("--hidden_dim", type=int, default=64, help="message_gnn only")
    p.add_argument("--base_matrix_path", type=str, default=None)
    p.add_argument("--lifting_factor", type=int, default=16)
    p.add_argument("--num_epochs", type=int, default=100)
    p.add_argument("--batch_size", type=int, default=32)
    p.add_argument("--learning_rate", type=float, default=0.001)
    p.add_argument("--momentum", type=float, default=0.9)
    p.add_argument("--weight_decay", type=float, default=0.0001)
    p.add_argument("--snr_min", type=int, default=-2)
    p.add_argument("--snr_max", type=int, default=6)
    p.add_argument("--snr_step", type=int, default=2)
    p.add_argument("--num_trials", type=int, default=100)
    p.add_argument("--compare_with_traditional", action="store_true")
    p.add_argument("--bp_max_iterations", type=int, default=50)
    p.add_argument("--ms_scaling_factor", type=float, default=0.75)
    p.add_argument("--model_path", type=str, default="ldpc_neural_decoder/models/saved_models/model.pt")
    p.add_argument("--results_dir", type=str, default="ldpc_neural_decoder/results")
    return p.parse_args(argv)


def load_code(args):
    """(H, base matrix or None) from --base_matrix_path / --lifting_factor, else the 3x4 example."""
    if args.base_matrix_path:
        base = load_base_matrix(args.base_matrix_path)
        return expand_base_matrix(base, args.lifting_factor), base
    return torch.tensor(_EXAMPLE_H, dtype=torch.float32), None


def create_model(args, H, base=None):
    """main.py:62-81 -> (model, converter or None, message types or None)."""
    if args.model_type == "standard":
        from ldpc_neural_decoder.models.decoder import LDPCNeuralDecoder
        return LDPCNeuralDecoder(num_nodes=int((H == 1).sum()), num_iterations=args.num_iterations,
                                 depth_L=args.depth_L), None, None
    if args.model_type == "message_gnn":
        from ldpc_neural_decoder.models.message_gnn_decoder import create_message_gnn_decoder
        Z = args.lifting_factor if base is not None else None
        model, conv = create_message_gnn_decoder(H, num_iterations=args.num_iterations, hidden_dim=args.hidden_dim,
                                                 base_graph=base, Z=Z)
        return model, conv, conv.get_message_types(base, Z)
    raise NotImplementedError("model_type 'tied' (TiedNeuralLDPCDecoder) is not part of this build")


def _setup(args):
    torch.manual_seed(args.seed)
    H, base = load_code(args)
    _, check_idx, var_idx, _ = create_LLR_mapping(H.T)
    model, conv, types = create_model(args, H, base)
    return H, check_idx, var_idx, model, conv, types


def _snr_range(args):
    return list(range(args.snr_min, args.snr_max + 1, args.snr_step))


def _trainer(args, model, conv, types):
    from ldpc_neural_decoder.training.trainer import LDPCDecoderTrainer
    return LDPCDecoderTrainer(model, device=args.device, converter=conv, message_types=types, seed=args.seed)


def train(args):
    """main.py:84-141."""
    H, check_idx, var_idx, model, conv, types = _setup(args)
    trainer = _trainer(args, model, conv, types)
    print(f"Training model with {args.num_epochs} epochs...")
    trainer.train(num_epochs=args.num_epochs, batch_size=args.batch_size, learning_rate=args.learning_rate,
                  check_index_tensor=check_idx, var_index_tensor=var_idx, snr_range=_snr_range(args),
                  variable_bit_length=H.shape[1], momentum=args.momentum, weight_decay=args.weight_decay)
    os.makedirs(os.path.dirname(args.model_path) or ".", exist_ok=True)
    trainer.save_model(args.model_path)
    print(f"Model saved to {args.model_path}")
    fig1, fig2 = trainer.plot_training_history()
    os.makedirs(args.results_dir, exist_ok=True)
    fig1.savefig(os.path.join(args.results_dir, "training_loss.png"))
    if fig2:
        fig2.savefig(os.path.join(args.results_dir, "error_rates.png"))
    return trainer


def evaluate(args):
    """main.py:143-205."""
    H, check_idx, var_idx, model, conv, types = _setup(args)
    trainer = _trainer(args, model, conv, types)
    trainer.load_model(args.model_path)
    print(f"Model loaded from {args.model_path}")
    snr_range = _snr_range(args)
    print(f"Evaluating model over SNR range {snr_range}...")
    ber, fer = trainer.evaluate_snr_range(snr_range=snr_range, batch_size=args.batch_size,
                                          num_trials=args.num_trials, check_index_tensor=check_idx,
                                          var_index_tensor=var_idx, variable_bit_length=H.shape[1])
    fig1, fig2 = trainer.plot_snr_performance(snr_range, ber, fer)
    os.makedirs(args.results_dir, exist_ok=True)
    fig1.savefig(os.path.join(args.results_dir, "ber_vs_snr.png"))
    fig2.savefig(os.path.join(args.results_dir, "fer_vs_snr.png"))
    results = {"snr_range": snr_range, "ber_results": ber, "fer_results": fer}
    torch.save(results, os.path.join(args.results_dir, "evaluation_results.pt"))
    print("Evaluation completed.")
    return results


def compare(args):
    """main.py:207-281."""
    from ldpc_neural_decoder.sweep import ComparativeEvaluator
    H, check_idx, var_idx, model, conv, types = _setup(args)
    neural = None
    if args.compare_with_traditional:
        neural = model
        checkpoint = torch.load(args.model_path, map_location="cpu", weights_only=True)
        neural.load_state_dict(checkpoint["model_state_dict"])
        neural.eval()
        print(f"Neural model loaded from {args.model_path}")
    evaluator = ComparativeEvaluator(H, neural_decoder=neural, device=args.device, converter=conv, seed=args.seed,
                                     message_types=types)
    snr_range = _snr_range(args)
    print(f"Comparing decoders over SNR range {snr_range}...")
    results = evaluator.evaluate_all(snr_range=snr_range, batch_size=args.batch_size, num_trials=args.num_trials,
                                     variable_bit_length=H.shape[1], check_index_tensor=check_idx,
                                     var_index_tensor=var_idx)
    os.makedirs(args.results_dir, exist_ok=True)
    evaluator.plot_ber_comparison(save_path=os.path.join(args.results_dir, "ber_comparison.png"))
    evaluator.plot_fer_comparison(save_path=os.path.join(args.results_dir, "fer_comparison.png"))
    evaluator.plot_iterations_comparison(save_path=os.path.join(args.results_dir, "iterations_comparison.png"))
    evaluator.save_results(os.path.join(args.results_dir, "comparison_results.pt"))
    evaluator.print_summary()
    print("Comparison completed.")
    return results


def visualize(args):
    """main.py:283-322."""
    path = os.path.join(args.results_dir, "evaluation_results.pt")
    if not os.path.exists(path):
        print(f"Results file not found: {path}")
        return
    results = torch.load(path, weights_only=True)
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    fig, axes = plt.subplots(1, 2, figsize=(10, 6))
    for ax, key, name in ((axes[0], "ber_results", "BER"), (axes[1], "fer_results", "FER")):
        ax.semilogy(results["snr_range"], results[key], "o-", label="Neural LDPC")
        ax.set_xlabel("SNR (dB)")
        ax.set_ylabel(name)
        ax.grid(True)
        ax.legend()
    fig.suptitle("LDPC Neural Decoder Performance")
    fig.tight_layout()
    fig.savefig(os.path.join(args.results_dir, "performance.png"))
    print("Visualization completed.")


def main(argv=None):
    args = parse_args(argv)
    return {"train": train, "evaluate": evaluate, "visualize": visualize, "compare": compare}[args.mode](args)


if __name__ == "__main__":
    main()
