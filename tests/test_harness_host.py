"""Harness and on-disk formats, host side: CLI flags and defaults, the
checkpoint/result dict schemas, and the var-major edge structure LDPCNeuralDecoder derives from
the reference's index tensors.  No GPU."""
import os

import numpy as np
import pytest
import torch

from conftest import code_path

from ldpc_neural_decoder import main as cli
from ldpc_neural_decoder.models.decoder import edge_variables
from ldpc_neural_decoder.training.trainer import HISTORY_KEYS
from ldpc_neural_decoder.utils import create_LLR_mapping, expand_base_matrix, load_base_matrix

# main.py:11-60 of the reference (flag -> default); the reference module cannot be imported (it
# imports the missing models/decoder.py), so the defaults are restated here with their lines
REFERENCE_DEFAULTS = {
    "mode": "train", "seed": 42, "model_type": "standard", "num_iterations": 5, "depth_L": 2,
    "base_matrix_path": None, "lifting_factor": 16, "num_epochs": 100, "batch_size": 32,
    "learning_rate": 0.001, "momentum": 0.9, "weight_decay": 0.0001, "snr_min": -2, "snr_max": 6,
    "snr_step": 2, "num_trials": 100, "compare_with_traditional": False, "bp_max_iterations": 50,
    "ms_scaling_factor": 0.75, "model_path": "ldpc_neural_decoder/models/saved_models/model.pt",
    "results_dir": "ldpc_neural_decoder/results",
}


def test_cli_defaults_match_reference():
    args = vars(cli.parse_args([]))
    for k, v in REFERENCE_DEFAULTS.items():
        assert args[k] == v, k
    assert args["device"] == ("cuda" if torch.cuda.is_available() else "cpu")


def test_cli_flags_parse():
    a = cli.parse_args(["--mode", "compare", "--compare_with_traditional", "--snr_min", "0", "--snr_max", "4",
                        "--snr_step", "1", "--model_type", "message_gnn", "--lifting_factor", "4"])
    assert a.mode == "compare" and a.compare_with_traditional and a.model_type == "message_gnn"
    assert cli._snr_range(a) == [0, 1, 2, 3, 4]
    with pytest.raises(SystemExit):
        cli.parse_args(["--mode", "bogus"])


def test_load_code_example_and_file():
    a = cli.parse_args([])
    H, base = cli.load_code(a)
    assert base is None and H.tolist() == [[1, 1, 0, 0], [0, 1, 1, 1], [1, 0, 0, 1]]
    a = cli.parse_args(["--base_matrix_path", code_path(4), "--lifting_factor", "4"])
    H, base = cli.load_code(a)
    assert H.shape == (42 * 4, 52 * 4) and base.shape == (42, 52)


def test_tied_model_is_refused():
    a = cli.parse_args(["--model_type", "tied"])
    with pytest.raises(NotImplementedError):
        cli.create_model(a, torch.tensor([[1.0, 1.0]]))


def test_history_keys_are_the_reference_checkpoint_schema():
    # trainer.py:344-350: torch.save({'model_state_dict', 'train_losses', 'val_losses',
    # 'ber_history', 'fer_history'})
    assert HISTORY_KEYS == ("train_losses", "val_losses", "ber_history", "fer_history")


@pytest.mark.parametrize("which", ["example", 4, 32])
def test_edge_variables_recover_var_major_numbering(which):
    if which == "example":
        H = torch.tensor([[1, 1, 0, 0], [0, 1, 1, 1], [1, 0, 0, 1]], dtype=torch.float32)
    else:
        H = expand_base_matrix(load_base_matrix(code_path(which)), which)
    _, _, var_idx, out_idx = create_LLR_mapping(H.T)
    var_of = edge_variables(var_idx)
    assert torch.equal(var_of, out_idx[0].long())       # create_LLR_mapping's own edge -> var map
    # the padded form the reference gathers with (-1 -> E) gives the same answer
    E = var_idx.shape[0]
    assert torch.equal(edge_variables(torch.where(var_idx < 0, torch.full_like(var_idx, E), var_idx)), var_of)


def test_oracle_neural_decoder_shapes(oracle_mod):
    H = expand_base_matrix(load_base_matrix(code_path(4)), 4)
    _, cidx, vidx, out_idx = create_LLR_mapping(H.T)
    E = cidx.shape[0]
    torch.manual_seed(0)
    params = [(torch.rand(E) + 0.5, torch.tensor([0.5, -0.25])) for _ in range(2)]
    llr = torch.randn(5, H.shape[1]) * 3
    gt = (torch.rand(5, H.shape[1]) < 0.5).float()
    soft, loss = oracle_mod.neural_decoder(params, llr, cidx, vidx, out_idx[0], 2, gt)
    assert soft.shape == (5, H.shape[1]) and loss.shape == (5,)
    assert torch.all((soft >= 0) & (soft <= 1)) and torch.all(loss >= 0)
    # one iteration, no variable layers: soft = sigmoid(-(llr + sum of min-sum c2v of the channel))
    soft1, _ = oracle_mod.neural_decoder([], llr, cidx, vidx, out_idx[0], 2)
    c = oracle_mod.check_layer(llr[:, out_idx[0]], cidx)
    app = torch.zeros_like(llr).index_add(1, out_idx[0], c)
    np.testing.assert_allclose(soft1.numpy(), torch.sigmoid(-(llr + app)).numpy(), rtol=1e-6)
