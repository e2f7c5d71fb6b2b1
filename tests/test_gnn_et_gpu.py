"""Per-frame early termination of the bf16 MessageGNN decoder (BASELINE cfg5) (GPU).

Parity unpinned: the reference has no early termination (message_gnn_decoder.py:247-265 always
runs every layer).  The feature is checked by construction instead:
  * a decoder whose decisions never form a codeword never stops, and its outputs are bitwise
    those of the full run;
  * a decoder built so that every layer's hard decision is the channel's own sign decision stops
    after layer 1 exactly on the frames whose channel decision is a codeword (oracle syndrome),
    runs to the end on the others, and again returns bitwise the full run's outputs."""
import numpy as np
import pytest
import torch

from conftest import code_path

from ldpc_neural_decoder.models import create_message_gnn_decoder
from ldpc_neural_decoder.utils import awgn_llr, expand_base_matrix, load_base_matrix

pytestmark = pytest.mark.gpu


def _decoder(z, layers, cuda, seed=0):
    torch.manual_seed(seed)
    # Z = 384 (5G's largest lifting): the BG2 shifts of the Z = 32 file lifted at 384, N = 19 968 --
    # the syndrome pass's variable sums no longer fit its LDS cache and are summed again instead
    base = load_base_matrix(code_path(32 if z == 384 else z))
    H = expand_base_matrix(base, z)
    dec, conv = create_message_gnn_decoder(H, num_iterations=layers, hidden_dim=64, base_graph=base, Z=z)
    with torch.no_grad():
        for p in dec.parameters():
            p.mul_(0.5)
    dec = dec.to(cuda)
    dec.precision = "bf16"
    return base, H, dec, conv


def _run(dec, conv, base, z, llr, et):
    dec.early_termination = et
    args = (llr, conv.message_to_var_index(), conv.get_message_types(base, z), conv.var_to_check_adjacency,
            conv.check_to_var_adjacency)
    with torch.no_grad():
        p = dec(*args)
    return p, dec.last_iterations.clone()


def test_no_stop_is_the_full_run(cuda):
    base, H, dec, conv = _decoder(4, 5, cuda)
    llr = awgn_llr(96, H.shape[1], 3.0, seed=5, device=cuda)
    p0, it0 = _run(dec, conv, base, 4, llr, False)
    p1, it1 = _run(dec, conv, base, 4, llr, True)
    assert torch.equal(it0, torch.full_like(it0, 5))
    assert torch.equal(it1, torch.full_like(it1, 5))  # random weights: no decision is a codeword
    assert torch.equal(p0, p1)


@pytest.mark.parametrize("compact", ["1", "0"])
@pytest.mark.parametrize("z,layers,B", [(4, 5, 512), (32, 4, 64), (32, 15, 64), (32, 3, 300), (384, 3, 8)])
def test_stops_exactly_on_codeword_decisions(cuda, oracle_mod, monkeypatch, z, layers, B, compact):
    """(compact: after a syndrome pass the layers walk the list of frames still decoding, or --
    LDPC_GNN_ET_COMPACT=0 -- every frame, skipping the finished ones; same results either way)"""
    monkeypatch.setenv("LDPC_GNN_ET_COMPACT", compact)
    base, H, dec, conv = _decoder(z, layers, cuda, seed=1)
    with torch.no_grad():  # second Linear of every MLP = 0: x = 0 after every layer
        for layer in dec.gnn_layers:
            for seq in (layer.var_to_check_update, layer.check_to_var_update):
                seq[2].weight.zero_()
                seq[2].bias.zero_()
        dec.gnn_layers[-1].output_projection.bias.zero_()
    # the decoder's P(bit = 1) = sigmoid(llr): feed -LLR so a hard 1 is a channel sign error
    llr = -awgn_llr(B, H.shape[1], 9.0 if z == 4 else 12.0, seed=11, device=cuda)
    p_full, it_full = _run(dec, conv, base, z, llr, False)
    p_et, it_et = _run(dec, conv, base, z, llr, True)
    hard = (llr > 0).to(torch.uint8).cpu().numpy()
    valid = oracle_mod.syndrome_valid(oracle_mod.Graph(H.numpy()), hard)
    assert 0 < valid.sum() < B  # both branches exercised
    expect = np.where(valid, 1, layers)
    np.testing.assert_array_equal(it_et.cpu().numpy(), expect)
    assert torch.equal(it_full, torch.full_like(it_full, layers))
    assert torch.equal(p_et, p_full)


def test_fp32_early_termination_is_refused(cuda):
    base, H, dec, conv = _decoder(4, 2, cuda)
    dec.precision = "fp32"
    llr = awgn_llr(4, H.shape[1], 3.0, device=cuda)
    with pytest.raises(NotImplementedError):
        _run(dec, conv, base, 4, llr, True)


def test_group_mean_grid_cap_is_bitwise_neutral(cuda, monkeypatch):
    """LDPC_GNN_GM_CAP: after the first syndrome pass the group-mean kernel strides a capped grid
    over the frames still decoding; every (frame, tile) item is computed exactly as before."""
    base, H, dec, conv = _decoder(32, 5, cuda, seed=6)
    llr = awgn_llr(300, H.shape[1], 4.0, seed=29, device=cuda)
    monkeypatch.setenv("LDPC_GNN_GM_CAP", "0")
    p1, it1 = _run(dec, conv, base, 32, llr, True)
    monkeypatch.setenv("LDPC_GNN_GM_CAP", "1")
    p2, it2 = _run(dec, conv, base, 32, llr, True)
    assert torch.equal(p1, p2) and torch.equal(it1, it2)
