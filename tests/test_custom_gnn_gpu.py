"""Hybrid GNN decoder (CustomVariableMessageGNNDecoder, message_gnn_decoder.py:758-879) on the GPU vs
the oracle (oracle/oracle.py custom_variable_forward, torch fp32).

The reference cannot run this decoder, so the end-to-end bar is this build's
stated definition (models/custom_decoders.py): "parity unpinned" beyond the components it shares with
MessageGNNDecoder (embeddings, check-side MLP, output heads -- pinned by gnn_z*.npz).  Bar: probs
within 2e-5 of the oracle, the fp32 GNN tolerance (float32 re-association inside the MLPs)."""
import numpy as np
import pytest
import torch

from conftest import code_path

from ldpc_neural_decoder.models import create_custom_variable_message_gnn_decoder
from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix

pytestmark = pytest.mark.gpu
TOL = 2e-5


def setup(z, layers, seed, hidden=64):
    base = load_base_matrix(code_path(z))
    H = expand_base_matrix(base, z)
    torch.manual_seed(seed)
    dec, conv = create_custom_variable_message_gnn_decoder(H, num_iterations=layers, hidden_dim=hidden,
                                                           base_graph=base, Z=z)
    types = conv.get_message_types(base, z)
    return H, dec, conv, types


@pytest.mark.parametrize("z,layers,B,identity", [(4, 3, 16, False), (4, 5, 7, True), (32, 4, 6, False)])
def test_hybrid_gnn_vs_oracle(cuda, oracle_mod, z, layers, B, identity):
    H, dec, conv, types = setup(z, layers, 100 + z + layers)
    llr = torch.randn(B, H.shape[1]) * 2.0 + 1.0
    Ac = None if identity else conv.check_to_var_adjacency
    Av = None if identity else conv.var_to_check_adjacency
    probs, loss = dec(llr.to(cuda), conv.message_to_var_index().to(cuda), types.to(cuda), Av, Ac)
    assert loss is None
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    ref = oracle_mod.custom_variable_forward(sd, llr, conv.edge_var, conv.edge_chk, H.shape[1], H.shape[0],
                                             types=types, check_identity=identity)
    np.testing.assert_allclose(probs.detach().cpu().numpy(), ref.numpy(), atol=TOL, rtol=0)


@pytest.mark.parametrize("hidden,z,identity", [(8, 4, False), (32, 4, True), (96, 32, False), (128, 4, False)])
def test_hybrid_gnn_any_hidden_dim_vs_oracle(cuda, oracle_mod, hidden, z, identity):
    """hidden_dim other than 64 (the reference's constructor takes any, MGD:765; its min-sum factory's
    default is 8, :1254): the check side of the generic fp32 kernels (group means, the tiled MLP with
    the layer's own head), the same variable update and output; against the oracle at the same bar."""
    H, dec, conv, types = setup(z, 3, 300 + hidden, hidden=hidden)
    llr = torch.randn(5, H.shape[1]) * 2.0 + 1.0
    Ac = None if identity else conv.check_to_var_adjacency
    Av = None if identity else conv.var_to_check_adjacency
    probs, _ = dec(llr.to(cuda), conv.message_to_var_index().to(cuda), types.to(cuda), Av, Ac)
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    ref = oracle_mod.custom_variable_forward(sd, llr, conv.edge_var, conv.edge_chk, H.shape[1], H.shape[0],
                                             types=types, check_identity=identity)
    np.testing.assert_allclose(probs.detach().cpu().numpy(), ref.numpy(), atol=TOL, rtol=0)


def test_hybrid_gnn_loss_decode_and_one_hot_mapping(cuda, oracle_mod):
    H, dec, conv, types = setup(4, 3, 7)
    llr = (torch.randn(9, H.shape[1]) + 1.5).to(cuda)
    gt = torch.zeros_like(llr)
    Av, Ac = conv.var_to_check_adjacency, conv.check_to_var_adjacency
    p1, loss = dec(llr, conv.message_to_var_mapping.to(cuda), types.to(cuda), Av, Ac, ground_truth=gt)
    p2, _ = dec(llr, conv.message_to_var_index().to(cuda), types.to(cuda), Av, Ac)
    assert torch.equal(p1, p2)
    want = torch.nn.functional.binary_cross_entropy(p1, gt, reduction="none").max(dim=1).values
    assert torch.allclose(loss, want)
    assert torch.equal(dec.decode(llr, conv.message_to_var_index().to(cuda), types.to(cuda), Av, Ac), (p1 > 0.5).float())
    sub, _ = dec(llr[2:5], conv.message_to_var_index().to(cuda), types.to(cuda), Av, Ac)
    assert torch.equal(sub, p1[2:5])


def test_hybrid_gnn_bench_size_chunks(cuda, oracle_mod):
    """The hybrid-gnn-z32 bench shape: B = 32 768 frames, 10 layers, which the forward splits into
    launches of at most ((1 << 31) // 16 - 1) // E = 21 291 frames (the kernels' per-launch message
    bound).  Sub-batches -- one straddling the chunk boundary -- decode bit-identically to the same
    frames inside the full batch, and four spot frames across both chunks match the oracle."""
    H, dec, conv, types = setup(32, 10, 77)
    from ldpc_neural_decoder.utils import awgn_llr
    B = 32768
    E = len(conv.messages)
    limit = ((1 << 31) // 16 - 1) // E
    assert limit < B  # two launches
    llr = awgn_llr(B, H.shape[1], 2.0, seed=20251015, device=cuda)
    io, ty = conv.message_to_var_index().to(cuda), types.to(cuda)
    Av, Ac = conv.var_to_check_adjacency, conv.check_to_var_adjacency
    with torch.no_grad():
        full, _ = dec(llr, io, ty, Av, Ac)
        for s, e in ((0, 7), (limit - 3, limit + 4), (B - 5, B)):
            part, _ = dec(llr[s:e].contiguous(), io, ty, Av, Ac)
            assert torch.equal(part, full[s:e]), (s, e)
    spots = [0, limit - 1, limit, B - 1]
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    ref = oracle_mod.custom_variable_forward(sd, llr[spots].cpu(), conv.edge_var, conv.edge_chk, H.shape[1],
                                             H.shape[0], types=types)
    np.testing.assert_allclose(full[spots].cpu().numpy(), ref.numpy(), atol=TOL, rtol=0)


def test_hybrid_training_is_refused_clearly(cuda):
    """No HIP backward for the hybrid decoders: the hybrid GNN's probs carry a grad_fn whose
    backward names the decoder (not torch's generic "does not require grad"); the hybrid min-sum
    reads no parameter (its alpha, MGD:974, is never used), so its probs need no grad at all."""
    H, dec, conv, types = setup(4, 2, 3)
    llr = (torch.randn(4, H.shape[1]) + 1.5).to(cuda)
    Av, Ac = conv.var_to_check_adjacency, conv.check_to_var_adjacency
    p, loss = dec(llr, conv.message_to_var_index().to(cuda), types.to(cuda), Av, Ac, ground_truth=torch.zeros_like(llr))
    assert p.requires_grad
    with pytest.raises(NotImplementedError, match="CustomVariableMessageGNNDecoder"):
        loss.mean().backward()
    from ldpc_neural_decoder.models import create_custom_minsum_message_gnn_decoder
    hdec, _ = create_custom_minsum_message_gnn_decoder(H, num_iterations=3)
    q = hdec(llr)
    assert not q.requires_grad
