"""MessageGNNDecoder with adjacencies other than TannerToMessageGraph's (GPU).

The reference multiplies whatever (E, E) matrices it is given with a dense bmm, after zero-padding
or cropping them to E (message_gnn_decoder.py:92-118).  This build aggregates the normalized
cliques as group means and any other matrix as a sparse bmm over its nonzeros (CSR plan, fp32).
Oracle: oracle.gnn_forward_dense, the reference's dense formulation restated (pinned to the
reference fixture in tests/test_oracle_golden.py).  Tolerance (stated, fp32): |dprobs| <= 2e-5
for normalized matrices; 1e-4 for the unnormalized clique (sums of up to 23 features)."""
import numpy as np
import pytest
import torch

from conftest import code_path

from ldpc_neural_decoder.models import create_message_gnn_decoder
from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix

pytestmark = pytest.mark.gpu


def _setup(hidden, cuda, seed=0):
    torch.manual_seed(seed)
    base = load_base_matrix(code_path(4))
    H = expand_base_matrix(base, 4)
    dec, conv = create_message_gnn_decoder(H, num_iterations=3, hidden_dim=hidden, base_graph=base, Z=4)
    with torch.no_grad():
        for p in dec.parameters():
            p.mul_(0.5)
    llr = torch.randn(6, H.shape[1], generator=torch.Generator().manual_seed(seed + 1)) * 2 + 1
    return base, H, dec.to(cuda), conv, llr


def _check(dec, conv, oracle_mod, llr, Av, Ac, types, cuda, tol):
    with torch.no_grad():
        p = dec(llr.to(cuda), conv.message_to_var_index(), types, Av, Ac).cpu().numpy()
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    ref = oracle_mod.gnn_forward_dense(sd, llr, conv.edge_var, llr.shape[1], Av.cpu(), Ac.cpu(), types).numpy()
    np.testing.assert_allclose(p, ref, atol=tol)
    return p


@pytest.mark.parametrize("hidden", [64, 16])
def test_padded_and_cropped_adjacency(cuda, oracle_mod, hidden):
    base, H, dec, conv, llr = _setup(hidden, cuda)
    types = conv.get_message_types(base, 4)
    Av, Ac = conv.var_to_check_adjacency, conv.check_to_var_adjacency
    E = Av.shape[0]
    # larger: the reference crops back to the top-left (E, E) block = the cliques again
    big_v, big_c = torch.rand(E + 6, E + 6), torch.rand(E + 6, E + 6)
    big_v[:E, :E], big_c[:E, :E] = Av, Ac
    p_big = _check(dec, conv, oracle_mod, llr, big_v, big_c, types, cuda, 2e-5)
    p_ref = _check(dec, conv, oracle_mod, llr, Av.clone(), Ac.clone(), types, cuda, 2e-5)
    np.testing.assert_allclose(p_big, p_ref, atol=2e-5)
    # smaller: zero rows / columns for the last messages (a general matrix: the CSR plan)
    _check(dec, conv, oracle_mod, llr, Av[:E - 20, :E - 20].clone(), Ac[:E - 20, :E - 20].clone(), types, cuda, 2e-5)


def test_non_clique_adjacency(cuda, oracle_mod):
    """An unnormalized clique (A + I, 0/1) on the variable side and the normalized check matrix:
    mixed pairs run as two CSR matrices."""
    base, H, dec, conv, llr = _setup(64, cuda, seed=3)
    ev = torch.as_tensor(conv.edge_var.astype(np.int64))
    Av = (ev.view(-1, 1) == ev.view(1, -1)).float()
    _check(dec, conv, oracle_mod, llr, Av, conv.check_to_var_adjacency.clone(), conv.get_message_types(base, 4),
           cuda, 1e-4)


def test_general_adjacency_refusals(cuda):
    base, H, dec, conv, llr = _setup(64, cuda)
    Av = conv.var_to_check_adjacency[:-3, :-3].clone()
    Ac = conv.check_to_var_adjacency[:-3, :-3].clone()
    args = (llr.to(cuda), conv.message_to_var_index(), None, Av, Ac)
    dec.precision = "bf16"
    with pytest.raises(NotImplementedError):
        with torch.no_grad():
            dec(*args)
    dec.precision = "fp32"
    with pytest.raises(AttributeError):
        dec(llr.to(cuda), conv.message_to_var_index(), None, None, None)
