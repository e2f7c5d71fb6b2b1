"""Oracle restatement of the index-gather layers (oracle.py) and the product's host-side LLR
mapping vs the reference's golden vectors (tests/golden/layers_z4.npz, made by
tests/golden/make_golden_layers.py).  CPU only."""
import numpy as np
import pytest
import torch

from conftest import code_path, golden

from ldpc_neural_decoder.utils import create_LLR_mapping, expand_base_matrix, get_LLR_indexes, load_base_matrix
from ldpc_neural_decoder.utils import matrix_utils


@pytest.fixture(scope="module")
def fx():
    return golden("layers_z4.npz")


@pytest.fixture(scope="module")
def H4():
    return expand_base_matrix(load_base_matrix(code_path(4)), 4)


def test_mapping_matches_reference(fx, H4):
    m, c, v, o = create_LLR_mapping(H4.T)
    assert np.array_equal(m.numpy(), fx["H_to_LLR_mapping_T"])
    assert np.array_equal(c.numpy(), fx["check_LLR"]) and c.dtype == torch.int64
    assert np.array_equal(v.numpy(), fx["var_LLR"]) and v.dtype == torch.int64
    assert np.array_equal(o.numpy(), fx["output_index"]) and tuple(o.shape) == (1, 788)
    c2, v2 = matrix_utils.get_LLR_indexes(m)
    assert torch.equal(c, c2) and torch.equal(v, v2)
    c3, v3 = get_LLR_indexes(m)
    assert torch.equal(c, c3) and torch.equal(v, v3)
    with pytest.raises(TypeError):  # matrix_utils.py:101 raises in the reference too
        matrix_utils.create_LLR_mapping(H4.T)


def test_oracle_forward_and_grads(oracle_mod, fx, H4):
    _, chk, var, _ = oracle_mod.llr_mapping(H4.numpy())
    x = torch.from_numpy(fx["x"]).requires_grad_(True)
    out = oracle_mod.check_layer(x, chk)
    assert np.array_equal(out.detach().numpy(), fx["check_out"])
    (out * torch.from_numpy(fx["check_grad_out"])).sum().backward()
    np.testing.assert_allclose(x.grad.numpy(), fx["check_grad_in"], rtol=1e-6, atol=1e-6)

    llr = torch.from_numpy(fx["llr"]).requires_grad_(True)
    msgs = torch.from_numpy(fx["check_out"]).requires_grad_(True)
    vo = oracle_mod.variable_layer(llr, msgs, var)
    np.testing.assert_allclose(vo.detach().numpy(), fx["var_out"], rtol=1e-6, atol=1e-5)
    (vo * torch.from_numpy(fx["var_grad_out"])).sum().backward()
    np.testing.assert_allclose(msgs.grad.numpy(), fx["var_grad_msgs"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(llr.grad.numpy(), fx["var_grad_llr"], rtol=0, atol=0)

    w_ch = torch.from_numpy(fx["res_w_ch"]).requires_grad_(True)
    w_res = torch.from_numpy(fx["res_w_res"]).requires_grad_(True)
    prevs = [torch.from_numpy(p).requires_grad_(True) for p in fx["res_prev"]]
    cm = torch.from_numpy(fx["res_cm"])
    ro = oracle_mod.residual_layer(torch.from_numpy(fx["llr"]), cm, prevs, w_ch, w_res)
    assert np.array_equal(ro.detach().numpy(), fx["res_out"])
    (ro * torch.from_numpy(fx["res_grad_out"])).sum().backward()
    np.testing.assert_allclose(w_ch.grad.numpy(), fx["res_grad_w_ch"], rtol=1e-5, atol=1e-5)
    np.testing.assert_allclose(w_res.grad.numpy(), fx["res_grad_w_res"], rtol=1e-5, atol=1e-4)

    fin = torch.from_numpy(fx["out_final"]).requires_grad_(True)
    soft, loss = oracle_mod.output_layer(fin, torch.from_numpy(fx["llr"]), torch.from_numpy(fx["out_gt"]))
    assert np.array_equal(soft.detach().numpy(), fx["out_soft"])
    np.testing.assert_allclose(loss.detach().numpy(), fx["out_max_loss"], rtol=1e-6)
    ((soft * torch.from_numpy(fx["out_grad_soft"])).sum() + (loss * torch.from_numpy(fx["out_grad_loss"])).sum()).backward()
    np.testing.assert_allclose(fin.grad.numpy(), fx["out_grad_final"], rtol=1e-5, atol=1e-6)
