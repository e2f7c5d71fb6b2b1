"""Native GNN backward (csrc/gnn_train.hip) vs torch autograd through the CPU oracle (GPU).

The reference trains with torch autograd (trainer.py:93-99: loss.backward() through
MessageGNNDecoder.forward + BCE, message_gnn_decoder.py:314).  The oracle's gnn_forward is the
same math in torch fp32 ops, so autograd on it gives the reference gradients.

Tolerance (floating point, stated): per parameter tensor, max |g - g_ref| <= 1e-3 * max|g_ref|
+ 1e-6.  Both sides are fp32; they differ only in summation order (segment sums vs index_add,
per-row fma chains vs MKL GEMMs), which leaves ~1e-6 relative error per layer."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import code_path

from ldpc_neural_decoder.models import create_message_gnn_decoder
from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix

pytestmark = pytest.mark.gpu
RTOL = 1e-3


def _setup(z, layers, hidden, B, seed=0, scale=0.5):
    torch.manual_seed(seed)
    base = load_base_matrix(code_path(z))
    H = expand_base_matrix(base, z)
    dec, conv = create_message_gnn_decoder(H, num_iterations=layers, hidden_dim=hidden, base_graph=base, Z=z)
    with torch.no_grad():
        for p in dec.parameters():
            p.mul_(scale)
    types = conv.get_message_types(base, z)
    llr = torch.randn(B, H.shape[1]) * 2 + 1.0
    gt = (torch.rand(B, H.shape[1]) < 0.3).float()
    return base, H, dec, conv, types, llr, gt


def _oracle_grads(oracle_mod, dec, conv, H, types, llr, gt):
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in dec.state_dict().items()}
    ev, ec = conv.edge_var, conv.edge_chk
    probs, loss = oracle_mod.gnn_forward(sd, llr, ev, ev, ec, H.shape[1], H.shape[0], types, ground_truth=gt)
    loss.backward()
    return probs.detach(), loss.detach(), {k: v.grad for k, v in sd.items()}


def _check(dec, ref_grads):
    seen = 0
    for name, p in dec.named_parameters():
        g_ref = ref_grads[name]
        if g_ref is None:
            assert p.grad is None, f"{name}: reference has no gradient, native has one"
            continue
        assert p.grad is not None, f"{name}: missing gradient"
        g = p.grad.detach().cpu()
        err = float((g - g_ref).abs().max())
        bound = RTOL * float(g_ref.abs().max()) + 1e-6
        assert err <= bound, f"{name}: max err {err:.3e} > {bound:.3e}"
        seen += 1
    return seen


@pytest.mark.parametrize("proj", ["1", "0", "serial", "fp32mfma", "recompute", "recompute-serial"])
@pytest.mark.parametrize("z,layers,hidden,B", [(4, 3, 64, 8), (4, 2, 32, 5), (32, 2, 64, 2)])
def test_backward_matches_autograd(cuda, oracle_mod, monkeypatch, z, layers, hidden, B, proj):
    """(proj: the H = 64 backward from the projected group rows the forward saved -- GEMM1 over c,
    the group part of dz once per group -- or, LDPC_GNN_TRAIN_PROJ=0, per message over [c; g];
    "serial": LDPC_GNN_TRAIN_OVERLAP=0; "fp32mfma": the backward MLP on fp32 MFMA instead of bf16x6
    splits, LDPC_GNN_TRAIN_S6=0; "recompute": LDPC_GNN_SAVED_PROJ=0, the backward recomputes the
    projections on the side stream, "recompute-serial" in line; same bar)"""
    monkeypatch.setenv("LDPC_GNN_TRAIN_PROJ", "0" if proj == "0" else "1")
    monkeypatch.setenv("LDPC_GNN_TRAIN_OVERLAP", "0" if proj.endswith("serial") else "1")
    monkeypatch.setenv("LDPC_GNN_TRAIN_S6", "0" if proj == "fp32mfma" else "1")
    monkeypatch.setenv("LDPC_GNN_SAVED_PROJ", "0" if proj.startswith("recompute") else "1")
    base, H, dec, conv, types, llr, gt = _setup(z, layers, hidden, B)
    ref_p, ref_loss, ref_g = _oracle_grads(oracle_mod, dec, conv, H, types, llr, gt)
    dec = dec.to(cuda)
    probs, loss = dec(llr.to(cuda), conv.message_to_var_index(), types, conv.var_to_check_adjacency,
                      conv.check_to_var_adjacency, ground_truth=gt.to(cuda))
    assert probs.requires_grad and loss.requires_grad
    np.testing.assert_allclose(probs.detach().cpu().numpy(), ref_p.numpy(), atol=2e-5)
    assert abs(loss.item() - ref_loss.item()) < 1e-5
    loss.backward()
    n = _check(dec, ref_g)
    assert n == 2 + 9 * layers + 2  # every used parameter compared
    # unused: output_projection of the non-last layers, output_layer
    assert dec.gnn_layers[0].output_projection.weight.grad is None
    assert dec.output_layer.weight.grad is None


def test_sgd_steps_track_reference(cuda, oracle_mod):
    """Three SGD steps with the trainer's optimizer settings (trainer.py:70: momentum 0.9,
    weight decay 1e-4) on the native path and on the oracle give the same parameters."""
    base, H, dec, conv, types, llr, gt = _setup(4, 2, 32, 6, seed=1)
    ref = {k: v.detach().clone().requires_grad_(True) for k, v in dec.state_dict().items()}
    used = [k for k in ref if not k.startswith("output_layer") and
            not (k.startswith("gnn_layers.0.output_projection"))]
    opt_ref = torch.optim.SGD([ref[k] for k in used], lr=0.05, momentum=0.9, weight_decay=1e-4)
    dec = dec.to(cuda)
    opt = torch.optim.SGD(dec.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    ev, ec = conv.edge_var, conv.edge_chk
    for step in range(3):
        opt_ref.zero_grad()
        _, loss_r = oracle_mod.gnn_forward(ref, llr, ev, ev, ec, H.shape[1], H.shape[0], types, ground_truth=gt)
        loss_r.backward()
        opt_ref.step()
        opt.zero_grad()
        _, loss = dec(llr.to(cuda), conv.message_to_var_index(), types, conv.var_to_check_adjacency,
                      conv.check_to_var_adjacency, ground_truth=gt.to(cuda))
        loss.backward()
        opt.step()
        assert abs(loss.item() - loss_r.item()) < 1e-4 * max(1.0, abs(loss_r.item()))
    sd = dec.state_dict()
    for k in used:
        np.testing.assert_allclose(sd[k].cpu().numpy(), ref[k].detach().numpy(), rtol=1e-3, atol=1e-5)


def test_no_grad_path_unchanged(cuda):
    """Inference (no grad) keeps the fast path: same probs, no graph."""
    base, H, dec, conv, types, llr, gt = _setup(4, 2, 64, 4)
    dec = dec.to(cuda)
    args = (llr.to(cuda), conv.message_to_var_index(), types, conv.var_to_check_adjacency,
            conv.check_to_var_adjacency)
    with torch.no_grad():
        p0 = dec(*args)
    p1 = dec(*args)
    assert not p0.requires_grad and p1.requires_grad
    np.testing.assert_allclose(p0.cpu().numpy(), p1.detach().cpu().numpy(), atol=1e-6)


@pytest.mark.parametrize("z,layers,hidden,B", [(4, 3, 64, 8), (4, 2, 32, 5), (32, 3, 64, 2)])
def test_deep_supervision_matches_autograd(cuda, oracle_mod, z, layers, hidden, B):
    """forward_all_layers (every layer's output through the last output_projection) and the
    backward of a loss over all of them (ldpc_gnn_layer_probs / ldpc_gnn_backward_ds) vs torch
    autograd through the oracle's all_layers forward.  Same tolerance as above.  Parity unpinned:
    the reference has no per-layer loss; the oracle restates its forward and head."""
    base, H, dec, conv, types, llr, gt = _setup(z, layers, hidden, B, seed=3)
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in dec.state_dict().items()}
    ev, ec = conv.edge_var, conv.edge_chk
    wts = torch.linspace(0.5, 1.0, layers)
    ref_p = oracle_mod.gnn_forward(sd, llr, ev, ev, ec, H.shape[1], H.shape[0], types, all_layers=True)
    ref_loss = sum(w * F.binary_cross_entropy(ref_p[i], gt) for i, w in enumerate(wts))
    ref_loss.backward()
    ref_g = {k: v.grad for k, v in sd.items()}
    dec = dec.to(cuda)
    p = dec.forward_all_layers(llr.to(cuda), conv.message_to_var_index(), types, conv.var_to_check_adjacency,
                               conv.check_to_var_adjacency)
    assert p.shape == (layers, B, H.shape[1])
    np.testing.assert_allclose(p.detach().cpu().numpy(), ref_p.detach().numpy(), atol=2e-5)
    g = gt.to(cuda)
    loss = sum(w * F.binary_cross_entropy(p[i], g) for i, w in enumerate(wts.tolist()))
    assert abs(loss.item() - ref_loss.item()) < 1e-4
    loss.backward()
    assert _check(dec, ref_g) == 2 + 9 * layers + 2
    # the same final probs as forward()
    with torch.no_grad():
        q = dec(llr.to(cuda), conv.message_to_var_index(), types, conv.var_to_check_adjacency,
                conv.check_to_var_adjacency)
    np.testing.assert_allclose(q.cpu().numpy(), p[-1].detach().cpu().numpy(), atol=2e-6)


@pytest.mark.parametrize("hidden", [96, 128, 200, 256])
def test_wide_hidden_matches_autograd(cuda, oracle_mod, hidden):
    """hidden_dim past 64 (message_gnn_decoder.py:22 takes any width): the training forward on
    gnn_mlp_tiled_kernel (never the wide MFMA path: gnn.hip carve(train)), the backward
    on train_mlp_bwd_wide_kernel, which recomputes the forward's products in the same fma order, and
    the tiled weight-gradient reductions (64 gradient rows x 128 columns per launch), against
    autograd through the oracle.  96 and 200 leave a partial 64-unit chunk.  Same tolerance as
    above; inference (no grad: the wide MFMA path where H = 32 k) gives the same probs at the
    forward bar."""
    base, H, dec, conv, types, llr, gt = _setup(4, 2, hidden, 3, seed=5)
    ref_p, ref_loss, ref_g = _oracle_grads(oracle_mod, dec, conv, H, types, llr, gt)
    dec = dec.to(cuda)
    args = (llr.to(cuda), conv.message_to_var_index(), types, conv.var_to_check_adjacency,
            conv.check_to_var_adjacency)
    probs, loss = dec(*args, ground_truth=gt.to(cuda))
    np.testing.assert_allclose(probs.detach().cpu().numpy(), ref_p.numpy(), atol=2e-5)
    assert abs(loss.item() - ref_loss.item()) < 1e-5
    loss.backward()
    assert _check(dec, ref_g) == 2 + 9 * 2 + 2
    with torch.no_grad():
        q = dec(*args)
    np.testing.assert_allclose(q.cpu().numpy(), probs.detach().cpu().numpy(), atol=2e-5)


@pytest.mark.parametrize("hidden", [320, 512])
def test_training_past_256_matches_autograd(cuda, oracle_mod, hidden):
    """Past H = 256 (the reference trains any width, message_gnn_decoder.py:22, :162): the training
    forward runs gnn_mlp_tiled_kernel (fma chains in k order, one wave of 128 H bytes of LDS) and the
    wide backward recomputes those products in the same order.  Same bar as above; inference (no
    grad) gives the same probs."""
    base, H, dec, conv, types, llr, gt = _setup(4, 2, hidden, 3, seed=6)
    ref_p, ref_loss, ref_g = _oracle_grads(oracle_mod, dec, conv, H, types, llr, gt)
    dec = dec.to(cuda)
    args = (llr.to(cuda), conv.message_to_var_index(), types, conv.var_to_check_adjacency,
            conv.check_to_var_adjacency)
    probs, loss = dec(*args, ground_truth=gt.to(cuda))
    np.testing.assert_allclose(probs.detach().cpu().numpy(), ref_p.numpy(), atol=2e-5)
    assert abs(loss.item() - ref_loss.item()) < 1e-5
    loss.backward()
    assert _check(dec, ref_g) == 2 + 9 * 2 + 2
    with torch.no_grad():
        q = dec(*args)
    np.testing.assert_allclose(q.cpu().numpy(), probs.detach().cpu().numpy(), atol=2e-5)


def _dense_grads(oracle_mod, dec, conv, H, types, llr, gt, Av, Ac):
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in dec.state_dict().items()}
    probs = oracle_mod.gnn_forward_dense(sd, llr, conv.edge_var, H.shape[1], Av, Ac, types)
    loss = F.binary_cross_entropy(probs, gt)
    loss.backward()
    return probs.detach(), loss.detach(), {k: v.grad for k, v in sd.items()}


@pytest.mark.parametrize("kind", ["cropped", "padded", "non-clique"])
@pytest.mark.parametrize("hidden", [64, 32, 96])
def test_general_adjacency_backward_matches_autograd(cuda, oracle_mod, kind, hidden):
    """Training through whatever adjacencies the caller passes (trainer.py:90-111 hands the
    converter's matrices to forward, and MessageGNNLayer backpropagates through bmm(A, c) for any A,
    message_gnn_decoder.py:92-118): a matrix smaller than E (zero-padded: the last messages aggregate
    nothing), one larger than E (cropped back), and an unnormalized 0/1 clique beside the normalized
    check matrix.  The general ones run on the CSR plan, whose backward applies A^T over the plan's
    transposed CSR.  Against autograd through oracle.gnn_forward_dense (the reference's dense bmm)
    at the bar above."""
    base, H, dec, conv, types, llr, gt = _setup(4, 2, hidden, 4, seed=11)
    Av0, Ac0 = conv.var_to_check_adjacency, conv.check_to_var_adjacency
    E = Av0.shape[0]
    if kind == "cropped":
        Av, Ac = Av0[:E - 20, :E - 20].clone(), Ac0[:E - 20, :E - 20].clone()
    elif kind == "padded":
        g = torch.Generator().manual_seed(5)
        Av, Ac = torch.rand(E + 6, E + 6, generator=g), torch.rand(E + 6, E + 6, generator=g)
        Av[:E, :E] = Av0 * (torch.rand(E, E, generator=g) < 0.7)  # no longer cliques: the CSR plan
        Ac[:E, :E] = Ac0
    else:
        ev = torch.as_tensor(conv.edge_var.astype(np.int64))
        Av, Ac = (ev.view(-1, 1) == ev.view(1, -1)).float(), Ac0.clone()
    ref_p, ref_loss, ref_g = _dense_grads(oracle_mod, dec, conv, H, types, llr, gt, Av, Ac)
    dec = dec.to(cuda)
    probs, loss = dec(llr.to(cuda), conv.message_to_var_index(), types, Av, Ac, ground_truth=gt.to(cuda))
    tol = 1e-4 if kind == "non-clique" else 2e-5  # unnormalized sums of up to 23 features
    np.testing.assert_allclose(probs.detach().cpu().numpy(), ref_p.numpy(), atol=tol)
    assert abs(loss.item() - ref_loss.item()) < 1e-4
    loss.backward()
    assert _check(dec, ref_g) == 2 + 9 * 2 + 2
