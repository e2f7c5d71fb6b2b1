"""MessageGNN on extreme and non-finite LLRs, and on weights of wide dynamic range (GPU).

The reference runs whatever float32 LLRs it is given through dense torch ops
(message_gnn_decoder.py:190-317): a NaN or inf stays inside its frame (bmm and the MLPs act on
one frame at a time) but reaches every message of that frame in the first layer, because its dense
bmm with the normalized adjacency multiplies it by the zeros too (0 * inf = 0 * NaN = NaN,
MGD:108, :118) -- so such a frame's probs are NaN everywhere (checked on oracle.gnn_forward_dense, the
reference's dense formulation).  Magnitudes far from the training range simply saturate the
sigmoid.
This build's fp32 MLP runs its products as scaled two-term f16 splits whose scales come from each
message column's largest magnitude (csrc/gnn.hpp col_exp / col_exp_w) and from one power of two
per call for the weights; these tests reach that range logic.

Bars (stated):
  * frames of only finite LLRs (0, +-1e4, normal): the fp32 path within 2e-5 of the fp32 oracle
    (the bar of test_gnn_gpu.py); the bf16 path within the bf16 bar (mean |dp| <= 5e-3, >= 99.5 % of
    confident decisions equal);
  * frames holding inf / NaN: every prob NaN, as the reference's dense bmm makes them;
  * no other frame changes by a bit: the batch with the special frames replaced by ordinary ones
    decodes the ordinary frames bit-identically;
  * weights whose rows span 1e-4 .. 1e2 and the trained cfg4 checkpoint at 3 seeds: the split MLP
    stays fp32-accurate (error against the float64 oracle within 2x that of the fp32 MFMA kernel or
    the fp32 oracle, + 1e-7; the bar of test_gnn_depth_gpu.py::test_split_mlp_is_fp32_accurate).
"""
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, code_path

from ldpc_neural_decoder.models import create_message_gnn_decoder
from ldpc_neural_decoder.utils import awgn_llr, expand_base_matrix, load_base_matrix

pytestmark = pytest.mark.gpu
TOL = 2e-5
KINDS = ("zero", "big", "posinf", "neginf", "nan", "mixed")


def _model(z, layers, cuda, seed, precision="fp32", scale=0.5, hidden=64):
    torch.manual_seed(seed)
    base = load_base_matrix(code_path(z))
    H = expand_base_matrix(base, z)
    dec, conv = create_message_gnn_decoder(H, num_iterations=layers, hidden_dim=hidden, base_graph=base, Z=z)
    with torch.no_grad():
        for p in dec.parameters():
            p.mul_(scale)
    dec = dec.to(cuda)
    dec.precision = precision
    return base, H, dec, conv, conv.get_message_types(base, z)


def _native(dec, conv, types, llr, cuda):
    io = conv.message_to_var_index().to(cuda).to(torch.int32)
    with torch.no_grad():
        return dec.native_forward(llr, io, types.to(cuda).to(torch.int32), conv.var_groups, conv.check_groups)


def _oracle(oracle_mod, dec, conv, H, types, llr, dtype=torch.float32):
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    return oracle_mod.gnn_forward(sd, llr.cpu(), conv.edge_var, conv.edge_var, conv.edge_chk, H.shape[1],
                                  H.shape[0], types, dtype=dtype).numpy()


def _special_batch(n, B, seed):
    """B ordinary frames, and a copy where frames 0, 3, 7, ... hold one special kind each."""
    g = torch.Generator().manual_seed(seed)
    base = torch.randn(B, n, generator=g) * 2 + 1.5
    llr = base.clone()
    where = {}
    slots = [0, 3, 7, 10, 14, B - 1]
    for f, kind in zip(slots, KINDS):
        pos = torch.randperm(n, generator=g)[:max(1, n // 50)]
        if kind == "zero":
            llr[f] = 0.0
        elif kind == "big":
            llr[f] = torch.where(torch.rand(n, generator=g) < 0.5, -1e4, 1e4)
        elif kind == "posinf":
            llr[f, pos] = float("inf")
        elif kind == "neginf":
            llr[f, pos] = float("-inf")
        elif kind == "nan":
            llr[f, pos] = float("nan")
        else:  # a few huge LLRs among ordinary ones
            llr[f, pos] = 1e4
        where[f] = kind
    return base, llr, where


def _bf16_ok(p, ref):
    d = np.abs(p - ref)
    sure = np.abs(ref - 0.5) > 0.05
    agree = ((p > 0.5) == (ref > 0.5))[sure].mean() if sure.any() else 1.0
    return d.mean() <= 5e-3 and agree >= 0.995, (float(d.mean()), float(agree))


@pytest.mark.parametrize("precision,z,layers,hidden", [("fp32", 4, 3, 64), ("fp32", 32, 3, 64), ("bf16", 4, 3, 64),
                                                      ("bf16", 32, 3, 64), ("fp32", 4, 3, 128), ("fp32", 4, 3, 40)])
def test_special_llr_frames(cuda, oracle_mod, precision, z, layers, hidden):
    """(hidden 128: the wide row GEMMs, whose per-row f16 scales come from recorded row maxima;
    hidden 40: the tiled fp32 kernel)"""
    base, H, dec, conv, types = _model(z, layers, cuda, seed=21, hidden=hidden)
    dec.precision = precision
    n = H.shape[1]
    ordinary, llr, where = _special_batch(n, 20, seed=z)
    p = _native(dec, conv, types, llr.to(cuda), cuda).cpu().numpy()
    q = _native(dec, conv, types, ordinary.to(cuda), cuda).cpu().numpy()
    others = [f for f in range(llr.shape[0]) if f not in where]
    # no ordinary frame changes by a bit
    assert np.array_equal(p[others], q[others], equal_nan=True)
    ref = _oracle(oracle_mod, dec, conv, H, types, llr)
    dense = None
    if z == 4:  # the reference's own formulation (dense bmm): small enough here
        sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
        dense = oracle_mod.gnn_forward_dense(sd, llr, conv.edge_var, n, conv.var_to_check_adjacency,
                                             conv.check_to_var_adjacency, types).numpy()
    for f in range(llr.shape[0]):
        kind = where.get(f, "ordinary")
        if not bool(torch.isfinite(llr[f]).all()):
            assert np.isnan(p[f]).all(), (f, kind, int(np.isnan(p[f]).sum()))
            if dense is not None:
                assert np.isnan(dense[f]).all(), (f, kind)
            continue
        assert np.isfinite(p[f]).all() and np.isfinite(ref[f]).all(), (f, kind)
        if dense is not None:
            assert float(np.abs(dense[f] - ref[f]).max()) <= TOL, (f, kind)
        if precision == "fp32":
            err = float(np.abs(p[f] - ref[f]).max())
            assert err <= TOL, (f, kind, err)
        else:
            good, stats = _bf16_ok(p[f], ref[f])
            assert good, (f, kind, stats)


def _spread_rows(dec, seed):
    """Scale row r of every W1 (and b1[r]) by s_r = 10^U(-4, 2) and column r of the W2 after it by
    1 / s_r: ReLU commutes with the positive scale, so the decoder computes the same function (its
    probs stay away from 0 / 1), while W1's rows and W2's columns span six orders of magnitude
    under the call's single power-of-two weight scale."""
    g = torch.Generator().manual_seed(seed)
    with torch.no_grad():
        for layer in dec.gnn_layers:
            for seq in (layer.var_to_check_update, layer.check_to_var_update):
                r = (10.0 ** (torch.rand(seq[0].weight.shape[0], generator=g) * 6 - 4)).to(seq[0].weight.device)
                seq[0].weight.mul_(r.view(-1, 1))
                seq[0].bias.mul_(r)
                seq[2].weight.div_(r.view(1, -1))


@pytest.mark.parametrize("weights", ["spread", "trained"])
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_split_mlp_fp32_accurate_wide_range(cuda, oracle_mod, monkeypatch, weights, seed):
    if weights == "trained":
        path = os.path.join(ROOT, "checkpoints", "gnn_bg2_z32_i10_h64.pt")
        ck = torch.load(path, map_location="cpu", weights_only=True)
        base, H, dec, conv, types = _model(32, 10, cuda, seed=seed, scale=1.0)
        dec.load_state_dict(ck["model_state_dict"])
        llr = awgn_llr(64, H.shape[1], seed - 5.0, seed=100 + seed, device=cuda)  # -4 .. -2 dB: probs in flight
    else:
        base, H, dec, conv, types = _model(32, 4, cuda, seed=seed)
        _spread_rows(dec, seed)
        llr = awgn_llr(16, H.shape[1], 1.0, seed=200 + seed, device=cuda)
    exact = _oracle(oracle_mod, dec, conv, H, types, llr, dtype=torch.float64)
    f32 = _oracle(oracle_mod, dec, conv, H, types, llr)
    err = {}
    for split in ("1", "0"):
        monkeypatch.setenv("LDPC_GNN_SPLIT", split)
        err[split] = float(np.abs(_native(dec, conv, types, llr, cuda).cpu().numpy() - exact).max())
    ref_err = float(np.abs(f32 - exact).max())
    unsure = float((np.abs(exact - 0.5) < 0.49).mean())
    print(f"{weights} seed {seed}: split {err['1']:.3e}  fp32-mfma {err['0']:.3e}  oracle-f32 {ref_err:.3e}  "
          f"(probs within 0.49 of 0.5: {unsure:.3f})")
    assert unsure > (0.01 if weights == "spread" else 0.001)  # the outputs are not all saturated
    if weights == "spread":  # beyond the splits' range: the decoder chose the fp32-MFMA products
        assert not dec._split_ok
    else:
        assert dec._split_ok
    assert err["1"] <= 2 * max(err["0"], ref_err) + 1e-7, (err, ref_err)


@pytest.mark.parametrize("weights", ["normal", "spread"])
@pytest.mark.parametrize("hidden", [128, 96, 192, 224])
def test_wide_split_fp32_accurate(cuda, oracle_mod, weights, hidden):
    """hidden_dim 96 / 128 / 192 (csrc/gnn_wide.hip's fused MLP: c split per row from its exact
    largest |c|, relu(h) per row and hidden slice under a running exponent) and 224 (the row GEMMs:
    each input row scaled by the largest |value| its producer recorded), both on scaled two-term f16
    splits, are fp32-accurate -- error against the float64 oracle within 2x the fp32 oracle's own,
    + 1e-7; with weights beyond the splits' range the decoder takes the three-term bf16 row GEMMs
    (LDPC_GNN_FP32_PRODUCTS), at the same bar."""
    base, H, dec, conv, types = _model(32, 4, cuda, seed=40 + hidden)
    from ldpc_neural_decoder.models import create_message_gnn_decoder as _c
    torch.manual_seed(40 + hidden)
    dec, conv = _c(H, num_iterations=4, hidden_dim=hidden, base_graph=base, Z=32)
    with torch.no_grad():
        for p in dec.parameters():
            p.mul_(0.5)
    dec = dec.to(cuda)
    if weights == "spread":
        _spread_rows(dec, hidden)
    llr = awgn_llr(24, H.shape[1], 1.0, seed=300 + hidden, device=cuda)
    exact = _oracle(oracle_mod, dec, conv, H, types, llr, dtype=torch.float64)
    f32 = _oracle(oracle_mod, dec, conv, H, types, llr)
    got = _native(dec, conv, types, llr, cuda).cpu().numpy()
    assert dec._split_ok == (weights == "normal")
    err, ref_err = float(np.abs(got - exact).max()), float(np.abs(f32 - exact).max())
    unsure = float((np.abs(exact - 0.5) < 0.49).mean())
    print(f"H={hidden} {weights}: native {err:.3e}  oracle-f32 {ref_err:.3e}  (unsaturated {unsure:.3f})")
    assert unsure > 0.01
    assert err <= 2 * ref_err + 1e-7, (err, ref_err)


@pytest.mark.parametrize("hidden", [96, 128, 192])
def test_wide_fused_hidden_slice_scales(cuda, oracle_mod, hidden):
    """The fused wide MLP (csrc/gnn_wide.hip gnn_wide_mlp_kernel) splits relu(h) per row and hidden
    slice of 32 units under a running exponent that only moves down, rescaling y's accumulators when
    a later slice holds larger values.  Rows of W1 (and b1) scaled by 2^U(-6, 6), the matching
    columns of W2 by the inverse (the same function): the slices' maxima then differ by up to 2^12
    inside the splits' range (the fused path runs), and the result stays fp32-accurate -- within 2x
    the fp32 oracle's own error against float64, + 1e-7."""
    base, H, dec, conv, types = _model(32, 4, cuda, seed=50 + hidden)
    from ldpc_neural_decoder.models import create_message_gnn_decoder as _c
    torch.manual_seed(50 + hidden)
    dec, conv = _c(H, num_iterations=4, hidden_dim=hidden, base_graph=base, Z=32)
    g = torch.Generator().manual_seed(hidden)
    with torch.no_grad():
        for p in dec.parameters():
            p.mul_(0.5)
        for layer in dec.gnn_layers:
            for seq in (layer.var_to_check_update, layer.check_to_var_update):
                r = 2.0 ** torch.floor(torch.rand(seq[0].weight.shape[0], generator=g) * 12 - 6)
                seq[0].weight.mul_(r.view(-1, 1))
                seq[0].bias.mul_(r)
                seq[2].weight.div_(r.view(1, -1))
    dec = dec.to(cuda)
    llr = awgn_llr(24, H.shape[1], 1.0, seed=500 + hidden, device=cuda)
    exact = _oracle(oracle_mod, dec, conv, H, types, llr, dtype=torch.float64)
    f32 = _oracle(oracle_mod, dec, conv, H, types, llr)
    got = _native(dec, conv, types, llr, cuda).cpu().numpy()
    assert dec._split_ok  # inside the splits' range: the fused MLP ran
    err, ref_err = float(np.abs(got - exact).max()), float(np.abs(f32 - exact).max())
    unsure = float((np.abs(exact - 0.5) < 0.49).mean())
    print(f"H={hidden}: native {err:.3e}  oracle-f32 {ref_err:.3e}  (unsaturated {unsure:.3f})")
    assert unsure > 0.01
    assert err <= 2 * ref_err + 1e-7, (err, ref_err)
