"""BASELINE cfg4 / cfg5 at their real depths and per-GPU batch (GPU).

cfg4: BG2 Z=32 MessageGNN, 10 layers, H=64, T=32, fp32, 32768 frames per GPU.
cfg5: the same code, 15 layers, bf16 message MLP on MFMA, per-frame early termination.

Tolerances (stated):
  * fp32 vs the torch-fp32 oracle (oracle.gnn_forward, a restatement of
    message_gnn_decoder.py:190-317 pinned by tests/golden/gnn_z*.npz): |dprobs| <= 2e-5.  The
    oracle in float64 differs from float32 by <= 1e-7 at these depths, so the bar is the MFMA
    summation order, not error growth over 10 residual layers.
  * bf16 vs the fp32 oracle: the bar of test_gnn_gpu.py::test_bf16_path_within_tolerance (mean
    |dp| <= 5e-3, max <= 0.1, >= 99.5 % of decisions with |p - 0.5| > 0.05 unchanged).
  * full-batch properties are exact: a frame's output depends only on that frame, so chunking and
    batch position must not change a single bit.
"""
import numpy as np
import pytest
import torch

from conftest import code_path

from ldpc_neural_decoder.models import create_message_gnn_decoder
from ldpc_neural_decoder.utils import awgn_llr, expand_base_matrix, load_base_matrix

pytestmark = pytest.mark.gpu
TOL = 2e-5
CFG_BATCH = 32768


def _model(layers, cuda, seed=0, precision="fp32", hidden=64):
    torch.manual_seed(seed)
    base = load_base_matrix(code_path(32))
    H = expand_base_matrix(base, 32)
    dec, conv = create_message_gnn_decoder(H, num_iterations=layers, hidden_dim=hidden, base_graph=base, Z=32)
    with torch.no_grad():
        for p in dec.parameters():
            p.mul_(0.5)
    dec = dec.to(cuda)
    dec.precision = precision
    types = conv.get_message_types(base, 32)
    return base, H, dec, conv, types


def _oracle(oracle_mod, dec, conv, H, types, llr):
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    return oracle_mod.gnn_forward(sd, llr.cpu(), conv.edge_var, conv.edge_var, conv.edge_chk,
                                  H.shape[1], H.shape[0], types).numpy()


def _native(dec, conv, types, llr, cuda, chunk=None):
    io = conv.message_to_var_index().to(cuda).to(torch.int32)
    t = types.to(cuda).to(torch.int32)
    with torch.no_grad():
        return dec.native_forward(llr, io, t, conv.var_groups, conv.check_groups, chunk=chunk)


@pytest.mark.parametrize("split", ["1", "0"])
def test_cfg4_depth_fp32_vs_oracle(cuda, oracle_mod, monkeypatch, split):
    """10-layer fp32 forward at Z=32, H=64 through native_forward, forward() under no_grad and
    decode() (which must take the inference path even with grad enabled).  split: the MLP's fp32
    products as scaled two-term f16 splits on the f16 MFMA (default) or on the fp32 MFMA
    (LDPC_GNN_SPLIT=0); same bar."""
    monkeypatch.setenv("LDPC_GNN_SPLIT", split)
    base, H, dec, conv, types = _model(10, cuda)
    llr = (torch.randn(8, H.shape[1], generator=torch.Generator().manual_seed(4)) * 2 + 1.5).to(cuda)
    ref = _oracle(oracle_mod, dec, conv, H, types, llr)
    p = _native(dec, conv, types, llr, cuda)
    np.testing.assert_allclose(p.cpu().numpy(), ref, atol=TOL)
    args = (llr, conv.message_to_var_index(), types, conv.var_to_check_adjacency, conv.check_to_var_adjacency)
    with torch.no_grad():
        q = dec(*args)
    assert torch.equal(p, q)
    assert torch.is_grad_enabled()
    bits = dec.decode(*args)                    # grad enabled: must not take the training path
    assert not bits.requires_grad
    sure = np.abs(ref - 0.5) > 1e-4
    assert np.array_equal(bits.cpu().numpy()[sure], (ref > 0.5)[sure].astype(np.float32))


def test_rowwalk_staged_check_rows_bitwise(cuda, monkeypatch):
    """The row walk reads each unit's projected check rows from LDS after the unit's first tile
    (default) or from global memory at every tile (LDPC_GNN_PCLDS=0: the kernel that codes with too
    many message types for the staging run): the same values, so the outputs are bit for bit equal."""
    base, H, dec, conv, types = _model(10, cuda, seed=3)
    llr = awgn_llr(512, H.shape[1], 1.0, seed=31, device=cuda)
    p = _native(dec, conv, types, llr, cuda)
    monkeypatch.setenv("LDPC_GNN_PCLDS", "0")
    q = _native(dec, conv, types, llr, cuda)
    assert torch.equal(p, q)


def test_cfg4_full_batch_properties(cuda, oracle_mod):
    """cfg4's per-GPU batch (32768 frames, 10 layers): the (B, E, H) buffers pass 2^31 elements,
    the 48 GB workspace budget chunks the batch.  Chunked (4096) == default chunking, a sub-batch
    decodes identically on its own, probs are finite, and spot frames match the oracle."""
    base, H, dec, conv, types = _model(10, cuda, seed=1)
    llr = awgn_llr(CFG_BATCH, H.shape[1], 2.0, seed=77, device=cuda)
    p = _native(dec, conv, types, llr, cuda)
    assert p.shape == (CFG_BATCH, H.shape[1]) and bool(torch.isfinite(p).all())
    q = _native(dec, conv, types, llr, cuda, chunk=4096)
    assert torch.equal(p, q)
    sub = _native(dec, conv, types, llr[20000:20077].contiguous(), cuda)
    assert torch.equal(sub, p[20000:20077])
    idx = torch.tensor([0, 12345, 20076, CFG_BATCH - 1])
    ref = _oracle(oracle_mod, dec, conv, H, types, llr[idx.to(cuda)])
    np.testing.assert_allclose(p[idx.to(cuda)].cpu().numpy(), ref, atol=TOL)


def test_cfg5_depth_bf16_et_vs_oracle(cuda, oracle_mod):
    """15-layer bf16 path with early termination on, against the fp32 oracle."""
    base, H, dec, conv, types = _model(15, cuda, seed=3, precision="bf16")
    dec.early_termination = True
    llr = (torch.randn(16, H.shape[1], generator=torch.Generator().manual_seed(5)) * 2 + 1.5).to(cuda)
    with torch.no_grad():
        p = dec(llr, conv.message_to_var_index(), types, conv.var_to_check_adjacency,
                conv.check_to_var_adjacency).cpu().numpy()
    ref = _oracle(oracle_mod, dec, conv, H, types, llr)
    assert torch.equal(dec.last_iterations.cpu(), torch.full((16,), 15, dtype=torch.int32))
    d = np.abs(p - ref)
    sure = np.abs(ref - 0.5) > 0.05
    agree = ((p > 0.5) == (ref > 0.5))[sure].mean()
    print(f"bf16 15 layers: mean {d.mean():.2e} max {d.max():.2e} agree {agree:.5f}")
    assert d.mean() <= 5e-3 and d.max() <= 0.1 and agree >= 0.995


def test_cfg5_full_batch_properties(cuda):
    """cfg5's per-GPU batch: 32768 frames, 15 bf16 layers, early termination on.  With random
    weights no decision is a codeword, so every frame runs 15 layers and the outputs equal the
    early-termination-off run bit for bit; chunking and sub-batches change nothing."""
    base, H, dec, conv, types = _model(15, cuda, seed=2, precision="bf16")
    llr = awgn_llr(CFG_BATCH, H.shape[1], 2.0, seed=78, device=cuda)
    dec.early_termination = True
    p = _native(dec, conv, types, llr, cuda)
    it = dec.last_iterations.clone()
    assert bool(torch.isfinite(p).all())
    assert bool(((it >= 1) & (it <= 15)).all())
    dec.early_termination = False
    p_off = _native(dec, conv, types, llr, cuda)
    if bool((it == 15).all()):
        assert torch.equal(p, p_off)
    dec.early_termination = True
    q = _native(dec, conv, types, llr, cuda, chunk=5000)
    assert torch.equal(p, q) and torch.equal(it, dec.last_iterations)
    sub = _native(dec, conv, types, llr[31000:31111].contiguous(), cuda)
    assert torch.equal(sub, p[31000:31111])


def test_split_mlp_is_fp32_accurate(cuda, oracle_mod, monkeypatch):
    """The split MLP (gnn_mlp2s_kernel: scaled two-term f16 splits, 3 MFMAs per product) is
    fp32-accurate: against the float64 oracle its error is within 2x (+1e-7) of the fp32-MFMA
    kernel's and of the float32 oracle's own, at 10 layers, Z=32."""
    base, H, dec, conv, types = _model(10, cuda, seed=5)
    llr = awgn_llr(16, H.shape[1], 1.0, seed=9, device=cuda)
    sd = {k: v.detach().cpu() for k, v in dec.state_dict().items()}
    args = (sd, llr.cpu(), conv.edge_var, conv.edge_var, conv.edge_chk, H.shape[1], H.shape[0], types)
    exact = oracle_mod.gnn_forward(*args, dtype=torch.float64).numpy()
    f32 = oracle_mod.gnn_forward(*args).numpy()
    err = {}
    for split in ("1", "0"):
        monkeypatch.setenv("LDPC_GNN_SPLIT", split)
        err[split] = float(np.abs(_native(dec, conv, types, llr, cuda).cpu().numpy() - exact).max())
    ref_err = float(np.abs(f32 - exact).max())
    assert err["1"] <= 2 * max(err["0"], ref_err) + 1e-7, (err, ref_err)


@pytest.mark.parametrize("hidden,layers", [(128, 10), (96, 6), (192, 4), (256, 3)])
def test_wide_hidden_mfma_vs_oracle(cuda, oracle_mod, hidden, layers):
    """hidden_dim = 32 k other than 64 (message_gnn_decoder.py:22, :162 take any width) on the MFMA
    kernels of gnn_wide.hip (scaled f16 two-term splits: fp32-accurate products; H = 96 / 128 / 192
    through the fused per-tile MLP, 256 through the row GEMMs): BG2 Z=32 against the oracle at the
    H = 64 bar (|dprobs| <= 2e-5), H = 128 at cfg4's 10 layers; a sub-batch decodes bit-identically
    to its rows of the full batch (a frame's output depends on that frame alone)."""
    base, H, dec, conv, types = _model(layers, cuda, seed=hidden, hidden=hidden)
    llr = awgn_llr(6, H.shape[1], 1.0, seed=hidden, device=cuda)
    got = _native(dec, conv, types, llr, cuda).cpu().numpy()
    ref = _oracle(oracle_mod, dec, conv, H, types, llr)
    err = float(np.abs(got - ref).max())
    assert err <= TOL, err
    sub = _native(dec, conv, types, llr[2:5].contiguous(), cuda).cpu().numpy()
    assert np.array_equal(sub, got[2:5])


@pytest.mark.parametrize("hidden", [96, 160, 224])
def test_wide_hidden_multi_tile_walk(cuda, oracle_mod, hidden):
    """H = 96 / 160 / 224: the projection's reduction (K = H; and GEMM1's at 224, where the row GEMMs
    run) has a k-step count that 4 does not divide, so gnn_wgemm_kernel's input ring runs 2 deep there
    (a 4-deep ring fed the next tile permuted chunks).  B = 48 frames at Z=32 give every
    wave several tiles to walk (and the fused MLP several passes at 96 / 160); the oracle checks
    every frame at the H = 64 bar."""
    base, H, dec, conv, types = _model(2, cuda, seed=hidden + 1, hidden=hidden)
    llr = awgn_llr(48, H.shape[1], 1.0, seed=hidden + 2, device=cuda)
    got = _native(dec, conv, types, llr, cuda).cpu().numpy()
    ref = _oracle(oracle_mod, dec, conv, H, types, llr)
    err = float(np.abs(got - ref).max())
    assert err <= TOL, err


@pytest.mark.parametrize("hidden,z,batch", [(128, 32, 1), (192, 32, 2), (96, 4, 1), (128, 4, 3)])
def test_wide_fused_tiny_batches(cuda, oracle_mod, hidden, z, batch):
    """The fused wide MLP (gnn_wide_mlp_kernel) on batches far smaller than its grid: most XCD tile
    ranges hold less than one pass, so workgroups run passes whose waves own no tile (they still
    take every slice's barrier and copy share) and Z = 4 leaves whole workgroups without a tile.
    Every frame against the oracle at the H = 64 bar."""
    torch.manual_seed(hidden + z)
    base = load_base_matrix(code_path(z))
    H = expand_base_matrix(base, z)
    dec, conv = create_message_gnn_decoder(H, num_iterations=3, hidden_dim=hidden, base_graph=base, Z=z)
    with torch.no_grad():
        for p in dec.parameters():
            p.mul_(0.5)
    dec = dec.to(cuda)
    types = conv.get_message_types(base, z)
    llr = awgn_llr(batch, H.shape[1], 1.0, seed=hidden + batch, device=cuda)
    got = _native(dec, conv, types, llr, cuda).cpu().numpy()
    ref = _oracle(oracle_mod, dec, conv, H, types, llr)
    err = float(np.abs(got - ref).max())
    assert err <= TOL, err
