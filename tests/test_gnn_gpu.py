"""HIP message-GNN forward vs the reference's golden outputs and the torch-fp32 oracle (GPU).

Tolerance (floating point, stated): |probs - ref| <= 2e-5 absolute for the fp32 path.  The
reference aggregates with a dense normalized-adjacency bmm and MKL GEMMs, this build with
segment means and the matrix cores: at H = 64 every fp32 product runs as a scaled two-term f16
split (22 significant bits per operand, three f16 MFMA products, fp32 accumulate; within 2x an
fp32 GEMM's error against float64, tests/test_gnn_depth_gpu.py::test_split_mlp_is_fp32_accurate),
in a different summation order, so results agree to float32 rounding, not bitwise."""
import numpy as np
import pytest
import torch

from conftest import code_path, golden

from ldpc_neural_decoder.models import MessageGNNDecoder, create_message_gnn_decoder
from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix

pytestmark = pytest.mark.gpu
TOL = 2e-5


def load_model(z):
    f = golden(f"gnn_z{z}.npz")
    base = load_base_matrix(code_path(z))
    H = expand_base_matrix(base, z)
    dec, conv = create_message_gnn_decoder(H, num_iterations=int(f["num_iterations"]),
                                           hidden_dim=int(f["hidden_dim"]), base_graph=base, Z=z)
    sd = {k[3:]: torch.from_numpy(f[k]) for k in f.files if k.startswith("w__")}
    dec.load_state_dict(sd)
    return f, base, dec, conv, sd


@pytest.mark.parametrize("z", [4, 32])
def test_forward_matches_reference(cuda, z):
    f, base, dec, conv, _ = load_model(z)
    dec = dec.to(cuda)
    llr = torch.from_numpy(f["llr"]).to(cuda)
    types = conv.get_message_types(base, z)
    mv = conv.message_to_var_index()
    Av, Ac = conv.var_to_check_adjacency, conv.check_to_var_adjacency
    p = dec(llr, mv, types, Av, Ac)
    np.testing.assert_allclose(p.detach().cpu().numpy(), f["probs"], atol=TOL)
    p = dec(llr, mv, None, Av, Ac)
    np.testing.assert_allclose(p.detach().cpu().numpy(), f["probs_no_types"], atol=TOL)
    p, loss = dec(llr, mv, types, Av, Ac, ground_truth=torch.from_numpy(f["ground_truth"]).to(cuda))
    assert abs(loss.item() - float(f["loss"])) < 1e-4
    bits = dec.decode(llr, mv, types, Av, Ac)
    ref_p = f["probs"]
    sure = np.abs(ref_p - 0.5) > 1e-4  # decisions away from the threshold must agree
    assert np.array_equal(bits.cpu().numpy()[sure].astype(np.uint8), f["decode_bits"][sure])


def test_2d_mapping_quirk(cuda):
    """The examples pass converter.message_to_var_mapping.long() (run_message_gnn.py:304-310):
    column 0 of the one-hot is used as the variable index (message_gnn_decoder.py:220-226)."""
    f, base, dec, conv, _ = load_model(4)
    dec = dec.to(cuda)
    llr = torch.from_numpy(f["llr"]).to(cuda)
    p = dec(llr, conv.message_to_var_mapping.long(), conv.get_message_types(base, 4),
            conv.var_to_check_adjacency, conv.check_to_var_adjacency)
    np.testing.assert_allclose(p.detach().cpu().numpy(), f["probs_2d_quirk"], atol=TOL)
    with pytest.raises(IndexError):  # the float one-hot fails in the reference too
        dec(llr, conv.message_to_var_mapping, None, conv.var_to_check_adjacency,
            conv.check_to_var_adjacency)


def test_untagged_adjacency_on_device(cuda):
    """Adjacencies that went through .to(device) lose the tag: groups are derived by probing."""
    f, base, dec, conv, _ = load_model(4)
    dec = dec.to(cuda)
    llr = torch.from_numpy(f["llr"]).to(cuda)
    p = dec(llr, conv.message_to_var_index(), conv.get_message_types(base, 4),
            conv.var_to_check_adjacency.to(cuda), conv.check_to_var_adjacency.to(cuda))
    np.testing.assert_allclose(p.detach().cpu().numpy(), f["probs"], atol=TOL)


@pytest.mark.parametrize("B,chunk", [(3, None), (70, 16)])
def test_z32_h64_vs_oracle(cuda, oracle_mod, B, chunk):
    """The MFMA path at the headline code (Z = 32, H = 64, 3 layers, random weights)."""
    torch.manual_seed(0)
    base = load_base_matrix(code_path(32))
    H = expand_base_matrix(base, 32)
    dec, conv = create_message_gnn_decoder(H, num_iterations=3, hidden_dim=64, base_graph=base, Z=32)
    with torch.no_grad():
        for p in dec.parameters():
            p.mul_(0.5)
    dec = dec.to(cuda)
    types = conv.get_message_types(base, 32)
    llr = (torch.randn(B, H.shape[1]) * 2 + 1.5).to(cuda)
    ev, ec = conv.edge_var, conv.edge_chk
    io = conv.message_to_var_index().to(cuda).to(torch.int32)
    vg, cg = conv.var_groups, conv.check_groups
    p = dec.native_forward(llr, io, types.to(cuda).to(torch.int32), vg, cg, chunk=chunk)
    sd = {k: v.cpu() for k, v in dec.state_dict().items()}
    ref = oracle_mod.gnn_forward(sd, llr.cpu(), ev, ev, ec, H.shape[1], H.shape[0], types)
    np.testing.assert_allclose(p.detach().cpu().numpy(), ref.numpy(), atol=TOL)


def test_state_dict_keys_match_reference():
    f = golden("gnn_z4.npz")
    dec = MessageGNNDecoder(788, 5, 64, 4)
    assert list(dec.state_dict().keys()) == list(f["state_keys"])


@pytest.mark.parametrize("z,layers", [(4, 5), (32, 3)])
def test_bf16_path_within_tolerance(cuda, oracle_mod, z, layers):
    """precision="bf16" (cfg5): bf16 feature storage and MFMA operands, fp32 accumulation.
    Stated tolerance vs the fp32 oracle: mean |dp| <= 5e-3, max |dp| <= 0.1, and >= 99.5 % of the
    decisions with |p - 0.5| > 0.05 unchanged."""
    torch.manual_seed(3)
    base = load_base_matrix(code_path(z))
    H = expand_base_matrix(base, z)
    dec, conv = create_message_gnn_decoder(H, num_iterations=layers, hidden_dim=64, base_graph=base, Z=z)
    with torch.no_grad():
        for p in dec.parameters():
            p.mul_(0.5)
    dec = dec.to(cuda)
    dec.precision = "bf16"
    types = conv.get_message_types(base, z)
    llr = (torch.randn(16, H.shape[1]) * 2 + 1.5).to(cuda)
    p = dec(llr, conv.message_to_var_index(), types, conv.var_to_check_adjacency,
            conv.check_to_var_adjacency).cpu().numpy()
    sd = {k: v.cpu() for k, v in dec.state_dict().items()}
    ref = oracle_mod.gnn_forward(sd, llr.cpu(), conv.edge_var, conv.edge_var, conv.edge_chk,
                                 H.shape[1], H.shape[0], types).numpy()
    d = np.abs(p - ref)
    sure = np.abs(ref - 0.5) > 0.05
    agree = ((p > 0.5) == (ref > 0.5))[sure].mean()
    print(f"bf16 z={z}: mean {d.mean():.2e} max {d.max():.2e} agree {agree:.5f}")
    assert d.mean() <= 5e-3 and d.max() <= 0.1 and agree >= 0.995


_KNOB_SCRIPT = r"""
import sys, torch
sys.path.insert(0, sys.argv[1])
from ldpc_neural_decoder.models import create_message_gnn_decoder
from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix
d = torch.load(sys.argv[2], weights_only=True)
base = load_base_matrix(d["code"]); H = expand_base_matrix(base, 32)
dec, conv = create_message_gnn_decoder(H, num_iterations=3, hidden_dim=64, base_graph=base, Z=32)
dec.load_state_dict(d["sd"]); dec = dec.to("cuda")
p = dec(d["llr"].cuda(), conv.message_to_var_index(), conv.get_message_types(base, 32),
        conv.var_to_check_adjacency, conv.check_to_var_adjacency)
torch.save(p.detach().cpu(), sys.argv[3])
"""


def test_fp32_group_mean_variants_bit_identical(cuda, tmp_path):
    """Per-message [c; g] kernels (LDPC_GNN_PROJ=0): the group-tile group-mean kernel and the
    degree-1 skip give the same probs, bit for bit, as the per-group kernel with every Mv row
    written (LDPC_GNN_GM=0 LDPC_GNN_D1=0).  Default (projected) path: its degree-1 message tiles
    (one combined W1v_left + W1v_right weight, rounded once) against every message on its projected
    group row (LDPC_GNN_D1=0): fp32 rounding apart, |dp| <= 1e-5.  The knobs are read once per
    process, so each variant runs in a child process."""
    import os
    import subprocess
    import sys
    base = load_base_matrix(code_path(32))
    H = expand_base_matrix(base, 32)
    torch.manual_seed(3)
    dec, conv = create_message_gnn_decoder(H, num_iterations=3, hidden_dim=64, base_graph=base, Z=32)
    llr = torch.randn(37, H.shape[1]) * 3.0 + 2.0
    torch.save({"code": code_path(32), "sd": dec.state_dict(), "llr": llr}, tmp_path / "in.pt")
    dec = dec.to(cuda)
    p = dec(llr.to(cuda), conv.message_to_var_index(), conv.get_message_types(base, 32),
            conv.var_to_check_adjacency, conv.check_to_var_adjacency).detach().cpu()
    pkg = os.path.dirname(os.path.dirname(os.path.abspath(
        sys.modules["ldpc_neural_decoder"].__file__)))
    def child(name, **knobs):
        env = dict(os.environ, **knobs)
        subprocess.run([sys.executable, "-c", _KNOB_SCRIPT, pkg, str(tmp_path / "in.pt"),
                        str(tmp_path / name)], env=env, check=True, timeout=180)
        return torch.load(tmp_path / name, weights_only=True)

    q_gm = child("gm.pt", LDPC_GNN_PROJ="0")
    q_pergroup = child("pergroup.pt", LDPC_GNN_PROJ="0", LDPC_GNN_GM="0", LDPC_GNN_D1="0")
    assert torch.equal(q_gm, q_pergroup)
    d = (p - child("nod1.pt", LDPC_GNN_D1="0")).abs().max().item()
    print(f"projected path, degree-1 tiles vs none: max |dp| {d:.2e}")
    assert d <= 1e-5
    # round 5: the row walk (check-group sums from the producing MLP, the default) against the tile
    # walk with gathered check means (LDPC_GNN_ROWWALK=0): summation order apart, |dp| <= 1e-5
    d = (p - child("norw.pt", LDPC_GNN_ROWWALK="0")).abs().max().item()
    print(f"row walk vs tile walk: max |dp| {d:.2e}")
    assert d <= 1e-5
