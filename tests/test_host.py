"""Host-side logic and the C-ABI library, without a GPU: the library loads and exports every
symbol of include/ldpc_amd.h; the Python drop-in layer's setup code matches the reference."""
import os
import re

import numpy as np
import pytest
import torch

from conftest import ROOT, code_path, golden

from ldpc_neural_decoder import _native as N
from ldpc_neural_decoder.models import message_gnn_decoder as MGD
from ldpc_neural_decoder.utils import ldpc_utils


def header_symbols():
    src = open(os.path.join(ROOT, "include", "ldpc_amd.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(ldpc_[a-z0-9_]+)\s*\(", src)))


def test_library_exports_every_header_symbol():
    lib = N.lib()
    syms = header_symbols()
    assert len(syms) >= 15
    assert lib.missing == ()
    for s in syms:
        assert hasattr(lib._handle, s), s
        assert s in N.SIGNATURES, f"{s} not bound in _native.SIGNATURES"
    assert lib.ldpc_version().decode().startswith("ldpc_amd")


def test_absent_symbol_raises_when_called():
    """An older library (A/B runs) loads; an entry point it lacks raises NativeError on use."""
    lib = N._Lib(N.lib()._handle, ["ldpc_not_in_this_build"])
    assert lib.ldpc_version().decode().startswith("ldpc_amd")
    with pytest.raises(N.NativeError, match="ldpc_not_in_this_build"):
        lib.ldpc_not_in_this_build(1, 2)


def test_library_is_gfx950():
    blob = open(N.LIB_PATH, "rb").read()
    assert b"gfx950" in blob


def test_no_gpu_means_loud_failure():
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(N.NativeError):
        N.device_of(None)


def test_weights_size_formula():
    H, T, L = 64, 4, 5
    want = 2 * H + L * (T * H + 2 * (2 * H * H + H + H * H + H) + H + 1)
    assert N.lib().ldpc_gnn_weights_size(H, T, L) == want
    dec = MGD.MessageGNNDecoder(788, L, H, T)
    n = sum(p.numel() for n_, p in dec.named_parameters() if not n_.startswith("output_layer"))
    assert n == want


@pytest.mark.parametrize("z", [4, 32])
def test_load_and_expand(z):
    c = golden(f"codes_z{z}.npz")
    base = ldpc_utils.load_base_matrix(code_path(z))
    assert base.dtype == torch.float32
    H = ldpc_utils.expand_base_matrix(base, z)
    assert H.dtype == torch.float32 and tuple(H.shape) == tuple(c["H_shape"])
    r, cc = np.nonzero(H.numpy())
    assert np.array_equal(r, c["H_rows"]) and np.array_equal(cc, c["H_cols"])


@pytest.mark.parametrize("z", [4, 32])
def test_tanner_to_message_graph(z):
    c = golden(f"codes_z{z}.npz")
    base = ldpc_utils.load_base_matrix(code_path(z))
    H = ldpc_utils.expand_base_matrix(base, z)
    conv = MGD.TannerToMessageGraph(H)
    assert conv.messages == [tuple(x) for x in c["messages"].tolist()]
    assert np.array_equal(conv.get_message_types(base, z).numpy(), c["message_types"])
    assert conv.get_message_types().sum() == 0
    E = len(conv.messages)
    assert conv.var_to_messages[0] == [i for i, (v, _) in enumerate(conv.messages) if v == 0]
    if z == 4:  # the dense matrices are E x E; check them at the small size
        Av = conv.var_to_check_adjacency.numpy()
        np.testing.assert_allclose(np.diag(Av), c["Av_diag"], rtol=1e-6)
        np.testing.assert_allclose(Av.sum(1), c["Av_rowsum"], rtol=1e-5)
        Ac = conv.check_to_var_adjacency.numpy()
        np.testing.assert_allclose(np.diag(Ac), c["Ac_diag"], rtol=1e-6)
        m = conv.message_to_var_mapping
        assert m.shape == (E, H.shape[1]) and m.sum() == E


def test_groups_from_adjacency_probe():
    base = ldpc_utils.load_base_matrix(code_path(4))
    H = ldpc_utils.expand_base_matrix(base, 4)
    conv = MGD.TannerToMessageGraph(H)
    E = len(conv.messages)
    A = conv.var_to_check_adjacency.clone()  # untagged copy -> derived by probing
    labels, n = MGD._groups_from_adjacency(A, E)
    ev = conv.edge_var
    # same partition as the variables (labels may be renumbered)
    assert n == len(np.unique(ev))
    for g in np.unique(labels)[:50]:
        assert len(np.unique(ev[labels == g])) == 1
    bad = A.clone()
    bad[0, 5] += 0.3
    with pytest.raises(NotImplementedError):
        MGD._groups_from_adjacency(bad, E)
    with pytest.raises(AttributeError):
        MGD._groups_from_adjacency(None, E)


def test_message_types_and_mapping_rules():
    t = MGD._types_for(torch.tensor([5, -2, 1]), 5, 4, "cpu")
    assert t.tolist() == [3, 0, 1, 0, 0]            # clamp + zero-pad (MGD:68-81)
    assert MGD._types_for(None, 3, 4, "cpu").tolist() == [0, 0, 0]
    assert MGD._types_for(torch.arange(6), 4, 9, "cpu").tolist() == [0, 1, 2, 3]  # truncate
    onehot = torch.zeros(4, 3).long()
    onehot[torch.arange(4), torch.tensor([0, 1, 0, 2])] = 1
    assert MGD._io_mapping(onehot, 4, 3, "cpu").tolist() == [1, 0, 1, 0]  # column-0 quirk
    assert MGD._io_mapping(torch.tensor([0, 2, -1, 1]), 4, 3, "cpu").tolist() == [0, 2, 2, 1]
    with pytest.raises(IndexError):
        MGD._io_mapping(onehot.float(), 4, 3, "cpu")  # the reference's float-mapping failure
    with pytest.raises(IndexError):
        MGD._io_mapping(torch.tensor([0, 1, 2, 3]), 4, 3, "cpu")


def test_checkpoint_roundtrip(tmp_path):
    """saved_models schema (trainer.py:344-350, run_comparison_all.py:124-143)."""
    f = golden("gnn_z4.npz")
    ck = torch.load(os.path.join(ROOT, "tests", "golden", "gnn_z4_ckpt.pt"), weights_only=True)
    keys = list(ck["model_state_dict"].keys())
    assert keys == list(f["state_keys"])
    base = ldpc_utils.load_base_matrix(code_path(4))
    H = ldpc_utils.expand_base_matrix(base, 4)
    dec, conv = MGD.create_message_gnn_decoder(H, num_iterations=5, hidden_dim=64, base_graph=base, Z=4)
    assert list(dec.state_dict().keys()) == keys
    dec.load_state_dict(ck["model_state_dict"])
    dec2, _ = MGD.load_message_gnn_model(os.path.join(ROOT, "tests", "golden", "gnn_z4_ckpt.pt"), H, "cpu")
    for (k, a), (_, b) in zip(dec.state_dict().items(), dec2.state_dict().items()):
        assert torch.equal(a, b), k
