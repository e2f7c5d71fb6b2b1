"""HIP index-gather layers (csrc/layers.hip) vs the reference's golden vectors and the oracle (GPU).

Tolerances (floating point, stated): CheckLayer forward bit-exact (signs and a min: no rounding);
ResidualLayer forward bit-exact (same fp32 operation sequence); VariableLayer forward and every
gradient within 1e-5 relative (summation order of the gathered terms / of the scatter-adds
differs from torch's reductions); OutputLayer within 2e-6 absolute (expf/log1pf vs SLEEF)."""
import numpy as np
import pytest
import torch

from conftest import code_path, golden

from ldpc_neural_decoder.models import CheckLayer, OutputLayer, ResidualLayer, VariableLayer
from ldpc_neural_decoder.utils import create_LLR_mapping, expand_base_matrix, load_base_matrix

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def fx():
    return golden("layers_z4.npz")


def t(a, dev, grad=False):
    x = torch.from_numpy(np.asarray(a)).to(dev)
    return x.requires_grad_(True) if grad else x


def close(a, b, rtol=1e-5, atol=1e-6):
    np.testing.assert_allclose(a.detach().cpu().numpy(), b, rtol=rtol, atol=atol)


def test_check_layer(cuda, fx):
    x = t(fx["x"], cuda, True)
    out = CheckLayer()(x, torch.from_numpy(fx["check_LLR"]))
    assert np.array_equal(out.detach().cpu().numpy(), fx["check_out"])
    (out * t(fx["check_grad_out"], cuda)).sum().backward()
    close(x.grad, fx["check_grad_in"])


def test_variable_layer(cuda, fx):
    llr, msgs = t(fx["llr"], cuda, True), t(fx["check_out"], cuda, True)
    out = VariableLayer()(llr, msgs, torch.from_numpy(fx["var_LLR"]))
    close(out, fx["var_out"], atol=1e-5)
    (out * t(fx["var_grad_out"], cuda)).sum().backward()
    close(msgs.grad, fx["var_grad_msgs"], atol=1e-5)
    close(llr.grad, fx["var_grad_llr"], rtol=0, atol=0)


def test_residual_layer(cuda, fx):
    E = fx["x"].shape[1]
    res = ResidualLayer(E, depth_L=2).to(cuda)
    with torch.no_grad():
        res.w_ch.copy_(t(fx["res_w_ch"], cuda))
        res.w_res.copy_(t(fx["res_w_res"], cuda))
    prevs = [t(p, cuda, True) for p in fx["res_prev"]]
    cm, llr = t(fx["res_cm"], cuda, True), t(fx["llr"], cuda, True)
    out = res(llr, cm, prevs)
    assert np.array_equal(out.detach().cpu().numpy(), fx["res_out"])
    (out * t(fx["res_grad_out"], cuda)).sum().backward()
    close(res.w_ch.grad, fx["res_grad_w_ch"])
    close(res.w_res.grad, fx["res_grad_w_res"], atol=1e-4)
    close(cm.grad, fx["res_grad_cm"], rtol=0, atol=0)
    close(llr.grad, fx["res_grad_llr"])
    for i in range(2):
        close(prevs[i].grad, fx["res_grad_prev"][i])
    assert prevs[2].grad is None  # beyond depth_L: not part of the graph


def test_output_layer(cuda, fx):
    fin = t(fx["out_final"], cuda, True)
    llr = t(fx["llr"], cuda)
    soft, loss = OutputLayer()(fin, llr, t(fx["out_gt"], cuda))
    close(soft, fx["out_soft"], rtol=0, atol=2e-6)
    close(loss, fx["out_max_loss"], rtol=1e-5, atol=2e-6)
    ((soft * t(fx["out_grad_soft"], cuda)).sum() + (loss * t(fx["out_grad_loss"], cuda)).sum()).backward()
    close(fin.grad, fx["out_grad_final"], atol=2e-6)
    s2, none = OutputLayer()(fin.detach(), llr)
    assert none is None
    close(s2, fx["out_soft_nogt"], rtol=0, atol=2e-6)


def test_unrolled_decoder_z32_vs_oracle(cuda, oracle_mod):
    """A small neural min-sum decoder built from the four layers at BG2 Z=32 (E = 6304), forward
    and backward through 3 iterations, against the same chain on the oracle with autograd."""
    torch.manual_seed(4)
    H = expand_base_matrix(load_base_matrix(code_path(32)), 32)
    _, chk, var, _ = create_LLR_mapping(H.T)
    E, B, iters = chk.shape[0], 4, 3
    llr0 = torch.randn(B, E) * 2 + 1
    gt = (torch.rand(B, E) < 0.1).float()
    w_ch = torch.rand(E) + 0.5
    w_res = torch.tensor([0.5, 0.25])

    def run(layers, dev, w_ch_t, w_res_t):
        ck, vl, rs, ol = layers
        llr = llr0.to(dev)
        v, prev = llr, []
        for _ in range(iters):
            c = ck(v)
            v = rs(llr, vl(llr, c), prev, w_ch_t, w_res_t)
            prev = [v] + prev
        return ol(v, llr, gt.to(dev))

    res = ResidualLayer(E).to(cuda)
    with torch.no_grad():
        res.w_ch.copy_(w_ch)
        res.w_res.copy_(w_res)
    hip_layers = (lambda v: CheckLayer()(v, chk), lambda l, c: VariableLayer()(l, c, var),
                  lambda l, cm, prev, a, b: res(l, cm, prev), lambda f, l, g: OutputLayer()(f, l, g))
    soft, loss = run(hip_layers, cuda, None, None)
    loss.sum().backward()

    w_ch_o, w_res_o = w_ch.clone().requires_grad_(True), w_res.clone().requires_grad_(True)
    ora = (lambda v: oracle_mod.check_layer(v, chk), lambda l, c: oracle_mod.variable_layer(l, c, var),
           lambda l, cm, prev, a, b: oracle_mod.residual_layer(l, cm, prev, a, b),
           lambda f, l, g: oracle_mod.output_layer(f, l, g))
    soft_o, loss_o = run(ora, "cpu", w_ch_o, w_res_o)
    loss_o.sum().backward()
    close(soft, soft_o.detach().numpy(), rtol=1e-4, atol=1e-5)
    close(loss, loss_o.detach().numpy(), rtol=1e-4, atol=1e-5)
    close(res.w_ch.grad, w_ch_o.grad.numpy(), rtol=1e-3, atol=1e-5)
    close(res.w_res.grad, w_res_o.grad.numpy(), rtol=1e-3, atol=1e-4)


@pytest.mark.parametrize("z", [4, 32])
def test_check_layer_groups_equal_gather(cuda, fx, z):
    """Without autograd, CheckLayer runs the per-check kernel (ldpc_check_groups_minsum) on
    create_LLR_mapping's index; its outputs are bit-identical to the per-edge gather kernel, on
    values that hit every rule: exact zeros, v = -1e-10 (sign 0), +-inf, ties, and padding."""
    from ldpc_neural_decoder import _native as N
    from ldpc_neural_decoder.models.layers import _check_groups, _check_index
    H = expand_base_matrix(load_base_matrix(code_path(z)), z)
    _, chk, _, _ = create_LLR_mapping(H.T)
    E = chk.shape[0]
    idx = _check_index(chk, E, cuda)
    assert _check_groups(idx, E) is not None
    g = torch.Generator().manual_seed(z)
    x = torch.randn(67, E, generator=g) * 4.0
    x[:, ::7] = 0.0
    x[:, 3::11] = -1e-10
    x[1::5, 5::13] = float("inf")
    x[2::5, 6::13] = -float("inf")
    x[:, 8::17] = 1.5  # ties within a check
    x[3::5, 9::19] = float("nan")
    x = x.to(cuda)
    with torch.no_grad():
        got = CheckLayer()(x, chk)
    K, n_out = idx.shape
    ref = torch.empty_like(got)
    N.check(N.lib().ldpc_gather_minsum(N.ptr(x), x.shape[0], E, N.ptr(idx), n_out, K, N.ptr(ref), None,
                                       N.stream_ptr(x.device)))
    torch.cuda.synchronize()
    a, b = got.cpu().numpy(), ref.cpu().numpy()
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))  # bitwise, incl. -0.0 and NaN
    if z == 4:  # the reference's own vectors, through the no-autograd path
        with torch.no_grad():
            out = CheckLayer()(t(fx["x"], cuda), torch.from_numpy(fx["check_LLR"]))
        assert np.array_equal(out.cpu().numpy(), fx["check_out"])


@pytest.mark.parametrize("z", [4, 32])
def test_variable_layer_groups_equal_gather(cuda, fx, z):
    """VariableLayer on create_LLR_mapping's index runs the per-variable kernel
    (ldpc_var_groups_sum: frame row in LDS, prefix + tail per run); its outputs are bit-identical
    to the per-edge gather kernel (ldpc_gather_sum), with and without the LLR term, on values with
    exact zeros, -0.0, +-inf and NaN.  An index without that structure keeps the gather."""
    from ldpc_neural_decoder import _native as N
    from ldpc_neural_decoder.models.layers import _check_index, _var_groups, gather_sum
    H = expand_base_matrix(load_base_matrix(code_path(z)), z)
    _, _, var, _ = create_LLR_mapping(H.T)
    E = var.shape[0]
    idx = _check_index(var, E, cuda, compact=True)
    assert _var_groups(idx, E) is not None
    g = torch.Generator().manual_seed(z + 1)
    x = torch.randn(67, E, generator=g) * 4.0
    x[:, ::7] = 0.0
    x[:, 3::11] = -0.0
    x[1::5, 5::13] = float("inf")
    x[2::5, 6::13] = -float("inf")
    x[3::5, 9::19] = float("nan")
    llr = (torch.randn(67, E, generator=g) * 2.0)
    llr[:, 1::9] = -0.0
    x, llr = x.to(cuda), llr.to(cuda)
    K, n_out = idx.shape
    for with_llr in (True, False):
        got = VariableLayer()(llr, x, var) if with_llr else gather_sum(x, idx)
        ref = torch.empty_like(got)
        N.check(N.lib().ldpc_gather_sum(N.ptr(llr) if with_llr else None, N.ptr(x), x.shape[0], E, N.ptr(idx),
                                        n_out, K, N.ptr(ref), N.stream_ptr(x.device)))
        torch.cuda.synchronize()
        a, b = got.detach().cpu().numpy(), ref.cpu().numpy()
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))  # bitwise, incl. -0.0 and NaN
    # a permuted index (rows no longer the ascending run of their variable) falls back to the gather
    perm = torch.flip(idx, dims=[0]).contiguous()
    assert _var_groups(perm, E) is None
    if z == 4:  # the reference's own vectors (grad path: the same forward kernel)
        out = VariableLayer()(t(fx["llr"], cuda), t(fx["check_out"], cuda), torch.from_numpy(fx["var_LLR"]))
        close(out, fx["var_out"], atol=1e-5)


def test_group_kernels_ragged_rows(cuda):
    """The per-check and per-variable kernels on a small hand-built graph whose edge count is not
    a multiple of 4 (the unvectorised staging path) and whose groups have degrees 1..5, against the
    per-edge gather kernels, bitwise (zeros, -0.0, inf and NaN among the values)."""
    from ldpc_neural_decoder import _native as N
    from ldpc_neural_decoder.models.layers import _check_groups, _check_index, _var_groups
    runs = [1, 2, 3, 4, 5, 1, 3]                 # variable runs over edges 0..18 (n = 19)
    n = sum(runs)
    var_rows, s = [], 0
    for d in runs:
        for i in range(s, s + d):
            var_rows.append([j for j in range(s, s + d) if j != i])
        s += d
    checks = [[0, 5, 9, 14], [1, 3, 18], [2, 6, 10, 15, 17], [4, 7], [8, 11, 12, 13, 16]]
    chk_rows = [None] * n
    for c in checks:
        for i in c:
            chk_rows[i] = [j for j in c if j != i]
    K = max(len(r) for r in chk_rows + var_rows)
    pad = lambda rows: torch.tensor([r + [-1] * (K - len(r)) for r in rows], dtype=torch.int64)
    chk, var = pad(chk_rows), pad(var_rows)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(37, n, generator=g) * 3.0
    x[:, ::5] = 0.0
    x[1::3, 2] = -0.0
    x[2::4, 7] = float("inf")
    x[3::6, 11] = float("nan")
    llr = torch.randn(37, n, generator=g)
    x, llr = x.to(cuda), llr.to(cuda)
    cidx = _check_index(chk, n, cuda)
    vidx = _check_index(var, n, cuda, compact=True)
    assert _check_groups(cidx, n) is not None and _var_groups(vidx, n) is not None
    with torch.no_grad():
        got_c = CheckLayer()(x, chk)
        got_v = VariableLayer()(llr, x, var)
    ref_c, ref_v = torch.empty_like(got_c), torch.empty_like(got_v)
    N.check(N.lib().ldpc_gather_minsum(N.ptr(x), 37, n, N.ptr(cidx), n, cidx.shape[0], N.ptr(ref_c), None,
                                       N.stream_ptr(x.device)))
    N.check(N.lib().ldpc_gather_sum(N.ptr(llr), N.ptr(x), 37, n, N.ptr(vidx), n, vidx.shape[0], N.ptr(ref_v),
                                    N.stream_ptr(x.device)))
    torch.cuda.synchronize()
    for a, b in ((got_c, ref_c), (got_v, ref_v)):
        a, b = a.cpu().numpy(), b.cpu().numpy()
        assert np.array_equal(a.view(np.uint32), b.view(np.uint32))


_IDX_F_SCRIPT = r"""
import sys, numpy as np, torch
sys.path[:0] = sys.argv[2:]
from conftest import code_path
from ldpc_neural_decoder.models import CheckLayer
from ldpc_neural_decoder.utils import create_LLR_mapping, expand_base_matrix, load_base_matrix
dev = torch.device("cuda", 0)
out = {}
runs = [1, 2, 3, 4, 5, 1, 3]
n = sum(runs)
checks = [[0, 5, 9, 14], [1, 3, 18], [2, 6, 10, 15, 17], [4, 7], [8, 11, 12, 13, 16]]
rows = [None] * n
for c in checks:
    for i in c:
        rows[i] = [j for j in c if j != i]
K = max(len(r) for r in rows)
graphs = {"ragged": torch.tensor([r + [-1] * (K - len(r)) for r in rows], dtype=torch.int64)}
H = expand_base_matrix(load_base_matrix(code_path(32)), 32)
graphs["z32"] = create_LLR_mapping(H.T)[1]
for name, chk in graphs.items():
    E = chk.shape[0]
    g = torch.Generator().manual_seed(11)
    x = torch.randn(41, E, generator=g) * 3.0
    x[:, ::5] = 0.0
    x[:, 1::9] = -1e-10
    x[1::3, 2::7] = -0.0
    x[2::4, 7::13] = float("inf")
    x[3::6, 11::17] = float("nan")
    with torch.no_grad():
        out[name] = CheckLayer()(x.to(dev), chk).cpu().numpy().view(np.uint32)
np.savez(sys.argv[1], **out)
"""


def test_check_group_kernels_idx_and_global_bit_equal(tmp_path):
    """check_group_idx_kernel (member lists staged in LDS, the default) and check_group_kernel (lists
    from global memory, LDPC_CHECK_IDX_F=0) share one per-check body; run each in a fresh process
    (the switch is read once) on a ragged graph and on BG2 Z=32, with zeros, -1e-10, -0.0, +-inf and
    NaN among the values: bit-equal outputs."""
    import os
    import subprocess
    import sys
    from conftest import ROOT, PKG
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    res = {}
    for f in ("0", "4"):
        path = str(tmp_path / f"idx{f}.npz")
        env = dict(os.environ, LDPC_CHECK_IDX_F=f)
        subprocess.run([sys.executable, "-c", _IDX_F_SCRIPT, path, os.path.join(ROOT, "tests"), PKG, ROOT],
                       env=env, check=True, timeout=120)
        res[f] = np.load(path)
    for name in ("ragged", "z32"):
        assert np.array_equal(res["0"][name], res["4"][name]), name
