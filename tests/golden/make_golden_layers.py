"""Golden vectors for the index-gather neural-BP layers (models/layers.py) and the var-major edge
mapping (utils/ldpc_utils.py:5-95, utils/matrix_utils.py:12-103) of the reference.

Run ONCE in the build container, where the reference is importable:
    PYTHONPATH=/root/reference PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden_layers.py
It imports the reference package and records, for BG2 Z=4, the mapping tensors and, on seeded
inputs (with exact zeros and padded rows mixed in), the forward outputs of CheckLayer,
VariableLayer, ResidualLayer and OutputLayer plus the gradients torch autograd gives for a
seeded upstream gradient.  Only .npz data is written; the reference itself never travels.
"""
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REF = "/root/reference"
sys.path.insert(0, REF)

from ldpc_neural_decoder.models.layers import CheckLayer, OutputLayer, ResidualLayer, VariableLayer  # noqa: E402
from ldpc_neural_decoder.utils.ldpc_utils import create_LLR_mapping, expand_base_matrix, load_base_matrix  # noqa: E402
from ldpc_neural_decoder.utils import matrix_utils  # noqa: E402


def main():
    torch.manual_seed(2025)
    base = load_base_matrix(os.path.join(REF, "5G LDPC CODES", "NR_2_0_4.txt"))
    H = expand_base_matrix(base, 4)
    HT = H.T.contiguous()
    m_T, chk, var, out_idx = create_LLR_mapping(HT)
    # matrix_utils.create_LLR_mapping raises TypeError at :101 (torch.tensor([row_indices])); its
    # get_LLR_indexes is the same function as ldpc_utils'
    chk2, var2 = matrix_utils.get_LLR_indexes(m_T)
    assert torch.equal(chk, chk2) and torch.equal(var, var2)
    E = chk.shape[0]
    B = 6
    x = torch.randn(B, E) * 3
    x[0, :7] = 0.0            # exact zeros: sign(0 + 1e-10) = 1 and |0| -> 1e10
    x[1, 10:12] = -1e-10      # sign(-1e-10 + 1e-10) = 0
    llr = torch.randn(B, E) * 2

    x_c = x.clone().requires_grad_(True)
    c_out = CheckLayer()(x_c, chk)
    g_c = torch.randn_like(c_out)
    (c_out * g_c).sum().backward()

    llr_v = llr.clone().requires_grad_(True)
    m_v = c_out.detach().clone().requires_grad_(True)
    v_out = VariableLayer()(llr_v, m_v, var)
    g_v = torch.randn_like(v_out)
    (v_out * g_v).sum().backward()

    res = ResidualLayer(E, depth_L=2)
    with torch.no_grad():
        res.w_ch.copy_(torch.rand(E) + 0.5)
        res.w_res.copy_(torch.tensor([0.7, -0.3]))
    prevs = [torch.randn(B, E).requires_grad_(True) for _ in range(3)]  # 3 > depth_L: third unused
    cm = torch.randn(B, E).requires_grad_(True)
    llr_r = llr.clone().requires_grad_(True)
    r_out = res(llr_r, cm, prevs)
    g_r = torch.randn_like(r_out)
    (r_out * g_r).sum().backward()

    fin = (torch.randn(B, E) * 4).requires_grad_(True)
    gt = (torch.rand(B, E) < 0.5).float()
    soft, max_loss = OutputLayer()(fin, llr, gt)
    g_soft = torch.randn_like(soft)
    g_loss = torch.randn_like(max_loss)
    (soft * g_soft).sum().backward(retain_graph=True)
    (max_loss * g_loss).sum().backward()
    soft_nogt, none = OutputLayer()(fin.detach(), llr)
    assert none is None

    np.savez_compressed(
        os.path.join(HERE, "layers_z4.npz"),
        H_to_LLR_mapping_T=m_T.numpy().astype(np.int32), check_LLR=chk.numpy(), var_LLR=var.numpy(),
        output_index=out_idx.numpy(), x=x.numpy(), llr=llr.numpy(),
        check_out=c_out.detach().numpy(), check_grad_out=g_c.numpy(), check_grad_in=x_c.grad.numpy(),
        var_out=v_out.detach().numpy(), var_grad_out=g_v.numpy(), var_grad_llr=llr_v.grad.numpy(),
        var_grad_msgs=m_v.grad.numpy(),
        res_w_ch=res.w_ch.detach().numpy(), res_w_res=res.w_res.detach().numpy(),
        res_prev=np.stack([p.detach().numpy() for p in prevs]), res_cm=cm.detach().numpy(),
        res_out=r_out.detach().numpy(), res_grad_out=g_r.numpy(), res_grad_w_ch=res.w_ch.grad.numpy(),
        res_grad_w_res=res.w_res.grad.numpy(), res_grad_cm=cm.grad.numpy(), res_grad_llr=llr_r.grad.numpy(),
        res_grad_prev=np.stack([p.grad.numpy() if p.grad is not None else np.zeros((B, E), np.float32)
                                for p in prevs]),
        out_final=fin.detach().numpy(), out_gt=gt.numpy(), out_soft=soft.detach().numpy(),
        out_max_loss=max_loss.detach().numpy(), out_grad_soft=g_soft.numpy(), out_grad_loss=g_loss.numpy(),
        out_grad_final=fin.grad.numpy(), out_soft_nogt=soft_nogt.numpy())
    print("wrote layers_z4.npz", E, chk.shape, var.shape)


if __name__ == "__main__":
    main()
