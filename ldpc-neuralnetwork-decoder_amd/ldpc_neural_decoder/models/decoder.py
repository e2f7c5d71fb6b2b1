"""Neural min-sum decoder assembled from the index-gather layers (models/layers.py).

The reference imports ``LDPCNeuralDecoder`` from ``ldpc_neural_decoder/models/decoder.py``
(main.py:6, constructed at main.py:66-71 as ``LDPCNeuralDecoder(num_nodes=E, num_iterations,
depth_L)``) and trains/evaluates it through the protocol of training/trainer.py:93,185,251:

    soft_bits, loss = decoder(llrs, check_index_tensor, var_index_tensor, transmitted_bits)
    hard_bits = decoder.decode(llrs, check_index_tensor, var_index_tensor)

with ``llrs`` (B, N) channel LLRs, the index tensors of create_LLR_mapping (utils/ldpc_utils.py:
62-95, var-major edge numbering) and ``loss`` a per-frame vector (the trainer takes ``.mean()``).
That file is not in the reference tree, so this module DEFINES the decoder on the reference's
layers -- parity at the decoder level is unpinned; every layer it is built from is pinned to the
reference by tests/golden/layers_z4.npz.  The structure follows the notebook prototype
LDPCDecoderResidual (EE4002R_2025.ipynb cell 11): check layer -> variable layer with channel and
residual weights -> output mapping.  Iteration l = 0..I-1 runs a check layer; every iteration
but the last is followed by a variable layer with its own ResidualLayer(E, depth_L) weights, and
the last check layer's messages feed the output mapping (as the prototype's forward does):

    x0[b, e]  = llrs[b, var(e)]                                  edge view of the channel LLRs
    c_l       = CheckLayer(v_{l-1}, check_index_tensor)          (v_{-1} = x0)
    v_l       = w_ch_l * x0 + sum_{e' in var(e), e' != e} c_l[e'] + sum_i w_res_l[i] v_{l-1-i}
    app[b, j] = sum_{e in var j} c_{I-1}[e]
    soft, max_loss = OutputLayer(-app, -llrs, ground_truth)      P(bit = 1) = sigmoid(-(llr + app))

The sign: the channel's LLR is log P(0)/P(1) (channel.py:127-148), so P(bit = 1) is
sigmoid(-LLR); the negation is explicit here rather than left to training (MessageGNN keeps the
reference's sigmoid(+LLR), message_gnn_decoder.py:307).  Every gather, min-sum, sum, residual
and output op runs in csrc/layers.hip; there is no CPU path.
"""
import torch
import torch.nn as nn

from ldpc_neural_decoder import _native as N
from ldpc_neural_decoder.models.layers import (
    OutputLayer, ResidualLayer, _check_index, check_minsum, gather_sum)

_STRUCT = {}


def edge_variables(var_index_tensor):
    """Variable of every var-major LLR index, from the "other edges of my variable" table: edge
    e starts a new variable unless e - 1 is one of its neighbours (utils/ldpc_utils.py:77
    numbers the edges variable by variable)."""
    v = torch.as_tensor(var_index_tensor).cpu().long()
    E = v.shape[0]
    if E == 0:
        return torch.zeros(0, dtype=torch.long)
    same = (v[1:] == torch.arange(E - 1).unsqueeze(1)).any(dim=1) if v.shape[1] else torch.zeros(E - 1, dtype=torch.bool)
    return torch.cat([torch.zeros(1, dtype=torch.long), torch.cumsum((~same).long(), 0)])


def _structure(var_index_tensor, n_vars, dev):
    """(x0 index (1, E), app index (dv_max, N)) in the kernels' prepared layout, cached per
    index tensor."""
    key = (id(var_index_tensor), var_index_tensor.data_ptr(), var_index_tensor._version, n_vars, str(dev))
    hit = _STRUCT.get(key)
    if hit is not None and hit[0] is var_index_tensor:
        return hit[1]
    var_of = edge_variables(var_index_tensor)
    E = var_of.numel()
    n_found = int(var_of[-1]) + 1 if E else 0
    if n_found != n_vars:
        raise RuntimeError(f"var_index_tensor describes {n_found} variables but llrs has {n_vars} columns")
    deg = torch.bincount(var_of, minlength=n_vars)
    start = torch.cumsum(deg, 0) - deg
    dmax = int(deg.max()) if E else 1
    slot = torch.arange(E) - start[var_of]
    app = torch.full((dmax, n_vars), -1, dtype=torch.int32)
    app[slot, var_of] = torch.arange(E, dtype=torch.int32)
    prepared = (var_of.to(torch.int32).unsqueeze(0).to(dev), app.to(dev))
    if len(_STRUCT) > 8:
        _STRUCT.clear()
    _STRUCT[key] = (var_index_tensor, prepared)
    return prepared


class LDPCNeuralDecoder(nn.Module):
    """Neural min-sum decoder with channel and residual weights (see module docstring)."""

    def __init__(self, num_nodes, num_iterations=5, depth_L=2):
        super().__init__()
        self.num_nodes = num_nodes
        self.num_iterations = num_iterations
        self.depth_L = depth_L
        if num_iterations < 1:
            raise ValueError("num_iterations must be >= 1")
        self.residual_layers = nn.ModuleList([ResidualLayer(num_nodes, depth_L)
                                              for _ in range(num_iterations - 1)])
        self.output_layer = OutputLayer()

    def forward(self, llrs, check_index_tensor, var_index_tensor, ground_truth=None):
        home = llrs.device
        dev = N.device_of(llrs)
        llr = llrs.to(dev, torch.float32).contiguous()
        B, n = llr.shape
        x0_idx, app_idx = _structure(torch.as_tensor(var_index_tensor), n, dev)
        E = x0_idx.shape[1]
        if E != self.num_nodes:
            raise RuntimeError(f"index tensors describe {E} LLR indices, decoder built for {self.num_nodes}")
        cidx = _check_index(check_index_tensor, E, dev)
        vidx = _check_index(var_index_tensor, E, dev, compact=True)
        x0 = gather_sum(llr, x0_idx)
        v, prevs = x0, []
        for res in self.residual_layers:
            c = check_minsum(v, cidx)
            v = res(x0, gather_sum(c, vidx), prevs)
            prevs = [v] + prevs[:max(self.depth_L - 1, 0)]
        app = gather_sum(check_minsum(v, cidx), app_idx)
        gt = None if ground_truth is None else ground_truth.to(dev, torch.float32)
        soft, loss = self.output_layer(-app, -llr, gt)
        if loss is None:
            return soft.to(home), None
        return soft.to(home), loss.to(home)

    @torch.no_grad()
    def decode(self, llrs, check_index_tensor, var_index_tensor):
        soft, _ = self.forward(llrs, check_index_tensor, var_index_tensor)
        return (soft > 0.5).float()

