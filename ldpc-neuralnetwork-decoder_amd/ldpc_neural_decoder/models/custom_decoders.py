"""Hybrid "Custom*" message decoders (drop-in for message_gnn_decoder.py:585-1291).

Two decoders: CustomMinSumMessageGNNDecoder (pure message passing, below) and
CustomVariableMessageGNNDecoder (the GNN's check side + a min-sum variable update, further down).

The reference's CustomMinSumMessageGNNDecoder (MGD:1137-1251) cannot run: its factory calls
TannerToMessageGraph() without H (MGD:1270), and its variable / check updates index per-node
tensors as if they were per-message (MGD:636-657, :999-1038).  This module
keeps its classes, constructors, parameters (state_dict keys) and forward signature, and defines
the decode by the updates those loops spell out -- per edge m = (check c, variable v), c2v = 0 at
the start (MGD:1193), for iteration = 0 .. num_iterations - 1:

  S_v   = sum of c2v over v's edges in ascending message order        (MGD:650, :1231)
  v2c_m = (llr_v + S_v) - c2v_m                 "total minus own"      (MGD:650-654)
  v2c_m = 0.5 v2c_m + 0.5 c2v_m     when iteration > 0 (damping)      (MGD:659-663)
  c2v_m = prod_{m' != m} sign(v2c_m') * min_{m' != m} |v2c_m'|        (MGD:1006-1038)
          unscaled: the learnable alpha of MGD:974 is never read by the update
  probs_v = sigmoid(llr_v + S_v)                                       (MGD:1214-1240)
  loss  = binary_cross_entropy(probs, ground_truth) (mean)             (MGD:1246-1249)

The whole decode runs in libldpc_amd (ldpc_custom_minsum_decode, csrc/flood.hip: streaming
kernels, any graph).  The check update is pinned to the reference's own check_layer_update
(tests/golden/make_custom_golden.py); the variable update and damping cannot execute in the
reference, so their restatement (oracle/ldpc_oracle.c) is the definition.
"""
import os
from collections import deque

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ldpc_neural_decoder import _native as N
from ldpc_neural_decoder.models.message_gnn_decoder import (
    MessageGNNDecoder, MessageGNNLayer, TannerToMessageGraph, _aggregation_specs, _io_mapping, _types_for)


class CustomVariableMessageGNNLayer(MessageGNNLayer):
    """MGD:585-755: a MessageGNNLayer plus the min-sum variable update's parameters (w_ch, w_res,
    unused by the update itself) and its residual storage."""

    def __init__(self, num_message_types=1, hidden_dim=64, depth_L=3):
        super().__init__(num_message_types, hidden_dim)
        self.depth_L = depth_L
        self.w_ch = nn.Parameter(torch.ones(1))
        self.w_res = nn.Parameter(torch.ones(depth_L))
        self.previous_VL_storage = deque(maxlen=depth_L + 1)

    def variable_layer_update(self, input_mapping_LLR, check_to_variable_messages, variable_index_tensor, iteration):
        """MGD:611-670 on its index rows: row m = [variable, incoming message ids..., -1].  Per frame
        b: v2c[b, m] = (llr[b, variable] + sum of the incoming c2v, ascending) - the row's last
        incoming c2v (the loop's last assignment); llr[b, variable] for a row without ids; from
        iteration 1 on, 0.5 v2c + 0.5 c2v[b, m] (MGD:659-663).  input_mapping_LLR (B, N) indexed by
        the row's variable; check_to_variable_messages (B, E).  HIP: ldpc_index_rows_varsum."""
        llr = torch.as_tensor(input_mapping_LLR)
        c2v = torch.as_tensor(check_to_variable_messages)
        home = llr.device
        dev = N.device_of(llr)
        rows = _index_rows(variable_index_tensor, llr.shape[1] if llr.dim() == 2 else 0,
                           c2v.shape[1] if c2v.dim() == 2 else 0, dev)
        if llr.dim() != 2 or c2v.dim() != 2 or llr.shape[0] != c2v.shape[0]:
            raise ValueError("input_mapping_LLR (B, N) and check_to_variable_messages (B, E) expected")
        B, R = llr.shape[0], rows.shape[0]
        damp = int(iteration) > 0
        if damp and R != c2v.shape[1]:
            raise RuntimeError(f"damping mixes {R} outputs with {c2v.shape[1]} input messages")
        x = llr.to(dev, torch.float32).contiguous()
        c = c2v.to(dev, torch.float32).contiguous()
        out = torch.empty((B, R), dtype=torch.float32, device=dev)
        N.check(N.lib().ldpc_index_rows_varsum(N.ptr(x), B, x.shape[1], N.ptr(c), c.shape[1], N.ptr(rows), R,
                                               rows.shape[1], int(damp), N.ptr(out), N.stream_ptr(dev)))
        return out.to(home) if home != dev else out


class CustomCheckMessageGNNLayer(MessageGNNLayer):
    """MGD:966-1082: a MessageGNNLayer plus the (unused) learnable min-sum scale alpha = 0.8."""

    def __init__(self, num_message_types, hidden_dim, depth=2, dropout=0.0):
        super().__init__(num_message_types, hidden_dim)
        self.alpha = nn.Parameter(torch.tensor(0.8))

    def check_layer_update(self, message_features, message_types, check_index_tensor):
        """MGD:976-1044 on its index rows: row m = [check, incoming message ids..., -1].  Per frame
        b: c2v[b, m] = prod sign(x) * min |x| over the row's valid ids except its last one (the
        loop's last assignment excludes it), torch.sign (sign(0) = sign(NaN) = 0) and torch.min (NaN
        wins) semantics, 0 with fewer than two valid ids.  message_features (B, E).  The learnable
        alpha is not used, as in the reference.  HIP: ldpc_index_rows_minsum."""
        x = torch.as_tensor(message_features)
        if x.dim() != 2:
            raise ValueError(f"message_features must be (batch, num_messages), got {tuple(x.shape)}")
        home = x.device
        dev = N.device_of(x)
        rows = _index_rows(check_index_tensor, None, x.shape[1], dev)
        xf = x.to(dev, torch.float32).contiguous()
        B, R = xf.shape[0], rows.shape[0]
        out = torch.empty((B, R), dtype=torch.float32, device=dev)
        N.check(N.lib().ldpc_index_rows_minsum(N.ptr(xf), B, xf.shape[1], N.ptr(rows), R, rows.shape[1], N.ptr(out),
                                               N.stream_ptr(dev)))
        return out.to(home) if home != dev else out


def _index_rows(index_tensor, n_nodes, n_msgs, device):
    """An index tensor (R, W) as int64 on `device`, validated as the reference's indexing would
    be: ids below n_msgs, every negative id is padding (the reference filters with ids >= 0,
    MGD:644, :1004), the node column in [0, n_nodes) when it is used."""
    t = torch.as_tensor(index_tensor)
    if t.dim() != 2 or t.shape[1] < 1:
        raise ValueError(f"index tensor must be (rows, 1 + max degree), got {tuple(t.shape)}")
    t = t.long()
    ids = t[:, 1:]
    if ids.numel() and int(ids.max()) >= n_msgs:
        raise IndexError(f"message id out of range for {n_msgs} messages")
    if n_nodes is not None and t.shape[0] and (int(t[:, 0].max()) >= n_nodes or int(t[:, 0].min()) < 0):
        raise IndexError(f"node index out of range for {n_nodes} nodes")
    return t.to(device).contiguous()


def _graph_from_index_tensors(check_index_tensor, variable_index_tensor, num_checks, num_variables):
    """Edges (check, variable) of the messages the two index tensors list (rows = nodes, entries =
    message ids, -1 padding), check-major with variables ascending."""
    ci = torch.as_tensor(check_index_tensor).cpu().numpy()
    vi = torch.as_tensor(variable_index_tensor).cpu().numpy()
    if ci.ndim != 2 or vi.ndim != 2 or ci.shape[0] != num_checks or vi.shape[0] != num_variables:
        raise ValueError("index tensors must be (num_checks, max_dc) and (num_variables, max_dv)")
    chk_of, var_of = {}, {}
    for c in range(ci.shape[0]):
        for m in ci[c][ci[c] >= 0]:
            chk_of[int(m)] = c
    for v in range(vi.shape[0]):
        for m in vi[v][vi[v] >= 0]:
            var_of[int(m)] = v
    if set(chk_of) != set(var_of):
        raise ValueError("the check and variable index tensors list different messages")
    pairs = sorted({(chk_of[m], var_of[m]) for m in chk_of})
    edge_chk = np.array([p[0] for p in pairs], dtype=np.int32)
    edge_var = np.array([p[1] for p in pairs], dtype=np.int32)
    return edge_chk, edge_var


class CustomMinSumMessageGNNDecoder(MessageGNNDecoder):
    """MGD:1137-1251.  forward(input_llrs, variable_adjacency, check_adjacency, message_types,
    variable_to_message_mapping, ground_truth=None) -> probs, or (probs, loss) with ground truth.
    The decode reads none of the module's parameters (the learnable alpha of MGD:974 included), so
    probs never require grad -- exactly the reference's autograd graph for these updates.
    The adjacency / type / mapping arguments are accepted for signature compatibility; the graph
    comes from the index tensors (set_variable_index_tensor / set_check_index_tensor), as in the
    reference's update loops."""

    def __init__(self, num_messages, num_iterations, hidden_dim, num_message_types=1, depth=2, dropout=0.0):
        super().__init__(num_messages, num_iterations, hidden_dim, num_message_types)
        self.variable_layer = CustomVariableMessageGNNLayer(num_message_types, hidden_dim, depth)
        self.check_layer = CustomCheckMessageGNNLayer(num_message_types, hidden_dim, depth, dropout)
        self.gnn_layers = nn.ModuleList([
            CustomCheckMessageGNNLayer(num_message_types, hidden_dim, depth, dropout)
            for _ in range(num_iterations)])
        self.variable_index_tensor = None
        self.check_index_tensor = None
        self._graphs = {}

    def set_variable_index_tensor(self, variable_index_tensor):
        self.variable_index_tensor = variable_index_tensor
        self._graphs = {}

    def set_check_index_tensor(self, check_index_tensor):
        self.check_index_tensor = check_index_tensor
        self._graphs = {}

    def _graph(self, num_variables, device):
        if self.variable_index_tensor is None or self.check_index_tensor is None:
            raise RuntimeError("set_variable_index_tensor / set_check_index_tensor first "
                               "(create_custom_minsum_message_gnn_decoder does)")
        key = str(device)
        if key not in self._graphs:
            M = torch.as_tensor(self.check_index_tensor).shape[0]
            ec, ev = _graph_from_index_tensors(self.check_index_tensor, self.variable_index_tensor, M, num_variables)
            self._graphs[key] = N.NativeGraph(ec, ev, M, num_variables, device)
        return self._graphs[key]

    def forward(self, input_llrs, variable_adjacency=None, check_adjacency=None, message_types=None,
                variable_to_message_mapping=None, ground_truth=None):
        home = input_llrs.device
        dev = N.device_of(input_llrs)
        x = input_llrs.to(dev, torch.float32).contiguous()
        if x.dim() != 2:
            raise ValueError(f"input_llrs must be (batch, num_variables), got {tuple(input_llrs.shape)}")
        B, n = x.shape
        g = self._graph(n, dev)
        if n != g.N:  # the graph's variable count comes from the index tensors (the reference indexes
            # past the LLR row and raises IndexError): the kernels take no N of their own
            raise ValueError(f"input_llrs has {n} variables, the index tensors describe {g.N}")
        probs = torch.empty((B, n), dtype=torch.float32, device=dev)
        if B:
            wsb = N.check(N.lib().ldpc_custom_minsum_workspace_size(g.handle, B))
            ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
            N.check(N.lib().ldpc_custom_minsum_decode(g.handle, N.ptr(x), B, int(self.num_iterations), N.ptr(probs),
                                                     N.ptr(ws), wsb, N.stream_ptr(dev)))
        if home != dev:
            probs = probs.to(home)
        if ground_truth is not None:
            return probs, F.binary_cross_entropy(probs, ground_truth.to(probs.device).float())
        return probs

    def decode(self, input_llrs, *args, **kwargs):
        """Hard decisions (probs > 0.5) -- the MessageGNNDecoder.decode convention (MGD:319-353)."""
        with torch.no_grad():
            probs = self.forward(input_llrs, *args, **kwargs)
        return (probs > 0.5).float()


def create_variable_index_tensor(H, converter):
    """MGD:938-964: (num_vars, max variable degree) message ids, -1 padding."""
    num_vars = H.shape[1]
    width = max(len(v) for v in converter.var_to_messages.values())
    out = -torch.ones((num_vars, width), dtype=torch.long)
    for v in range(num_vars):
        msgs = converter.var_to_messages[v]
        out[v, :len(msgs)] = torch.as_tensor(msgs, dtype=torch.long)
    return out


def create_check_index_tensor(H, message_type_map=None):
    """MGD:1085-1134: (num_checks, max check degree), -1 padding.  With message_type_map
    ({(check, variable): message id}) the entries are message ids; without it the reference's
    fallback id c * num_variables + v."""
    Hn = np.asarray(torch.as_tensor(H).cpu())
    M, Nv = Hn.shape
    width = int(Hn.sum(axis=1).max())
    out = torch.full((M, width), -1, dtype=torch.long)
    for c in range(M):
        k = 0
        for v in np.nonzero(Hn[c] > 0)[0]:
            if message_type_map is not None:
                m = message_type_map.get((c, int(v)))
                if m is None:
                    continue
            else:
                m = c * Nv + int(v)
            out[c, k] = m
            k += 1
    return out


def create_custom_minsum_message_gnn_decoder(H, num_iterations=5, hidden_dim=8, depth=2, dropout=0.0):
    """MGD:1254-1292 -> (decoder, converter), with the converter built from H (the reference's
    TannerToMessageGraph() call without H fails) and the index tensors in message ids."""
    converter = TannerToMessageGraph(H)
    num_messages = len(converter.messages)
    num_message_types = 1
    decoder = CustomMinSumMessageGNNDecoder(num_messages, num_iterations, hidden_dim, num_message_types, depth,
                                            dropout)
    decoder.set_variable_index_tensor(create_variable_index_tensor(H, converter))
    decoder.set_check_index_tensor(create_check_index_tensor(H, converter.message_type_map))
    return decoder, converter


def _one_hot_index(mapping, E, Nv, device):
    """The reference multiplies by message_to_var_mapping (MGD:829-830, :858-864): the (E, N) one-hot of
    TannerToMessageGraph.message_to_var_mapping.  Accepted as that matrix or as its 1-D index."""
    m = torch.as_tensor(mapping)
    if m.dim() == 2:
        if m.shape != (E, Nv):
            raise ValueError(f"message_to_var_mapping must be ({E}, {Nv}), got {tuple(m.shape)}")
        mf = m.float()
        if not bool(((mf == 0) | (mf == 1)).all()) or not bool((mf.sum(dim=1) == 1).all()):
            raise NotImplementedError("message_to_var_mapping must be one-hot per message")
        m = mf.argmax(dim=1)
    return _io_mapping(m.long(), E, Nv, device)


class CustomVariableMessageGNNDecoder(MessageGNNDecoder):
    """MGD:758-879.  The reference cannot run it (IndexError at MGD:829-834 /
    :637-654, and MGD:745 calls a Linear(1, H) the layer does not have).  This build defines each
    layer i by the steps MGD:672-755 spell out, per frame and message m (check c, variable v):

      c    = x + emb_i[type]                                                   (:704-709)
      b    = A_c c  (the check adjacency; the identity when none is given, :825-826)
      F    = check_to_var_update_i([c; b])                                     (:724-726)
      l_m  = output_projection_i(F_m)                                          (:729)
      v2c_m = (llr_v + sum_{m' -> v} l_m') - l_m, then 0.5 v2c_m + 0.5 l_m     (:650-663; the
             decoder passes iteration i + 1 >= 1, :851, so the damping applies at every layer)
      x    = input_embedding(v2c_m) + F_m    (the decoder's Linear(1, H))      (:745-753)

    and the output (:855-877): out_m = output_projection_L(x_m), probs_v = sigmoid(mean over v's
    messages of out_m + llr_v).  forward(...) returns (probs, None), or (probs, max over bits of
    the per-bit BCE) with ground truth, as the reference does.  Any hidden_dim up to 1024 (the
    reference's constructor takes any, MGD:765: 64 runs the split-MFMA kernels, other widths the tiled
    fp32 kernels); clique / identity check adjacencies.  Kernels: ldpc_gnn_custom_var_forward
    (csrc/gnn.hip).  Oracle: oracle/oracle.py custom_variable_forward.

    Training: this build has no backward for the hybrid GNN.  With grad enabled and trainable
    parameters the probs carry a grad_fn whose backward raises NotImplementedError (naming this
    decoder), instead of torch's generic "does not require grad".  The layers' w_ch / w_res
    (MGD:605-606) are never read by any forward in the reference (nor here): their gradient is None
    by construction, whatever the backward."""

    def __init__(self, num_messages, num_iterations=5, hidden_dim=64, num_message_types=1, depth_L=3):
        if not 0 < hidden_dim <= 1024:  # refused up front rather than at the first forward
            raise ValueError(f"CustomVariableMessageGNNDecoder: this build's kernels run the hybrid GNN at "
                             f"hidden_dim 1 .. 1024 (got hidden_dim={hidden_dim})")
        super().__init__(num_messages, num_iterations, hidden_dim, num_message_types)
        self.gnn_layers = nn.ModuleList([
            CustomVariableMessageGNNLayer(num_message_types, hidden_dim, depth_L) for _ in range(num_iterations)])
        self.variable_index_tensor = None

    def set_variable_index_tensor(self, variable_index_tensor):
        self.variable_index_tensor = variable_index_tensor

    def forward(self, input_llr, message_to_var_mapping, message_types=None, var_to_check_adjacency=None,
                check_to_var_adjacency=None, ground_truth=None):
        home = input_llr.device
        dev = N.device_of(input_llr)
        E = self.num_messages
        llr = input_llr.to(dev, torch.float32).contiguous()
        B, Nv = llr.shape
        io_map = _one_hot_index(message_to_var_mapping, E, Nv, dev)
        T = self.gnn_layers[0].message_type_embeddings.shape[0]
        types = _types_for(message_types, E, T, dev)
        vspec = (io_map.cpu().numpy().astype(np.int64), Nv)  # the plan's var side (unused by the kernels)
        if check_to_var_adjacency is None:
            cspec = (np.arange(E, dtype=np.int64), E)          # torch.eye (:825-826): every message alone
        else:
            if var_to_check_adjacency is None:
                # the reference takes eye(E) for A_v (MGD:822-823) and resizes nothing: a mis-sized
                # A_c then fails in its bmm
                if tuple(check_to_var_adjacency.shape) != (E, E):
                    raise RuntimeError(f"check_to_var_adjacency must be ({E}, {E}) when var_to_check_adjacency "
                                       f"is None, got {tuple(check_to_var_adjacency.shape)}")
                _, cspec = _aggregation_specs(check_to_var_adjacency, check_to_var_adjacency, E)
            else:
                _, cspec = _aggregation_specs(var_to_check_adjacency, check_to_var_adjacency, E)
            if isinstance(cspec[0], str) and cspec[0] == "csr":
                raise NotImplementedError("the hybrid GNN runs with clique (TannerToMessageGraph) or identity "
                                          "check adjacencies")
        plan = self._plan(vspec, cspec, dev)
        blob = self._weights_blob(dev)
        L = len(self.gnn_layers)
        probs = torch.empty((B, Nv), dtype=torch.float32, device=dev)
        if B:
            lib = N.lib()
            Hd = self.hidden_dim
            ws1 = N.check(lib.ldpc_gnn_custom_var_workspace_size(plan.handle, Hd, Nv, 1, L))
            per = N.check(lib.ldpc_gnn_custom_var_workspace_size(plan.handle, Hd, Nv, 2, L)) - ws1
            budget = int(os.environ.get("LDPC_GNN_WORKSPACE_BYTES", 48 << 30))
            limit = max(1, ((1 << 31) // 16 - 1) // E)  # the kernels' per-launch message bound
            chunk = max(1, min(B, limit, max(1, (budget - ws1) // max(per, 1))))
            wsb = N.check(lib.ldpc_gnn_custom_var_workspace_size(plan.handle, Hd, Nv, chunk, L))
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            with torch.no_grad():
                for s in range(0, B, chunk):
                    n = min(chunk, B - s)
                    N.check(lib.ldpc_gnn_custom_var_forward(
                        plan.handle, Hd, T, L, N.ptr(blob), N.ptr(types), N.ptr(io_map), N.ptr(llr[s:s + n]), Nv, n,
                        N.ptr(probs[s:s + n]), N.ptr(ws), wsb, N.stream_ptr(dev)))
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            probs = _NoHybridBackward.apply(probs, *[p for p in self.parameters() if p.requires_grad])
        if home != dev:
            probs = probs.to(home)
        if ground_truth is not None:
            loss = F.binary_cross_entropy(probs, ground_truth.to(probs.device).float(), reduction="none")
            return probs, torch.max(loss, dim=1).values
        return probs, None

    def decode(self, input_llr, message_to_var_mapping, message_types=None, var_to_check_adjacency=None,
               check_to_var_adjacency=None):
        with torch.no_grad():
            probs, _ = self.forward(input_llr, message_to_var_mapping, message_types, var_to_check_adjacency,
                                    check_to_var_adjacency)
        return (probs > 0.5).float()


class _NoHybridBackward(torch.autograd.Function):
    """Identity on probs that refuses the backward with a clear error (see the decoder's docstring)."""

    @staticmethod
    def forward(ctx, probs, *params):
        return probs.view_as(probs)

    @staticmethod
    def backward(ctx, grad):
        raise NotImplementedError(
            "CustomVariableMessageGNNDecoder is inference-only in this build: there is no HIP backward for "
            "the hybrid GNN (its w_ch / w_res are never read by the forward, MGD:605-606, so they would get "
            "no gradient in any case); decode() / torch.no_grad() for inference")


def create_custom_variable_message_gnn_decoder(H, num_iterations=5, hidden_dim=64, depth_L=3, base_graph=None, Z=None):
    """MGD:882-936 -> (decoder, converter)."""
    converter = TannerToMessageGraph(H)
    num_messages = len(converter.messages)
    if base_graph is not None and Z is not None:
        base = np.asarray(torch.as_tensor(base_graph).cpu())
        shifts = {int(v) for v in base.ravel() if v >= 0}
        num_message_types = len(shifts) if shifts else 1
    else:
        num_message_types = 1
    decoder = CustomVariableMessageGNNDecoder(num_messages=num_messages, num_iterations=num_iterations,
                                              hidden_dim=hidden_dim, num_message_types=num_message_types,
                                              depth_L=depth_L)
    decoder.set_variable_index_tensor(create_variable_index_tensor(H, converter))
    return decoder, converter
