"""Index-gather neural-BP layers (drop-in for models/layers.py of the reference, :5-208).

Same modules, signatures and parameters; the gathers and reductions run in csrc/layers.hip
through the C ABI, with HIP backward kernels behind torch autograd Functions (the reference
trains through these layers with autograd).  CPU inputs are moved to the HIP device and the
outputs moved back; there is no CPU fallback.
"""
import ctypes

import torch
import torch.nn as nn

from ldpc_neural_decoder import _native as N


def _dev_f32(t, dev):
    return t.to(dev, torch.float32).contiguous()


_PREPARED = {}  # (tensor identity, version, n_in, device) -> (K, n_out) int32 device index


def _check_index(idx, n_in, dev, compact=False):
    """The reference gathers from (B, n_in + 1) after mapping -1 to the zero column n_in: any
    other index outside [0, n_in] is torch.gather's out-of-bounds RuntimeError.  Returns the
    kernels' layout -- transposed (K, n_out) int32, -1 for padding -- built and validated once
    per index tensor (the decoders call every layer with the same index tensors).  compact (for
    the sums): each row's padding moved to its end, order of the real entries kept, K cut to the
    longest row -- padding adds an exact +0.0, and the sum kernels stop at the first -1."""
    idx = torch.as_tensor(idx)
    key = (id(idx), idx.data_ptr(), idx._version, tuple(idx.shape), n_in, str(dev), compact)
    hit = _PREPARED.get(key)
    if hit is not None and hit[0] is idx:
        return hit[1]
    if idx.dim() != 2:
        raise RuntimeError("index tensor must be 2-D (num_nodes, max_neighbors)")
    if idx.dtype.is_floating_point:
        raise RuntimeError("gather(): Expected dtype int64 for index")
    if idx.numel() and (int(idx.max()) > n_in or int(idx.min()) < -1):
        raise RuntimeError(f"index out of bounds for a dimension of size {n_in + 1}")
    prepared = torch.where(idx == n_in, torch.full_like(idx, -1), idx)
    if compact and prepared.numel():
        order = torch.argsort((prepared < 0).to(torch.int8), dim=1, stable=True)
        prepared = torch.gather(prepared, 1, order)
        keep = max(int((prepared >= 0).sum(dim=1).max()), 1)
        prepared = prepared[:, :keep]
    prepared = prepared.to(torch.int32).t().contiguous().to(dev)
    if len(_PREPARED) > 16:
        _PREPARED.clear()
    _PREPARED[key] = (idx, prepared)
    return prepared


_GROUPS = {}  # (prepared index identity, n_in) -> (gptr, gmem) device int32, or None


def _check_groups(idx, n_in):
    """Checks of a prepared CheckLayer index, or None: usable when every row i holds exactly the
    other members of one set S (i in S, no duplicates), and every member of S has that row --
    the structure create_LLR_mapping gives (each edge's row = the other edges of its check).
    Returns (gptr (G + 1), gmem (n)) int32 on the index's device, members ascending."""
    key = (id(idx), idx.data_ptr(), n_in)
    hit = _GROUPS.get(key)
    if hit is not None and hit[0] is idx:
        return hit[1]
    res = None
    K, n_out = idx.shape
    if n_out == n_in:
        rows = idx.t().cpu().tolist()
        sets, ok = {}, True
        for i, r in enumerate(rows):
            real = [j for j in r if j >= 0]
            s = frozenset(real)
            if len(s) != len(real) or i in s:
                ok = False
                break
            sets.setdefault(s | {i}, []).append(i)
        if ok and all(sorted(m) == sorted(k) for k, m in sets.items()):
            groups = sorted(sorted(m) for m in sets.values())
            ptr = [0]
            for m in groups:
                ptr.append(ptr[-1] + len(m))
            res = (torch.tensor(ptr, dtype=torch.int32, device=idx.device),
                   torch.tensor([j for m in groups for j in m], dtype=torch.int32, device=idx.device))
    if len(_GROUPS) > 16:
        _GROUPS.clear()
    _GROUPS[key] = (idx, res)
    return res


_VGROUPS = {}  # (prepared index identity, n_in) -> gptr device int32, or None


def _var_groups(idx, n_in):
    """Variable groups of a prepared (compacted) VariableLayer index, or None: usable when every
    row i holds exactly the other members of a run [s, s + d) containing i, in ascending order, and
    the runs tile [0, n) -- the structure create_LLR_mapping gives (each edge's row = the other
    edges of its variable, variable-major edge numbering).  Then summing a row in order equals
    ldpc_var_groups_sum's prefix-and-tail walk bit for bit.  Returns gptr (G + 1) int32."""
    key = (id(idx), idx.data_ptr(), n_in)
    hit = _VGROUPS.get(key)
    if hit is not None and hit[0] is idx:
        return hit[1]
    res = None
    K, n_out = idx.shape
    if n_out == n_in:
        rows = idx.t().cpu().tolist()
        ptr, i, ok = [0], 0, True
        while ok and i < n_in:
            d = len([j for j in rows[i] if j >= 0]) + 1
            run = list(range(i, i + d))  # i is the first member of its run
            if i + d > n_in:
                ok = False
                break
            for q in run:
                if [j for j in rows[q] if j >= 0] != [j for j in run if j != q]:
                    ok = False
                    break
            i += d
            ptr.append(i)
        if ok:
            res = torch.tensor(ptr, dtype=torch.int32, device=idx.device)
    if len(_VGROUPS) > 16:
        _VGROUPS.clear()
    _VGROUPS[key] = (idx, res)
    return res


def _var_sum(llr, msgs, idx):
    """out = llr + the gathered sums (llr None: the sums alone), through the variable-group kernel
    when the index has that structure, else the per-edge gather."""
    B, n_in = msgs.shape
    K, n_out = idx.shape
    out = torch.empty((B, n_out), dtype=torch.float32, device=msgs.device)
    grp = _var_groups(idx, n_in) if B else None
    if grp is not None:
        rc = N.lib().ldpc_var_groups_sum(N.ptr(llr) if llr is not None else None, N.ptr(msgs), B, n_in, N.ptr(grp),
                                         grp.numel() - 1, N.ptr(out), N.stream_ptr(msgs.device))
        if rc != N.LDPC_EUNSUPPORTED:  # rows too long for LDS: the per-edge gather below
            N.check(rc)
            return out
    N.check(N.lib().ldpc_gather_sum(N.ptr(llr) if llr is not None else None, N.ptr(msgs), B, n_in, N.ptr(idx),
                                    n_out, K, N.ptr(out), N.stream_ptr(msgs.device)))
    return out


class _CheckFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, idx):
        B, n_in = x.shape
        K, n_out = idx.shape
        out = torch.empty((B, n_out), dtype=torch.float32, device=x.device)
        am = torch.empty((B, n_out), dtype=torch.int32, device=x.device)
        N.check(N.lib().ldpc_gather_minsum(N.ptr(x), B, n_in, N.ptr(idx), n_out, K, N.ptr(out), N.ptr(am),
                                           N.stream_ptr(x.device)))
        ctx.save_for_backward(x, idx, am)
        return out

    @staticmethod
    def backward(ctx, g):
        x, idx, am = ctx.saved_tensors
        B, n_in = x.shape
        K, n_out = idx.shape
        gin = torch.empty_like(x)
        N.check(N.lib().ldpc_gather_minsum_backward(N.ptr(g.contiguous()), N.ptr(x), B, n_in, N.ptr(idx), n_out, K,
                                                    N.ptr(am), N.ptr(gin), N.stream_ptr(x.device)))
        return gin, None


def check_minsum(x, idx):
    """CheckLayer's min-sum on a prepared index.  Without autograd (inference, or an input that
    needs no gradient) the argmin the backward would need is not written."""
    if torch.is_grad_enabled() and x.requires_grad:
        return _CheckFn.apply(x, idx)
    B, n_in = x.shape
    K, n_out = idx.shape
    out = torch.empty((B, n_out), dtype=torch.float32, device=x.device)
    grp = _check_groups(idx, n_in)
    if grp is not None and B:
        gptr, gmem = grp
        rc = N.lib().ldpc_check_groups_minsum(N.ptr(x), B, n_in, N.ptr(gptr), N.ptr(gmem), gptr.numel() - 1, K,
                                              N.ptr(out), N.stream_ptr(x.device))
        if rc != N.LDPC_EUNSUPPORTED:  # rows too long for LDS: the per-edge gather below
            N.check(rc)
            return out
    N.check(N.lib().ldpc_gather_minsum(N.ptr(x), B, n_in, N.ptr(idx), n_out, K, N.ptr(out), None,
                                       N.stream_ptr(x.device)))
    return out


class _VarFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, llr, msgs, idx):
        B, n_in = msgs.shape
        out = _var_sum(llr, msgs, idx)
        ctx.save_for_backward(idx)
        ctx.shape = (B, n_in)
        return out

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        B, n_in = ctx.shape
        K, n_out = idx.shape
        g = g.contiguous()
        gm = torch.empty((B, n_in), dtype=torch.float32, device=g.device)
        N.check(N.lib().ldpc_gather_sum_backward(N.ptr(g), B, n_in, N.ptr(idx), n_out, K, N.ptr(gm),
                                                 N.stream_ptr(g.device)))
        return g, gm, None


class _SumFn(torch.autograd.Function):
    """out[:, i] = sum_k msgs[:, idx[k, i]] (ldpc_gather_sum with no LLR term)."""

    @staticmethod
    def forward(ctx, msgs, idx):
        B, n_in = msgs.shape
        out = _var_sum(None, msgs, idx)
        ctx.save_for_backward(idx)
        ctx.shape = (B, n_in)
        return out

    @staticmethod
    def backward(ctx, g):
        (idx,) = ctx.saved_tensors
        B, n_in = ctx.shape
        K, n_out = idx.shape
        gm = torch.empty((B, n_in), dtype=torch.float32, device=g.device)
        N.check(N.lib().ldpc_gather_sum_backward(N.ptr(g.contiguous()), B, n_in, N.ptr(idx), n_out, K, N.ptr(gm),
                                                 N.stream_ptr(g.device)))
        return gm, None


def gather_sum(msgs, prepared_idx):
    """Device-side segment sum over a prepared (K, n_out) int32 index (see _check_index)."""
    return _SumFn.apply(msgs, prepared_idx)


class _ResFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, llr, cm, w_ch, w_res, *prevs):
        B, n = llr.shape
        out = torch.empty_like(llr)
        arr = (ctypes.c_void_p * max(1, len(prevs)))(*[p.data_ptr() for p in prevs])
        N.check(N.lib().ldpc_residual(N.ptr(llr), N.ptr(w_ch), N.ptr(cm), N.ptr(w_res), arr, len(prevs), B, n,
                                      N.ptr(out), N.stream_ptr(llr.device)))
        ctx.save_for_backward(llr, w_ch, w_res, *prevs)
        return out

    @staticmethod
    def backward(ctx, g):
        llr, w_ch, w_res, *prevs = ctx.saved_tensors
        B, n = llr.shape
        g = g.contiguous()
        g_llr = torch.empty_like(llr) if ctx.needs_input_grad[0] else None
        g_wch = torch.empty_like(w_ch)
        g_wres = torch.zeros_like(w_res)  # entries past len(prevs) get no gradient
        g_prev = [torch.empty_like(p) for p in prevs]
        arr = (ctypes.c_void_p * max(1, len(prevs)))(*[p.data_ptr() for p in prevs])
        garr = (ctypes.c_void_p * max(1, len(prevs)))(*[p.data_ptr() for p in g_prev])
        N.check(N.lib().ldpc_residual_backward(N.ptr(g), N.ptr(llr), N.ptr(w_ch), N.ptr(w_res), arr, len(prevs), B,
                                               n, N.ptr(g_llr), N.ptr(g_wch), N.ptr(g_wres), garr,
                                               N.stream_ptr(g.device)))
        return (g_llr, g, g_wch, g_wres, *g_prev)


class _OutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, final, llr, gt):
        B, n = final.shape
        soft = torch.empty_like(final)
        loss = torch.empty(B, dtype=torch.float32, device=final.device) if gt is not None else None
        am = torch.empty(B, dtype=torch.int32, device=final.device) if gt is not None else None
        N.check(N.lib().ldpc_output_layer(N.ptr(final), N.ptr(llr), N.ptr(gt), B, n, N.ptr(soft), N.ptr(loss),
                                          N.ptr(am), N.stream_ptr(final.device)))
        ctx.save_for_backward(soft, gt, am)
        ctx.has_gt = gt is not None
        if gt is None:
            return soft
        return soft, loss

    @staticmethod
    def backward(ctx, g_soft, g_loss=None):
        soft, gt, am = ctx.saved_tensors
        B, n = soft.shape
        gz = torch.empty_like(soft)
        gs = g_soft.contiguous() if g_soft is not None else None
        gl = g_loss.contiguous() if g_loss is not None else None
        N.check(N.lib().ldpc_output_layer_backward(N.ptr(soft), N.ptr(gt), N.ptr(gs), N.ptr(gl), N.ptr(am), B, n,
                                                   N.ptr(gz), N.stream_ptr(soft.device)))
        return gz, gz, None


def _home_and_dev(t):
    return t.device, N.device_of(t)


class CheckLayer(nn.Module):
    """layers.py:5-66: min-sum check update over an (num_nodes, max_neighbors) index tensor."""

    def forward(self, input_tensor, check_index_tensor):
        home, dev = _home_and_dev(input_tensor)
        x = _dev_f32(input_tensor, dev)
        idx = _check_index(check_index_tensor, x.shape[1], dev)
        return check_minsum(x, idx).to(home)


class VariableLayer(nn.Module):
    """layers.py:69-125: input_llr + the sum of the gathered check messages."""

    def forward(self, input_llr, check_messages, var_index_tensor):
        home, dev = _home_and_dev(check_messages)
        msgs = _dev_f32(check_messages, dev)
        idx = _check_index(var_index_tensor, msgs.shape[1], dev, compact=True)
        llr = _dev_f32(input_llr, dev)
        if llr.shape != (msgs.shape[0], idx.shape[1]):
            raise RuntimeError(f"input_llr of shape {tuple(llr.shape)} does not match the summed messages "
                               f"{(msgs.shape[0], idx.shape[1])}")
        return _VarFn.apply(llr, msgs, idx).to(home)


class ResidualLayer(nn.Module):
    """layers.py:128-168: llr * w_ch + check messages + sum_i w_res[i] * prev_i (i < depth_L)."""

    def __init__(self, num_nodes, depth_L=2):
        super().__init__()
        self.num_nodes = num_nodes
        self.depth_L = depth_L
        self.w_ch = nn.Parameter(torch.ones(num_nodes))
        self.w_res = nn.Parameter(torch.ones(depth_L))

    def forward(self, input_llr, check_messages, prev_var_messages):
        home, dev = _home_and_dev(input_llr)
        prevs = [_dev_f32(p, dev) for p in list(prev_var_messages)[:self.depth_L]]
        if len(prevs) > 8:
            raise NotImplementedError("depth_L > 8")
        llr, cm = _dev_f32(input_llr, dev), _dev_f32(check_messages, dev)
        # the reference raises a broadcast error on these (layers.py:160-166); the kernel would
        # read w_ch / prev out of bounds
        if llr.dim() != 2 or self.w_ch.numel() != llr.shape[1]:
            raise RuntimeError(f"w_ch has {self.w_ch.numel()} entries for LLRs of shape {tuple(llr.shape)}")
        for i, t in enumerate([cm] + prevs):
            if t.shape != llr.shape:
                raise RuntimeError(f"{'check_messages' if i == 0 else f'prev_var_messages[{i - 1}]'} has shape "
                                   f"{tuple(t.shape)}, expected {tuple(llr.shape)}")
        out = _ResFn.apply(llr, cm, self.w_ch.to(dev),
                           self.w_res.to(dev), *prevs)
        return out.to(home)


class OutputLayer(nn.Module):
    """layers.py:171-208: (sigmoid(final + input), per-frame max of the BCE or None)."""

    def forward(self, final_llr, input_llr, ground_truth=None):
        home, dev = _home_and_dev(final_llr)
        fin, llr = _dev_f32(final_llr, dev), _dev_f32(input_llr, dev)
        if ground_truth is None:
            return _OutFn.apply(fin, llr, None).to(home), None
        soft, loss = _OutFn.apply(fin, llr, _dev_f32(ground_truth, dev))
        return soft.to(home), loss.to(home)
