"""Message-centred GNN decoder (drop-in for models/message_gnn_decoder.py:15-582 of the reference).

Same classes, constructor arguments, parameter names (so the same state_dict keys and
saved_models checkpoints) and forward/decode signatures as the reference; the forward pass
runs in libldpc_amd (csrc/gnn.hip): segment-mean aggregation instead of the dense E x E
normalized-adjacency bmm, the four message MLPs on the matrix cores, and the input embedding,
residuals, output projection, per-variable sum and sigmoid fused around them.  fp32 contract:
H = 64 runs each fp32 product as a scaled two-term f16 split (three v_mfma_f32_32x32x16_f16
products, fp32 accumulate; <= 2x an fp32 GEMM's error against float64), other widths as bf16x6
splits (H = 96..256) or fp32 fma chains; precision="bf16" is bf16 features and bf16 MFMA.

Compatibility notes (each mirrors the reference line cited):
  * a 2-D ``message_to_var_mapping`` uses its column 0 as the variable index (:220-226, :287-292),
    so the one-hot ``.long()`` mapping of the examples reproduces the reference's output exactly
    as the reference computes it; a float mapping raises IndexError as torch indexing does.
  * ``message_types`` None -> all zeros (:240-241); shorter/longer -> zero-pad/truncate (:68-78);
    values clamped to [0, T-1] (:81).
  * ``var_to_check_adjacency`` / ``check_to_var_adjacency`` are required (None fails like the
    reference, :93).  A mis-sized pair is zero-padded / cropped as :92-104 does.  The
    normalized cliques TannerToMessageGraph builds (:410-469) are recognised (groups read off the
    matrix once, verified by probing A @ r == group-mean(r)) and aggregated as group means; any
    other matrix runs as a general sparse bmm(A, c) over its nonzeros (fp32 only; trainable: the
    backward applies A^T over the plan's transposed CSR).
  * the unused ``output_layer`` (:188) is kept so state_dicts round-trip.
  * with grad enabled and trainable parameters, forward() runs the fp32 training path (every
    layer's features saved for the HIP backward, csrc/gnn_train.hip); otherwise the inference
    path (fp32 or bf16, chunked to LDPC_GNN_WORKSPACE_BYTES).  ``decode()`` is always inference.
    ``ground_truth`` returns (probs, BCE loss) as in :313-315.
"""
import os

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ldpc_neural_decoder import _native as N
from ldpc_neural_decoder.utils.ldpc_utils import edge_list


class MessageGNNLayer(nn.Module):
    """message_gnn_decoder.py:15-152 (parameters only; the math runs in the HIP kernels)."""

    def __init__(self, num_message_types=1, hidden_dim=64):
        super().__init__()
        self.message_type_embeddings = nn.Parameter(torch.randn(num_message_types, hidden_dim))
        self.var_to_check_update = nn.Sequential(
            nn.Linear(hidden_dim * 2, hidden_dim), nn.ReLU(), nn.Linear(hidden_dim, hidden_dim))
        self.check_to_var_update = nn.Sequential(
            nn.Linear(hidden_dim * 2, hidden_dim), nn.ReLU(), nn.Linear(hidden_dim, hidden_dim))
        self.output_projection = nn.Linear(hidden_dim, 1)

    def decode_messages(self, message_features):
        """message_gnn_decoder.py:131-152: project features to one LLR per message."""
        llr_values = self.output_projection(message_features).squeeze(-1)
        if llr_values.dim() == 1:
            llr_values = llr_values.unsqueeze(0)
        elif llr_values.shape[0] != message_features.shape[0]:
            llr_values = llr_values.transpose(0, 1)
        return llr_values

    def flat_weights(self):
        """This layer's section of the C-ABI weight blob (include/ldpc_amd.h)."""
        v, c = self.var_to_check_update, self.check_to_var_update
        parts = [self.message_type_embeddings, v[0].weight, v[0].bias, v[2].weight, v[2].bias,
                 c[0].weight, c[0].bias, c[2].weight, c[2].bias, self.output_projection.weight,
                 self.output_projection.bias]
        return [p.detach().reshape(-1) for p in parts]


def _types_for(message_types, E, T, device):
    """message_gnn_decoder.py:68-81 and :240-241."""
    if message_types is None:
        t = torch.zeros(E, dtype=torch.long, device=device)
    else:
        t = torch.as_tensor(message_types, device=device).long().reshape(-1)
        if t.numel() < E:
            t = torch.cat([t, torch.zeros(E - t.numel(), dtype=torch.long, device=device)])
        elif t.numel() > E:
            t = t[:E]
    return torch.clamp(t, 0, T - 1).to(torch.int32).contiguous()


def _io_mapping(mapping, E, N_vars, device):
    """message_gnn_decoder.py:218-229 / 285-295: the message -> variable index actually used."""
    m = torch.as_tensor(mapping)
    if m.dim() > 1:
        m = m[:, 0]  # the reference's column-0 rule
    if m.dtype.is_floating_point or m.dtype == torch.bool or m.dtype == torch.uint8:
        raise IndexError("tensors used as indices must be long, int, byte or bool tensors")
    m = m.to(device).long()
    if m.numel() != E:
        raise RuntimeError(f"message_to_var_mapping selects {m.numel()} values for {E} messages")
    if m.numel() and (int(m.max()) >= N_vars or int(m.min()) < -N_vars):
        raise IndexError(f"index out of range for {N_vars} variables")
    m = torch.where(m < 0, m + N_vars, m)
    return m.to(torch.int32).contiguous()


def _clique_groups(A, E):
    """Read the message groups off a normalized clique adjacency (message_gnn_decoder.py:410-469).

    Returns (labels (E,) int64 numpy, number of groups), or None when A is not such a matrix.  The
    labels are the first nonzero column of every row, renumbered densely; the matrix is then
    probed with random vectors to check that A @ r equals the group mean of r (the only property
    the group-mean kernels rely on)."""
    dev = A.device  # setup-time structure probe, on whichever device holds the matrix
    Ad = A.to(torch.float32)
    nz = Ad != 0
    if not bool(nz.any(dim=1).all()):
        return None  # an all-zero row (e.g. after the reference's zero-pad) is no clique
    first = torch.argmax(nz.to(torch.int8), dim=1)
    uniq, labels = torch.unique(first, return_inverse=True)
    n = int(uniq.numel())
    gen = torch.Generator(device="cpu").manual_seed(1234)
    for _ in range(2):
        r = torch.rand(E, generator=gen).to(dev)
        sums = torch.zeros(n, device=dev).index_add_(0, labels, r)
        cnt = torch.zeros(n, device=dev).index_add_(0, labels, torch.ones(E, device=dev))
        want = (sums / cnt)[labels]
        got = Ad @ r
        if not torch.allclose(got, want, rtol=1e-4, atol=1e-5):
            return None
    return labels.cpu().numpy().astype(np.int64), n


def _csr_of(A):
    """(ptr (E+1,), col, val) of a dense matrix: row m lists its nonzero columns ascending."""
    Ad = A.detach().to("cpu", torch.float32)
    rows, cols = torch.nonzero(Ad, as_tuple=True)  # row-major: rows ascending, cols ascending in a row
    ptr = torch.zeros(Ad.shape[0] + 1, dtype=torch.int64)
    ptr[1:] = torch.cumsum(torch.bincount(rows, minlength=Ad.shape[0]), 0)
    return ptr.numpy(), cols.numpy(), Ad[rows, cols].numpy()


def _resize_like_reference(Av, Ac, E):
    """message_gnn_decoder.py:92-104: when the var adjacency is not (E, E), both matrices are
    replaced by (E, E) zeros holding the top-left min(rows of A_v, E) block of each (the check
    matrix is resized by the var matrix's size, exactly as the reference does)."""
    if Av.size(0) == E and Av.size(1) == E:
        return Av, Ac
    new_v = torch.zeros((E, E), device=Av.device)
    new_c = torch.zeros((E, E), device=Av.device)
    k = min(Av.size(0), E)
    new_v[:k, :k] = Av[:k, :k]
    new_c[:k, :k] = Ac[:k, :k]
    return new_v, new_c


def _aggregation_specs(Av, Ac, E):
    """The two aggregation specs the native plan is built from, per side either
    ("groups", labels, n) -- a normalized clique adjacency, aggregated as group means -- or
    ("csr", ptr, col, val) -- any other matrix, aggregated as bmm(A, c) over its nonzeros.
    Cached on the caller's tensors (the reference rebuilds nothing per call either)."""
    if Av is None or Ac is None:
        raise AttributeError("'NoneType' object has no attribute 'size'")  # as MGD:93 fails
    cached = getattr(Av, "_ldpc_specs", None)
    if cached is not None and cached[0] == E and cached[1] is Ac:
        return cached[2]
    tagged = getattr(Av, "_ldpc_groups", None), getattr(Ac, "_ldpc_groups", None)
    if tagged[0] is not None and tagged[1] is not None and Av.shape == (E, E) and Ac.shape == (E, E):
        specs = (("groups",) + tuple(tagged[0]), ("groups",) + tuple(tagged[1]))
    else:
        v, c = _resize_like_reference(Av, Ac, E)
        if c.dim() != 2 or c.shape[0] != E or c.shape[1] != E:
            raise RuntimeError(f"check_to_var_adjacency of shape {tuple(c.shape)} cannot multiply {E} messages")
        out = []
        for A in (v, c):
            g = _clique_groups(A, E)
            out.append(("groups",) + g if g is not None else ("csr",) + _csr_of(A))
        specs = tuple(out)
        if specs[0][0] != specs[1][0]:  # a mixed pair runs as two CSR matrices
            specs = tuple(s_ if s_[0] == "csr" else ("csr",) + _csr_of(A) for s_, A in zip(specs, (v, c)))
    try:
        Av._ldpc_specs = (E, Ac, specs)
    except Exception:
        pass
    return specs


def _groups_from_adjacency(A, E):
    """The (labels, count) groups of a normalized clique adjacency of E messages (see
    _clique_groups); NotImplementedError for any other matrix."""
    tagged = getattr(A, "_ldpc_groups", None)
    if tagged is not None:
        return tagged
    if A is None:
        raise AttributeError("'NoneType' object has no attribute 'size'")
    g = _clique_groups(A, E) if A.dim() == 2 and A.shape == (E, E) else None
    if g is None:
        raise NotImplementedError("not a normalized clique adjacency of message groups")
    return g


class MessageGNNDecoder(nn.Module):
    """message_gnn_decoder.py:155-353."""

    def __init__(self, num_messages, num_iterations=5, hidden_dim=64, num_message_types=1):
        super().__init__()
        self.num_messages = num_messages
        self.num_iterations = num_iterations
        self.hidden_dim = hidden_dim
        self.input_embedding = nn.Linear(1, hidden_dim)
        self.gnn_layers = nn.ModuleList([MessageGNNLayer(num_message_types, hidden_dim)
                                         for _ in range(num_iterations)])
        self.output_layer = nn.Linear(hidden_dim, 1)  # unused by forward (:188), kept for state_dicts
        self.precision = "fp32"  # or "bf16": bf16 MLP operands, fp32 accumulate
        self.default_chunk = 0   # frames per native launch (0 = the whole batch, within budget)
        # cfg5 per-frame early termination (bf16 path; no reference counterpart): a frame stops
        # after the first layer whose hard decision (through the last layer's output projection)
        # satisfies every parity check.  last_iterations holds the layers each frame used.
        self.early_termination = False
        self.last_iterations = None
        self._plans = {}
        self._blob_key = None
        self._blob = None
        self._split_ok = True

    # -------------------------------------------------------------- native plumbing
    def _blob_params(self):
        """The parameters in weight-blob order (include/ldpc_amd.h); output_layer is unused."""
        ps = [self.input_embedding.weight, self.input_embedding.bias]
        for layer in self.gnn_layers:
            v, c = layer.var_to_check_update, layer.check_to_var_update
            ps += [layer.message_type_embeddings, v[0].weight, v[0].bias, v[2].weight, v[2].bias,
                   c[0].weight, c[0].bias, c[2].weight, c[2].bias, layer.output_projection.weight,
                   layer.output_projection.bias]
        return ps

    def _weights_blob(self, device):
        params = [self.input_embedding.weight, self.input_embedding.bias]
        params += [p for layer in self.gnn_layers for p in layer.parameters()]
        key = (str(device),) + tuple((p.data_ptr(), p._version) for p in params)
        if key != self._blob_key:
            parts = [self.input_embedding.weight.detach().reshape(-1),
                     self.input_embedding.bias.detach().reshape(-1)]
            for layer in self.gnn_layers:
                parts += layer.flat_weights()
            blob = torch.cat([p.to(device, torch.float32) for p in parts]).contiguous()
            T = self.gnn_layers[0].message_type_embeddings.shape[0]
            want = N.check(N.lib().ldpc_gnn_weights_size(self.hidden_dim, T, len(self.gnn_layers)))
            assert blob.numel() == want, (blob.numel(), want)
            self._blob, self._blob_key = blob, key
            self._split_ok = self._split_range_ok()
        return self._blob

    SPLIT_RANGE = 2.0 ** -17

    def _split_range_ok(self):
        """Whether the fp32 kernels' f16 splits hold every weight row to fp32 accuracy: each weight
        group shares one power-of-two scale, and a row keeps 22 bits while its largest |w| is >= 2^-17
        of its group's.  H = 64 (csrc/gnn.hip): the projection's W1v / W1c right halves; the MLP's
        left halves, W2v, W2c and W1v_left + W1v_right.  H = 96..256 (csrc/gnn_wide.hip): each side's
        W1 right half (the projections: one scale per workgroup slice; checked per whole matrix, which
        is stricter), both sides' W1 left halves together and W2v | W2c (the fused MLP's two scales).
        Checked once per weight version; otherwise the forward runs the products on the fp32 MFMA /
        as bf16x6 splits (LDPC_GNN_FP32_PRODUCTS)."""
        H = self.hidden_dim
        wide = H != 64 and H % 32 == 0 and 96 <= H <= 256
        if H != 64 and not wide:
            return True  # fp32 fma chains
        with torch.no_grad():
            for layer in self.gnn_layers:
                v, c = layer.var_to_check_update, layer.check_to_var_update
                w1v, w1c = v[0].weight.detach().float(), c[0].weight.detach().float()
                w2v, w2c = v[2].weight.detach().float(), c[2].weight.detach().float()
                if wide:
                    groups = ((w1v[:, H:],), (w1c[:, H:],), (w1v[:, :H], w1c[:, :H]),
                              (torch.cat([w2v, w2c], dim=1),))
                else:
                    groups = ((w1v[:, H:], w1c[:, H:]), (w1v[:, :H], w1c[:, :H], w2v, w2c, w1v[:, :H] + w1v[:, H:]))
                for g in groups:
                    rows = torch.cat([w.abs().amax(dim=1) for w in g])
                    live = rows[rows > 0]
                    if live.numel() and bool(live.min() < rows.max() * self.SPLIT_RANGE):
                        return False
        return True

    def _plan(self, vspec, cspec, device):
        """vspec / cspec: (labels, count) or ("groups", labels, count) or ("csr", ptr, col, val)."""
        norm = lambda sp: sp if isinstance(sp[0], str) else ("groups",) + tuple(sp)
        vspec, cspec = norm(vspec), norm(cspec)
        key = (str(device), vspec[0]) + tuple(np.asarray(a).tobytes() for a in vspec[1:] + cspec[1:])
        plan = self._plans.get(key)
        if plan is None:
            if vspec[0] == "groups" and cspec[0] == "groups":
                plan = N.NativeGnnPlan(vspec[1], vspec[2], cspec[1], cspec[2], device)
            else:
                plan = N.NativeGnnPlan.csr(self.num_messages, vspec[1:], cspec[1:], device)
            self._plans = {key: plan}  # keep one plan; graphs rarely change
        return plan

    def native_forward(self, llr, io_map, types, vgroups, cgroups, chunk=None):
        """llr (B, N) on a HIP device; io_map/types (E,) int32; vgroups / cgroups = (labels, count)
        group specs, or ("csr", ptr, col, val) general adjacencies (fp32 only)."""
        dev = llr.device
        B, Nv = llr.shape
        T = self.gnn_layers[0].message_type_embeddings.shape[0]
        L = len(self.gnn_layers)
        plan = self._plan(vgroups, cgroups, dev)
        if plan.weighted and self.precision != "fp32":
            raise NotImplementedError("a general (non-clique) adjacency runs on the fp32 path only")
        blob = self._weights_blob(dev)
        prec = 1 if self.precision == "bf16" else 0
        flags = N.LDPC_GNN_EARLY_STOP if self.early_termination else 0
        if flags and prec != 1:
            raise NotImplementedError("early termination is implemented on the bf16 path (precision='bf16')")
        if prec == 0 and not self._split_ok:
            flags |= N.LDPC_GNN_FP32_PRODUCTS  # weights beyond the f16 splits' range (_split_range_ok)
        probs = torch.empty((B, Nv), dtype=torch.float32, device=dev)
        iters = torch.empty(B, dtype=torch.int32, device=dev)
        self.last_iterations = iters
        if B == 0:
            return probs
        ws1 = N.check(N.lib().ldpc_gnn_workspace_size(plan.handle, self.hidden_dim, Nv, 1, L, prec))
        per_frame = N.check(N.lib().ldpc_gnn_workspace_size(plan.handle, self.hidden_dim, Nv, 2, L, prec)) - ws1
        budget = int(os.environ.get("LDPC_GNN_WORKSPACE_BYTES", 48 << 30))
        # frames per launch: bounded by the workspace budget and by LDPC_GNN_CHUNK (speed only)
        chunk = chunk or int(os.environ.get("LDPC_GNN_CHUNK", 0)) or self.default_chunk
        chunk = max(1, min(B, chunk or B, max(1, (budget - ws1) // max(per_frame, 1))))
        wsb = N.check(N.lib().ldpc_gnn_workspace_size(plan.handle, self.hidden_dim, Nv, chunk, L, prec))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        for s in range(0, B, chunk):
            n = min(chunk, B - s)
            N.check(N.lib().ldpc_gnn_forward_ex(
                plan.handle, self.hidden_dim, T, L, N.ptr(blob), N.ptr(types), N.ptr(io_map),
                N.ptr(llr[s:s + n]), Nv, n, prec, flags, N.ptr(probs[s:s + n]), N.ptr(iters[s:s + n]),
                N.ptr(ws), wsb, N.stream_ptr(dev)))
        return probs

    # -------------------------------------------------------------- reference API
    def forward(self, input_llr, message_to_var_mapping, message_types=None,
                var_to_check_adjacency=None, check_to_var_adjacency=None, ground_truth=None):
        """message_gnn_decoder.py:190-317 -> probs (B, N) [, BCE loss]."""
        home = input_llr.device
        dev = N.device_of(input_llr)
        E = self.num_messages
        vg, cg = _aggregation_specs(var_to_check_adjacency, check_to_var_adjacency, E)
        llr = input_llr.to(dev, torch.float32).contiguous()
        io_map = _io_mapping(message_to_var_mapping, E, llr.shape[1], dev)
        T = self.gnn_layers[0].message_type_embeddings.shape[0]
        types = _types_for(message_types, E, T, dev)
        params = self._blob_params()
        if self.precision == "fp32" and torch.is_grad_enabled() and any(p.requires_grad for p in params):
            # training: fp32 forward that saves every layer's features + the HIP backward
            # (precision="bf16" is an inference setting: it always takes the no-grad path)
            plan = self._plan(vg, cg, dev)
            probs, _ = _NativeGnnTrain.apply(self, llr, io_map, types, plan, False, *params)
        else:
            with torch.no_grad():
                probs = self.native_forward(llr, io_map, types, vg, cg)
        if home != dev:
            probs = probs.to(home)
        if ground_truth is not None:
            loss = F.binary_cross_entropy(probs, ground_truth.to(probs.device).float())
            return probs, loss
        return probs

    def forward_all_layers(self, input_llr, message_to_var_mapping, message_types=None,
                           var_to_check_adjacency=None, check_to_var_adjacency=None):
        """Training extension (no reference counterpart): the soft decisions after EVERY layer,
        (L, B, N), each layer's output features through the last layer's output_projection and the
        decoder's output stage; the last entry is forward()'s probs.  A loss on all of them (deep
        supervision) trains the intermediate layers to decode, which is what lets the bf16 path's
        per-frame early termination (cfg5) stop before the last layer -- its syndrome check reads
        exactly these decisions.  fp32, any adjacency, with autograd through the HIP backward
        (ldpc_gnn_backward_ds)."""
        dev = N.device_of(input_llr)
        E = self.num_messages
        vg, cg = _aggregation_specs(var_to_check_adjacency, check_to_var_adjacency, E)
        llr = input_llr.to(dev, torch.float32).contiguous()
        io_map = _io_mapping(message_to_var_mapping, E, llr.shape[1], dev)
        T = self.gnn_layers[0].message_type_embeddings.shape[0]
        types = _types_for(message_types, E, T, dev)
        plan = self._plan(vg, cg, dev)
        if self.precision != "fp32":
            raise NotImplementedError("forward_all_layers runs the fp32 training forward")
        probs, layer_probs = _NativeGnnTrain.apply(self, llr, io_map, types, plan, True, *self._blob_params())
        return torch.cat([layer_probs, probs.unsqueeze(0)], 0).to(input_llr.device)

    def decode(self, input_llr, message_to_var_mapping, message_types=None,
               var_to_check_adjacency=None, check_to_var_adjacency=None):
        """message_gnn_decoder.py:319-353: hard decision (probs > 0.5) as float32.  A hard
        decision has no gradient, so this always takes the inference path (chunked to the
        workspace budget), whatever the grad mode of the caller."""
        with torch.no_grad():
            soft_bits = self.forward(input_llr, message_to_var_mapping, message_types,
                                     var_to_check_adjacency, check_to_var_adjacency)
        return (soft_bits > 0.5).float()


def _saved_projections():
    """LDPC_GNN_SAVED_PROJ=0 makes the backward recompute the projections (A/B runs, tests)."""
    import os
    return os.environ.get("LDPC_GNN_SAVED_PROJ", "1") != "0"


class _NativeGnnTrain(torch.autograd.Function):
    """Autograd node of the native fp32 forward (message_gnn_decoder.py:190-307): forward saves
    each layer's features, backward is ldpc_gnn_backward (csrc/gnn_train.hip).  Replaces torch's
    autograd graph through the reference's forward for loss.backward() (trainer.py:93-99)."""

    @staticmethod
    def forward(ctx, dec, llr, io_map, types, plan, all_layers, *params):
        ctx.set_materialize_grads(False)
        dev = llr.device
        H, L = dec.hidden_dim, len(dec.gnn_layers)
        T = dec.gnn_layers[0].message_type_embeddings.shape[0]
        if H > 1024:
            raise NotImplementedError("the native backward supports hidden_dim <= 1024 (the widths of the tiled "
                                      "training forward, whose products it recomputes bit for bit)")
        B, Nv = llr.shape
        E = dec.num_messages
        blob = torch.cat([p.detach().reshape(-1).to(dev, torch.float32) for p in params]).contiguous()
        wsb = N.check(N.lib().ldpc_gnn_train_workspace_size(plan.handle, H, Nv, max(B, 1), L))
        # the forward's projected group rows and group means, kept for the backward (0 where the
        # path has none): no recompute there
        npj = N.check(N.lib().ldpc_gnn_train_proj_floats(plan.handle, H, B, L)) if _saved_projections() else 0
        need = L * B * E * H * 4 + npj * 4 + wsb
        free = torch.cuda.mem_get_info(dev)[0]
        free += torch.cuda.memory_reserved(dev) - torch.cuda.memory_allocated(dev)  # torch's cache
        if need > free:
            raise RuntimeError(
                f"training forward for {B} frames needs {need / 2**30:.1f} GiB of device memory "
                f"(every layer's (B, E, H) fp32 features are saved for the backward) but "
                f"{free / 2**30:.1f} GiB are free: use a smaller batch, or decode() / torch.no_grad() "
                f"for inference, which is chunked")
        probs = torch.empty((B, Nv), dtype=torch.float32, device=dev)
        saved = torch.empty((L, B, E, H), dtype=torch.float32, device=dev)
        proj = torch.empty(npj, dtype=torch.float32, device=dev)
        if B:
            ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
            N.check(N.lib().ldpc_gnn_forward_train_ex(
                plan.handle, H, T, L, N.ptr(blob), N.ptr(types), N.ptr(io_map), N.ptr(llr), Nv, B,
                N.ptr(probs), N.ptr(saved), N.ptr(proj) if npj else None, N.ptr(ws), wsb, N.stream_ptr(dev)))
        layer_probs = torch.empty((max(L - 1, 0) if all_layers else 0, B, Nv), dtype=torch.float32, device=dev)
        if all_layers and B and L > 1:
            N.check(N.lib().ldpc_gnn_layer_probs(
                plan.handle, H, T, L, N.ptr(blob), N.ptr(io_map), N.ptr(llr), Nv, B, N.ptr(saved),
                N.ptr(layer_probs), N.ptr(ws), wsb, N.stream_ptr(dev)))
        ctx.save_for_backward(llr, io_map, types, blob, probs, saved, layer_probs, proj)
        ctx.meta = (plan, H, T, L, [p.shape for p in params])
        return probs, layer_probs

    @staticmethod
    def backward(ctx, grad_probs, grad_layer_probs):
        llr, io_map, types, blob, probs, saved, layer_probs, proj = ctx.saved_tensors
        plan, H, T, L, shapes = ctx.meta
        dev = llr.device
        B, Nv = llr.shape
        grad = torch.empty_like(blob)
        wsb = N.check(N.lib().ldpc_gnn_train_workspace_size(plan.handle, H, Nv, B, L))
        ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
        g = (grad_probs.to(dev, torch.float32).contiguous() if grad_probs is not None
             else torch.zeros_like(probs))
        gl = None
        if grad_layer_probs is not None and layer_probs.numel():
            gl = grad_layer_probs.to(dev, torch.float32).contiguous()
        N.check(N.lib().ldpc_gnn_backward_ds_ex(
            plan.handle, H, T, L, N.ptr(blob), N.ptr(types), N.ptr(io_map), N.ptr(llr), Nv, B,
            N.ptr(probs), N.ptr(g), N.ptr(saved), N.ptr(proj) if proj.numel() else None,
            N.ptr(layer_probs) if gl is not None else None,
            N.ptr(gl) if gl is not None else None, N.ptr(grad), N.ptr(ws), wsb, N.stream_ptr(dev)))
        grads, off = [], 0
        for s in shapes:
            n = int(torch.Size(s).numel())
            grads.append(grad[off:off + n].view(s))
            off += n
        # only the last layer's output_projection takes part in the forward (:270): the others
        # get no gradient, exactly like the reference's autograd graph
        for layer in range(L - 1):
            grads[2 + layer * 11 + 9] = None
            grads[2 + layer * 11 + 10] = None
        return (None, None, None, None, None, None, *grads)


class TannerToMessageGraph:
    """message_gnn_decoder.py:356-536.  Same attributes; the two dense (E, E) adjacencies and the
    (E, N) one-hot mapping are built on first access (vectorised) and carry their message groups
    so the decoder never has to re-derive them."""

    def __init__(self, H):
        self.H = H
        self.num_checks, self.num_variables = H.shape
        self.edge_chk, self.edge_var = edge_list(H)  # check-major (:397-406)
        self.messages = list(zip(self.edge_var.tolist(), self.edge_chk.tolist()))
        self.var_to_messages = {i: [] for i in range(self.num_variables)}
        self.check_to_messages = {i: [] for i in range(self.num_checks)}
        for idx, (v, c) in enumerate(self.messages):
            self.var_to_messages[v].append(idx)
            self.check_to_messages[c].append(idx)
        self._adj = None
        self._map = None

    @property
    def var_groups(self):
        return self.edge_var.astype(np.int64), self.num_variables

    @property
    def check_groups(self):
        return self.edge_chk.astype(np.int64), self.num_checks

    def _build_adjacency(self):
        E = len(self.messages)
        dev = self.H.device if torch.is_tensor(self.H) else torch.device("cpu")
        out = []
        for lab, groups in ((self.edge_var, self.var_groups), (self.edge_chk, self.check_groups)):
            lab_t = torch.as_tensor(lab.astype(np.int64))
            deg = torch.bincount(lab_t).float()
            A = (lab_t.view(-1, 1) == lab_t.view(1, -1)).float()  # clique incl. self (:426-441 + eye)
            dis = deg[lab_t].pow(-0.5)
            A = (dis.view(-1, 1) * A) * dis.view(1, -1)            # D^-1/2 (A+I) D^-1/2 (:449-469)
            A = A.to(dev)
            A._ldpc_groups = groups
            out.append(A)
        self._adj = tuple(out)
        assert out[0].shape == (E, E)

    @property
    def var_to_check_adjacency(self):
        if self._adj is None:
            self._build_adjacency()
        return self._adj[0]

    @property
    def check_to_var_adjacency(self):
        if self._adj is None:
            self._build_adjacency()
        return self._adj[1]

    @property
    def message_to_var_mapping(self):
        """(E, N) float one-hot (:471-488)."""
        if self._map is None:
            E = len(self.messages)
            m = torch.zeros((E, self.num_variables))
            m[torch.arange(E), torch.as_tensor(self.edge_var.astype(np.int64))] = 1.0
            self._map = m
        return self._map

    @property
    def message_type_map(self):
        """{(check, variable): message id} -- what the reference's Custom* factory expects of its
        converter (MGD:1273-1286)."""
        return {(c, v): m for m, (v, c) in enumerate(self.messages)}

    def message_to_var_index(self):
        """The 1-D message -> variable index (the mapping form the decoder wants)."""
        return torch.as_tensor(self.edge_var.astype(np.int64))

    def get_message_types(self, base_graph=None, Z=None):
        """:490-536: index of the block's shift among the sorted distinct shifts (0 without args)."""
        E = len(self.messages)
        if base_graph is None or Z is None:
            return torch.zeros(E, dtype=torch.long)
        base = np.asarray(torch.as_tensor(base_graph).cpu(), dtype=np.float64)
        shifts = sorted({int(s) for s in base.ravel() if s >= 0})
        idx = {s: i for i, s in enumerate(shifts)}
        sh = base[self.edge_chk // Z, self.edge_var // Z]
        return torch.tensor([idx[int(s)] if s >= 0 else 0 for s in sh], dtype=torch.long)


def create_message_gnn_decoder(H, num_iterations=5, hidden_dim=64, base_graph=None, Z=None):
    """message_gnn_decoder.py:539-582 -> (decoder, converter)."""
    converter = TannerToMessageGraph(H)
    num_messages = len(converter.messages)
    if base_graph is not None and Z is not None:
        base = np.asarray(torch.as_tensor(base_graph).cpu())
        shifts = {int(s) for s in base.ravel() if s >= 0}
        num_message_types = len(shifts) if shifts else 1
    else:
        num_message_types = 1
    decoder = MessageGNNDecoder(num_messages=num_messages, num_iterations=num_iterations,
                                hidden_dim=hidden_dim, num_message_types=num_message_types)
    return decoder, converter


def load_message_gnn_model(model_path, H, device):
    """run_comparison_all.py:124-143: rebuild a decoder from a saved_models checkpoint
    ({'model_state_dict', ['num_iterations'], ['hidden_dim']}); loaded with weights_only=True."""
    checkpoint = torch.load(model_path, map_location="cpu", weights_only=True)
    num_iterations = checkpoint.get("num_iterations", 5)
    hidden_dim = checkpoint.get("hidden_dim", 64)
    sd = checkpoint["model_state_dict"]
    T = sd["gnn_layers.0.message_type_embeddings"].shape[0]
    decoder, converter = create_message_gnn_decoder(H, num_iterations=num_iterations,
                                                    hidden_dim=hidden_dim)
    if T != 1:
        decoder = MessageGNNDecoder(len(converter.messages), num_iterations, hidden_dim, T)
    decoder.load_state_dict(sd)
    return decoder.to(device), converter


# Hybrid Custom* decoders (MGD:585-1291), importable from here as in the reference
from ldpc_neural_decoder.models.custom_decoders import (  # noqa: E402
    CustomCheckMessageGNNLayer, CustomMinSumMessageGNNDecoder, CustomVariableMessageGNNDecoder,
    CustomVariableMessageGNNLayer, create_check_index_tensor, create_custom_minsum_message_gnn_decoder,
    create_custom_variable_message_gnn_decoder, create_variable_index_tensor)
