"""Python side of the CPU oracle.  TEST INFRASTRUCTURE ONLY — never imported by the product.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this module.
It is pinned against the golden fixtures in tests/golden/ (made by importing the reference
itself, tests/golden/make_golden.py); see tests/test_oracle_golden.py.

Contents
  load_base / expand / edge_lists   restate utils/ldpc_utils.py:97-147 and the check-major edge
                                    order of message_gnn_decoder.py:397-406
  flood_decode                      ctypes front-end of oracle/ldpc_oracle.c (min-sum / BP,
                                    traditional_decoders.py:42-134, 177-285)
  gnn_forward                       torch-fp32 restatement of MessageGNNDecoder.forward
                                    (message_gnn_decoder.py:51-129, 190-317) with the normalized
                                    clique adjacency written as a segment mean (the identity
                                    D^-1/2 (A+I) D^-1/2 = group mean, message_gnn_decoder.py:423-469)
  message_types                     restates TannerToMessageGraph.get_message_types (MGD:490-536)
"""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(HERE, "_build", "libldpc_oracle.so")
_lib = None


def build():
    subprocess.run(["make", "-s", "-C", HERE], check=True)


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        P = ctypes.c_void_p
        _lib.ldpc_oracle_flood_decode.restype = ctypes.c_int
        _lib.ldpc_oracle_flood_decode.argtypes = [
            ctypes.c_int, ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P, P,
            ctypes.c_int64, ctypes.c_int, ctypes.c_float, ctypes.c_int, P, P, P]
        _lib.ldpc_oracle_expand.argtypes = [P, ctypes.c_int, ctypes.c_int, ctypes.c_int, P]
        _lib.ldpc_oracle_syndrome.argtypes = [ctypes.c_int, P, P, ctypes.c_int, P,
                                              ctypes.c_int64, P]
        _lib.ldpc_oracle_set_threads.argtypes = [ctypes.c_int]
        _lib.ldpc_oracle_set_threads.restype = ctypes.c_int
        _lib.ldpc_oracle_custom_minsum.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_int, P, P, P, P, P,
                                                   ctypes.c_int64, ctypes.c_int, P]
        _lib.ldpc_oracle_custom_minsum.restype = ctypes.c_int
    return _lib


def set_threads(n):
    """Host threads of flood_decode's frame loop (OpenMP); returns the count in use.  Only the
    timed CPU baseline (bench.py) uses more than 1."""
    return lib().ldpc_oracle_set_threads(int(n))


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


# --------------------------------------------------------------------------- codes
def load_base(path):
    """utils/ldpc_utils.py:127-147: whitespace floats, one row per line."""
    with open(path) as f:
        rows = [[float(x) for x in line.split()] for line in f if line.strip()]
    return np.array(rows, dtype=np.float64)


def expand(base, z):
    """utils/ldpc_utils.py:97-125 via the C restatement -> dense uint8 H (M, N)."""
    b = np.ascontiguousarray(base, dtype=np.int32)
    H = np.zeros((b.shape[0] * z, b.shape[1] * z), dtype=np.uint8)
    lib().ldpc_oracle_expand(_p(b), b.shape[0], b.shape[1], z, _p(H))
    return H


class Graph:
    """Check-major edge list of a dense H (message_gnn_decoder.py:397-406)."""

    def __init__(self, H):
        H = np.asarray(H)
        self.M, self.N = H.shape
        chk, var = np.nonzero(H == 1)  # row-major nonzero = checks ascending, vars ascending
        self.edge_chk = chk.astype(np.int32)
        self.edge_var = var.astype(np.int32)
        self.E = len(chk)
        self.chk_ptr = np.zeros(self.M + 1, dtype=np.int32)
        np.cumsum(np.bincount(chk, minlength=self.M), out=self.chk_ptr[1:])
        order = np.lexsort((chk, var))  # by var, then ascending check
        self.var_edge = order.astype(np.int32)
        self.var_ptr = np.zeros(self.N + 1, dtype=np.int32)
        np.cumsum(np.bincount(var, minlength=self.N), out=self.var_ptr[1:])


def flood_decode(graph, llr, algo, max_iter, alpha=0.75, early_stop=0):
    """algo 'minsum' | 'bp'.  Returns (bits uint8 (B,N), app f32 (B,N), iterations, iters[B])."""
    llr = np.ascontiguousarray(llr, dtype=np.float32)
    B = llr.shape[0]
    bits = np.zeros((B, graph.N), dtype=np.uint8)
    app = np.zeros((B, graph.N), dtype=np.float32)
    iters = np.zeros(B, dtype=np.int32)
    r = lib().ldpc_oracle_flood_decode(
        0 if algo == "minsum" else 1, graph.M, graph.N, graph.E, _p(graph.chk_ptr),
        _p(graph.edge_var), _p(graph.var_ptr), _p(graph.var_edge), _p(llr), B, max_iter,
        float(alpha), int(early_stop), _p(bits), _p(app), _p(iters))
    if r < 0:
        raise MemoryError("oracle allocation failed")
    return bits, app, r, iters


def custom_minsum(graph, llr, iterations):
    """Hybrid min-sum (CustomMinSumMessageGNNDecoder, message_gnn_decoder.py:1167-1251) under the
    semantics this build defines for it (ldpc_oracle.c).  Returns probs f32 (B, N)."""
    llr = np.ascontiguousarray(llr, dtype=np.float32)
    probs = np.zeros_like(llr)
    r = lib().ldpc_oracle_custom_minsum(graph.M, graph.N, graph.E, _p(graph.chk_ptr), _p(graph.edge_var),
                                        _p(graph.var_ptr), _p(graph.var_edge), _p(llr), llr.shape[0],
                                        int(iterations), _p(probs))
    if r < 0:
        raise MemoryError("oracle allocation failed")
    return probs


def syndrome_valid(graph, bits):
    bits = np.ascontiguousarray(bits, dtype=np.uint8)
    valid = np.zeros(bits.shape[0], dtype=np.uint8)
    lib().ldpc_oracle_syndrome(graph.M, _p(graph.chk_ptr), _p(graph.edge_var), graph.N,
                               _p(bits), bits.shape[0], _p(valid))
    return valid.astype(bool)


def message_types(graph, base, z):
    """TannerToMessageGraph.get_message_types (message_gnn_decoder.py:490-536)."""
    base = np.asarray(base)
    shifts = sorted({int(s) for s in base.ravel() if s >= 0})
    idx = {s: i for i, s in enumerate(shifts)}
    sh = base[graph.edge_chk // z, graph.edge_var // z]
    return np.array([idx[int(s)] if s >= 0 else 0 for s in sh], dtype=np.int64)


# --------------------------------------------------------------------------- GNN (torch fp32)
def gnn_forward(sd, llr, msg_var_io, edge_var, edge_chk, num_vars, num_checks, types=None,
                ground_truth=None, all_layers=False, dtype=None):
    """MessageGNNDecoder.forward restated (message_gnn_decoder.py:190-317).

    all_layers  (training extension, no reference counterpart) return the (L, B, N) probs of every
                layer's output through the LAST layer's output_projection (the decoder's
                forward_all_layers / deep supervision); the last entry is the reference's probs.
    dtype       None: float32, the reference's arithmetic; torch.float64 gives the exact-arithmetic
                yardstick the fp32 kernels' errors are measured against

    sd          state_dict (tensors) in the reference's key schema
    msg_var_io  (E,) int64 message->variable index used for the LLR gather and the output sum
                (the reference's `message_to_var_mapping`, 1-D form; MGD:218-229, 285-295)
    edge_var/edge_chk  the Tanner-graph groups that the normalized adjacencies encode
    """
    import torch
    import torch.nn.functional as F

    dt = dtype or torch.float32
    llr = torch.as_tensor(llr).to(dt)
    if dtype is not None:
        sd = {k: v.to(dt) for k, v in sd.items()}
    B, E = llr.shape[0], len(edge_var)
    mv = torch.as_tensor(msg_var_io, dtype=torch.long)
    ev = torch.as_tensor(edge_var, dtype=torch.long)
    ec = torch.as_tensor(edge_chk, dtype=torch.long)
    n_layers = len({k.split(".")[1] for k in sd if k.startswith("gnn_layers.")})
    x = llr[:, mv].unsqueeze(-1) * sd["input_embedding.weight"][:, 0] + sd["input_embedding.bias"]
    t = torch.zeros(E, dtype=torch.long) if types is None else torch.as_tensor(types).long()
    deg_v = torch.bincount(ev, minlength=num_vars).to(dt)
    deg_c = torch.bincount(ec, minlength=num_checks).to(dt)

    def seg_mean(c, idx, deg, n):
        s = torch.zeros(B, n, c.shape[-1], dtype=dt).index_add_(1, idx, c)
        return (s / deg.clamp(min=1).view(1, -1, 1))[:, idx]

    def mlp(p, z):
        h = torch.relu(z @ sd[p + ".0.weight"].T + sd[p + ".0.bias"])
        return h @ sd[p + ".2.weight"].T + sd[p + ".2.bias"]

    last = f"gnn_layers.{n_layers - 1}.output_projection."

    def head(x):
        out = (x @ sd[last + "weight"][0]) + sd[last + "bias"][0]
        var_llrs = torch.zeros(B, num_vars, dtype=dt).index_add_(1, mv, out)
        return torch.sigmoid(var_llrs + llr)

    per_layer = []
    for i in range(n_layers):
        p = f"gnn_layers.{i}."
        emb = sd[p + "message_type_embeddings"]
        c = x + emb[t.clamp(0, emb.shape[0] - 1)]
        a = seg_mean(c, ev, deg_v, num_vars)
        b = seg_mean(c, ec, deg_c, num_checks)
        y = mlp(p + "var_to_check_update", torch.cat([c, a], 2)) + \
            mlp(p + "check_to_var_update", torch.cat([c, b], 2))
        x = y + x if i > 0 else y
        if all_layers and i < n_layers - 1:
            per_layer.append(head(x))
    probs = head(x)
    if all_layers:
        return torch.stack(per_layer + [probs])
    if ground_truth is not None:
        return probs, F.binary_cross_entropy(probs, torch.as_tensor(ground_truth).float())
    return probs


def custom_variable_forward(sd, llr, msg_var_io, edge_chk, num_vars, num_checks, types=None, check_identity=False,
                            ground_truth=None):
    """CustomVariableMessageGNNDecoder.forward (message_gnn_decoder.py:798-879, layer :672-755) under the
    semantics this build defines for it (models/custom_decoders.py; the reference cannot run it):
    per layer the check side's MLP over [c; A_c c] (A_c = group mean over the check's messages, or the
    identity), the layer's output head on it, the damped min-sum variable update on those LLRs and the
    decoder's Linear(1, H) back to features; output = sigmoid(mean of the last head over a variable's
    messages + llr).  torch fp32; returns probs, or (probs, max per-bit BCE) with ground truth."""
    import torch
    import torch.nn.functional as F

    llr = torch.as_tensor(llr, dtype=torch.float32)
    mv = torch.as_tensor(msg_var_io, dtype=torch.long)
    ec = torch.as_tensor(edge_chk, dtype=torch.long)
    B, E = llr.shape[0], mv.numel()
    n_layers = len({k.split(".")[1] for k in sd if k.startswith("gnn_layers.")})
    w_in, b_in = sd["input_embedding.weight"][:, 0], sd["input_embedding.bias"]
    x = llr[:, mv].unsqueeze(-1) * w_in + b_in
    t = torch.zeros(E, dtype=torch.long) if types is None else torch.as_tensor(types).long()
    deg_c = torch.bincount(ec, minlength=num_checks).float()
    deg_v = torch.bincount(mv, minlength=num_vars).float()

    def mlp(p, z):
        h = torch.relu(z @ sd[p + ".0.weight"].T + sd[p + ".0.bias"])
        return h @ sd[p + ".2.weight"].T + sd[p + ".2.bias"]

    for i in range(n_layers):
        p = f"gnn_layers.{i}."
        emb = sd[p + "message_type_embeddings"]
        c = x + emb[t.clamp(0, emb.shape[0] - 1)]
        if check_identity:
            b = c
        else:
            s = torch.zeros(B, num_checks, c.shape[-1]).index_add_(1, ec, c)
            b = (s / deg_c.clamp(min=1).view(1, -1, 1))[:, ec]
        Fm = mlp(p + "check_to_var_update", torch.cat([c, b], 2))
        lm = Fm @ sd[p + "output_projection.weight"][0] + sd[p + "output_projection.bias"][0]
        tot = llr + torch.zeros(B, num_vars).index_add_(1, mv, lm)
        v2c = tot[:, mv] - lm
        v2c = 0.5 * v2c + 0.5 * lm
        x = (v2c.unsqueeze(-1) * w_in + b_in) + Fm
    last = f"gnn_layers.{n_layers - 1}.output_projection."
    out = (x @ sd[last + "weight"][0]) + sd[last + "bias"][0]
    w = 1.0 / (deg_v + 1e-10)
    var_llrs = torch.zeros(B, num_vars).index_add_(1, mv, out * w[mv])
    probs = torch.sigmoid(var_llrs + llr)
    if ground_truth is not None:
        loss = F.binary_cross_entropy(probs, torch.as_tensor(ground_truth).float(), reduction="none")
        return probs, loss.max(dim=1).values
    return probs


def gnn_forward_dense(sd, llr, msg_var_io, num_vars, Av, Ac, types=None):
    """MessageGNNDecoder.forward restated with the reference's own aggregation: dense
    bmm(A, x + emb) with whatever adjacencies are given, zero-padded / cropped to E as
    message_gnn_decoder.py:92-104 does (MessageGNNLayer.forward :51-129, decoder :190-317).  Used
    to pin the general-adjacency path; gnn_forward above is the segment-mean form of the same math
    for the TannerToMessageGraph cliques."""
    import torch

    llr = torch.as_tensor(llr, dtype=torch.float32)
    mv = torch.as_tensor(msg_var_io, dtype=torch.long)
    B, E = llr.shape[0], mv.numel()
    n_layers = len({k.split(".")[1] for k in sd if k.startswith("gnn_layers.")})
    x = llr[:, mv].unsqueeze(-1) * sd["input_embedding.weight"][:, 0] + sd["input_embedding.bias"]
    t = torch.zeros(E, dtype=torch.long) if types is None else torch.as_tensor(types).long()
    Av, Ac = torch.as_tensor(Av, dtype=torch.float32), torch.as_tensor(Ac, dtype=torch.float32)
    if Av.size(0) != E or Av.size(1) != E:  # :92-104
        nv, nc = torch.zeros(E, E), torch.zeros(E, E)
        k = min(Av.size(0), E)
        nv[:k, :k] = Av[:k, :k]
        nc[:k, :k] = Ac[:k, :k]
        Av, Ac = nv, nc

    def mlp(p, z):
        h = torch.relu(z @ sd[p + ".0.weight"].T + sd[p + ".0.bias"])
        return h @ sd[p + ".2.weight"].T + sd[p + ".2.bias"]

    for i in range(n_layers):
        p = f"gnn_layers.{i}."
        emb = sd[p + "message_type_embeddings"]
        c = x + emb[t.clamp(0, emb.shape[0] - 1)]
        a = torch.bmm(Av.unsqueeze(0).expand(B, -1, -1), c)
        b = torch.bmm(Ac.unsqueeze(0).expand(B, -1, -1), c)
        y = mlp(p + "var_to_check_update", torch.cat([c, a], 2)) + mlp(p + "check_to_var_update", torch.cat([c, b], 2))
        x = y + x if i > 0 else y
    last = f"gnn_layers.{n_layers - 1}.output_projection."
    out = (x @ sd[last + "weight"][0]) + sd[last + "bias"][0]
    var_llrs = torch.zeros(B, num_vars).index_add_(1, mv, out)
    return torch.sigmoid(var_llrs + llr)


# --------------------------------------------------------------------------- index-gather layers
# Restatement of models/layers.py:5-208 and utils/ldpc_utils.py:5-95 (var-major edge mapping),
# in torch ops so that autograd gives the reference gradients (test infrastructure only).
def llr_mapping(H):
    """ldpc_utils.py:62-95 with H_T = H.T: LLR index i = i-th nonzero of H_T in row-major order
    (variables outer, checks inner); neighbour lists in ascending LLR index, -1 padded."""
    import torch
    HT = np.asarray(H, dtype=np.float32).T
    rows, cols = np.nonzero(HT == 1)
    E = len(rows)
    m = np.full(HT.shape, -1, dtype=np.int64)
    m[rows, cols] = np.arange(E)
    mT = m.T  # (checks, vars)
    def neighbours(mat):
        lists = [[] for _ in range(E)]
        for r in range(mat.shape[0]):
            ids = mat[r][mat[r] >= 0]
            for a in ids:
                lists[a] = [int(b) for b in ids if b != a]
        K = max(len(x) for x in lists)
        out = np.full((E, K), -1, dtype=np.int64)
        for a, x in enumerate(lists):
            out[a, :len(x)] = x
        return out
    return (torch.from_numpy(mT.copy()), torch.from_numpy(neighbours(mT)),
            torch.from_numpy(neighbours(m)), torch.from_numpy(rows.astype(np.int64)[None, :]))


def _gathered(x, idx):
    import torch
    valid = idx >= 0
    v = x[:, idx.clamp(min=0)]                       # (B, n_out, K)
    return torch.where(valid.unsqueeze(0), v, torch.zeros_like(v)), valid


def check_layer(x, idx):
    """layers.py:14-66: prod sign(v + 1e-10) * min |v| (|0| -> 1e10, padding -> 0)."""
    import torch
    v, _ = _gathered(x, idx)
    sp = torch.prod(torch.sign(v + 1e-10), dim=2)
    a = torch.abs(v)
    a = torch.where(a == 0, torch.full_like(a, 1e10), a)
    return sp * torch.min(a, dim=2).values


def variable_layer(llr, msgs, idx):
    """layers.py:78-125: llr + sum of the gathered messages (padding -> 0)."""
    import torch
    v, _ = _gathered(msgs, idx)
    return llr + torch.sum(v, dim=2)


def residual_layer(llr, cm, prevs, w_ch, w_res):
    """layers.py:143-168."""
    r = llr * w_ch.unsqueeze(0) + cm
    for i, p in enumerate(prevs):
        if i < w_res.shape[0]:
            r = r + w_res[i] * p
    return r


def output_layer(final, llr, gt=None):
    """layers.py:180-208: sigmoid(final + llr); with gt, the per-frame max of the elementwise BCE."""
    import torch
    import torch.nn.functional as F
    soft = torch.sigmoid(final + llr)
    if gt is None:
        return soft, None
    return soft, torch.max(F.binary_cross_entropy(soft, gt, reduction="none"), dim=1).values


def neural_decoder(params, llr, check_idx, var_idx, var_of_edge, depth_L, gt=None):
    """models/decoder.py's LDPCNeuralDecoder composed from the layer restatements above (the
    reference's models/decoder.py is missing: the composition is the build's definition, the
    layers are the reference's).  params: [(w_ch, w_res)] per variable layer; var_of_edge (E,)."""
    import torch
    n = llr.shape[1]
    x0 = llr[:, var_of_edge]
    v, prevs = x0, []
    zero = torch.zeros_like(x0)
    for w_ch, w_res in params:
        c = check_layer(v, check_idx)
        v = residual_layer(x0, variable_layer(zero, c, var_idx), prevs, w_ch, w_res)
        prevs = [v] + prevs[:max(depth_L - 1, 0)]
    c = check_layer(v, check_idx)
    app = torch.zeros((llr.shape[0], n), dtype=llr.dtype).index_add(1, var_of_edge, c)
    return output_layer(-app, -llr, gt)


# --------------------------------------------------------------------------- Philox-4x32-10
def philox4x32_10(ctr, key):
    """Random123 Philox-4x32-10 (Salmon et al., SC'11) on uint32 arrays.
    ctr: (n, 4) uint32, key: (2,) uint32 -> (n, 4) uint32.  Used to pin the HIP channel RNG."""
    M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
    W0, W1 = np.uint32(0x9E3779B9), np.uint32(0xBB67AE85)
    c = np.array(ctr, dtype=np.uint32).reshape(-1, 4).copy()
    k0 = np.full(c.shape[0], key[0], dtype=np.uint32)
    k1 = np.full(c.shape[0], key[1], dtype=np.uint32)
    mask = np.uint64(0xFFFFFFFF)
    for _ in range(10):
        p0 = M0 * c[:, 0].astype(np.uint64)
        p1 = M1 * c[:, 2].astype(np.uint64)
        hi0, lo0 = (p0 >> np.uint64(32)).astype(np.uint32), (p0 & mask).astype(np.uint32)
        hi1, lo1 = (p1 >> np.uint64(32)).astype(np.uint32), (p1 & mask).astype(np.uint32)
        c = np.stack([hi1 ^ c[:, 1] ^ k0, lo1, hi0 ^ c[:, 3] ^ k1, lo0], axis=1)
        k0 = k0 + W0
        k1 = k1 + W1
    return c


def awgn_llr(batch, n, snr_db, seed, frame_offset=0, bits=None, bpsk=False):
    """Restatement of the fused on-device channel (csrc/channel.hip) in float64 numpy: the Philox
    stream above, Box-Muller, then the reference's float32 formulas (utils/channel.py:39 and
    :81-86 / :137-143 for QPSK, :217-230 for BPSK AWGNChannel.transmit).  The noise generator is
    this build's (Philox + Box-Muller instead of torch's mt19937), so this pins the kernel's
    arithmetic, not the reference's draws.  Returns (batch, n) float64."""
    snr = 10.0 ** (snr_db / 10.0)
    if bpsk:
        std = np.float32(1.0 / np.sqrt(snr))
        denom = np.float32(float(std) ** 2)
    else:
        std = np.float32(np.sqrt((1.0 / snr) / 2.0))
        denom = np.float32(1.0 / snr)
    quads = (n + 3) // 4
    j = np.tile(np.arange(quads, dtype=np.uint64), batch)
    fr = np.repeat(np.arange(batch, dtype=np.uint64) + np.uint64(frame_offset), quads)
    tag = 0xC4A77E11 ^ (1 if bpsk else 0)
    ctr = np.stack([j.astype(np.uint32), (fr & np.uint64(0xFFFFFFFF)).astype(np.uint32),
                    (fr >> np.uint64(32)).astype(np.uint32), np.full(j.shape, tag, np.uint32)], 1)
    w = philox4x32_10(ctr, [seed & 0xFFFFFFFF, (seed >> 32) & 0xFFFFFFFF]).astype(np.float64)
    u = (np.floor(w / 256.0) + 0.5) / 16777216.0          # 24 bits centred: never 0 or 1
    r0, r1 = np.sqrt(-2 * np.log(u[:, 0])), np.sqrt(-2 * np.log(u[:, 2]))
    t0, t1 = 2 * np.pi * u[:, 1], 2 * np.pi * u[:, 3]
    noise = np.stack([r0 * np.cos(t0), r0 * np.sin(t0), r1 * np.cos(t1), r1 * np.sin(t1)], 1)
    noise = noise.reshape(batch, quads * 4)[:, :n]
    b = np.zeros((batch, n)) if bits is None else np.asarray(bits, dtype=np.float64)
    if bpsk:
        sym = 1.0 - 2.0 * b
    else:
        sym = float(np.float32(1 / np.sqrt(2))) - b * float(np.float32(np.sqrt(2)))
    return 2.0 * (sym + noise * float(std)) / float(denom)
