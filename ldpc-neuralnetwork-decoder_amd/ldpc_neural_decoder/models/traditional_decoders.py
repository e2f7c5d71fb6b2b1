"""Flooding sum-product and scaled min-sum decoders (drop-in for models/traditional_decoders.py).

Same constructors, attributes and ``decode(llr) -> (decoded_bits, iterations)`` contract as the
reference (traditional_decoders.py:4-285); the iteration loop runs in libldpc_amd's
LDS-resident HIP kernel (csrc/flood.hip).  Min-sum decisions are bitwise identical to the
reference; BP agrees within float32 tolerance (see DESIGN.md "Parity").

Differences by design:
  * llr on the CPU is moved to the current HIP device and the bits are moved back (the
    reference follows llr.device); there is no CPU compute path.
  * ``early_stopping=True`` keeps the reference's batch-global rule (stop at the first iteration
    at which EVERY frame satisfies H x = 0, :104-107).  ``early_stopping="frame"`` selects the
    per-frame freeze, an extension with no reference counterpart.
"""
import numpy as np
import torch

from ldpc_neural_decoder import _native as N
from ldpc_neural_decoder.utils.ldpc_utils import edge_list


class _FloodDecoder:
    _algo = None

    def __init__(self, H, max_iterations=50, early_stopping=True):
        self.H = H
        self.max_iterations = max_iterations
        self.early_stopping = early_stopping
        self._graphs = {}
        self._precompute_indices()

    def _precompute_indices(self):
        """traditional_decoders.py:26-40: check_to_var / var_to_check lists (ascending)."""
        m, n = self.H.shape
        self._edge_chk, self._edge_var = edge_list(self.H)
        self.check_to_var = [[] for _ in range(m)]
        self.var_to_check = [[] for _ in range(n)]
        for i, j in zip(self._edge_chk.tolist(), self._edge_var.tolist()):
            self.check_to_var[i].append(j)
            self.var_to_check[j].append(i)

    def graph(self, device):
        key = str(device)
        if key not in self._graphs:
            m, n = self.H.shape
            self._graphs[key] = N.NativeGraph(self._edge_chk, self._edge_var, m, n, device)
        return self._graphs[key]

    def _es_mode(self):
        if self.early_stopping == "frame":
            return N.LDPC_ES_FRAME
        return N.LDPC_ES_BATCH if self.early_stopping else N.LDPC_ES_OFF

    def _alpha(self):
        return 0.0

    def decode(self, llr, out_dtype=torch.float32, counters=None, return_frame_iters=False):
        """llr (B, N) float32 -> (decoded_bits (B, N) float32 0/1, iterations: int).

        counters: optional int64[4] device tensor += [bit errors vs all-zero, frame errors,
        frames, iteration sum] (the sweep's fused BER/FER counting).  `iterations` is a Python int
        as in the reference (traditional_decoders.py:107-109): with early stopping that is one host
        sync (the sweep uses decode_async, which never waits)."""
        out = self.decode_async(llr, out_dtype, counters, return_frame_iters)
        it = out[1]
        if torch.is_tensor(it):
            it = int(it.item())
        return (out[0], it) + tuple(out[2:])

    def decode_async(self, llr, out_dtype=torch.float32, counters=None, return_frame_iters=False):
        """decode() without a host sync: with early stopping `iterations` is a device int32 scalar
        (its value is also in the counters' iteration sum).  The sweep's entry point."""
        if self.max_iterations < 1:
            # the reference's loop never binds decoded_bits (traditional_decoders.py:109)
            raise UnboundLocalError("local variable 'decoded_bits' referenced before assignment")
        home = llr.device
        dev = N.device_of(llr)
        x = llr.to(dev, torch.float32).contiguous()
        if x.dim() != 2 or x.shape[1] != self.H.shape[1]:
            raise ValueError(f"llr must be (batch, {self.H.shape[1]}), got {tuple(llr.shape)}")
        g = self.graph(dev)
        B = x.shape[0]
        es = self._es_mode()
        bits = torch.empty((B, g.N), dtype=out_dtype, device=dev)
        kind = N.LDPC_OUT_F32 if out_dtype == torch.float32 else N.LDPC_OUT_U8
        batch_iters = torch.zeros(1, dtype=torch.int32, device=dev)
        frame_iters = torch.empty(B, dtype=torch.int32, device=dev) if return_frame_iters else None
        wsb = N.check(N.lib().ldpc_flood_workspace_size(g.handle, B, self.max_iterations, es))
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
        N.check(N.lib().ldpc_flood_decode(
            g.handle, self._algo, N.ptr(x), B, int(self.max_iterations), float(self._alpha()), es,
            kind, N.ptr(bits), N.ptr(frame_iters), N.ptr(batch_iters), N.ptr(counters), N.ptr(ws),
            wsb, N.stream_ptr(dev)))
        if es == N.LDPC_ES_OFF:
            iterations = self.max_iterations
        else:
            iterations = batch_iters[0]
        if home != dev:
            bits = bits.to(home)
        if return_frame_iters:
            return bits, iterations, frame_iters
        return bits, iterations

    def _check_valid_codeword(self, decoded_bits):
        """traditional_decoders.py:111-134: (B,) bool, True where H x = 0 (mod 2)."""
        Hd = torch.as_tensor(self.H, dtype=torch.float32, device=decoded_bits.device)
        par = torch.remainder(decoded_bits.float() @ Hd.T, 2.0)
        return (par == 0).all(dim=1)


class BeliefPropagationDecoder(_FloodDecoder):
    """Flooding sum-product (traditional_decoders.py:4-134)."""
    _algo = N.LDPC_ALGO_BP

    def __init__(self, H, max_iterations=50, early_stopping=True):
        super().__init__(H, max_iterations, early_stopping)


class MinSumScaledDecoder(_FloodDecoder):
    """Scaled min-sum (traditional_decoders.py:137-285); c2v = prod sign * (alpha * min)."""
    _algo = N.LDPC_ALGO_MINSUM

    def __init__(self, H, max_iterations=50, scaling_factor=0.75, early_stopping=True):
        self.scaling_factor = scaling_factor
        super().__init__(H, max_iterations, early_stopping)

    def _alpha(self):
        return self.scaling_factor
