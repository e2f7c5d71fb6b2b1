"""Systematic encoder for a parity-check matrix (training data for the message GNN).

The reference never encodes: every harness sends the all-zero codeword (comparative_evaluation.py:133,
run_comparison_all.py:163) and its trainer draws random bits that are not codewords
(trainer.py:85).  A decoder trained on non-codewords can only learn a per-bit detector, so the
checkpoint this build ships (tools/train_gnn_checkpoint.py) trains on random codewords instead.

For H = [A | P] with the parity part P (the last M columns) invertible over GF(2) -- true for the 5G
base graphs, whose parity part is the dual-diagonal core plus the identity extension -- the
codeword of information bits u (the first N - M positions) is [u, P^-1 A u mod 2].  P^-1 A is
computed once on the host by Gauss-Jordan elimination on bit-packed rows; encoding is one matmul
on the device (exact: at most K ones are summed in float32, K < 2^24).
"""
import numpy as np
import torch


def _gf2_solve(P, A):
    """X with P X = A over GF(2) (P square invertible, uint8 0/1), by elimination on packed rows."""
    M = P.shape[0]
    K = A.shape[1]
    aug = np.concatenate([P, A], axis=1).astype(np.uint8)
    packed = np.packbits(aug, axis=1)  # rows as bytes
    for col in range(M):
        byte, bit = divmod(col, 8)
        mask = np.uint8(0x80 >> bit)
        rows = np.nonzero(packed[col:, byte] & mask)[0]
        if len(rows) == 0:
            raise ValueError("the parity part of H is singular over GF(2): no systematic encoder")
        piv = col + rows[0]
        if piv != col:
            packed[[col, piv]] = packed[[piv, col]]
        hit = np.nonzero(packed[:, byte] & mask)[0]
        hit = hit[hit != col]
        packed[hit] ^= packed[col]
    return np.unpackbits(packed, axis=1)[:, M:M + K]


class SystematicEncoder:
    """encode(u) -> codewords (B, N) float32 0/1 on the device of u; random(B) draws u uniformly."""

    def __init__(self, H, device=None):
        Hn = np.asarray(torch.as_tensor(H).cpu(), dtype=np.float32).astype(np.uint8)
        M, N = Hn.shape
        self.M, self.N, self.K = M, N, N - M
        parity = _gf2_solve(Hn[:, self.K:], Hn[:, :self.K])  # (M, K): p = parity @ u
        self.device = torch.device(device) if device is not None else torch.device("cpu")
        self._par = torch.from_numpy(parity.astype(np.float32)).to(self.device)
        self._H = torch.from_numpy(Hn.astype(np.float32)).to(self.device)

    def encode(self, u):
        u = torch.as_tensor(u, dtype=torch.float32, device=self.device)
        p = torch.remainder(u @ self._par.T, 2.0)
        return torch.cat([u, p], dim=1)

    def random(self, batch, generator=None):
        u = torch.randint(0, 2, (batch, self.K), device=self.device, generator=generator).float()
        return self.encode(u)

    def syndrome_ok(self, c):
        """(B,) bool: H c = 0 (mod 2)."""
        return (torch.remainder(c.float() @ self._H.T, 2.0) == 0).all(dim=1)
