"""The systematic encoder behind the GNN checkpoint's training data (utils/encoding.py; CPU)."""
import numpy as np
import pytest
import torch

from conftest import code_path

from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix
from ldpc_neural_decoder.utils.encoding import SystematicEncoder


@pytest.mark.parametrize("z", [4, 32])
def test_codewords_satisfy_every_check(z):
    H = expand_base_matrix(load_base_matrix(code_path(z)), z)
    enc = SystematicEncoder(H)
    assert enc.K == H.shape[1] - H.shape[0] == 10 * z
    g = torch.Generator().manual_seed(z)
    c = enc.random(33, generator=g)
    assert c.shape == (33, H.shape[1])
    Hn = H.numpy().astype(np.int64)
    assert not ((c.numpy().astype(np.int64) @ Hn.T) % 2).any()
    assert bool(enc.syndrome_ok(c).all())
    # systematic: the information bits come first; linear: c(u1 ^ u2) = c(u1) ^ c(u2)
    u = c[:, :enc.K]
    assert torch.equal(enc.encode(u), c)
    u2 = torch.roll(u, 1, dims=0)
    assert torch.equal(enc.encode((u + u2) % 2), (enc.encode(u) + enc.encode(u2)) % 2)


def test_singular_parity_part_refused():
    H = torch.tensor([[1, 1, 0, 0], [0, 0, 1, 1]], dtype=torch.float32)  # parity part [[0,0],[1,1]]
    with pytest.raises(ValueError):
        SystematicEncoder(H)
