"""The sharded on-device harness around the REAL HIP decoders (GPU): two gloo ranks share the card
(torch.distributed.run in a child process), deal the trials round-robin, draw disjoint Philox
frames and sum their counters with one all-reduce (sweep.py).  The sharded BER / FER /
avg_iterations must equal a single-process run exactly (integer counts), for the classic decoders
(ComparativeEvaluator.evaluate_all, comparative_evaluation.py:40-166) and the message GNN
(evaluate_message_gnn, run_comparison_all.py:245-295)."""
import os
import subprocess
import sys

import pytest
import torch

from conftest import ROOT, code_path

from ldpc_neural_decoder.models import create_message_gnn_decoder
from ldpc_neural_decoder.sweep import ComparativeEvaluator, evaluate_message_gnn
from ldpc_neural_decoder.utils import expand_base_matrix, load_base_matrix

pytestmark = pytest.mark.gpu


def test_two_rank_sweep_equals_single_process(cuda, tmp_path):
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    out = tmp_path / "dist.pt"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(port),
           os.path.join(ROOT, "tests", "dist_sweep_worker.py"), code_path(4), "4", str(out)]
    r = subprocess.run(cmd, env=env, timeout=240, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    d = torch.load(out, weights_only=True)
    assert d["world"] == 2

    base = load_base_matrix(code_path(4))
    H = expand_base_matrix(base, 4)
    snrs = [0.0, 2.0, 4.0]
    ev = ComparativeEvaluator(H, device=cuda, seed=17)
    ev.bp_decoder.max_iterations = ev.ms_decoder.max_iterations = 8
    single = ev.evaluate_all(snrs, batch_size=48, num_trials=5)
    assert d["results"] == single
    assert single["min_sum_scaled"]["ber"][0] > 0  # errors present: the comparison is not trivial
    dec, conv = create_message_gnn_decoder(H, num_iterations=3, hidden_dim=32, base_graph=base, Z=4)
    dec.load_state_dict(d["sd"])
    gnn = evaluate_message_gnn(dec, conv, snrs, 40, 3, cuda, seed=23, message_types=conv.get_message_types(base, 4))
    assert tuple(d["gnn"]) == tuple(gnn)
