"""Harness and on-disk formats on the GPU: the assembled index-gather decoder
(models/decoder.py) against its oracle composition, the trainer (trainer.py:21-364 API), the
evaluator's results file, and the CLI's train -> evaluate -> compare -> visualize chain.

Parity: LDPCNeuralDecoder's composition is the build's definition (the reference's
models/decoder.py is missing) -- unpinned at that level; the layers are pinned by
tests/golden/layers_z4.npz.  Tolerance (fp32, stated): soft bits and per-frame losses within
1e-5 abs / 1e-5 rel of the oracle; parameter gradients within 1e-4 * max|g_ref| + 1e-6.  The
harness counts (BER/FER) are integers and compared exactly with a hand loop."""
import os

import numpy as np
import pytest
import torch

from conftest import code_path

from ldpc_neural_decoder.models import LDPCNeuralDecoder, create_message_gnn_decoder
from ldpc_neural_decoder.sweep import ComparativeEvaluator
from ldpc_neural_decoder.training import LDPCDecoderTrainer
from ldpc_neural_decoder.utils import awgn_llr, create_LLR_mapping, expand_base_matrix, load_base_matrix

pytestmark = pytest.mark.gpu


def _code(z):
    base = load_base_matrix(code_path(z))
    H = expand_base_matrix(base, z)
    _, cidx, vidx, out_idx = create_LLR_mapping(H.T)
    return base, H, cidx, vidx, out_idx[0]


def _decoder(E, iters, depth, seed=0):
    torch.manual_seed(seed)
    dec = LDPCNeuralDecoder(E, num_iterations=iters, depth_L=depth)
    with torch.no_grad():
        for res in dec.residual_layers:
            res.w_ch.copy_(torch.rand(E) + 0.5)
            res.w_res.copy_(torch.randn(depth) * 0.3)
    return dec


@pytest.mark.parametrize("z,iters,depth,B", [(4, 3, 2, 7), (4, 1, 2, 3), (32, 4, 3, 5)])
def test_neural_decoder_matches_oracle(cuda, oracle_mod, z, iters, depth, B):
    base, H, cidx, vidx, var_of = _code(z)
    dec = _decoder(cidx.shape[0], iters, depth)
    llr = torch.randn(B, H.shape[1]) * 3
    llr[0, :5] = 0.0                                  # exact zeros reach the check layer
    gt = (torch.rand(B, H.shape[1]) < 0.5).float()
    params = [(r.w_ch.detach().clone().requires_grad_(True), r.w_res.detach().clone().requires_grad_(True))
              for r in dec.residual_layers]
    ref_soft, ref_loss = oracle_mod.neural_decoder(params, llr, cidx, vidx, var_of, depth, gt)
    if params:                         # iters = 1: a single check layer, nothing to train
        ref_loss.mean().backward()
    dec = dec.to(cuda)
    soft, loss = dec(llr.to(cuda), cidx, vidx, gt.to(cuda))
    np.testing.assert_allclose(soft.detach().cpu().numpy(), ref_soft.detach().numpy(), atol=1e-5, rtol=1e-5)
    np.testing.assert_allclose(loss.detach().cpu().numpy(), ref_loss.detach().numpy(), atol=1e-5, rtol=1e-5)
    if params:
        loss.mean().backward()
    for res, (w_ch, w_res) in zip(dec.residual_layers, params):
        for g, g_ref in ((res.w_ch.grad, w_ch.grad), (res.w_res.grad, w_res.grad)):
            if g_ref is None:          # first variable layer: no previous layers, w_res unused
                g_ref = torch.zeros_like(g.cpu())
            err = float((g.cpu() - g_ref).abs().max())
            assert err <= 1e-4 * float(g_ref.abs().max()) + 1e-6
    hard = dec.decode(llr.to(cuda), cidx, vidx)
    assert torch.equal(hard.cpu(), (ref_soft.detach() > 0.5).float())


def test_neural_decoder_rejects_mismatched_shapes(cuda):
    base, H, cidx, vidx, _ = _code(4)
    dec = LDPCNeuralDecoder(cidx.shape[0] + 1, 2).to(cuda)
    with pytest.raises(RuntimeError):
        dec(torch.zeros(2, H.shape[1], device=cuda), cidx, vidx)
    dec = LDPCNeuralDecoder(cidx.shape[0], 2).to(cuda)
    with pytest.raises(RuntimeError):
        dec(torch.zeros(2, H.shape[1] + 3, device=cuda), cidx, vidx)


def test_trainer_train_validate_checkpoint(cuda, tmp_path):
    base, H, cidx, vidx, _ = _code(4)
    dec = LDPCNeuralDecoder(cidx.shape[0], num_iterations=3)
    tr = LDPCDecoderTrainer(dec, device=cuda, seed=3)
    hist = tr.train(num_epochs=4, batch_size=64, learning_rate=0.01, check_index_tensor=cidx, var_index_tensor=vidx,
                    snr_range=[0, 2, 4], variable_bit_length=H.shape[1], validation_interval=2)
    assert set(hist) == {"train_losses", "val_losses", "ber_history", "fer_history"}
    assert len(hist["train_losses"]) == 4 and len(hist["val_losses"]) == 2 and len(hist["ber_history"]) == 2
    assert all(np.isfinite(hist["train_losses"])) and all(0 <= b <= 1 for b in hist["ber_history"])
    assert dec.residual_layers[0].w_ch.grad is not None       # SGD stepped through the HIP backward
    path = tmp_path / "model.pt"
    tr.save_model(str(path))
    ck = torch.load(str(path), weights_only=True)             # trainer.py:344-350 schema
    assert set(ck) == {"model_state_dict", "train_losses", "val_losses", "ber_history", "fer_history"}
    assert ck["train_losses"] == hist["train_losses"]
    dec2 = LDPCNeuralDecoder(cidx.shape[0], num_iterations=3)
    tr2 = LDPCDecoderTrainer(dec2, device=cuda)
    tr2.load_model(str(path))
    for (k, a), (_, b) in zip(dec.state_dict().items(), dec2.state_dict().items()):
        assert torch.equal(a.cpu(), b.cpu()), k
    assert tr2.fer_history == hist["fer_history"]


def test_evaluate_snr_range_counts_exactly(cuda):
    """evaluate_snr_range (trainer.py:205-262) = a hand loop over the same LLRs (same Philox
    stream) with the decisions counted on the host."""
    base, H, cidx, vidx, _ = _code(4)
    dec = _decoder(cidx.shape[0], 3, 2).to(cuda)
    tr = LDPCDecoderTrainer(dec, device=cuda, seed=11)
    snrs, B, T, n = [-1, 2, 5], 48, 3, H.shape[1]
    ber, fer = tr.evaluate_snr_range(snrs, B, T, cidx, vidx, n)
    for si, snr in enumerate(snrs):
        bit_err = frame_err = 0
        for t in range(T):
            llr = awgn_llr(B, n, snr, seed=11, frame_offset=(si * T + t) * B, device=cuda)
            hard = dec.decode(llr, cidx, vidx).cpu().numpy()
            bit_err += int(hard.sum())
            frame_err += int((hard.sum(1) > 0).sum())
        assert ber[si] == bit_err / (T * B * n) and fer[si] == frame_err / (T * B)
    assert ber[0] > ber[-1]


def test_trainer_message_gnn(cuda):
    base, H, cidx, vidx, _ = _code(4)
    torch.manual_seed(0)
    dec, conv = create_message_gnn_decoder(H, num_iterations=2, hidden_dim=32, base_graph=base, Z=4)
    tr = LDPCDecoderTrainer(dec, device=cuda, converter=conv, message_types=conv.get_message_types(base, 4))
    before = {k: v.detach().clone() for k, v in dec.state_dict().items()}
    hist = tr.train(num_epochs=2, batch_size=16, learning_rate=0.01, check_index_tensor=None, var_index_tensor=None,
                    snr_range=[1, 3], validation_interval=1)
    assert len(hist["train_losses"]) == 2 and len(hist["val_losses"]) == 2
    changed = [k for k, v in dec.state_dict().items() if not torch.equal(v, before[k])]
    assert any(k.startswith("gnn_layers.1.") for k in changed)   # SGD stepped through the HIP backward
    ber, fer = tr.evaluate_snr_range([0, 4], 16, 2, None, None, H.shape[1])
    assert len(ber) == 2 and all(0 <= x <= 1 for x in ber + fer)


def test_comparative_evaluator_results_file(cuda, tmp_path):
    base, H, cidx, vidx, _ = _code(4)
    dec = _decoder(cidx.shape[0], 3, 2)
    ev = ComparativeEvaluator(H, neural_decoder=dec, device=cuda, seed=5)
    res = ev.evaluate_all([0, 3], batch_size=32, num_trials=2, check_index_tensor=cidx, var_index_tensor=vidx)
    assert set(res) == {"snr_range", "belief_propagation", "min_sum_scaled", "neural_decoder"}
    assert set(res["belief_propagation"]) == {"ber", "fer", "avg_iterations"}
    assert set(res["neural_decoder"]) == {"ber", "fer"}
    p = tmp_path / "comparison_results.pt"
    ev.save_results(str(p))
    loaded = torch.load(str(p), weights_only=True)   # what visualization/plot_comparison.py reads
    assert loaded == res
    ev2 = ComparativeEvaluator(H, device=cuda)
    ev2.load_results(str(p))
    ev2.print_summary()
    for f in (ev2.plot_ber_comparison, ev2.plot_fer_comparison, ev2.plot_iterations_comparison):
        f(save_path=str(tmp_path / "x.png"))
    # without index tensors (and no converter) the neural decoder is skipped, as :77
    assert "neural_decoder" not in ev.evaluate_all([0], batch_size=8, num_trials=1)


@pytest.mark.parametrize("model_type", ["standard", "message_gnn"])
def test_cli_train_evaluate_compare_visualize(cuda, tmp_path, model_type):
    from ldpc_neural_decoder import main as cli
    common = ["--base_matrix_path", code_path(4), "--lifting_factor", "4", "--num_iterations", "2",
              "--batch_size", "16", "--snr_min", "0", "--snr_max", "4", "--snr_step", "4", "--num_trials", "2",
              "--model_path", str(tmp_path / "m" / "model.pt"), "--results_dir", str(tmp_path / "r"),
              "--model_type", model_type, "--hidden_dim", "16", "--device", "cuda"]
    cli.main(["--mode", "train", "--num_epochs", "2"] + common)
    ck = torch.load(str(tmp_path / "m" / "model.pt"), weights_only=True)
    assert len(ck["train_losses"]) == 2
    res = cli.main(["--mode", "evaluate"] + common)
    ev = torch.load(str(tmp_path / "r" / "evaluation_results.pt"), weights_only=True)
    assert ev == res and ev["snr_range"] == [0, 4] and len(ev["ber_results"]) == 2
    cli.main(["--mode", "compare", "--compare_with_traditional"] + common)
    cmp_ = torch.load(str(tmp_path / "r" / "comparison_results.pt"), weights_only=True)
    assert "neural_decoder" in cmp_ and cmp_["snr_range"] == [0, 4]
    cli.main(["--mode", "visualize"] + common)
    for f in ("training_loss.png", "ber_vs_snr.png", "fer_vs_snr.png", "ber_comparison.png", "performance.png"):
        assert os.path.exists(tmp_path / "r" / f), f


def test_cli_default_example_code(cuda, tmp_path):
    """The reference CLI's default code is the 3x4 example H (main.py:93-98): E = 7 edges, a
    degree-1 variable, rows of unequal degree -- the smallest graph the layer kernels see."""
    from ldpc_neural_decoder import main as cli
    common = ["--num_iterations", "3", "--batch_size", "8", "--snr_min", "0", "--snr_max", "2", "--snr_step", "2",
              "--num_trials", "2", "--model_path", str(tmp_path / "model.pt"), "--results_dir", str(tmp_path / "r"),
              "--device", "cuda"]
    trainer = cli.main(["--mode", "train", "--num_epochs", "2"] + common)
    assert len(trainer.train_losses) == 2 and all(np.isfinite(trainer.train_losses))
    res = cli.main(["--mode", "evaluate"] + common)
    assert res["snr_range"] == [0, 2] and all(0 <= x <= 1 for x in res["ber_results"] + res["fer_results"])
    cmp_ = cli.main(["--mode", "compare", "--compare_with_traditional"] + common)
    assert set(cmp_) == {"snr_range", "belief_propagation", "min_sum_scaled", "neural_decoder"}


def _fixture_llr_fn(llrs, dev):
    """An llr_fn for run_sweep that replays the reference's own seeded channel LLRs
    (tests/golden/channel_z4.npz): trial t of SNR index si starts at frame (si*T + t)*B."""
    B = llrs.shape[1]

    def fn(b, n, snr, off):
        assert b == B and off % B == 0
        return torch.from_numpy(llrs[off // B]).to(dev)
    return fn


@pytest.mark.parametrize("algo,alpha,es", [("bp", None, 0), ("bp", None, 1), ("ms", 0.75, 0), ("ms", 0.75, 1),
                                           ("ms", 0.8, 0), ("ms", 0.8, 1)])
def test_sweep_matches_reference_ber_fer(cuda, algo, alpha, es):
    """run_sweep + rates (the on-device harness) on the reference's fixture LLRs reproduce the
    per-SNR BER/FER that the reference's compute_ber_fer returned (make_golden.py:110-112) and its
    decode() iteration counts as avg_iterations (comparative_evaluation.py:146-159).  Min-sum is
    exact (the reference's float32 mean of a 0/1 tensor of 13 312 bits is the count / 13 312 to
    float32 rounding); BP within the BP bar (<= 0.1 % of bits; measured 0)."""
    from golden_util import trad_key
    from ldpc_neural_decoder.models import BeliefPropagationDecoder, MinSumScaledDecoder
    from ldpc_neural_decoder.sweep import rates, run_sweep
    from conftest import golden
    ch, fx = golden("channel_z4.npz"), golden("trad_z4.npz")
    base, H, *_ = _code(4)
    key = trad_key(algo, alpha, es)
    llrs, snrs = ch["llrs"], ch["snrs"].tolist()
    B, n = llrs.shape[1:]
    dec = (BeliefPropagationDecoder(H, 5, early_stopping=bool(es)) if algo == "bp"
           else MinSumScaledDecoder(H, 5, alpha, early_stopping=bool(es)))
    counts = run_sweep(lambda llr, c: dec.decode(llr, out_dtype=torch.uint8, counters=c),
                       _fixture_llr_fn(llrs, cuda), snrs, B, 1, n, device=cuda)
    ber, fer, avg_it = rates(counts, n)
    ref = fx[key + "_ber_fer"]
    assert avg_it == [float(i) for i in fx[key + "_iters"]]
    bit_err = counts[:, 0].cpu().numpy()
    ref_err = np.rint(ref[:, 0] * B * n)
    if algo == "ms":
        assert np.array_equal(bit_err, ref_err)
        np.testing.assert_allclose(ber, ref[:, 0], rtol=1e-6, atol=0)
        np.testing.assert_allclose(fer, ref[:, 1], rtol=0, atol=1e-7)
    else:
        assert np.all(np.abs(bit_err - ref_err) <= 1e-3 * B * n)
        np.testing.assert_allclose(fer, ref[:, 1], atol=2 / B)


def test_comparative_evaluator_vs_reference_fixtures(cuda):
    """ComparativeEvaluator.evaluate_all end to end (comparative_evaluation.py:40-166) with its
    channel replaced by the reference's fixture LLRs and the fixtures' 5 iterations: the results
    dict holds the reference's BER/FER and avg_iterations for both classic decoders."""
    from conftest import golden
    ch, fx = golden("channel_z4.npz"), golden("trad_z4.npz")
    base, H, *_ = _code(4)
    ev = ComparativeEvaluator(H, device=cuda)
    ev.bp_decoder.max_iterations = ev.ms_decoder.max_iterations = 5
    ev._llr_fn = lambda: _fixture_llr_fn(ch["llrs"], cuda)
    snrs = ch["snrs"].tolist()
    res = ev.evaluate_all(snrs, batch_size=ch["llrs"].shape[1], num_trials=1)
    for name, key in (("belief_propagation", "bp_es1"), ("min_sum_scaled", "ms_a0.75_es1")):
        bp = name == "belief_propagation"  # BP: within the BP bar; min-sum: exact counts
        assert res[name]["avg_iterations"] == [float(i) for i in fx[key + "_iters"]]
        np.testing.assert_allclose(res[name]["ber"], fx[key + "_ber_fer"][:, 0], rtol=1e-6, atol=1e-3 if bp else 0)
        np.testing.assert_allclose(res[name]["fer"], fx[key + "_ber_fer"][:, 1], atol=2 / 64 if bp else 1e-7)


def test_trainer_keeps_data_on_its_device(cuda):
    """Bits, LLRs and counters are made on trainer.device (not the current device), so the HIP
    backward's gradients land next to the parameters.  With one GPU the explicit
    device is also the current one; with several the trainer is put on the last one."""
    base, H, cidx, vidx, _ = _code(4)
    dev = torch.device("cuda", torch.cuda.device_count() - 1)
    torch.manual_seed(0)
    dec, conv = create_message_gnn_decoder(H, num_iterations=2, hidden_dim=16, base_graph=base, Z=4)
    tr = LDPCDecoderTrainer(dec, device=dev, converter=conv, message_types=conv.get_message_types(base, 4))
    bits = tr._random_bits(8, H.shape[1])
    assert bits.device == dev and tr._channel(bits, 2.0).device == dev
    assert all(p.device == dev for p in dec.parameters())
    with torch.cuda.device(0):
        hist = tr.train(num_epochs=1, batch_size=8, learning_rate=0.01, check_index_tensor=None,
                        var_index_tensor=None, snr_range=[2], validation_interval=1)
    assert len(hist["train_losses"]) == 1 and all(p.grad is None or p.grad.device == dev for p in dec.parameters())
