"""On-device SNR sweep: the reference's evaluation harness with nothing leaving the GPU.

Replaces the per-(SNR, trial) Python loops of
  ComparativeEvaluator._evaluate_traditional_decoder  training/comparative_evaluation.py:108-166
  ComparativeEvaluator.evaluate_all                   training/comparative_evaluation.py:40-106
  evaluate_message_gnn                                run_comparison_all.py:245-295
with: fused channel kernel (all-zero codeword -> QPSK -> AWGN -> LLR, Philox keyed by the global
frame index) -> decoder -> fused integer BER/FER counters.  The only host sync is at the end.

Semantics kept from the reference:
  * every trial transmits the all-zero codeword (:133) in a batch of `batch_size` frames;
  * BER/FER per SNR = mean over trials of the per-trial means (equal batch sizes, so it is the
    global mean of the integer counts);
  * avg_iterations = mean over trials of the decoder's returned iteration count (batch-global
    early stop: every frame of a trial reports the trial's count);
  * results dict keyed as comparative_evaluation.py:86-104.

Multi-GPU: trials are dealt round-robin to ranks (trial t -> rank t % world) so the batch-global
early-stop rule still sees whole trials; the only collective is one SUM all-reduce of the
(n_snr, 4) int64 counter matrix at the end (RCCL over xGMI, or gloo in the CPU tests).
"""
import torch

COUNTER_FIELDS = ("bit_errors", "frame_errors", "frames", "iteration_sum")


def run_sweep(decode_fn, llr_fn, snr_range, batch_size, num_trials, n, rank=0, world=1,
              device="cpu", all_reduce=None):
    """Generic sharded sweep.

    llr_fn(batch, n, snr_db, frame_offset) -> (batch, n) float32 LLRs on `device`
    decode_fn(llr, counters) -> None; adds [bit errs, frame errs, frames, iteration sum] into
        the int64[4] `counters` (the flood decoders do it inside the kernel epilogue)
    all_reduce(tensor) -> sums a tensor over ranks in place (None for a single process)
    Returns the (len(snr_range), 4) int64 counter matrix (summed over ranks).
    """
    counts = torch.zeros((len(snr_range), 4), dtype=torch.int64, device=device)
    for si, snr in enumerate(snr_range):
        for t in range(rank, num_trials, world):
            offset = (si * num_trials + t) * batch_size  # global frame index of the trial
            llr = llr_fn(batch_size, n, snr, offset)
            decode_fn(llr, counts[si])
    if all_reduce is not None:
        all_reduce(counts)
    return counts


def rates(counts, n):
    """Counter matrix -> (ber list, fer list, avg_iterations list)."""
    c = counts.double().cpu()
    frames = c[:, 2].clamp(min=1)
    ber = (c[:, 0] / (frames * n)).tolist()
    fer = (c[:, 1] / frames).tolist()
    avg_it = (c[:, 3] / frames).tolist()
    return ber, fer, avg_it


def _dist_all_reduce():
    """(all_reduce fn, rank, world) of the initialised process group.  RCCL ("nccl") reduces the
    device tensor in place over xGMI; gloo (CPU tests, multi-rank rehearsals sharing one card)
    reduces a host copy.  Any initialised group reduces, a world of one included (BENCH_DIST=1 runs
    the RCCL branch on one GPU)."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        if dist.get_backend() == "gloo":
            def ar(t):
                h = t.cpu()
                dist.all_reduce(h, op=dist.ReduceOp.SUM)
                t.copy_(h)
        else:
            def ar(t):
                dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return ar, dist.get_rank(), dist.get_world_size()
    return None, 0, 1


class ComparativeEvaluator:
    """comparative_evaluation.py:10-106,335-390 on the GPU (BP and min-sum: 50 iterations,
    batch-global early stop, alpha 0.75, as :34-35).  ``neural_decoder`` is either a decoder of
    the reference protocol (``decode(llrs, check_index_tensor, var_index_tensor)``, evaluated when
    evaluate_all gets both index tensors, as :77) or a MessageGNNDecoder with its
    TannerToMessageGraph passed as ``converter``.  ``device`` is where results and decoders live;
    the compute always runs on the HIP device (a CPU ``device`` selects the current one)."""

    def __init__(self, H, neural_decoder=None, device=None, converter=None, seed=0, message_types=None):
        from ldpc_neural_decoder import _native as N
        from ldpc_neural_decoder.models import BeliefPropagationDecoder, MinSumScaledDecoder
        self.device = N.device_of(None) if device is None else torch.device(device)
        self._dev = self.device if self.device.type == "cuda" else N.device_of(None)
        self.H = H
        self.neural_decoder = neural_decoder
        if neural_decoder is not None:
            neural_decoder.to(self._dev)
            neural_decoder.eval()
        self.converter = converter
        self.message_types = message_types
        self.seed = seed
        self.bp_decoder = BeliefPropagationDecoder(H, max_iterations=50, early_stopping=True)
        self.ms_decoder = MinSumScaledDecoder(H, max_iterations=50, scaling_factor=0.75, early_stopping=True)
        self.results = {}

    def _llr_fn(self):
        from ldpc_neural_decoder.utils.channel import awgn_llr
        dev, seed = self._dev, self.seed
        return lambda b, n, snr, off: awgn_llr(b, n, snr, seed=seed, frame_offset=off, device=dev)

    def _flood(self, dec, snr_range, batch_size, num_trials):
        ar, rank, world = _dist_all_reduce()
        n = self.H.shape[1]

        def decode(llr, counters):
            dec.decode_async(llr, out_dtype=torch.uint8, counters=counters)

        counts = run_sweep(decode, self._llr_fn(), snr_range, batch_size, num_trials, n, rank, world,
                           self._dev, ar)
        return rates(counts, n)

    def _evaluate_traditional_decoder(self, decoder, snr_range, batch_size, num_trials, variable_bit_length=None):
        return self._flood(decoder, snr_range, batch_size, num_trials)

    def _evaluate_neural_decoder(self, snr_range, batch_size, num_trials, variable_bit_length=None,
                                 check_index_tensor=None, var_index_tensor=None):
        """:168-223 -> (ber list, fer list)."""
        if self.converter is not None:
            return evaluate_message_gnn(self.neural_decoder, self.converter, snr_range, batch_size,
                                        num_trials, self._dev, seed=self.seed, message_types=self.message_types)
        from ldpc_neural_decoder.utils.channel import count_errors
        ar, rank, world = _dist_all_reduce()
        n = self.H.shape[1] if variable_bit_length is None else variable_bit_length
        cidx, vidx = check_index_tensor.to(self._dev), var_index_tensor.to(self._dev)
        dec = self.neural_decoder

        def decode(llr, counters):
            with torch.no_grad():
                count_errors(dec.decode(llr, cidx, vidx).to(self._dev), counters=counters)

        counts = run_sweep(decode, self._llr_fn(), snr_range, batch_size, num_trials, n, rank, world,
                           self._dev, ar)
        ber, fer, _ = rates(counts, n)
        return ber, fer

    def evaluate_all(self, snr_range, batch_size=32, num_trials=100, variable_bit_length=None,
                     check_index_tensor=None, var_index_tensor=None):
        """:40-106.  The results dict holds plain Python lists (loadable with weights_only=True)."""
        snr_range = list(snr_range)
        bp = self._flood(self.bp_decoder, snr_range, batch_size, num_trials)
        ms = self._flood(self.ms_decoder, snr_range, batch_size, num_trials)
        self.results = {
            "snr_range": snr_range,
            "belief_propagation": {"ber": bp[0], "fer": bp[1], "avg_iterations": bp[2]},
            "min_sum_scaled": {"ber": ms[0], "fer": ms[1], "avg_iterations": ms[2]},
        }
        if self.neural_decoder is not None and (
                self.converter is not None or (check_index_tensor is not None and var_index_tensor is not None)):
            ber, fer = self._evaluate_neural_decoder(snr_range, batch_size, num_trials, variable_bit_length,
                                                     check_index_tensor, var_index_tensor)
            self.results["neural_decoder"] = {"ber": ber, "fer": fer}
        return self.results

    def _plot(self, field, ylabel, save_path, log=True):
        """:225-333 (presentation only): one curve per decoder that has `field`."""
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        fig, ax = plt.subplots(figsize=(10, 6))
        snr = self.results["snr_range"]
        for key, label, style in (("belief_propagation", "Belief Propagation", "o-"),
                                  ("min_sum_scaled", "Min-Sum Scaled", "s-"), ("neural_decoder", "Neural Decoder", "^-")):
            if field in self.results.get(key, {}):
                (ax.semilogy if log else ax.plot)(snr, self.results[key][field], style, label=label)
        ax.set_xlabel("SNR (dB)")
        ax.set_ylabel(ylabel)
        ax.grid(True)
        ax.legend()
        if save_path:
            fig.savefig(save_path)
            plt.close(fig)  # saved: do not keep it in pyplot's figure list
        return fig

    def plot_ber_comparison(self, save_path=None):
        return self._plot("ber", "Bit Error Rate (BER)", save_path)

    def plot_fer_comparison(self, save_path=None):
        return self._plot("fer", "Frame Error Rate (FER)", save_path)

    def plot_iterations_comparison(self, save_path=None):
        return self._plot("avg_iterations", "Average Iterations", save_path, log=False)

    def save_results(self, path):
        """:335-345."""
        if not self.results:
            raise ValueError("No results to save. Run evaluate_all() first.")
        torch.save(self.results, path)

    def load_results(self, path):
        """:347-354 (weights_only: the file holds lists and floats)."""
        self.results = torch.load(path, weights_only=True)

    def print_summary(self):
        """:356-390."""
        if not self.results:
            raise ValueError("No results to summarize. Run evaluate_all() first.")
        print("Evaluation Summary")
        print("=================")
        print(f"SNR Range: {self.results['snr_range']}")
        print()
        for key, title in (("belief_propagation", "Belief Propagation Decoder"),
                           ("min_sum_scaled", "Min-Sum Scaled Decoder"), ("neural_decoder", "Neural Decoder")):
            if key not in self.results:
                continue
            r = self.results[key]
            print(title)
            print("-" * len(title))
            print(f"BER: {r['ber']}")
            print(f"FER: {r['fer']}")
            if "avg_iterations" in r:
                print(f"Average Iterations: {r['avg_iterations']}")
            print()


def evaluate_message_gnn(decoder, converter, snr_range, batch_size, num_trials, device=None, seed=0,
                         message_types=None):
    """run_comparison_all.py:245-295 on the GPU -> (ber list, fer list).  message_types=None uses
    converter.get_message_types() (all zero) as :273 does."""
    from ldpc_neural_decoder import _native as N
    from ldpc_neural_decoder.utils.channel import awgn_llr, count_errors
    dev = N.device_of(None) if device is None else torch.device(device)
    decoder = decoder.to(dev)
    ar, rank, world = _dist_all_reduce()
    n = converter.num_variables
    io = converter.message_to_var_index().to(dev).to(torch.int32)
    T = decoder.gnn_layers[0].message_type_embeddings.shape[0]
    from ldpc_neural_decoder.models.message_gnn_decoder import _types_for
    types = _types_for(converter.get_message_types() if message_types is None else message_types,
                       len(converter.messages), T, dev)
    vg, cg = converter.var_groups, converter.check_groups

    def decode(llr, counters):
        probs = decoder.native_forward(llr, io, types, vg, cg)
        count_errors((probs > 0.5).to(torch.uint8), counters=counters)

    def llr_fn(b, nn_, snr, off):
        return awgn_llr(b, nn_, snr, seed=seed, frame_offset=off, device=dev)

    counts = run_sweep(decode, llr_fn, snr_range, batch_size, num_trials, n, rank, world, dev, ar)
    ber, fer, _ = rates(counts, n)
    return ber, fer
