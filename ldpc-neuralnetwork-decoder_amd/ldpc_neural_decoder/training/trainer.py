"""Trainer (drop-in for the reference's training/trainer.py:21-364).

Same class, methods, arguments, defaults and on-disk checkpoint dict as the reference:
  * ``train`` (TR:45-140): SGD(lr, momentum=0.9, weight_decay=1e-4) (TR:70), one batch of random
    bits per SNR per epoch, ``loss.mean().backward()``, validation every ``validation_interval``
    epochs, history dict {'train_losses', 'val_losses', 'ber_history', 'fer_history'};
  * ``validate`` (TR:142-203): mean over SNRs of (loss, BER, FER) with soft > 0.5 decisions;
  * ``evaluate_snr_range`` (TR:205-262): all-zero codeword, ``num_trials`` batches per SNR,
    ``decoder.decode`` -> (ber list, fer list);
  * ``save_model`` / ``load_model`` (TR:337-364): {'model_state_dict', 'train_losses',
    'val_losses', 'ber_history', 'fer_history'}; loads with ``weights_only=True``.

What runs where: the channel is the fused on-device kernel (utils.channel.awgn_llr: QPSK + AWGN
+ LLR from a Philox stream keyed by (seed, frame index), the same LLR law as TR:80-88's
qpsk_modulate -> awgn_channel -> qpsk_demodulate), error counting is the integer counter kernel,
and the decoder's forward/backward are the HIP kernels behind its autograd Functions.  Losses
and counters stay on the device inside an epoch / SNR point; the host syncs once per epoch
(the reference calls .item() per batch).

Decoders: anything with the reference protocol ``decoder(llrs, check_index_tensor,
var_index_tensor, bits) -> (soft, loss)`` and ``decoder.decode(llrs, check_index_tensor,
var_index_tensor)`` (models.decoder.LDPCNeuralDecoder), or a MessageGNNDecoder together with
its TannerToMessageGraph ``converter`` (then the index-tensor arguments are unused and may be
None; the loss is the decoder's BCE, message_gnn_decoder.py:313-315).
"""
import functools

import torch

from ldpc_neural_decoder import _native as N
from ldpc_neural_decoder.sweep import rates, run_sweep, _dist_all_reduce
from ldpc_neural_decoder.utils.channel import awgn_llr, count_errors

HISTORY_KEYS = ("train_losses", "val_losses", "ber_history", "fer_history")


def _on_device(fn):
    """Run a trainer method with self.device as the current HIP device, so every tensor it makes
    (bits, LLRs, counters, losses) lands where the decoder's parameters are."""
    @functools.wraps(fn)
    def wrapper(self, *args, **kwargs):
        with torch.cuda.device(self.device):
            return fn(self, *args, **kwargs)
    return wrapper


class LDPCDecoderTrainer:
    def __init__(self, decoder, device=None, converter=None, message_types=None, seed=0):
        self.decoder = decoder
        # the decoders compute on the HIP device only: a CPU `device` (the reference's default
        # without CUDA) selects the current HIP device rather than a CPU path
        dev = torch.device(device) if device is not None else None
        self.device = dev if dev is not None and dev.type == "cuda" else N.device_of(None)
        self.decoder.to(self.device)
        self.converter = converter
        self.message_types = message_types
        self.seed = seed
        self._frames = 0  # Philox frame counter: every generated frame gets fresh noise
        self.train_losses = []
        self.val_losses = []
        self.ber_history = []
        self.fer_history = []

    # ------------------------------------------------------------------ decoder protocol
    def _gnn_args(self):
        conv = self.converter
        types = self.message_types if self.message_types is not None else conv.get_message_types()
        return (conv.message_to_var_index(), types, conv.var_to_check_adjacency, conv.check_to_var_adjacency)

    def _forward(self, llrs, check_index_tensor, var_index_tensor, bits):
        if self.converter is not None:
            return self.decoder(llrs, *self._gnn_args(), ground_truth=bits)
        return self.decoder(llrs, check_index_tensor, var_index_tensor, bits)

    def _decode(self, llrs, check_index_tensor, var_index_tensor):
        if self.converter is not None:
            return self.decoder.decode(llrs, *self._gnn_args())
        return self.decoder.decode(llrs, check_index_tensor, var_index_tensor)

    def _channel(self, bits, snr_db):
        """Random (or given) bits -> LLRs on the compute device; advances the frame counter."""
        B, n = bits.shape
        llrs = awgn_llr(B, n, snr_db, seed=self.seed, frame_offset=self._frames, bits=bits,
                        device=self.device)
        self._frames += B
        return llrs

    def _bits_per_frame(self, variable_bit_length):
        if variable_bit_length is not None:
            return int(variable_bit_length)
        if self.converter is not None:
            return self.converter.num_variables
        raise ValueError("variable_bit_length is required")

    def _random_bits(self, batch_size, n):
        return torch.randint(0, 2, (batch_size, n), device=self.device).float()

    @staticmethod
    def _to(t, dev):
        return None if t is None else torch.as_tensor(t).to(dev)

    # ------------------------------------------------------------------ reference API
    @_on_device
    def train(self, num_epochs, batch_size, learning_rate, check_index_tensor, var_index_tensor,
              snr_range=None, variable_bit_length=None, validation_interval=5, momentum=0.9, weight_decay=0.0001):
        """TR:45-140."""
        check_index_tensor = self._to(check_index_tensor, self.device)
        var_index_tensor = self._to(var_index_tensor, self.device)
        optimizer = torch.optim.SGD(self.decoder.parameters(), lr=learning_rate, momentum=momentum,
                                    weight_decay=weight_decay)
        if snr_range is None:
            snr_range = [-2, 0, 2, 4]
        variable_bit_length = self._bits_per_frame(variable_bit_length)
        for epoch in range(num_epochs):
            self.decoder.train()
            epoch_loss = torch.zeros((), dtype=torch.float64, device=self.device)
            num_batches = 0
            for snr_db in snr_range:
                bits = self._random_bits(batch_size, variable_bit_length)
                llrs = self._channel(bits, snr_db)
                optimizer.zero_grad()
                _, loss = self._forward(llrs, check_index_tensor, var_index_tensor, bits)
                batch_loss = loss.mean()
                batch_loss.backward()
                optimizer.step()
                epoch_loss += batch_loss.detach().to(epoch_loss.device, torch.float64)
                num_batches += 1
            avg_epoch_loss = float(epoch_loss) / max(num_batches, 1)
            self.train_losses.append(avg_epoch_loss)
            print(f"Epoch {epoch+1}/{num_epochs} - Loss: {avg_epoch_loss:.6f}")
            if (epoch + 1) % validation_interval == 0:
                val_loss, ber, fer = self.validate(batch_size, check_index_tensor, var_index_tensor,
                                                   snr_range, variable_bit_length)
                self.val_losses.append(val_loss)
                self.ber_history.append(ber)
                self.fer_history.append(fer)
                print(f"Validation - Loss: {val_loss:.6f}, BER: {ber:.6f}, FER: {fer:.6f}")
        return {k: getattr(self, k) for k in HISTORY_KEYS}

    @_on_device
    def validate(self, batch_size, check_index_tensor, var_index_tensor, snr_range, variable_bit_length):
        """TR:142-203 -> (avg_loss, avg_ber, avg_fer), averaged over the SNR points."""
        self.decoder.eval()
        variable_bit_length = self._bits_per_frame(variable_bit_length)
        dev = self.device
        total_loss = torch.zeros((), dtype=torch.float64, device=dev)
        per_snr = torch.zeros((len(snr_range), 4), dtype=torch.int64, device=dev)
        with torch.no_grad():
            for i, snr_db in enumerate(snr_range):
                bits = self._random_bits(batch_size, variable_bit_length)
                llrs = self._channel(bits, snr_db)
                soft, loss = self._forward(llrs, check_index_tensor, var_index_tensor, bits)
                total_loss += loss.mean().to(dev, torch.float64)
                count_errors((soft.to(dev) > 0.5).to(torch.uint8), ref=bits, counters=per_snr[i])
        n = max(len(snr_range), 1)
        ber, fer, _ = rates(per_snr, variable_bit_length)
        return float(total_loss) / n, sum(ber) / n, sum(fer) / n

    @_on_device
    def evaluate_snr_range(self, snr_range, batch_size, num_trials, check_index_tensor, var_index_tensor,
                           variable_bit_length):
        """TR:205-262 -> (ber_results, fer_results).  With torch.distributed initialised the
        trials are dealt to ranks and the counters summed once (sweep.run_sweep)."""
        self.decoder.eval()
        variable_bit_length = self._bits_per_frame(variable_bit_length)
        check_index_tensor = self._to(check_index_tensor, self.device)
        var_index_tensor = self._to(var_index_tensor, self.device)
        dev = self.device
        ar, rank, world = _dist_all_reduce()
        base = self._frames

        def llr_fn(b, n, snr, off):
            return awgn_llr(b, n, snr, seed=self.seed, frame_offset=base + off, device=dev)

        def decode(llrs, counters):
            with torch.no_grad():
                hard = self._decode(llrs, check_index_tensor, var_index_tensor)
            count_errors(hard.to(dev), counters=counters)

        counts = run_sweep(decode, llr_fn, snr_range, batch_size, num_trials, variable_bit_length, rank, world,
                           dev, ar)
        self._frames += len(snr_range) * num_trials * batch_size
        ber, fer, _ = rates(counts, variable_bit_length)
        return ber, fer

    def plot_training_history(self):
        """TR:264-297 (matplotlib; presentation only)."""
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        fig1, ax = plt.subplots(figsize=(10, 6))
        ax.plot(self.train_losses, label="Training Loss")
        if self.val_losses:
            step = max(len(self.train_losses) // len(self.val_losses), 1)
            ax.plot(list(range(0, len(self.train_losses), step))[:len(self.val_losses)], self.val_losses, "o-",
                    label="Validation Loss")
        ax.set_xlabel("Epoch")
        ax.set_ylabel("Loss")
        ax.legend()
        fig2 = None
        if self.ber_history:
            fig2, ax2 = plt.subplots(figsize=(10, 6))
            ax2.semilogy(self.ber_history, label="BER")
            ax2.semilogy(self.fer_history, label="FER")
            ax2.legend()
        return fig1, fig2

    def plot_snr_performance(self, snr_range, ber_results, fer_results, comparison_ber=None, comparison_fer=None):
        """TR:299-335 (matplotlib; presentation only)."""
        import matplotlib
        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
        figs = []
        for ys, cmp, name in ((ber_results, comparison_ber, "BER"), (fer_results, comparison_fer, "FER")):
            fig, ax = plt.subplots(figsize=(10, 6))
            ax.semilogy(snr_range, ys, "o-", label="Neural Decoder")
            if cmp is not None:
                ax.semilogy(snr_range, cmp, "s-", label="Conventional Decoder")
            ax.set_xlabel("SNR (dB)")
            ax.set_ylabel(name)
            ax.legend()
            figs.append(fig)
        return tuple(figs)

    def save_model(self, path):
        """TR:337-350."""
        torch.save({"model_state_dict": self.decoder.state_dict(),
                    **{k: list(getattr(self, k)) for k in HISTORY_KEYS}}, path)

    def load_model(self, path):
        """TR:352-364 (missing history keys default to empty lists)."""
        checkpoint = torch.load(path, map_location=self.device, weights_only=True)
        self.decoder.load_state_dict(checkpoint["model_state_dict"])
        for k in HISTORY_KEYS:
            setattr(self, k, list(checkpoint.get(k, [])))
