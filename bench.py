#!/usr/bin/env python3
"""Benchmark of the decoding hot path (contract: see README / DESIGN.md "Measurement").

    python bench.py [--gpus N] [--steps K] [--warmup W] [--workload minsum-z32|...]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

`--gpus N` without a launcher starts the N ranks itself (torch.distributed.run, before anything
touches the GPU); under a launcher it must equal WORLD_SIZE, and with RCCL every rank needs its own
GPU -- otherwise the run exits 2 instead of timing fewer GPUs than it reports
(BENCH_DIST_BACKEND=gloo: the rehearsal with ranks sharing a card).

One step = one decode pass over this rank's batch of synthetic frames that are already resident
in HBM (all-zero codeword through the on-device QPSK/AWGN channel at a fixed SNR).  Frames shard
across ranks (weak scaling, no collective on the data path); the BER/FER counters and the timing
are reduced over ranks once at the end.  Rank 0 prints ONE JSON line.

Workloads (BASELINE.json configs):
  minsum-z32  cfg3 (default): BG2 Z=32, scaled min-sum alpha 0.75, 10 iterations, B=65536/GPU
  minsum-z32-stream  cfg3 on the streaming kernels (messages in HBM; the path of graphs that do
              not fit LDS), for the HBM roofline of SURVEY 8(d)'s byte model
  minsum-z384 BG2 lifted to Z=384 (5G's largest; the NR_2_0_32 shifts taken mod 384), streaming
  bp-z4       cfg1 sizes on the GPU: BG2 Z=4, BP, 5 iterations, B=64 (x --batch)
  gnn-z4      cfg2: BG2 Z=4, MessageGNN 5 layers, H=64, T=4, B=4096, fp32
  gnn-z32     cfg4 per GPU: BG2 Z=32, MessageGNN 10 layers, H=64, T=32, B=32768/GPU, fp32
  gnn-z32-bf16 cfg5 per GPU: same code, 15 layers, bf16 features + bf16 MFMA (fp32 accumulate),
              per-frame early-termination syndrome check after every layer (avg_layers reported)
  gnn-z32-bf16-i10  cfg4 shape (10 layers) on the bf16 path: the north-star "10 iterations" GNN line
  gnn-z32-h128  cfg4's code and depth at hidden_dim 128 (the reference builds any width, MGD:22/:162):
              gnn_wide.hip (group means, projections, the fused per-tile MLP), fp32, random weights
  gnn-z32-h192  the same at hidden_dim 192 (the fused MLP at one wave per SIMD)
  gnn-z32-sweep  cfg4 as BASELINE states it: the on-device SNR sweep 0..6 dB step 1 (sweep.py
              evaluate_message_gnn = run_comparison_all.py:245-295), fp32, B frames per GPU per SNR;
              one step = one whole sweep (channel + decode + counters, RCCL all-reduce at the end)
  lay-z32     the index-gather layers (models/layers.py): 10 iterations of CheckLayer ->
              VariableLayer -> ResidualLayer(depth 2) + OutputLayer on the var-major edge vector
  gnn-train-z32 / gnn-train-z4  one training step (fp32 forward saving features, BCE, HIP backward,
                SGD with the trainer's momentum 0.9 / weight decay 1e-4), frames/s
  hybrid-minsum-z32  CustomMinSumMessageGNNDecoder as this build defines it (models/custom_decoders.py):
              damped, unscaled min-sum on the streaming kernels, soft output, 10 iterations
  hybrid-gnn-z32     CustomVariableMessageGNNDecoder as defined there: check-side MLP + damped
              min-sum variable update, 10 layers, fp32
"""
import argparse
import json
import os
import platform
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "ldpc-neuralnetwork-decoder_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

HBM_PEAK_GBS = 8000.0       # MI355X HBM3E, MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_GINST = 1024 * 2.4 / 2  # wave64 VALU instructions/s (1e9): 1024 SIMDs, 2.4 GHz, 2 cycles each
FP32_MFMA_PEAK_TFS = 157.3  # MI355X fp32 matrix (spec), same guide
BF16_MFMA_PEAK_TFS = 2500.0  # MI355X bf16 dense MFMA (spec, no sparsity)

HIDDEN = {"gnn-z32-h128": 128, "gnn-z32-h192": 192}  # hidden_dim of the GNN workloads (default 64)

WORKLOADS = {
    # name: (decoder, Z, iterations, default batch per GPU, SNR dB)
    "minsum-z32": ("minsum", 32, 10, 65536, 2.0),
    "minsum-z32-stream": ("minsum", 32, 10, 65536, 2.0),
    "minsum-z384": ("minsum", 384, 10, 8192, 2.0),
    "bp-z4": ("bp", 4, 5, 64, 2.0),
    "bp-z32": ("bp", 32, 10, 65536, 2.0),
    "gnn-z4": ("gnn", 4, 5, 4096, 2.0),
    "gnn-z32": ("gnn", 32, 10, 32768, 2.0),
    "gnn-z32-h128": ("gnn", 32, 10, 8192, 2.0),
    "gnn-z32-h192": ("gnn", 32, 10, 8192, 2.0),
    "gnn-z32-bf16": ("gnn-bf16", 32, 15, 32768, 2.0),
    "gnn-z4-bf16": ("gnn-bf16", 4, 5, 4096, 2.0),
    "gnn-z32-bf16-i10": ("gnn-bf16", 32, 10, 32768, 2.0),
    "gnn-z32-sweep": ("gnn-sweep", 32, 10, 32768, None),
    "gnn-train-z32": ("gnn-train", 32, 10, 256, 2.0),
    "lay-z32": ("lay", 32, 10, 4096, 2.0),
    "gnn-train-z4": ("gnn-train", 4, 5, 4096, 2.0),
    "hybrid-minsum-z32": ("hybrid-minsum", 32, 10, 65536, 2.0),
    "hybrid-gnn-z32": ("hybrid-gnn", 32, 10, 32768, 2.0),
}


def flood_bytes_per_cw(E, N, iters):
    """every edge message read + written once per iteration (fp32), every APP read
    + written once per iteration, the LLR read once (4N) and the decision written once (N)."""
    return iters * 8 * (E + N) + 5 * N


def valu_roofline(B, n, kern_ms, traffic, pmc, pmc_path, alg_bytes):
    """The flood decoders keep every message in LDS: HBM sees the LLRs once and the decisions once,
    so SURVEY 8(d)'s streaming byte model is not their bound.  Their bound is VALU issue: the
    reference's exact float32 operation order (ascending, exclusive variable sums) is a fixed
    instruction stream per frame-iteration.  achieved = VALU wave64 instructions per launch (PMC
    SQ_INSTS_VALU of the same workload, scaled to this batch) / the live kernel time; peak = 1024
    SIMDs x 2.4 GHz / 2 cycles per wave64 VALU instruction (MI355X_MICROARCH.md: a SIMD issues a
    wave64 VALU instruction over 2 cycles)."""
    c = (pmc or {}).get("counters_per_launch", {})
    scale = B / pmc["batch"] if pmc and pmc.get("batch") else 1.0
    insts = c.get("SQ_INSTS_VALU")
    achieved = insts * scale / (kern_ms * 1e-3) / 1e9 if insts else None
    comp = 5 * n * B  # LLR read (4N) + uint8 decision written (N)
    notes = {
        "pmc_source": os.path.relpath(pmc_path, ROOT) if pmc_path else None,
        "valu_insts_per_launch": insts * scale if insts else None,
        "survey_streaming_bytes_per_launch": alg_bytes,
        "survey_streaming_GBps": alg_bytes / (kern_ms * 1e-3) / 1e9,
        "compulsory_bytes_per_launch": comp,
        "compulsory_frac_of_hbm_peak": comp / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
        "traffic_over_compulsory": (traffic / comp) if traffic else None,
    }
    notes.update((pmc or {}).get("derived", {}))
    return achieved, notes


# mangled-name prefix of the kernel a workload's PMC summary counts (flood_fixed_kernel<G, ALGO, ES>)
PMC_KERNEL_SYMBOL = {
    "minsum-z32": "_ZN4ldpc18flood_fixed_kernelINS_5fixed7BG2_Z32ELi0ELi0E",
    "bp-z32": "_ZN4ldpc18flood_fixed_kernelINS_5fixed7BG2_Z32ELi1ELi0E",
    "bp-z4": "_ZN4ldpc18flood_fixed_kernelINS_5fixed6BG2_Z4ELi1ELi0E",
    # the dominant kernel's translation unit (its PMC summary also sums the small gnn.hip output pass)
    "gnn-z32-bf16": "gnn_bf16_mlp_kernel",
    "gnn-z32-bf16-i10": "gnn_bf16_mlp_kernel",
    "gnn-z32-h128": "gnn_wide",
    "gnn-z32-h192": "gnn_wide",
    "lay-z32": "check_group",
    # the fp32 GNN's dominant kernels (projection + split MLP) share gnn.hip's code object
    "gnn-z32": "gnn_mlp2s_kernel",
    "gnn-z4": "gnn_mlp2s_kernel",
}


def sha256_file(path):
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", default="minsum-z32", choices=sorted(WORKLOADS))
    ap.add_argument("--batch", type=int, default=0, help="frames per GPU (0 = workload default)")
    ap.add_argument("--snr", type=float, default=None)
    ap.add_argument("--iterations", type=int, default=0, help="override the workload's iteration count")
    ap.add_argument("--early-termination", choices=("auto", "on", "off"), default="auto",
                    help="bf16 GNN per-frame early termination (auto: on for gnn-z32-bf16 = cfg5 only)")
    ap.add_argument("--early-stop", choices=("off", "batch", "frame"), default="off",
                    help="min-sum / BP stopping rule: off (cfg3: every iteration), batch (the reference's "
                         "batch-global rule, traditional_decoders.py:104-107), frame (per-frame freeze)")
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0,
                    help="target CPU work for the oracle baseline sample (0 disables)")
    ap.add_argument("--data", choices=("auto", "zero", "codewords"), default="auto",
                    help="transmitted frames: the all-zero codeword (every reference harness, e.g. "
                         "comparative_evaluation.py:133) or random codewords (utils/encoding.py), whose BER / "
                         "FER show a neural decoder's decoding on typical frames.  auto: codewords when the "
                         "bf16 GNN's early termination is on (the all-zero frame stops early by construction: "
                         "the checkpoint saw it in every batch), the all-zero codeword otherwise")
    ap.add_argument("--checkpoint", default=None,
                    help="MessageGNN weights (a trainer checkpoint dict, loaded weights_only); default: "
                         "checkpoints/gnn_bg2_z<Z>_i<layers>_h64.pt when present, else random weights")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC traffic summary (profiles/*_pmc.json) to report as roofline.traffic")
    return ap.parse_args()


def resolve_launch(gpus, env, device_count):
    """What `bench.py --gpus N` does, before anything touches the GPU:
      ("run", None)    this process is the job (N = 1), or one rank of a launcher's job
                       (WORLD_SIZE set, equal to N);
      ("spawn", None)  N > 1 and no launcher: start N ranks under torch.distributed.run and exit with
                       their status (the parent never initialises HIP);
      ("error", msg)   a run that would misreport: --gpus differs from the launcher's WORLD_SIZE, or
                       fewer GPUs are visible than ranks with RCCL.  BENCH_DIST_BACKEND=gloo is the
                       explicit rehearsal of the multi-rank path with ranks sharing fewer cards."""
    gloo = env.get("BENCH_DIST_BACKEND", "nccl") == "gloo"
    world = env.get("WORLD_SIZE")
    if gpus < 1:
        return "error", f"--gpus {gpus}: need at least one"
    if world is None:
        if gpus == 1:
            return "run", None
        if not gloo and device_count < gpus:
            return "error", f"--gpus {gpus} but {device_count} GPU(s) visible (RCCL needs one per rank)"
        return "spawn", None
    if int(world) != gpus:
        return "error", f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks"
    if not gloo and device_count < int(world):
        return "error", f"WORLD_SIZE={world} but {device_count} GPU(s) visible (RCCL needs one per rank)"
    return "run", None


def spawn_ranks(gpus, argv):
    """torch.distributed.run with one rank per GPU on this node, rendezvous on 127.0.0.1 at a free
    port; returns its exit status.  The ranks inherit stdout: rank 0's JSON line is this run's."""
    import socket
    import subprocess
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    env = dict(os.environ, BENCH_LAUNCH="self", MASTER_ADDR="127.0.0.1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    return subprocess.call(cmd, env=env)


def setup_dist():
    """One process per GPU.  A process group is created for more than one rank, or for one rank
    with BENCH_DIST=1 (the RCCL branch exercised on a single GPU: tests/test_dist_rccl_gpu.py)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or os.environ.get("BENCH_DIST") == "1":
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        # BENCH_DIST_BACKEND=gloo with more ranks than GPUs is a rehearsal of the multi-rank path
        # on a 1-GPU box (ranks share the card); the measured runs use RCCL ("nccl"), one GPU each
        backend = os.environ.get("BENCH_DIST_BACKEND", "nccl")
        dev_i = local % max(torch.cuda.device_count(), 1) if backend == "gloo" else local
        torch.cuda.set_device(dev_i)
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_i))
        else:
            dist.init_process_group(backend)
    else:
        torch.cuda.set_device(0)
    return world, rank, torch.device("cuda", torch.cuda.current_device())


def barrier(world):
    if dist.is_initialized():
        dist.barrier()


def cpu_baseline(workload, z, iters, target_s):
    """The CPU restatement of the same workload (oracle/: ldpc_oracle.c single-threaded for the
    flooding decoders, the reference's literal loop order; oracle.gnn_forward in torch fp32 on
    torch's CPU threads for the GNN) on a bounded sample of ~target_s seconds, on this host."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle
    kind, _, _, _, snr = WORKLOADS[workload]
    base = oracle.load_base(os.path.join(ROOT, "codes", f"NR_2_0_{z if z in (4, 32) else 32}.txt"))
    H = oracle.expand(base, z)
    g = oracle.Graph(H)
    rng = np.random.default_rng(0)
    s = 10 ** (snr / 10)
    cpu = platform.processor() or platform.machine()

    def sample(b):
        noise = rng.normal(0.0, np.sqrt(1 / (2 * s)), size=(b, g.N))
        return (2 * s * (1 / np.sqrt(2) + noise)).astype(np.float32)

    if kind.startswith("hybrid"):
        if kind == "hybrid-minsum":
            def run(b):
                oracle.custom_minsum(g, sample(b), iters)
            what = "oracle/ldpc_oracle.c custom_minsum, 1 thread"
        else:
            from ldpc_neural_decoder.models import create_custom_variable_message_gnn_decoder
            torch.manual_seed(7)
            dec, conv = create_custom_variable_message_gnn_decoder(torch.from_numpy(H), num_iterations=iters,
                                                                   hidden_dim=64, base_graph=torch.from_numpy(base),
                                                                   Z=z)
            sd = {k: v.detach() for k, v in dec.state_dict().items()}
            types = conv.get_message_types(torch.from_numpy(base), z)

            def run(b):
                with torch.no_grad():
                    oracle.custom_variable_forward(sd, torch.from_numpy(sample(b)), conv.edge_var, conv.edge_chk,
                                                   g.N, g.M, types)
            what = f"oracle.custom_variable_forward (torch CPU, {torch.get_num_threads()} threads)"
        run(1)
        b = 2
        t0 = time.perf_counter()
        run(b)
        dt = max(time.perf_counter() - t0, 1e-6)
        b = int(min(1 << 16, max(2, b * target_s / dt)))
        t0 = time.perf_counter()
        run(b)
        dt = time.perf_counter() - t0
        cores = 1 if kind == "hybrid-minsum" else torch.get_num_threads()
        return {"value": b / dt, "unit": "codewords/s", "cores": cores, "kind": "port",
                "sample": f"{b} frames, BG2 Z={z}, {iters} iterations, {what} on {cpu}, {dt:.1f} s"}
    if kind.startswith("gnn"):
        snr = 2.0 if snr is None else snr
        from ldpc_neural_decoder.models import create_message_gnn_decoder
        torch.manual_seed(7)
        dec, conv = create_message_gnn_decoder(torch.from_numpy(H), num_iterations=iters,
                                               hidden_dim=HIDDEN.get(workload, 64), base_graph=torch.from_numpy(base), Z=z)
        sd = {k: v.detach() for k, v in dec.state_dict().items()}
        types = conv.get_message_types(torch.from_numpy(base), z)
        ev, ec = conv.edge_var, conv.edge_chk

        train = kind == "gnn-train"
        if train:
            sd = {k: v.requires_grad_(True) for k, v in sd.items()}

        def run(b):
            x = torch.from_numpy(sample(b))
            if train:
                _, loss = oracle.gnn_forward(sd, x, ev, ev, ec, g.N, g.M, types,
                                             ground_truth=torch.zeros(b, g.N))
                loss.backward()
                return
            with torch.no_grad():
                oracle.gnn_forward(sd, x, ev, ev, ec, g.N, g.M, types)
        run(1)  # warm-up (thread pool, allocator)
        b = 2
        t0 = time.perf_counter()
        run(b)
        dt = max(time.perf_counter() - t0, 1e-6)
        b = int(min(4096, max(2, b * target_s / dt)))
        t0 = time.perf_counter()
        run(b)
        dt = time.perf_counter() - t0
        return {"value": b / dt, "unit": "codewords/s", "cores": torch.get_num_threads(), "kind": "port",
                "sample": f"{b} frames, BG2 Z={z}, MessageGNN {iters} layers H={HIDDEN.get(workload, 64)} fp32, {snr} dB, "
                          f"{'forward + BCE + autograd backward' if train else 'forward'}, "
                          f"oracle.gnn_forward (torch CPU, segment means) on {cpu} with "
                          f"{torch.get_num_threads()} threads, {dt:.1f} s"}
    if kind == "lay":
        _, chk, var, oidx = oracle.llr_mapping(H)
        E = chk.shape[0]
        w_ch, w_res = torch.ones(E), torch.ones(2)

        def run_lay(b):
            llr = torch.from_numpy(sample(b))[:, oidx[0]].contiguous()
            with torch.no_grad():
                v, prev = llr, []
                for _ in range(iters):
                    v = oracle.residual_layer(llr, oracle.variable_layer(llr, oracle.check_layer(v, chk), var),
                                              prev, w_ch, w_res)
                    prev = [v] + prev
                oracle.output_layer(v, llr)
        run_lay(1)
        b = 2
        t0 = time.perf_counter()
        run_lay(b)
        dt = max(time.perf_counter() - t0, 1e-6)
        b = int(min(4096, max(2, b * target_s / dt)))
        t0 = time.perf_counter()
        run_lay(b)
        dt = time.perf_counter() - t0
        return {"value": b / dt, "unit": "codewords/s", "cores": torch.get_num_threads(), "kind": "port",
                "sample": f"{b} frames, BG2 Z={z} (E={E} edge LLRs), {iters} iterations of the index-gather "
                          f"layers, oracle (torch CPU) on {cpu} with {torch.get_num_threads()} threads, {dt:.1f} s"}
    algo = "minsum" if kind == "minsum" else "bp"

    def timed(threads, seconds):
        oracle.set_threads(threads)
        b = 16 * threads
        t0 = time.perf_counter()
        oracle.flood_decode(g, sample(b), algo, iters, 0.75, 0)
        dt = max(time.perf_counter() - t0, 1e-6)
        b = int(min(1 << 18, max(16 * threads, b * seconds / dt)))
        x = sample(b)
        t0 = time.perf_counter()
        oracle.flood_decode(g, x, algo, iters, 0.75, 0)
        return b, time.perf_counter() - t0

    # all cores of this process's share (OMP_NUM_THREADS: 16 per GPU on the bench boxes, whose
    # os.cpu_count() counts the whole machine) and one core, the literal loop order in C both times
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count() or 1
    b1, dt1 = timed(1, target_s / 3)
    bn, dtn = timed(threads, target_s)
    oracle.set_threads(1)
    return {"value": bn / dtn, "unit": "codewords/s", "cores": threads, "kind": "port",
            "value_1core": b1 / dt1,
            "sample": f"{bn} frames, BG2 Z={z}, {algo} {iters} it, {snr} dB, oracle/ldpc_oracle.c (the "
                      f"reference's loop order) with an OpenMP frame loop on {threads} threads of {cpu} "
                      f"(os.cpu_count()={os.cpu_count()}), {dtn:.1f} s; 1 thread: {b1} frames in {dt1:.1f} s"}


def main():
    a = parse()
    # torch.cuda.device_count() does not initialise the GPU on this image (a launcher parent may
    # still spawn its ranks after it)
    action, msg = resolve_launch(a.gpus, os.environ, torch.cuda.device_count())
    if action == "error":
        print(f"bench.py: {msg}", file=sys.stderr, flush=True)
        sys.exit(2)
    if action == "spawn":
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:]))
    world, rank, dev = setup_dist()
    kind, z, iters, bdef, snr = WORKLOADS[a.workload]
    snr = a.snr if a.snr is not None else snr
    sweep = snr is None  # gnn-z32-sweep: every step sweeps 0..6 dB
    snr = 0.0 if sweep else snr
    iters = a.iterations or iters
    B = a.batch or bdef
    if a.data == "auto":
        et_on = kind == "gnn-bf16" and (a.early_termination == "on" or
                                        (a.early_termination == "auto" and a.workload == "gnn-z32-bf16"))
        a.data = "codewords" if et_on else "zero"

    from ldpc_neural_decoder import _native as N
    from ldpc_neural_decoder.utils import awgn_llr, expand_base_matrix, load_base_matrix

    if a.workload.endswith("-stream"):
        os.environ["LDPC_FLOOD_STREAM"] = "1"
    base = load_base_matrix(os.path.join(ROOT, "codes", f"NR_2_0_{z if z in (4, 32) else 32}.txt"))
    H = expand_base_matrix(base, z)
    n = H.shape[1]
    ref_bits = None
    if a.data == "codewords":
        from ldpc_neural_decoder.utils.encoding import SystematicEncoder
        gen = torch.Generator(device=dev)
        gen.manual_seed(20251015 + rank)
        ref_bits = SystematicEncoder(H, dev).random(B, generator=gen).to(torch.uint8)
    llr = awgn_llr(B, n, snr, seed=20251015, frame_offset=rank * B, bits=ref_bits, device=dev)
    counters = torch.zeros(4, dtype=torch.int64, device=dev)
    scratch = torch.zeros(4, dtype=torch.int64, device=dev)  # fused counters of a codeword run (iterations only)

    weights = None
    if kind in ("minsum", "bp"):
        from ldpc_neural_decoder.models import BeliefPropagationDecoder, MinSumScaledDecoder
        dec = (MinSumScaledDecoder(H, iters, 0.75, early_stopping=False) if kind == "minsum"
               else BeliefPropagationDecoder(H, iters, early_stopping=False))
        g = dec.graph(dev)
        bits = torch.empty((B, n), dtype=torch.uint8, device=dev)
        algo = N.LDPC_ALGO_MINSUM if kind == "minsum" else N.LDPC_ALGO_BP
        stream = N.stream_ptr(dev)
        es = {"off": N.LDPC_ES_OFF, "batch": N.LDPC_ES_BATCH, "frame": N.LDPC_ES_FRAME}[a.early_stop]
        wsb = N.check(N.lib().ldpc_flood_workspace_size(g.handle, B, iters, es))
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)

        def step(count):
            # the fused counters count bit errors against the all-zero codeword: a codeword run takes
            # only their iteration sum (index 3: the iterations actually run, early stop included)
            # and counts its errors against the transmitted codewords
            cnt = None if not count else (counters if ref_bits is None else scratch.zero_())
            N.check(N.lib().ldpc_flood_decode(
                g.handle, algo, N.ptr(llr), B, iters, 0.75, es, N.LDPC_OUT_U8,
                N.ptr(bits), None, None, N.ptr(cnt) if cnt is not None else None, N.ptr(ws), wsb, stream))
            if count and ref_bits is not None:
                from ldpc_neural_decoder.utils import count_errors
                count_errors(bits, ref=ref_bits, counters=counters)
                counters[3] += scratch[3]

        dtype = "f32"
        per_launch_alg = flood_bytes_per_cw(g.E, g.N, iters) * B
        streaming = a.workload.endswith("-stream") or z not in (4, 32)
        if streaming:  # messages stream through HBM every iteration: SURVEY 8(d)'s byte model is the bound
            bound, unit, peak = "hbm", "GB/s", HBM_PEAK_GBS
            dominant = f"stream_check_kernel<{kind}> + stream_var_kernel (all iterations)"
        else:
            bound, unit, peak = "valu", "Ginst/s", VALU_PEAK_GINST
            fixed = os.environ.get("LDPC_FLOOD_FIXED", "1") != "0"
            dominant = f"flood_fixed_kernel<BG2_Z{z}, {kind}>" if fixed else f"flood_kernel<{kind}>"
    elif kind == "hybrid-minsum":
        from ldpc_neural_decoder.models import create_custom_minsum_message_gnn_decoder
        from ldpc_neural_decoder.utils import count_errors
        hdec, _ = create_custom_minsum_message_gnn_decoder(H, num_iterations=iters)
        g = hdec._graph(n, dev)
        probs = torch.empty((B, n), dtype=torch.float32, device=dev)
        wsb = N.check(N.lib().ldpc_custom_minsum_workspace_size(g.handle, B))
        ws = torch.empty(max(wsb, 1), dtype=torch.uint8, device=dev)
        stream = N.stream_ptr(dev)

        def step(count):
            N.check(N.lib().ldpc_custom_minsum_decode(g.handle, N.ptr(llr), B, iters, N.ptr(probs), N.ptr(ws), wsb,
                                                      stream))
            if count:
                # probs = sigmoid(llr + S) (MGD:1214-1240) is P(bit = 0) for a channel LLR log P(0)/P(1):
                # counted with the flooding decoders' rule, bit = 1 where the APP is negative (TD:101)
                count_errors((probs < 0.5).to(torch.uint8), ref=ref_bits, counters=counters)

        dtype = "f32"
        # per frame-iteration, messages in HBM: variable phase reads + writes every edge message and
        # reads the LLRs; check phase reads + writes every edge message (fp32); + LLR transpose and
        # the output pass once
        per_launch_alg = (iters * (4 * g.E * 4 + g.N * 4) + 3 * g.N * 4 + g.E * 4) * B
        bound, unit, peak = "hbm", "GB/s", HBM_PEAK_GBS
        dominant = "custom_var_kernel + stream_check_kernel<minsum> (all iterations)"
    elif kind == "lay":
        from ldpc_neural_decoder.models import CheckLayer, OutputLayer, ResidualLayer, VariableLayer
        from ldpc_neural_decoder.utils import create_LLR_mapping
        _, chk, var, out_idx = create_LLR_mapping(H.T)
        E = chk.shape[0]
        chk_d, var_d = chk.to(dev), var.to(dev)
        # edge-vector LLRs: each edge carries its variable's channel LLR (out_idx = variable of edge)
        ellr = llr[:, out_idx[0].to(dev)].contiguous()
        ck, vl, ol = CheckLayer(), VariableLayer(), OutputLayer()
        rs = ResidualLayer(E, depth_L=2).to(dev)

        def step(count):
            with torch.no_grad():
                v, prev = ellr, []
                for _ in range(iters):
                    v = rs(ellr, vl(ellr, ck(v, chk_d), var_d), prev)
                    prev = [v] + prev
                ol(v, ellr)

        dtype = "f32"
        # per frame-iteration: read v + write c (check), read c + llr + write (variable),
        # read llr, c-sum, 2 prev + write (residual) -- 11 passes over the E-vector, fp32
        per_launch_alg = iters * 11 * 4 * E * B
        bound, unit, peak = "hbm", "GB/s", HBM_PEAK_GBS
        dominant = "index-gather layers (all iterations)"
    else:
        from ldpc_neural_decoder.models import create_message_gnn_decoder
        torch.manual_seed(7)
        hid = HIDDEN.get(a.workload, 64)
        gdec, conv = create_message_gnn_decoder(H, num_iterations=iters, hidden_dim=hid,
                                                base_graph=base, Z=z)
        ckpt = a.checkpoint or os.path.join(ROOT, "checkpoints", f"gnn_bg2_z{z}_i{iters}_h{hid}.pt")
        if kind != "hybrid-gnn" and os.path.exists(ckpt):
            # a checkpoint written by the trainer (tools/train_gnn_checkpoint.py): tensors and plain data only
            ck = torch.load(ckpt, map_location="cpu", weights_only=True)
            gdec.load_state_dict(ck["model_state_dict"])
            weights = {"weights": "trained", "checkpoint": os.path.relpath(ckpt, ROOT),
                       "train_config": ck.get("train_config")}
        else:
            weights = {"weights": "random (torch.manual_seed(7))", "checkpoint": None}
        gdec = gdec.to(dev)
        if kind == "gnn-bf16":
            gdec.precision = "bf16"
            # cfg5 = 15 iterations + per-frame early-termination syndrome check
            gdec.early_termination = (a.workload == "gnn-z32-bf16" if a.early_termination == "auto"
                                      else a.early_termination == "on")
        types = conv.get_message_types(base, z).to(dev).to(torch.int32)
        io = conv.message_to_var_index().to(dev).to(torch.int32)
        probs = torch.empty((B, n), dtype=torch.float32, device=dev)
        vg, cg = conv.var_groups, conv.check_groups
        g_m, g_n = H.shape
        sweep_snrs = [float(x) for x in range(0, 7)]
        sweep_out = {}

        if kind == "hybrid-gnn":
            from ldpc_neural_decoder.models import create_custom_variable_message_gnn_decoder
            from ldpc_neural_decoder.utils import count_errors
            torch.manual_seed(7)
            hdec, hconv = create_custom_variable_message_gnn_decoder(H, num_iterations=iters, hidden_dim=64,
                                                                     base_graph=base, Z=z)
            hdec = hdec.to(dev)
            Avh, Ach = hconv.var_to_check_adjacency, hconv.check_to_var_adjacency

            def step(count):
                p, _ = hdec(llr, io, types, Avh, Ach)
                if count:
                    count_errors((p > 0.5).to(torch.uint8), ref=ref_bits, counters=counters)
        elif kind == "gnn-sweep":
            from ldpc_neural_decoder.sweep import evaluate_message_gnn

            def step(count):  # trial t of each SNR -> rank t: every rank decodes B frames per SNR
                sweep_out["ber_fer"] = evaluate_message_gnn(gdec, conv, sweep_snrs, B, world, dev, seed=20251015,
                                                            message_types=types)
        elif kind == "gnn-train":
            opt = torch.optim.SGD(gdec.parameters(), lr=1e-3, momentum=0.9, weight_decay=1e-4)
            gt = torch.zeros((B, n), dtype=torch.float32, device=dev) if ref_bits is None else ref_bits.float()
            Av, Ac = conv.var_to_check_adjacency, conv.check_to_var_adjacency

            def step(count):  # trainer.py:90-102: zero_grad, forward + BCE, backward, SGD step
                opt.zero_grad()
                p, loss = gdec(llr, io, types, Av, Ac, ground_truth=gt)
                loss.backward()
                opt.step()
                if count:
                    from ldpc_neural_decoder.utils import count_errors
                    count_errors((p.detach() > 0.5).to(torch.uint8), ref=ref_bits, counters=counters)
        else:
            def step(count):
                p = gdec.native_forward(llr, io, types, vg, cg)
                if count:
                    from ldpc_neural_decoder.utils import count_errors
                    count_errors((p > 0.5).to(torch.uint8), ref=ref_bits, counters=counters)

        dtype = "bf16" if kind == "gnn-bf16" else "f32"
        E = len(conv.messages)
        # fp32 forward FLOPs per frame-layer as executed: the reference's MLPs cost 12 H^2 per message
        # (two sides x (W1 over [c; g]: 4 H^2 + W2: 2 H^2)); W1's group half is applied once per group
        # (gnn.hip, gnn_group_proj_kernel), so 8 H^2 per message + 2 H^2 per var / check group
        fwd_flops = 8 * hid * hid * E + 2 * hid * hid * (g_n + g_m)
        mlp_flops = 8 * hid * hid * E  # of which on the MLP kernel (f16 splits)
        nominal_flops = 12 * hid * hid * E
        if kind == "hybrid-gnn":
            # check side only: 4 H^2 per message (W1 over c + W2) + 2 H^2 per check group (projection)
            per_launch_alg = (4 * 64 * 64 * E + 2 * 64 * 64 * g_m) * B * iters
            bound, unit, peak = "mfma", "TFLOP/s", FP32_MFMA_PEAK_TFS
        elif kind == "gnn" and hid != 64:
            # gnn_wide.hip (f16 two-term splits) is HBM-bound: SURVEY 8(d)'s per frame-layer bytes (3
            # passes over the (E, H) fp32 features + the group rows written and read) as the
            # algorithmic figure; the design's own traffic in the notes: at H = 96 / 128 the fused MLP
            # (x read twice, both sides' projected group rows gathered, y written: 5 E H words, + 3 (N +
            # M) H for the group means and projections), else the row GEMMs (12 E H: h round-trips HBM
            # between GEMM1 and GEMM2)
            wide_fused = (hid in (96, 128, 160, 192) and os.environ.get("LDPC_GNN_WIDE_FUSED", "1") != "0"
                          and hid <= int(os.environ.get("LDPC_GNN_WIDE_FUSED_MAX", "192")))
            per_launch_alg = (3 * E * hid * 4 + 2 * (g_n + g_m) * hid * 4) * B * iters
            wide_design_bytes = ((5 if wide_fused else 12) * E * hid * 4 + 3 * (g_n + g_m) * hid * 4) * B * iters
            bound, unit, peak = "hbm", "GB/s", HBM_PEAK_GBS
        elif kind in ("gnn-sweep", "gnn"):
            # SURVEY 8(d) cfg2 / cfg4, HBM: per frame-layer 3 passes over the fp32 features (E x 64) +
            # the group rows written and read ((N + M) x 64 fp32, twice; 3.99 MB per cfg2 codeword).
            # The binding resource of this build's fp32 path at both sizes: its kernels move their
            # bytes at 4-5 TB/s while the matrix pipe (fp32 products as f16 two-term splits) is a
            # fraction busy (roofline_notes)
            fp32_layer_bytes = (3 * E * 64 * 4 + 2 * (g_n + g_m) * 64 * 4) * B
            per_launch_alg = fp32_layer_bytes * iters * (len(sweep_snrs) if kind == "gnn-sweep" else 1)
            bound, unit, peak = "hbm", "GB/s", HBM_PEAK_GBS
        elif kind == "gnn-bf16":
            # HBM-bound; per frame-layer 3 passes over the bf16 features
            # (group-mean read, MLP read + write) + the fp32-sized group-mean rows written + read
            bf16_layer_bytes = (3 * E * 64 * 2 + 2 * (g_n + g_m) * 64 * 4) * B  # all frames, one layer
            per_launch_alg = iters * bf16_layer_bytes
            bound, unit, peak = "hbm", "GB/s", HBM_PEAK_GBS
        elif kind == "gnn-train":
            # forward 12 H^2 E + backward 24 H^2 E (recomputed GEMM1, W2^T, W1^T, 4 weight-grad
            # outer products) per frame-layer, fp32 (VALU fp32 peak = fp32 MFMA peak)
            per_launch_alg = 36 * 64 * 64 * E * B * iters
            bound, unit, peak = "mfma", "TFLOP/s", FP32_MFMA_PEAK_TFS
        else:
            # the reference's useful FLOPs, 12 H^2 E per frame-layer
            # (this build executes fewer: see the notes' executed_frac)
            per_launch_alg = nominal_flops * B * iters
            bound, unit, peak = "mfma", "TFLOP/s", FP32_MFMA_PEAK_TFS
        dominant = {"gnn-train": "gnn training step", "gnn-sweep": "SNR sweep (7 x channel + gnn forward + count)",
                    "hybrid-gnn": "hybrid gnn forward (all layers)"}.get(
            kind, "gnn forward (all layers)")

    for _ in range(a.warmup):
        step(False)
    torch.cuda.synchronize()
    barrier(world)
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(a.steps)]
    torch.cuda.synchronize()
    barrier(world)
    t0 = time.perf_counter()
    for i in range(a.steps):
        ev[i][0].record()
        step(i == a.steps - 1)
        ev[i][1].record()
    torch.cuda.synchronize()
    barrier(world)
    elapsed = time.perf_counter() - t0
    kern_ms = float(np.mean([s.elapsed_time(e) for s, e in ev]))
    t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
    tot = counters.clone()
    if dist.is_initialized():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
    elapsed, kern_ms = t.tolist()
    avg_layers = None
    if kind.startswith("gnn") and kind != "gnn-train" and getattr(gdec, "last_iterations", None) is not None:
        avg_layers = float(gdec.last_iterations.double().mean())  # this rank's last step
    be, fe, fr, itsum = tot.tolist()

    if kind == "gnn-bf16" and avg_layers is not None:
        # early termination: the layers actually run (the frames' mean), not the maximum
        per_launch_alg = avg_layers * bf16_layer_bytes
    if rank == 0:
        total_frames = B * world * a.steps * (7 if kind == "gnn-sweep" else 1)
        value = total_frames / elapsed
        achieved = None if bound == "valu" else per_launch_alg / (kern_ms * 1e-3) / (1e9 if unit == "GB/s" else 1e12)
        traffic = None
        tj = a.traffic_json
        if tj is None:  # the newest PMC summary of this workload (profiles/<round>_pmc_<workload>.json)
            import glob
            import re
            found = glob.glob(os.path.join(ROOT, "profiles", f"*_pmc_{a.workload.replace('-', '_')}.json"))
            natural = lambda p: [int(t) if t.isdigit() else t for t in re.split(r"(\d+)", os.path.basename(p))]
            tj = max(found, key=natural) if found else ""
        tjd = None
        pmc_stale = None
        if os.path.exists(tj):
            tjd = json.load(open(tj))
            # a PMC summary describes the library build it profiled (tools/gpu_profile.sh stamps the
            # sha256 of the .so it loaded): from any other build its counts are not this run's
            lib_sha = sha256_file(N.LIB_PATH)
            # ... or of the gfx950 code object that holds the benched kernel (tools/code_object_sha.py):
            # a rebuild after a change in another translation unit leaves that one untouched
            needle = PMC_KERNEL_SYMBOL.get(a.workload)
            code_sha = None
            if needle:
                sys.path.insert(0, os.path.join(ROOT, "tools"))
                from code_object_sha import kernel_code_sha
                code_sha = kernel_code_sha(N.LIB_PATH, needle)
            if tjd.get("lib_sha256") != lib_sha and (code_sha is None
                                                     or code_sha not in tjd.get("code_objects_sha256", [])):
                pmc_stale = {"pmc_source": os.path.relpath(tj, ROOT), "pmc_lib_sha256": tjd.get("lib_sha256"),
                             "loaded_lib_sha256": lib_sha,
                             "note": "the PMC summary was measured on another libldpc_amd.so build: its "
                                     "instruction / byte counts are not reported for this one"}
                tjd = None
        if tjd is not None:
            # the PMC pass ran the same workload at the default batch; scale per launch to this B
            traffic = tjd.get("bytes_per_launch")
            if traffic is not None and tjd.get("batch") and tjd["batch"] != B:
                traffic = traffic * B / tjd["batch"]
        notes = None
        if kind in ("gnn", "gnn-sweep"):
            reps = len(sweep_snrs) if kind == "gnn-sweep" else 1
            split = os.environ.get("LDPC_GNN_SPLIT", "1") != "0" and hid == 64
            secs = kern_ms * 1e-3
            notes = {"flop_model": "the reference's per-message MLPs cost 12 H^2 E FLOP per frame-layer (SURVEY 8(d)); "
                                   "this build executes 8 H^2 E + 2 H^2 (N + M) fp32-equivalent FLOPs (W1's group half "
                                   "once per group). Reported for reference only: roofline.bound names the binding resource",
                     "nominal_fp32_tflops": nominal_flops * B * iters * reps / secs / 1e12,
                     "nominal_frac_of_fp32_mfma": nominal_flops * B * iters * reps / secs / 1e12 / FP32_MFMA_PEAK_TFS,
                     "executed_flops_per_launch": fwd_flops * B * iters * reps}
            if hid != 64:  # gnn_wide.hip: the bytes its kernels move by design, and their rate
                notes["wide_design_bytes_per_launch"] = wide_design_bytes
                notes["wide_design_GBps"] = wide_design_bytes / secs / 1e9
                notes["wide_design_frac_of_hbm_peak"] = wide_design_bytes / secs / 1e9 / HBM_PEAK_GBS
                notes["wide_products"] = ("scaled two-term f16 splits on v_mfma_f32_32x32x16_f16: one power of two "
                                          "per weight matrix and per input row, h's per row and hidden slice under a "
                                          "running exponent" if wide_fused else
                                          "scaled two-term f16 splits on v_mfma_f32_32x32x16_f16, one power of two "
                                          "per weight slice and per input row (recorded by its producer)")
                notes["wide_mlp"] = ("fused per 32-row tile (gnn_wide_mlp_kernel: GEMM1 -> GEMM2 -> head, h in "
                                     "registers)" if wide_fused else "row GEMMs (gnn_wgemm_kernel), h through HBM")
            if split:
                # gnn_mlp2s_kernel: the per-message products (8 H^2 E) as three f16 products each on the
                # f16 MFMA (scaled two-term splits); the group projection (2 H^2 (N + M)) stays on the
                # fp32 MFMA
                mlp_f16 = 3 * mlp_flops * B * iters * reps
                notes["mlp_products"] = ("scaled two-term f16 split, 3 f16 MFMA products per fp32 product "
                                         "(fp32-accurate: tests/test_gnn_depth_gpu.py::test_split_mlp_is_fp32_accurate)")
                notes["mlp_f16_mfma_flops_per_launch"] = mlp_f16
                notes["mlp_f16_mfma_frac_whole_forward"] = mlp_f16 / (kern_ms * 1e-3) / 1e12 / BF16_MFMA_PEAK_TFS
                if nominal_flops * B * iters * reps / secs / 1e12 > FP32_MFMA_PEAK_TFS:
                    notes["nominal_over_fp32_peak"] = ("the reference's FLOPs per second exceed the fp32 MFMA "
                                                       "peak: the products run on the f16 MFMA (three per product)")
        if bound == "valu":
            achieved, notes = valu_roofline(B, n, kern_ms, traffic, tjd, tj if tjd else None, per_launch_alg)
            if tjd is None:
                achieved = None  # no same-build PMC count: the VALU fraction is not measured
            if a.early_stop != "off" or a.iterations or a.snr is not None:
                # the PMC pass ran the default workload (10 iterations, no stop): its instruction
                # count does not describe this run
                achieved = None
                notes = {"valu": "not measured for this variant (the PMC pass is of the default workload)"}
        if pmc_stale is not None:
            notes = dict(notes or {}, pmc_stale=pmc_stale)
        if kind in ("minsum", "bp"):
            # work-normalised rate beside the VALU fraction (which counts instructions, not decoding
            # work): every edge gets one check-to-variable and one variable-to-check update per iteration
            notes = dict(notes or {}, edge_updates_per_s=2.0 * g.E * iters * B / (kern_ms * 1e-3),
                         edge_update_basis="2 E iterations per frame (c2v + v2c), B frames per launch / kernel time")
        # BER / FER of a neural decoder with random weights say nothing about decoding: not reported
        no_rates = kind == "lay" or (weights is not None and weights["checkpoint"] is None)
        if no_rates and weights is not None:
            notes = dict(notes or {}, ber_fer="not reported: random weights (no trained checkpoint for this "
                                              "configuration; tools/train_gnn_checkpoint.py makes one)")
        cpu = None
        if world == 1 and a.cpu_baseline_seconds > 0:
            cpu = cpu_baseline(a.workload, z, iters, a.cpu_baseline_seconds)
        out = {
            "metric": ("training codewords/s (BG2, %d layers, fwd+bwd+SGD)" % iters if kind == "gnn-train"
                       else "codewords/s at fixed SNR (BG2, %d iters)" % iters),
            "value": value,
            "unit": "codewords/s",
            "coded_bits_per_s": value * n,
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": elapsed / a.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": dtype,
            "data": f"synthetic: {'random codewords (utils/encoding.py)' if ref_bits is not None else 'all-zero codeword'}"
                    f" through the on-device QPSK/AWGN channel at "
                    f"{'0..6 (step 1)' if sweep else snr} dB "
                    f"(Philox seed 20251015, frame offset rank*B), resident in HBM",
            "config": {"workload": a.workload, "code": f"5G NR BG2 Z={z} (N={n})",
                       "decoder": kind, "iterations": iters, "batch_per_gpu": B,
                       "early_stop": a.early_stop if kind in ("minsum", "bp") else None,
                       "global_batch": B * world, "snr_db": "0..6" if sweep else snr,
                       "parallelism": f"dp{world}"},
            "ber": None if no_rates else (sweep_out["ber_fer"][0] if kind == "gnn-sweep" else be / max(fr * n, 1)),
            "fer": None if no_rates else (sweep_out["ber_fer"][1] if kind == "gnn-sweep" else fe / max(fr, 1)),
            "model": weights,
            "roofline": {"bound": bound, "kernel": dominant, "achieved": achieved, "peak": peak,
                         "unit": unit, "frac": None if achieved is None else achieved / peak, "traffic": traffic,
                         "kernel_ms": kern_ms,
                         "algorithmic_per_launch": None if bound == "valu" else per_launch_alg,
                         # the MEASURED HBM rate beside the algorithmic one: PMC bytes of
                         # this build per launch / the same live kernel time, and its fraction of peak
                         "traffic_GBps": None if traffic is None else traffic / (kern_ms * 1e-3) / 1e9,
                         "traffic_frac": None if traffic is None else traffic / (kern_ms * 1e-3) / 1e9 / HBM_PEAK_GBS},
            "roofline_notes": notes,
            "avg_layers": avg_layers,
            "avg_iterations": itsum / max(fr, 1) if kind in ("minsum", "bp") else None,
            "cpu_baseline": cpu,
            "dist_backend": dist.get_backend() if dist.is_initialized() else None,
            # the process group's own rank count (the GPUs that did the work) beside the launch
            "world_size": dist.get_world_size() if dist.is_initialized() else 1,
            "launch": ("bench.py --gpus (self-spawned ranks)" if os.environ.get("BENCH_LAUNCH") == "self"
                       else "torch.distributed.run" if "WORLD_SIZE" in os.environ else "single process"),
            # the last step's counters summed over ranks (bits / frames in error, frames counted)
            "counters": {"bit_errors": be, "frame_errors": fe, "frames": fr, "iterations_sum": itsum},
        }
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
