"""The RCCL branch of the multi-GPU path, executed on one GPU (GPU).

SURVEY 8(e) / north_star: frames shard by rank, RCCL over xGMI only for the final counter
all-reduce.  The driver's 8-GPU bench is the only run with several GPUs; this test makes the RCCL
code path itself run on the one-GPU box: bench.py under `torch.distributed.run --nproc-per-node 1`
with BENCH_DIST=1 initialises a `nccl` (= RCCL) process group of one rank, and every counter /
timing reduction (bench.py) and the sweep's all_reduce (sweep.py _dist_all_reduce) goes through
RCCL on device tensors.  The counters must equal the plain single-process run's exactly.

Each run is a fresh subprocess started from here (no exec from a process that touched the GPU);
the launcher and its worker initialise the GPU themselves.
"""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _bench(args, dist):
    env = dict(os.environ)
    env.pop("BENCH_DIST", None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if dist:
        env["BENCH_DIST"] = "1"
        env["MASTER_ADDR"] = "127.0.0.1"
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
               "--master-addr", "127.0.0.1", "--master-port", "29533", "bench.py"] + args
    else:
        cmd = [sys.executable, "bench.py"] + args
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [x for x in r.stdout.splitlines() if x.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.parametrize("workload,extra", [
    ("minsum-z32", ["--batch", "4096", "--snr", "-2.0"]),
    ("gnn-z32-sweep", ["--batch", "256"]),
])
def test_rccl_world_of_one_equals_single_process(workload, extra):
    args = ["--workload", workload, "--steps", "2", "--warmup", "1", "--cpu-baseline-seconds", "0"] + extra
    plain = _bench(args, dist=False)
    ranked = _bench(args, dist=True)
    print(f"{workload}: plain ber {plain['ber']} fer {plain['fer']} | rccl ber {ranked['ber']} fer {ranked['fer']} "
          f"({ranked['dist_backend']}, {ranked['value']:.4g} cw/s)")
    assert plain["dist_backend"] is None
    assert ranked["dist_backend"] == "nccl" and ranked["n_gpus"] == 1
    assert ranked["ber"] == plain["ber"] and ranked["fer"] == plain["fer"]
    if workload == "minsum-z32":
        assert plain["ber"] > 0  # -2 dB: the counters carry errors, so equality means something


def _run(args, extra_env=None, timeout=300):
    env = dict(os.environ)
    for k in ("BENCH_DIST", "BENCH_DIST_BACKEND", "WORLD_SIZE", "RANK", "LOCAL_RANK", "BENCH_LAUNCH"):
        env.pop(k, None)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.update(extra_env or {})
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, env=env, capture_output=True, text=True,
                          timeout=timeout)


def test_bench_gpus_2_self_launches_two_ranks():
    """`bench.py --gpus 2` (no launcher) starts two ranks itself.  Rehearsed on one card with
    BENCH_DIST_BACKEND=gloo (the ranks share it): the line reports 2 GPUs, a 2 B global batch and a
    process group of 2, and the counters summed over the ranks equal one process decoding the
    same 2 B frames (rank r decodes Philox frames r B .. r B + B - 1)."""
    B = 4096
    common = ["--workload", "minsum-z32", "--steps", "2", "--warmup", "1", "--snr", "-2.0", "--cpu-baseline-seconds", "0"]
    r = _run(["--gpus", "2", "--batch", str(B)] + common, {"BENCH_DIST_BACKEND": "gloo"})
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 alone prints
    two = json.loads(lines[0])
    one = _bench(["--batch", str(2 * B)] + common, dist=False)
    print(f"2 ranks: {two['counters']} ({two['value']:.4g} cw/s) | 1 process: {one['counters']}")
    assert two["n_gpus"] == 2 and two["world_size"] == 2 and two["dist_backend"] == "gloo"
    assert two["config"]["global_batch"] == 2 * B and two["launch"].startswith("bench.py --gpus")
    assert one["n_gpus"] == 1 and one["world_size"] == 1
    assert two["counters"] == one["counters"] and one["counters"]["bit_errors"] > 0
    assert one["counters"]["frames"] == 2 * B


def test_bench_gpus_2_with_rccl_on_one_gpu_refuses():
    """With RCCL (the default backend) `--gpus 2` on a one-GPU box must fail, not time one GPU."""
    import torch
    if torch.cuda.device_count() >= 2:
        pytest.skip("more than one GPU visible")
    r = _run(["--gpus", "2", "--workload", "minsum-z32", "--steps", "1", "--warmup", "0", "--batch", "64",
              "--cpu-baseline-seconds", "0"], timeout=120)
    assert r.returncode == 2, (r.returncode, r.stderr[-2000:])
    assert "GPU(s) visible" in r.stderr and not [x for x in r.stdout.splitlines() if x.startswith("{")]
