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
