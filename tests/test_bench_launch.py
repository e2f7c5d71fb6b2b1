"""bench.py's launch logic (CPU): `--gpus N` against the launcher's WORLD_SIZE and the visible GPUs
(the driver's multi-GPU run must never time one GPU under an N-GPU label)."""
import os
import subprocess
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402


@pytest.mark.parametrize("gpus,env,count,want", [
    (1, {}, 0, "run"),                                          # plain single process
    (1, {}, 8, "run"),
    (2, {}, 8, "spawn"),                                        # no launcher: start the ranks
    (8, {}, 8, "spawn"),
    (8, {}, 1, "error"),                                        # RCCL: one GPU per rank
    (2, {"BENCH_DIST_BACKEND": "gloo"}, 1, "spawn"),            # the explicit rehearsal
    (2, {"BENCH_DIST_BACKEND": "gloo"}, 0, "spawn"),
    (4, {"WORLD_SIZE": "4"}, 8, "run"),                         # a rank of the driver's launcher
    (8, {"WORLD_SIZE": "8"}, 8, "run"),
    (1, {"WORLD_SIZE": "1", "BENCH_DIST": "1"}, 1, "run"),      # the RCCL branch at world size 1
    (1, {"WORLD_SIZE": "8"}, 8, "error"),                       # --gpus disagrees with the launcher
    (8, {"WORLD_SIZE": "2"}, 8, "error"),
    (2, {"WORLD_SIZE": "2"}, 1, "error"),                       # RCCL ranks sharing one GPU
    (2, {"WORLD_SIZE": "2", "BENCH_DIST_BACKEND": "gloo"}, 1, "run"),
    (0, {}, 8, "error"),
])
def test_resolve_launch(gpus, env, count, want):
    action, msg = bench.resolve_launch(gpus, env, count)
    assert action == want, (action, msg)
    assert (msg is None) == (want != "error")


def test_gpus_2_without_gpus_exits_nonzero():
    """No GPU visible (this container): `--gpus 2` refuses before any device work."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "BENCH_DIST_BACKEND")}
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1"],
                       cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    if r.returncode == 0:
        pytest.fail("bench.py --gpus 2 succeeded without GPUs")
    assert r.returncode == 2 and "GPU(s) visible" in r.stderr, r.stderr[-1000:]
