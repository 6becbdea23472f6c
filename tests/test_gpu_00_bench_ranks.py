"""`bench.py --gpus N` on the GPU (config C4's launcher path): without a
launcher it starts its own N ranks (torch.distributed.run, one process per
GPU), refuses more ranks than visible GPUs, and with --allow-shared (a
rehearsal of N ranks on one GPU) gathers every rank's tile ImageBlocks to
rank 0, checks the assembled frame against a whole-frame render and runs the
parity leg on it.  This file runs first among the GPU tests (its name sorts
first) and never initialises the GPU in the pytest process itself: the ranks
are child processes, and a process that has initialised the GPU must not
start programs (the device count here comes from torch, which does not
initialise it)."""
import json
import os
import subprocess
import sys

import pytest

import bench
from conftest import REPO

pytestmark = pytest.mark.gpu


def _bench(args, timeout=600):
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *args], capture_output=True, text=True,
                          timeout=timeout, cwd=REPO)


SMALL = ["--workload", "cbox", "--width", "320", "--height", "180", "--spp", "16", "--steps", "2", "--warmup", "1",
         "--no-cpu"]


def test_bench_two_ranks_gather_and_check_the_frame():
    r = _bench(["--gpus", "2", "--allow-shared", *SMALL])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [line for line in r.stdout.splitlines() if line.startswith("{")]
    assert len(lines) == 1, r.stdout[-3000:]
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2
    assert out["devices"]["distinct"] >= 1 and len(out["devices"]["pci"]) == 2
    assert out["assembly"]["pass"], out["assembly"]
    assert out["parity"]["pass"], out["parity"]
    assert "assembled from all 2 ranks" in out["parity"]["tiles"]


@pytest.mark.skipif(bench.visible_gpus() >= 2, reason="needs a box with fewer than 2 GPUs")
def test_bench_refuses_two_ranks_on_one_gpu():
    r = _bench(["--gpus", "2", *SMALL], timeout=300)
    assert r.returncode != 0
    assert "refusing" in r.stderr, r.stderr[-2000:]
    assert not [line for line in r.stdout.splitlines() if line.startswith("{")]
