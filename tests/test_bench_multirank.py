"""bench.py's multi-rank path, executed: the driver's 8-GPU scaling run
launches `torch.distributed.run --nproc-per-node N bench.py --gpus N`; here 2 fresh rank
processes share the one GPU of the box (POLAR_BENCH_BACKEND=gloo for the collectives, HIP for
the decodes), with short steps, the C4 scatter / gather flow and the secondary C3 / C5 entries.
Checks the rank-count all-reduce, the per-rank C5 shard (512 frames over 2 ranks), the error
totals against the per-rank counts, and the scatter -> decode -> gather result."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_two_ranks_gloo(pkg, cuda):
    env = dict(os.environ, POLAR_BENCH_BACKEND="gloo", OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1", "--io", "scatter",
           "--no-ebn0-sweep", "--settle-ms", "0", "--check", "8"]
    res = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    assert res.returncode == 0, res.stderr[-4000:]
    lines = [ln for ln in res.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, res.stdout[-2000:]   # rank 0 prints the one JSON line
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["config"]["frames_per_gpu"] == 65536
    assert r["parity_check"]["bit_exact"]
    e = r["errors_all_ranks"]
    assert e["frames"] == 2 * 65536 and len(e["per_rank"]) == 2
    assert e["frame_errors"] == sum(p["frame_errors"] for p in e["per_rank"])
    assert e["bit_errors"] == sum(p["bit_errors"] for p in e["per_rank"])
    sg = r["scatter_gather"]
    assert sg["gathered_equals_single_decode"] is True and sg["frames_per_step"] == 2 * 65536
    c5 = r["secondary"]["c5"]
    assert c5["frames_per_gpu"] == 256 and c5["frames_all_ranks"] == 512
    assert c5["parity_check"]["bit_exact"] and r["secondary"]["c3"]["parity_check"]["bit_exact"]
    assert "c5_share64" not in r["secondary"]   # at N > 1 the c5 entry is the per-rank share
