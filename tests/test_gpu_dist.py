"""GPU: bench.py's N>1 path end to end (torch.distributed.run, one process
per rank). On a one-GPU box the two ranks share cuda:0 and synchronise over
gloo (bench.py's rehearsal mode); on a multi-GPU node the same command runs
one rank per GPU over RCCL. Checks the single JSON line: weak scaling, the
whole-job value, and that each rank parsed its own shard without errors."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_ranks():
    n = 1 << 20
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1",
           "--config", "c3", "--packets", str(n), "--no-c5"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["scaling"] == "weak" and r["steps"] == 3
    assert r["config"]["frames_per_gpu"] == n
    assert r["value"] > 0 and r["unit"] == "Mpkt/s"
    # value = frames of all ranks / max-over-ranks time
    assert abs(r["value"] - 2 * n * 3 / (r["ms_per_step"] * 3 * 1e-3) / 1e6) < 0.02 * r["value"]
    assert "cpu_baseline" not in r            # rank 0 at N=1 only


def test_bench_spawns_ranks_itself():
    """`python bench.py --gpus 2` with no launcher around it (the driver's
    command) starts both ranks itself and reports n_gpus == 2."""
    n = 1 << 20
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--packets", str(n), "--c5-frames", "2M"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["scaling"] == "weak"
    assert r["config"]["frames_per_gpu"] == n and r["config"]["job_frames"] == 2 * n
    assert abs(r["value"] - 2 * n * 3 / (r["ms_per_step"] * 3 * 1e-3) / 1e6) < 0.02 * r["value"]


def test_bench_config5_and_host_path_over_ranks():
    """The driver's multi-GPU command also measures BASELINE config 5 (the IMIX
    stream split over the ranks, strong scaling) and the PCIe-inclusive rate
    of every rank at once: plain `python bench.py --gpus 2
    --c5-frames 8M`, no launcher around it."""
    total = 8 << 20
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3",
           "--warmup", "1", "--packets", str(1 << 20), "--c5-frames", "8M"]
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    c5 = r["config5"]
    assert c5["frames_total"] == total and c5["scaling"] == "strong" and c5["steps"] == 3
    # the rank shards tile the stream [0, total) in rank order
    assert c5["shards"][0][0] == 0 and c5["shards"][-1][1] == total and len(c5["shards"]) == 2
    assert all(a[1] == b[0] for a, b in zip(c5["shards"], c5["shards"][1:]))
    assert c5["rejected_per_rank"] == [0, 0]
    assert abs(c5["mpkt_s"] - total * 3 / (c5["ms_per_step"] * 3e-3) / 1e6) < 0.02 * c5["mpkt_s"]
    assert len(c5["frac_per_rank"]) == 2 and all(0 < f < 1 for f in c5["frac_per_rank"])
    h = r["h2d_d2h_inclusive"]
    assert h["ranks"] == 2 and h["sample_frames"] == 2 * (1 << 20) and h["gb_per_s"] > 0
    assert len(h["per_rank_gb_per_s"]) == 2


def test_bench_rccl_path_one_rank():
    """The RCCL branch of the multi-GPU line (init_process_group("nccl",
    device_id=...), barrier(device_ids=...), the all-reduces of the timing
    and of the per-rank rows) on one GPU: `torch.distributed.run
    --nproc-per-node 1 bench.py --gpus 1 --dist` (a one-GPU box cannot start
    two RCCL ranks; the 8-GPU node runs the same code with one rank per GPU)."""
    n = 1 << 20
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}",
           os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dist", "--steps", "3",
           "--warmup", "1", "--config", "c3", "--packets", str(n), "--c5-frames", "2M",
           "--no-cpu"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 1 and r["config"]["dist_backend"] == "nccl"
    pl = r["roofline"]["placement"]                       # the arena's read probe
    assert pl["read_gbs"] > 0 and pl["arena_bytes"] >= r["config"]["bytes_per_gpu"] - 16
    assert r["config5"]["rejected_per_rank"] == [0] and r["h2d_d2h_inclusive"]["ranks"] == 1
    assert abs(r["value"] - n * 3 / (r["ms_per_step"] * 3 * 1e-3) / 1e6) < 0.02 * r["value"]
