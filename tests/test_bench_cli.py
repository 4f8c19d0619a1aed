"""CPU: bench.py's rank-count guard. Under a launcher, --gpus must equal
WORLD_SIZE; the check runs before anything touches the GPU, so it is
testable here."""
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_gpus_must_match_world_size():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "3"],
                         cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 2
    assert "WORLD_SIZE=2" in out.stderr
    assert not [l for l in out.stdout.splitlines() if l.startswith("{")]


def test_host_cores_reports_affinity():
    sys.path.insert(0, ROOT)
    import bench
    threads, visible, quota = bench.host_cores()
    assert visible == len(os.sched_getaffinity(0))
    assert 1 <= threads <= visible
    if quota is not None:
        assert threads <= max(1, int(quota))


def test_parse_count_suffixes():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.parse_count("8M") == 8 << 20
    assert bench.parse_count("256m") == 1 << 28
    assert bench.parse_count("4096") == 4096
    assert bench.parse_count("2K") == 2048
    assert bench.parse_count(str(bench.C5_TOTAL)) == bench.C5_TOTAL
