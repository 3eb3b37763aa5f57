"""bench.py --gpus N outside a launcher starts N ranks itself (torch.distributed.run
as a child, before anything touches a GPU) and they must all join one
communicator: a 2-rank gloo rehearsal of that plumbing on the CPU."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_gpus_2_launches_two_ranks():
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo")
    env.pop("WORLD_SIZE", None)
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--plumbing-check"], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["ranks_seen"] == 2


def test_bench_rejects_mismatched_world_size():
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--plumbing-check"], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0


def test_bench_missing_rank_fails_loudly():
    """A rank whose peer never joins must not hang the run: the communicator's
    start runs under bench.py's watchdog (BENCH_DIST_TIMEOUT_S) and the rank
    exits non-zero with a message naming the phase."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, BENCH_DIST_BACKEND="gloo", BENCH_DIST_TIMEOUT_S="8", WORLD_SIZE="2", RANK="0",
               LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                          "--plumbing-check"], env=env, capture_output=True, text=True, timeout=120)
    assert out.returncode != 0
    assert "joining the gloo communicator" in out.stderr, out.stderr[-2000:]
    assert not [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
