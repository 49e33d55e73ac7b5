"""CPU: ``bench.py --gpus N`` starts N ranks itself (the driver's command
shape has no torch.distributed launcher around it).  The dry run goes through
the same launcher and rendezvous over gloo, without the GPU workload."""
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, timeout=180):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    return subprocess.run([sys.executable, os.path.join(REPO, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=timeout)


def test_bench_gpus2_launches_two_ranks():
    p = _run(["--gpus", "2", "--dry-run", "--backend", "gloo"])
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout  # rank 0 only
    assert json.loads(lines[0])["n_gpus"] == 2
    found = re.findall(r"\[rank (\d+)/2\] local_rank \d+ pid (\d+)", p.stderr)
    assert sorted(r for r, _ in found) == ["0", "1"], p.stderr
    assert len({pid for _, pid in found}) == 2  # two distinct worker processes


def test_bench_gpus1_stays_single_process():
    p = _run(["--gpus", "1", "--dry-run"])
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip().splitlines()[-1])["n_gpus"] == 1
    assert "[launcher]" not in p.stderr


def test_bench_launcher_propagates_rank_failure():
    # a bad backend name makes every rank fail in init_process_group
    p = _run(["--gpus", "2", "--dry-run", "--backend", "no-such-backend"])
    assert p.returncode != 0
