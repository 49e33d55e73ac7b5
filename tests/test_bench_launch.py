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


def test_bench_layout_plan_config4_and_din_batches():
    """--gpus N --shard catalog lays the work out as BASELINE's configs: recall
    catalog-sharded (config 4, whole screen tiles, every item block and user
    once) and the 165 DIN Dice batches round-robin (batch b on rank b mod N)."""
    p = _run(["--gpus", "3", "--shard", "catalog", "--dry-run", "--backend", "gloo"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    plan = line["layout"]
    rec, din = plan["recall"], plan["din"]
    assert rec["layout"] == "catalog" and "config 4" in rec["parallelism"]
    nblk = -(-364_047 // 32)
    blocks = [r["blocks"] for r in rec["per_rank"]]
    assert blocks[0][0] == 0 and blocks[-1][1] == nblk
    assert all(a[1] == b[0] for a, b in zip(blocks, blocks[1:]))
    assert all(lo % rec["tile_blocks"] == 0 for lo, _ in blocks)
    users = [r["users"] for r in rec["per_rank"]]
    assert users[0][0] == 0 and users[-1][1] == 250_000 and all(a[1] == b[0] for a, b in zip(users, users[1:]))
    assert din["batches"] == 165 and [r["batches"] for r in din["per_rank"]] == [55, 55, 55]
    assert sum(r["samples"] for r in din["per_rank"]) == 675_653
    assert [r["short_batch"] for r in din["per_rank"]] == [False, False, True]  # batch 164 -> rank 2
    assert line["covered"] == {"item_blocks": nblk, "users": 250_000, "din_samples": 675_653, "din_batches": 165}


def test_bench_default_layout_is_users_sharded():
    """The N > 1 headline is users-sharded (weak scaling, no data-path
    collective); config 4 is measured beside it."""
    p = _run(["--gpus", "2", "--dry-run", "--backend", "gloo"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    rec = line["layout"]["recall"]
    assert rec["layout"] == "users" and all(r["users"] == [0, 250_000] for r in rec["per_rank"])


def test_bench_layout_plan_users_and_single():
    from importlib import import_module
    import argparse

    sys.path[:0] = [REPO, os.path.join(REPO, "news-recommendation-tc_amd")]
    bench = import_module("bench")
    a = argparse.Namespace(users=250_000, items=364_047, dim=32, din_samples=675_653, shard="users")
    plan = bench.layout_plan(a, 8)
    assert plan["recall"]["layout"] == "users"
    assert all(r["users"] == [0, 250_000] for r in plan["recall"]["per_rank"])
    assert [r["batches"] for r in plan["din"]["per_rank"]] == [21, 21, 21, 21, 21, 20, 20, 20]
    one = bench.layout_plan(a, 1)
    assert one["recall"]["parallelism"] == "single" and one["din"]["per_rank"][0]["samples"] == 675_653
    mine, rows = bench.din_batches(675_653, 4096, 8, 4)
    assert mine == list(range(4, 165, 8)) and rows[-1] == 675_652  # batch 164 = 4 mod 8: the short one, last


def test_bench_layout_plan_grid():
    """Config 4 as a rank grid: --gpus 4 --user-groups 2 (nrk.dist.layout_2d;
    the default is one group) -- each user group's ranks split the
    catalog in whole tiles, every user once, every item block once per group."""
    p = _run(["--gpus", "4", "--shard", "catalog", "--user-groups", "2", "--dry-run", "--backend", "gloo"])
    assert p.returncode == 0, p.stderr[-2000:]
    line = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][0])
    rec = line["layout"]["recall"]
    assert rec["user_groups"] == 2 and "2 user groups x 2 catalog shards" in rec["parallelism"]
    nblk = -(-364_047 // 32)
    per = rec["per_rank"]
    assert [r["group_users"] for r in per] == [[0, 125_000], [0, 125_000], [125_000, 250_000], [125_000, 250_000]]
    assert [r["blocks"][0] for r in per] == [0, per[0]["blocks"][1], 0, per[2]["blocks"][1]]
    assert per[1]["blocks"][1] == nblk and per[3]["blocks"][1] == nblk
    users = [r["users"] for r in per]
    assert users[0][0] == 0 and users[-1][1] == 250_000 and all(a[1] == b[0] for a, b in zip(users, users[1:]))
    assert line["covered"]["item_blocks"] == 2 * nblk and line["covered"]["users"] == 250_000
    from importlib import import_module
    import argparse

    sys.path[:0] = [REPO, os.path.join(REPO, "news-recommendation-tc_amd")]
    bench = import_module("bench")
    a = argparse.Namespace(users=250_000, items=364_047, dim=32, din_samples=675_653, shard="catalog", topk=30,
                           user_groups=None)
    assert bench.layout_plan(a, 8)["recall"]["user_groups"] == 1
    a.user_groups = 2
    assert bench.layout_plan(a, 8)["recall"]["user_groups"] == 2
