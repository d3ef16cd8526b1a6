"""Multi-GPU sharding logic on CPU: LPT partition properties and a
world_size-2 gloo run (every rank derives the same partition independently,
the shards tile the job list, and the counter reduction gives max time /
summed bytes / all-ok).  SURVEY.md §8e."""
import os
import random
import socket

import pytest

import shard


def test_lpt_partition_tiles_jobs():
    rng = random.Random(7)
    costs = [rng.randint(1, 1 << 22) for _ in range(4096)]
    for world in (1, 2, 4, 8):
        shards = shard.lpt_partition(costs, world)
        flat = sorted(i for s in shards for i in s)
        assert flat == list(range(len(costs)))
        loads = shard.shard_loads(costs, shards)
        # LPT bound: max load <= avg + largest job
        assert max(loads) <= sum(costs) / world + max(costs)


def test_lpt_partition_deterministic_and_balanced():
    costs = [5, 5, 4, 4, 3, 3, 3]
    a = shard.lpt_partition(costs, 2)
    b = shard.lpt_partition(list(costs), 2)
    assert a == b
    loads = shard.shard_loads(costs, a)
    assert max(loads) - min(loads) <= 3
    assert shard.lpt_partition([], 3) == [[], [], []]
    with pytest.raises(ValueError):
        shard.lpt_partition(costs, 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, costs, q):
    import torch.distributed as dist

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = shard.my_shard(costs, rank, world)
        gathered = [None] * world
        dist.all_gather_object(gathered, mine)
        nbytes = sum(costs[i] for i in mine)
        t, b, ok = shard.reduce_counters(0.5 + rank, nbytes, True)
        _, _, ok_one_bad = shard.reduce_counters(0.0, 0, rank == 0)
        q.put((rank, gathered, t, b, ok and not ok_one_bad))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_shards_and_counters():
    import torch.multiprocessing as mp

    rng = random.Random(11)
    costs = [rng.randint(1, 1 << 20) for _ in range(257)]
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, costs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    g0 = res[0][1]
    assert all(r[1] == g0 for r in res)  # every rank derived the same partition
    assert sorted(i for s in g0 for i in s) == list(range(len(costs)))
    for rank, _, t, b, ok in res:
        assert t == 1.5  # max over ranks
        assert b == sum(costs)
        assert ok


def test_bench_self_launch_dry_run():
    """bench.py --gpus 2 with no launcher starts its own 2 ranks (gloo in the
    dry run); by default (weak scaling) each rank decodes its own 64-stream
    batch, with --scaling strong its LPT share of one batch; rank 0 prints one
    line with the reduced counters."""
    import json
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}

    def run(*extra):
        r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--dry-run", "--gpus", "2", "--stream-mib",
                            "1", "--steps", "1", "--warmup", "0", *extra], capture_output=True, text=True, timeout=300,
                           env=env)
        assert r.returncode == 0, r.stderr[-2000:]
        lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
        assert len(lines) == 1, r.stdout
        return json.loads(lines[0])

    d = run("--c5-streams", "64", "--c5-leg-kib", "4")
    assert d["dry_run"] and d["n_gpus"] == 2 and d["verified_bit_exact"] and d["scaling"] == "weak"
    # configs[4] beside the weak headline: the fixed batch split across both ranks (strong)
    c5 = d["c5"]
    assert c5["scaling"] == "strong" and c5["streams_total"] == 64 and c5["verified_bit_exact"], c5
    assert [r["rank"] for r in c5["ranks"]] == [0, 1] and sum(r["streams"] for r in c5["ranks"]) == 64
    assert [r["streams"] for r in c5["ranks"]] == [len(shard.bench_shard(64, k, 2, shard.c5_kind)) for k in (0, 1)]
    assert d["config"]["streams_total"] == 128 and d["rank_streams"] == list(range(64))
    d = run("--scaling", "strong", "--no-c5-leg")
    assert d["dry_run"] and d["n_gpus"] == 2 and d["verified_bit_exact"] and d["scaling"] == "strong"
    assert d["config"]["streams_total"] == 64
    assert d["rank_streams"] == shard.bench_shard(64, 0, 2, shard.c2_kind)
    both = sorted(shard.bench_shard(64, 0, 2, shard.c2_kind) + shard.bench_shard(64, 1, 2, shard.c2_kind))
    assert both == list(range(64))
    # balanced: each rank gets half of the Zipf and half of the line-text streams
    for rk in (0, 1):
        ids = shard.bench_shard(64, rk, 2, shard.c2_kind)
        assert sum(shard.c2_kind(i) == "zipf" for i in ids) == 16


def test_bench_shards_cover_c5():
    for world in (1, 2, 4, 8):
        parts = [shard.bench_shard(4096, r, world, shard.c5_kind) for r in range(world)]
        assert sorted(i for p in parts for i in p) == list(range(4096))
        loads = [sum(2 if shard.c5_kind(i) == "zipf" else 1 for i in p) for p in parts]
        assert max(loads) - min(loads) <= 2
