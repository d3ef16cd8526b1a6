"""Stream sharding across GPUs: one process per GPU, independent streams.

Inflate has no exchange step between streams, so a multi-GPU
batch is a partition of the job list: every rank decodes its own shard with
one zs_inflate_batch() call and no collective touches the data.  The only
collectives are the bench contract's barrier and the reduction of per-rank
counters (elapsed time: max; bytes: sum; verification: min).

Partitioning is greedy LPT on a per-job cost (compressed size by default, the
decompressed size when known, e.g. a gzip ISIZE trailer): jobs in decreasing
cost order, each to the currently least-loaded rank (ties: lowest rank, then
lowest job index), which is deterministic, so every rank computes the same
partition without communicating.
"""
import heapq


def lpt_partition(costs, world):
    """Return `world` lists of job indices; each list is in ascending index order."""
    if world < 1:
        raise ValueError("world must be >= 1")
    order = sorted(range(len(costs)), key=lambda i: (-int(costs[i]), i))
    heap = [(0, r) for r in range(world)]
    shards = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        shards[r].append(i)
        heapq.heappush(heap, (load + int(costs[i]), r))
    return [sorted(s) for s in shards]


def corpus_costs(stream_ids, kind_of):
    """Per-stream LPT costs for the bench corpora, known before any stream is
    generated: a Zipf-text stream compresses to ~2x the bytes of a line-text
    stream of the same size (ratio ~3-4 vs ~6-8 at zlib L6) and decodes in
    ~2x the time, so it costs 2 and a line-text stream 1."""
    return [2 if kind_of(i) == "zipf" else 1 for i in stream_ids]


def c2_kind(i):
    """configs[1] stream i: Zipf text for i % 64 < 32, line text otherwise (tests/corpus.py)."""
    return "zipf" if i % 64 < 32 else "lines"


def c5_kind(k):
    """configs[4] stream k: Zipf text for k % 4 < 2, line text otherwise (tests/corpus.py:c5_stream)."""
    return "zipf" if k % 4 < 2 else "lines"


def bench_shard(nstreams, rank, world, kind_of):
    """Stream ids of `rank` when `nstreams` bench streams are split across `world`
    ranks (strong scaling: the node decodes the same batch whatever the world)."""
    ids = list(range(nstreams))
    return [ids[i] for i in lpt_partition(corpus_costs(ids, kind_of), world)[rank]]


def my_shard(costs, rank, world):
    """Job indices of `rank` under lpt_partition(costs, world)."""
    return lpt_partition(costs, world)[rank]


def shard_loads(costs, shards):
    return [sum(int(costs[i]) for i in s) for s in shards]


def reduce_counters(elapsed_s, nbytes, ok, device=None):
    """All-reduce of one rank's counters over the default process group:
    (max elapsed seconds, sum of bytes, all ranks ok).  With no initialised
    process group the values are returned unchanged."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()):
        return elapsed_s, nbytes, bool(ok)
    t = torch.tensor([float(elapsed_s)], dtype=torch.float64, device=device)
    b = torch.tensor([int(nbytes)], dtype=torch.int64, device=device)
    k = torch.tensor([1 if ok else 0], dtype=torch.int32, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.all_reduce(b, op=dist.ReduceOp.SUM)
    dist.all_reduce(k, op=dist.ReduceOp.MIN)
    return float(t.item()), int(b.item()), bool(k.item())
