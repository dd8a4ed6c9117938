"""N>1 bench bookkeeping on CPU (gloo, world_size 2): barrier-bracketed timing, max over
ranks, whole-job unit sums, and the partition assignment.  The data path itself has no
collective: each rank encodes its own partitions, so only these scalars cross
ranks.  Each rank's step here writes its partition's file with the CPU oracle (no GPU on this
host); the GPU writer path is the same per-rank code in bench.write_file."""
import os
import socket
import sys
import time

import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world))
    os.environ.pop("KPW_PIN_CACHE_GB", None)
    sys.path.insert(0, ROOT)
    for p in ("synth", "oracle", "kafka-parquet-writer_amd"):
        sys.path.insert(0, os.path.join(ROOT, p))
    import bench
    dist = bench.dist_init(world, rank, backend="gloo")
    calls = []
    import oracle
    import synth
    seeds = bench.partition_seeds("c2", rank, world)
    data, offs = synth.generate(synth.KIND_REC8, seeds[0][0], 2000 * (rank + 1))
    fb = oracle.encode_file(synth.REC8, data, offs, oracle.make_props(codec=oracle.SNAPPY))

    def step(i):
        calls.append(i)
        assert oracle.encode_file(synth.REC8, data, offs, oracle.make_props(codec=oracle.SNAPPY)) == fb
        time.sleep(0.05 * (rank + 1))   # rank 1 is the slow one
        return rank

    elapsed, outs = bench.timed_steps(step, steps=3, warmup=2, dist=dist)
    units = bench.reduce_scalar(100 * (rank + 1), dist)
    # the per-rank host-memory budget bench.py reports at N>1 (library caps, no GPU call)
    mem = bench.rank_memory(dist, pinned_sets=[(data, offs)])
    q.put((rank, elapsed, calls, outs, units, mem))
    dist.destroy_process_group()


def test_two_rank_timing_and_units():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, e0, c0, o0, u0, m0), (r1, e1, c1, o1, u1, m1) = res
    assert c0 == c1 == [0, 1, 2, 3, 4]         # warmup 2 + exactly 3 timed steps
    assert o0 == [0, 0, 0] and o1 == [1, 1, 1]
    assert e0 == pytest.approx(e1)             # every rank reports the max over ranks
    assert e0 >= 3 * 0.1 * 0.95                # ... which is the slow rank's time
    assert u0 == u1 == 300                     # whole-job units = sum over ranks
    # pinned cache cap shared by the node's ranks: 48 GB / LOCAL_WORLD_SIZE per process
    assert m0["pin_cache_cap_gb"] == m1["pin_cache_cap_gb"] == pytest.approx(48 * 2 ** 30 / 2 / 1e9, rel=1e-3)
    assert m0["local_world_size"] == 2
    # every rank's worst-case pinned total: its record sets + the cache cap (max over ranks)
    assert m0["pinned_budget_gb_max_over_ranks"] == m1["pinned_budget_gb_max_over_ranks"]
    assert m0["pinned_budget_gb_max_over_ranks"] >= m0["pin_cache_cap_gb"]


def test_partition_assignment_disjoint():
    """C5: 64 partitions over 8 GPUs, 8 writers each, every partition exactly once; C2 at N>1:
    one distinct partition per rank; the timed steps of a rank cycle over distinct batches."""
    sys.path.insert(0, ROOT)
    import bench
    c5 = [sd for r in range(8) for ss in bench.partition_seeds("c5", r, 8) for sd in ss]
    assert len(c5) == 64 and len(set(c5)) == 64 and min(c5) == 0xC0FFEE05
    for w in (1, 2, 4, 8):
        c2 = [bench.partition_seeds("c2", r, w) for r in range(w)]
        flat = [sd for sets in c2 for ss in sets for sd in ss]
        assert len(set(flat)) == len(flat) == 2 * w
    assert bench.partition_seeds("c2", 0, 1)[0] == [0xC0FFEE02]
