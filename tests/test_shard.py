"""Multi-rank path of bench.py / the sharded scan, on CPU with gloo (world 2)."""
import os
import socket

import pytest

from grom_amd.shard import assign_chromosomes


def test_assign_chromosomes_lpt():
    # GRCh38-like lengths: every chromosome lands on exactly one rank, the
    # assignment is deterministic and balanced within one chromosome
    lengths = [248, 242, 198, 190, 181, 171, 159, 145, 138, 134, 135, 133, 114, 107, 102, 90, 83, 80, 59, 64,
               47, 51, 156, 57]
    for world in (1, 2, 4, 8):
        shards = assign_chromosomes(lengths, world)
        assert sorted(i for s in shards for i in s) == list(range(len(lengths)))
        assert shards == assign_chromosomes(lengths, world)
        loads = [sum(lengths[i] for i in s) for s in shards]
        assert max(loads) - min(loads) <= max(lengths)
    assert assign_chromosomes([5], 2) == [[0], []]
    with pytest.raises(ValueError):
        assign_chromosomes([1], 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import time
    import torch.distributed as dist
    from grom_amd.shard import max_over_ranks, timed_steps
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []

        def step():
            calls.append(1)
            time.sleep(0.05 * (rank + 1))  # rank 1 is the slow one

        dt = timed_steps(step, 3, dist.barrier)
        q.put((rank, len(calls), dt, max_over_ranks(dt)))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_timing_is_max_over_ranks():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, n0, dt0, m0), (r1, n1, dt1, m1) = res
    assert (r0, r1) == (0, 1) and n0 == n1 == 3
    # both ranks report the same max, and it covers the slow rank's 3 x 0.1 s
    assert m0 == m1 == max(dt0, dt1)
    assert m0 >= 0.3


def test_timed_concurrent_runs_every_step_once():
    from grom_amd.shard import timed_concurrent
    seen = []
    fns = [lambda i, k=k: seen.append((k, i)) for k in range(3)]
    dt = timed_concurrent(fns, 8, lambda: None)
    assert dt >= 0
    assert sorted(i for _, i in seen) == list(range(8))
    assert all(i % 3 == k for k, i in seen)
