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


# ---- a genome sharded over two ranks: the merged output equals one rank's ----
SHARD_LENGTHS = [1_300_000, 1_000_000, 900_000, 700_000, 600_000]
SHARD_NAMES = ["chr1", "chr2", "chr3", "chrX", "chrY"]


def _stub_scan(i):
    """A CPU stand-in for the GPU scan: the chromosome's synthetic reads
    (generated in this process) summarised into one deterministic line."""
    import zlib
    import numpy as np
    import grom_amd
    p = grom_amd.default_params()
    probe = grom_amd.SynthBatch.genome_chrom([2_000_000], 0, p, coverage=8.0, seed=4)
    probe.close()
    b = grom_amd.SynthBatch.genome_chrom(SHARD_LENGTHS, i, p, names=SHARD_NAMES, coverage=8.0, sv_per_mb=3.0,
                                         dup_frac=0.02, seed=4)
    try:
        pos = np.ctypeslib.as_array(grom_amd.C.cast(b.reads.pos, grom_amd.C.POINTER(grom_amd.C.c_int32)),
                                    shape=(b.reads.n,))
        crc = zlib.crc32(pos.tobytes())
        return f"{b.chrom.name.decode()}\t{b.reads.n}\t{b.reads.n_aux}\t{b.chrom.p_last}\t{crc:08x}\n"
    finally:
        b.close()


def _shard_worker(rank, world, port, q):
    import torch.distributed as dist
    from grom_amd.shard import gather_to_rank0, sharded_genome_text
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        text = sharded_genome_text(_stub_scan, SHARD_LENGTHS, world, rank, gather_to_rank0)
        q.put((rank, text))
    finally:
        dist.destroy_process_group()


def test_gloo_world2_sharded_genome_matches_one_rank():
    import torch.multiprocessing as mp
    from grom_amd.shard import sharded_genome_text
    one = sharded_genome_text(_stub_scan, SHARD_LENGTHS, 1, 0)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[1] is None
    assert res[0] == one
    assert one.count("\n") == len(SHARD_LENGTHS) and "chrx" in one and "chry" in one


def test_sharded_text_rejects_gaps_and_overlaps():
    from grom_amd.shard import sharded_genome_text
    with pytest.raises(RuntimeError):
        sharded_genome_text(lambda i: "x", [5, 4], 2, 0, gather=lambda d: [d, d])  # same chromosome twice
    with pytest.raises(RuntimeError):
        sharded_genome_text(lambda i: "x", [5, 4], 2, 0, gather=lambda d: [d])  # rank 1's share missing


def test_sharded_text_carries_ctx_rows_to_the_postpass():
    """With (vcf, raw CTX) per chromosome, rank 0 joins both in chromosome order
    and runs the translocation post-pass over the whole genome's CTX rows."""
    from grom_amd.shard import sharded_genome_text
    parts = {0: {0: ("v0\n", "c0\n"), 2: ("v2\n", "c2\n")}, 1: {1: ("v1\n", "c1\n")}}
    out = sharded_genome_text(lambda i: None, [5, 4, 3], 2, 0, gather=lambda d: [parts[0], parts[1]],
                              ctx_post=lambda raw: raw.upper())
    assert out == ("v0\nv1\nv2\n", "C0\nC1\nC2\n")


def test_ctx_postpass_pairs_translocations():
    """grom_ctx_postpass (main's post-pass, GROM.c:22400-22770) on two raw CTX
    rows that are each other's mates: both kept, as BND rows naming the mate."""
    import grom_amd
    # raw row: type chr pos binom ev rd conc other mchr mpos rs re hez
    raw = ("CTX_F\tchr1\t1000\t1e-10\t5.0\t30\t10\t0\t1\t-5000\t900\t990\t1e-5\n"
           "CTX_R\tchr2\t5000\t1e-10\t5.0\t30\t10\t0\t0\t1000\t5010\t5100\t1e-5\n")
    text = grom_amd.ctx_postpass(raw, ["chr1", "chr2"], 600, 150)
    rows = text.splitlines()
    assert len(rows) == 2 and all("SVTYPE=BND" in r for r in rows), text
    assert rows[0].startswith("chr1\t1001\t") and "chr2:5000" in rows[0]


# ---- the parallel merge of the ranks' VCFs (bench.py --gpus N) ----

_MERGE_CHROMS = ["chr1", "chr2", "chr3", "chr4", "chr5"]


def _rank_vcf(path, chroms, seg_path=None):
    """A rank's CLI output: the header, then each of its chromosomes' rows
    together (different row counts per chromosome; chr4 has none)."""
    hdr = "##fileformat=VCFv4.1\n#CHROM\tPOS\tID\tREF\tALT\n"
    rows = {c: "".join(f"{c}\t{p}\t.\tA\tT\n" for p in range(1, 1 + 3 * (i + 1)))
            for i, c in enumerate(_MERGE_CHROMS) if c != "chr4"}
    body, segs, at = "", [], len(hdr)
    for c in chroms:
        t = rows.get(c, "")
        if t:
            segs.append(f"{c}\t{at}\t{len(t)}\n")
        body += t
        at += len(t)
    with open(path, "w") as f:
        f.write(hdr + body)
    if seg_path:
        with open(seg_path, "w") as f:
            f.write("".join(segs))


def _merge_worker(rank, world, port, d, use_segs, q):
    import torch.distributed as dist
    from grom_amd.shard import all_gather_objects, merge_rank_outputs_parallel
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = [c for i, c in enumerate(_MERGE_CHROMS) if i % world == rank]
        merge_rank_outputs_parallel(rank, os.path.join(d, f"r{rank}.vcf"), mine, _MERGE_CHROMS,
                                    os.path.join(d, "merged.vcf"), all_gather_objects, dist.barrier,
                                    segs_path=os.path.join(d, f"r{rank}.segs") if use_segs else None)
        q.put((rank, "ok"))
    except BaseException as e:  # noqa: BLE001 -- reported to the test
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("use_segs", [True, False], ids=["segment_index", "scan"])
def test_gloo_world2_parallel_merge_matches_rank0_merge(tmp_path, use_segs):
    """bench.py's N>1 merge: every rank copies its chromosomes' rows to their
    offsets in the merged VCF (from the CLI's GROM_VCF_SEGS index, or by
    scanning its file); the bytes equal rank 0's merge_rank_outputs join."""
    import torch.multiprocessing as mp
    from grom_amd.shard import merge_rank_outputs
    world = 2
    for r in range(world):
        mine = [c for i, c in enumerate(_MERGE_CHROMS) if i % world == r]
        _rank_vcf(tmp_path / f"r{r}.vcf", mine, tmp_path / f"r{r}.segs")
        (tmp_path / f"r{r}.ctxraw").write_text("")
    want, _ = merge_rank_outputs([str(tmp_path / f"r{r}.vcf") for r in range(world)],
                                 [str(tmp_path / f"r{r}.ctxraw") for r in range(world)], _MERGE_CHROMS,
                                 _MERGE_CHROMS, 600, 150)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_merge_worker, args=(r, world, port, str(tmp_path), use_segs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=300) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == {0: "ok", 1: "ok"}, res
    assert (tmp_path / "merged.vcf").read_text() == want
    assert want.count("\n") == 2 + 3 + 6 + 9 + 15


def test_vcf_segments_rejects_interleaved_rows():
    from grom_amd.shard import vcf_segments
    data = b"#h\nchr1\t1\nchr2\t1\nchr1\t2\n"
    with pytest.raises(RuntimeError):
        vcf_segments(data, ["chr1", "chr2"])
    assert vcf_segments(b"#h\nchr1\t1\nchr1\t2\nchr2\t1\n", ["chr1", "chr2"]) == (3, {"chr1": (3, 17), "chr2": (17, 24)})


def test_gloo_world2_merge_fails_fast_on_every_rank(tmp_path):
    """A rank whose segment index does not validate (it used to
    raise alone, leaving the other rank in the next collective until the
    process-group timeout): both ranks raise within seconds."""
    import time

    import torch.multiprocessing as mp
    world = 2
    for r in range(world):
        mine = [c for i, c in enumerate(_MERGE_CHROMS) if i % world == r]
        _rank_vcf(tmp_path / f"r{r}.vcf", mine, tmp_path / f"r{r}.segs")
    (tmp_path / "r1.segs").write_text("chr2\t0\t5\n")  # does not tile rank 1's file
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    t0 = time.time()
    procs = [ctx.Process(target=_merge_worker, args=(r, world, port, str(tmp_path), True, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert time.time() - t0 < 100
    assert all("merge failed on rank(s) 1" in res[r] for r in range(world)), res
