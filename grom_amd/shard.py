"""Chromosome sharding and multi-rank timing (one process per GPU).

The per-chromosome scan has no cross-chromosome state (every
array of count_discordant_pairs is local to one call, GROM.c:1432), so ranks
split the chromosomes and never exchange data on the scan path.  The one
genome-wide step after the scans is main's translocation post-pass
(GROM.c:22400-22770), which pairs CTX rows across chromosomes: ranks hand
their raw CTX rows to rank 0 with the VCF text and rank 0 runs it
(grom_amd.ctx_postpass).  torch.distributed (RCCL on the GPU box, gloo in the
CPU tests) carries that gather, the barrier around the timed region and the
max-over-ranks of its duration.
"""
import time
from typing import Callable, List, Sequence


def assign_chromosomes(lengths: Sequence[int], world: int) -> List[List[int]]:
    """Longest-processing-time assignment of chromosome indices to ranks.

    The reference already processes chromosomes longest-first
    (GROM.c:22318-22336); each chromosome goes to the least-loaded rank, ties
    to the lower rank, so the result is deterministic."""
    if world < 1:
        raise ValueError("world size must be >= 1")
    order = sorted(range(len(lengths)), key=lambda i: (-lengths[i], i))
    load = [0] * world
    shards: List[List[int]] = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        shards[r].append(i)
        load[r] += lengths[i]
    for s in shards:
        s.sort()
    return shards


def timed_steps(step: Callable[[], None], steps: int, barrier: Callable[[], None]) -> float:
    """Seconds for exactly `steps` calls of step(), bracketed by barrier()."""
    barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    barrier()
    return time.perf_counter() - t0


def timed_concurrent(steps_of: "list[Callable[[int], None]]", steps: int, barrier: Callable[[], None]) -> float:
    """Seconds for exactly `steps` steps dealt round-robin over len(steps_of)
    host threads (thread k runs steps k, k+F, ...; one library context each),
    bracketed by barrier().  Any step's exception is re-raised."""
    import threading
    F = len(steps_of)
    errs = []

    def worker(k):
        try:
            for i in range(k, steps, F):
                steps_of[k](i)
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            errs.append(e)

    barrier()
    t0 = time.perf_counter()
    ths = [threading.Thread(target=worker, args=(k,)) for k in range(F)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    barrier()
    dt = time.perf_counter() - t0
    if errs:
        raise errs[0]
    return dt


def run_queue(workers: "list[Callable[[int], None]]", items: Sequence[int]) -> None:
    """One pass over `items`: len(workers) host threads (one library context
    each) take the next item in the given order -- longest chromosome first --
    until none is left (greedy list scheduling).  Any exception is re-raised
    after every thread has stopped."""
    import threading
    lock = threading.Lock()
    nxt = [0]
    errs = []

    def loop(k):
        try:
            while True:
                with lock:
                    if errs or nxt[0] >= len(items):
                        return
                    i = items[nxt[0]]
                    nxt[0] += 1
                workers[k](i)
        except BaseException as e:  # noqa: BLE001 -- re-raised below
            with lock:
                errs.append(e)

    ths = [threading.Thread(target=loop, args=(k,)) for k in range(len(workers))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    if errs:
        raise errs[0]


def sharded_genome_text(scan_chrom: "Callable[[int], object]", lengths: Sequence[int], world: int, rank: int,
                        gather: "Callable[[dict], list] | None" = None, ctx_post: "Callable[[str], str] | None" = None):
    """The genome's output text with its chromosomes scanned across ranks:
    rank r scans its longest-processing-time share (assign_chromosomes), the
    per-chromosome texts are gathered on rank 0 (the only exchange, off the
    scan path) and joined in chromosome order -- the order a one-rank run, and
    GROM's serial loop over the FASTA, writes them.  Returns the text on rank
    0, None elsewhere.  `gather(obj)` returns every rank's obj on rank 0
    (torch.distributed.gather_object); None means a single rank.

    When scan_chrom returns (vcf, raw_ctx) pairs, rank 0 also joins the raw
    CTX rows in chromosome order and returns (vcf, ctx_post(raw)) -- the
    translocation post-pass over the whole genome's CTX rows."""
    mine = assign_chromosomes(lengths, world)[rank] if world > 1 else list(range(len(lengths)))
    texts = {i: scan_chrom(i) for i in mine}
    parts = [texts] if gather is None else gather(texts)
    if rank != 0:
        return None
    merged = {}
    for d in parts:
        for i, t in d.items():
            if i in merged:
                raise RuntimeError(f"chromosome {i} scanned by two ranks")
            merged[i] = t
    missing = [i for i in range(len(lengths)) if i not in merged]
    if missing:
        raise RuntimeError(f"chromosomes {missing} scanned by no rank")
    vals = [merged[i] for i in range(len(lengths))]
    if vals and isinstance(vals[0], tuple):
        vcf = "".join(v[0] for v in vals)
        raw = "".join(v[1] for v in vals)
        return vcf, (ctx_post(raw) if ctx_post else raw)
    return "".join(vals)


def gather_to_rank0(obj):
    """torch.distributed.gather_object onto rank 0 (gloo or RCCL)."""
    import torch.distributed as dist
    out = [None] * dist.get_world_size() if dist.get_rank() == 0 else None
    dist.gather_object(obj, out, dst=0)
    return out


def max_over_ranks(value: float, device=None) -> float:
    """Max of `value` over all ranks (identity without a process group)."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def merge_rank_outputs(vcf_paths: Sequence[str], raw_ctx_paths: Sequence[str], chrom_order: Sequence[str],
                       target_names: Sequence[str], insert_max: int, lseq: int):
    """Join several ranks' drop-in CLI runs over disjoint chromosome shares
    (GROM_CHROMS, each with GROM_CTX_RAW) into one run's output: the VCF
    header of the first file, every chromosome's rows in `chrom_order` (the
    order a one-process run writes them: GROM's loop over the BAM targets),
    and the translocation post-pass (grom_ctx_postpass, GROM.c:22400-22770)
    over all ranks' raw CTX rows in the same order.  Rows are grouped by their
    chromosome column (VCF column 1, raw CTX column 2).  Returns
    (vcf_text, bnd_rows)."""
    from . import ctx_postpass
    header, rows, raw = [], {}, {}
    for k, path in enumerate(vcf_paths):
        with open(path) as f:
            for line in f:
                if line.startswith("#"):
                    if k == 0:
                        header.append(line)
                    continue
                rows.setdefault(line.split("\t", 1)[0], []).append(line)
    for path in raw_ctx_paths:
        with open(path) as f:
            for line in f:
                raw.setdefault(line.split("\t", 2)[1], []).append(line)
    unknown = (set(rows) | set(raw)) - set(chrom_order)
    if unknown:
        raise ValueError(f"rows of chromosomes outside the plan: {sorted(unknown)[:5]}")
    vcf = "".join(header) + "".join("".join(rows.get(c, [])) for c in chrom_order)
    bnd = ctx_postpass("".join("".join(raw.get(c, [])) for c in chrom_order), list(target_names), insert_max, lseq)
    return vcf, bnd
