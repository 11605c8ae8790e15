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


def vcf_segments(data: bytes, chroms: Sequence[str]):
    """One rank's VCF as bytes: (end of its header, {chromosome: (start,
    end)}) for the chromosomes of `chroms` (in the file's order) that have
    rows.  The CLI writes a chromosome's rows together; that is checked here:
    no row of a chromosome lies outside its segment."""
    pos = 0
    while pos < len(data) and data[pos:pos + 1] == b"#":
        nl = data.find(b"\n", pos)
        pos = len(data) if nl < 0 else nl + 1
    hdr_end = pos
    starts = []
    for c in chroms:
        key = b"\n" + c.encode() + b"\t"
        if data.startswith(key[1:], hdr_end):
            starts.append((hdr_end, c))
        else:
            k = data.find(key, max(hdr_end - 1, 0))
            if k >= 0:
                starts.append((k + 1, c))
    starts.sort()
    segs = {}
    for j, (s, c) in enumerate(starts):
        e = starts[j + 1][0] if j + 1 < len(starts) else len(data)
        key = b"\n" + c.encode() + b"\t"
        if data.find(key, max(hdr_end - 1, 0), max(s - 1, 0)) >= 0 or data.find(key, max(e - 1, s)) >= 0:
            raise RuntimeError(f"rows of {c} are not contiguous in the rank's VCF")
        if s < 1 or data.count(key, s - 1, e - 1) != data.count(b"\n", s, e):
            raise RuntimeError(f"rows of other chromosomes among {c}'s in the rank's VCF")
        segs[c] = (s, e)
    rest = data[hdr_end:starts[0][0]] if starts else data[hdr_end:]
    if rest:
        raise RuntimeError("rows of chromosomes outside the rank's share")
    return hdr_end, segs


def read_vcf_segments(segs_path: str, file_size: int):
    """The CLI's GROM_VCF_SEGS index ("chromosome<TAB>offset<TAB>bytes" per
    chromosome with rows, in file order): (end of the header, {chromosome:
    (start, end)}).  The segments must tile the file after its header."""
    segs, order = {}, []
    with open(segs_path) as f:
        for line in f:
            c, o, n = line.rstrip("\n").split("\t")
            segs[c] = (int(o), int(o) + int(n))
            order.append(c)
    hdr_end = segs[order[0]][0] if order else file_size
    at = hdr_end
    for c in order:
        if segs[c][0] != at:
            raise RuntimeError(f"{segs_path}: the segment of {c} does not follow the one before")
        at = segs[c][1]
    if at != file_size:
        raise RuntimeError(f"{segs_path}: the segments end at {at}, the file at {file_size}")
    return hdr_end, segs


def merge_rank_outputs_parallel(rank: int, vcf_path: str, chroms_mine: Sequence[str], chrom_order: Sequence[str],
                                out_vcf: str, all_gather: "Callable[[object], list]", barrier: Callable[[], None],
                                raw_ctx_paths: Sequence[str] = (), target_names: Sequence[str] = (),
                                insert_max: int = 0, lseq: int = 0, out_ctx: "str | None" = None,
                                segs_path: "str | None" = None):
    """merge_rank_outputs with every rank writing its own rows: each rank
    knows its chromosomes' row segments in its VCF (the CLI's GROM_VCF_SEGS
    index, or vcf_segments over the file's bytes), the ranks exchange the
    segment sizes (all_gather, a few integers per rank), rank 0 writes the
    header and sizes the output file, and every rank copies its segments to
    their offsets in chromosome order (copy_file_range into the one file on
    the node).  Rank 0 then runs the translocation post-pass over all ranks'
    raw CTX rows (a few hundred rows) into out_ctx.  Same bytes as
    merge_rank_outputs; rank 0 no longer reads and re-joins the genome's
    ~440 MB of rows alone (4.4 s in Python)."""
    import os

    def agree(ok_err, payload=None):
        """all_gather of (rank, error or None, payload): a rank that failed makes
        every rank raise at once (a rank that raised alone would leave the
        others waiting in the next collective until its timeout)."""
        got = all_gather((rank, ok_err, payload))
        bad = [(r, e) for r, e, _ in got if e is not None]
        if bad:
            raise RuntimeError("merge failed on rank(s) " + "; ".join(f"{r}: {e}" for r, e in bad))
        return got

    hdr_end, segs, err = 0, {}, None
    try:
        size = os.path.getsize(vcf_path)
        if segs_path is not None:
            hdr_end, segs = read_vcf_segments(segs_path, size)
            missing = set(segs) - set(chroms_mine)
            if missing:
                raise RuntimeError(f"rows of chromosomes outside the rank's share: {sorted(missing)[:5]}")
        else:
            with open(vcf_path, "rb") as f:
                hdr_end, segs = vcf_segments(f.read(), chroms_mine)
    except (OSError, RuntimeError, ValueError) as e:
        err = f"{type(e).__name__}: {e}"
    info = agree(err, (hdr_end, {c: e - s for c, (s, e) in segs.items()}))
    hdr_len, sizes = 0, {}
    for r, _, (h, d) in info:
        if r == 0:
            hdr_len = h
        for c, n in d.items():
            if c in sizes:
                raise RuntimeError(f"chromosome {c} written by two ranks")
            sizes[c] = n
    unknown = set(sizes) - set(chrom_order)
    if unknown:
        raise ValueError(f"rows of chromosomes outside the plan: {sorted(unknown)[:5]}")
    off, base = {}, hdr_len
    for c in chrom_order:
        off[c] = base
        base += sizes.get(c, 0)
    err = None
    try:
        if rank == 0:
            with open(out_vcf, "wb") as f, open(vcf_path, "rb") as g:
                f.write(g.read(hdr_end))
                f.truncate(base)
    except OSError as e:
        err = f"OSError: {e}"
    agree(err)
    err = None
    try:
        src = os.open(vcf_path, os.O_RDONLY)
        try:
            dst = os.open(out_vcf, os.O_WRONLY)
            try:
                for c, (s, e) in segs.items():
                    done = 0
                    while done < e - s:
                        k = os.copy_file_range(src, dst, e - s - done, s + done, off[c] + done)
                        if k <= 0:
                            raise OSError(f"copy_file_range returned {k}")
                        done += k
            finally:
                os.close(dst)
        finally:
            os.close(src)
    except OSError as e:
        err = f"OSError: {e}"
    agree(err)
    if rank == 0 and out_ctx is not None:
        from . import ctx_postpass
        raw = {}
        for path in raw_ctx_paths:
            with open(path) as f:
                for line in f:
                    raw.setdefault(line.split("\t", 2)[1], []).append(line)
        bnd = ctx_postpass("".join("".join(raw.get(c, [])) for c in chrom_order), list(target_names), insert_max, lseq)
        with open(out_ctx, "w") as f:
            f.write(bnd)


def all_gather_objects(obj):
    """torch.distributed.all_gather_object (gloo or RCCL)."""
    import torch.distributed as dist
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out
