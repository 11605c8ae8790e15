"""bench.py -- GROM's per-chromosome scan on MI355X, whole genome, whole run.

Metric (BASELINE.json): "Mbases/sec scanned (whole genome)" -- SURVEY 8(d):
genome bases / wall time of the whole run, BAM in, VCF out.

Default workload (BASELINE.json configs[2]): a synthetic 30x 2x150 bp
paired-end human-shape genome -- the 24 GRCh38 contig lengths (3.09 Gb), SNVs
and indels, breakpoint SVs (DEL/DUP/INV/INS and CTX, with split reads and
discordant pairs), copy-number regions, 5% PCR duplicates -- written once as
a BAM + BAI + FASTA by grom_synth, and scanned with `-M -g 1` (the male
genome: chrY is processed too, so all 24 contigs are scanned).

One step = one whole run of the drop-in CLI (grom_amd/bin/grom) as a fresh
process: BAM index, each chromosome's compressed BGZF run read ahead into
pinned memory and copied to HBM, inflated and parsed on the GPU piece by
piece (ddecode.hip; the insert statistics from the first run's pieces),
every chromosome's scan (pileup/SNV, duplicate filter, breakpoint evidence
and tests, SV/INDEL rows, CTX records, read-depth CNV path and rows), the VCF
and the translocation post-pass (.ctx.vcf).  The BAM sits in the page cache
(the first warmup run reads it from disk).
value = genome bases * steps / (time of the steps).

--gpus N (torch.distributed.run, one rank per GPU): the chromosomes are
assigned longest-processing-time-first to ranks (configs[3]); each rank runs
its own CLI process on its GPU over its share (GROM_CHROMS: the serial
stream's plan is kept, so each chromosome gets exactly a one-process run's
input; the insert statistics come from <bam>.mean, which a plan-only run of
rank 0 writes first, as the reference's -c children load it);
after a barrier rank 0 joins the shares in chromosome order and runs the
translocation post-pass over all raw CTX rows (grom_amd.shard.merge_rank_outputs)
-- inside the timed step.  The step time is the max over ranks.  There is no
data-path collective: chromosomes are independent.

The JSON line also carries:
  identical_to_oracle_full_scale  every timed run's VCF and .ctx.vcf rows
                  against the oracle's on the same full-scale genome (sha256
                  of the non-header rows, tests/golden/oracle_genome_s100.json;
                  each step writes its own files, hashed after the timed
                  region: oracle_full_scale.identical_runs "k/K");
  footprint_rank0 the run's peak device memory (the CLI's footprint line);
and (rank 0, N=1):
  roofline        the pileup kernel (k_scan_tile) in the timed whole runs:
                  algorithmic bytes of every launch (read records, CIGAR,
                  packed bases + qualities, reference, caf arrays)
                  / the launches' HIP-event durations, against 8 TB/s HBM;
                  SURVEY 8(d)'s 158.8 B/base model beside it; PMC traffic from
                  profiles/pmc_genome_30x.json;
  device_resident the same genome generated on the host (grom_synth_chrom_stream:
                  each chromosome as the BAM's serial stream hands it to its
                  scan) and kept in HBM, scanned with two chromosomes in flight:
                  the device-only throughput, and its rows compared with the
                  whole run's VCF and .ctx.vcf (decode + staging checked at
                  full scale); skipped when --budget-s would be exceeded;
  cpu_baseline    the CPU restatement of the reference (oracle/, "port"), one
                  thread, on a bounded 3-contig 6 Mb sample of the same
                  generator and flags;
  concordance     the GPU CLI on that sample against the oracle, byte for byte.
"""
import argparse
import ctypes
import hashlib
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile
import threading
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak (spec)
SURVEY_BYTES_PER_BASE = 158.8  # SURVEY.md 8(d), pileup kernel at 30x, 2x150
READ_LEN = 150
CPU_SAMPLE_LENS = (3_000_000, 2_000_000, 1_000_000)  # the bounded cpu_baseline / concordance sample: 3 contigs
PILEUP_KERNEL = "k_scan_tile"
FILEDATE, SEED = "20260101", "7"

GRCH38 = [("chr1", 248956422), ("chr2", 242193529), ("chr3", 198295559), ("chr4", 190214555),
          ("chr5", 181538259), ("chr6", 170805979), ("chr7", 159345973), ("chr8", 145138636),
          ("chr9", 138394717), ("chr10", 133797422), ("chr11", 135086622), ("chr12", 133275309),
          ("chr13", 114364328), ("chr14", 107043718), ("chr15", 101991189), ("chr16", 90338345),
          ("chr17", 83257441), ("chr18", 80373285), ("chr19", 58617616), ("chr20", 64444167),
          ("chr21", 46709983), ("chr22", 50818468), ("chrX", 156040895), ("chrY", 57227415)]

# 2,000 DEL/DUP/INV/INS + 200 CTX, 500 CNVs of 10 kb-1 Mb,
# 5% PCR duplicates, seed 3, run with -M (and -g 1: every contig processed)
C3 = dict(coverage=30.0, dup_frac=0.05, sv_per_mb=2200 / 3088.3, cnv_rate=500 / 3.0883e9,
          cnv_range=(10_000, 1_000_000), seed=3)
C2 = dict(coverage=30.0, dup_frac=0.0, sv_per_mb=0.0, cnv_rate=0.0, cnv_range=(0, 0), seed=2)
GENOME_FLAGS = ["-M", "-g", "1"]

FOOTPRINT = re.compile(r"^footprint: peak ([\d.]+) GB of device memory \(([^)]*)\).*buffers: peak ([\d.]+) GB together.*"
                       r"; (\d+) allocations waited ([\d.]+) s(?:.*; (\d+) slow hipMalloc calls ([\d.]+) s)?")
ORACLE_FULL = os.path.join(REPO, "tests", "golden", "oracle_genome_s100.json")
CHROM_LINE = re.compile(r"^(\S+): (\d+) reads, ([\d.]+) ms on GPU .*; pileup ([\d.]+) ms, cnv ([\d.]+) ms, "
                        r"cigar_ops (\d+), bases (\d+), len (\d+)$")


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def cpu_quota() -> int:
    """CPUs this container may use: the cgroup quota (cpu.max) if any, else the online CPUs."""
    n = os.cpu_count() or 1
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max" and int(period) > 0:
            n = min(n, max(1, -(-int(q) // int(period))))
    except (OSError, ValueError):
        pass
    return n


def launch_bytes(reads, cigar_ops, bases, chrom_len) -> int:
    """Bytes the pileup kernel must move once per launch: every read record it
    ingests (SoA metadata, CIGAR, packed bases, qualities), the reference and
    the three whole-chromosome read-depth arrays it writes."""
    per_read = 4 + 2 + 1 + 4 + 4 + 4 + 4 + 4 + 8 + 4  # pos flag mapq mtid mpos isize lqseq cig_off base_off name
    return reads * per_read + cigar_ops * 4 + bases // 2 + bases + chrom_len * (1 + 3 * 4)


def synth_args(knobs, lengths):
    a = ["-L", ",".join(str(x) for x in lengths), "-s", str(knobs["seed"]), "-c", str(knobs["coverage"]),
         "-l", str(READ_LEN)]
    if knobs["dup_frac"]:
        a += ["-D", str(knobs["dup_frac"])]
    if knobs["sv_per_mb"]:
        a += ["-X", str(knobs["sv_per_mb"])]
    if knobs["cnv_rate"]:
        a += ["-V", str(knobs["cnv_rate"]), "-W", "%d,%d" % knobs["cnv_range"]]
    return a


def run_heartbeat(cmd, what, timeout, **kw):
    """Run a long child with a progress line every 30 s (silent runs look hung)."""
    t0 = time.perf_counter()
    p = subprocess.Popen(cmd, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, **kw)
    while True:
        try:
            out, err = p.communicate(timeout=30)
            break
        except subprocess.TimeoutExpired:
            if time.perf_counter() - t0 > timeout:
                p.kill()
                p.communicate()
                raise RuntimeError(f"{what}: timed out after {timeout} s")
            log(f"{what}: {time.perf_counter() - t0:.0f} s")
    if p.returncode != 0:
        raise RuntimeError(f"{what} failed ({p.returncode}): {out[-2000:]} {err[-2000:]}")
    return out, time.perf_counter() - t0


def write_genome(work, knobs, lengths, names):
    from grom_amd import SYNTH_BIN
    prefix = os.path.join(work, "genome")
    _, dt = run_heartbeat([SYNTH_BIN, "-o", prefix] + synth_args(knobs, lengths) + ["-n", ",".join(names)],
                          "grom_synth", 1500)
    bam = prefix + ".bam"
    log(f"genome BAM written: {sum(lengths) / 1e9:.3f} Gb, {os.path.getsize(bam) / 1e9:.2f} GB in {dt:.1f} s")
    return bam, prefix + ".fa", dt


def cli_env(extra=None):
    e = dict(os.environ, GROM_FILEDATE=FILEDATE, GROM_SEED=SEED, GROM_VERBOSE="1")
    e.update(extra or {})
    return e


def whole_run(work, bam, fa, out, flags, env_extra=None, timeout=900):
    """The drop-in CLI as a fresh process; (seconds, stdout)."""
    from grom_amd import GROM_BIN
    t0 = time.perf_counter()
    r = subprocess.run([GROM_BIN, "-i", bam, "-r", fa, "-o", out] + flags, cwd=work, env=cli_env(env_extra),
                       capture_output=True, text=True, timeout=timeout)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError(f"grom failed ({r.returncode}): {r.stdout[-3000:]} {r.stderr[-3000:]}")
    slow = [ln for ln in r.stderr.splitlines() if ln.startswith("grom:") and " took " in ln]
    if slow:
        log(f"{len(slow)} slow device allocations in the run: " + "; ".join(ln[6:] for ln in slow[:12]))
    return dt, r.stdout


def chrom_stats(stdout):
    out = {}
    for line in stdout.splitlines():
        m = CHROM_LINE.match(line)
        if m:
            out[m.group(1)] = dict(reads=int(m.group(2)), ms_total=float(m.group(3)), ms_pileup=float(m.group(4)),
                                   ms_cnv=float(m.group(5)), cigar_ops=int(m.group(6)), bases=int(m.group(7)),
                                   len=int(m.group(8)))
    return out


def footprint(stdout):
    """the CLI's footprint line (GROM_VERBOSE): peak device memory of the run"""
    for line in stdout.splitlines():
        m = FOOTPRINT.match(line)
        if m:
            return {"peak_gb": float(m.group(1)), "measured_as": m.group(2), "buffers_peak_gb": float(m.group(3)),
                    "allocations_waited": int(m.group(4)), "wait_s": float(m.group(5)),
                    "slow_hipmalloc": int(m.group(6) or 0), "slow_hipmalloc_s": float(m.group(7) or 0.0)}
    return None


def oracle_full_scale(vcf, ctx):
    """The timed whole run's rows against the oracle's at the same full-scale
    workload (tests/golden/oracle_genome_s100.json, tools/make_golden_genome.py:
    the oracle, one thread, about three hours in the build container)."""
    if not os.path.exists(ORACLE_FULL):
        return None
    g = json.load(open(ORACLE_FULL))
    nv, dv = rows_digest(vcf)
    nc, dc = rows_digest(ctx)
    return {"identical": (nv, dv, nc, dc) == (g["vcf_rows"], g["vcf_rows_sha256"], g["ctx_rows"], g["ctx_rows_sha256"]),
            "vcf_rows": nv, "ctx_rows": nc, "oracle_vcf_rows": g["vcf_rows"], "oracle_ctx_rows": g["ctx_rows"],
            "oracle_seconds": g.get("oracle_seconds"), "golden": os.path.relpath(ORACLE_FULL, REPO)}


def rows_digest(path):
    """(rows, sha256) of a VCF's non-header lines."""
    h, n = hashlib.sha256(), 0
    with open(path, "rb") as f:
        for line in f:
            if not line.startswith(b"#"):
                h.update(line)
                n += 1
    return n, h.hexdigest()


def inflate_roofline(dec_line):
    """The GPU BGZF inflater (k_inflate, the largest event time of a whole
    run) beside the pileup's roofline: algorithmic bytes = the compressed
    bytes read + the inflated bytes written, over the CLI's summed HIP-event
    time of the inflate launches (the decode line of the last timed run)."""
    if not dec_line or not dec_line.startswith("device decode"):
        return None
    m = re.search(r"([\d.]+) GB compressed.*?([\d.]+) GB inflated.*?GPU inflate ([\d.]+) s", dec_line)
    if not m:
        return None
    comp, infl, sec = float(m.group(1)), float(m.group(2)), float(m.group(3))
    if sec <= 0:
        return None
    achieved = (comp + infl) / sec
    return {"bound": "hbm", "kernel": "k_inflate", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
            "bytes_model": "compressed bytes read + inflated bytes written per genome (DESIGN.md 4.5)",
            "event_s": sec, "gb_in": comp, "gb_out": infl,
            "note": "latency-bound (one DEFLATE block per lane, each match an L2 round trip); its launches "
                    "share the chip with the scans"}


def roofline_of(per_launch, alone=None):
    """per_launch: [(bytes, ms, chrom_len)] of the pileup kernel's launches."""
    byt = sum(b for b, _, _ in per_launch)
    sec = sum(ms for _, ms, _ in per_launch) / 1e3
    bases = sum(L for _, _, L in per_launch)
    achieved = byt / sec / 1e9
    survey = SURVEY_BYTES_PER_BASE * bases / sec / 1e9
    traffic = None
    pmc = os.path.join(REPO, "profiles", "pmc_genome_30x.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get(f"{PILEUP_KERNEL}_hbm_bytes_per_launch")
        except (OSError, ValueError):
            traffic = None
    r = {"bound": "hbm", "kernel": PILEUP_KERNEL, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
         "bytes_model": "this build (DESIGN.md 7): read records + CIGAR + 1.5 B per read base + 13 B per reference "
                        "base, summed over the timed launches (HIP events on the scan stream)",
         "launches": len(per_launch), "launch_ms_mean": round(sec * 1e3 / max(len(per_launch), 1), 3),
         "bytes_per_100mb": round(byt / bases * 1e8), "survey_bytes_per_base": SURVEY_BYTES_PER_BASE,
         "survey_achieved": round(survey, 1), "survey_frac": round(survey / HBM_PEAK_GBS, 4)}
    if alone:
        r["alone"] = alone
    return r


def cpu_baseline_and_concordance(work_dir, knobs, flags):
    """The oracle (CPU port of GROM's scan, one thread) on a bounded 3-contig
    sample of the workload's generator, whole run (BAM decode + scan + VCF);
    then the GPU CLI on the same files, compared byte for byte."""
    from grom_amd import cli_main, last_error, run_synth
    total = sum(CPU_SAMPLE_LENS)
    sample = f"{len(CPU_SAMPLE_LENS)} contigs, {total / 1e6:g} Mb"
    bam, fa = run_synth(os.path.join(work_dir, "sample"), *synth_args(knobs, CPU_SAMPLE_LENS))
    env = dict(os.environ, GROM_FILEDATE=FILEDATE, GROM_SEED=SEED)
    oracle = os.path.join(REPO, "oracle", "grom_oracle")
    t0 = time.perf_counter()
    r = subprocess.run([oracle, "-i", bam, "-r", fa, "-o", "cpu.vcf"] + flags, cwd=work_dir, env=env,
                       capture_output=True, text=True, timeout=900)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError("oracle failed: " + r.stderr[-2000:])
    cpu = {"value": round(total / dt / 1e6, 4), "unit": "Mbases/s", "cores": 1, "kind": "port",
           "sample": f"{sample} synthetic genome of the bench generator "
                     f"(grom_synth {' '.join(synth_args(knobs, CPU_SAMPLE_LENS))}), flags {' '.join(flags) or '-'}; "
                     f"whole oracle run (BAM decode + scan + VCF) in {dt:.2f} s, 1 thread"}
    t0 = time.perf_counter()
    # (the in-process CLI prints its report on fd 1: sent to stderr, so that
    # stdout holds only the bench's one JSON line)
    sys.stdout.flush()
    saved_fd = os.dup(1)
    os.dup2(2, 1)
    try:
        rc = cli_main(["-i", bam, "-r", fa, "-o", "gpu.vcf"] + flags,
                      env={"GROM_FILEDATE": FILEDATE, "GROM_SEED": SEED}, cwd=work_dir)
    finally:
        ctypes.CDLL(None).fflush(None)
        os.dup2(saved_fd, 1)
        os.close(saved_fd)
    dt_gpu = time.perf_counter() - t0
    if rc != 0:
        raise RuntimeError(f"GPU CLI failed on the concordance sample: {last_error()}")
    same = all(open(os.path.join(work_dir, "gpu" + ext), "rb").read() ==
               open(os.path.join(work_dir, "cpu" + ext), "rb").read() for ext in (".vcf", ".ctx.vcf"))
    rows = sum(1 for ln in open(os.path.join(work_dir, "gpu.vcf")) if not ln.startswith("#"))
    conc = {"sample": f"the cpu_baseline sample ({sample}) through the GPU CLI (grom_cli_main)",
            "vcf_rows": rows, "identical_to_oracle": same,
            "cli_end_to_end_s": round(dt_gpu, 2), "cli_end_to_end_mbases_per_s": round(total / dt_gpu / 1e6, 2)}
    return cpu, conc


def resident_leg(local, knobs, lengths, names, bam, whole_vcf, steps, inflight):
    """The genome generated on the host as the BAM's serial stream hands each
    chromosome to its scan (grom_synth_chrom_stream), kept in HBM, scanned
    with `inflight` chromosomes in flight; device-only Mbases/s, the pileup
    kernel alone on the largest chromosome, and the rows against the whole
    run's VCF / .ctx.vcf."""
    import grom_amd
    from grom_amd.shard import run_queue
    imean, lseq, imin, imax = (int(x) for x in open(bam + ".mean").read().split()[:4])
    params = grom_amd.default_params()
    params.rmdup, params.gender = 1, 1
    grom_amd.lib().grom_params_set_insert(ctypes.byref(params), imean, imin, imax, lseq)
    order = sorted(range(len(lengths)), key=lambda i: (-lengths[i], i))  # longest first, as GROM.c:22318-22336
    res, info = {}, {}
    lock = threading.Lock()
    t_gen = time.perf_counter()

    def make(i):
        b = grom_amd.SynthBatch.genome_chrom(lengths, i, params, names=names, coverage=knobs["coverage"],
                                             read_len=READ_LEN, dup_frac=knobs["dup_frac"],
                                             sv_per_mb=knobs["sv_per_mb"], cnv_rate=knobs["cnv_rate"],
                                             cnv_range=knobs["cnv_range"], seed=knobs["seed"], stream=True)
        try:
            r = grom_amd.Resident(local, b.chrom, b.reads)
            r.chrom.seed = int(SEED)  # what the CLI's scans get (GROM_SEED)
            with lock:
                res[i] = r
                info[i] = {"bytes": launch_bytes(b.reads.n, b.reads.n_cigar_ops, b.reads.n_bases, lengths[i]),
                           "resident_bytes": r.bytes}
        finally:
            b.close()

    run_queue([make] * max(1, min(cpu_quota(), 16, len(order))), order)
    t_gen = time.perf_counter() - t_gen
    log(f"resident genome generated in {t_gen:.1f} s ({sum(v['resident_bytes'] for v in info.values()) / 1e9:.1f} GB)")
    devs = [grom_amd.Device(local, params, slot=local + 8 * k) for k in range(inflight)]
    texts, rec = {}, []
    try:
        def scanner(k, record):
            def scan(i):
                vcf, ctx, st = devs[k].scan_rows(res[i].chrom, res[i].reads, device_resident=True)
                with lock:
                    if record is None:
                        texts[i] = (vcf, ctx)
                    else:
                        record.append((i, st.ms_pileup))
            return scan
        run_queue([scanner(k, None) for k in range(inflight)], order)  # warm pass; keeps the rows
        _, st_alone = devs[0].scan(res[order[0]].chrom, res[order[0]].reads, device_resident=True)
        t0 = time.perf_counter()
        for _ in range(steps):
            run_queue([scanner(k, rec) for k in range(inflight)], order)
        dt = time.perf_counter() - t0
    finally:
        for d in reversed(devs):
            d.close()
        for r in res.values():
            r.close()
    # rows: the resident pass against the whole run
    vcf = "".join(texts[i][0] for i in range(len(lengths)))
    bnd = grom_amd.ctx_postpass("".join(texts[i][1] for i in range(len(lengths))), names, params.insert_max_size,
                                params.lseq)
    n_whole, d_whole = rows_digest(whole_vcf)
    n_ctx, d_ctx = rows_digest(whole_vcf[:-4] + ".ctx.vcf")
    same_vcf = (vcf.count("\n"), hashlib.sha256(vcf.encode()).hexdigest()) == (n_whole, d_whole)
    same_ctx = (bnd.count("\n"), hashlib.sha256(bnd.encode()).hexdigest()) == (n_ctx, d_ctx)
    big = order[0]
    alone_ach = info[big]["bytes"] / (st_alone.ms_pileup / 1e3) / 1e9
    out = {"value": round(sum(lengths) * steps / dt / 1e6, 1), "unit": "Mbases/s", "passes": steps,
           "ms_per_pass": round(dt / steps * 1e3, 1), "scans_in_flight": inflight,
           "host_generate_s": round(t_gen, 1),
           "hbm_resident_gb": round(sum(v["resident_bytes"] for v in info.values()) / 1e9, 1),
           "rows_identical_to_whole_run": same_vcf, "ctx_identical_to_whole_run": same_ctx,
           "vcf_rows": n_whole, "bnd_rows": n_ctx,
           "note": "inputs already in HBM when the pass starts (no BAM decode, no host->device copies); the rows "
                   "are compared with the timed whole run's VCF and .ctx.vcf (sha256 of the rows)"}
    alone = {"chrom": names[big], "launch_ms": round(st_alone.ms_pileup, 3), "achieved": round(alone_ach, 1),
             "frac": round(alone_ach / HBM_PEAK_GBS, 4),
             "survey_frac": round(SURVEY_BYTES_PER_BASE * lengths[big] / (st_alone.ms_pileup / 1e3) / 1e9
                                  / HBM_PEAK_GBS, 4)}
    launches = [(info[i]["bytes"], ms, lengths[i]) for i, ms in rec]
    return out, alone, launches


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["genome", "chrom"], default="genome",
                    help="genome: configs[2]/[3] human-shape 3.09 Gb genome; chrom: configs[1] 100 Mb chromosome")
    ap.add_argument("--scale", type=float, default=1.0, help="scale every contig length (tests / quick runs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-resident", action="store_true", help="skip the device-resident leg")
    ap.add_argument("--resident-steps", type=int, default=2)
    ap.add_argument("--inflight", type=int, default=2, help="resident leg: chromosome scans in flight per GPU")
    ap.add_argument("--budget-s", type=float, default=540.0,
                    help="skip the resident leg when it would end the run after this many seconds")
    ap.add_argument("--workdir", default="", help="keep the BAM here (default: a temporary directory)")
    args = ap.parse_args()
    t_start = time.perf_counter()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # GROM_BENCH_ONE_GPU=1 (a rehearsal of the multi-rank path on a one-GPU
    # box): every rank runs its CLI on GPU 0 and the ranks talk over gloo
    # (RCCL refuses two ranks on one GPU)
    one_gpu = os.environ.get("GROM_BENCH_ONE_GPU") == "1"
    if one_gpu:
        local = 0
    if world > 1:
        torch.cuda.set_device(local)
        if one_gpu:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import grom_amd
    from grom_amd.shard import all_gather_objects, assign_chromosomes, max_over_ranks, merge_rank_outputs_parallel

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    genome = args.workload == "genome"
    if genome:
        knobs, flags = C3, list(GENOME_FLAGS)
        names = [n for n, _ in GRCH38]
        lengths = [max(int(L * args.scale), 1_000_000) for _, L in GRCH38]
    else:
        knobs, flags = C2, []
        names = ["chr1"]
        lengths = [max(int(100_000_000 * args.scale), 1_000_000)]
    total = sum(lengths)
    shares = assign_chromosomes(lengths, world)
    mine = shares[rank]

    # one shared directory on this node (rank 0 writes the BAM)
    work = args.workdir or os.path.join(tempfile.gettempdir(), f"grom_bench_{os.environ.get('MASTER_PORT', 'solo')}")
    if rank == 0:
        shutil.rmtree(work, ignore_errors=True)
        os.makedirs(work, exist_ok=True)
        bam, fa, t_synth = write_genome(work, knobs, lengths, names)
    barrier()
    bam, fa = os.path.join(work, "genome.bam"), os.path.join(work, "genome.fa")

    # the rank's CLI: its chromosomes, its GPU, its share of the CPUs.  The
    # CLI sees only its own GPU (HIP_VISIBLE_DEVICES): a process that could
    # see all eight would initialise the HIP runtime over all of them, a fixed
    # cost every rank pays inside the timed step
    cpus = cpu_quota()
    vis = os.environ.get("HIP_VISIBLE_DEVICES") or os.environ.get("CUDA_VISIBLE_DEVICES")
    vis_list = [v for v in vis.split(",") if v.strip()] if vis else []
    env = {"GROM_DEVICE": "0", "HIP_VISIBLE_DEVICES": vis_list[local] if local < len(vis_list) else str(local)}
    if world > 1:
        env.update(GROM_CHROMS=",".join(names[i].lower() for i in mine),
                   GROM_DECODE_THREADS=str(max(1, cpus // world)),
                   GROM_CTX_RAW=os.path.join(work, f"rank{rank}.ctxraw"),
                   GROM_VCF_SEGS=os.path.join(work, f"rank{rank}.segs"))
    hdr_names = names  # BAM target names (the CTX post-pass maps mate ids to them)

    def outs(k):
        """step k's output files (each timed step keeps its own, so every
        step's rows are compared with the oracle after the timed region)"""
        return os.path.join(work, f"rank{rank}_s{k}.vcf"), os.path.join(work, f"merged_s{k}.vcf")

    def step(k):
        out, merged = outs(k)
        dt, so = whole_run(work, bam, fa, out, flags, env)
        if world > 1:
            # every rank copies its own chromosomes' rows into the merged VCF
            # at their offsets (the CLI's segment index, an all-gather of the
            # segment sizes); rank 0 adds the header and the CTX post-pass
            barrier()
            m = open(bam + ".mean").read().split()  # insert mean, lseq, min, max (save_insert_mean)
            merge_rank_outputs_parallel(rank, out, [names[i].lower() for i in mine], [n.lower() for n in names],
                                        merged, all_gather_objects, barrier,
                                        [os.path.join(work, f"rank{r}.ctxraw") for r in range(world)], hdr_names,
                                        int(m[3]), int(m[1]), merged[:-4] + ".ctx.vcf",
                                        segs_path=os.path.join(work, f"rank{rank}.segs"))
        return dt, so

    def drop(k):
        for p in outs(k):
            for q in (p, p[:-4] + ".ctx.vcf"):
                if os.path.exists(q):
                    os.remove(q)

    if world > 1 and rank == 0:
        # the side files every rank's CLI reads (<bam>.mean, <fasta>.info) are
        # written once here, before the ranks run concurrently (a plan-only run
        # over no chromosome: the insert-statistics head of the file only)
        whole_run(work, bam, fa, os.path.join(work, "prewarm.vcf"), flags, {"GROM_PLAN_ONLY": "1", "GROM_CHROMS": "-"})
    barrier()
    for w in range(args.warmup):
        dt, _ = step(-1 - w)
        drop(-1 - w)
        log(f"warmup run {w + 1}: {dt:.2f} s")
    barrier()
    t0 = time.perf_counter()
    runs, last, run_out = [], "", []
    for k in range(args.steps):
        t1 = time.perf_counter()
        _, last = step(k)
        runs.append(time.perf_counter() - t1)
        run_out.append(last)
        ph = [ln[len("cli phases (s from start): "):] for ln in last.splitlines() if ln.startswith("cli phases")]
        rd = re.search(r"file reads ([\d.]+) s \(read ahead; waited for ([\d.]+) s\)", last)
        log(f"timed run {k + 1}: {runs[-1]:.2f} s" + (f"; {ph[0]}" if ph else "") +
            (f"; file reads {rd.group(1)} s, waited {rd.group(2)} s" if rd else ""))
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0, device="cpu" if one_gpu else "cuda")
    value = total * args.steps / dt / 1e6
    stats = chrom_stats(last)  # this rank's chromosomes, last timed run
    feet = [footprint(so) for so in run_out]
    feet = [f for f in feet if f]
    dec = [ln for ln in last.splitlines() if ln.startswith(("streamed decode:", "device decode:"))]
    phases = [ln for ln in last.splitlines() if ln.startswith("cli phases")]

    launches = [(launch_bytes(s["reads"], s["cigar_ops"], s["bases"], s["len"]), s["ms_pileup"], s["len"])
                for s in stats.values()]
    resident, alone = None, None
    if rank == 0 and world == 1:
        remaining = args.budget_s - (time.perf_counter() - t_start)
        est = 0.55 * (t_synth if genome else 30.0) + 20.0  # host generation (no compression) + passes
        if args.no_resident:
            resident = {"skipped": "--no-resident"}
        elif est > remaining:
            resident = {"skipped": f"time budget (--budget-s {args.budget_s:g}: {remaining:.0f} s left, the leg "
                                   f"takes about {est:.0f} s)"}
        else:
            resident, alone, rl = resident_leg(local, knobs, lengths, names, bam, outs(args.steps - 1)[0], args.resident_steps,
                                               max(1, min(args.inflight, 8)))
            log(f"device-resident: {resident['value']} Mbases/s, rows identical: "
                f"{resident['rows_identical_to_whole_run']}/{resident['ctx_identical_to_whole_run']}")
    if rank == 0:
        cpu = conc = None
        if world == 1 and not args.no_cpu_baseline:
            with tempfile.TemporaryDirectory() as d:
                cpu, conc = cpu_baseline_and_concordance(d, knobs, flags)
        # every timed step's rows against the oracle's full-scale digest
        # (after the timed region; each step wrote its own files)
        final_of = [outs(k)[0] if world == 1 else outs(k)[1] for k in range(args.steps)]
        final_vcf = final_of[-1]
        n_rows, _ = rows_digest(final_vcf)
        full = None
        if genome and args.scale == 1.0:
            per = [oracle_full_scale(v, v[:-4] + ".ctx.vcf") for v in final_of]
            full = per[-1]
            if full is not None:
                full["identical_runs"] = f"{sum(1 for p in per if p and p['identical'])}/{len(per)}"
                full["identical"] = all(p and p["identical"] for p in per)
        else:
            # a reduced workload has no oracle digest: the steps' rows must at least agree with each other
            d0 = [rows_digest(v) + rows_digest(v[:-4] + ".ctx.vcf") for v in final_of]
            full_steps_agree = all(d == d0[0] for d in d0)
            log(f"timed steps' rows identical to each other: {full_steps_agree}")
        wl = ("BASELINE configs[2]: synthetic 30x 2x150 bp human-shape genome, 24 GRCh38 contigs "
              f"({total / 1e9:.3f} Gb), SNV/indel, {knobs['sv_per_mb']:.2f} breakpoint SVs/Mb "
              "(DEL/DUP/INV/INS/CTX with split reads + discordant pairs), 500 CNVs/3.1 Gb, 5% PCR duplicates, "
              "flags -M -g 1" + ("; chromosomes LPT-sharded over ranks, one CLI process per GPU (configs[3])"
                                 if world > 1 else "")
              if genome else "BASELINE configs[1]: one 100 Mb chromosome, 30x 2x150 bp, SNV/indel")
        line = {
            "metric": "Mbases/sec scanned (whole genome) + VCF concordance vs ref",
            "value": round(value, 3),
            "unit": "Mbases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded generator grom_amd/csrc/synth.c, written as BAM + BAI + FASTA by grom_synth)",
            "config": {
                "workload": wl + "; step = one whole run of the drop-in CLI (grom_amd/bin/grom, a fresh process): "
                                 "BAM index, compressed BGZF runs copied to HBM and inflated + parsed on the GPU, every "
                                 "chromosome's scan (pileup/SNV, duplicate filter, breakpoint evidence + tests, "
                                 "SV/INDEL rows, CTX records, read-depth CNV path + rows), VCF + CTX post-pass",
                "genome_bases": total, "chromosomes": len(lengths), "chromosomes_rank0": len(mine),
                "coverage": knobs["coverage"], "read_len": READ_LEN, "flags": " ".join(flags),
                "bam_bytes": os.path.getsize(bam), "synth_s": round(t_synth, 1),
                "run_s": [round(x, 3) for x in runs],
                "vcf_rows": n_rows,
                "host_cpus": cpus, "decode": "device (GPU inflate + parse)" if dec and dec[-1].startswith("device") else "host threads",
                "decode_rank0": dec[-1] if dec else None,
                "phases_rank0": phases[-1] if phases else None,
                "reads_rank0": sum(s["reads"] for s in stats.values()),
                "pileup_ms_rank0": round(sum(s["ms_pileup"] for s in stats.values()), 1),
                "cnv_ms_rank0": round(sum(s["ms_cnv"] for s in stats.values()), 1),
                "footprint_rank0": {"peak_gb_max": max(f["peak_gb"] for f in feet),
                                    "buffers_peak_gb_max": max(f["buffers_peak_gb"] for f in feet),
                                    "measured_as": feet[0]["measured_as"],
                                    "allocations_waited": sum(f["allocations_waited"] for f in feet),
                                    "wait_s": round(sum(f["wait_s"] for f in feet), 3),
                                    "slow_hipmalloc_runs": sum(1 for f in feet if f["slow_hipmalloc"]),
                                    "slow_hipmalloc_s": round(sum(f["slow_hipmalloc_s"] for f in feet), 3)}
                if feet else None,
            },
            "identical_to_oracle_full_scale": full["identical"] if full else None,
            "oracle_full_scale": full,
            "roofline": roofline_of(launches, alone) if launches else None,
            "roofline_inflate": inflate_roofline(dec[-1] if dec else None),
            "cpu_baseline": cpu,
            "concordance": conc,
            "device_resident": resident,
        }
        if full is None and not (genome and args.scale == 1.0):
            line["steps_rows_identical"] = full_steps_agree
        print(json.dumps(line), flush=True)
    barrier()
    for k in range(args.steps):
        drop(k)
    if rank == 0 and not args.workdir:
        shutil.rmtree(work, ignore_errors=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
