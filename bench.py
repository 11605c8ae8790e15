"""bench.py -- GROM per-chromosome scan on MI355X, whole genome.

Default workload (BASELINE.json configs[2]): a synthetic 30x 2x150 bp
paired-end human-shape genome -- the 24 GRCh38 contig lengths (3.09 Gb), SNVs
and indels, breakpoint SVs (DEL/DUP/INV/INS and CTX, with split reads and
discordant pairs), copy-number regions, 5% PCR duplicates -- scanned with
`-M`.  Every chromosome's reads are generated on the host (grom_synth_chrom,
the generator behind grom_synth) and kept resident in HBM (grom_resident_new);
the timed region starts with all inputs in HBM.

One step = one whole-genome pass: every chromosome through
grom_scan_chrom_device -- pileup/SNV kernels, duplicate filter, breakpoint
evidence and tests, SV assembly and rows, CTX records, the read-depth CNV path
and its rows -- with --inflight F chromosomes in flight per GPU (F library
contexts, one host thread each, longest chromosome first).  value = genome
bases / step time.

--gpus N (torch.distributed.run, one rank per GPU): the chromosomes are
assigned longest-processing-time-first to ranks (configs[3]: the same genome
sharded by chromosome, strong scaling); ranks never exchange data on the scan
path -- RCCL carries only the barrier and the max-over-ranks of the step time.
--workload chrom is configs[1] (one 100 Mb chromosome per rank, weak scaling).

The JSON line also carries
  roofline      the pileup kernel (k_scan_tile): algorithmic bytes of every
                timed launch / their summed durations (HIP events on the
                library's stream), against 8 TB/s HBM, for this build's byte
                model (`bytes_model`) and for SURVEY.md 8(d)'s 158.8 B/base,
                with PMC-measured traffic when profiles/pmc_<tag>.json exists;
  cpu_baseline  the CPU restatement of the reference (oracle/, "port"), one
                thread, on a bounded 3-contig 6 Mb sample of the same
                generator and flags (rank 0, N=1);
  concordance   the GPU CLI on that same sample's BAM/FASTA against the
                oracle's VCF and .ctx.vcf, byte for byte, with the CLI's
                end-to-end time (BAM decode and upload included);
  cli_whole_run the drop-in CLI (grom_amd/bin/grom, a fresh process) on a
                >=100 Mb 24-contig 30x BAM of the same generator (the GRCh38
                contigs scaled by --cli-scale): SURVEY 8(d)'s metric as
                defined, bases / wall time of the whole run (BAM decode on
                the host's cores, pinned pieces streamed to HBM, scans, VCF),
                with its VCF and .ctx.vcf compared byte for byte against the
                oracle run on the same files (rank 0, N=1).
"""
import argparse
import ctypes
import json
import os
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

GRCH38 = [("chr1", 248956422), ("chr2", 242193529), ("chr3", 198295559), ("chr4", 190214555),
          ("chr5", 181538259), ("chr6", 170805979), ("chr7", 159345973), ("chr8", 145138636),
          ("chr9", 138394717), ("chr10", 133797422), ("chr11", 135086622), ("chr12", 133275309),
          ("chr13", 114364328), ("chr14", 107043718), ("chr15", 101991189), ("chr16", 90338345),
          ("chr17", 83257441), ("chr18", 80373285), ("chr19", 58617616), ("chr20", 64444167),
          ("chr21", 46709983), ("chr22", 50818468), ("chrX", 156040895), ("chrY", 57227415)]

# 2,000 DEL/DUP/INV/INS + 200 CTX, 500 CNVs of 10 kb-1 Mb,
# 5% PCR duplicates, seed 3, run with -M
C3 = dict(coverage=30.0, dup_frac=0.05, sv_per_mb=2200 / 3088.3, cnv_rate=500 / 3.0883e9,
          cnv_range=(10_000, 1_000_000), seed=3)
C2 = dict(coverage=30.0, dup_frac=0.0, sv_per_mb=0.0, cnv_rate=0.0, cnv_range=(0, 0), seed=2)


def algorithmic_bytes(reads, chrom_len) -> int:
    """Bytes the pileup kernel must move once per launch: every read record it ingests
    (SoA metadata, CIGAR, packed bases, qualities), the reference, and the three
    whole-chromosome read-depth arrays it writes ('Roofline')."""
    per_read = 4 + 2 + 1 + 4 + 4 + 4 + 4 + 4 + 8 + 4  # pos flag mapq mtid mpos isize lqseq cig_off base_off name
    return (reads.n * per_read + reads.n_cigar_ops * 4 + reads.n_bases // 2 + reads.n_bases
            + chrom_len * (1 + 3 * 4))


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


def cpu_baseline_and_concordance(work_dir, knobs, flags):
    """The oracle (CPU port of GROM's scan, one thread) on a bounded 3-contig
    sample of the workload's generator, whole run (BAM decode + scan + VCF);
    then the GPU CLI on the same files, timed end to end (BAM decode, host
    batches, upload, scans, rows) and compared byte for byte."""
    from grom_amd import cli_main, last_error, run_synth
    total = sum(CPU_SAMPLE_LENS)
    sample = f"{len(CPU_SAMPLE_LENS)} contigs, {total / 1e6:g} Mb"
    bam, fa = run_synth(os.path.join(work_dir, "sample"), *synth_args(knobs, CPU_SAMPLE_LENS))
    env = dict(os.environ, GROM_FILEDATE="20260101", GROM_SEED="7")
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
    rc = cli_main(["-i", bam, "-r", fa, "-o", "gpu.vcf"] + flags, env={"GROM_FILEDATE": "20260101", "GROM_SEED": "7"},
                  cwd=work_dir)
    dt_gpu = time.perf_counter() - t0
    if rc != 0:
        raise RuntimeError(f"GPU CLI failed on the concordance sample: {last_error()}")
    same = all(open(os.path.join(work_dir, "gpu" + ext), "rb").read() ==
               open(os.path.join(work_dir, "cpu" + ext), "rb").read() for ext in (".vcf", ".ctx.vcf"))
    rows = sum(1 for ln in open(os.path.join(work_dir, "gpu.vcf")) if not ln.startswith("#"))
    conc = {"sample": f"the cpu_baseline sample ({sample}) through the GPU CLI (grom_cli_main)",
            "vcf_rows": rows, "identical_to_oracle": same,
            "cli_end_to_end_s": round(dt_gpu, 2), "cli_end_to_end_mbases_per_s": round(total / dt_gpu / 1e6, 2),
            "cli_note": "whole CLI run: insert pre-pass, BAM decode (host), upload, scans, VCF; on a sample this "
                        "small the fixed costs (binomial tables, contexts) dominate"}
    return cpu, conc


def cli_whole_run_start(work_dir, knobs, flags, scale):
    """Write the >=100 Mb BAM, start the oracle on it in the background (its
    VCF is compared at the end), then time the GPU CLI twice as a fresh process."""
    from grom_amd import GROM_BIN, run_synth
    names = [n for n, _ in GRCH38]
    lengths = [max(int(L * scale), 1_000_000) for _, L in GRCH38]
    total = sum(lengths)
    src = os.path.join(work_dir, "src")
    os.makedirs(src, exist_ok=True)
    t0 = time.perf_counter()
    bam, fa = run_synth(os.path.join(src, "cli"), *synth_args(knobs, lengths), "-n", ",".join(names), timeout=1200)
    t_synth = time.perf_counter() - t0
    print(f"[bench] whole-run BAM written: {total / 1e6:.1f} Mb, {os.path.getsize(bam) / 1e9:.2f} GB in {t_synth:.1f} s",
          file=sys.stderr, flush=True)
    env = dict(os.environ, GROM_FILEDATE="20260101", GROM_SEED="7")
    dirs = {}
    for side in ("gpu", "cpu"):  # own copies of the side files (.mean, .info); same paths in the VCF header
        d = os.path.join(work_dir, side)
        os.makedirs(d, exist_ok=True)
        for f, t in (("cli.bam", bam), ("cli.bam.bai", bam + ".bai"), ("cli.fa", fa)):
            os.symlink(t, os.path.join(d, f))
        dirs[side] = d
    args = ["-i", "cli.bam", "-r", "cli.fa", "-o", "out.vcf"] + flags
    runs = []
    for _ in range(2):
        t1 = time.perf_counter()
        r = subprocess.run([GROM_BIN] + args, cwd=dirs["gpu"], env=dict(env, GROM_VERBOSE="1"), capture_output=True,
                           text=True, timeout=600)
        runs.append(time.perf_counter() - t1)
        print(f"[bench] CLI whole run {len(runs)}: {runs[-1]:.2f} s", file=sys.stderr, flush=True)
        if r.returncode != 0:
            raise RuntimeError("GPU CLI failed on the whole-run BAM: " + r.stdout[-2000:] + r.stderr[-2000:])
    dec = [ln for ln in r.stdout.splitlines() if ln.startswith("streamed decode:")]
    info = {"bam": f"{len(lengths)} GRCh38 contigs x {scale:g} ({total / 1e6:.1f} Mb), same generator and flags "
                   f"as the workload (grom_synth {' '.join(synth_args(knobs, ['...']))})",
            "bam_bytes": os.path.getsize(bam), "genome_bases": total, "synth_s": round(t_synth, 1),
            "cli_wall_s": [round(x, 3) for x in runs],
            "value": round(total / min(runs) / 1e6, 2), "unit": "Mbases/s",
            "value_first_run": round(total / runs[0] / 1e6, 2),
            "decode": dec[-1] if dec else None,
            "note": "grom_amd/bin/grom as a fresh process (process start, HIP init, BAM index + parallel decode on "
                    "the host, pinned pieces -> HBM, scans, VCF + .ctx.vcf); best of two runs, the BAM in the page "
                    "cache"}
    # the oracle runs after the timed region (cli_whole_run_finish): beside
    # it, it took host cores from the scans' row threads (1,640 vs 1,458 ms
    # per pass in round 3)
    return {"info": info, "args": args, "env": env, "dirs": dirs, "total": total}


def cli_whole_run_finish(st):
    info = st["info"]
    oracle = os.path.join(REPO, "oracle", "grom_oracle")
    st["t_oracle"] = time.perf_counter()
    st["proc"] = subprocess.Popen([oracle] + st["args"], cwd=st["dirs"]["cpu"], env=st["env"],
                                  stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
    while True:  # a line every 30 s while the oracle runs (long silent runs look hung)
        try:
            err = st["proc"].communicate(timeout=30)[1]
            break
        except subprocess.TimeoutExpired:
            print(f"[bench] oracle on the whole-run BAM: {time.perf_counter() - st['t_oracle']:.0f} s", file=sys.stderr,
                  flush=True)
    dt = time.perf_counter() - st["t_oracle"]
    if st["proc"].returncode != 0:
        info["identical_to_oracle"] = None
        info["oracle_error"] = (err or "")[-500:]
        return info
    same = all(open(os.path.join(st["dirs"]["gpu"], "out" + ext), "rb").read() ==
               open(os.path.join(st["dirs"]["cpu"], "out" + ext), "rb").read() for ext in (".vcf", ".ctx.vcf"))
    info["identical_to_oracle"] = same
    info["vcf_rows"] = sum(1 for ln in open(os.path.join(st["dirs"]["gpu"], "out.vcf")) if not ln.startswith("#"))
    info["oracle_s"] = round(dt, 1)
    info["oracle_mbases_per_s"] = round(st["total"] / dt / 1e6, 3)
    return info


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--workload", choices=["genome", "chrom"], default="genome",
                    help="genome: configs[2]/[3] human-shape 3.09 Gb genome; chrom: configs[1] 100 Mb chromosome")
    ap.add_argument("--scale", type=float, default=1.0, help="scale every contig length (tests / quick runs)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inflight", type=int, default=2,
                    help="chromosome scans in flight per GPU: library context slots on the same device, one host "
                         "thread each")
    ap.add_argument("--gen-workers", type=int, default=0, help="host generator threads (0: auto)")
    ap.add_argument("--cnv-rate", type=float, default=None, help="override the copy-number region rate (tests)")
    ap.add_argument("--sweep-inflight", default="", help="e.g. 1,2,3,4: time one pass per value first (stderr)")
    ap.add_argument("--cli-scale", type=float, default=0.04,
                    help="contig scale of the whole-run CLI leg's BAM (0.04: 24 contigs, 124 Mb); 0 skips it")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    import grom_amd
    from grom_amd.shard import assign_chromosomes, max_over_ranks, run_queue

    genome = args.workload == "genome"
    if genome:
        knobs, flags = C3, ["-M"]
        names = [n for n, _ in GRCH38]
        lengths = [max(int(L * args.scale), 1_000_000) for _, L in GRCH38]
        mine = assign_chromosomes(lengths, world)[rank] if world > 1 else list(range(len(lengths)))
    else:
        knobs, flags = C2, []
        names = ["chr1"]
        lengths = [max(int(100_000_000 * args.scale), 1_000_000)]
        mine = [0]
    if args.cnv_rate is not None:
        knobs = dict(knobs, cnv_rate=args.cnv_rate)
    params = grom_amd.default_params()
    params.rmdup = 1 if "-M" in flags else 0
    gen = dict(coverage=knobs["coverage"], read_len=READ_LEN, dup_frac=knobs["dup_frac"],
               sv_per_mb=knobs["sv_per_mb"], cnv_rate=knobs["cnv_rate"], cnv_range=knobs["cnv_range"],
               seed=knobs["seed"] + (rank if not genome else 0))
    # the whole-run CLI leg first, while HBM is empty (its oracle runs meanwhile)
    cli_state, cli_dir = None, None
    if genome and rank == 0 and world == 1 and args.cli_scale > 0 and not args.no_cpu_baseline:
        cli_dir = tempfile.TemporaryDirectory()
        cli_state = cli_whole_run_start(cli_dir.name, knobs, flags, args.cli_scale)
        print(f"[bench] CLI whole run: {cli_state['info']['cli_wall_s']} s, {cli_state['info']['value']} Mbases/s",
              file=sys.stderr, flush=True)
    # genome-wide insert statistics (find_insert_mean runs once per BAM): the
    # same generator on a 2 Mb probe, identical on every rank
    probe = grom_amd.SynthBatch.genome_chrom([2_000_000], 0, params, **dict(gen, sv_per_mb=0.0, cnv_rate=0.0))
    probe.close()

    # generate each chromosome on the host and keep its inputs in HBM
    order = sorted(mine, key=lambda i: (-lengths[i], i))  # longest first, as GROM.c:22318-22336
    workers = args.gen_workers or max(1, min(8, 16 // max(world, 1), len(order)))
    res, info = {}, {}
    lock = threading.Lock()
    mem_reserve = 48 << 30  # scratch of the scan contexts on the largest chromosome

    def make(i):
        b = grom_amd.SynthBatch.genome_chrom(lengths, i, params, names=names, **gen)
        try:
            r = grom_amd.Resident(local, b.chrom, b.reads)
            with lock:
                res[i] = r
                info[i] = {"reads": b.reads.n, "bytes": algorithmic_bytes(b.reads, lengths[i]),
                           "resident_bytes": r.bytes}
            free = grom_amd.lib().grom_device_mem_free(local)
            print(f"[bench] {names[i]}: {b.reads.n} reads generated and resident ({r.bytes / 1e9:.1f} GB), "
                  f"{free / 2**30:.0f} GiB HBM free, {time.perf_counter() - t_gen:.0f} s", file=sys.stderr, flush=True)
            if 0 <= free < mem_reserve:
                raise RuntimeError(f"HBM nearly full after uploading {names[i]} ({free / 2**30:.1f} GiB free)")
        finally:
            b.close()

    t_gen = time.perf_counter()
    run_queue([make] * workers, order)
    t_gen = time.perf_counter() - t_gen

    if args.sweep_inflight:
        for f in [int(v) for v in args.sweep_inflight.split(",")]:
            dv = [grom_amd.Device(local, params, slot=local + 8 * k) for k in range(f)]
            ot = [grom_amd.Out() for _ in dv]

            def sw(k):
                return lambda i: dv[k].scan(res[i].chrom, res[i].reads, device_resident=True, out=ot[k])
            run_queue([sw(k) for k in range(f)], order)  # warm
            t1 = time.perf_counter()
            run_queue([sw(k) for k in range(f)], order)
            t1 = time.perf_counter() - t1
            print(f"[bench] inflight {f}: {t1 * 1e3:.0f} ms per pass, {sum(lengths[i] for i in mine) / t1 / 1e6:.1f} "
                  f"Mbases/s, {grom_amd.lib().grom_device_mem_free(local) / 2**30:.0f} GiB HBM free", file=sys.stderr,
                  flush=True)
            for o in ot:
                grom_amd.lib().grom_out_free(ctypes.byref(o))
            for d in reversed(dv):
                d.close()
    F = max(1, min(args.inflight, 8))
    devs = [grom_amd.Device(local, params, slot=local + 8 * k) for k in range(F)]
    outs = [grom_amd.Out() for _ in devs]
    pile_ms, pile_bytes, cnv_ms = [], [], []
    rows = {}

    def scanner(k, record):
        def scan(i):
            vcf_len, st = devs[k].scan(res[i].chrom, res[i].reads, device_resident=True, out=outs[k])
            if record is not None:
                with lock:
                    record.append((i, st.ms_pileup, st.ms_cnv))
            else:
                rows[i] = ctypes.string_at(outs[k].vcf, vcf_len).count(b"\n")
        return scan

    # warmup passes (the first also counts each chromosome's VCF rows)
    for w in range(args.warmup):
        run_queue([scanner(k, None if w == 0 else []) for k in range(F)], order)
    # the pileup kernel alone (nothing else on the GPU), on the largest chromosome
    _, st_alone = devs[0].scan(res[order[0]].chrom, res[order[0]].reads, device_resident=True, out=outs[0])

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    rec = []
    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        run_queue([scanner(k, rec) for k in range(F)], order)
    barrier()
    dt = max_over_ranks(time.perf_counter() - t0, device="cuda")
    for o in outs:
        grom_amd.lib().grom_out_free(ctypes.byref(o))

    total_bases = sum(lengths) if genome else lengths[0] * world
    value = total_bases * args.steps / dt / 1e6
    launch_bytes = sum(info[i]["bytes"] for i, _, _ in rec)
    launch_s = sum(ms for _, ms, _ in rec) / 1e3
    achieved = launch_bytes / launch_s / 1e9
    bases_launched = sum(lengths[i] for i, _, _ in rec)
    survey_achieved = SURVEY_BYTES_PER_BASE * bases_launched / launch_s / 1e9
    big = order[0]
    alone_ach = info[big]["bytes"] / (st_alone.ms_pileup / 1e3) / 1e9
    tag = "genome_30x" if genome else f"{lengths[0] // 1_000_000}Mb_30x"
    traffic = None
    pmc = os.path.join(REPO, "profiles", f"pmc_{tag}.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get(f"{PILEUP_KERNEL}_hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        cpu = conc = None
        if world == 1 and not args.no_cpu_baseline:
            with tempfile.TemporaryDirectory() as d:
                cpu, conc = cpu_baseline_and_concordance(d, knobs, flags)
        cli_info = cli_whole_run_finish(cli_state) if cli_state else None
        if cli_dir:
            cli_dir.cleanup()
        wl = ("BASELINE configs[2]: synthetic 30x 2x150 bp human-shape genome, 24 GRCh38 contigs "
              f"({sum(lengths) / 1e9:.3f} Gb), SNV/indel, {knobs['sv_per_mb']:.2f} breakpoint SVs/Mb "
              "(DEL/DUP/INV/INS/CTX with split reads + discordant pairs), 500 CNVs/3.1 Gb, 5% PCR duplicates, -M"
              + ("; chromosomes LPT-sharded over ranks (configs[3])" if world > 1 else "")
              if genome else
              "BASELINE configs[1]: one 100 Mb chromosome per GPU, 30x 2x150 bp, SNV/indel")
        line = {
            "metric": "Mbases/sec scanned (whole genome) + VCF concordance vs ref",
            "value": round(value, 3),
            "unit": "Mbases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong" if genome else "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded generator grom_amd/csrc/synth.c, inputs resident in HBM)",
            "config": {
                "workload": wl + "; step = every chromosome through grom_scan_chrom_device (pileup/SNV, "
                                 "duplicate filter, breakpoint evidence + tests, SV/INDEL rows, CTX records, "
                                 "read-depth CNV path + rows)",
                "genome_bases": total_bases, "chromosomes": len(lengths), "chromosomes_rank0": len(mine),
                "coverage": knobs["coverage"], "read_len": READ_LEN, "flags": " ".join(flags),
                "reads_rank0": sum(info[i]["reads"] for i in mine),
                "vcf_rows_rank0": sum(rows.values()),
                "hbm_resident_gb_rank0": round(sum(info[i]["resident_bytes"] for i in mine) / 1e9, 1),
                "host_generate_s": round(t_gen, 1), "generator_threads": workers,
                "scans_in_flight_per_gpu": F,
                "cnv_ms_per_step_rank0": round(sum(c for _, _, c in rec) / args.steps, 1),
            },
            "roofline": {
                "bound": "hbm", "kernel": PILEUP_KERNEL,
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "bytes_model": "this build (DESIGN.md 6): read records + CIGAR + 1.5 B per read base + 13 B per "
                               "reference base, summed over the timed launches",
                "launches": len(rec), "launch_ms_mean": round(launch_s * 1e3 / len(rec), 3),
                "bytes_per_100mb": round(launch_bytes / bases_launched * 1e8),
                "survey_bytes_per_base": SURVEY_BYTES_PER_BASE,
                "survey_achieved": round(survey_achieved, 1),
                "survey_frac": round(survey_achieved / HBM_PEAK_GBS, 4),
                "alone": {"chrom": names[big], "launch_ms": round(st_alone.ms_pileup, 3),
                          "achieved": round(alone_ach, 1), "frac": round(alone_ach / HBM_PEAK_GBS, 4),
                          "survey_frac": round(SURVEY_BYTES_PER_BASE * lengths[big] / (st_alone.ms_pileup / 1e3)
                                               / 1e9 / HBM_PEAK_GBS, 4)},
            },
            "cpu_baseline": cpu,
            "concordance": conc,
            "cli_whole_run": cli_info,
        }
        print(json.dumps(line), flush=True)
    for d in reversed(devs):
        d.close()
    for r in res.values():
        r.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
