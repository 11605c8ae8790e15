"""bench.py -- GROM per-chromosome scan on MI355X.

One step = one pass of the scan (grom_scan_chrom_device: the pileup/SNV HIP
kernels, the host SNV-list flush and VCF formatting, the CIGAR indel-evidence
pass, and the read-depth CNV
path -- GC windows, depth blocks, detect_del_dup and its rows) over one
synthetic 100 Mb, 30x,
2x150 bp paired-end chromosome whose reads are already resident in HBM
(BASELINE.json configs[1]).  With --gpus N (torch.distributed.run, one rank per
GPU) every rank scans its own chromosome: chromosomes shard with no data-path
collective, so scaling is weak and `value` is all bases scanned / max-rank time.

With --inflight F (default 2) each GPU runs F scans at once: F library
contexts on the device (grom_ctx_init), one host thread each, steps dealt
round-robin, all K finished inside the timed region.  The pileup kernel then
shares the GPU, so its launch time over the timed region (roofline.launch_ms)
is longer than alone; roofline.launch_ms_alone / frac_alone give the kernel
measured one scan at a time during warmup.

The JSON line also carries
  roofline      the pileup kernel's (k_scan_tile; k_scan_scatter with
                GROM_PILEUP=scatter) algorithmic bytes per launch / its mean
                duration
                (HIP events on the library's stream) against 8 TB/s HBM,
                with PMC-measured traffic when profiles/pmc_<tag>.json exists;
  cpu_baseline  the CPU restatement of the reference (oracle/, "port"), one
                thread, on a bounded sample of the same workload (rank 0, N=1).
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

CHROM_LEN = 100_000_000
COVERAGE = 30.0
READ_LEN = 150
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md, HBM3E peak (spec)
CPU_SAMPLE_LEN = 6_000_000
PILEUP_KERNEL = "k_scan_scatter" if os.environ.get("GROM_PILEUP") == "scatter" else "k_scan_tile"


def algorithmic_bytes(batch) -> int:
    """Bytes the pileup kernel must move once per launch: every read record it ingests
    (SoA metadata, CIGAR, packed bases, qualities), the reference, and the three
    whole-chromosome read-depth arrays it writes ('Roofline')."""
    r = batch.reads
    per_read = 4 + 2 + 1 + 4 + 4 + 4 + 4 + 4 + 8 + 4  # pos flag mapq mtid mpos isize lqseq cig_off base_off name
    return (r.n * per_read + r.n_cigar_ops * 4 + r.n_bases // 2 + r.n_bases
            + batch.chrom.len * (1 + 3 * 4))


def cpu_baseline(work_dir):
    """Oracle (CPU port of GROM's scan, single thread) on a 6 Mb / 30x sample."""
    from grom_amd import run_synth
    prefix = os.path.join(work_dir, "cpu_sample")
    bam, fa = run_synth(prefix, "-L", str(CPU_SAMPLE_LEN), "-s", "3", "-c", str(COVERAGE), "-l", str(READ_LEN))
    oracle = os.path.join(REPO, "oracle", "grom_oracle")
    t0 = time.perf_counter()
    r = subprocess.run([oracle, "-i", bam, "-r", fa, "-o", os.path.join(work_dir, "cpu.vcf")], cwd=work_dir,
                       capture_output=True, text=True, timeout=900)
    dt = time.perf_counter() - t0
    if r.returncode != 0:
        raise RuntimeError("oracle failed: " + r.stderr[-2000:])
    return {"value": round(CPU_SAMPLE_LEN / dt / 1e6, 4), "unit": "Mbases/s", "cores": 1, "kind": "port",
            "sample": f"{CPU_SAMPLE_LEN // 1_000_000} Mb synthetic chromosome, {COVERAGE:g}x 2x{READ_LEN} bp, "
                      f"whole oracle run (BAM decode + scan + VCF) in {dt:.2f} s, 1 thread"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--chrom-len", type=int, default=CHROM_LEN)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inflight", type=int, default=2,
                    help="chromosome scans in flight per GPU: library context slots on the same device, one host "
                         "thread each (a genome's chromosomes are independent scans)")
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
    from grom_amd.shard import max_over_ranks, timed_concurrent

    t_gen = time.perf_counter()
    batch = grom_amd.SynthBatch(args.chrom_len, COVERAGE, READ_LEN, 500.0, 50.0, seed=1000 + rank)
    t_gen = time.perf_counter() - t_gen
    F = max(1, min(args.inflight, 8))
    dev = grom_amd.Device(local, batch.params)
    # more contexts on the same GPU (slots local + 8k); they scan the reads uploaded once by the first
    devs = [dev] + [grom_amd.Device(local, batch.params, slot=local + 8 * k) for k in range(1, F)]
    dchrom, dreads = dev.upload(batch.chrom, batch.reads)
    alone_ms = []  # the pileup kernel with nothing else on the GPU (warmup, one scan at a time)
    for _ in range(args.warmup):
        for d in devs:
            _, st = d.scan(dchrom, dreads, device_resident=True)
            alone_ms.append(st.ms_pileup)

    def barrier():
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()

    pile_ms = []
    tot_ms = []
    cnv_ms = []
    outs = [grom_amd.Out() for _ in devs]  # VCF text buffers, reused across steps (grom_out)
    last = [0] * F

    def step_on(k):
        def step(i):
            vcf_len, st = devs[k].scan(dchrom, dreads, device_resident=True, out=outs[k])
            pile_ms.append(st.ms_pileup)
            tot_ms.append(st.ms_total)
            cnv_ms.append(st.ms_cnv)
            last[k] = vcf_len
        return step

    dt = timed_concurrent([step_on(k) for k in range(F)], args.steps, barrier)
    texts = [ctypes.string_at(outs[k].vcf, last[k]) for k in range(F) if last[k]]
    rows = texts[0].count(b"\n") if texts else 0
    if any(t != texts[0] for t in texts):
        raise RuntimeError("contexts produced different VCF text for the same chromosome")
    for o in outs:
        grom_amd.lib().grom_out_free(ctypes.byref(o))
    dt = max_over_ranks(dt, device="cuda")

    bases = args.chrom_len * world * args.steps
    value = bases / dt / 1e6
    abytes = algorithmic_bytes(batch)
    pile_s = sum(pile_ms) / len(pile_ms) / 1e3
    achieved = abytes / pile_s / 1e9
    tag = f"{args.chrom_len // 1_000_000}Mb_{int(COVERAGE)}x"
    traffic = None
    pmc = os.path.join(REPO, "profiles", f"pmc_{tag}.json")
    if os.path.exists(pmc):
        try:
            traffic = json.load(open(pmc)).get(f"{PILEUP_KERNEL}_hbm_bytes_per_launch")
        except Exception:
            traffic = None

    if rank == 0:
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            with tempfile.TemporaryDirectory() as d:
                cpu = cpu_baseline(d)
        line = {
            "metric": "Mbases/sec scanned (whole genome) + VCF concordance vs ref",
            "value": round(value, 3),
            "unit": "Mbases/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int32",
            "data": "synthetic (seeded generator, grom_amd/csrc/synth.c)",
            "config": {
                "workload": "BASELINE configs[1]: 1 chromosome of 100 Mb per GPU, 30x 2x150 bp paired-end, "
                            "SNV/indel, reads resident in HBM; step = pileup/SNV scan + SNV flush + VCF text + CIGAR "
                            "indel evidence + read-depth CNV path (GC windows, depth blocks, detect_del_dup, CNV rows)",
                "chrom_len": args.chrom_len, "coverage": COVERAGE, "read_len": READ_LEN,
                "reads_per_gpu": batch.n_reads, "vcf_rows_per_step": rows,
                "device_ms_per_step": round(sum(tot_ms) / len(tot_ms), 3),
                "cnv_ms_per_step": round(sum(cnv_ms) / len(cnv_ms), 3),
                "host_generate_s": round(t_gen, 1),
                "scans_in_flight_per_gpu": F,
            },
            "roofline": {
                "bound": "hbm", "kernel": PILEUP_KERNEL,
                "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                "bytes_per_launch": abytes, "launch_ms": round(pile_s * 1e3, 3),
                "launch_ms_alone": round(sum(alone_ms) / len(alone_ms), 3) if alone_ms else None,
                "frac_alone": (round(abytes / (sum(alone_ms) / len(alone_ms) / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                               if alone_ms else None),
            },
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    for d in reversed(devs):
        d.close()
    batch.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
