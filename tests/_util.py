"""Test helpers: synthetic datasets, the oracle (CPU restatement) and the product CLI."""
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_BIN = os.path.join(REPO, "oracle", "grom_oracle")
ORACLE_LIB = os.path.join(REPO, "oracle", "liboracle.so")
GROM_BIN = os.path.join(REPO, "grom_amd", "bin", "grom")
SYNTH_BIN = os.path.join(REPO, "grom_amd", "bin", "grom_synth")
GOLDEN_VCF = os.path.join(REPO, "tests", "golden", "tilapia_v1.0.0.vcf")
GOLDEN_CTX = os.path.join(REPO, "tests", "golden", "tilapia_v1.0.0.ctx.vcf")
# the reference's own test FASTA (test_data/oreNil2_GL831235-1.fa, 2.65 Mb,
# soft-masked, N runs), copied as a data fixture: SURVEY 8(d)'s C1s stand-in
# for the bundled tilapia BAM (a missing blob) simulates reads from it
TILAPIA_FA = os.path.join(REPO, "tests", "fixtures", "oreNil2_GL831235-1.fa")
NCOUNT = 40
FILEDATE = "20260101"
SEED = "7"  # GROM_SEED: pins the CNV sampling generator (srand(time()) at GROM.c:1584)

# synthetic parity cases: name -> grom_synth arguments
CASES = {
    "one_chr": ["-L", "400000", "-s", "11"],
    "three_chr": ["-L", "250000,180000,220000", "-s", "12"],
    "lowmapq_clip": ["-L", "300000", "-s", "13", "-Q", "0.2", "-C", "0.08", "-q", "0.1", "-U", "0.01"],
    "dups": ["-L", "300000", "-s", "14", "-D", "0.15"],
    "empty_middle": ["-L", "200000,200000,200000", "-s", "15", "-c", "30,0,30"],
    # CIGAR indels at 10x the default rate, half of them multi-allelic (two
    # lengths at one base: the evidence "other" slots and their swaps), with
    # low-MAPQ reads (zero-weight evidence) and PCR duplicates for -M
    "indels": ["-L", "400000", "-s", "21", "-I", "0.001", "-J", "0.5", "-Q", "0.1", "-D", "0.1"],
    # copy-number regions (0x, 0.5x, 1.5x, 2x depth) for the read-depth CNV path
    "cnv": ["-L", "1500000", "-s", "16", "-V", "0.000004", "-W", "20000,150000", "-Q", "0.05"],
    "cnv_multi": ["-L", "700000,900000", "-s", "17", "-V", "0.000005", "-W", "15000,80000", "-Q", "0.08"],
    # long copy-number regions (0.3-1 Mb, as in BASELINE configs[2]): calls whose
    # window search spans the region (the walk's wave-cooperative phases)
    "cnv_long": ["-L", "4000000", "-s", "18", "-V", "0.0000008", "-W", "300000,1000000", "-Q", "0.05", "-D", "0.05"],
    # BASELINE configs[4] shape: 60x tetraploid donor (allele fractions k/4),
    # a male genome (chrX and chrY at half depth), run with -p 4 -g 1
    "c5_tetra_male": ["-L", "500000,400000,300000", "-n", "chr1,chrX,chrY", "-c", "60,30,30", "-P", "4", "-s", "5",
                      "-X", "4", "-D", "0.02"],
    # BASELINE configs[2] shape: six contigs with SNVs/indels, breakpoint SVs,
    # copy-number regions and 5% PCR duplicates, run with -M
    "c3_genome": ["-L", "500000,420000,380000,300000,260000,220000", "-s", "3", "-D", "0.05", "-X", "6",
                  "-V", "0.000002", "-W", "20000,120000"],
    # breakpoint evidence: deletions, duplications, inversions, insertions and
    # translocations with split reads (SA tags), a 300 kb partner chromosome
    "sv": ["-L", "600000,300000", "-s", "31", "-X", "30", "-I", "0.0003", "-J", "0.3", "-Q", "0.05"],
    # dense breakpoint SVs: >= 50 rows of every <DEL>/<DUP>/<INV>/<INS> class and
    # translocation (BND) pairs in .ctx.vcf
    "sv_many": ["-L", "3000000,1500000", "-s", "33", "-X", "80", "-I", "0.0003", "-J", "0.3", "-Q", "0.05"],
    # reads simulated from the reference's tilapia FASTA at
    # 5x, 2x100 bp, seed 1 (the bundled test's contig, names and case kept)
    "c1s": ["-F", TILAPIA_FA, "-c", "5", "-l", "100", "-s", "1"],
    # a 30 Mb contig whose every window has one GC content: one GC bin gets
    # more than g_sample_lists_len (100,000) depth samples, so the reservoir
    # draws of GROM.c:18385-18451 run at the reference's own cap
    "cnv_reservoir": ["-L", "30000000", "-R", "50", "-s", "41", "-V", "0.0000002", "-W", "50000,300000", "-Q", "0.05"],
    # a 2.2 kb insert library (mean above the 1536 of the 32-bit GC-window
    # kernel: k_cnv_gc's 64-bit instance), with copy-number regions and SVs
    # a 20 kb insert library: above k_cnv_gc's 16,384 LDS halo, the GC windows
    # come from chromosome-wide prefixes (k_cnv_gc_global)
    "huge_insert": ["-L", "2500000", "-s", "23", "-m", "20000", "-d", "1500", "-V", "0.000003", "-W", "60000,300000",
                    "-Q", "0.05"],
    # amplicon depth: tiles of 256 positions holding about 60-72k reads, on both
    # sides of the register builds' 16-bit counter bound (PACK_MAX_READS,
    # 65,535: heavier tiles go to k_scan_tile_mem); contig ends ramp the depth
    # down through the bound
    "amplicon": ["-L", "30000,20000", "-c", "24500,23000", "-s", "51"],
    "wide_insert": ["-L", "1500000", "-s", "19", "-m", "2200", "-d", "200", "-V", "0.000004", "-W", "20000,150000",
                    "-Q", "0.05", "-X", "5"],
}


def synth(datadir, name, args):
    prefix = os.path.join(str(datadir), name)
    bam = prefix + ".bam"
    if not os.path.exists(bam):
        r = subprocess.run([SYNTH_BIN, "-o", prefix] + list(args), capture_output=True, text=True)
        assert r.returncode == 0, r.stderr
    return bam, prefix + ".fa"


def run(binary, args, cwd, env_extra=None):
    env = dict(os.environ)
    env["GROM_FILEDATE"] = FILEDATE
    env["GROM_SEED"] = SEED
    if env_extra:
        env.update(env_extra)
    r = subprocess.run([binary] + list(args), cwd=cwd, env=env, capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, f"{binary} failed: {r.stdout[-3000:]}\n{r.stderr[-3000:]}"
    return r


def run_oracle(datadir, bam, fa, out, extra=(), dump=None):
    env = {"GROM_ORACLE_DUMP": dump} if dump else None
    return run(ORACLE_BIN, ["-i", bam, "-r", fa, "-o", out] + list(extra), str(datadir), env)


def run_grom(datadir, bam, fa, out, extra=(), dump=None, env_extra=None):
    """The product CLI, called in this process through the C ABI so the HIP
    library is loaded (and checked) by the test process itself."""
    import grom_amd
    env = {"GROM_FILEDATE": FILEDATE, "GROM_SEED": SEED}
    if dump:
        env["GROM_DUMP"] = dump
    if env_extra:
        env.update(env_extra)
    rc = grom_amd.cli_main(["-i", bam, "-r", fa, "-o", out] + list(extra), env=env, cwd=str(datadir))
    assert rc == 0, f"grom_cli_main returned {rc}: {grom_amd.last_error()}"
    return rc


INDEL_DTYPE = np.dtype([(n, "<i4") for n in ("pos", "ins", "ins_len", "del_f", "del_f_len", "del_f_rd", "del_r",
                                             "del_r_len", "del_r_rd", "other_len")] +
                       [("ins_seq", "S52"), ("pad", "<i4")])


def load_indels(path):
    """grom_indel_rec / orc_indel records (include/grom_amd.h)."""
    return np.fromfile(path, dtype=INDEL_DTYPE)


def load_counts(path):
    a = np.fromfile(path, dtype=np.int32)
    return a.reshape(-1, NCOUNT)
