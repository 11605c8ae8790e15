"""tools/make_golden_genome.py -- golden digests of the oracle on inputs too
large for it to run inside a GPU test:

  genome_s010   a 24-contig genome at 0.1 of GRCh38's contig lengths (BASELINE
                configs[2]'s shape: 30x, SVs, copy-number regions, 5% PCR
                duplicates), run with -M -g 1 -- about 7 minutes of oracle;
  genome_s100   the bench's own workload, BASELINE configs[2] at full GRCh38
                contig lengths (3.09 Gb, 20 GB BAM), -M -g 1 -- about 3 hours of
                oracle; bench.py compares its timed whole run's rows with it
                (identical_to_oracle_full_scale);
  c4_20mb_60x   BASELINE configs[4]'s shape at 20 Mb: a 60x tetraploid male
                donor (chr1 at 60x, chrX/chrY at 30x), SVs, copy-number regions,
                2% duplicates, run with -p 4 -g 1 -M -V 1 -- about 90 s.

For each case tests/golden/oracle_<case>.json keeps the grom_synth arguments,
the CLI flags and the sha256 and row counts of the oracle's VCF and .ctx.vcf, and the sha256 of
their non-header rows alone (the ##reference header names the FASTA path).
tests/test_gpu_parity.py::test_oracle_digest_cases writes the same BAM on the
GPU box (grom_synth is deterministic per seed) and checks the GPU CLI's
outputs against these digests.

    python tools/make_golden_genome.py CASE [workdir]
"""
import hashlib
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402


def cases():
    lengths = [max(int(l * 0.1), 1_000_000) for _, l in bench.GRCH38]
    names = [n for n, _ in bench.GRCH38]
    return {
        "genome_s010": (bench.synth_args(bench.C3, lengths) + ["-n", ",".join(names)], list(bench.GENOME_FLAGS)),
        "genome_s100": (bench.synth_args(bench.C3, [l for _, l in bench.GRCH38]) + ["-n", ",".join(names)],
                        list(bench.GENOME_FLAGS)),
        "c4_20mb_60x": (["-L", "12000000,5000000,3000000", "-n", "chr1,chrX,chrY", "-c", "60,30,30", "-P", "4", "-s",
                         "5", "-X", "4", "-D", "0.02", "-V", "0.0000004", "-W", "20000,300000", "-l", "150"],
                        ["-p", "4", "-g", "1", "-M", "-V", "1"]),
    }


def digest(path):
    """(sha256 of the file, rows, sha256 of the non-header rows)"""
    h, hr = hashlib.sha256(), hashlib.sha256()
    rows = 0
    with open(path, "rb") as f:
        for line in f:
            h.update(line)
            if not line.startswith(b"#"):
                hr.update(line)
                rows += 1
    return h.hexdigest(), rows, hr.hexdigest()


def main():
    case = sys.argv[1]
    work = sys.argv[2] if len(sys.argv) > 2 else f"/tmp/golden_{case}"
    os.makedirs(work, exist_ok=True)
    args, flags = cases()[case]
    env = dict(os.environ, GROM_FILEDATE="20260101", GROM_SEED="7")
    subprocess.run([os.path.join(REPO, "grom_amd", "bin", "grom_synth"), "-o", "genome"] + args, cwd=work, env=env,
                   check=True, stdout=subprocess.DEVNULL)
    t0 = time.time()
    subprocess.run([os.path.join(REPO, "oracle", "grom_oracle"), "-i", "genome.bam", "-r", "genome.fa", "-o",
                    "o.vcf"] + flags, cwd=work, env=env, check=True, stdout=subprocess.DEVNULL)
    dt = time.time() - t0
    vcf, nv, vcf_rows = digest(os.path.join(work, "o.vcf"))
    ctx, nc, ctx_rows = digest(os.path.join(work, "o.ctx.vcf"))
    rec = {"generator": f"tools/make_golden_genome.py {case}", "synth_args": args, "cli_flags": flags,
           "env": {"GROM_FILEDATE": "20260101", "GROM_SEED": "7"}, "oracle_seconds": round(dt, 1),
           "vcf_sha256": vcf, "vcf_rows": nv, "ctx_sha256": ctx, "ctx_rows": nc,
           "vcf_rows_sha256": vcf_rows, "ctx_rows_sha256": ctx_rows}
    with open(os.path.join(REPO, "tests", "golden", f"oracle_{case}.json"), "w") as f:
        json.dump(rec, f, indent=1)
        f.write("\n")
    print(json.dumps(rec))


if __name__ == "__main__":
    main()
