"""CPU baseline of BASELINE configs[4]'s path (`snap-rna paired`, PairedAligner.cpp:421-689) on bench.py's
RNA workload, measured with the reference itself (oracle/_ref/snap-rna, compiled from /root/reference by
oracle/Makefile.ref) in the build container -- the reference cannot travel to the GPU box.

Workload: the same inputs as bench.py's `extras.rna_paired` and golden.json["rna_bench"]: the C2
synthetic genome, the 2,000-gene synthetic GTF and tests/rna_synth.py's 2 x 150 pairs (deterministic).
The reference runs `snap-rna paired <C2 index> <transcriptome> synth.gtf r1 r2 -t T` over a bounded sample
(--blocks blocks of --block pairs, spread over the 100k pairs), and its own stats line (AlignerContext::
printStats, AlignerContext.cpp:372-393: "... Reads/s (at: <ms>)") gives the alignment time, which
excludes loading the index, the transcriptome and the GTF.  reads/s = 2 x pairs / sum of the blocks'
alignment times.  Blocks on which the reference crashes at the end of the run (AnalyzeReadIntervals,
DESIGN.md section 8) are skipped and listed.

    python3 tests/golden/rna_cpu_baseline.py [--blocks 6] [--block 2000] [--threads 1] [--opt N]

--opt N times oracle/_ref/snap-rna-O<N> (`make -f oracle/Makefile.ref rna-variants`: BaseAligner.cpp at -O<N>,
the rest as in snap-rna) instead of snap-rna, whose BaseAligner.cpp is built at -O0 (oracle/Makefile.ref:
CharacterizeSeeds' missing return); each block is then also run through the -O0 binary and the two SAM
outputs compared (records equal or not, and where the optimised build crashed).

Writes the run into tests/golden/rna_cpu_baseline.json under "threads_<T>" (or "threads_<T>_O<N>"); bench.py
prints the records as extras.rna_paired.cpu_baseline.
"""
import json
import os
import platform
import re
import shutil
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, HERE)

import snapgpu  # noqa: E402
from golden_common import C2  # noqa: E402

SNAP = os.path.join(ROOT, "oracle", "_ref", "snap-rna")
STATS = re.compile(r"\t(\d+)\t(\d+) \(at: (\d+)\)")


def cpu_model():
    for line in open("/proc/cpuinfo"):
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    return platform.processor()


def main():
    a = sys.argv
    blocks = int(a[a.index("--blocks") + 1]) if "--blocks" in a else 6
    block = int(a[a.index("--block") + 1]) if "--block" in a else 2000
    threads = int(a[a.index("--threads") + 1]) if "--threads" in a else 1
    opt = a[a.index("--opt") + 1] if "--opt" in a else "0"   # 1, 2, 3 (g++) or 3c (clang -fno-strict-return)
    opt = 0 if opt == "0" else opt
    snap = SNAP + (f"-O{opt}" if opt else "")
    from rna_synth import synth_rna_workload
    work = tempfile.mkdtemp(prefix="rnacpu")
    try:
        gg = snapgpu.Genome.synthetic(**C2["genome"])
        gfa = os.path.join(work, "c2.fa")
        gg.write_fasta(gfa)
        gtf, fq0, fq1, info = synth_rna_workload(gg._h, work, n_pairs=100_000)
        gidx = os.path.join(work, "gidx")
        subprocess.run([SNAP, "index", gfa, gidx], check=True, capture_output=True)
        twd = os.path.join(work, "tx")
        os.makedirs(twd)
        subprocess.run([SNAP, "transcriptome", gtf, gfa, "tidx", "-O1000"], check=True, capture_output=True, cwd=twd)
        recs = [open(x).read().splitlines() for x in (fq0, fq1)]
        n = len(recs[0]) // 4
        stride = n // blocks
        runs, crashed = [], []
        for b in range(blocks):
            first = b * stride
            idx = range(first, min(n, first + block))
            d = tempfile.mkdtemp(dir=work, prefix="blk")
            for k in range(2):
                with open(os.path.join(d, f"r_{k}.fq"), "w") as f:
                    f.write("".join("\n".join(recs[k][4 * i:4 * i + 4]) + "\n" for i in idx))
            def run(binary, out):
                return subprocess.run([binary, "paired", gidx, os.path.join(twd, "tidx"), gtf, os.path.join(d, "r_0.fq"),
                                       os.path.join(d, "r_1.fq"), "-t", str(threads), "-o", os.path.join(d, out)],
                                      capture_output=True, text=True, cwd=d)

            def records(out):   # (sorted: with -t > 1 the writer threads interleave pairs differently per run)
                with open(os.path.join(d, out)) as f:
                    return sorted(l for l in f if not l.startswith("@PG"))
            r = run(snap, "out.sam")
            m = STATS.search(r.stdout)
            if r.returncode != 0 or not m:
                crashed.append({"first_pair": first, "returncode": r.returncode,
                                "stderr_tail": (r.stderr or r.stdout).strip().splitlines()[-1:]})
            else:
                runs.append({"first_pair": first, "pairs": len(idx), "total_reads": int(m.group(1)),
                             "reads_per_s_printed": int(m.group(2)), "align_ms": int(m.group(3))})
                if opt:   # the same block through the -O0 build: are the records the same?
                    r0 = run(SNAP, "out_O0.sam")
                    runs[-1]["records_equal_to_O0"] = (r0.returncode == 0 and STATS.search(r0.stdout) is not None
                                                       and records("out.sam") == records("out_O0.sam"))
            shutil.rmtree(d, ignore_errors=True)
            print(runs[-1] if runs and runs[-1]["first_pair"] == first else {"crashed": first}, flush=True)
        if not runs:
            print(json.dumps({"opt": opt, "threads": threads, "every_block_crashed": crashed}))
            return
        pairs = sum(x["pairs"] for x in runs)
        ms = sum(x["align_ms"] for x in runs)
        out = {"value": 2 * pairs / (ms / 1000.0), "unit": "reads/s", "cores": threads,
               "kind": "reference, build container", "base_aligner_opt": f"-O{opt}",
               "sample": f"{pairs} of bench.py's 100k 2x150 RNA pairs ({len(runs)} blocks of {block}, spread over the "
                         f"set), `snap-rna paired <C2 index> <transcriptome> synth.gtf r1 r2 -t {threads}` with "
                         f"BaseAligner.cpp compiled at -O{opt} (the other SNAPLib files at -O3, the UB files at -O0: "
                         "oracle/Makefile.ref); time = the reference's own alignment time (AlignerContext::printStats), "
                         "index load excluded",
               "host": {"cpu": cpu_model(), "nproc": os.cpu_count()},
               "blocks": runs, "crashed_blocks": crashed, "workload": info}
        path = os.path.join(HERE, "rna_cpu_baseline.json")
        allr = json.load(open(path)) if os.path.exists(path) else {}
        if opt:
            out["records_equal_to_O0"] = all(x.get("records_equal_to_O0") for x in runs) and bool(runs)
        allr[f"threads_{threads}" + (f"_O{opt}" if opt else "")] = out   # one record per thread count / level
        with open(path, "w") as f:
            json.dump(allr, f, indent=1)
        print(json.dumps({k: v for k, v in out.items() if k not in ("blocks", "workload")}))
    finally:
        shutil.rmtree(work, ignore_errors=True)


if __name__ == "__main__":
    main()
