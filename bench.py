#!/usr/bin/env python3
"""Benchmark: aligned reads/s of the MI355X BaseAligner::AlignRead hot path.

Workload (BASELINE.json configs[1] shape): a chr21-sized
(46,709,983 bp) synthetic repeat-rich genome indexed with seed 20 and resident in
HBM; 1,000,000 wgsim-like 100 bp single-end reads per GPU in (pinned) host memory;
defaults maxHits 300, maxK 14, 25 seeds, extraSearchDepth 2.  `--workload c3` is the
per-GPU shard of configs[2]: a ~3.1 Gb, 25-contig genome and 6,250,000 reads per GPU.

One step = one batched AlignRead over the rank's reads at the SURVEY.md 8(d) d1
boundary: reads in host memory -> records in host memory, i.e. H2D of the reads, the
GPU passes, D2H of the records and the host MAPQ fix-ups (snapgpu_align_batch, which
pipelines chunks over two HIP streams).  The device-resident rate (inputs already in
HBM, records left there) is reported beside it as `resident`.

Multi-GPU: one process per GPU (torch.distributed.run), reads sharded by rank, the
index built once per node (rank 0, shared through /dev/shm) and uploaded by every rank;
no data-path collective -- gloo carries only the barriers and the max-over-ranks time.

Prints ONE JSON line on rank 0 (contract in the task statement), including `roofline`
(algorithmic bytes of the alignment kernel per launch / its HIP-event time per launch)
and `cpu_baseline` (the oracle/ C restatement on the host cores, same reads).
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0    # MI355X_MICROARCH.md: 8.0 TB/s spec
READ_LEN = 100
MAX_K = 31
METRIC = "aligned reads/sec (100 bp SE, k=20 seed) at 1/2/4/8 GPUs + CPU baseline"

WORKLOADS = {
    # configs[1]: GRCh38 chr21-sized index in HBM, 1M reads on 1 GPU
    "c2": dict(genome_bases=46_709_983, n_contigs=1, reads=1_000_000, families=200, paired_pairs=500_000,
               desc="C2: chr21-sized (46,709,983 bp) synthetic repeat-rich genome, seed-20 index in HBM, "
                    "{reads} x 100 bp SE reads per GPU (configs[1] shape)"),
    # configs[2]: full GRCh38-sized index, 50M reads over 8 GPUs -> the per-GPU shard
    # (its paired leg: configs[3]'s 25M 2 x 101 pairs over 8 GPUs -> 3,125,000 pairs per GPU)
    "c3": dict(genome_bases=3_100_000_000, n_contigs=25, reads=6_250_000, families=2000, paired_pairs=3_125_000,
               desc="C3 per-GPU shard: ~3.1 Gb 25-contig synthetic repeat-rich genome, seed-20 index in HBM, "
                    "{reads} x 100 bp SE reads per GPU (configs[2]: 50M reads / 8 GPUs)"),
}


def algorithmic_bytes(res, ref_probes=None):
    """B_read = 2*readLen + 16 + 12*P + 4*(H + V) + (readLen + MAX_K)*S, in the reference's
    units: P = SNAPHashTable slot probes (12-B entries), which the oracle counts on the same reads
    (`ref_probes`, its records' nProbes; the device counts 64-B bucket lines instead, which only
    granule_bytes prices), a byte genome window per LV-scored candidate.  Without an oracle run P falls back
    to the device's line count at 12 B each (marked in the returned units).  Also returns the same formula
    on the device's own layout: 3-bit genome planes, ceil((readLen + MAX_K) * 3 / 8) bytes per window."""
    H = res["nHitWords"].astype(np.int64).sum()
    V = res["nOverflowLists"].astype(np.int64).sum()
    S = res["nLocationsScored"].astype(np.int64).sum()
    n = len(res)
    if ref_probes is not None:
        P, p_unit = int(np.asarray(ref_probes, dtype=np.int64).sum()), "reference slot probes (oracle, same reads)"
    else:
        P, p_unit = int(res["nProbes"].astype(np.int64).sum()), "device bucket lines (no oracle run: P unpinned)"
    base = n * (2 * READ_LEN + 16) + 12 * P + 4 * (H + V)
    byte_genome = int(base + (READ_LEN + MAX_K) * S)
    planes = int(base + -(-(READ_LEN + MAX_K) * 3 // 8) * S)
    return byte_genome, dict(P=P / n, H=H / n, V=V / n, S=S / n), planes, p_unit


def granule_bytes(res):
    """SURVEY.md 8(d) d3, granule-adjusted: every random access moves whole 64-B lines -- the read's
    bases and qualities, its record, one line per bucket line probed, per overflow list
    ceil(4 H / 64) hit lines (the list length travels in the bucket entry), and per LV-scored candidate the genome window's lines
    (64 * ceil((readLen + MAX_K) / 64), the byte genome of the reference's layout)."""
    P = res["nProbes"].astype(np.int64)
    H = res["nHitWords"].astype(np.int64)
    V = res["nOverflowLists"].astype(np.int64)
    S = res["nLocationsScored"].astype(np.int64)
    line = 64
    per_read = (2 * line * -(-READ_LEN // line) + line + line * P + line * ((4 * H + line - 1) // line) +
                line * -(-(READ_LEN + MAX_K) // line) * S)
    return int(per_read.sum())


def lib_sha256():
    import snapgpu._ffi as F
    h = hashlib.sha256()
    with open(F.LIB_PATH, "rb") as f:
        h.update(f.read())
    return h.hexdigest()


def kernel_source_sha256():
    """Identity of the device code: the HIP sources and headers, the ABI header and the
    Makefile's compiler flags (a rebuild from the same sources elsewhere gives other .so bytes --
    hipcc embeds paths -- but the same kernels)."""
    import glob
    h = hashlib.sha256()
    files = sorted(glob.glob(os.path.join(ROOT, "snap-rnaseq_amd", "csrc", "*.hip")) +
                   glob.glob(os.path.join(ROOT, "snap-rnaseq_amd", "csrc", "*.h")))
    files += [os.path.join(ROOT, "include", "snapgpu.h"), os.path.join(ROOT, "snap-rnaseq_amd", "Makefile")]
    for f in files:
        h.update(os.path.basename(f).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def load_pmc(sha, src_sha):
    """Per-read HBM bytes / VALU instructions of align_kernel<128> from the committed rocprofv3
    PMC summary (profiles/pmc_traffic.json), only if it was collected on this library or on a
    build of the same device sources."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if not os.path.exists(p):
        return None, "no profiles/pmc_traffic.json"
    d = json.load(open(p))
    if d.get("lib_sha256") != sha and d.get("kernel_source_sha256") != src_sha:
        return None, (f"profiles/pmc_traffic.json was collected on another build (library "
                      f"{str(d.get('lib_sha256'))[:12]}, kernel sources {str(d.get('kernel_source_sha256'))[:12]})")
    return d, d.get("source")


def issue_rates():
    """Issue capacity of the CU's pipes, measured by tools/gpu/issue_rates.hip (profiles/r05/issue_rates.json):
    shader cycles per wave64 VALU instruction per SIMD and per SALU instruction per CU once enough waves issue,
    at the occupancy the aligner runs (20 waves per CU).  Without the file: the guide's 2 cycles per wave64
    VALU on a SIMD-32 (MI355X_MICROARCH.md "Wave scheduling") and one SALU per cycle per CU (marked)."""
    p = os.path.join(ROOT, "profiles", "r05", "issue_rates.json")
    if os.path.exists(p):
        d = json.load(open(p))
        rate = {r["instruction"]: r for r in d["rates"]}
        key = "wpc20"
        v = rate["v_add_u32"][key]["cycles_per_instr_per_cu"] * 4   # per SIMD: 4 SIMDs per CU
        sc = rate["s_add_u32"][key]["cycles_per_instr_per_cu"]
        br = rate["s_cmp_eq_u32 + s_cbranch_scc1 (not taken)"][key]["cycles_per_instr_per_cu"]
        return {"valu_cycles_per_simd": v, "salu_cycles_per_cu": sc, "branch_pair_cycles_per_cu": br,
                "source": "profiles/r05/issue_rates.json (tools/gpu/issue_rates.hip, 20 waves per CU)"}
    return {"valu_cycles_per_simd": 2.0, "salu_cycles_per_cu": 1.0, "branch_pair_cycles_per_cu": None,
            "source": "MI355X_MICROARCH.md (2 cycles per wave64 VALU); SALU rate unmeasured"}


def issue_roofline(pmc, reads_launch, kms_launch, n_cu):
    """Instruction-issue roofline of align_kernel<128> (verdict r4 item 3): the PMC instruction counts per read
    of this build (SQ_INSTS_*, exact counts) against what the SIMDs can issue in the measured kernel time.
      valu_pipe_busy   VALU instructions x cycles per wave64 VALU / SIMD-cycles available
      salu_busy        SALU instructions x cycles per SALU per CU / CU-cycles available (the scalar pipe's
                       scope -- per CU or per SIMD -- is what issue_rates.hip measures)
      issue_frac       every instruction (VALU, SALU, branch, LDS, VMEM, SMEM) at one issue slot per SIMD-cycle
    SQ_ACTIVE/WAIT counters are quad-cycles (MI355X_MICROARCH.md): the wave-state shares are ratios of them."""
    if not pmc or not pmc.get("valu_insts_per_read") or not n_cu:
        return None
    rates = issue_rates()
    clk = 2.4e9
    simd_cyc = 4 * n_cu * clk * (kms_launch / 1000.0) / reads_launch   # SIMD-cycles per read
    cu_cyc = simd_cyc / 4
    ins = {k: pmc.get(f"{k}_insts_per_read") for k in ("valu", "salu", "branch", "lds", "vmem", "smem")}
    total = sum(v for v in ins.values() if v)
    valu = ins["valu"] * rates["valu_cycles_per_simd"] / simd_cyc
    salu = ins["salu"] * rates["salu_cycles_per_cu"] / cu_cyc if ins["salu"] else None
    out = {"insts_per_read": {k: (round(v, 1) if v else v) for k, v in ins.items()}, "insts_total_per_read": round(total, 1),
           "simd_cycles_per_read": simd_cyc, "clock_ghz": 2.4, "simds": 4 * n_cu,
           "valu_pipe_busy": valu, "salu_busy": salu, "issue_frac": total / simd_cyc,
           "valu_pipe_busy_guide_2cyc": ins["valu"] * 2.0 / simd_cyc,
           "rates": rates, "wave_state": pmc.get("wave_state"), "source": pmc.get("source")}
    wc = pmc.get("wave_cycles_per_read")
    if wc:
        out["wave_cycles_per_read"] = wc
        out["waves_per_simd_effective"] = wc / simd_cyc
    return out


def cpu_info():
    """Host cores this process can use: the affinity mask, capped by a cgroup CPU quota (the
    GPU boxes expose every core of the host but give each job a quota)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()
        if q != "max":
            quota = int(q) / int(per)
    except (OSError, ValueError):
        try:   # cgroup v1 (csrc/host/threads.cpp reads the same two files)
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            if q > 0 and per > 0:
                quota = q / per
        except (OSError, ValueError):
            pass
    usable = min(aff, int(quota)) if quota else aff
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"nproc": os.cpu_count(), "affinity": aff, "cgroup_quota_cpus": quota, "usable": max(1, usable),
            "model": model}


def log(rank, msg, t0=[time.time()]):
    """Progress on stderr (stdout carries only the JSON line)."""
    if rank == 0:
        print(f"[bench {time.time() - t0[0]:7.1f}s] {msg}", file=sys.stderr, flush=True)


_RESULT_OUT = sys.stdout   # where the one JSON line goes (the real stdout; see _stdout_to_stderr)


def _stdout_to_stderr():
    """stdout carries exactly rank 0's JSON line: everything else written to fd 1 from here on --
    gloo's "[Gloo] Rank i is connected to ..." lines, HIP/ROCm warnings, library prints -- goes to
    stderr, and the line is written to a duplicate of the original stdout."""
    global _RESULT_OUT
    sys.stdout.flush()
    saved = os.dup(1)
    os.dup2(2, 1)
    _RESULT_OUT = os.fdopen(saved, "w")


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def self_launch(args, argv):
    """`python bench.py --gpus N` (N > 1) without a launcher around it: start N rank processes
    through torch.distributed.run (one per GPU, 127.0.0.1 rendezvous) and exit with its code --
    the reference's model is one worker per device over disjoint read ranges
    (ParallelTask.h:127-137).  Runs before anything here imports snapgpu or touches a GPU; the
    ranks inherit stdout, so rank 0's JSON line is this process's output.  Returns only when
    this process is itself a rank (WORLD_SIZE set) or N == 1."""
    if "WORLD_SIZE" in os.environ or args.gpus <= 1:
        return
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    print(f"[bench] launching {args.gpus} ranks: {' '.join(cmd)}", file=sys.stderr, flush=True)
    sys.exit(subprocess.call(cmd, env=env))


def init_distributed():
    """One process per GPU (torch.distributed.run sets RANK/LOCAL_RANK/WORLD_SIZE); gloo
    carries only barriers and the max-over-ranks reduction -- reads are independent, the
    index is replicated, no data-path collective."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo", rank=rank, world_size=world)
    return world, rank, local, dist


def paired_leg(args, idx, local, rank, cpus):
    """SURVEY.md 8(f) f2 (BASELINE configs[3] shape on this workload's genome): wgsim-like
    2 x 101 bp pairs (insert 500 +- 50) through ChimericPairedEndAligner::align on the GPU
    (intersecting kernel, then the single-end fallback), host buffers in and out; the C
    restatement on the job's CPUs beside it, and parity of every record field on a sample."""
    import snapgpu
    n = args.paired_pairs
    r0, r1 = snapgpu.Reads.synthetic_pairs(idx.genome_handle(), n, seed=7 + rank, read_length=101)
    pa = snapgpu.PairedAligner(idx, device=local)
    pa.align(r0, r1)
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        res = pa.align(r0, r1)
        ts.append(time.perf_counter() - t0)
    t0 = time.perf_counter()
    inter = pa.intersect(r0, r1)
    t_int = time.perf_counter() - t0
    dt = float(np.median(ts))
    together = int(res["fromAlignTogether"].sum())
    out = {"value": 2 * n / dt, "unit": "reads/s", "pairs_per_s": n / dt, "pairs": n, "ms_per_batch": dt * 1000.0,
           "intersect_only_ms": t_int * 1000.0, "aligned_together": together, "fallback_pairs": int(n - together),
           "status_pairs": {int(k): int(v) for k, v in zip(*np.unique(res["status"][:, 0], return_counts=True))},
           "deferred_to_pass2": int(((inter["flags"] & snapgpu.PFLAG_DEFERRED) != 0).sum()),
           "params": "paired CLI defaults: maxHits 16000, maxDist 15, 8 seeds, extra 2, spacing 50..1000",
           "workload": args.workload + (" (configs[3] per-GPU shard: 25M pairs / 8 GPUs)" if n == 3_125_000 else ""),
           "boundary": "host pairs in -> host PairedAlignmentResult out (snapgpu_paired_align_batch)"}
    if not args.no_cpu_baseline:
        from oracle_ffi import oracle_paired
        ns = min(n, 200_000)
        s0, s1 = r0.slice(0, ns), r1.slice(0, ns)
        nthr = cpus["usable"]
        c0 = time.perf_counter()
        cres = oracle_paired(idx, s0, s1, pa.params, chimeric=True, n_threads=nthr)
        cdt = time.perf_counter() - c0
        fields = ("status", "location", "direction", "score", "mapq", "fromAlignTogether", "alignedAsPair",
                  "nLocationsScored", "nSingleScored")
        bad = np.zeros(ns, dtype=bool)
        for f in fields:
            bad |= (res[f][:ns] != cres[f]).reshape(ns, -1).any(axis=1)
        out["cpu_baseline"] = {"value": 2 * ns / cdt, "unit": "reads/s", "cores": nthr, "kind": "port",
                               "sample": f"the first {ns} pairs, oracle/snap_oracle.c paired section, {nthr} threads"}
        out["parity"] = {"pairs_compared": ns, "mismatches": int(bad.sum()), "fields": list(fields)}
    return out


def rna_parity(args, pa, ta, gtf, r0, r1, work):
    """One more (untimed) run of the RNA leg writing its SAM file; SHA-256 of its records against
    the reference CLI's own output on the same workload (tests/golden/golden.json "rna_bench",
    made by make_golden.py --only-rna-bench: `snap-rna paired` over blocks of these pairs)."""
    import snapgpu
    ref = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json"))).get("rna_bench")
    if not ref:
        return {"compared": False, "why": "no rna_bench digest in tests/golden/golden.json"}
    if args.workload != "c2" or args.genome_bases or ref["pairs"] != args.rna_pairs:
        return {"compared": False, "why": "the reference digest covers the default C2 workload with "
                                          f"{ref['pairs']} pairs only"}
    sam = os.path.join(work, "rna_parity.sam")
    gtf.reset_counts()
    snapgpu.rna_paired_align(pa, ta, gtf, r0, r1, sam)
    drop = {f"rp{i}" for i in ref["dropped_pairs"]}
    h = hashlib.sha256()
    nrec = 0
    with open(sam) as f:
        for line in f:
            if line.startswith("@") or line.split("\t", 1)[0] in drop:
                continue
            h.update(line.encode())
            nrec += 1
    os.unlink(sam)
    return {"compared": True, "records": nrec, "reference_records": ref["records"],
            "sha256_match": h.hexdigest() == ref["sha256"], "reference_runs": ref["reference_runs"],
            "dropped_pairs": len(ref["dropped_pairs"]),
            "what": "SAM records of the whole batch vs the reference CLI (`snap-rna paired -t 1`) on the same "
                    "pairs, genome, GTF"}


def rna_roofline(ta, r0, tidx=None, n_threads=1):
    """Roofline of the RNA leg's dominant kernel, align_kernel<256> (the 2 x 150 mates' pass), on the
    transcriptome aligner over end 0 (untimed extra call): SURVEY 8(d) d3 algorithmic bytes of the
    records (each read at its own length) / the pass-2+3 kernel time (HIP events).  P is in the
    headline's unit: the reference's SNAPHashTable slot probes at 12 B, counted by the oracle on the
    same reads with the same parameters (`tidx` given: the CPU-baseline leg), else the device's bucket
    lines at 12 B each (marked unpinned)."""
    res = ta.AlignReads(r0)
    ks, ovf = [], 0
    for _ in range(3):
        ta.AlignReads(r0, out=res)
        t = ta.timing()
        ks.append(t["spillKernelMs"])
        ovf = int(t["nArenaOverflow"])
    lens = np.array([len(r0.get(i)[0]) for i in range(r0.n)], dtype=np.int64)
    P = res["nProbes"].astype(np.int64)
    p_unit = "device bucket lines at 12 B (no oracle run: P unpinned)"
    if tidx is not None:
        from oracle_ffi import mismatches, oracle_align
        c0 = time.perf_counter()
        cres = oracle_align(tidx, r0, ta.params, n_threads=n_threads)
        oracle_s = time.perf_counter() - c0
        bad = int(len(mismatches(res, cres)))
        P = cres["nProbes"].astype(np.int64)
        p_unit = (f"reference slot probes at 12 B (oracle on the same {r0.n} reads, {oracle_s:.1f} s on "
                  f"{n_threads} threads; {bad} records differ from the GPU's)")
    H = res["nHitWords"].astype(np.int64)
    V = res["nOverflowLists"].astype(np.int64)
    S = res["nLocationsScored"].astype(np.int64)
    b = int((2 * lens + 16 + 12 * P + 4 * (H + V) + (lens + MAX_K) * S).sum())
    b_planes = int((2 * lens + 16 + 12 * P + 4 * (H + V) + -(-(lens + MAX_K) * 3 // 8) * S).sum())
    ms = float(min(ks))
    return {"kernel": "align_kernel<256, false> (+ the <512> byte pass and the big-arena pass over the reads "
                      "that outgrew a capped arena)", "reads": int(r0.n), "arena_overflow_reads": ovf,
            "kernel_ms": ms, "algorithmic_bytes": b, "achieved": b / (ms / 1000.0) / 1e9, "peak": HBM_PEAK_GBS,
            "unit": "GB/s", "frac": b / (ms / 1000.0) / 1e9 / HBM_PEAK_GBS,
            "per_read": {"P": float(P.mean()), "H": float(H.mean()), "V": float(V.mean()), "S": float(S.mean())},
            "algorithmic_bytes_note": "SURVEY 8(d) d3 in the headline's units: P = " + p_unit + ", a byte-genome "
                                      "window of readLen + MAX_K bytes per scored candidate",
            "plane_layout": {"algorithmic_bytes": b_planes, "frac": b_planes / (ms / 1000.0) / 1e9 / HBM_PEAK_GBS,
                             "note": "the same formula on the 3-bit genome planes the device reads"},
            "params": "transcriptome aligner of the RNA path: maxHits 16000, maxK 15, 8 seeds, extra 2",
            "note": "end 0 of the batch through snapgpu_align_batch (plain AlignRead; the product path's "
                    "multi-hit calls run the EXT twin of the same kernel)"}


def rna_cpu_baseline(args):
    """configs[4]'s CPU baseline: the reference CLI itself (`snap-rna paired -t T`) on a sample of this
    leg's workload, timed by its own stats line in the build container (tests/golden/rna_cpu_baseline.py;
    the reference does not travel to the GPU box).  Only for the default C2 workload it was run on."""
    path = os.path.join(ROOT, "tests", "golden", "rna_cpu_baseline.json")
    if not os.path.exists(path) or args.workload != "c2" or args.genome_bases:
        return None
    runs = json.load(open(path))
    out = {}
    for key, r in sorted(runs.items()):
        out[key] = {x: r.get(x) for x in ("value", "unit", "cores", "kind", "sample", "host", "crashed_blocks",
                                          "base_aligner_opt", "records_equal_to_O0")}
    # the headline: one thread, BaseAligner.cpp at the highest optimisation that completes (clang -O3
    # -fno-strict-return; every g++ level above -O0 aborts on CharacterizeSeeds' missing return)
    one = runs.get("threads_1_O3c") or runs.get("threads_1")
    if one:
        out.update({x: one.get(x) for x in ("value", "unit", "cores", "kind", "sample", "base_aligner_opt")})
        out["note"] = ("snap-rna's own build of BaseAligner.cpp at -O0 is listed as threads_1; g++ -O1/-O2/-O3 "
                       "builds abort ('double free') on every block (oracle/Makefile.ref rna-variants)")
    return out


def single_leg(args, idx, local, build_threads):
    """SURVEY.md 8(f) f1, timed (verdict r5 #4): the `snap-rna single` product path (SingleAligner.cpp:
    140-320; the reference's product metric is this end-to-end Reads/s, AlignerContext.cpp:382-393) on the
    C2 genome, the RNA leg's 2,000-gene GTF and transcriptome, and 1M 100-bp single-end reads
    (tests/rna_synth.py): host FASTQ file in -> SAM file out.  Timed per call: FASTQ parsing
    (snapgpu_reads_from_fastq) + snapgpu_single_align (clipping, pre-filter, transcriptome and genome
    AlignRead batches, AlignmentFilter::FilterSingle, both CIGAR batches, splice junctions, SAM lines,
    the file write, gene read counts); median of 3 calls after a warm-up.  Parity: SHA-256 of the SAM
    records against the reference CLI's own output on the same reads (golden.json "single_bench",
    tests/golden/make_golden.py --only-single-bench)."""
    import shutil
    import tempfile
    import snapgpu
    from rna_synth import synth_single_reads
    work = tempfile.mkdtemp(prefix="snapgpu_single_", dir="/dev/shm" if os.path.isdir("/dev/shm") else None)
    try:
        t0 = time.time()
        gtf_path, fq, info = synth_single_reads(idx.genome_handle(), work, n_reads=args.single_reads)
        gtf = snapgpu.Gtf.load(gtf_path)
        tfa = os.path.join(work, "transcriptome.fa")
        gtf.write_transcriptome(idx.genome_handle(), tfa)
        tidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(tfa, 500), 20, build_threads)
        t_prep = time.time() - t0
        ga = snapgpu.BaseAligner(idx, device=local)     # `snap-rna single` defaults for both aligners
        ta = snapgpu.BaseAligner(tidx, device=local)
        sam = os.path.join(work, "out.sam")
        ts, sts, parse = [], [], []
        for it in range(4):   # a warm-up, then 3 timed calls
            gtf.reset_counts()
            c0 = time.perf_counter()
            reads = snapgpu.Reads.from_fastq(fq)
            c1 = time.perf_counter()
            st = snapgpu.single_align(ga, ta, gtf, reads, sam)
            c2 = time.perf_counter()
            del reads
            if it:
                ts.append(c2 - c0)
                parse.append(c1 - c0)
                sts.append(st)
        k = int(np.argsort(ts)[1])
        dt, st = ts[k], sts[k]
        n = int(st["totalReads"])
        kern = {}
        for name, al in (("transcriptome", ta), ("genome", ga)):   # the last call's GPU passes per aligner
            t = al.timing()
            kern[name] = {"align_kernel_busy_ms": round(t["mainKernelBusyMs"], 2), "lookup_busy_ms": round(t["lookupKernelBusyMs"], 2),
                          "call_wall_ms": round(t["wallMs"], 2)}
        ref = json.load(open(os.path.join(ROOT, "tests", "golden", "golden.json"))).get("single_bench")
        if not ref:
            parity = {"compared": False, "why": "no single_bench digest in tests/golden/golden.json"}
        elif args.workload != "c2" or args.genome_bases or ref["reads"] != args.single_reads:
            parity = {"compared": False, "why": f"the reference digest covers the default C2 workload with "
                                                f"{ref['reads']} reads only"}
        else:
            drop = {f"rp{i}" for i in ref["dropped_reads"]}
            h = hashlib.sha256()
            nrec = 0
            with open(sam) as f:
                for line in f:
                    if line.startswith("@") or line.split("\t", 1)[0].split("/")[0] in drop:
                        continue
                    h.update(line.encode())
                    nrec += 1
            parity = {"compared": True, "records": nrec, "reference_records": ref["records"],
                      "sha256_match": h.hexdigest() == ref["sha256"], "reference_runs": ref["reference_runs"],
                      "dropped_reads": len(ref["dropped_reads"]),
                      "what": "SAM records of the whole batch vs the reference CLI (`snap-rna single -t 1`) on the "
                              "same reads, genome, GTF"}
        cpu = None
        if ref and args.workload == "c2" and not args.genome_bases:
            cb = ref.get("cpu_baseline") or {}
            one = cb.get("threads_1")
            if one:
                cpu = {x: one.get(x) for x in ("value", "unit", "cores", "kind", "sample", "base_aligner_opt",
                                               "records_equal_to_O0")}
                cpu["threads_8"] = {x: (cb.get("threads_8") or {}).get(x) for x in ("value", "cores", "sample")}
        return {"value": n / dt, "unit": "reads/s", "reads": n, "ms_per_batch": dt * 1e3,
                "read_len": 100, "workload": info, "transcriptome_bases": tidx.info()["nBases"],
                "stage_ms": {"fastq_parse": round(float(parse[k]) * 1e3, 2),
                             **{x: round(st[x], 2) for x in ("prepMs", "alignMs", "filterMs", "cigarMs", "writeMs",
                                                              "formatMs", "ioMs", "wallMs")}},
                "records": {x: int(st[x]) for x in ("usefulReads", "singleHits", "multiHits", "notFound",
                                                    "transcriptomeRecords")},
                "aligners": kern,
                "sam_bytes": os.path.getsize(sam), "prep_s": round(t_prep, 1),
                "parity": parity, "cpu_baseline": cpu,
                "params": "`snap-rna single` defaults: both aligners maxHits 300, maxK 14, 25 seeds, extra 2; "
                          "filter maxDist 14, confDiff 2",
                "boundary": "host FASTQ file in -> SAM file out (" + ("/dev/shm" if work.startswith("/dev/shm")
                                                                       else "temp dir") + "), the gene read counters "
                            "advanced (snapgpu_reads_from_fastq + snapgpu_single_align)"}
    finally:
        shutil.rmtree(work, ignore_errors=True)


def rna_leg(args, idx, local, build_threads):
    """SURVEY.md 8(f) f4 (BASELINE configs[4] shape on this workload's genome): the RNA paired
    product path (`snap-rna paired`: transcriptome multi-hit + chimeric genome aligners,
    AlignmentFilter::Filter with the GPU seed census, GPU CIGARs, SAM lines, GTF read counts) on
    a synthetic GTF (2,000 genes) and 2 x 150 bp pairs, host FASTQ batches in -> SAM lines out."""
    import shutil
    import tempfile
    import snapgpu
    from rna_synth import synth_rna_workload
    work = tempfile.mkdtemp(prefix="snapgpu_rna_")
    try:
        t0 = time.time()
        gtf_path, fq0, fq1, info = synth_rna_workload(idx.genome_handle(), work, n_pairs=args.rna_pairs)
        gtf = snapgpu.Gtf.load(gtf_path)
        tfa = os.path.join(work, "transcriptome.fa")
        gtf.write_transcriptome(idx.genome_handle(), tfa)
        tidx = snapgpu.GenomeIndex.build(snapgpu.Genome.from_fasta(tfa, 500), 20, build_threads)
        t_prep = time.time() - t0
        pa = snapgpu.PairedAligner(idx, device=local)
        ta = snapgpu.BaseAligner(tidx, maxHitsToConsider=16000, maxK=15, maxSeedsToUse=8, extraSearchDepth=2,
                                 device=local)
        r0, r1 = snapgpu.Reads.from_fastq(fq0), snapgpu.Reads.from_fastq(fq1)
        snapgpu.rna_paired_align(pa, ta, gtf, r0, r1)   # warm-up
        ts, sts = [], []
        for _ in range(3):
            gtf.reset_counts()
            c0 = time.perf_counter()
            res, st = snapgpu.rna_paired_align(pa, ta, gtf, r0, r1)
            ts.append(time.perf_counter() - c0)
            sts.append(st)
        k = int(np.argsort(ts)[1])
        dt, st = ts[k], sts[k]
        n = r0.n
        parity = rna_parity(args, pa, ta, gtf, r0, r1, work)
        roof = rna_roofline(ta, r0, None if args.no_cpu_baseline else tidx, build_threads)
        return {"parity": parity, "roofline": roof, "cpu_baseline": rna_cpu_baseline(args), "value": 2 * n / dt, "unit": "reads/s", "pairs_per_s": n / dt, "pairs": n, "ms_per_batch": dt * 1e3,
                "read_len": 150, "workload": info, "transcriptome_bases": tidx.info()["nBases"],
                "stage_ms": {x: round(st[x], 2) for x in ("prepMs", "alignMs", "filterMs", "seedMs", "countMs", "cigarMs",
                                                          "writeMs", "wallMs")},
                "sub_batches": st["subBatches"],
                "stage_note": "stage times are sums over the pipelined sub-batches (stage A: the GPU aligners of "
                              "sub-batch s+1 overlaps stage B: filter, seed census, CIGARs, records of s)",
                "records": {x: st[x] for x in ("singleHits", "multiHits", "notFound", "transcriptomeRecords")},
                "partial_pairs": st["partialPairs"], "partial_matches": st["partialMatches"],
                "seed_runs": st["seedRuns"], "prep_s": round(t_prep, 1),
                "boundary": "host FASTQ batches in -> SAM lines + read counters (snapgpu_rna_paired_align; "
                            "lines formatted, not written to disk)"}
    finally:
        shutil.rmtree(work, ignore_errors=True)


def timed_steps(step, steps, dist, sync, own=None):
    """Barrier + sync on both sides of exactly `steps` steps; returns the max over ranks (this
    rank's own time is appended to `own` when given)."""
    if dist:
        dist.barrier()
    sync()
    t_start = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    t_end = time.perf_counter()
    if dist:
        dist.barrier()
    elapsed = t_end - t_start
    if own is not None:
        own.append(elapsed)
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def gather_per_rank(dist, world, mine):
    """Every rank's own figures (reads/s on its shard, its index upload time, ...) on every rank
    (gloo all_gather_object; not on the data path)."""
    if not dist:
        return [mine]
    got = [None] * world
    dist.all_gather_object(got, mine)
    return got


def shard_tag(reads):
    """Short identity of a rank's read shard (its first read's bases)."""
    return hashlib.sha256(bytes(reads.get(0)[0])).hexdigest()[:16]


def standin_main(args, wl, world, rank, local, dist):
    """--oracle-standin: the launch / sharding / index-sharing / reduction path of an N-rank run
    with the CPU oracle in place of the GPU aligner, so the CPU suite can check `bench.py --gpus N`
    end to end (tests/test_multirank.py).  Never a measurement: the line says so."""
    import snapgpu
    from snapgpu import shared_index
    from oracle_ffi import oracle_align
    gen = dict(seed=2121, n_contigs=wl["n_contigs"], n_repeat_families=wl["families"])
    idx, index_info = shared_index.build_once(snapgpu, wl["genome_bases"], gen, 20, 2, rank, world, dist)
    reads = snapgpu.Reads.synthetic(idx.genome_handle(), wl["reads"], seed=99 + rank)
    params = snapgpu.default_params()
    box = {}

    def step():
        box["res"] = oracle_align(idx, reads, params, n_threads=1)

    for _ in range(args.warmup):
        step()
    own = []
    elapsed = timed_steps(step, args.steps, dist, lambda: None, own)
    per_rank = gather_per_rank(dist, world, {
        "rank": rank, "device": None, "reads": wl["reads"], "elapsed_s": round(own[0], 4),
        "reads_per_s": wl["reads"] * args.steps / own[0], "index_built_here": bool(index_info.get("built_by_this_rank")),
        "index_attached": bool(index_info.get("attached")), "shared_file": index_info.get("shared_file"),
        "shard_first_read": shard_tag(reads),
        "single_hits": int((box["res"]["result"] == snapgpu.SingleHit).sum())})
    result = None
    if rank == 0:
        result = {"metric": METRIC, "value": wl["reads"] * world * args.steps / elapsed, "unit": "reads/s",
                  "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                  "ms_per_step": elapsed * 1000.0 / args.steps, "higher_is_better": True, "scaling": "weak",
                  "vs_baseline": None, "dtype": "u8",
                  "standin": "oracle (CPU test of the N-rank launch path; NOT a GPU measurement)",
                  "data": "synthetic", "config": {"workload": args.workload, "genome_bases": wl["genome_bases"],
                                                  "reads_per_gpu": wl["reads"], "index": index_info,
                                                  "per_rank": per_rank}}
        print(json.dumps(result), file=_RESULT_OUT, flush=True)
    if dist:
        dist.barrier()
        shared_index.cleanup(rank, world)
        dist.destroy_process_group()
    return result


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--reads", type=int, default=None, help="reads per GPU (default: the workload's)")
    ap.add_argument("--genome-bases", type=int, default=None)
    ap.add_argument("--resident-steps", type=int, default=5)
    ap.add_argument("--paired-pairs", type=int, default=None,
                    help="extras.paired: 2 x 101 bp pairs through the GPU ChimericPairedEndAligner (0: skip; default: "
                         "the workload's -- 500k on c2, configs[3]'s per-GPU shard of 3,125,000 on c3)")
    ap.add_argument("--rna-pairs", type=int, default=100_000,
                    help="extras.rna_paired: 2 x 150 bp pairs through the RNA paired product path (0: skip)")
    ap.add_argument("--single-reads", type=int, default=1_000_000,
                    help="reads of the `snap-rna single` product-path leg (extras.single_e2e; 0 = skip)")
    ap.add_argument("--mode", choices=("stream", "sync"), default="stream",
                    help="stream: submit every step, wait once (a streaming caller); sync: one blocking call per step")
    ap.add_argument("--cpu-sample", type=int, default=1_000_000, help="reads timed on the CPU baseline")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extras", action="store_true", help="skip ceilings, CIGAR/SAM and parity legs")
    ap.add_argument("--oracle-standin", action="store_true",
                    help="CPU test of the N-rank launch path only: each rank runs the oracle/ restatement on its "
                         "shard instead of the GPU aligner; the line is marked `standin` and is not a measurement")
    args = ap.parse_args()
    self_launch(args, sys.argv[1:])
    _stdout_to_stderr()
    wl = dict(WORKLOADS[args.workload])
    if args.paired_pairs is None:
        args.paired_pairs = wl["paired_pairs"]
    if args.reads:
        wl["reads"] = args.reads
    if args.genome_bases:
        wl["genome_bases"] = args.genome_bases

    world, rank, local, dist = init_distributed()
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but {world} rank(s) were launched (WORLD_SIZE); refusing to report "
              f"a {world}-GPU run as {args.gpus}", file=sys.stderr, flush=True)
        if dist:
            dist.destroy_process_group()
        sys.exit(2)
    if args.oracle_standin:
        return standin_main(args, wl, world, rank, local, dist)

    import snapgpu
    from snapgpu import shared_index
    cpus = cpu_info()
    build_threads = min(cpus["usable"], 64)
    t0 = time.time()
    gen = dict(seed=2121, n_contigs=wl["n_contigs"], n_repeat_families=wl["families"])
    log(rank, f"workload {args.workload}: genome + index ({wl['genome_bases']} bases, {build_threads} threads)")
    idx, index_info = shared_index.build_once(snapgpu, wl["genome_bases"], gen, 20, build_threads, rank, world, dist)
    t_index = time.time() - t0
    log(rank, f"index ready {index_info}")
    # one GPU per local rank; more ranks than GPUs (a multi-rank rehearsal on a smaller box) share them
    ndev = snapgpu.device_count()
    if ndev > 0:
        local = local % ndev
    t1 = time.time()
    aligner = snapgpu.BaseAligner(idx, device=local)   # index + genome upload to this GPU's HBM
    t_upload = time.time() - t1
    log(rank, f"index uploaded in {t_upload:.1f}s")
    # rank r aligns shard r of a world x reads batch (its own read-generator seed: disjoint shards)
    reads = snapgpu.Reads.synthetic(idx.genome_handle(), wl["reads"], seed=99 + rank)
    out = np.zeros(wl["reads"], dtype=snapgpu.RESULT_DTYPE)
    log(rank, f"{wl['reads']} reads generated")

    outs = [out, np.zeros(wl["reads"], dtype=snapgpu.RESULT_DTYPE)]
    for _ in range(args.warmup):
        aligner.AlignReads(reads, out=out)
    kernel_ms, lookup_ms, launches, fix_ms, busy_ms, lk_busy_ms = [], [], [], [], [], []

    def record(t, k):
        kernel_ms.append(t["mainKernelMs"] / k)
        lookup_ms.append(t["lookupKernelMs"] / k)
        launches.append(t["nLaunches"] / k)
        fix_ms.append(t["fixupMs"] / k)
        busy_ms.append(t["mainKernelBusyMs"] / k)
        lk_busy_ms.append(t["lookupKernelBusyMs"] / k)

    if args.mode == "stream":
        # a streaming caller: batch k+1 is submitted while batch k's last chunks are on the GPU
        # (snapgpu_align_batch_submit), records land in alternating host arrays, one wait at the end
        n_sub = [0]

        def step():
            aligner.submit(reads, outs[n_sub[0] & 1])
            n_sub[0] += 1

        def sync():
            aligner.wait()
            if n_sub[0]:
                record(aligner.timing(), n_sub[0])
                n_sub[0] = 0
    else:
        def step():
            aligner.AlignReads(reads, out=out)
            record(aligner.timing(), 1)

        def sync():
            pass

    own = []
    elapsed = timed_steps(step, args.steps, dist, sync, own)
    if args.mode == "stream":
        assert np.array_equal(outs[0].view(np.uint8), outs[1].view(np.uint8))
    log(rank, f"timed {args.steps} steps: {elapsed:.3f}s")
    res = out
    total_reads = wl["reads"] * world * args.steps
    value = total_reads / elapsed
    ms_per_step = elapsed * 1000.0 / args.steps
    per_rank = gather_per_rank(dist, world, {
        "rank": rank, "device": local, "reads": wl["reads"], "elapsed_s": round(own[0], 4),
        "reads_per_s": wl["reads"] * args.steps / own[0], "index_upload_s": round(t_upload, 2),
        "index_built_here": bool(index_info.get("built_by_this_rank")), "index_attached": bool(index_info.get("attached")),
        "shard_first_read": shard_tag(reads)})

    result = None
    if rank == 0:
        counts = {int(k): int(v) for k, v in zip(*np.unique(res["result"], return_counts=True))}
        extras = {}
        copy_peak_gbs = None
        if not args.no_extras:
            # device-resident rate: the same pass sets without the copies or the host tail
            dev = aligner.upload(reads)
            dev.run()
            dev.synchronize()
            r0 = time.perf_counter()
            for _ in range(args.resident_steps):
                dev.run()
            dev.synchronize()
            r_s = time.perf_counter() - r0
            rres = dev.results()
            extras["resident"] = {"value": wl["reads"] * args.resident_steps / r_s, "unit": "reads/s",
                                  "ms_per_step": r_s * 1000.0 / args.resident_steps,
                                  "same_results": bool(np.array_equal(rres.view(np.uint8), res.view(np.uint8))),
                                  "note": "reads already in HBM, records left in HBM (snapgpu_align_resident)"}
            # seed_lookup_kernel (pass 0) measured with the two streams' pass sets serialised, so
            # no align kernel shares the GPU with it: read bytes + offsets/lengths + 16 records of
            # 16 B per read, then per looked-up seed its table's (bucket base, count), 64 B per
            # bucket line loaded, 4 B per saturated overflow count re-read from its list
            # (own lists: `launches` / `busy_ms` of the timed steps feed the align kernel's roofline)
            aligner.set_overlap(False)
            lk_busy_ms, lk_launches = [], []
            for _ in range(3):
                dev.run()
                dev.synchronize()
                t = aligner.timing()
                lk_busy_ms.append(t["lookupKernelBusyMs"])
                lk_launches.append(t["nLaunches"])
            aligner.set_overlap(True)
            lk_bytes = int(wl["reads"] * (READ_LEN + 12 + 256) + 12 * t["lookupSeeds"] + 64 * t["lookupProbes"] +
                           4 * t["lookupOverflowReads"]) / t["nLaunches"]
            lk_s = float(np.mean(lk_busy_ms)) / float(np.mean(lk_launches)) / 1000.0
            lookup = {"kernel": "seed_lookup_kernel", "kernel_ms_per_launch": lk_s * 1000.0,
                      "achieved": lk_bytes / lk_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": lk_bytes / lk_s / 1e9 / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": lk_bytes,
                      "seeds_per_launch": t["lookupSeeds"] / t["nLaunches"],
                      "probes_per_launch": t["lookupProbes"] / t["nLaunches"],
                      # pass 0 looks up SEEDS_PER_READ (16) seeds of every read speculatively; a read
                      # applies fewer (the reference stops after <= 13 lookups), so its record's nProbes
                      # (the probes of the seeds it used, from pass 0's records or probed in the align
                      # kernel) is not pass 0's count plus an in-kernel remainder: both are reported
                      "pass0_probes_per_read": t["lookupProbes"] / len(res),
                      "pass0_probes_per_seed": t["lookupProbes"] / max(1, t["lookupSeeds"]),
                      "applied_probes_per_read": float(res["nProbes"].astype(np.int64).sum()) / len(res)}
            # measured ceilings: random 64-B bucket-line gathers from the resident image (2^28 lines) and a
            # streaming copy (4 GiB read + 4 GiB written)
            n_g = 1 << 28
            g_ms = aligner.gather_peak_ms(n_g)
            lookup["gather_peak"] = {"loads": n_g, "ms": g_ms, "loads_per_s": n_g / (g_ms / 1000.0),
                                     "note": "independent random 64-B bucket-line loads, best of 3"}
            lookup["bucket_image"] = aligner.bucket_info()
            lookup["probe_rate_frac_of_gather_peak"] = (lookup["probes_per_launch"] / lk_s) / (n_g / (g_ms / 1000.0))
            c_bytes = 4 << 30
            c_ms = aligner.copy_peak_ms(c_bytes)
            copy_gbs = 2 * c_bytes / (c_ms / 1000.0) / 1e9
            extras["copy_peak"] = {"GBps": copy_gbs, "ms": c_ms, "bytes_moved": 2 * c_bytes,
                                   "note": "copy_peak_kernel, 16-B loads + stores, best of 3"}
            copy_peak_gbs = copy_gbs
            lookup["frac_of_measured_copy_peak"] = lookup["achieved"] / copy_gbs
            extras["lookup_roofline"] = lookup
            # SAM records: GPU CIGARs of the resident records, then host SAM lines
            cig_ms = []
            for _ in range(3):
                dev.run_cigars()
                cig_ms.append(aligner.cigar_ms())
            cig = dev.cigars()
            cig_bytes = wl["reads"] * (8 + 4 + 64 + READ_LEN + READ_LEN + 128 + 4 + 4 + 256)
            cig_s = float(np.mean(cig_ms)) / 1000.0
            ids = [f"read{i}" for i in range(wl["reads"])]
            s0 = time.perf_counter()
            sam_t = {}
            sam = snapgpu.sam_format(idx, reads, ids, res, cig, timing=sam_t)
            sam_s = time.perf_counter() - s0
            extras["sam_records"] = {"kernel": "cigar_kernel", "kernel_ms": cig_s * 1000.0,
                                     "reads_per_s": wl["reads"] / cig_s,
                                     "with_cigar": int((cig.editDistance >= 0).sum()),
                                     "achieved": cig_bytes / cig_s / 1e9, "unit": "GB/s",
                                     "frac": cig_bytes / cig_s / 1e9 / HBM_PEAK_GBS,
                                     "sam_format_reads_per_s": wl["reads"] / sam_t["format_s"],
                                     "sam_format_note": "snapgpu_sam_format (host threads) alone; with the Python "
                                                        "id/buffer plumbing around it: "
                                                        f"{wl['reads'] / sam_s / 1e6:.2f} M lines/s",
                                     "sam_bytes": len(sam)}
            del sam, dev
            if args.paired_pairs:
                extras["paired"] = paired_leg(args, idx, local, rank, cpus)
            if args.single_reads:
                extras["single_e2e"] = single_leg(args, idx, local, build_threads)
                log(rank, "single_e2e done")
            if args.rna_pairs:
                extras["rna_paired"] = rna_leg(args, idx, local, build_threads)
        log(rank, "extras done")
        cpu = None
        parity = None
        if not args.no_cpu_baseline and world == 1:   # CPU baseline: rank 0 at N=1 only
            from oracle_ffi import mismatches, oracle_align
            nthr = cpus["usable"]
            ns = min(args.cpu_sample, wl["reads"])
            sample = reads if ns == wl["reads"] else reads.slice(0, ns)
            c0 = time.perf_counter()
            cres = oracle_align(idx, sample, aligner.params, n_threads=nthr)
            cdt = time.perf_counter() - c0
            cpu = {"value": ns / cdt, "unit": "reads/s", "cores": nthr, "kind": "port",
                   "sample": f"the first {ns} reads of the rank-0 shard of the timed workload, oracle/snap_oracle.c "
                             f"(bit-exact C restatement of BaseAligner, calibrated at 1.01x the reference's speed), "
                             f"{nthr} threads, {cdt:.2f} s wall",
                   "per_core_reads_per_s": ns / cdt / nthr, "host": cpus,
                   "note": "cores = the CPUs this job may use (affinity mask capped by the cgroup quota); "
                           "nproc counts the whole host"}
            parity = {"reads_compared": ns, "mismatches": int(len(mismatches(res[:ns], cres))),
                      "against": "oracle/snap_oracle.c (pinned bit-exact to the compiled reference by "
                                 "tests/test_oracle_golden.py)" + (
                                     "; the reference's own digest of all C2 records is tests/test_gpu_golden.py's"
                                     if args.workload == "c2" else
                                     "; no reference digest at this size (the compiled reference needs more RAM "
                                     "than the build container has)")}
            if "sam_records" in extras:   # CIGAR parity on a 20k-read sample
                from oracle_ffi import oracle_cigars
                nc = min(20000, wl["reads"])
                loc, dirs = snapgpu.cigar_inputs(res[:nc])
                want = oracle_cigars(idx, [reads.get(i)[0] for i in range(nc)], loc, dirs, 0)
                extras["sam_records"]["parity"] = {"reads_compared": nc, "mismatches": sum(
                    1 for i in range(nc) if (int(cig.editDistance[i]), cig.string(i)) != want[i])}
        # ---- roofline of the dominant kernel (after the CPU leg: its oracle run counts the reference's
        # own slot probes on these reads, the P of the algorithmic bytes)
        sha = lib_sha256()
        src_sha = kernel_source_sha256()
        ref_probes = cres["nProbes"] if cpu is not None and len(cres) == len(res) else None
        bytes_all, per_read, bytes_planes, p_unit = algorithmic_bytes(res, ref_probes)
        n_launch = float(np.mean(launches))
        bytes_launch = bytes_all / n_launch
        # the two lanes' launches overlap (one fills the other's tail): a launch's own HIP-event
        # duration (= rocprof's per-dispatch duration) double-counts the shared time, so the
        # roofline uses the align kernel's GPU-busy time per step (union of the launch intervals)
        kms_launch_own = float(np.sum(kernel_ms)) / float(np.sum(launches))
        busy_step = float(np.mean(busy_ms))
        kms_launch = busy_step / n_launch
        achieved = bytes_launch / (kms_launch / 1000.0) / 1e9
        pmc, pmc_src = load_pmc(sha, src_sha)
        reads_launch = wl["reads"] / n_launch
        traffic = pmc["hbm_bytes_per_read"] * reads_launch if pmc else None
        issue = issue_roofline(pmc, reads_launch, kms_launch, snapgpu.device_cu_count(local))
        if issue:
            ws = issue.get("wave_state") or {}
            binding = (f"instruction issue and dependent latency, not HBM (frac below) and not MFMA (no matrix work): "
                       f"{issue['insts_total_per_read']:.0f} instructions per read ({issue['insts_per_read']['valu']:.0f} VALU, "
                       f"{issue['insts_per_read']['salu']:.0f} SALU, {issue['insts_per_read']['branch']:.0f} branch) fill "
                       f"{issue['issue_frac']:.2f} of the SIMDs' issue slots (one per SIMD-cycle); the VALU pipe is "
                       f"{issue['valu_pipe_busy']:.2f} busy at {issue['rates']['valu_cycles_per_simd']:.2f} cycles per wave64 "
                       f"instruction, the scalar pipe {issue['salu_busy']:.2f} at {issue['rates']['salu_cycles_per_cu']:.2f} "
                       f"cycles per SALU per CU ({issue['rates']['source']}); waves spend "
                       f"{ws.get('SQ_WAIT_ANY', 0):.0%} of their time waiting on memory counters, "
                       f"{ws.get('SQ_WAIT_INST_ANY', 0):.0%} on dependencies, {ws.get('SQ_ACTIVE_INST_ANY', 0):.0%} issuing "
                       "(DESIGN.md section 4)")
        else:
            binding = ("instruction issue and dependent latency (DESIGN.md section 4), not HBM bandwidth (no PMC data of "
                       "this build: " + str(pmc_src) + ")")
        granule = granule_bytes(res)
        roofline = {"bound": "issue", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                    "bound_note": "the kernel is bound by neither HBM nor MFMA: `bound` names what binds "
                                  "(binding_resource, issue_roofline); achieved / peak / frac / traffic are the "
                                  "contract's HBM roofline of the same launches",
                    "issue_roofline": issue,
                    "kernel": "align_kernel<128, false>", "kernel_ms_per_launch": kms_launch,
                    "kernel_busy_ms_per_step": busy_step,
                    "launch_duration_ms": kms_launch_own,
                    "achieved_on_launch_durations": bytes_launch / (kms_launch_own / 1000.0) / 1e9,
                    "timing_note": "kernel_ms_per_launch = union of the step's align-kernel launch intervals / "
                                   "launches (HIP events); launch_duration_ms = mean of each launch's own "
                                   "interval (what rocprofv3 reports per dispatch; launches of the two "
                                   "streams overlap)",
                    "algorithmic_bytes_note": "SURVEY 8(d) d3 in the reference's units: P = " + p_unit +
                                              " at 12 B, a byte-genome window of readLen + MAX_K bytes per scored "
                                              "candidate (round 4 charged 64 B per device bucket line instead)",
                    "plane_layout": {"bytes_per_read": bytes_planes / len(res),
                                     "achieved": bytes_planes / n_launch / (kms_launch / 1000.0) / 1e9,
                                     "frac": bytes_planes / n_launch / (kms_launch / 1000.0) / 1e9 / HBM_PEAK_GBS,
                                     "note": "the same formula on the layout the device reads: 3-bit genome planes, "
                                             "ceil(131 * 3 / 8) = 50 B per window"},
                    "granule_adjusted": {"bytes_per_read": granule / len(res),
                                         "achieved": granule / n_launch / (kms_launch / 1000.0) / 1e9,
                                         "frac": granule / n_launch / (kms_launch / 1000.0) / 1e9 / HBM_PEAK_GBS,
                                         "note": "64-B lines per random access, device bucket lines (SURVEY 8(d) d3)"},
                    "launches_per_step": n_launch, "reads_per_launch": reads_launch,
                    "algorithmic_bytes_per_launch": bytes_launch, "algorithmic_bytes_per_read": bytes_all / len(res),
                    "binding_resource": binding,
                    "pmc_source": pmc_src, "lib_sha256": sha, "kernel_source_sha256": src_sha}
        if copy_peak_gbs:
            roofline["frac_of_measured_copy_peak"] = achieved / copy_peak_gbs
        result = {
            "metric": METRIC,
            "value": value,
            "unit": "reads/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms_per_step,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (deterministic repeat-rich genome + wgsim-like reads generated in-process)",
            "config": {
                "workload": wl["desc"].format(reads=wl["reads"]),
                "genome_bases": wl["genome_bases"], "contigs": wl["n_contigs"], "reads_per_gpu": wl["reads"],
                "read_len": READ_LEN, "seed_len": 20, "maxHits": 300, "maxK": 14, "numSeeds": 25,
                "extraSearchDepth": 2,
                "parallelism": f"reads sharded over {world} GPU(s), index built once per node and replicated",
                "boundary": "host reads in (pinned) -> host records out: H2D, passes, D2H, MAPQ fix-ups "
                            "(chunks pipelined over 2 HIP streams; " + (
                                "mode stream: snapgpu_align_batch_submit per step, one snapgpu_align_batch_wait, "
                                "records alternate between two host arrays)" if args.mode == "stream" else
                                "mode sync: one blocking snapgpu_align_batch per step)"),
                "mode": args.mode,
                "results": {"SingleHit": counts.get(1, 0), "MultipleHits": counts.get(2, 0),
                            "NotFound": counts.get(0, 0)},
                "per_read": {k: round(float(v), 2) for k, v in per_read.items()},
                "host_tail_ms_per_step": float(np.mean(fix_ms)),
                "index_build_s": round(t_index, 2),
                "index_upload_s": round(t_upload, 2),
                "index": index_info,
                "per_rank": per_rank,
            },
            "roofline": roofline,
            "cpu_baseline": cpu,
            "parity": parity,
        }
        result.update(extras)
        print(json.dumps(result), file=_RESULT_OUT, flush=True)
    if dist:
        dist.barrier()
        shared_index.cleanup(rank, world)
        dist.destroy_process_group()
    return result


if __name__ == "__main__":
    main()
