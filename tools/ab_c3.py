"""A/B timing of library builds on the C3 genome (bench --workload c3 shape) without rebuilding
the 3.1 Gb index per variant: `build` writes the index once to /dev/shm (snapgpu_index_share),
`run` (one process per library, SNAPGPU_LIB=...) attaches it, aligns N resident reads three
times and prints the best time and a digest of the records.
  python tools/ab_c3.py build [path]
  SNAPGPU_LIB=... python tools/ab_c3.py run [path] [n_reads]"""
import hashlib
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
import snapgpu  # noqa: E402

mode = sys.argv[1]
path = sys.argv[2] if len(sys.argv) > 2 else "/dev/shm/snapgpu_ab_c3.bin"
if mode == "build":
    t0 = time.time()
    g = snapgpu.Genome.synthetic(3_100_000_000, seed=2121, n_contigs=25, n_repeat_families=2000)
    idx = snapgpu.GenomeIndex.build(g, 20, 16)
    idx.share(path)
    print(f"built and shared in {time.time() - t0:.1f} s", flush=True)
else:
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 1_000_000
    idx = snapgpu.GenomeIndex.attach(path)
    reads = snapgpu.Reads.synthetic(idx.genome_handle(), n, seed=99)
    al = snapgpu.BaseAligner(idx, device=0)
    dev = al.upload(reads)
    dev.run()
    dev.synchronize()
    ts = []
    for _ in range(3):
        t0 = time.perf_counter()
        dev.run()
        dev.synchronize()
        ts.append(time.perf_counter() - t0)
    res = dev.results()
    dg = hashlib.sha256(res.tobytes()).hexdigest()[:16]
    print(f"{os.path.basename(os.environ.get('SNAPGPU_LIB', 'libsnapgpu.so'))} reads {n} best_ms {min(ts) * 1e3:.1f} "
          f"reads_per_s {n / min(ts) / 1e6:.2f}M digest {dg}", flush=True)
