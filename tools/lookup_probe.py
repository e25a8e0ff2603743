"""seed_lookup_kernel timing two ways on the same dispatches: HIP events around the launch
(snapgpu timing: lookupKernelMs / lookupKernelBusyMs) and the rocprofv3 kernel trace when run under
it.  C2 genome, 1M resident reads, the two streams' pass sets serialised (set_overlap(False)).
  rocprofv3 --kernel-trace --stats -d <dir> -o run --output-format csv -- python3 tools/lookup_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
import snapgpu  # noqa: E402

g = snapgpu.Genome.synthetic(46_709_983, seed=2121, n_contigs=1)
idx = snapgpu.GenomeIndex.build(g, 20, 16)
reads = snapgpu.Reads.synthetic(idx.genome_handle(), 1_000_000, seed=99)
al = snapgpu.BaseAligner(idx, device=0)
al.set_overlap(False)
dev = al.upload(reads)
for i in range(6):
    dev.run()
    dev.synchronize()
    t = al.timing()
    print(f"run {i}: lookup event ms {t['lookupKernelMs']:.4f} busy {t['lookupKernelBusyMs']:.4f} "
          f"align {t['mainKernelMs']:.3f} launches {t['nLaunches']}", flush=True)
