"""Diagnostic: how much of align_kernel<128>'s time is the persistent kernel's tail?  The C2 batch
(1M reads) aligned in its own order, then with the same reads permuted -- heaviest first (by the
nLocationsScored of the first run: perfect knowledge of each read's cost), only the heaviest 5 %
moved to the front, and a random permutation as the control.  Prints the align kernel's busy
milliseconds per 1M reads (best of 3) for each order.
  python tools/order_probe.py [--reads N]"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
import numpy as np  # noqa: E402
import snapgpu  # noqa: E402
from snapgpu import lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--reads", type=int, default=1_000_000)
ap.add_argument("--genome-bases", type=int, default=46_709_983)
ap.add_argument("--contigs", type=int, default=1)
ap.add_argument("--families", type=int, default=200)
args = ap.parse_args()
g = snapgpu.Genome.synthetic(args.genome_bases, seed=2121, n_contigs=args.contigs, n_repeat_families=args.families)
reads = snapgpu.Reads.synthetic(g, args.reads, seed=99)
idx = snapgpu.GenomeIndex.build(g, 20, 16)
del g
al = snapgpu.BaseAligner(idx, device=0)


def permuted(rd, perm):
    r = rd._p.contents
    n = r.n
    offs = np.ctypeslib.as_array(C.cast(r.offsets, C.POINTER(C.c_uint64)), shape=(n,))[perm].copy()
    lens = np.ctypeslib.as_array(C.cast(r.lengths, C.POINTER(C.c_uint32)), shape=(n,))[perm].copy()
    p = lib().snapgpu_reads_from_arrays(n, C.cast(r.bases, C.c_char_p), C.cast(r.quals, C.c_char_p),
                                        offs.ctypes.data_as(C.POINTER(C.c_uint64)),
                                        lens.ctypes.data_as(C.POINTER(C.c_uint32)))
    return snapgpu.Reads(p)


def kernel_ms(rd):
    best, res = None, None
    for _ in range(3):
        res = al.AlignReads(rd)
        t = al.timing()
        ms = t["mainKernelMs"]
        best = ms if best is None else min(best, ms)
    return best, res


out = {"reads": args.reads}
ms, res = kernel_ms(reads)
out["input_order_ms"] = ms
w = res["nLocationsScored"].astype(np.int64)
n = len(w)
heavy = np.argsort(-w, kind="stable")
out["heaviest_first_ms"], r1 = kernel_ms(permuted(reads, heavy))
top = heavy[: n // 20]
mask = np.ones(n, bool)
mask[top] = False
out["top5pct_first_ms"], _ = kernel_ms(permuted(reads, np.concatenate([top, np.nonzero(mask)[0]])))
rng = np.random.default_rng(7)
out["random_order_ms"], _ = kernel_ms(permuted(reads, rng.permutation(n)))
out["same_results_heaviest_first"] = bool(np.array_equal(r1["location"], res["location"][heavy]))
out["cost_share_top5pct"] = float(w[top].sum() / max(1, w.sum()))
print(json.dumps(out))
