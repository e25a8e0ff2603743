import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "snap-rnaseq_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

PRODUCT_SO = os.path.join(ROOT, "snap-rnaseq_amd", "snapgpu", "libsnapgpu.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")
    config.addinivalue_line("markers", "reference: needs /root/reference + oracle/_ref (this container only)")


def _ensure_built():
    if not os.path.exists(PRODUCT_SO):
        subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "snap-rnaseq_amd")], check=True)
    if not os.path.exists(os.path.join(ROOT, "oracle", "liboracle.so")):
        subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "oracle", "Makefile")], check=True, cwd=ROOT)


_ensure_built()


@pytest.fixture(scope="session")
def gpu_available():
    import snapgpu
    n = snapgpu.device_count()
    if n <= 0:
        pytest.fail("no HIP device visible, but a gpu-marked test was selected")
    return n


@pytest.fixture(scope="session")
def small_world():
    """1 Mb, 3-contig repeat-rich genome + index + wgsim-like reads (config C1 shape)."""
    import snapgpu
    g = snapgpu.Genome.synthetic(1_000_000, seed=2121, n_contigs=3, n_repeat_families=60)
    ref_genome = snapgpu.Genome.synthetic(1_000_000, seed=2121, n_contigs=3, n_repeat_families=60)
    idx = snapgpu.GenomeIndex.build(g, 20, 8)
    reads = snapgpu.Reads.synthetic(ref_genome, 4000, seed=99, random_read_fraction=0.01)
    return {"genome": ref_genome, "index": idx, "reads": reads}
