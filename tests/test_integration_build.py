"""The SNAPLib drop-in (snap-rnaseq_amd/integration/) builds against the reference itself.

GpuBaseAligner (an Aligner) and GpuSingleExtension (the AlignerExtension hook of
SingleAlignerContext, AlignerContext.h:132-163) are compiled with the reference's headers
and dialect (g++ -std=gnu++98) and linked with the reference's SNAPLib objects and
libsnapgpu.so into `snap-rna-gpu`, apps/snap/Main.cpp's single command with the extension
plugged in.  Build container only (the binary contains reference code and never travels to a
GPU box): here it runs end to end up to the aligner construction and must fail loudly, not
fall back to the CPU aligner."""
import os
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
G = os.path.join(HERE, "golden")
REF = os.path.join(ROOT, "oracle", "_ref")


@pytest.mark.reference
def test_extension_builds_against_reference_and_fails_loudly_without_gpu(tmp_path):
    if not os.path.exists(os.path.join(REF, "snap-rna")) or not os.path.isdir("/root/reference/SNAPLib"):
        pytest.skip("reference build (oracle/_ref) not available: build container only")
    subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "snap-rnaseq_amd", "integration", "Makefile")], check=True)
    exe = os.path.join(REF, "integration", "snap-rna-gpu")
    assert os.access(exe, os.X_OK)
    snap = os.path.join(REF, "snap-rna")
    subprocess.run([snap, "index", os.path.join(G, "small.fa"), str(tmp_path / "gidx")], check=True,
                   capture_output=True)
    subprocess.run([snap, "transcriptome", os.path.join(G, "small.gtf"), os.path.join(G, "small.fa"), "tidx", "-O1000"],
                   check=True, capture_output=True, cwd=tmp_path)
    import snapgpu
    if snapgpu.device_count() > 0:
        pytest.skip("GPU present: the no-GPU failure path is what this container checks")
    p = subprocess.run([exe, "single", str(tmp_path / "gidx"), str(tmp_path / "tidx"), os.path.join(G, "small.gtf"),
                        os.path.join(G, "single_reads.fq"), "-t", "1", "-o", str(tmp_path / "o.sam")],
                       capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert "MI355X aligner" in p.stdout + p.stderr and "no such HIP device" in p.stdout + p.stderr


@pytest.mark.reference
def test_paired_dropin_builds_and_fails_loudly_without_gpu(tmp_path):
    """GpuPairedEndAligner (a PairedEndAligner, PairedEndAligner.h:60-78) in the same binary:
    `snap-rna-gpu pairs` must stop at the GPU aligner's construction here, not fall back."""
    if not os.path.exists(os.path.join(REF, "snap-rna")) or not os.path.isdir("/root/reference/SNAPLib"):
        pytest.skip("reference build (oracle/_ref) not available: build container only")
    subprocess.run(["make", "-s", "-f", os.path.join(ROOT, "snap-rnaseq_amd", "integration", "Makefile")], check=True)
    exe = os.path.join(REF, "integration", "snap-rna-gpu")
    subprocess.run([os.path.join(REF, "snap-rna"), "index", os.path.join(G, "small.fa"), str(tmp_path / "gidx")],
                   check=True, capture_output=True)
    import snapgpu
    if snapgpu.device_count() > 0:
        pytest.skip("GPU present: the no-GPU failure path is what this container checks")
    p = subprocess.run([exe, "pairs", str(tmp_path / "gidx"), os.path.join(G, "paired_1.fq"),
                        os.path.join(G, "paired_2.fq")], capture_output=True, text=True, timeout=120)
    assert p.returncode != 0
    assert "MI355X paired aligner" in p.stdout + p.stderr and "no such HIP device" in p.stdout + p.stderr
