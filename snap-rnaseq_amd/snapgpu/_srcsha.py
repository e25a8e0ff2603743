"""Identity of the sources libsnapgpu.so is built from (no imports beyond the stdlib).

SHA-256 over every file under snap-rnaseq_amd/csrc (*.hip, *.h, *.cpp), include/snapgpu.h and
snap-rnaseq_amd/Makefile, in sorted relative-path order, each as `path NUL content NUL`.  The
Makefile embeds it into the library (snapgpu_source_sha256); snapgpu._ffi refuses to load a
library whose embedded identity differs from the sources beside it, so a stale prebuilt .so
cannot run in place of the sources it ships with.

    python3 snap-rnaseq_amd/snapgpu/_srcsha.py     # prints the identity (the Makefile's SNAPGPU_SRC_SHA)
"""
import hashlib
import os

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))   # snap-rnaseq_amd
ROOT = os.path.dirname(PKG)


def source_files():
    out = []
    for d, _, fs in os.walk(os.path.join(PKG, "csrc")):
        for f in fs:
            if f.endswith((".hip", ".h", ".cpp")):
                out.append(os.path.join(d, f))
    out += [os.path.join(ROOT, "include", "snapgpu.h"), os.path.join(PKG, "Makefile")]
    return sorted(os.path.relpath(p, ROOT) for p in out)


def source_sha256():
    """-> hex digest, or None when the sources are not beside the package."""
    h = hashlib.sha256()
    files = source_files()
    if not os.path.exists(os.path.join(ROOT, "include", "snapgpu.h")):
        return None
    for rel in files:
        h.update(rel.encode() + b"\0")
        with open(os.path.join(ROOT, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()


if __name__ == "__main__":
    print(source_sha256())
