"""Build the in-tree native extensions.

* ``serann_host`` -- C++17 host runtime (Levenshtein, genotype statistics), g++.
* ``serann_hip``  -- HIP/CDNA4 kernels for gfx950, hipcc ``--offload-arch=gfx950`` (cross-compiles
  without a GPU).  Written directly for CDNA4: no hipify, no CUDA shims.

Both land in ``serann/_native`` (git-ignored, but shipped with the repo snapshot).

    python -m serann.build [--only host|hip] [--jobs N]
"""
from __future__ import annotations

import argparse
import os
import shutil
import subprocess
import sys
import sysconfig
from concurrent.futures import ThreadPoolExecutor
from pathlib import Path

PKG = Path(__file__).resolve().parent
NATIVE = PKG / "_native"
CSRC = PKG / "csrc"
OFFLOAD_ARCH = os.environ.get("SERANN_OFFLOAD_ARCH", "gfx950")


def _pybind_includes():
    import pybind11
    return [f"-I{sysconfig.get_paths()['include']}", f"-I{pybind11.get_include()}"]


def _run(cmd):
    print("+", " ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)


def _ext_suffix():
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def build_host():
    NATIVE.mkdir(exist_ok=True)
    out = NATIVE / f"serann_host{_ext_suffix()}"
    _run(["g++", "-O3", "-std=c++17", "-shared", "-fPIC", "-pthread", *_pybind_includes(),
          str(CSRC / "host" / "serann_host.cpp"), "-o", str(out)])
    return out


def _hipcc():
    for c in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if c and os.path.exists(c):
            return c
    raise FileNotFoundError("hipcc not found")


# gchain.hip keeps its MFMA accumulators in VGPRs: they are read by VALU epilogues every tile, and the
# AGPR form costs a v_accvgpr_read per element
PER_FILE_FLAGS = {"gchain.hip": ["-mllvm", "-amdgpu-mfma-vgpr-form"]}
# sources compiled as several objects (-D<macro>=0..n-1), each instantiating a part of the kernels: gemm3.hip's
# launcher is split in four (its template instantiations are most of the build time)
MULTI_PART = {"gemm3.hip": ("GEMM3_PART", 4)}


def build_hip(jobs: int = 4):
    NATIVE.mkdir(exist_ok=True)
    build_dir = PKG / "_build"
    build_dir.mkdir(exist_ok=True)
    hipcc = _hipcc()
    srcs = sorted((CSRC / "hip").glob("*.hip"))
    flags = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={OFFLOAD_ARCH}", "-mcode-object-version=5",
             "-Wno-unused-result", f"-I{CSRC / 'hip'}", *_pybind_includes()]
    objs = []

    hdr_mtime = max((h.stat().st_mtime for h in (CSRC / "hip").glob("*.h")), default=0.0)
    # the sources' digest goes into module.hip (src_hash()); the loader checks it against the tree
    sys.path.insert(0, str(PKG))
    from utils.native import hip_source_hash
    sys.path.pop(0)
    digest = hip_source_hash(CSRC / "hip")
    stamp = build_dir / "src_hash.txt"
    stale_digest = not stamp.exists() or stamp.read_text().strip() != digest

    units = []
    for src in srcs:
        if src.name in MULTI_PART:
            macro, n = MULTI_PART[src.name]
            units += [(src, f"{src.stem}_p{i}", [f"-D{macro}={i}"]) for i in range(n)]
        else:
            units.append((src, src.stem, []))
    for stale in build_dir.glob("*.o"):           # objects of a former unit layout
        if stale.stem not in {u[1] for u in units}:
            stale.unlink()

    def compile_one(unit):
        src, stem, defs = unit
        obj = build_dir / (stem + ".o")
        extra = PER_FILE_FLAGS.get(src.name, []) + defs
        if src.name == "module.hip":
            extra = extra + [f'-DSERANN_SRC_HASH="{digest}"']
        # incremental: an object newer than its source and every header is reused
        if obj.exists() and obj.stat().st_mtime > max(src.stat().st_mtime, hdr_mtime) and not (
                src.name == "module.hip" and stale_digest):
            return obj
        _run([hipcc, *flags, *extra, "-c", str(src), "-o", str(obj)])
        return obj

    # heaviest units first, so the pool does not end on one long compile
    units.sort(key=lambda u: -u[0].stat().st_size)
    with ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        objs = list(ex.map(compile_one, units))
    out = NATIVE / f"serann_hip{_ext_suffix()}"
    _run([hipcc, "-shared", "-fPIC", f"--offload-arch={OFFLOAD_ARCH}", *map(str, objs), "-o", str(out)])
    stamp.write_text(digest)
    return out


def build_all(jobs: int = 4):
    return [build_host(), build_hip(jobs)]


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", choices=["host", "hip"], default=None)
    ap.add_argument("--jobs", type=int, default=4)
    a = ap.parse_args()
    if a.only in (None, "host"):
        build_host()
    if a.only in (None, "hip"):
        build_hip(a.jobs)
