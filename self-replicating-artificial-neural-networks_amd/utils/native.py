"""Loader for the in-tree native extensions (built by ``__graft_entry__.build`` /
``python -m serann.build``).  Extensions live in ``serann/_native`` so they travel with the repo
snapshot; nothing is installed into site-packages."""
from __future__ import annotations

import hashlib
import importlib.util
import os
import sysconfig
from pathlib import Path

NATIVE_DIR = Path(__file__).resolve().parent.parent / "_native"
HIP_SRC_DIR = Path(__file__).resolve().parent.parent / "csrc" / "hip"
_cache = {}


def hip_source_hash(src_dir: Path = HIP_SRC_DIR) -> str:
    """Digest of the HIP kernel sources (every .hip / .h in csrc/hip).  ``build_hip`` compiles it into the
    extension; the loader compares it with the sources beside it, so a stale .so -- one whose kernels
    expect other descriptor or tile layouts than this tree's Python planners write -- fails loudly at import
    instead of faulting the GPU."""
    h = hashlib.sha256()
    for f in sorted(list(src_dir.glob("*.hip")) + list(src_dir.glob("*.h"))):
        h.update(f.name.encode())
        h.update(f.read_bytes())
    return h.hexdigest()[:16]


def load(name: str, required: bool = False):
    """Import ``serann/_native/<name><EXT_SUFFIX>``; returns None (or raises) if absent."""
    if name in _cache:
        return _cache[name]
    suffix = sysconfig.get_config_var("EXT_SUFFIX") or ".so"
    # SERANN_NATIVE_DIR: load the extensions of another in-tree build (A/B timing of two kernel versions);
    # an extension that directory does not hold comes from the in-tree build
    path = NATIVE_DIR / f"{name}{suffix}"
    alt = os.environ.get("SERANN_NATIVE_DIR")
    if alt and (Path(alt) / f"{name}{suffix}").exists():
        path = Path(alt) / f"{name}{suffix}"
    mod = None
    if path.exists():
        if name.startswith("serann_hip"):
            import torch  # noqa: F401  -- HIP runtime must come from torch's bundled libamdhip64
        spec = importlib.util.spec_from_file_location(name, str(path))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        if name == "serann_hip" and not alt and HIP_SRC_DIR.is_dir():
            built = mod.src_hash() if hasattr(mod, "src_hash") else "unknown"
            want = hip_source_hash()
            if built != want:
                raise ImportError(f"{path.name} was built from other kernel sources (hash {built}, tree {want}): "
                                  f"rebuild it (`python -c 'import __graft_entry__ as g; g.build()'`)")
    elif required:
        raise ImportError(f"native extension {name} not built (expected {path}); "
                          f"run `python -c 'import __graft_entry__ as g; g.build()'`")
    _cache[name] = mod
    return mod
