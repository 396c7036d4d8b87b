"""Loader for the in-tree HIP extension ``_C`` (built by ``build.py``).

Policy (the framework must never silently fall back on a GPU box):
  * CPU tensors always use the PyTorch reference implementations in
    ``mift.ops.reference``;
  * GPU tensors use the HIP kernels.  If the extension failed to import and a
    kernel is requested for a GPU tensor, ``require()`` raises with the import
    error — unless the user explicitly opted out with ``MIFT_KERNELS=0``
    (used only by the torch-eager comparison baseline in bench.py).
"""
import importlib.util
import os
import sys

_C = None
_ERR = None


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return
    here = os.path.dirname(os.path.abspath(__file__))
    so = os.environ.get("MIFT_EXT_SO")  # explicit build (A/B runs of two builds on one device)
    if not so:
        cands = sorted(f for f in os.listdir(here) if f.startswith("_C") and f.endswith(".so"))
        if "_C.so" in cands:
            cands.remove("_C.so")
            cands.insert(0, "_C.so")
        so = os.path.join(here, cands[0]) if cands else None
    if so is None:
        _ERR = ImportError(f"mift extension not built (no _C*.so in {here}); run `python -m mift.build`")
        return
    try:
        import torch  # noqa: F401  (libtorch must be loaded first)
        spec = importlib.util.spec_from_file_location("mift._C", so)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        if not os.environ.get("MIFT_EXT_SO") and os.environ.get("MIFT_ALLOW_STALE_EXT", "0") != "1":
            _check_provenance(mod, so, here)
        sys.modules["mift._C"] = mod
        _C = mod
    except Exception as e:  # pragma: no cover - depends on build
        _ERR = e


def _check_provenance(mod, so, here):
    """The binary must have been built from the csrc/ tree next to it (build.py stamps the
    sha256 of every source into the .so); a stale or foreign _C.so fails loudly."""
    if not os.path.isdir(os.path.join(here, "csrc")):
        return
    import importlib
    build = importlib.import_module(__package__ + ".build") if __package__ else None
    want = build.source_digest(debug=os.path.basename(so).startswith("_C_debug")) if build else None
    got = mod.source_hash() if hasattr(mod, "source_hash") else "<unstamped>"
    if want is not None and got != want:
        raise ImportError(f"stale extension {so}: built from sources {got[:12]}, tree is {want[:12]}; "
                          f"rebuild with `python -m mift.build` (MIFT_ALLOW_STALE_EXT=1 to override)")


def available() -> bool:
    _load()
    return _C is not None


def kernels_enabled() -> bool:
    return os.environ.get("MIFT_KERNELS", "1") != "0"


def require():
    """Return the extension module or raise loudly."""
    _load()
    if _C is None:
        raise RuntimeError(f"mift HIP extension unavailable: {_ERR!r}")
    return _C


def error():
    _load()
    return _ERR
