"""Loader for the in-tree native extensions.

``_pbx_hip``  -- hand-written gfx950 kernels (GPU table, dedup, pull/push,
                 seqpool+CVM, data_norm, FM, loss, AUC, Adam).
``_pbx_host`` -- native C++ host runtime (CPU parameter server, slot dataset,
                 parser, metrics, archive, thread pool).

On a GPU box the HIP extension is mandatory: GPU ops call :func:`hip` which
raises if the extension is missing instead of silently falling back to eager
PyTorch.  CPU tensors use the reference implementations in
``paddlebox_amd.ops.reference`` (that is the CPU device path, not a fallback).
"""
from __future__ import annotations

import importlib

import torch  # noqa: F401  (loads libc10 / libtorch for the extensions)
import os

_hip_mod = None
_host_mod = None
_hip_err = None
_host_err = None


def _try_import(name):
    try:
        return importlib.import_module(f"paddlebox_amd.{name}"), None
    except Exception as e:  # pragma: no cover - depends on build state
        return None, e


def hip():
    """Return the HIP extension module or raise loudly."""
    global _hip_mod, _hip_err
    if _hip_mod is None:
        _hip_mod, _hip_err = _try_import("_pbx_hip")
        if _hip_mod is None:
            raise RuntimeError(
                "paddlebox_amd._pbx_hip (gfx950 kernels) is not built/loadable: "
                f"{_hip_err!r}. Run `python setup.py build_ext --inplace`."
            )
    return _hip_mod


def host():
    """Return the native host runtime module or raise loudly."""
    global _host_mod, _host_err
    if _host_mod is None:
        _host_mod, _host_err = _try_import("_pbx_host")
        if _host_mod is None:
            raise RuntimeError(
                "paddlebox_amd._pbx_host (native host runtime) is not built/loadable: "
                f"{_host_err!r}. Run `python setup.py build_ext --inplace`."
            )
    return _host_mod


def hip_available() -> bool:
    try:
        hip()
        return True
    except RuntimeError:
        return False


def host_available() -> bool:
    try:
        host()
        return True
    except RuntimeError:
        return False


def so_paths():
    """Paths of the native libraries actually loaded (for diagnostics)."""
    out = {}
    for name, mod in (("_pbx_hip", _hip_mod), ("_pbx_host", _host_mod)):
        if mod is not None:
            out[name] = os.path.abspath(mod.__file__)
    return out


# ---------------------------------------------------------------- build provenance
_SRC_DIRS = ("csrc",)
_SRC_SUFFIXES = (".hip", ".cpp", ".cc", ".h")


def sources_digest(root: str = None) -> str:
    """sha256 over the native sources (path + bytes, sorted): what the in-tree
    libraries must have been built from."""
    import hashlib

    root = root or os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    h = hashlib.sha256()
    files = []
    for d in _SRC_DIRS:
        for dp, _, fns in os.walk(os.path.join(root, d)):
            files += [os.path.join(dp, f) for f in fns if f.endswith(_SRC_SUFFIXES)]
    for f in sorted(files):
        h.update(os.path.relpath(f, root).encode())
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def build_info() -> dict:
    """Provenance of the loaded libraries: the stamp written by the build
    (__graft_entry__.build: sources digest, hipcc version, arch, time) and
    whether the sources in this tree still match it (False = stale binary)."""
    import json

    here = os.path.dirname(os.path.abspath(__file__))
    info = {"stamp": None, "sources_now": None, "matches_tree": None}
    try:
        with open(os.path.join(here, "_build_info.json")) as f:
            info["stamp"] = json.load(f)
    except (OSError, ValueError):
        return info
    try:
        info["sources_now"] = sources_digest()
        info["matches_tree"] = info["sources_now"] == info["stamp"].get("sources")
    except OSError:
        pass
    return info
