"""Locations of in-tree build artefacts (native agent binaries, pybind module, HIP library)."""

from __future__ import annotations

import os
from pathlib import Path

PACKAGE_DIR = Path(__file__).resolve().parent.parent
REPO_ROOT = PACKAGE_DIR.parent
LIB_DIR = PACKAGE_DIR / "_lib"
BIN_DIR = LIB_DIR / "bin"


class NativeArtifactMissing(FileNotFoundError):
    """A native artefact was not built; run ``python -c 'import __graft_entry__ as g; g.build()'``."""


def native_bin(name: str) -> Path:
    """Path of a native executable (``discover``, ``netop-lldp-tx``, ``netop-topo`` ...)."""
    override = os.environ.get("NETOP_BIN_DIR")
    for d in ([Path(override)] if override else []) + [BIN_DIR, LIB_DIR]:
        p = d / name
        if p.is_file() and os.access(p, os.X_OK):
            return p
    raise NativeArtifactMissing(f"native binary {name!r} not built (looked in {BIN_DIR}); run __graft_entry__.build()")


def hip_library() -> Path:
    p = LIB_DIR / "libnetop_hip.so"
    if not p.is_file():
        raise NativeArtifactMissing(f"{p} not built; run __graft_entry__.build()")
    return p
