"""Python access to the native (C++17) node agent.

``native()`` returns the pybind11 module ``_netop_native`` (LLDP codec, Port-Description
parser, rtnetlink client, sysfs/KFD topology).  The agent itself is the ``discover``
executable (see ``network_operator_amd.utils.native_bin``); Python never sits on the node
agent's hot path.
"""

from __future__ import annotations

import importlib
import sys

from ..utils.paths import LIB_DIR, NativeArtifactMissing

_mod = None


def native():
    global _mod
    if _mod is None:
        if str(LIB_DIR) not in sys.path:
            sys.path.insert(0, str(LIB_DIR))
        try:
            _mod = importlib.import_module("_netop_native")
        except ImportError as e:  # pragma: no cover - exercised when not built
            raise NativeArtifactMissing(f"_netop_native not built in {LIB_DIR}: {e}") from e
    return _mod


__all__ = ["native"]
