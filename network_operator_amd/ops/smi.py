"""xGMI link state and traffic counters (ctypes over ``libnetop_smi.so`` -> amd-smi).

``snapshot()`` -> {"gpus": [{"bdf", "link_status", "xgmi_read_kb", "xgmi_write_kb", "links": [...]}]}
``traffic(before, after)`` -> per-GPU, per-link bytes moved between two snapshots, and how
many *up* links carried traffic — the "every link is used" check of BASELINE.json.
"""

from __future__ import annotations

import ctypes
import json
from typing import Optional

from ..utils.paths import LIB_DIR, NativeArtifactMissing

_lib = None


def lib():
    global _lib
    if _lib is None:
        p = LIB_DIR / "libnetop_smi.so"
        if not p.is_file():
            raise NativeArtifactMissing(f"{p} not built; run __graft_entry__.build()")
        L = ctypes.CDLL(str(p))
        L.netop_smi_snapshot.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.netop_smi_snapshot.restype = ctypes.c_int
        _lib = L
    return _lib


def snapshot() -> dict:
    buf = ctypes.create_string_buffer(1 << 20)
    rc = lib().netop_smi_snapshot(buf, len(buf))
    doc = json.loads(buf.value.decode() or "{}")
    if rc != 0:
        raise RuntimeError(doc.get("error", f"amd-smi failed ({rc})"))
    return doc


def traffic(before: dict, after: dict, min_bytes: int = 1 << 20) -> dict:
    """Bytes per link between two snapshots (read + write counters, KB -> bytes)."""
    prev = {g["bdf"]: g for g in before.get("gpus", [])}
    out = {"gpus": [], "links_up": 0, "links_with_traffic": 0}
    for g in after.get("gpus", []):
        p = prev.get(g["bdf"])
        if not p or "xgmi_read_kb" not in g:
            continue
        status: Optional[str] = g.get("link_status")
        peers = [(ln.get("peer") or "").lower() for ln in g.get("links") or []]
        per_link = []
        for i, (r, w) in enumerate(zip(g["xgmi_read_kb"], g["xgmi_write_kb"])):
            d = ((r - p["xgmi_read_kb"][i]) + (w - p["xgmi_write_kb"][i])) * 1024
            per_link.append(d)
            up = status is not None and i < len(status) and status[i] == "U"
            out["links_up"] += int(up)
            out["links_with_traffic"] += int(up and d >= min_bytes)
        out["gpus"].append({"bdf": g["bdf"], "link_status": status, "bytes_per_link": per_link,
                            "peer_per_link": peers[:len(per_link)]})
    return out
