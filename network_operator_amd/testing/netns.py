"""Synthetic-switch network-namespace harness (veth pairs + injected LLDP).

Full harness: see ``NodeSim`` below.  ``available()`` reports whether this process can
create private network namespaces and raw packet sockets (root in the build container;
the unprivileged GPU boxes cannot).
"""

from __future__ import annotations

import ctypes
import ctypes.util
import os
import shutil
import socket
import subprocess

CLONE_NEWNET = 0x40000000
CLONE_NEWUSER = 0x10000000


def available() -> tuple[bool, str]:
    """True when ``unshare -rn`` works and AF_PACKET sockets can be opened inside it."""
    if not shutil.which("unshare"):
        return False, "unshare(1) not installed"
    probe = ("import socket; s=socket.socket(socket.AF_PACKET, socket.SOCK_RAW, 0); "
             "n=socket.socket(socket.AF_NETLINK, socket.SOCK_RAW, 0); print('ok')")
    try:
        r = subprocess.run(["unshare", "-rn", "python3", "-c", probe], capture_output=True, text=True, timeout=60)
    except Exception as e:  # pragma: no cover
        return False, f"unshare failed: {e}"
    if r.returncode != 0 or "ok" not in r.stdout:
        return False, (r.stderr.strip().splitlines() or ["unshare -rn failed"])[-1]
    return True, "ok"
