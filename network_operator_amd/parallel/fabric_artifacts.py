"""Apply the node agent's RCCL artifacts to a collective run, and read back what RCCL made of them.

The reference's node artifact exists to be consumed by the collective library: HCCL reads
``gaudinet.json`` (reference cmd/discover/gaudinet.go:28-89, README.md:25).  Here the agent's
counterpart is ``rccl.env`` (+ the ``NCCL_TOPO_FILE`` XML it names), and the consumer is RCCL.
This module closes that loop for ``bench.py`` and ``validate.py``:

* :func:`generate` runs the agent itself, unprivileged (``discover --dry-run``), against this
  node's sysfs: it writes ``rccl-topo.xml`` and the intra-node part of ``rccl.env``
  (``NCCL_TOPO_FILE`` + site settings; no HCA / GID / socket interface, since nothing was
  configured) into a scratch directory.
* :func:`load_env_dir` reads an artifact directory the way a job sources it (``rccl.env``, then
  the validation Job's ``rccl-tuned.env`` on top).
* :func:`rccl_view` parses RCCL's own topology dump (``NCCL_TOPO_DUMP_FILE``) of a run made with
  the file: the xGMI links RCCL sees per GPU, and whether each GPU's and NIC's PCIe ancestry in
  RCCL's dump equals the file's.  :func:`links_verdict` turns that into the check "RCCL sees at
  least n-1 xGMI links per GPU under the file".
"""

from __future__ import annotations

import hashlib
import json
import os
import subprocess
import time
import xml.etree.ElementTree as ET
from pathlib import Path
from typing import Dict, Iterable, List, Optional

from ..utils.paths import native_bin

ENV_FILE = "rccl.env"
TUNED_FILE = "rccl-tuned.env"
TOPO_FILE = "rccl-topo.xml"
DUMP_FILE = "rccl-topo-dump.xml"


def parse_env_text(text: str) -> Dict[str, str]:
    """KEY=VALUE lines of an env-file (comments and blanks skipped; the value is everything after
    the first ``=``, so ``NCCL_IB_HCA==mlx5_0:1`` keeps RCCL's exact-match ``=`` prefix)."""
    out: Dict[str, str] = {}
    for line in text.splitlines():
        line = line.strip()
        if not line or line.startswith("#") or "=" not in line:
            continue
        k, v = line.split("=", 1)
        k = k.strip()
        if k.startswith("export "):
            k = k[len("export "):].strip()
        if k:
            out[k] = v
    return out


def load_env_dir(artifact_dir: str) -> Dict[str, str]:
    """What a job on the node gets: ``rccl.env``, then ``rccl-tuned.env`` overriding it."""
    env: Dict[str, str] = {}
    for name in (ENV_FILE, TUNED_FILE):
        p = Path(artifact_dir) / name
        if p.is_file():
            env.update(parse_env_text(p.read_text()))
    return env


def _sha256(path: str) -> Optional[str]:
    try:
        return hashlib.sha256(Path(path).read_bytes()).hexdigest()
    except OSError:
        return None


def generate(out_dir: str, sysfs_root: Optional[str] = None, env_extra: str = "", timeout: float = 60) -> dict:
    """Runs ``discover --dry-run`` into ``out_dir``; returns the artifacts' description:
    ``{"applied": False, "env": {...}, "topo_file", "topo_file_bytes", "topo_sha256", "agent_ms",
    "agent_status"}`` or ``{"error": ...}``.  ``applied`` is set by the caller once the env is live."""
    out = Path(out_dir)
    out.mkdir(parents=True, exist_ok=True)
    topo, envf, status = out / TOPO_FILE, out / ENV_FILE, out / "agent-status.json"
    cmd = [str(native_bin("discover")), "--dry-run", "--xgmi-expect=0", f"--rccl-topo={topo}", f"--rccl-env={envf}",
           f"--status-file={status}"]
    if env_extra:
        cmd.append(f"--rccl-env-extra={env_extra}")
    env = dict(os.environ)
    if sysfs_root:
        env["SYSFS_ROOT"] = sysfs_root
    t = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env)
    ms = (time.perf_counter() - t) * 1e3
    if r.returncode != 0 or not envf.is_file():
        return {"error": f"discover --dry-run rc={r.returncode}: {(r.stderr or r.stdout)[-600:]}", "agent_ms": ms}
    doc = {"source": "discover --dry-run on this node's sysfs" + (f" ({sysfs_root})" if sysfs_root else ""),
           "dir": str(out), "env_file": str(envf), "env": parse_env_text(envf.read_text()), "agent_ms": round(ms, 3),
           "topo_file": str(topo) if topo.is_file() else None,
           "topo_file_bytes": topo.stat().st_size if topo.is_file() else 0, "topo_sha256": _sha256(str(topo))}
    try:
        st = json.loads(status.read_text())
        doc["agent_status"] = {k: st[k] for k in ("xgmi_pairs", "xgmi_links", "xgmi_error", "gpudirect_rdma", "phases_ms",
                                                  "not_in_netns", "nics_without_rdma") if k in st}
    except (OSError, ValueError):
        pass
    if doc["env"].get("NCCL_TOPO_FILE") != doc["topo_file"]:
        doc["error"] = f"rccl.env names NCCL_TOPO_FILE={doc['env'].get('NCCL_TOPO_FILE')!r}, expected {doc['topo_file']!r}"
    return doc


def apply(env: Dict[str, str], target: Optional[dict] = None) -> dict:
    """Exports ``env`` into ``target`` (default ``os.environ``); returns what this process now
    sees for those keys plus the hash of the topology file it will load (a per-rank record)."""
    target = os.environ if target is None else target
    for k, v in env.items():
        target[k] = v
    seen = {k: target.get(k) for k in env}
    topo = target.get("NCCL_TOPO_FILE")
    return {"env": seen, "topo_sha256": _sha256(topo) if topo else None}


def strip(env: dict, keys: Iterable[str]) -> dict:
    """A copy of ``env`` without the artifact keys (a run with RCCL's defaults)."""
    drop = set(keys) | {"NCCL_TOPO_DUMP_FILE"}
    return {k: v for k, v in env.items() if k not in drop}


# ------------------------------------------------------------------------------------------
# RCCL's topology dump
# ------------------------------------------------------------------------------------------
def _chains(root: ET.Element):
    """busid -> [cpu numaid, outer pci busid, ..., busid] for every <pci>; net name -> the chain
    of the <pci> it sits under."""
    pci: Dict[str, List[str]] = {}
    net: Dict[str, List[str]] = {}

    def walk(el, path):
        for c in el:
            if c.tag == "cpu":
                walk(c, path + [c.get("numaid")])
            elif c.tag == "pci":
                here = path + [(c.get("busid") or "").lower()]
                pci[here[-1]] = here
                walk(c, here)
            elif c.tag == "net":
                net[c.get("name", "")] = path
            else:
                walk(c, path)
    walk(root, [])
    return pci, net


def rccl_view(dump_xml: str, file_xml: Optional[str] = None) -> dict:
    """What RCCL made of the node: per GPU of the dump (one per rank of the communicator) the
    xGMI links to the other GPUs of the dump (``<xgmi target=... count=...>`` children of
    ``<gpu>``), and — when ``file_xml`` is given — whether each GPU's and NIC's ancestry in the
    dump equals the file's."""
    root = ET.fromstring(dump_xml)
    pci, net = _chains(root)
    gpus: Dict[str, dict] = {}

    def walk(el, parent):
        for c in el:
            if c.tag == "gpu" and parent is not None and parent.tag == "pci":
                busid = (parent.get("busid") or "").lower()
                links: Dict[str, int] = {}
                for x in c:
                    if x.tag in ("xgmi", "nvlink"):
                        t = (x.get("target") or "").lower()
                        links[t] = links.get(t, 0) + int(x.get("count") or 1)
                gpus[busid] = {"rank": c.get("rank"), "dev": c.get("dev"), "gcn": c.get("gcn"), "links": links}
            walk(c, c)
    walk(root, None)
    xgmi_elements = sum(len(g["links"]) for g in gpus.values())
    per_gpu = {b: sum(1 for t in g["links"] if t in gpus and t != b) for b, g in gpus.items()}
    view = {"gpus": len(gpus), "gpu_busids": sorted(gpus), "xgmi_elements": xgmi_elements,
            "xgmi_links_per_gpu": per_gpu, "min_xgmi_links": min(per_gpu.values()) if per_gpu else 0,
            "xgmi_link_count_per_gpu": {b: sum(c for t, c in g["links"].items() if t in gpus) for b, g in gpus.items()},
            "nets": sorted(net)}
    if file_xml is not None:
        fpci, fnet = _chains(ET.fromstring(file_xml))
        gdiff = {b: {"file": fpci.get(b), "rccl": pci.get(b)} for b in gpus if fpci.get(b) != pci.get(b)}
        ndiff = {n: {"file": fnet[n], "rccl": net[n]} for n in net if n in fnet and fnet[n] != net[n]}
        view.update(gpu_ancestry_equal=not gdiff, gpu_ancestry_diff=gdiff,
                    nic_ancestry_equal=(not ndiff) if any(n in fnet for n in net) else None, nic_ancestry_diff=ndiff,
                    nets_from_file=sorted(n for n in net if n in fnet))
    return view


def read_view(dump_path: str, file_path: Optional[str] = None) -> Optional[dict]:
    p = Path(dump_path)
    if not p.is_file() or p.stat().st_size == 0:
        return None
    try:
        return rccl_view(p.read_text(), Path(file_path).read_text() if file_path and Path(file_path).is_file() else None)
    except (ET.ParseError, OSError) as e:
        return {"error": f"unparseable RCCL topology dump {dump_path}: {e}"}


def traffic_view(job_bdfs: List[str], traffic: Optional[dict], min_bytes: int = 1 << 20) -> Optional[dict]:
    """From amd-smi's per-link counters around the timed loop (``ops.smi.traffic``): for each of
    the job's GPUs, the xGMI links *to another GPU of the job* that moved at least ``min_bytes``.
    Hardware's account of what RCCL used, independent of RCCL's dump."""
    if not traffic or not traffic.get("gpus"):
        return None
    job = {b.lower() for b in job_bdfs}
    per = {}
    for g in traffic["gpus"]:
        b = g["bdf"].lower()
        if b not in job:
            continue
        peers = g.get("peer_per_link") or []
        per[b] = sum(1 for i, d in enumerate(g["bytes_per_link"])
                     if i < len(peers) and peers[i] in job and peers[i] != b and d >= min_bytes)
    if not per:
        return None
    return {"gpus": len(per), "links_with_traffic_per_gpu": per, "min_links_with_traffic": min(per.values())}


def links_verdict(n: int, with_file: Optional[dict], defaults: Optional[dict],
                  traffic: Optional[dict] = None) -> dict:
    """The dump-based verdict (:func:`dump_verdict`), with the hardware counters as a one-way
    tie breaker: when every one of the job's GPUs moved data over n-1 xGMI links during the timed
    loop (``traffic_view``), RCCL used every link, whatever its dump says.  Fewer used links do
    not fail the check (RCCL's rings may leave a link idle); they are reported."""
    v = dump_verdict(n, with_file, defaults)
    if traffic is not None:
        v["min_links_with_traffic"] = traffic["min_links_with_traffic"]
        counters_ok = traffic["gpus"] >= n and traffic["min_links_with_traffic"] >= max(n - 1, 0)
        if v["status"] != "ok" and counters_ok:
            v = dict(v, status="ok", dump_status=v["status"],
                     why=f"amd-smi: every GPU moved data over {n - 1} xGMI link(s) to the others during the timed "
                         f"loop (RCCL's dump: {v['status']}: {v.get('why', '')})")
        elif n > 1 and not counters_ok:
            # Informational only: which links a collective uses is RCCL's choice of rings and
            # channels (a 4-GPU ring may leave the diagonals idle).  "RCCL sees the link" is the
            # topology's question, answered by the dump.
            v = dict(v, counters_note=f"amd-smi: a GPU moved data over {traffic['min_links_with_traffic']} of "
                                      f"{n - 1} xGMI links during the timed loop")
    return v


def dump_verdict(n: int, with_file: Optional[dict], defaults: Optional[dict]) -> dict:
    """"RCCL sees at least n-1 xGMI links per GPU under the agent's file."

    * ``ok`` — every GPU of the dump has >= n-1 xGMI peers among the job's GPUs (and the dump
      holds all n GPUs), and the file did not cost a link RCCL sees without it.
    * ``failed`` — fewer, while RCCL without the file sees more (the file lost links:
      ``file_blamed``), or the dump is missing / shows fewer than n-1 with xGMI elements present.
    * ``degraded`` — fewer than n-1, but the same without the file: the node's mesh, not the file.
    * ``unverifiable`` — RCCL's dump carries no ``<xgmi>`` elements with *or* without the file
      (this RCCL build records the links elsewhere): the file cannot be blamed, say so.
    """
    need = max(n - 1, 0)
    if n <= 1:
        return {"status": "ok", "expected_per_gpu": 0, "why": "n=1: no peer GPU"}
    if not with_file or "error" in with_file:
        return {"status": "failed", "expected_per_gpu": need,
                "why": (with_file or {}).get("error", "RCCL wrote no topology dump under the agent's file")}
    got = with_file["min_xgmi_links"]
    base = defaults.get("min_xgmi_links") if defaults and "error" not in defaults else None
    out = {"expected_per_gpu": need, "min_with_file": got, "min_with_rccl_defaults": base,
           "gpus_in_dump": with_file["gpus"]}
    if with_file["gpus"] < n:
        return dict(out, status="failed", why=f"RCCL's dump holds {with_file['gpus']} of {n} GPUs")
    if got >= need and (base is None or got >= base):
        return dict(out, status="ok")
    if base is not None and base > got:
        return dict(out, status="failed", file_blamed=True,
                    why=f"with the agent's file RCCL sees {got} xGMI peers per GPU (min), without it {base}: the "
                        "file costs links")
    if with_file["xgmi_elements"] == 0 and (base is None or defaults.get("xgmi_elements", 0) == 0):
        return dict(out, status="unverifiable",
                    why="RCCL's topology dump has no <xgmi> elements with the agent's file, and "
                        + ("none without it either" if base is not None else "no dump without it to compare"))
    if base is not None and base == got:
        # RCCL sees the same deficit without the file: the node's mesh (or how this RCCL build
        # records it), not the agent's artifacts.  Reported, not blamed on the file.
        return dict(out, status="degraded",
                    why=f"RCCL sees {got} xGMI peers per GPU (min) of {need}, with and without the agent's file")
    return dict(out, status="failed", why=f"RCCL sees {got} xGMI peers per GPU (min), {need} expected")
