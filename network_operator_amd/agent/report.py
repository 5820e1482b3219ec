"""Is this node ready for the operator?  One read-only look, without privileges, at everything the
agent checks before it labels a node: each GPU's scale-out rail (the NIC behind its PCIe switch,
the NIC's driver and RDMA device), both ends' PCIe links as trained, the xGMI mesh (KFD) and
every xGMI link's state (gpu_metrics), GPUDirect RDMA, and each rail's Ethernet link as the kernel
has it now (state, negotiated speed, MTU).  When the agent has written its RCCL topology file
(``--artifact-dir``, default /etc/amd/scale-out), the report also checks that the file places each
GPU and its NIC as this node's PCIe tree does, and that ``rccl.env`` names the rails' current RDMA
devices and, when it pins ``NCCL_IB_GID_INDEX``, a slot that holds a RoCE v2 GID on every one.

    python -m network_operator_amd.agent.report            # a table
    python -m network_operator_amd.agent.report --json     # the same as one JSON document
    python -m network_operator_amd.agent.report --min-link-speed-gbps 400   # the policy's floor too
    SYSFS_ROOT=/path/to/sys python -m network_operator_amd.agent.report

It reads what the agent reads, through the same native code (``_netop_native``), so a problem
shown here is the reason the agent would give.  Nothing is changed.  The exit status is 1 when
something would keep the label off the node with the policy defaults plus `requireFullPcieLink`
and `gpuDirectRdma: Any` (and `minLinkSpeedGbps`, when given).  A link that is down is not a
problem by itself: the agent brings the rails up.
"""

from __future__ import annotations

import argparse
import json
import os
import platform
import sys
from typing import List

from . import native


def _netdev(root: str, bdf: str, ifname: str) -> dict:
    """The rail's Ethernet link as ``ip link`` and ethtool show it, read under its PCI function
    (a container in its own network namespace has no /sys/class/net entry for the host's NICs).
    The kernel reports speed -1 (or refuses the read) while there is no carrier."""
    d = os.path.join(root, "bus", "pci", "devices", bdf, "net", ifname)
    if not bdf or not os.path.isdir(d):
        d = os.path.join(root, "class", "net", ifname)

    def attr(name: str) -> str:
        try:
            with open(os.path.join(d, name)) as f:
                return f.read().strip()
        except OSError:
            return ""

    speed = attr("speed")
    mbps = int(speed) if speed.lstrip("-").isdigit() else -1
    mtu = attr("mtu")
    return {"operstate": attr("operstate") or "unknown", "speed_gbps": mbps / 1000 if mbps > 0 else None,
            "mtu": int(mtu) if mtu.isdigit() else None}


def _link_str(link: dict) -> str:
    out = link["operstate"]
    if link["speed_gbps"]:
        out += f" {link['speed_gbps']:g}G"
    if link["mtu"]:
        out += f" mtu {link['mtu']}"
    return out


def collect(root: str, min_link_speed_gbps: float = 0, artifact_dir: str = "") -> dict:
    n = native()
    d = n.discover(root)
    nics = {x["ifname"]: x for x in d["nics"]}
    rails = []
    for p in d["pairs"]:
        nic = nics.get(p["nic"], {})
        rails.append({"gpu": p["gpu"], "nic": p["nic"], "path": p["path"], "driver": nic.get("driver", ""),
                      "rdma_dev": nic.get("rdma_dev", ""), "nic_pcie": n.read_pcie_link(root, nic.get("bdf", "")),
                      "gpu_pcie": n.read_pcie_link(root, p["gpu"]), "link": _netdev(root, nic.get("bdf", ""), p["nic"])})
    x = n.read_xgmi(root)
    # Bounded like the agent's own read: a wedged SMU is a finding, not a hung report.
    health = n.read_xgmi_health(root, [g["bdf"] for g in d["gpus"]], 5000)
    gdr = n.detect_gdr(root, platform.release())
    problems: List[str] = []
    paired = {r["gpu"] for r in rails}
    problems += [f"GPU {g['bdf']}: no scale-out NIC behind its PCIe switch" for g in d["gpus"] if g["bdf"] not in paired]
    problems += [f"{r['nic']}: no RDMA device (load its RDMA driver)" for r in rails if not r["rdma_dev"]]
    for r in rails:
        if r["nic_pcie"]["degraded"]:
            problems.append(f"{r['nic']}: PCIe link {r['nic_pcie']['str']}")
        if r["gpu_pcie"]["known"] and r["gpu_pcie"]["width"] < r["gpu_pcie"]["max_width"]:
            problems.append(f"GPU {r['gpu']}: PCIe link {r['gpu_pcie']['str']}")
        speed = r["link"]["speed_gbps"]
        if min_link_speed_gbps and speed and speed < min_link_speed_gbps:
            problems.append(f"{r['nic']}: link negotiated {speed:g} Gb/s, below the required {min_link_speed_gbps:g}")
    if x["pairs_connected"] < x["pairs_expected"]:
        problems.append(f"xGMI mesh: {x['pairs_connected']} of {x['pairs_expected']} GPU pairs linked")
    for h in health:
        if h.get("late"):
            problems.append(f"GPU {h['bdf']}: gpu_metrics did not answer in 5s (a wedged or resetting SMU?)")
        down = [i for i, s in enumerate(h["status"]) if s == 0]
        if down:
            problems.append(f"GPU {h['bdf']}: xGMI link(s) {', '.join(map(str, down))} down")
    if gdr["mode"] == "none":
        problems.append("GPUDirect RDMA unavailable (no amdkfd peer-memory client, no RDMA dma-buf)")
    topo_file = None
    tf = os.path.join(artifact_dir, "rccl-topo.xml") if artifact_dir else ""
    if tf and os.path.isfile(tf):
        from ..models.topology import NodeTopology
        from ..validate import topo_file_agrees

        import xml.etree.ElementTree as ET

        with open(tf, errors="replace") as f:
            text = f.read()
        try:
            topo_file = dict(topo_file_agrees(text, NodeTopology.discover(root, with_xgmi=False)), path=tf)
        except ET.ParseError as e:  # torn or foreign: RCCL would refuse it too
            topo_file = {"ok": False, "gpus_missing": [], "pairs_split": [], "path": tf, "error": str(e)}
            problems.append(f"{tf}: not a topology file RCCL can read ({e})")
        if topo_file["gpus_missing"]:
            problems.append(f"{tf}: GPU(s) {', '.join(topo_file['gpus_missing'])} missing (a stale file?)")
        for gpu, nic in topo_file["pairs_split"]:
            problems.append(f"{tf}: places {nic} under another switch than GPU {gpu} (a stale file?)")
    rccl_env = _check_rccl_env(root, os.path.join(artifact_dir, "rccl.env") if artifact_dir else "", rails, problems)
    return {"sysfs_root": root, "gpus": len(d["gpus"]), "rails": rails,
            "xgmi": {"pairs": f"{x['pairs_connected']}/{x['pairs_expected']}", "links": health},
            "gpudirect_rdma": gdr["mode"], "kernel": gdr["kernel"], "left_alone": d.get("excluded", {}),
            "rccl_topology_file": topo_file, "rccl_env": rccl_env,
            "problems": problems}


def _check_rccl_env(root: str, path: str, rails: List[dict], problems: List[str]):
    """The agent's rccl.env against the node as it is now: every rail's current RDMA device named
    (a driver reload renumbers them), none that is gone, and, when it pins NCCL_IB_GID_INDEX=k,
    slot k of every named device holding a RoCE v2 GID (the RDMA core re-adds a netdev's GIDs in
    whatever slot is free after its link went down)."""
    if not path or not os.path.isfile(path):
        return None
    env = {}
    with open(path, errors="replace") as f:  # whatever is in the file, the report says what it found
        for line in f:
            k, sep, v = line.strip().partition("=")
            if sep and not k.startswith("#"):
                env[k] = v
    named = [h for h in env.get("NCCL_IB_HCA", "").lstrip("=^").split(",") if h]
    devs = {h.split(":", 1)[0]: int(h.split(":", 1)[1]) if ":" in h and h.split(":", 1)[1].isdigit() else 1 for h in named}
    current = {r["rdma_dev"] for r in rails if r["rdma_dev"]}
    out = {"path": path, "hcas": sorted(devs), "gid_index": env.get("NCCL_IB_GID_INDEX"), "bad_gid_slots": []}
    for dev in sorted(set(devs) - current):
        problems.append(f"{path}: names RDMA device {dev}, which no rail has now (a driver reload renumbered it?)")
    for r in rails:
        if r["rdma_dev"] and devs and r["rdma_dev"] not in devs:
            problems.append(f"{path}: does not name {r['nic']}'s RDMA device {r['rdma_dev']}")
    gid = env.get("NCCL_IB_GID_INDEX", "")
    if gid.isdigit():
        for dev, port in sorted(devs.items()):
            base = os.path.join(root, "class", "infiniband", dev, "ports", str(port))
            try:
                with open(os.path.join(base, "gids", gid), errors="replace") as f:
                    value = f.read().strip()
                with open(os.path.join(base, "gid_attrs", "types", gid), errors="replace") as f:
                    kind = f.read().strip()
            except (OSError, ValueError):  # (ValueError: a NUL in a device name from the file)
                value, kind = "", ""
            # (L3 pins an IPv4-mapped GID, L2 the link-local one: either, as long as it is RoCE v2)
            if kind != "RoCE v2" or not value or set(value) <= {"0", ":"}:
                out["bad_gid_slots"].append(dev)
                problems.append(f"{path}: NCCL_IB_GID_INDEX={gid}, but slot {gid} of {dev} port {port} holds no RoCE v2 "
                                f"GID ({value or 'unreadable'}{', ' + kind if kind else ''}): a stale index?")
    return out


def render(r: dict) -> str:
    out = [f"{r['gpus']} GPU(s), {len(r['rails'])} scale-out rail(s); xGMI pairs {r['xgmi']['pairs']}; "
           f"GPUDirect RDMA {r['gpudirect_rdma']} (kernel {r['kernel']})", ""]
    out.append(f"{'GPU':14} {'NIC':14} {'path':5} {'driver':10} {'RDMA':10} {'link':20} {'NIC PCIe':30} {'GPU PCIe':30}")
    for x in r["rails"]:
        out.append(f"{x['gpu']:14} {x['nic']:14} {x['path']:5} {x['driver'] or '-':10} {x['rdma_dev'] or 'none':10} "
                   f"{_link_str(x['link']):20} {x['nic_pcie']['str']:30} {x['gpu_pcie']['str']:30}")
    known = [h for h in r["xgmi"]["links"] if h["known"]]
    if known:
        letter = {1: "U", 0: "D", -1: "X"}
        out += ["", "xGMI links (gpu_metrics " + known[0]["revision"] + "; U up, D down, X no link):"]
        for h in known:
            out.append(f"  {h['bdf']}  {''.join(letter[s] for s in h['status'])}  x{h['width']} at {h['speed_gbps']} Gb/s")
    elif r["xgmi"]["links"]:
        out += ["", "xGMI link state not read: " + r["xgmi"]["links"][0]["error"]]
    if r.get("rccl_topology_file"):
        t = r["rccl_topology_file"]
        out += ["", f"RCCL topology file {t['path']}: " + ("matches this node" if t["ok"] else "does not match this node")]
    if r.get("rccl_env"):
        e = r["rccl_env"]
        out += [f"RCCL environment {e['path']}: HCAs {', '.join(e['hcas']) or '-'}, GID index {e['gid_index'] or 'not pinned'}"]
    out += ["", "Problems:" if r["problems"] else "No problems found."]
    out += [f"  - {p}" for p in r["problems"]]
    return "\n".join(out)


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m network_operator_amd.agent.report", description=__doc__.split("\n\n")[0])
    ap.add_argument("--json", action="store_true", help="one JSON document instead of the table")
    ap.add_argument("--min-link-speed-gbps", type=float, default=0,
                    help="also name a rail whose link negotiated below this (the policy's minLinkSpeedGbps)")
    ap.add_argument("--artifact-dir", default="/etc/amd/scale-out",
                    help="where the agent writes rccl-topo.xml (checked against this node when present)")
    a = ap.parse_args(argv)
    r = collect(os.environ.get("SYSFS_ROOT", "/sys/"), a.min_link_speed_gbps, a.artifact_dir)
    print(json.dumps(r, indent=1) if a.json else render(r))
    return 1 if r["problems"] else 0


if __name__ == "__main__":
    sys.exit(main())
