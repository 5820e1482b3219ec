"""The agent binary itself on a real MI355X node (``-m gpu``: runs on the GPU box).

The box gives no NET_ADMIN / NET_RAW and no user namespaces, so the agent runs with
``--dry-run``: the real discovery, xGMI and GPUDirect checks and topology writer against the
box's own /sys, with no link, address or label change.  The pieces that need privileges run in
the netns harness (tests/test_netns_integration.py, tests/test_e2e.py).
"""

import json
import os
import re
import subprocess
from pathlib import Path

import pytest

from network_operator_amd.agent import native
from network_operator_amd.utils.paths import native_bin


@pytest.mark.gpu
def test_agent_dry_run_on_this_node(tmp_path):
    topo, status = tmp_path / "rccl-topo.xml", tmp_path / "status.json"
    r = subprocess.run([str(native_bin("discover")), "--dry-run", "--mode=L3", "--mtu=9000", "--xgmi-expect=0",
                        f"--rccl-topo={topo}", f"--status-file={status}", "-v=2"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-3000:]
    st = json.loads(status.read_text())
    root = os.environ.get("SYSFS_ROOT", "/sys/")
    want = native().discover(root, "affine")
    index = {g["bdf"]: g["index"] for g in want["gpus"]}
    pairs = re.findall(r"GPU (\d+) \((\S+)\) <-> NIC (\S+) \((\S+), ", r.stderr)
    assert [(g, b, n) for g, b, n, _ in pairs] == [(str(index[p["gpu"]]), p["gpu"], p["nic"]) for p in want["pairs"]]
    x = native().read_xgmi(root)
    assert st["xgmi_pairs"] == f"{x['pairs_connected']}/{x['pairs_expected']}"
    # Rails whose NIC has no RDMA device (RDMA driver not loaded) are named, exactly those.
    bare = sorted(p["nic"] for p in want["pairs"] if not any(n["ifname"] == p["nic"] and n["rdma_dev"]
                                                              for n in want["nics"]))
    assert sorted(filter(None, st.get("nics_without_rdma", "").split(","))) == bare, (st, bare)
    assert st["dry_run"] == "true" and st["ready"] is False
    xml = topo.read_text()
    assert xml.startswith('<system version="2">') and xml.count("<net ") == len(want["pairs"])
    out = Path(os.environ.get("GRAFT_REPO_ROOT", ".")) / "gpurun_out"
    if out.is_dir():  # evidence for profiles/ when run through gpurun
        (out / "agent_dry_run_box.json").write_text(json.dumps({"status": st, "pairs": pairs,
                                                                "log_tail": r.stderr[-4000:]}, indent=1))


# ------------------------------------------------------------------------------------------
# An independent oracle for the GPU <-> NIC pairing: plain Python over sysfs, no native code.
# ------------------------------------------------------------------------------------------
_BDF = re.compile(r"^[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.[0-7]$")


def _read(path, default=""):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return default


def sysfs_oracle(root="/sys/"):
    """GPUs (amdgpu PCI functions), physical PCI network functions with a netdev (and their RDMA
    device, if any) and, per GPU, the NICs behind the same PCIe switch, from realpaths alone.
    The rule, stated independently of the agent: a NIC is affine to a GPU when their deepest
    common PCI ancestor is below the root port (a switch port); among those, the closest
    (deepest common ancestor) is the GPU's rail NIC.  No driver allow-list: a NIC family the
    agent does not know shows up here as an unpaired affine NIC."""
    root = root.rstrip("/")

    def chain(dev_path):
        real = os.path.realpath(dev_path)
        parts = real.split("/devices/", 1)[1].split("/") if "/devices/" in real else []
        return [p for p in parts if p]

    gpus = {}
    drv = os.path.join(root, "bus/pci/drivers/amdgpu")
    for name in sorted(os.listdir(drv)) if os.path.isdir(drv) else []:
        if _BDF.match(name):
            dev = os.path.join(root, "bus/pci/devices", name)
            gpus[name] = {"chain": chain(dev), "numa": _read(os.path.join(dev, "numa_node"), "-1")}
    nics = {}
    cls = os.path.join(root, "class/net")
    for ifname in sorted(os.listdir(cls)) if os.path.isdir(cls) else []:
        dev = os.path.join(cls, ifname, "device")
        if not os.path.exists(dev):
            continue  # virtual
        c = chain(dev)
        if not c or not _BDF.match(c[-1]):
            continue
        if not _read(os.path.join(dev, "class")).startswith("0x02"):
            continue  # not a network controller
        ib = os.path.join(dev, "infiniband")
        rdma = sorted(os.listdir(ib)) if os.path.isdir(ib) else []
        nics[ifname] = {"chain": c, "bdf": c[-1], "rdma": rdma[0] if rdma else None,
                        "numa": _read(os.path.join(dev, "numa_node"), "-1"),
                        "driver": os.path.basename(os.path.realpath(os.path.join(dev, "driver")))}
    affine = {}
    for g, gd in gpus.items():
        cands = []
        for n, nd in nics.items():
            k = 0
            while k < min(len(gd["chain"]), len(nd["chain"])) and gd["chain"][k] == nd["chain"][k]:
                k += 1
            # chain[0] is the host bridge (pciDDDD:BB), chain[1] the root port: a common
            # component past those is a switch both sit below.
            if k >= 3:
                cands.append((k, n))
        best = max((k for k, _ in cands), default=None)
        affine[g] = {"closest": sorted(n for k, n in cands if k == best), "all": sorted(n for _, n in cands)}
    return {"gpus": gpus, "nics": nics, "affine": affine}


@pytest.mark.gpu
def test_pairing_matches_an_independent_sysfs_oracle(tmp_path):
    """the agent's pairs (the `discover` binary's log and its NCCL_TOPO_FILE)
    checked against plain-Python sysfs walking, whichever NIC family (mlx5, ionic, ...) the box
    has."""
    import xml.etree.ElementTree as ET

    root = os.environ.get("SYSFS_ROOT", "/sys/")
    o = sysfs_oracle(root)
    if not o["gpus"]:
        pytest.skip("no amdgpu GPU in this sysfs")
    topo = tmp_path / "rccl-topo.xml"
    r = subprocess.run([str(native_bin("discover")), "--dry-run", "--xgmi-expect=-1", f"--rccl-topo={topo}"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-3000:]
    pairs = re.findall(r"GPU (\d+) \((\S+)\) <-> NIC (\S+) \((\S+), (no rdma|\S+), path (\w+)\)", r.stderr)
    got = {b: n for _, b, n, _, _, _ in pairs}
    # not vacuous: the oracle sees affine NICs on every box of this pool, and so must the agent
    assert any(a["all"] for a in o["affine"].values()) == bool(pairs), (o["affine"], r.stderr[-2000:])
    # 1. every GPU with an affine RDMA NIC is paired, with one of its closest NICs (or, when a
    #    closer one went to an earlier GPU, another affine one); no NIC twice.
    assert len(set(got.values())) == len(got)
    for g, a in o["affine"].items():
        if not a["all"]:
            assert g not in got, (g, got.get(g))
            continue
        assert g in got, (g, a)
        assert got[g] in a["all"], (g, got[g], a)
        if got[g] not in a["closest"]:
            assert all(n in got.values() for n in a["closest"]), (g, got[g], a)
    # 2. each pair's PCI function and RDMA device as sysfs has them
    for _, b, n, bdf, rdma, _ in pairs:
        want_rdma = o["nics"][n]["rdma"] or "no rdma"
        assert o["nics"][n]["bdf"] == bdf and want_rdma == rdma, (n, o["nics"][n], bdf, rdma)
        assert o["nics"][n]["numa"] == o["gpus"][b]["numa"], (n, b)
    # 3. the NCCL_TOPO_FILE names each pair's RDMA device under the GPU's own top switch
    xml = ET.fromstring(topo.read_text())
    top_of = {}
    for cpu in xml.findall("cpu"):
        for top in cpu.findall("pci"):
            for p in top.iter("pci"):
                top_of[p.get("busid")] = top.get("busid")
            for net in top.iter("net"):
                top_of["net:" + net.get("name")] = top.get("busid")
    for _, b, n, _, rdma, _ in pairs:
        net = n if rdma == "no rdma" else rdma  # RCCL's name for it: the IB device, else the netdev
        assert top_of.get("net:" + net) == top_of.get(b), (b, n, net)
    families = sorted({o["nics"][n]["driver"] + (" (RDMA)" if o["nics"][n]["rdma"] else " (no RDMA device)")
                       for n in got.values()})
    out = Path(os.environ.get("GRAFT_REPO_ROOT", ".")) / "gpurun_out"
    if out.is_dir():
        (out / "pairing_oracle_box.json").write_text(json.dumps(
            {"nic_families_paired": families, "pairs": pairs, "oracle_affine": o["affine"],
             "rdma_nics": {n: {k: v for k, v in d.items() if k != "chain"} for n, d in o["nics"].items()}}, indent=1))


@pytest.mark.gpu
def test_rdma_discovery_on_this_node_leaves_every_gpu_rail_alone():
    """Round 4, on the box's real PCIe tree: host-nic (rdma) discovery takes no NIC that sits
    below a GPU's PCIe switch.  Checked against the independent oracle above: every NIC the oracle
    finds affine to some GPU is left out (named with a GPU), and what discovery keeps is disjoint
    from the amd-so agent's pairs."""
    root = os.environ.get("SYSFS_ROOT", "/sys/")
    o = sysfs_oracle(root)
    if not o["gpus"]:
        pytest.skip("no amdgpu GPU in this sysfs")
    d = native().discover(root, mode="rdma", drivers=[])  # every PCI NIC driver: the widest host-nic policy
    affine = {n for a in o["affine"].values() for n in a["all"]}
    rdma_affine = {n for n in affine if o["nics"][n]["rdma"]}
    assert rdma_affine <= set(d["excluded"]), (sorted(rdma_affine), d["excluded"])
    assert all("scale-out rail of GPU" in why for why in d["excluded"].values())
    pairs = {p["nic"] for p in native().discover(root, "affine", drivers=[])["pairs"]}
    assert not set(d["ifnames"]) & pairs, (d["ifnames"], sorted(pairs))
    out = Path(os.environ.get("GRAFT_REPO_ROOT", ".")) / "gpurun_out"
    if out.is_dir():
        (out / "rdma_discovery_box.json").write_text(json.dumps(
            {"host_nics_kept": d["ifnames"], "left_alone": d["excluded"], "gpu_affine_rdma_nics": sorted(rdma_affine),
             "amd_so_pairs": sorted(pairs)}, indent=1))


def test_oracle_agrees_with_agent_on_the_captured_node(tmp_path):
    """The oracle itself, against the fake tree of the captured 8x MI355X node (CPU-side
    counterpart of the box test; the fixture's rail NICs are mlx5)."""
    from network_operator_amd.testing import fakesysfs

    fakesysfs.build_mi355x_node(tmp_path)
    o = sysfs_oracle(str(tmp_path) + "/")
    want = native().discover(str(tmp_path) + "/", "affine")
    assert len(o["gpus"]) == 8 and all(len(a["closest"]) == 1 for a in o["affine"].values())
    assert {p["gpu"]: p["nic"] for p in want["pairs"]} == {g: a["closest"][0] for g, a in o["affine"].items()}


@pytest.mark.gpu
def test_xgmi_link_state_from_gpu_metrics_matches_amd_smi(tmp_path):
    """The agent reads each GPU's trained xGMI links from amdgpu's gpu_metrics without amd-smi;
    on this box, for every GPU amd-smi sees (netop-xgmi-counters, the library), the link status,
    width and bit rate agree, and the agent's dry run reports every GPU of the node."""
    from network_operator_amd.utils.paths import LIB_DIR

    root = os.environ.get("SYSFS_ROOT", "/sys/")
    gpus = [g["bdf"] for g in native().discover(root, "affine")["gpus"]]  # (KFD filters the GPUs we cannot open)
    if not gpus:
        pytest.skip("no amdgpu GPU in this sysfs")
    mine = {h["bdf"]: h for h in native().read_xgmi_health(root, gpus)}
    assert len(mine) == len(gpus)
    assert all(h["known"] for h in mine.values()), {b: h["error"] for b, h in mine.items()}
    r = subprocess.run([str(LIB_DIR / "netop-xgmi-counters")], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    smi = json.loads(r.stdout)["gpus"]
    assert smi, r.stdout
    letter = {1: "U", 0: "D", -1: "X"}
    for g in smi:
        h = mine[g["bdf"]]
        assert "".join(letter[s] for s in h["status"]) == g["link_status"], (h, g)
        assert (h["width"], h["speed_gbps"]) == (g["xgmi_link_width"], g["xgmi_link_speed"]), (h, g)
    status = tmp_path / "status.json"
    d = subprocess.run([str(native_bin("discover")), "--dry-run", "--xgmi-expect=0", f"--status-file={status}"],
                       capture_output=True, text=True, timeout=60)
    assert d.returncode == 0, d.stderr[-3000:]
    st = json.loads(status.read_text())
    up = sum(s == 1 for h in mine.values() for s in h["status"])
    down = sum(s == 0 for h in mine.values() for s in h["status"])
    assert st["xgmi_links"].startswith(f"{up} up, {down} down on {len(mine)} GPUs"), st
    out = Path(os.environ.get("GRAFT_REPO_ROOT", ".")) / "gpurun_out"
    if out.is_dir():
        (out / "xgmi_health_box.json").write_text(json.dumps(
            {"agent_status_xgmi_links": st["xgmi_links"], "gpu_metrics": list(mine.values()), "amd_smi": smi}, indent=1))


@pytest.mark.gpu
def test_pcie_links_of_every_rail_read_as_sysfs_has_them():
    """--require-full-pcie on the box's real PCIe tree: the agent's reading of every paired GPU's
    and NIC's trained and maximum link agrees with the raw sysfs text.  Which links trained below
    their maximum is recorded, not asserted (that is the hardware's state, not the agent's)."""
    root = os.environ.get("SYSFS_ROOT", "/sys/")
    o = sysfs_oracle(root)
    want = native().discover(root, "affine")
    if not want["pairs"]:
        pytest.skip("no GPU <-> NIC pair in this sysfs")
    seen = {}
    for p in want["pairs"]:
        for bdf in (p["gpu"], o["nics"][p["nic"]]["bdf"]):
            got = native().read_pcie_link(root, bdf)
            d = os.path.join(root, "bus/pci/devices", bdf)
            raw = {a: _read(os.path.join(d, a)) for a in ("current_link_speed", "current_link_width", "max_link_speed",
                                                          "max_link_width")}
            assert got["known"], (bdf, raw)
            assert got["speed_gts"] == float(raw["current_link_speed"].split()[0]), (bdf, raw, got)
            assert got["width"] == int(raw["current_link_width"]) and got["max_width"] == int(raw["max_link_width"]), (bdf, raw)
            seen[bdf] = got["str"]
    for bdf, text in seen.items():  # "of" exactly when the link is below its maximum
        got = native().read_pcie_link(root, bdf)
        assert (" of " in text) == got["degraded"], (bdf, text, got)
    out = Path(os.environ.get("GRAFT_REPO_ROOT", ".")) / "gpurun_out"
    if out.is_dir():
        (out / "pcie_links_rails_box.json").write_text(json.dumps(seen, indent=1))


@pytest.mark.gpu
def test_node_report_on_this_node():
    """The read-only node report on the box: one rail per paired GPU, the xGMI link state of every
    GPU read, GPUDirect RDMA detected; its problems (if any) are the hardware's, recorded."""
    import sys

    r = subprocess.run([sys.executable, "-m", "network_operator_amd.agent.report", "--json"], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode in (0, 1), r.stderr[-2000:]
    rep = json.loads(r.stdout)
    want = native().discover(os.environ.get("SYSFS_ROOT", "/sys/"), "affine")
    assert sorted((x["gpu"], x["nic"]) for x in rep["rails"]) == sorted((p["gpu"], p["nic"]) for p in want["pairs"])
    assert all(h["known"] for h in rep["xgmi"]["links"]), rep["xgmi"]
    assert rep["gpudirect_rdma"] != "none", rep
    assert all(x["link"]["operstate"] != "unknown" for x in rep["rails"]), rep["rails"]  # read under the PCI function
    assert (r.returncode == 1) == bool(rep["problems"])
    out = Path(os.environ.get("GRAFT_REPO_ROOT", ".")) / "gpurun_out"
    if out.is_dir():
        (out / "node_report_box.json").write_text(json.dumps(rep, indent=1))
        (out / "node_report_box.txt").write_text(subprocess.run(
            [sys.executable, "-m", "network_operator_amd.agent.report"], capture_output=True, text=True,
            timeout=60).stdout)


@pytest.mark.gpu
def test_topo_tool_on_this_node():
    """``netop-topo`` (the agent image's look at a node): on the box, every GPU's xGMI links and
    PCIe link read, agreeing with the report's readings (Python binding, same sysfs)."""
    r = subprocess.run([str(native_bin("netop-topo"))], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-2000:]
    j = json.loads(r.stdout)
    root = os.environ.get("SYSFS_ROOT", "/sys/")
    health = {h["bdf"]: h for h in native().read_xgmi_health(root, [g["bdf"] for g in j["gpus"]])}
    assert j["gpus"]
    for g in j["gpus"]:
        h, x = health[g["bdf"]], g["xgmi_links"]
        assert x["known"] == h["known"], (g, h)
        if x["known"]:
            assert x["up"] == sum(s == 1 for s in h["status"]) and x["width"] == h["width"], (g, h)
        assert g["pcie"]["known"], g  # amdgpu functions carry current_link_* on every box seen
    out = Path(os.environ.get("GRAFT_REPO_ROOT", ".")) / "gpurun_out"
    if out.is_dir():
        (out / "netop_topo_box.json").write_text(json.dumps(j, indent=1))


@pytest.mark.gpu
def test_require_rdma_dry_run_on_this_node_names_every_rail_without_an_rdma_device(tmp_path):
    """VERDICT r5 #1 on the box: with --require-rdma (the operator's default), a dry run says which
    rails a real start would wait for -- on this pool's Pollara boxes all 8 (ionic, no
    ionic_rdma) -- and, where every rail has its device, nothing.  The bounded gpu_metrics reads
    (--sysfs-read-timeout) answer within the timeout on a healthy SMU."""
    status = tmp_path / "status.json"
    r = subprocess.run([str(native_bin("discover")), "--dry-run", "--require-rdma", "--mode=L3", "--xgmi-expect=0",
                        "--sysfs-read-timeout=5s", f"--status-file={status}", "-v=1"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-3000:]
    st = json.loads(status.read_text())
    bare = sorted(filter(None, st.get("nics_without_rdma", "").split(",")))
    waits = re.findall(r"a real start would wait for RDMA devices on (\d+) rails?", r.stderr)
    assert (waits == [str(len(bare))]) if bare else not waits, (waits, bare, r.stderr[-2000:])
    assert "did not answer" not in st.get("xgmi_error", ""), st
    out = Path(os.environ.get("GRAFT_REPO_ROOT", ".")) / "gpurun_out"
    if out.is_dir():
        (out / "agent_dry_run_require_rdma_box.json").write_text(json.dumps(
            {"status": st, "waits_for": waits, "log_tail": r.stderr[-4000:]}, indent=1))
