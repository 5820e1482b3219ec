"""NCCL_TOPO_FILE written by the agent (native/src/artifacts.cpp generate_rccl_topo).

CPU: golden XML for the captured 8x MI355X node (tests/fixtures/mi355x_node_topology.json ->
fake sysfs), the structure RCCL needs (GPU and NIC functions folded under the same switch as
RCCL folds them), and the agent's rccl.env pointing at it.

GPU (-m gpu): RCCL itself loads the file generated from the box's real /sys — a fresh process
per case, because RCCL reads NCCL_TOPO_FILE once at communicator init — and its topology dump
(NCCL_TOPO_DUMP_FILE) must place the GPU (and, when RCCL's network plugin can use one of the
file's NICs, that NIC) exactly where the file put it.  The reference's counterpart is the
HCCL-consumed gaudinet.json (reference cmd/discover/gaudinet.go:28-89).
"""

import json
import os
import subprocess
import sys
import textwrap
import xml.etree.ElementTree as ET
from pathlib import Path

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from network_operator_amd.testing import fakesysfs

ROOT = Path(__file__).resolve().parent.parent
GOLDEN = ROOT / "tests" / "fixtures" / "mi355x_rccl_topo.xml"


def _chain(root: ET.Element, busid: str):
    """[cpu numaid, outer pci busid, ..., busid] for the pci element `busid`, or None."""
    def walk(el, path):
        for c in el:
            here = path + [c.get("numaid") if c.tag == "cpu" else c.get("busid")] if c.tag in ("cpu", "pci") else path
            if c.tag == "pci" and c.get("busid") == busid:
                return here
            r = walk(c, here)
            if r:
                return r
        return None
    return walk(root, [])


def _net_chain(root: ET.Element, name: str):
    def walk(el, path):
        for c in el:
            if c.tag == "net" and c.get("name") == name:
                return path
            here = path + [c.get("numaid") if c.tag == "cpu" else c.get("busid")] if c.tag in ("cpu", "pci") else path
            r = walk(c, here)
            if r:
                return r
        return None
    return walk(root, [])


def test_topo_xml_golden_for_captured_node(native, tmp_path):
    fakesysfs.build_mi355x_node(tmp_path)
    xml = native.rccl_topo_xml(str(tmp_path) + "/", cpu=fakesysfs.MI355X_HOST_CPU)
    assert xml == GOLDEN.read_text()


def test_topo_xml_gpu_and_nic_share_rccl_switch(native, tmp_path):
    fx = fakesysfs.build_mi355x_node(tmp_path)
    root = ET.fromstring(native.rccl_topo_xml(str(tmp_path) + "/", cpu=fakesysfs.MI355X_HOST_CPU))
    assert root.tag == "system" and root.get("version") == "2"
    for cpu in root.iter("cpu"):  # RCCL refuses a <cpu> without these (its xml.h "Attribute arch ... not found")
        assert {"numaid", "affinity", "arch", "vendor", "familyid", "modelid"} <= set(cpu.keys())
    gpus = [p.get("busid") for p in root.iter("pci") if p.get("class") == "0x120000"]
    assert sorted(gpus) == sorted(g["bdf"] for g in fx["gpus"])
    nets = [n.get("name") for n in root.iter("net")]
    assert len(nets) == 8 and len(set(nets)) == 8  # the scale-out NICs only, not the management ports
    assert not list(root.iter("xgmi")) and not list(root.iter("gpu"))  # left to RCCL (see artifacts.hpp)
    pairs = {p["gpu"]: p["nic"] for p in native.discover(str(tmp_path) + "/")["pairs"]}
    rdma = {n["ifname"]: n["rdma_dev"] for n in native.discover(str(tmp_path) + "/")["nics"]}
    for gpu, nic in pairs.items():
        g, n = _chain(root, gpu), _net_chain(root, rdma[nic])
        assert g[0] == n[0] and g[1] == n[1], (gpu, nic, g, n)  # same CPU, same top switch
        assert len(g) == 5 and len(n) == 4  # cpu > 01 > 06 > 08 > GPU;  cpu > 01 > 03 > NIC (RCCL folding)


def test_validate_checks_topology_file_against_live_tree(native, tmp_path):
    """validate.py's rccl_topology_file check: the golden file agrees with the fixture node; a
    file that puts a rail NIC under another GPU's switch does not."""
    from network_operator_amd import validate
    from network_operator_amd.models.topology import NodeTopology

    fakesysfs.build_mi355x_node(tmp_path)
    topo = NodeTopology.discover(str(tmp_path) + "/")
    good = GOLDEN.read_text()
    assert validate.topo_file_agrees(good, topo)["ok"]
    bad = good.replace('<net name="mlx5_1" port="1"/>', '<net name="tmp" port="1"/>').replace(
        '<net name="mlx5_3" port="1"/>', '<net name="mlx5_1" port="1"/>')
    r = validate.topo_file_agrees(bad, topo)
    assert not r["ok"] and len(r["pairs_split"]) == 2, r


def test_topo_xml_extra_interface_without_rdma(native, tmp_path):
    fakesysfs.build_mi355x_node(tmp_path)
    root = ET.fromstring(native.rccl_topo_xml(str(tmp_path) + "/", interfaces=["ens9np0", "lo"], cpu=fakesysfs.MI355X_HOST_CPU))
    # ens9np0 (a management port, not GPU-affine) is listed under its RDMA device name, the
    # name RCCL's IB plugin gives it; lo is virtual -> nothing PCIe to pin.
    names = [n.get("name") for n in root.iter("net")]
    assert "mlx5_8" in names and len(names) == 9 and "lo" not in names
    # Without an RDMA device the socket plugin's name (the netdev) is used.
    import shutil

    for ib in tmp_path.glob("devices/**/infiniband/mlx5_8"):
        shutil.rmtree(ib)
    root = ET.fromstring(native.rccl_topo_xml(str(tmp_path) + "/", interfaces=["ens9np0"], cpu=fakesysfs.MI355X_HOST_CPU))
    assert "ens9np0" in [n.get("name") for n in root.iter("net")]


# ------------------------------------------------------------------------------------------
# On the GPU box: RCCL loads the file.
# ------------------------------------------------------------------------------------------
_RCCL_INIT = textwrap.dedent("""
    import os, sys, torch, torch.distributed as dist
    d = torch.device("cuda", 0); torch.cuda.set_device(d)
    dist.init_process_group("nccl", init_method="file://" + os.environ["NETOP_TEST_STORE"], rank=0, world_size=1,
                            device_id=d)
    x = torch.ones(4096, device=d); dist.all_reduce(x); torch.cuda.synchronize()
    dist.destroy_process_group()
""")


def _rccl_dump(tmp_path, topo_file, extra_env=None, tag="run"):
    dump = tmp_path / f"dump_{tag}.xml"
    env = dict(os.environ, NETOP_TEST_STORE=str(tmp_path / f"store_{tag}"),
               NCCL_TOPO_DUMP_FILE=str(dump), NCCL_DEBUG="INFO", NCCL_DEBUG_SUBSYS="INIT,GRAPH,NET")
    if topo_file:
        env["NCCL_TOPO_FILE"] = str(topo_file)
    env.update(extra_env or {})
    r = subprocess.run([sys.executable, "-c", _RCCL_INIT], env=env, capture_output=True, text=True, timeout=110)
    return r, (ET.parse(dump).getroot() if dump.exists() else None)


def _ipv4_ifaces():
    import psutil

    out = {}
    for name, addrs in psutil.net_if_addrs().items():
        for a in addrs:
            if a.family == 2:
                out[name] = a.address
    return out


@pytest.mark.gpu
def test_rccl_loads_generated_topology(native, tmp_path):
    xml = native.rccl_topo_xml("/sys/")
    topo = tmp_path / "rccl-topo.xml"
    topo.write_text(xml)
    mine = ET.fromstring(xml)
    r, dump = _rccl_dump(tmp_path, topo, tag="file")
    assert r.returncode == 0, r.stderr[-3000:]
    assert f"Loading topology file {topo}" in r.stdout + r.stderr or "NCCL_TOPO_FILE set by environment" in r.stdout + r.stderr
    assert dump is not None and dump.get("version") == mine.get("version")
    # the visible GPU's pci element in the dump, and its ancestry there vs in our file
    seen = [p.get("busid") for p in dump.iter("pci") if p.find("gpu") is not None]
    assert len(seen) == 1, ET.tostring(dump)[:2000]
    busid = seen[0]
    assert _chain(dump, busid) == _chain(mine, busid), (ET.tostring(dump)[:3000], _chain(mine, busid))
    # RCCL's own detection without the file agrees with it (the file mirrors RCCL's folding).
    r0, auto = _rccl_dump(tmp_path, None, tag="auto")
    assert r0.returncode == 0, r0.stderr[-2000:]
    assert _chain(auto, busid) == _chain(mine, busid)
    # Attribute by attribute, the file says what RCCL would have read from sysfs itself
    # (NCCL's link rule included: slower of device and port speed, narrower width).
    attrs = ("class", "vendor", "device", "subsystem_vendor", "subsystem_device", "link_speed", "link_width")
    by_bus = lambda root: {p.get("busid"): p for p in root.iter("pci")}  # noqa: E731
    for b in _chain(mine, busid)[1:]:
        got, want = by_bus(auto)[b], by_bus(mine)[b]
        assert {a: got.get(a) for a in attrs} == {a: want.get(a) for a in attrs}, b
    cpu_auto = [c for c in auto.iter("cpu") if c.get("numaid") == _chain(mine, busid)[0]][0]
    cpu_mine = [c for c in mine.iter("cpu") if c.get("numaid") == _chain(mine, busid)[0]][0]
    for a in ("affinity", "arch", "vendor", "familyid", "modelid"):
        assert cpu_auto.get(a) == cpu_mine.get(a), a
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "rccl_topo_loaded.json").write_text(json.dumps({
        "gpu_busid": busid, "chain_in_file": _chain(mine, busid), "chain_in_rccl_dump": _chain(dump, busid),
        "dump_version": dump.get("version"), "nets_in_dump": [n.get("name") for n in dump.iter("net")]}, indent=1))


@pytest.mark.gpu
def test_rccl_places_socket_nic_from_topology_file(native, tmp_path):
    """With NCCL_SOCKET_IFNAME on one of the file's NICs, RCCL's socket plugin uses it and the
    dump shows that net where the file put it (under the GPU's switch for a rail NIC)."""
    d = native.discover("/sys/")
    ipv4 = _ipv4_ifaces()
    usable = [p["nic"] for p in d["pairs"] if p["nic"] in ipv4]
    if not usable:
        pytest.skip(f"no scale-out NIC of this box has an IPv4 address in this network namespace "
                    f"(paired: {[p['nic'] for p in d['pairs']]}; with IPv4: {sorted(ipv4)})")
    nic = usable[0]
    xml = native.rccl_topo_xml("/sys/")
    topo = tmp_path / "rccl-topo.xml"
    topo.write_text(xml)
    r, dump = _rccl_dump(tmp_path, topo, {"NCCL_SOCKET_IFNAME": "=" + nic, "NCCL_IB_DISABLE": "1"}, tag="nic")
    assert r.returncode == 0, r.stderr[-3000:]
    assert _net_chain(dump, nic) == _net_chain(ET.fromstring(xml), nic)


@pytest.mark.gpu
def test_rccl_takes_nic_placement_from_the_topology_file(native, tmp_path, cuda_device):
    """The mechanism the agent's file relies on, shown on a box whose rail NICs RCCL cannot use:
    RCCL places a network device where the topology file puts it.  The file generated from this
    box's sysfs names the visible GPU's rail NIC; here that <net> is renamed to the interface
    RCCL's socket plugin really uses (a container veth without a PCI path), and RCCL's dump must
    show that interface under the rail NIC's PCI function, i.e. behind the GPU's PCIe switch."""
    from network_operator_amd.parallel.rail import device_bdf

    gpu = device_bdf(0)
    d = native.discover("/sys/")
    pair = next((p for p in d["pairs"] if p["gpu"].lower() == gpu.lower()), None)
    if pair is None:
        pytest.skip(f"visible GPU {gpu} has no GPU-affine NIC on this box")
    rdma = {n["ifname"]: n["rdma_dev"] for n in d["nics"]}
    rail_name = rdma.get(pair["nic"]) or pair["nic"]
    socket_if = next((i for i in sorted(_ipv4_ifaces()) if i != "lo"), None)
    if socket_if is None:
        pytest.skip("no IPv4 interface for RCCL's socket plugin")
    xml = native.rccl_topo_xml("/sys/").replace(f'<net name="{rail_name}"', f'<net name="{socket_if}"')
    mine = ET.fromstring(xml)
    want = _net_chain(mine, socket_if)
    nic_bdf = next(n["bdf"] for n in d["nics"] if n["ifname"] == pair["nic"])
    assert want and want[-1] == nic_bdf, (want, nic_bdf)
    topo = tmp_path / "rccl-topo.xml"
    topo.write_text(xml)
    r, dump = _rccl_dump(tmp_path, topo, {"NCCL_SOCKET_IFNAME": "=" + socket_if, "NCCL_IB_DISABLE": "1"},
                         tag="placed")
    assert r.returncode == 0, r.stderr[-3000:]
    got = _net_chain(dump, socket_if)
    assert got == want, (got, want, ET.tostring(dump)[:3000])
    # ... and that is the GPU's switch: GPU and NIC share the outermost switch below the CPU.
    assert _chain(dump, gpu.lower())[:2] == got[:2]
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "rccl_topo_nic_placed.json").write_text(json.dumps(
        {"gpu": gpu, "rail_nic": pair["nic"], "socket_if": socket_if, "net_chain_in_file": want,
         "net_chain_in_rccl_dump": got, "gpu_chain_in_rccl_dump": _chain(dump, gpu.lower())}, indent=1))


def _nccl_fold(components):
    """Independent re-statement of NCCL's ncclTopoGetXmlFromSys parent walk (src/graph/xml.cc):
    from a device's sysfs path, strip one component at a time; a non-BDF component is the root
    complex (-> CPU); every second BDF component is the next parent.  Returns the parents,
    outermost first."""
    path = list(components)
    parents = []
    while True:
        count = 0
        parent = None
        while len(path) > 1:
            path.pop()
            count += 1
            last = path[-1]
            is_bdf = len(last) == 12 and last[4] == ":" and last[7] == ":" and last[10] == "."
            if not is_bdf:
                return list(reversed(parents))  # CPU
            if count == 2:
                parent = last
                break
        if parent is None:
            return list(reversed(parents))
        parents.append(parent)


@settings(max_examples=60, deadline=None)
@given(depth=st.integers(min_value=1, max_value=9), seed=st.integers(min_value=0, max_value=2 ** 16))
def test_pci_folding_matches_nccl_walk(native, depth, seed):
    import random
    import tempfile

    rng = random.Random(seed)
    bus = rng.randrange(0, 0xe0)
    comps = [f"pci0000:{bus:02x}"] + [f"0000:{(bus + i) % 256:02x}:{rng.randrange(32):02x}.{rng.randrange(8)}"
                                      for i in range(depth)]
    with tempfile.TemporaryDirectory() as t:
        root = Path(t)
        d = root / "devices" / "/".join(comps)
        for k in range(1, len(comps) + 1):
            p = root / "devices" / "/".join(comps[:k])
            p.mkdir(parents=True, exist_ok=True)
            if k > 1:
                (p / "class").write_text("0x060400\n")
                (p / "numa_node").write_text("0\n")
        (d / "class").write_text("0x120000\n")
        (d / "vendor").write_text("0x1002\n")
        drv = root / "bus" / "pci" / "drivers" / "amdgpu"
        drv.mkdir(parents=True)
        (drv / comps[-1]).symlink_to(d)
        (d / "driver").symlink_to(drv)
        xml = ET.fromstring(native.rccl_topo_xml(str(root) + "/", cpu=fakesysfs.MI355X_HOST_CPU))
        chain = _chain(xml, comps[-1])
        assert chain is not None
        assert chain[1:-1] == _nccl_fold(comps), (comps, chain)


@pytest.mark.gpu
def test_bench_measures_with_the_agents_file_and_reads_rccl_dump(tmp_path):
    """bench.py's headline runs RCCL with the agent's NCCL_TOPO_FILE / rccl.env (discover
    --dry-run on this box) and reads RCCL's dump back: the GPU where the file puts it, and the
    xGMI link check (n - 1 = 0 here).  The RCCL-defaults A/B dumps too, for comparison."""
    r = subprocess.run([sys.executable, str(ROOT / "bench.py"), "--gpus", "1", "--steps", "3", "--warmup", "1",
                        "--sweep", "", "--node-ready", "off", "--native-rccl", "0", "--gpu-side", "0",
                        "--deadline-s", "100"], capture_output=True, text=True, timeout=115, cwd=tmp_path)
    assert r.returncode == 0, r.stderr[-3000:]
    j = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    a = j["agent_artifacts"]
    assert a["applied"] is True and a["ranks_applied"] == 1 and a["topo_file_bytes"] > 1000, a
    d = a["rccl_dump"]
    assert "error" not in d, d
    assert d["gpus"] == 1 and d["gpu_ancestry_equal"] is True, d
    assert a["xgmi_links_check"]["status"] == "ok"
    base = j["rccl_defaults"]["rccl_dump"]
    assert base["gpus"] == 1 and base["gpu_busids"] == d["gpu_busids"]
    (ROOT / "gpurun_out").mkdir(exist_ok=True)
    (ROOT / "gpurun_out" / "bench_artifacts_n1.json").write_text(json.dumps(
        {"agent_artifacts": a, "rccl_defaults": j["rccl_defaults"], "ms_per_step": j["ms_per_step"]}, indent=1))


def test_validation_names_a_rail_whose_pcie_link_trained_low(tmp_path):
    """validate.py's rail_pcie_links check: every rail at full PCIe passes; a NIC trained at Gen4,
    or a GPU at x8, fails and is named; a GPU only slower (idle downshift) does not."""
    from network_operator_amd import validate
    from network_operator_amd.models.topology import NodeTopology

    fx = fakesysfs.build_mi355x_node(tmp_path, n_gpus=4)
    topo = NodeTopology.discover(str(tmp_path))
    c = validate.rail_pcie_check(topo, str(tmp_path))
    assert c["ok"] and len(c["links"]) == 4 and c["degraded"] == []
    gpus = sorted(g["bdf"] for g in fx["gpus"])[:4]
    fakesysfs.set_pcie_link(tmp_path, gpus[0], 16.0, 16)  # idle GPU: speed only
    assert validate.rail_pcie_check(topo, str(tmp_path))["ok"]
    fakesysfs.set_pcie_link(tmp_path, gpus[1], 32.0, 8)
    nic = topo.nic_for_gpu(gpus[2])
    fakesysfs.set_pcie_link(tmp_path, fakesysfs.nic_pci_dir(tmp_path, nic).name, 16.0, 16)
    c = validate.rail_pcie_check(topo, str(tmp_path))
    assert not c["ok"] and sorted(c["degraded"]) == sorted([topo.nic_for_gpu(gpus[1]), nic]), c
    assert c["links"][nic]["nic"] == "16.0 GT/s x16 of 32.0 GT/s x16"


def test_node_report_checks_the_agents_rccl_topology_file(tmp_path):
    """The node report checks the agent's rccl-topo.xml (``--artifact-dir``) against the node: the
    golden file matches the fixture node; a file that puts a rail NIC under another GPU's switch
    is named as a problem (exit 1)."""
    root, art = tmp_path / "sys", tmp_path / "scale-out"
    fakesysfs.build_mi355x_node(root)
    (root / "module" / "ib_uverbs").mkdir(parents=True)
    art.mkdir()

    def report():
        r = subprocess.run([sys.executable, "-m", "network_operator_amd.agent.report", "--json", f"--artifact-dir={art}"],
                           capture_output=True, text=True, timeout=60, env=dict(os.environ, SYSFS_ROOT=str(root)))
        return r.returncode, json.loads(r.stdout)

    rc, rep = report()
    assert rep["rccl_topology_file"] is None  # the agent has not run here
    good = GOLDEN.read_text()
    (art / "rccl-topo.xml").write_text(good)
    rc, rep = report()
    assert rep["rccl_topology_file"]["ok"] and not [p for p in rep["problems"] if "rccl-topo" in p], rep
    (art / "rccl-topo.xml").write_text(good.replace('<net name="mlx5_1" port="1"/>', '<net name="tmp" port="1"/>').replace(
        '<net name="mlx5_3" port="1"/>', '<net name="mlx5_1" port="1"/>'))
    rc, rep = report()
    assert rc == 1 and len([p for p in rep["problems"] if "rccl-topo.xml: places" in p]) == 2, rep["problems"]
