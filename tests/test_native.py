"""Native agent building blocks: C++ unit suite, pybind11 bindings, property-based fuzzing,
and discovery on a fake sysfs copy of a real 8x MI355X node."""

import errno
import ipaddress
import json
import os
import subprocess

import pytest
from hypothesis import given, settings
from hypothesis import strategies as st

from network_operator_amd.testing import fakesysfs
from network_operator_amd.utils import native_bin


def test_cpp_unit_suite():
    r = subprocess.run([str(native_bin("netop-unit-tests"))], capture_output=True, text=True, timeout=540)  # (pytest-timeout: 600)
    assert r.returncode == 0, r.stdout[-4000:] + r.stderr[-2000:]
    assert "FAIL" not in r.stdout


def test_discover_help_lists_reference_flags():
    out = subprocess.run([str(native_bin("discover")), "--help"], capture_output=True, text=True).stdout
    for flag in ("--mode", "--configure", "--disable-networkmanager", "--interfaces", "--wait", "--keep-running",
                 "--systemd-networkd", "--mtu", "--rccl-net", "--v"):
        assert flag in out, flag


def test_every_agent_flag_is_documented():
    """Each flag `discover --help` lists is explained in the docs (USER_GUIDE / ARCHITECTURE / README)."""
    import re
    from pathlib import Path
    out = subprocess.run([str(native_bin("discover")), "--help"], capture_output=True, text=True).stdout
    flags = re.findall(r"^\s+(--[a-z0-9_-]+)", out, re.M)
    assert len(flags) > 60
    root = Path(__file__).resolve().parent.parent
    docs = "".join(p.read_text() for p in [root / "README.md", *sorted((root / "docs").glob("*.md"))])
    assert [f for f in flags if not re.search(re.escape(f) + r"(?![a-z0-9-])", docs)] == []
    # and the operator manager's
    import sys
    out = subprocess.run([sys.executable, "-m", "network_operator_amd.operator.manager", "--help"],
                         capture_output=True, text=True).stdout
    flags = re.findall(r"^\s+(--[a-z0-9_-]+)", out, re.M)
    assert len(flags) > 15
    assert [f for f in flags if not re.search(re.escape(f) + r"(?![a-z0-9-])", docs)] == []


def test_discover_rejects_bad_flags():
    r = subprocess.run([str(native_bin("discover")), "--wait=90"], capture_output=True, text=True)
    assert r.returncode == 2 and "invalid duration" in r.stderr
    r = subprocess.run([str(native_bin("discover")), "--mode=L4", "--nic-discovery=none", "--interfaces=lo"],
                       capture_output=True, text=True)
    assert r.returncode == 1 and "Invalid mode 'L4'" in r.stderr


# --- LLDP codec ------------------------------------------------------------------------------
MAC = st.lists(st.integers(0, 255), min_size=6, max_size=6).map(lambda b: ":".join(f"{x:02x}" for x in b))
TEXT = st.text(alphabet=st.characters(min_codepoint=32, max_codepoint=126), max_size=200)


@settings(max_examples=300, deadline=None)
@given(mac=MAC, sysname=TEXT, port=TEXT.filter(bool), desc=TEXT, ttl=st.integers(0, 65535),
       vlan=st.one_of(st.none(), st.integers(1, 4094)))
def test_lldp_roundtrip_property(native, mac, sysname, port, desc, ttl, vlan):
    frame = native.lldp_switch_frame(mac, sysname, port, desc, ttl, vlan)
    d = native.lldp_decode(frame)
    assert d["port_description"] == desc
    assert d["system_name"] == sysname
    assert d["port_id"] == port.encode()[:255]
    assert d["ttl"] == ttl
    assert d["peer_mac"] == mac
    assert d["vlan"] == vlan


@settings(max_examples=500, deadline=None)
@given(data=st.binary(max_size=300))
def test_lldp_decode_never_crashes_on_garbage(native, data):
    frame = bytes.fromhex("0180c200000e020000aabbcc88cc") + data
    try:
        native.lldp_decode(frame)
    except ValueError:
        pass


def test_lldp_peer_mac_port_overrides_chassis(native):
    f = native.lldp_encode("02:00:00:00:00:01", 4, bytes.fromhex("020000000001"), 3, bytes.fromhex("020000000002"))
    assert native.lldp_decode(f)["peer_mac"] == "02:00:00:00:00:02"
    f = native.lldp_encode("02:00:00:00:00:01", 4, bytes.fromhex("020000000001"), 5, b"Ethernet1")
    assert native.lldp_decode(f)["peer_mac"] == "02:00:00:00:00:01"


# --- Port Description -> /30 -------------------------------------------------------------------
@settings(max_examples=400, deadline=None)
@given(a=st.integers(0, 2**32 - 1), tag=st.sampled_from(["no-alert", "x", "uplink-7"]))
def test_port_description_matches_ipaddress_model(native, a, tag):
    ip = ipaddress.IPv4Address(a)
    desc = f"{tag} {ip}/30"
    net = ipaddress.IPv4Network(f"{ip}/30", strict=False)
    if ip in (net.network_address, net.broadcast_address):
        with pytest.raises(ValueError):
            native.parse_port_description(desc, "compat")
        return
    r = native.parse_port_description(desc, "compat")
    local = ipaddress.IPv4Address(int(ip) ^ 3)
    assert r["peer"] == str(ip) and r["local"] == str(local)
    assert r["p2p_network"] == str(net)
    assert r["routed_network"] == str(ipaddress.IPv4Network(f"{local}/16", strict=False))


@pytest.mark.parametrize("desc,policy,local", [
    ("no-alert 10.200.10.2/30", "compat", "10.200.10.1"),
    ("to leaf1 eth1/1 10.1.1.2/30", "compat-then-last", "10.1.1.1"),
    ("uplink 7 10.5.5.6/30 via tor", "any", "10.5.5.5"),
])
def test_port_description_policies(native, desc, policy, local):
    assert native.parse_port_description(desc, policy)["local"] == local


@pytest.mark.parametrize("desc", ["no-alert", "a 10.0.0.2/24", "a 10.0.0.0/30", "a  10.0.0.2/30", "a 1.2.3/30"])
def test_port_description_compat_rejects(native, desc):
    with pytest.raises(ValueError):
        native.parse_port_description(desc, "compat")


# --- Topology on the real MI355X node layout ------------------------------------------------
def test_real_mi355x_topology_discovery(native, tmp_path):
    fx = fakesysfs.build_mi355x_node(tmp_path)
    d = native.discover(str(tmp_path))
    assert [g["bdf"] for g in d["gpus"]] == sorted(g["bdf"] for g in fx["gpus"])
    assert all(g["device"] == 0x75A3 for g in d["gpus"])
    assert len(d["pairs"]) == 8
    # Every GPU pairs with the mlx5 NIC behind its own PCIe switch; management NICs excluded.
    assert "ens9np0" not in d["ifnames"] and "ens49np1" not in d["ifnames"]
    for p in d["pairs"]:
        assert p["path"] == "PXB" and p["common_depth"] == 3
        g = [x for x in fx["gpus"] if x["bdf"] == p["gpu"]][0]
        n = [x for x in fx["nics"] if x["ifname"] == p["nic"]][0]
        assert g["path"].split("/")[:3] == n["pcipath"].split("/")[:3]
    x = native.read_xgmi(str(tmp_path))
    assert x["pairs_expected"] == 28 and x["pairs_connected"] == 28 and x["full_mesh"]
    assert x["per_gpu_bw_mbs"] == 7 * 76000


def test_rdma_discovery_on_the_mi355x_node_leaves_the_eight_rails_to_amd_so(native, tmp_path):
    """host-nic discovery (rdma, default drivers) on the captured node, where all ten NICs are
    mlx5 with an RDMA device: the eight GPU rails are left out (each named with its GPU), so an
    amd-so and a host-nic policy on one node never share a NIC.  The reference cannot reach another
    agent's NIC at all: it only enumerates netdevs under the accelerator's own PCI functions
    (reference cmd/discover/network.go:34,88-119)."""
    fx = fakesysfs.build_mi355x_node(tmp_path)
    rails = fakesysfs.real_nic_order()
    d = native.discover(str(tmp_path), mode="rdma")
    assert sorted(d["ifnames"]) == ["ens49np1", "ens9np0"]
    assert sorted(d["excluded"]) == sorted(rails)
    pairs = {p["nic"]: p["gpu"] for p in native.discover(str(tmp_path))["pairs"]}
    for nic, why in d["excluded"].items():
        assert why.startswith(f"scale-out rail of GPU {pairs[nic]} (amdgpu, path PXB)"), why
    # Disjoint from what the amd-so agent takes, and together they cover every RDMA NIC.
    assert not set(d["ifnames"]) & set(pairs)
    assert set(d["ifnames"]) | set(pairs) == {n["ifname"] for n in fx["nics"]}
    # --rdma-include-gpu-rails (explicit opt-in) takes them all.
    assert len(native.discover(str(tmp_path), mode="rdma", include_gpu_rails=True)["ifnames"]) == 10


def test_topo_tool_json(tmp_path):
    """``netop-topo`` (in the agent image, which has no Python): the node's topology, and each
    GPU's and NIC's PCIe link and each GPU's xGMI links as trained."""
    fx = fakesysfs.build_mi355x_node(tmp_path, drop_xgmi_pairs=[(1, 2)])
    gpu1 = sorted(g["bdf"] for g in fx["gpus"])[1]
    fakesysfs.set_xgmi_link(tmp_path, gpu1, 2, False)
    fakesysfs.set_pcie_link(tmp_path, gpu1, 32.0, 8)
    out = subprocess.run([str(native_bin("netop-topo")), f"--sysfs-root={tmp_path}"], capture_output=True, text=True,
                         check=True).stdout
    j = json.loads(out)
    assert len(j["gpus"]) == 8 and len(j["pairs"]) == 8
    links = {g["bdf"]: g["xgmi_links"] for g in j["gpus"]}
    assert links[gpu1]["status"] == "XUDUUUUU" and links[gpu1]["down"] == 1 and links[gpu1]["up"] == 6, links[gpu1]
    assert all(v["known"] and v["revision"] == "1.8" and v["width"] == 16 for v in links.values())
    assert sum(v["down"] for v in links.values()) == 1
    pcie = {g["bdf"]: g["pcie"] for g in j["gpus"]}
    assert pcie[gpu1] == {"known": True, "degraded": True, "str": "32.0 GT/s x8 of 32.0 GT/s x16"}
    assert all(n["pcie"]["known"] and not n["pcie"]["degraded"] for n in j["nics"] if n["ifname"] in
               {p["nic"] for p in j["pairs"]})
    assert j["xgmi"]["pairs_connected"] == 27 and not j["xgmi"]["full_mesh"]
    # What a host-nic policy would take from sysfs: the two host NICs; the rails are amd-so's.
    assert sorted(j["host_nics"]["ifnames"]) == ["ens49np1", "ens9np0"]
    assert sorted(j["host_nics"]["left_alone"]) == sorted(p["nic"] for p in j["pairs"])


def test_accel_mode_reference_layout(native, tmp_path):
    # Reference fixture layout: netdevs directly under the accelerator function
    # (reference cmd/discover/network_test.go:94-116).
    dev = tmp_path / "devices" / "pci0000:00" / "0000:00:02.0" / "0000:33:00.0"
    for n in ("eth_a", "eth_b"):
        (dev / "net" / n).mkdir(parents=True)
    drv = tmp_path / "bus" / "pci" / "drivers" / "habanalabs"
    drv.mkdir(parents=True)
    (drv / "0000:33:00.0").symlink_to(dev)
    d = native.discover(str(tmp_path), mode="accel", accel_driver="habanalabs")
    assert sorted(d["ifnames"]) == ["eth_a", "eth_b"]


def test_gid_lookup(native, tmp_path):
    fakesysfs.add_rocev2_gids(tmp_path, "mlx5_0", ["10.9.8.1", "10.9.8.5"])
    assert native.find_rocev2_gid_index(str(tmp_path), "mlx5_0", 1, "10.9.8.1") == 3
    assert native.find_rocev2_gid_index(str(tmp_path), "mlx5_0", 1, "10.9.8.5") == 5
    assert native.find_rocev2_gid_index(str(tmp_path), "mlx5_0", 1, "10.9.8.9") is None


def test_topology_model(tmp_path):
    from network_operator_amd.models import NodeTopology

    fakesysfs.build_mi355x_node(tmp_path)
    t = NodeTopology.discover(str(tmp_path))
    assert len(t.gpus) == 8 and len(t.pairs) == 8 and t.xgmi.full_mesh
    assert t.nic_for_gpu("0000:0a:00.0") == "enp5s0np0"
    assert t.xgmi.busbw_ceiling_GBps() == 532.0


def test_rccl_bench_cli():
    exe = str(native_bin("netop-rccl-bench"))
    r = subprocess.run([exe, "--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "--id-file" in r.stderr
    r = subprocess.run([exe, "-o", "gather"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 2


def test_rccl_bench_command_and_parse():
    from network_operator_amd.parallel import rccl_bench

    cmd = rccl_bench.command(op="alltoall", gpus=8, max_bytes=1 << 30, graph=True)
    assert cmd[1:5] == ["-o", "alltoall", "-g", "8"] and "--graph" in cmd
    rows = rccl_bench.parse('# x\n{"op":"all_reduce","bytes":8,"count":8,"dtype":"bf16","ranks":2,"time_us":9.5,'
                            '"algbw_GBps":0.001,"busbw_GBps":0.001,"wrong":0,"checked":true,"inplace":false,'
                            '"graph":false}\n')
    assert rows[0].ranks == 2 and rows[0].time_us == 9.5


def test_xgmi_allreduce_cli():
    from network_operator_amd.parallel import xgmi_allreduce as X

    r = subprocess.run(X.command(mode="pull")[:1] + ["--help"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0 and "--mode" in r.stderr
    assert "--ranks" in X.command(ranks=8)
    with pytest.raises(ValueError):
        X.command(mode="ring")


def test_gdr_detection_binding(native, tmp_path):
    assert native.detect_gdr(str(tmp_path), "6.8.0")["mode"] == "none"
    (tmp_path / "module" / "ib_uverbs").mkdir(parents=True)
    d = native.detect_gdr(str(tmp_path), "6.8.0")
    assert d["mode"] == "dmabuf" and d["kernel"] == "6.8.0"


def test_dcb_netlink_requests_reach_the_kernel(native):
    """The DCB netlink request the agent sends to read a NIC's DCBX mode is well-formed: the
    kernel parses it and answers for the named device.  lo has no DCB interface (EOPNOTSUPP) and
    an unknown name has no device (ENODEV): both read as "no DCB interface", never as an error.
    A malformed request would fail with EINVAL and raise.  Setting needs CAP_NET_ADMIN and a DCB
    driver: on lo it is refused either way."""
    r = native.Rtnl()
    assert r.dcbx_mode("lo") is None
    assert r.dcbx_mode("netop-nosuch0") is None
    with pytest.raises(OSError) as e:
        r.set_dcbx_mode("lo", 0x09)
    assert any(os.strerror(c) in str(e.value) for c in (errno.EOPNOTSUPP, errno.EPERM)), e.value


def test_ipv6_addresses_are_read_from_the_kernel(native):
    """The agent treats a global / ULA IPv6 address on a NIC as the node's (ownership check), so
    the rtnetlink address dump must carry IPv6 addresses with their scope: lo's ::1 is host scope
    (254), which the agent ignores like link-local (253)."""
    if not os.path.exists("/proc/net/if_inet6"):
        pytest.skip("kernel without IPv6")
    r = native.Rtnl()
    lo = r.link_by_name("lo")["index"]
    got = r.addr6_list(lo)
    if not got:
        pytest.skip("no IPv6 address on lo in this namespace")
    assert {"address": "::1", "prefixlen": 128, "scope": 254, "ifindex": lo} in got
    assert all(a["address"] for a in r.addr6_list(0))


def test_pattern_swar_sum_matches_the_per_rank_reference():
    """The device's rank sum (netop_hip.hip group_sum: even / odd 3-bit fields of every rank
    added as 6-bit slots without a shift, flushed every 9 ranks, each rank's word the previous
    one plus h d) equals the sum of the per-rank reference (collectives.pattern_reference) for
    1..64 ranks and rank ranges -- emulated here with Python integers, line for line."""
    import random

    import torch

    from network_operator_amd.parallel.collectives import pattern_reference

    M32 = 0xFFFFFFFF
    EVEN = (7 << 5) | (7 << 11) | (7 << 17) | (7 << 23)
    ODD = EVEN << 3

    def group_hash(g):
        x = ((g & M32) * 0x9E3779B1 & M32) ^ (((g >> 32) & M32) * 0x85EBCA77 & M32)
        x ^= x >> 15
        x = x * 0x2C1B3C6D & M32
        return x ^ (x >> 12)

    def base_mult(seed):
        k = ((seed + 0x632BE5AB) & M32) * 0xC2B2AE3D & M32
        return (k ^ (k >> 16)) | 1

    def step_mult(seed):
        k = ((seed ^ 0x27D4EB2F) & M32) * 0x165667B1 & M32
        return (((k ^ (k >> 15)) << 1) | 2) & M32

    def group_sum(g, seed, lo, n):
        h, s = group_hash(g), [-4 * n] * 8
        d = step_mult(seed)
        dx = h * d & M32
        x = h * ((base_mult(seed) + lo * d) & M32) & M32
        for r0 in range(0, n, 9):
            even = odd = 0
            for _ in range(r0, min(r0 + 9, n)):
                even = (even + (x & EVEN)) & M32
                odd = (odd + (x & ODD)) & M32
                x = (x + dx) & M32
            for k in range(4):
                s[2 * k] += (even >> (5 + 6 * k)) & 63
                s[2 * k + 1] += (odd >> (8 + 6 * k)) & 63
        return s

    rng = random.Random(7)
    groups = 64
    for lo, n in [(0, 1), (3, 1), (0, 8), (0, 9), (0, 10), (5, 18), (0, 64), (17, 27)]:
        seed = rng.randrange(1 << 32)
        ref = sum(pattern_reference(groups * 8, seed, r) for r in range(lo, lo + n))
        dev = torch.tensor([v for g in range(groups) for v in group_sum(g, seed, lo, n)], dtype=torch.float32)
        assert torch.equal(dev, ref), (lo, n)
        assert ref.abs().max() <= 256  # exact in bf16


def test_dry_run_reports_an_xgmi_link_down_without_failing(native, tmp_path):
    """A dry run says what a real start would fail on and goes on: with a GPU's xGMI link down in
    gpu_metrics, it exits 0, logs "a real start would fail", and status.json names the link;
    every other GPU's links are read and counted (the fake node's blobs are the live MI355X's)."""
    fx = fakesysfs.build_mi355x_node(tmp_path / "sys", n_gpus=8)
    bdfs = [g["bdf"] for g in fx["gpus"]]
    fakesysfs.set_xgmi_link(tmp_path / "sys", bdfs[2], 6, False)
    health = native.read_xgmi_health(str(tmp_path / "sys"), bdfs)
    assert [h["status"].count(0) for h in health] == [0, 0, 1, 0, 0, 0, 0, 0]
    status = tmp_path / "status.json"
    r = subprocess.run([str(native_bin("discover")), "--dry-run", "--xgmi-expect=0", f"--status-file={status}"],
                       capture_output=True, text=True, timeout=60, env=dict(os.environ, SYSFS_ROOT=str(tmp_path / "sys")))
    assert r.returncode == 0, r.stderr[-2000:]
    assert f"dry run: a real start would fail: xGMI: GPU {bdfs[2]}: link 6 down" in r.stderr
    st = json.loads(status.read_text())
    assert st["xgmi_links"] == "55 up, 1 down on 8 GPUs, x16 at 38 Gb/s (gpu_metrics)"
    assert st["xgmi_error"] == f"GPU {bdfs[2]}: link 6 down"


def test_a_rail_without_an_rdma_device_is_named(native, tmp_path):
    """A scale-out NIC whose RDMA driver is not loaded (no /sys/class/infiniband device) leaves RCCL
    only TCP sockets on that rail: the agent names it (log, status.json ``nics_without_rdma``);
    with --require-gdr it is a failure.  (Boxes of this pool with Pollara NICs look like this.)"""
    import shutil

    fx = fakesysfs.build_mi355x_node(tmp_path / "sys", n_gpus=2)
    first_rail = native.discover(str(tmp_path / "sys"))["pairs"][0]["nic"]
    victim = next(n for n in fx["nics"] if n["ifname"] == first_rail)
    shutil.rmtree(tmp_path / "sys" / "devices" / victim["pcipath"] / "infiniband")
    for dev in list((tmp_path / "sys" / "class" / "infiniband").iterdir()):
        if not dev.exists():
            dev.unlink()
    status = tmp_path / "status.json"
    r = subprocess.run([str(native_bin("discover")), "--dry-run", "--xgmi-expect=0", f"--status-file={status}"],
                       capture_output=True, text=True, timeout=60, env=dict(os.environ, SYSFS_ROOT=str(tmp_path / "sys")))
    assert r.returncode == 0, r.stderr[-2000:]
    st = json.loads(status.read_text())
    assert st.get("nics_without_rdma") == victim["ifname"], (st, victim)
    assert "without an RDMA device: " + victim["ifname"] in r.stderr


def test_node_report_names_what_would_keep_the_label_off(tmp_path):
    """``python -m network_operator_amd.agent.report``: the agent's own readings of a node, read
    only.  A healthy fake node (GPUDirect RDMA via dma-buf) reports no problem and exits 0; a rail
    trained at x8, an xGMI link down and a missing RDMA device are each named, exit 1; so is a link
    below ``--min-link-speed-gbps`` (a link that is down is not: the agent brings it up)."""
    import shutil
    import sys

    root = tmp_path / "sys"
    fx = fakesysfs.build_mi355x_node(root, n_gpus=4)
    (root / "module" / "ib_uverbs").mkdir(parents=True)

    def report(*args):
        r = subprocess.run([sys.executable, "-m", "network_operator_amd.agent.report", "--json", *args], capture_output=True,
                           text=True, timeout=60, env=dict(os.environ, SYSFS_ROOT=str(root)))
        return r.returncode, json.loads(r.stdout)

    rc, rep = report()
    assert rc == 0 and rep["problems"] == [] and len(rep["rails"]) == 4, rep
    assert rep["gpudirect_rdma"] == "dmabuf" and rep["xgmi"]["pairs"] == "6/6"
    rail0 = rep["rails"][0]
    assert rail0["link"] == {"operstate": "unknown", "speed_gbps": None, "mtu": None}
    net = root / "class" / "net"
    for i, x in enumerate(rep["rails"]):  # as a host shows them: rail 1 negotiated 200G, rail 2 has no carrier
        (net / x["nic"] / "operstate").write_text("down\n" if i == 2 else "up\n")
        (net / x["nic"] / "speed").write_text("-1\n" if i == 2 else ("200000\n" if i == 1 else "400000\n"))
        (net / x["nic"] / "mtu").write_text("9000\n")
    rc, rep = report()
    assert rc == 0 and rep["rails"][0]["link"] == {"operstate": "up", "speed_gbps": 400, "mtu": 9000}
    assert rep["rails"][2]["link"]["speed_gbps"] is None
    rc, rep = report("--min-link-speed-gbps", "400")
    assert rc == 1 and rep["problems"] == [f"{rep['rails'][1]['nic']}: link negotiated 200 Gb/s, below the required 400"]
    (net / rep["rails"][1]["nic"] / "speed").write_text("400000\n")
    fakesysfs.set_pcie_link(root, fakesysfs.nic_pci_dir(root, rail0["nic"]).name, 16.0, 8)
    fakesysfs.set_xgmi_link(root, fx["gpus"][1]["bdf"], 2, False)
    victim = next(n for n in fx["nics"] if n["ifname"] == rep["rails"][3]["nic"])
    shutil.rmtree(root / "devices" / victim["pcipath"] / "infiniband")
    rc, rep = report()
    assert rc == 1
    assert rep["problems"] == [f"{victim['ifname']}: no RDMA device (load its RDMA driver)",
                               f"{rail0['nic']}: PCIe link 16.0 GT/s x8 of 32.0 GT/s x16",
                               f"GPU {fx['gpus'][1]['bdf']}: xGMI link(s) 2 down"], rep["problems"]


def test_node_report_checks_rccl_env_against_the_rails_devices_and_gid_slots(tmp_path):
    """The report reads the agent's rccl.env against the node as it is now: an HCA renumbered by a
    driver reload (named but gone, the new one not named) and a pinned NCCL_IB_GID_INDEX whose slot
    holds no RoCE v2 IPv4 GID on a device are each a problem; a current file is not."""
    import sys

    root = tmp_path / "sys"
    fakesysfs.build_mi355x_node(root, n_gpus=2)
    (root / "module" / "ib_uverbs").mkdir(parents=True)
    art = tmp_path / "art"
    art.mkdir()

    def report():
        r = subprocess.run([sys.executable, "-m", "network_operator_amd.agent.report", "--json", "--artifact-dir", str(art)],
                           capture_output=True, text=True, timeout=60, env=dict(os.environ, SYSFS_ROOT=str(root)))
        return r.returncode, json.loads(r.stdout)

    rc, rep = report()
    devs = [x["rdma_dev"] for x in rep["rails"]]
    assert rc == 0 and all(devs) and rep["rccl_env"] is None
    for i, dev in enumerate(devs):
        fakesysfs.add_rocev2_gids(root, dev, [f"10.20{i}.0.1"])  # IPv4 RoCE v2 GID at slot 3
    (art / "rccl.env").write_text(f"NCCL_IB_HCA=={devs[0]}:1,{devs[1]}:1\nNCCL_IB_GID_INDEX=3\n")
    rc, rep = report()
    assert rc == 0 and rep["problems"] == [] and rep["rccl_env"]["hcas"] == sorted(devs), rep
    (art / "rccl.env").write_text(f"NCCL_IB_HCA=={devs[0]}:1,mlx5_9:1\nNCCL_IB_GID_INDEX=2\n")  # slot 2: RoCE v1
    rc, rep = report()
    env = str(art / "rccl.env")
    assert rc == 1
    assert f"{env}: names RDMA device mlx5_9, which no rail has now (a driver reload renumbered it?)" in rep["problems"]
    assert f"{env}: does not name {rep['rails'][1]['nic']}'s RDMA device {devs[1]}" in rep["problems"]
    assert any(p.startswith(f"{env}: NCCL_IB_GID_INDEX=2, but slot 2 of {devs[0]} port 1 holds no RoCE v2 GID")
               for p in rep["problems"]), rep["problems"]
    (art / "rccl.env").write_text(f"NCCL_IB_HCA=={devs[0]}:1,{devs[1]}:1\nNCCL_IB_GID_INDEX=1\n")  # L2: link-local v2
    rc, rep = report()
    assert rc == 0 and rep["problems"] == [], rep["problems"]
    (art / "rccl.env").write_text(f"NCCL_IB_HCA=={devs[0]}:1,{devs[1]}:1\nNCCL_IB_GID_INDEX=7\n")  # an empty slot
    rc, rep = report()
    assert rc == 1 and len(rep["rccl_env"]["bad_gid_slots"]) == 2


def test_node_report_names_a_torn_topology_file(tmp_path):
    import sys

    root = tmp_path / "sys"
    fakesysfs.build_mi355x_node(root, n_gpus=2)
    art = tmp_path / "art"
    art.mkdir()
    (art / "rccl-topo.xml").write_bytes(b'<system version="1"><cpu numaid="0"><pci busid="0000:0')
    r = subprocess.run([sys.executable, "-m", "network_operator_amd.agent.report", "--json", "--artifact-dir", str(art)],
                       capture_output=True, text=True, timeout=60, env=dict(os.environ, SYSFS_ROOT=str(root)))
    rep = json.loads(r.stdout)
    assert r.returncode == 1 and rep["rccl_topology_file"]["ok"] is False
    assert any("not a topology file RCCL can read" in p for p in rep["problems"]), rep["problems"]


@settings(max_examples=150, deadline=None)
@given(data=st.one_of(st.binary(max_size=300),
                      st.lists(st.sampled_from(["NCCL_IB_HCA==mlx5_0:1,mlx5_9", "NCCL_IB_HCA=^", "NCCL_IB_HCA=a:b:c,,",
                                                "NCCL_IB_GID_INDEX=3", "NCCL_IB_GID_INDEX=99999999999", "NCCL_IB_GID_INDEX=-1",
                                                "NCCL_IB_HCA=../../..:1", "NCCL_IB_HCA=x\x00y:1", "# c", "=", "\xff\xfe"]),
                               max_size=6).map(lambda ls: "\n".join(ls).encode("utf-8", "surrogatepass"))))
def test_node_report_rccl_env_check_never_crashes_on_a_garbled_file(tmp_path_factory, data):
    """Whatever bytes sit in rccl.env (a torn write, another tool's file), the report's check returns
    what it found and names problems; it never raises."""
    from network_operator_amd.agent.report import _check_rccl_env

    d = tmp_path_factory.mktemp("env")
    (d / "rccl.env").write_bytes(data)
    problems = []
    out = _check_rccl_env(str(d / "sys"), str(d / "rccl.env"),
                          [{"nic": "ens0", "rdma_dev": "mlx5_0"}, {"nic": "ens1", "rdma_dev": ""}], problems)
    assert isinstance(out["hcas"], list) and all(isinstance(p, str) for p in problems)


def test_a_gpu_metrics_read_that_never_returns_neither_hangs_the_start_nor_hides_the_reason(native, tmp_path):
    """every start-path sysfs join has a deadline.  GPU 2's gpu_metrics is a FIFO
    nobody writes (a wedged SMU: the read never returns).  The dry run ends after
    --sysfs-read-timeout, names the GPU in status.json and its log, and the other GPUs' links are
    still read (concurrently)."""
    import time

    fakesysfs.build_mi355x_node(tmp_path / "sys", n_gpus=8)
    bdfs = sorted(g["bdf"] for g in native.discover(str(tmp_path / "sys"))["gpus"])
    gm = tmp_path / "sys" / "bus" / "pci" / "devices" / bdfs[2] / "gpu_metrics"
    gm.unlink()
    os.mkfifo(gm)
    status = tmp_path / "status.json"
    t0 = time.monotonic()
    r = subprocess.run([str(native_bin("discover")), "--dry-run", "--xgmi-expect=0", "--sysfs-read-timeout=1s",
                        f"--status-file={status}"], capture_output=True, text=True, timeout=30,
                       env=dict(os.environ, SYSFS_ROOT=str(tmp_path / "sys")))
    took = time.monotonic() - t0
    assert r.returncode == 0, r.stderr[-2000:]
    assert took < 5, took
    st = json.loads(status.read_text())
    assert st["xgmi_error"] == f"gpu_metrics of {bdfs[2]} did not answer in 1s", st
    assert st["xgmi_links"] == "49 up, 0 down on 7 GPUs, x16 at 38 Gb/s (gpu_metrics)", st
    assert f"a real start would fail: xGMI: gpu_metrics of {bdfs[2]} did not answer in 1s" in r.stderr


def test_a_pollara_node_without_ionic_rdma_would_wait_for_rdma_devices(native, tmp_path):
    """VERDICT r5 #1, the box's case (profiles/r5_agent_dry_run_box_ionic.json): every rail is an
    ionic NIC without an RDMA device.  With --require-rdma (what the operator passes by default)
    the dry run says a real start would wait for RDMA devices on all 8 rails."""
    fx = fakesysfs.build_mi355x_node(tmp_path / "sys", n_gpus=8, rail_driver="ionic")
    rails = [p["nic"] for p in native.discover(str(tmp_path / "sys"))["pairs"]]
    for nif in rails:
        fakesysfs.remove_rdma(tmp_path / "sys", nif)
    status = tmp_path / "status.json"
    r = subprocess.run([str(native_bin("discover")), "--dry-run", "--require-rdma", "--xgmi-expect=0",
                        f"--status-file={status}"], capture_output=True, text=True, timeout=30,
                       env=dict(os.environ, SYSFS_ROOT=str(tmp_path / "sys")))
    assert r.returncode == 0, r.stderr[-2000:]
    assert "dry run: a real start would wait for RDMA devices on 8 rails" in r.stderr, r.stderr[-2000:]
    assert sorted(json.loads(status.read_text())["nics_without_rdma"].split(",")) == sorted(rails)
    assert fx["nics"]


def test_an_unknown_gpu_metrics_layout_is_said_once_and_in_the_status(native, tmp_path):
    """gpu_metrics layouts other than 1.8 (other firmware) are not decoded.  The agent
    says so at warning level and in status.json's xgmi_links, not only at -v=1; the KFD mesh check
    still runs and passes."""
    fakesysfs.build_mi355x_node(tmp_path / "sys", n_gpus=2)
    for g in native.discover(str(tmp_path / "sys"))["gpus"]:
        f = tmp_path / "sys" / "bus" / "pci" / "devices" / g["bdf"] / "gpu_metrics"
        b = bytearray(f.read_bytes())
        b[3] = 9  # content revision 1.9
        f.write_bytes(bytes(b))
    status = tmp_path / "status.json"
    r = subprocess.run([str(native_bin("discover")), "--dry-run", "--xgmi-expect=0", f"--status-file={status}"],
                       capture_output=True, text=True, timeout=60, env=dict(os.environ, SYSFS_ROOT=str(tmp_path / "sys")))
    assert r.returncode == 0, r.stderr[-2000:]
    st = json.loads(status.read_text())
    assert st["xgmi_links"] == ("not checked: gpu_metrics 1.9 is not a layout this agent reads (1.8): xGMI link state "
                                "not checked"), st
    assert st["xgmi_pairs"] == "1/1" and "xgmi_error" not in st
    assert r.stderr.count("xGMI link state not checked on any of the 2 GPU(s)") == 1, r.stderr[-2000:]


def test_a_stalled_bridge_read_leaves_the_topology_file_out_instead_of_hanging(native, tmp_path):
    """Bound every wait on the start path, the topology worker's included: its walk
    reads every bridge's PCI attributes above the GPUs and NICs, and a function in error recovery
    can stall such a read.  Here the root port above GPU 0 has a max_link_speed that never answers
    (a FIFO): the dry run finishes after --sysfs-read-timeout, rccl.env names no NCCL_TOPO_FILE
    (RCCL then reads the topology itself), and the log says why."""
    import time

    fx = fakesysfs.build_mi355x_node(tmp_path / "sys", n_gpus=2)
    parts = fx["gpus"][0]["path"].split("/")
    attr = tmp_path / "sys" / "devices" / "/".join(parts[:2]) / "max_link_speed"
    attr.unlink()
    os.mkfifo(attr)
    t0 = time.monotonic()
    r = subprocess.run([str(native_bin("discover")), "--dry-run", "--xgmi-expect=0", "--sysfs-read-timeout=1s",
                        f"--rccl-topo={tmp_path / 'rccl-topo.xml'}", f"--rccl-env={tmp_path / 'rccl.env'}",
                        f"--status-file={tmp_path / 'status.json'}"], capture_output=True, text=True, timeout=30,
                       env=dict(os.environ, SYSFS_ROOT=str(tmp_path / "sys")))
    took = time.monotonic() - t0
    assert r.returncode == 0, r.stderr[-2000:]
    assert took < 5, took
    assert "The RCCL topology file was not generated within 1s" in r.stderr, r.stderr[-2000:]
    assert not (tmp_path / "rccl-topo.xml").exists()
    assert "NCCL_TOPO_FILE" not in (tmp_path / "rccl.env").read_text()


def test_agent_start_timing_on_a_fake_mi355x_node(native, tmp_path):
    """network_operator_amd/agent/start_timing.py (bench.py's node_ready_gpu_side.agent_binary,
    tools/agent_start_box.py): the real discover binary's dry run, repeated, on a fake sysfs copy
    of an 8-GPU node: its own phase timings and the process wall time."""
    from network_operator_amd.agent import start_timing

    fakesysfs.build_mi355x_node(tmp_path / "sys", n_gpus=8)
    r = start_timing.measure(runs=3, sysfs=str(tmp_path / "sys") + "/")
    assert "error" not in r, r
    assert r["runs"] == 3 and r["xgmi_pairs"] == "28/28"
    assert {"discover", "xgmi", "gdr", "rccl_topo"} <= set(r["phases_ms"])
    assert 0 < r["process_wall_ms"]["p50"] <= r["process_wall_ms"]["max"]
    assert len(r["nics_not_in_this_netns"]) == 8  # the fake node's rails are not in this namespace
