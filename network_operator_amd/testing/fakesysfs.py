"""Fake sysfs trees for the node agent (``SYSFS_ROOT``).

``build_mi355x_node`` reproduces the PCIe / KFD topology of a real 8x MI355X node (captured
from a GPU box, see ``tests/fixtures/mi355x_node_topology.json``): eight 0x75a3 GPUs, each
behind a PCIe switch shared with one mlx5 RoCE NIC (its scale-out rail), two more mlx5 NICs on
their own root ports (frontend / management / storage: host NICs), and the KFD io_links of the
28-pair xGMI mesh.  NIC netdev names can be remapped so
the agent's affinity discovery finds the veth "NICs" of the netns harness.

The reference's equivalent is its tmpdir + ``SYSFS_ROOT`` fake tree
(reference cmd/discover/network_test.go:94-116,226-252).
"""

from __future__ import annotations

import json
import os
from pathlib import Path
from typing import Dict, Optional

FIXTURE = Path(__file__).resolve().parents[2] / "tests" / "fixtures" / "mi355x_node_topology.json"


def _w(path: Path, content: str) -> None:
    path.parent.mkdir(parents=True, exist_ok=True)
    path.write_text(content)


def _link(target: Path, link: Path) -> None:
    link.parent.mkdir(parents=True, exist_ok=True)
    if not link.exists() and not link.is_symlink():
        os.symlink(os.path.relpath(target, link.parent), link)


def _pci(root: Path, pcipath: str, driver: str, vendor: str, device: str, numa: int, cls: str) -> Path:
    d = root / "devices" / pcipath
    d.mkdir(parents=True, exist_ok=True)
    _w(d / "vendor", vendor + "\n")
    _w(d / "device", device + "\n")
    _w(d / "numa_node", f"{numa}\n")
    _w(d / "class", cls + "\n")
    _w(d / "subsystem_vendor", vendor + "\n")
    _w(d / "subsystem_device", device + "\n")
    _w(d / "max_link_speed", "32.0 GT/s PCIe\n")
    _w(d / "max_link_width", "16\n")
    _w(d / "current_link_speed", "32.0 GT/s PCIe\n")  # trained at the maximum, as on the live node
    _w(d / "current_link_width", "16\n")
    # Bridges above the function (root port, switch up/downstream ports): the attributes RCCL's
    # topology reads from each of them (Broadcom PEX switch ports, like the live node).
    parts = pcipath.split("/")
    for k in range(1, len(parts) - 1):
        b = root / "devices" / "/".join(parts[: k + 1])
        if not (b / "class").exists():
            _w(b / "class", "0x060400\n")
            _w(b / "vendor", "0x1000\n")
            _w(b / "device", "0xc030\n")
            _w(b / "subsystem_vendor", "0x1000\n")
            _w(b / "subsystem_device", "0x0072\n")
            _w(b / "numa_node", f"{numa}\n")
            # PCIe 5 x16 on every port
            _w(b / "max_link_speed", "32.0 GT/s PCIe\n")
            _w(b / "max_link_width", "16\n")
    drv = root / "bus" / "pci" / "drivers" / driver
    drv.mkdir(parents=True, exist_ok=True)
    _link(drv, d / "driver")
    _link(d, root / "bus" / "pci" / "devices" / d.name)  # /sys/bus/pci/devices/<bdf>, as on a host
    return d


# NIC driver -> (PCI vendor id, RDMA device name prefix) for rail_driver.
RAIL_DRIVERS = {"mlx5_core": ("0x15b3", "mlx5"), "ionic": ("0x1dd8", "ionic"), "bnxt_en": ("0x14e4", "bnxt_re")}


def build_mi355x_node(root: Path, nic_names: Optional[Dict[str, str]] = None, nic_macs: Optional[Dict[str, str]] = None,
                      n_gpus: int = 8, with_kfd: bool = True, drop_xgmi_pairs=(), rail_driver: str = "") -> dict:
    """Writes the tree under ``root``; returns the fixture (with applied renames).

    nic_names: {original ifname -> new ifname}; nic_macs: {new ifname -> MAC}.
    drop_xgmi_pairs: iterable of (gpu_i, gpu_j) KFD-order indices whose xGMI link is removed.
    n_gpus < 8: a smaller node of the same layout, so the rails of the GPUs left out (the NICs
    behind their PCIe switches) are left out too.
    rail_driver: the scale-out NICs (one behind each GPU's PCIe switch) are of this driver, with
    its RDMA device names (``ionic``: AMD Pollara, ``ionic_<n>``; ``bnxt_en``: ``bnxt_re<n>``)
    instead of the captured node's ConnectX-7 (``mlx5_core``); the host NICs stay mlx5.
    """
    fx = json.loads(FIXTURE.read_text())
    if rail_driver:
        vendor, prefix = RAIL_DRIVERS[rail_driver]
        rails = {tuple(g["path"].split("/")[:3]) for g in fx["gpus"]}
        for n in fx["nics"]:
            if tuple(n["pcipath"].split("/")[:3]) in rails:
                n.update(driver=rail_driver, vendor=vendor)
        k = 0
        for r in sorted(fx["rdma"], key=lambda r: r["dev"]):
            if tuple(r["pcipath"].split("/")[:3]) in rails:
                r["dev"] = f"{prefix}_{k}" if prefix != "bnxt_re" else f"{prefix}{k}"
                k += 1
    nic_names = nic_names or {}
    nic_macs = nic_macs or {}
    root = Path(root)
    gpus = sorted(fx["gpus"], key=lambda g: g["bdf"])[:n_gpus]
    for g in gpus:
        d = _pci(root, g["path"], "amdgpu", g["vendor"], g["device"], g["numa"], "0x120000")
        _link(d, root / "bus" / "pci" / "drivers" / "amdgpu" / g["bdf"])
    nics = []
    built = {tuple(g["path"].split("/")[:3]) for g in gpus}
    every = {tuple(g["path"].split("/")[:3]) for g in fx["gpus"]}
    for n in fx["nics"]:
        under = tuple(n["pcipath"].split("/")[:3])
        if under in every and under not in built:
            continue  # the rail of a GPU this node does not have
        name = nic_names.get(n["ifname"], n["ifname"])
        d = _pci(root, n["pcipath"], n["driver"], n.get("vendor", "0x15b3"), "0x1021", 0 if n["pcipath"] < "pci0000:80" else 1,
                 "0x020000")
        net = d / "net" / name
        _w(net / "address", nic_macs.get(name, n["mac"]) + "\n")
        _w(net / "dev_port", "0\n")
        _link(d, net / "device")  # /sys/class/net/<if>/device -> the PCI function, as on a host
        _link(net, root / "class" / "net" / name)
        nics.append(dict(n, ifname=name))
    kept = {n["pcipath"] for n in nics}
    for r in fx["rdma"]:
        if r["pcipath"] not in kept:
            continue
        d = root / "devices" / r["pcipath"] / "infiniband" / r["dev"]
        d.mkdir(parents=True, exist_ok=True)
        _link(d, root / "class" / "infiniband" / r["dev"])
    # Two NUMA nodes of 128 CPUs each, interleaved like the live box's cpumaps.
    _w(root / "devices" / "system" / "node" / "node0" / "cpumap",
       "00000000,00000000,ffffffff,ffffffff,00000000,00000000,ffffffff,ffffffff\n")
    _w(root / "devices" / "system" / "node" / "node1" / "cpumap",
       "ffffffff,ffffffff,00000000,00000000,ffffffff,ffffffff,00000000,00000000\n")
    _w(root / "devices" / "virtual" / "net" / "lo" / "address", "00:00:00:00:00:00\n")
    _link(root / "devices" / "virtual" / "net" / "lo", root / "class" / "net" / "lo")

    if with_kfd:
        base = root / "class" / "kfd" / "kfd" / "topology" / "nodes"
        _w(base / "0" / "properties", "cpu_cores_count 128\nsimd_count 0\n")
        _w(base / "1" / "properties", "cpu_cores_count 128\nsimd_count 0\n")
        drop = {tuple(sorted(p)) for p in drop_xgmi_pairs}
        for i, g in enumerate(gpus):
            node = i + 2
            bus, dev, fn = (int(x, 16) for x in g["bdf"][5:].replace(".", ":").split(":"))
            loc = (bus << 8) | (dev << 3) | fn
            _w(base / str(node) / "properties",
               f"simd_count 1024\nvendor_id 4098\ndevice_id {int(g['device'], 16)}\nlocation_id {loc}\ndomain 0\n"
               f"hive_id {fx['kfd_gpu_node']['hive_id']}\nnum_xcc 8\n")
            _w(base / str(node) / "gpu_id", f"{1000 + i}\n")
            li = 0
            _w(base / str(node) / "io_links" / str(li) / "properties",
               f"type 2\nnode_from {node}\nnode_to {g['numa']}\nweight 20\nmax_bandwidth 64000\n")
            li += 1
            for j in range(len(gpus)):
                if j == i or tuple(sorted((i, j))) in drop:
                    continue
                _w(base / str(node) / "io_links" / str(li) / "properties",
                   f"type 11\nnode_from {node}\nnode_to {j + 2}\nweight 15\nmin_bandwidth 76000\nmax_bandwidth 76000\n")
                li += 1
        # amdgpu's gpu_metrics (as captured on a live MI355X, 1.8): every GPU's 7 xGMI links up.
        blob = GPU_METRICS_FIXTURE.read_bytes()
        for g in gpus:
            (root / "devices" / g["path"] / "gpu_metrics").write_bytes(blob)
    fx["nics"] = nics
    fx["gpus"] = gpus
    return fx


GPU_METRICS_FIXTURE = FIXTURE.parent / "gpu_metrics_v1_8.bin"
_GM18_XGMI_STATUS = 264  # u16 per link slot: 1 up, 0 down, 0xffff no link


def set_pcie_link(root: Path, bdf: str, speed_gts: float, width: int) -> None:
    """The PCIe link a function trained at (a card in a worn slot: 16 GT/s x8 of 32 GT/s x16)."""
    d = Path(root) / "bus" / "pci" / "devices" / bdf
    _w(d / "current_link_speed", f"{speed_gts:.1f} GT/s PCIe\n")
    _w(d / "current_link_width", f"{width}\n")


def set_xgmi_link(root: Path, bdf: str, slot: int, up: bool) -> None:
    """Writes one xGMI link's state into a GPU's gpu_metrics, as the firmware would when the link
    trains or drops (the file is replaced whole, like a sysfs read sees one snapshot)."""
    f = Path(root) / "bus" / "pci" / "devices" / bdf / "gpu_metrics"
    b = bytearray(f.read_bytes())
    b[_GM18_XGMI_STATUS + 2 * slot:_GM18_XGMI_STATUS + 2 * slot + 2] = (1 if up else 0).to_bytes(2, "little")
    tmp = f.with_name("gpu_metrics.tmp")
    tmp.write_bytes(bytes(b))
    tmp.replace(f)


def add_rocev2_gids(root: Path, rdma_dev: str, ips, port: int = 1) -> None:
    """Populates a GID table like mlx5 does after an IPv4 address is configured."""
    p = Path(root) / "class" / "infiniband" / rdma_dev / "ports" / str(port)
    _w(p / "gids" / "0", "fe80:0000:0000:0000:0000:00ff:fe00:0001\n")
    _w(p / "gid_attrs" / "types" / "0", "IB/RoCE v1\n")
    _w(p / "gids" / "1", "fe80:0000:0000:0000:0000:00ff:fe00:0001\n")
    _w(p / "gid_attrs" / "types" / "1", "RoCE v2\n")
    idx = 2
    for ip in ips:
        a, b, c, d = (int(x) for x in ip.split("."))
        gid = f"0000:0000:0000:0000:0000:ffff:{a:02x}{b:02x}:{c:02x}{d:02x}"
        for t in ("IB/RoCE v1", "RoCE v2"):
            _w(p / "gids" / str(idx), gid + "\n")
            _w(p / "gid_attrs" / "types" / str(idx), t + "\n")
            idx += 1


# CPU identity of the live MI355X boxes as RCCL records it (its topology dump: Zen 5,
# familyid 191 / modelid 2) -- fixed so golden files do not depend on the build machine's CPU.
MI355X_HOST_CPU = {"arch": "x86_64", "vendor": "AuthenticAMD", "family": 191, "model": 2}


def nic_pci_dir(root: Path, ifname: str) -> Path:
    """The PCI function directory behind a netdev of the tree."""
    return (Path(root) / "class" / "net" / ifname).resolve().parent.parent


def unbind_driver(root: Path, ifname: str) -> None:
    """The NIC's kernel driver is not loaded: the function has no ``driver`` link."""
    (nic_pci_dir(root, ifname) / "driver").unlink(missing_ok=True)


def bind_driver(root: Path, ifname: str, driver: str) -> None:
    """What loading a NIC driver (the host-nic KMD container) does to sysfs: the function binds."""
    drv = Path(root) / "bus" / "pci" / "drivers" / driver
    drv.mkdir(parents=True, exist_ok=True)
    link = nic_pci_dir(root, ifname) / "driver"
    link.unlink(missing_ok=True)
    os.symlink(os.path.relpath(drv, link.parent), link)


def remove_rdma(root: Path, ifname: str) -> str:
    """The NIC's RDMA driver (mlx5_ib, ionic_rdma, bnxt_re) is not loaded: its function has no
    ``infiniband/`` device.  Returns the device name it had ("" if none)."""
    import shutil

    ib = nic_pci_dir(root, ifname) / "infiniband"
    devs = sorted(os.listdir(ib)) if ib.is_dir() else []
    shutil.rmtree(ib, ignore_errors=True)
    for d in devs:
        (Path(root) / "class" / "infiniband" / d).unlink(missing_ok=True)
    return devs[0] if devs else ""


def bind_rdma(root: Path, ifname: str, dev: str, ips=()) -> None:
    """What loading the NIC's RDMA driver does to sysfs: the function gets its ``infiniband/<dev>``
    device (and /sys/class/infiniband/<dev>), and the RDMA core fills the port's GID table from the
    netdev's addresses (RoCE v2 GIDs of `ips`)."""
    d = nic_pci_dir(root, ifname) / "infiniband" / dev
    d.mkdir(parents=True, exist_ok=True)
    _link(d, Path(root) / "class" / "infiniband" / dev)
    if ips:
        add_rocev2_gids(root, dev, list(ips))


def _main(argv=None) -> int:
    """Against $SYSFS_ROOT, the simulated driver containers of the end-to-end harness
    (testing/e2e.py):

    * ``bind <driver> <ifname>...``: the NIC kernel driver binds the functions (host-nic KMD);
    * ``bind-rdma <ifname>=<rdma-dev>[@<ipv4>] ...``: the NICs' RDMA driver registers their RDMA
      devices (amd-so ``driverImage``)."""
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("op", choices=["bind", "bind-rdma"])
    ap.add_argument("args", nargs="+")
    a = ap.parse_args(argv)
    root = Path(os.environ["SYSFS_ROOT"])
    if a.op == "bind":
        driver, ifnames = a.args[0], a.args[1:]
        for i in ifnames:
            bind_driver(root, i, driver)
        print(f"bound {', '.join(ifnames)} to {driver}")
        return 0
    for spec in a.args:
        ifname, rest = spec.split("=", 1)
        dev, _, ip = rest.partition("@")
        bind_rdma(root, ifname, dev, [ip] if ip else [])
    print(f"registered RDMA devices for {', '.join(x.split('=')[0] for x in a.args)}")
    return 0


def real_nic_order() -> list:
    """Fixture's scale-out NIC names in GPU (BDF) order — what affine discovery returns."""
    fx = json.loads(FIXTURE.read_text())
    return [n["ifname"] for n in fx["nics"] if n["ifname"].startswith("enp")]


if __name__ == "__main__":
    import sys

    sys.exit(_main())
