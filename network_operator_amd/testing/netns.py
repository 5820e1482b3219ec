"""Synthetic-switch network-namespace harness (veth pairs + injected LLDP).

What it builds (all inside ``unshare -rn``, so nothing touches the host network):

    node netns (this process)                 switch netns (forked child)
    enp5s0np0 ... (one veth end per NIC)  <->  swp0 ... (netop-lldp-tx: LLDP with
    discover (the real C++ agent binary)        "<tag> a.b.c.d/30" Port Descriptions)
    SYSFS_ROOT = fake MI355X node tree          optional 802.1AB-2009 fast start

Node-side veths are named like the real node's mlx5 scale-out NICs, and the fake sysfs
(``fakesysfs.build_mi355x_node``) places them behind the same PCIe switches as the GPUs,
so the agent runs its normal affinity discovery, xGMI verification and L3 configuration.

Measured: t(agent start) -> t(NFD readiness label visible), plus the agent's own phase
timings.  For the same run the harness also reports the *reference model*: the time the
switch's first periodic LLDPDU reaches the last NIC (what an agent that never solicits
fast start, like the reference's pcap listener, waits for at best).

The reference has no such harness ("How multi-node is tested without a
cluster: it isn't").
"""

from __future__ import annotations

import argparse
import ctypes
import ctypes.util
import json
import os
import random
import shutil
import signal
import statistics
import subprocess
import sys
import tempfile
import time
from pathlib import Path
from typing import Optional

CLONE_NEWNET = 0x40000000


def unshare_cmd() -> list[str]:
    """Real root: a plain network namespace (a user namespace would lose DAC access to
    directories owned by other users); otherwise user + network namespaces."""
    return ["unshare", "-n"] if os.geteuid() == 0 else ["unshare", "-rn"]


def unavailable() -> dict | None:
    """None when a private network namespace with AF_PACKET and netlink sockets can be made; else
    ``{"code": ..., "why": ...}``.  The reason is taken from what failed, never from whatever a
    process happened to print last: a child under a profiler (rocprofv3's preloaded tool logs at
    exit) or any other wrapper adds lines of its own.

    codes: ``no-unshare`` (util-linux missing), ``unshare`` (the kernel refused the namespace:
    no user namespaces, a container without CAP_SYS_ADMIN), ``sockets`` (namespace made, but no
    AF_PACKET / netlink socket in it), ``timeout``, ``spawn``."""
    if not shutil.which("unshare"):
        return {"code": "no-unshare", "why": "unshare(1) not installed"}
    probe = ("import socket\n"
             "try:\n"
             " socket.socket(socket.AF_PACKET, socket.SOCK_RAW, 0); socket.socket(socket.AF_NETLINK, socket.SOCK_RAW, 0)\n"
             "except OSError as e:\n"
             " print('NETOP-PROBE sockets ' + str(e)); raise SystemExit(3)\n"
             "print('NETOP-PROBE ok')")
    try:
        r = subprocess.run([*unshare_cmd(), sys.executable, "-c", probe], capture_output=True, text=True, timeout=60)
    except subprocess.TimeoutExpired:
        return {"code": "timeout", "why": "unshare: the probe did not finish in 60 s"}
    except OSError as e:  # pragma: no cover
        return {"code": "spawn", "why": f"unshare: {e}"}
    marks = [ln.split(" ", 2)[1:] for ln in r.stdout.splitlines() if ln.startswith("NETOP-PROBE ")]
    if r.returncode == 0 and ["ok"] in marks:
        return None
    for m in marks:
        if m and m[0] == "sockets":
            return {"code": "sockets", "why": "no AF_PACKET / netlink socket in the namespace: " + (m[1] if len(m) > 1 else "")}
    # unshare(1) itself failed: its own message ("unshare: unshare failed: Operation not permitted").
    own = [ln.strip() for ln in r.stderr.splitlines() if ln.strip().startswith("unshare:")]
    return {"code": "unshare", "why": own[0] if own else f"unshare exited with status {r.returncode}"}


def available() -> tuple[bool, str]:
    """True when a private network namespace with AF_PACKET sockets can be created; else why not."""
    u = unavailable()
    return (True, "ok") if u is None else (False, u["why"])


# ---------------------------------------------------------------------------
# Address plans
# ---------------------------------------------------------------------------
def random_plan(n: int, rng: random.Random) -> list[dict]:
    """n distinct /30 links inside one random /16; peer is .1 or .2 of each /30."""
    second = rng.randrange(0, 256)
    blocks = rng.sample(range(16384), n)
    tags = ["no-alert", "scale-out", "gpu-fabric", "leaf-port"]
    plan = []
    for b in blocks:
        base = (10 << 24) | (second << 16) | (b * 4)
        host = rng.choice((1, 2))
        peer = base + host
        local = peer ^ 3
        fmt = lambda v: ".".join(str((v >> s) & 255) for s in (24, 16, 8, 0))  # noqa: E731
        plan.append({"peer": fmt(peer), "local": fmt(local), "p2p": fmt(base) + "/30",
                     "routed": f"10.{second}.0.0/16", "desc": f"{rng.choice(tags)} {fmt(peer)}/30"})
    return plan


# ---------------------------------------------------------------------------
# Inside the namespace
# ---------------------------------------------------------------------------
def _native():
    here = Path(__file__).resolve().parents[2]
    if str(here) not in sys.path:
        sys.path.insert(0, str(here))
    from network_operator_amd.agent import native

    return native()


def _wait_for(path: Path, timeout: float, proc=None, poll: float = 0.0005) -> float | None:
    """Monotonic time at which `path` appeared; None on timeout or if `proc` exited first."""
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if path.exists():
            return time.monotonic()
        if proc is not None and proc.poll() is not None:
            return time.monotonic() if path.exists() else None
        time.sleep(poll)
    return None


def _in_netns(pid: int, fn) -> int:
    """Runs fn() in a forked child that joined the network namespace of `pid`."""
    libc = ctypes.CDLL(ctypes.util.find_library("c"), use_errno=True)
    child = os.fork()
    if child == 0:
        code = 1
        try:
            fd = os.open(f"/proc/{pid}/ns/net", os.O_RDONLY)
            if libc.setns(fd, CLONE_NEWNET) != 0:
                os._exit(3)
            fn()
            code = 0
        finally:
            os._exit(code)
    _, status = os.waitpid(child, 0)
    return os.waitstatus_to_exitcode(status)


def set_switch_port(pid: int, port: str, up: bool) -> None:
    def go():
        rt = _native().Rtnl()
        idx = rt.link_by_name(port)["index"]
        (rt.link_set_up if up else rt.link_set_down)(idx)
    if _in_netns(pid, go) != 0:
        raise RuntimeError(f"could not set {port} {'up' if up else 'down'} in the switch namespace")


def _tx_packets() -> dict:
    """Transmitted packets per interface of this network namespace (/proc/net/dev follows it)."""
    out = {}
    for line in Path("/proc/net/dev").read_text().splitlines()[2:]:
        name, data = line.split(":", 1)
        out[name.strip()] = int(data.split()[9])
    return out


def egress_matrix(nic_names: list, plan: list, packets: int = 20) -> list:
    """For each NIC k: send UDP datagrams from a socket bound to NIC k's address to an off-link
    address of the routed /16 and count which NICs transmitted them.  Row k is the per-NIC
    packet delta; with per-rail tables all of row k lands on NIC k."""
    import ipaddress
    import socket

    rows = []
    for p in plan:
        dst = str(ipaddress.ip_network(p["routed"]).broadcast_address - 1)  # x.y.255.254: behind the switch
        before = _tx_packets()
        with socket.socket(socket.AF_INET, socket.SOCK_DGRAM) as s:
            s.bind((p["local"], 0))
            for _ in range(packets):
                s.sendto(b"rail-probe", (dst, 9))
        time.sleep(0.05)
        after = _tx_packets()
        rows.append([after.get(n, 0) - before.get(n, 0) for n in nic_names])
    return rows


class NetnsHolder:
    """An empty network namespace kept alive by a sleeping child (another node of the fabric).
    ``enter()`` is a ``preexec_fn`` that moves a new child process into it."""

    def __init__(self):
        libc = ctypes.CDLL(ctypes.util.find_library("c"), use_errno=True)
        r, w = os.pipe()
        pid = os.fork()
        if pid == 0:
            try:
                os.close(r)
                if libc.unshare(CLONE_NEWNET) != 0:
                    os._exit(3)
                os.write(w, b"1")
                signal.pause()
            finally:
                os._exit(0)
        os.close(w)
        os.read(r, 1)
        os.close(r)
        self.pid = pid

    def enter(self) -> None:
        libc = ctypes.CDLL(ctypes.util.find_library("c"), use_errno=True)
        fd = os.open(f"/proc/{self.pid}/ns/net", os.O_RDONLY)
        if libc.setns(fd, CLONE_NEWNET) != 0:
            raise OSError(ctypes.get_errno(), "setns")
        os.close(fd)

    def run(self, fn) -> int:
        """fn() in a forked child inside the namespace; its exit code."""
        return _in_netns(self.pid, fn)

    def stop(self) -> None:
        if self.pid:
            os.kill(self.pid, signal.SIGKILL)
            os.waitpid(self.pid, 0)
            self.pid = 0


class SyntheticSwitch:
    """The switch namespace: a forked child unshares its network namespace, receives one veth peer
    (``swp<i>``) per node NIC, and runs ``netop-lldp-tx`` with each port's Port Description from
    `plan`.  The last `silent_nics` ports send no LLDP."""

    def __init__(self, nic_names: list, plan: list, rng: random.Random, interval: str = "30s", phase: str = "random",
                 fast_start: bool = True, silent_nics: int = 0, remote: Optional[list] = None, forward: bool = False,
                 system_name: str = "", port_system_names: Optional[dict] = None, max_frame_size: int = 0):
        """`remote`: (network-namespace pid, ifname) of NICs of other nodes, wired to the ports after
        this namespace's `nic_names` (`plan` covers both).  `forward`: the switch routes between its
        /30s (a leaf of an L3 fabric), so nodes reach each other over their /16 routes."""
        from ..utils.paths import native_bin

        self.nic_names, self.plan = list(nic_names), plan
        self.remote = list(remote or [])
        self.forward = forward
        self.ports = [f"swp{i}" for i in range(len(self.nic_names) + len(self.remote))]
        self.args = [str(native_bin("netop-lldp-tx")), f"--interval={interval}", f"--phase={phase}", "--assign-ip",
                     f"--seed={rng.randrange(1, 1 << 30)}"]
        if fast_start:
            self.args.append("--fast-start")
        if max_frame_size:  # LLDP 802.3 Maximum Frame Size TLV (the switch ports' MTU)
            self.args.append(f"--max-frame-size={max_frame_size}")
        if system_name:  # "{port}": one leaf per rail
            self.args.append(f"--system-name={system_name}")
        for sp, name in (port_system_names or {}).items():
            self.args.append(f"--port-system-name={sp}={name}")
        for i, (sp, p) in enumerate(zip(self.ports, plan)):
            if i >= len(plan) - silent_nics:
                self.args.append(f"--silent-port={sp}")  # up (carrier) but never sends LLDP
                continue
            self.args.append(f"--port={sp}={p['desc']}")
        self.pid = 0
        self.first_periodic: dict = {}  # port -> seconds (switch clock) of its first periodic frame
        self._out = None

    def start(self, rt) -> float:
        """Creates the veth pairs (node ends keep the NIC names) and starts the switch; returns the
        monotonic time at which the switch got its ports."""
        has_ports = any(a.startswith(("--port=", "--silent-port=")) for a in self.args)
        libc = ctypes.CDLL(ctypes.util.find_library("c"), use_errno=True)
        r1, w1 = os.pipe()
        r2, w2 = os.pipe()
        out_r, out_w = os.pipe()
        pid = os.fork()
        if pid == 0:  # switch: own netns, wait for the ports, exec lldp-tx
            try:
                os.close(r1)
                os.close(w2)
                os.close(out_r)
                if libc.unshare(CLONE_NEWNET) != 0:
                    os._exit(3)
                if self.forward:
                    with open("/proc/sys/net/ipv4/ip_forward", "w") as f:
                        f.write("1")
                os.write(w1, b"1")
                os.read(r2, 1)
                os.dup2(out_w, 1)
                if not has_ports:  # no port sends anything
                    signal.pause()
                os.execv(self.args[0], self.args)
            finally:
                os._exit(4)
        self.pid = pid
        os.close(w1)
        os.close(r2)
        os.close(out_w)
        os.read(r1, 1)
        for node_if, sp in zip(self.nic_names, self.ports):
            rt.veth_add(node_if, sp)
            rt.link_set_netns_pid(rt.link_by_name(sp)["index"], pid)
        for k, ((node_pid, node_if), sp) in enumerate(zip(self.remote, self.ports[len(self.nic_names):])):
            tmp_if = f"rn{k}"  # created here, moved, then renamed inside the node's namespace
            rt.veth_add(tmp_if, sp)
            rt.link_set_netns_pid(rt.link_by_name(sp)["index"], pid)
            rt.link_set_netns_pid(rt.link_by_name(tmp_if)["index"], node_pid)

            def rename(old=tmp_if, new=node_if):
                r = _native().Rtnl()
                r.link_set_name(r.link_by_name(old)["index"], new)
            if _in_netns(node_pid, rename) != 0:
                raise RuntimeError(f"could not name {node_if} in namespace of pid {node_pid}")
        t_switch = time.monotonic()
        os.write(w2, b"1")
        self._out = os.fdopen(out_r)
        if has_ports:
            for line in self._out:
                if line.startswith("first "):
                    _, ifn, ns = line.split()
                    self.first_periodic[ifn] = int(ns) / 1e9
                if line.strip() == "ready":
                    break
        return t_switch

    def stop(self) -> None:
        if self.pid:
            os.kill(self.pid, signal.SIGTERM)
            os.waitpid(self.pid, 0)
            self.pid = 0
        if self._out is not None:
            self._out.close()
            self._out = None


def run_scenario(n_nics: int = 8, mode: str = "L3", seed: int | None = None, interval: str = "30s",
                 fast_start: bool = True, announce: bool = True, phase: str = "random", wait: str = "90s",
                 mtu: int = 9000, pipeline: bool = True, bad_nics: int = 0, silent_nics: int = 0,
                 xgmi_expect: int = 0, keep_tmp: bool = False, sigterm: bool = True, verbose: int = 2,
                 drop_xgmi: list | None = None, extra_args: list | None = None, flap_port: int | None = None,
                 crash_restart: bool = False, crash_after_s: float = 0.0, gid_delay_s: float = 0.0,
                 egress_probe: bool = False, nm_bus: bool = False, nm_restore: bool = True, lldp_cache: bool = False,
                 soak_cycles: int = 0, arp_silent_ports: int = 0, switch_name: str = "",
                 port_switch_names: dict | None = None, nic_speeds_mbps: list | None = None,
                 switch_max_frame: int = 0, dark_port: int | None = None,
                 dark_port_up_after: float | None = None, kill_mid_config: int = 0, rail_driver: str = "",
                 xgmi_down_at_start: tuple | None = None, xgmi_up_after: float | None = None,
                 xgmi_link_flap: tuple | None = None, pcie_degraded: dict | None = None,
                 link_state: bool = True, pcie_flap: int | None = None, rails_without_rdma: int = 0,
                 rdma_bind_after: float | None = None, label_holddown: str | None = None,
                 flap_burst: tuple | None = None, gpu_metrics_stall: bool = False,
                 sysfs_read_timeout: str = "", require_rdma: bool = True,
                 pcie_restored_after: float | None = None) -> dict:
    """Runs one node bring-up.  Must already be inside a private user+net namespace.

    nm_bus: run the agent with --disable-networkmanager against a real ``dbus-daemon`` on which a
    NetworkManager stand-in owns the name (testing/fakedbus.py), with an NM keyfile directory,
    and record both before and after SIGTERM.

    lldp_cache: run the agent with --lldp-cache; with crash_restart, also record how long after
    the restart the switch's frames confirmed every cached Port Description.

    dark_port: that switch port is down when the agent starts (the NIC has no carrier); once the
    agent has said why it is not ready, the port comes up and the label must follow.
    dark_port_up_after: instead, the port comes up that many seconds after the agent started (an
    optic still training its link); every reason and status the agent wrote meanwhile is kept.

    kill_mid_config: SIGKILL the agent that many times part-way through configuring the node
    (after 1, 2, ... of its NICs are configured, by its own log) and start it again each time;
    the last start runs to readiness and is what the result describes.  ``mid_config_kills``
    records the state each kill left behind.

    rail_driver: the scale-out NICs' driver and RDMA names (fakesysfs.build_mi355x_node).

    xgmi_down_at_start / xgmi_link_flap: (GPU index, link slot) whose xGMI link is down in the
    GPU's gpu_metrics before the agent starts / goes down after readiness and comes back.
    xgmi_up_after: the link down at start comes up that many seconds after the agent started;
    the reasons the agent gave meanwhile are kept.

    pcie_flap: after readiness that rail's NIC retrains its PCIe link at 16 GT/s x8, then back.

    pcie_degraded: {NIC index (an int, or its str after JSON): (GT/s, width)} -- that rail's NIC trained its PCIe link below the
    maximum (32 GT/s x16); {"gpu<i>": (GT/s, width)} the same for GPU i.  pcie_restored_after:
    those links retrain at the maximum that many seconds after the agent started ("pcie_restore").

    require_rdma: pass --require-rdma, as the operator does for every amd-so policy unless
    ``requireRdma: false`` (off: that policy, or an agent build older than the flag).

    rails_without_rdma: the first k rails' NICs have no RDMA device (their RDMA driver is not
    loaded) when the agent starts; with rdma_bind_after, the devices (and their GIDs) appear that
    many seconds after the agent started, and the reasons and files meanwhile are kept ("rdma").

    label_holddown: the agent's --label-holddown (default: "0s" for the scenarios that time a
    republication, else the agent's own).  flap_burst: (switch port, count, period s) -- after
    readiness that port flaps `count` times, one period each; every label transition is recorded.

    gpu_metrics_stall: after readiness GPU 0's gpu_metrics becomes a FIFO nobody writes (a wedged
    SMU: the read never returns) and switch port 0 then loses carrier: how fast the label goes
    while the read is stalled, and what the agent says once the read times out
    (sysfs_read_timeout, the agent's --sysfs-read-timeout)."""
    from . import fakesysfs

    nat = _native()
    from ..utils.paths import native_bin

    rng = random.Random(seed)
    rt = nat.Rtnl()
    rt.link_set_up(rt.link_by_name("lo")["index"])
    tmp = Path(tempfile.mkdtemp(prefix="netop-sim-"))
    try:
        fx = fakesysfs.build_mi355x_node(tmp / "sys", n_gpus=n_nics, rail_driver=rail_driver,
                                         drop_xgmi_pairs=[tuple(p) for p in (drop_xgmi or [])])
        degraded_bdfs = []
        for key, (gts, width) in (pcie_degraded or {}).items():
            if isinstance(key, str) and key.startswith("gpu"):
                bdf = fx["gpus"][int(key[3:])]["bdf"]
            else:
                bdf = fakesysfs.nic_pci_dir(tmp / "sys", nat.discover(str(tmp / "sys"))["pairs"][int(key)]["nic"]).name
            fakesysfs.set_pcie_link(tmp / "sys", bdf, gts, width)
            degraded_bdfs.append(bdf)
        if xgmi_down_at_start is not None:
            fakesysfs.set_xgmi_link(tmp / "sys", fx["gpus"][xgmi_down_at_start[0]]["bdf"], xgmi_down_at_start[1], False)
        pairs = nat.discover(str(tmp / "sys"))["pairs"]
        nic_names = [p["nic"] for p in pairs][:n_nics]
        rdma_removed = {nif: fakesysfs.remove_rdma(tmp / "sys", nif) for nif in nic_names[:rails_without_rdma]}
        plan = random_plan(len(nic_names), rng)
        for nif, mbps in zip(nic_names, nic_speeds_mbps or []):  # what the NIC driver negotiated
            (tmp / "sys" / "class" / "net" / nif / "speed").write_text(f"{mbps}\n")
        for i, p in enumerate(plan):
            if i < bad_nics:
                p["desc"] = "no-alert not-an-address"
        rdma = {n["ifname"]: "" for n in fx["nics"]}
        # GID tables as mlx5 would populate them once the address is configured.
        disc = nat.discover(str(tmp / "sys"))
        gid_jobs = []
        for n in disc["nics"]:
            if n["ifname"] in nic_names and n["rdma_dev"]:
                gid_jobs.append((n["rdma_dev"], plan[nic_names.index(n["ifname"])]["local"]))
                rdma[n["ifname"]] = n["rdma_dev"]

        def add_gids():
            for dev, ip in gid_jobs:
                fakesysfs.add_rocev2_gids(tmp / "sys", dev, [ip])

        if gid_delay_s > 0:
            # Like the RDMA core: the RoCE v2 GID shows up a little after the address is added.
            import threading

            threading.Timer(gid_delay_s, add_gids).start()
        else:
            add_gids()

        sw = SyntheticSwitch(nic_names, plan, rng, interval=interval, phase=phase, fast_start=fast_start,
                             silent_nics=silent_nics, system_name=switch_name, port_system_names=port_switch_names,
                             max_frame_size=switch_max_frame)
        t_switch = sw.start(rt)
        pid, sw_ports, first_periodic = sw.pid, sw.ports, sw.first_periodic
        for sp in sw_ports[len(sw_ports) - arp_silent_ports:] if arp_silent_ports else []:
            # A switch port that has its LLDP Port Description but does not answer on that /30
            # (arp_ignore 8: no ARP replies at all) — what --verify-peers is for.
            def mute(port=sp):
                Path(f"/proc/sys/net/ipv4/conf/{port}/arp_ignore").write_text("8")
            if _in_netns(pid, mute) != 0:
                raise RuntimeError(f"could not silence ARP on {sp}")

        feat = tmp / "features.d"
        feat.mkdir()
        label = feat / "scale-out-readiness.txt"
        args = [str(native_bin("discover")), "--configure=true", "--keep-running", f"--mode={mode}", f"--mtu={mtu}",
                f"--wait={wait}", f"--rccl-net={tmp / 'rccl-net.json'}", f"--rccl-env={tmp / 'rccl.env'}",
                f"--rccl-topo={tmp / 'rccl-topo.xml'}", f"--status-file={tmp / 'status.json'}", f"--nfd-features-dir={feat}", f"--xgmi-expect={xgmi_expect}",
                f"--pipeline={'true' if pipeline else 'false'}", f"--lldp-announce={'true' if announce else 'false'}",
                f"--systemd-networkd={tmp / 'networkd'}", f"-v={verbose}", *(extra_args or [])]
        if link_state:  # as the operator passes it (off: an agent build older than the flag, bench/agent_ab.py)
            args.append(f"--link-state={tmp / 'link-state'}")
        if require_rdma:  # likewise (the CRD default requireRdma: true)
            args.append("--require-rdma")
        if label_holddown is None and (flap_port is not None or soak_cycles or xgmi_link_flap is not None
                                       or pcie_flap is not None or gpu_metrics_stall):
            label_holddown = "0s"  # these time the republication itself
        if label_holddown is not None:
            args.append(f"--label-holddown={label_holddown}")
        if sysfs_read_timeout:
            args.append(f"--sysfs-read-timeout={sysfs_read_timeout}")
        if lldp_cache:
            args.append(f"--lldp-cache={tmp / 'lldp-cache'}")
        env = dict(os.environ, SYSFS_ROOT=str(tmp / "sys"), NODE_NAME="mi355x-node-0")
        bus = nm = None
        keyfile = tmp / "NetworkManager" / "conf.d" / "99-amd-network-operator.conf"
        if nm_bus:
            from .fakedbus import BusDaemon, NetworkManagerOnBus

            (tmp / "dbus").mkdir()
            (tmp / "NetworkManager").mkdir()
            bus = BusDaemon(str(tmp / "dbus"))
            nm = NetworkManagerOnBus(bus.address, {**{n: True for n in nic_names}, "eth9": True})
            env["DBUS_SYSTEM_BUS_ADDRESS"] = bus.address
            args += ["--disable-networkmanager", f"--nm-keyfile-dir={keyfile.parent}"]
            if nm_restore:
                args.append("--nm-restore")
        # The agent's log goes to a file, not a pipe nobody reads until the end: a long run
        # (soak_cycles) logs more than a pipe buffer holds and would block the agent.
        agent_log = tmp / "agent.log"

        def spawn():
            with open(agent_log, "a") as logf:
                return subprocess.Popen(args, env=env, stdout=logf, stderr=subprocess.STDOUT, text=True)
        if dark_port is not None:
            set_switch_port(pid, sw_ports[dark_port], False)
        t0 = time.monotonic()
        agent = spawn()
        budget = 5.0 + float(wait.rstrip("s"))
        mid_kills = []
        for k in range(kill_mid_config):
            # An OOM kill or a node-agent crash half-way: some NICs have their address (and rail
            # rule and table), the rest nothing.  Progress is read from this run's own log, since
            # the addresses of earlier runs are still on the links.
            want = 1 + k % max(1, len(nic_names) - 1)
            start = agent_log.stat().st_size if agent_log.exists() else 0
            done = 0
            end = time.monotonic() + budget
            while time.monotonic() < end and agent.poll() is None and done < want:
                with open(agent_log, errors="replace") as f:
                    f.seek(start)
                    tail = f.read()
                done = tail.count("Configured address and route") + tail.count("already configured with address")
                time.sleep(0.0005)
            agent.kill()
            agent.wait()
            addressed = sum(1 for n in nic_names if rt.addr_list(rt.link_by_name(n)["index"]))
            rules = [r for r in rt.rule_list() if 0 < r["priority"] < 32766]
            mid_kills.append({"after_configured": done, "wanted": want, "nics_with_address": addressed,
                              "rules": len(rules), "label": label.exists(), "rc": agent.returncode})
            t0 = time.monotonic()
            agent = spawn()
        dark: dict = {}
        if dark_port is not None and dark_port_up_after is not None:
            reason, status = tmp / "status.json.not-ready", tmp / "status.json"
            seen_reasons, seen_flags = [], set()
            while time.monotonic() < t0 + dark_port_up_after and agent.poll() is None:
                try:
                    why = reason.read_text()
                    if why and why not in seen_reasons:
                        seen_reasons.append(why)
                except OSError:
                    pass
                try:
                    for i in json.loads(status.read_text()).get("interfaces", []):
                        seen_flags |= {f"{i['name']}:{k}" for k in ("awaiting_carrier", "no_carrier") if i.get(k)}
                except (OSError, ValueError):
                    pass
                time.sleep(0.05)
            dark["reasons_seen"], dark["status_flags_seen"] = seen_reasons, sorted(seen_flags)
            dark["label_while_dark"] = label.exists()
            t_up = time.monotonic()
            set_switch_port(pid, sw_ports[dark_port], True)
            t_ready = _wait_for(label, 10, agent)
            dark["port_up_s"] = t_up - t0
            dark["port_up_to_label_s"] = (t_ready - t_up) if t_ready else None
        elif dark_port is not None:
            reason = tmp / "status.json.not-ready"
            t_why = _wait_for(reason, budget, agent)
            # Past --carrier-wait: "waiting for carrier" turns into the fault.
            while t_why and time.monotonic() < t0 + budget and agent.poll() is None:
                try:
                    if "waiting for carrier" not in reason.read_text():
                        break
                except OSError:
                    pass
                time.sleep(0.02)
            t_why = time.monotonic() if t_why else None
            dark["reason_s"] = (t_why - t0) if t_why else None
            dark["label_while_dark"] = label.exists()
            dark["reason"] = reason.read_text() if reason.exists() else None
            # The agent writes the probe's reason first and status.json right after it: give the
            # second write its moment (a sanitizer build widens the gap).
            t_end = time.monotonic() + 2.0
            while True:
                try:
                    st = json.loads((tmp / "status.json").read_text())
                    dark["status_ready"] = st.get("ready")
                    dark["status_no_carrier"] = [i["name"] for i in st["interfaces"] if i.get("no_carrier")]
                except (OSError, ValueError, KeyError):
                    dark["status_ready"] = dark["status_no_carrier"] = None
                if dark["status_no_carrier"] or time.monotonic() >= t_end:
                    break
                time.sleep(0.02)
            pr = subprocess.run([str(native_bin("discover")), "--ready-check", f"--nfd-features-dir={feat}",
                                 f"--status-file={tmp / 'status.json'}"], capture_output=True, text=True, timeout=10)
            dark["ready_check"] = {"rc": pr.returncode, "stdout": pr.stdout.strip()}
            t_up = time.monotonic()
            set_switch_port(pid, sw_ports[dark_port], True)
            t_ready = _wait_for(label, 10, agent)
            dark["port_up_to_label_s"] = (t_ready - t_up) if t_ready else None
        elif pcie_degraded and pcie_restored_after is not None:
            # The narrow link retrains at full width while the agent runs (a reseat needs none,
            # but PCIe error recovery or a hot reset can): the monitor configures the NIC it left
            # unconfigured and labels the node, no restart needed.
            reason, seen = tmp / "status.json.not-ready", []
            while time.monotonic() < t0 + pcie_restored_after and agent.poll() is None:
                try:
                    why = reason.read_text()
                    if why and why not in seen:
                        seen.append(why)
                except OSError:
                    pass
                time.sleep(0.02)
            dark["reasons_seen"], dark["label_while_narrow"] = seen, label.exists()
            dark["running_while_narrow"] = agent.poll() is None
            t_fix = time.monotonic()
            for bdf in degraded_bdfs:
                fakesysfs.set_pcie_link(tmp / "sys", bdf, 32.0, 16)
            t_ready = _wait_for(label, 10, agent)
            dark["restore_to_label_s"] = (t_ready - t_fix) if t_ready else None
        elif rails_without_rdma and rdma_bind_after is not None:
            # The rails' RDMA driver is loaded while the agent runs (a driver container, the node):
            # until then the agent configures, stays up unlabelled and says why; then it labels.
            reason, seen, env_seen = tmp / "status.json.not-ready", [], False
            while time.monotonic() < t0 + rdma_bind_after and agent.poll() is None:
                try:
                    why = reason.read_text()
                    if why and why not in seen:
                        seen.append(why)
                except OSError:
                    pass
                env_seen |= (tmp / "rccl.env").exists()
                time.sleep(0.02)
            dark["reasons_seen"], dark["label_while_missing"] = seen, label.exists()
            dark["rccl_env_while_missing"], dark["running_while_missing"] = env_seen, agent.poll() is None
            try:
                st = json.loads((tmp / "status.json").read_text())
                dark["configured_while_missing"] = [i["name"] for i in st["interfaces"] if i.get("configured")]
            except (OSError, ValueError, KeyError):
                dark["configured_while_missing"] = None
            t_bind = time.monotonic()
            for nif, dev in rdma_removed.items():
                fakesysfs.bind_rdma(tmp / "sys", nif, dev, [plan[nic_names.index(nif)]["local"]])
            t_ready = _wait_for(label, 10, agent)
            dark["bind_to_label_s"] = (t_ready - t_bind) if t_ready else None
        elif xgmi_down_at_start is not None and xgmi_up_after is not None:
            reason, seen = tmp / "status.json.not-ready", []
            while time.monotonic() < t0 + xgmi_up_after and agent.poll() is None:
                try:
                    why = reason.read_text()
                    if why and why not in seen:
                        seen.append(why)
                except OSError:
                    pass
                time.sleep(0.05)
            dark["reasons_seen"], dark["label_while_down"] = seen, label.exists()
            t_up = time.monotonic()
            fakesysfs.set_xgmi_link(tmp / "sys", fx["gpus"][xgmi_down_at_start[0]]["bdf"], xgmi_down_at_start[1], True)
            t_ready = _wait_for(label, 10, agent)
            dark["link_up_to_label_s"] = (t_ready - t_up) if t_ready else None
        else:
            t_ready = _wait_for(label, budget, agent)
        res: dict = {"n_nics": len(nic_names), "mode": mode, "fast_start": fast_start, "announce": announce,
                     "interval": interval, "pipeline": pipeline, "plan": plan, "nics": nic_names}
        res["ready"] = t_ready is not None
        res["latency_s"] = (t_ready - t0) if t_ready else None
        if dark:
            res["dark"] = dark
        if kill_mid_config:
            res["mid_config_kills"] = mid_kills
        try:  # CPU of the process so far (coarse: clock ticks; the status has getrusage at readiness)
            f = Path(f"/proc/{agent.pid}/stat").read_text().rsplit(")", 1)[1].split()
            res["agent_cpu_ms"] = (int(f[11]) + int(f[12])) * 1000.0 / os.sysconf("SC_CLK_TCK")
        except (OSError, IndexError, ValueError):
            res["agent_cpu_ms"] = None
        try:  # resource envelope (the DaemonSet requests 45Mi / limits 90Mi, like the reference)
            st = Path(f"/proc/{agent.pid}/status").read_text()
            res["agent_rss_kib"] = int(next(x for x in st.splitlines() if x.startswith("VmHWM:")).split()[1])
            res["agent_threads"] = int(next(x for x in st.splitlines() if x.startswith("Threads:")).split()[1])
        except (OSError, StopIteration, ValueError):
            res["agent_rss_kib"] = None
        if first_periodic:
            res["reference_model_s"] = max(0.0, max(first_periodic.values()) - t0)
        # Inspect the configured node.
        state = {}
        for node_if, p in zip(nic_names, plan):
            try:
                link = rt.link_by_name(node_if)
                state[node_if] = {"up": link["up"], "mtu": link["mtu"], "addrs": rt.addr_list(link["index"]),
                                  "routes": [r for r in rt.route_list() if r["ifindex"] == link["index"]]}
            except OSError as e:
                state[node_if] = {"error": str(e)}
        res["state"] = state
        res["rules"] = [r for r in rt.rule_list() if 0 < r["priority"] < 32766]  # not the kernel's defaults
        if egress_probe and t_ready:
            res["egress"] = egress_matrix(nic_names, plan)
        res["rail_tables"] = {r["table"]: rt.route_list(r["table"]) for r in res["rules"]}
        if t_ready:  # the agent writes status.json (ready=true) right after the label
            end = time.monotonic() + 5
            while time.monotonic() < end and agent.poll() is None:
                try:
                    if json.loads((tmp / "status.json").read_text()).get("ready"):
                        break
                except (OSError, ValueError):
                    pass
                time.sleep(0.001)
        for f in ("rccl-net.json", "status.json"):
            fp = tmp / f
            res[f.split(".")[0].replace("-", "_")] = json.loads(fp.read_text()) if fp.exists() else None
        res["rccl_env"] = (tmp / "rccl.env").read_text() if (tmp / "rccl.env").exists() else None
        res["rccl_topo"] = (tmp / "rccl-topo.xml").read_text() if (tmp / "rccl-topo.xml").exists() else None
        res["label"] = label.read_text() if label.exists() else None
        if nm is not None:
            res["nm_keyfile_while_ready"] = keyfile.read_text() if keyfile.exists() else None
            res["nm_managed_while_ready"] = dict(nm.devices)
        res["networkd_files"] = sorted(os.listdir(tmp / "networkd")) if (tmp / "networkd").exists() else []
        if crash_restart and t_ready:
            # The agent dies without cleaning up (OOM kill, node agent crash): the label, the
            # addresses and the switch's neighbour entry are all stale.  The restarted agent
            # must start from scratch and still be ready in fast-start time.
            time.sleep(crash_after_s)  # e.g. let the switch's fast-transmission window run out
            agent.kill()
            agent.wait()
            res["stale_label_after_crash"] = label.exists()
            wall = time.time_ns()
            t_r = time.monotonic()
            restart_log_at = agent_log.stat().st_size if agent_log.exists() else 0
            agent = spawn()
            back = None
            end = t_r + budget
            while time.monotonic() < end and agent.poll() is None:
                try:
                    if label.stat().st_mtime_ns >= wall:
                        back = time.monotonic()
                        break
                except FileNotFoundError:
                    pass
                time.sleep(0.0005)
            res["restart_latency_s"] = (back - t_r) if back else None
            if lldp_cache and back:
                def sources():
                    try:
                        st = json.loads((tmp / "status.json").read_text())
                    except (OSError, ValueError):
                        return None
                    return [i.get("lldp_source") for i in st["interfaces"]]

                # How each NIC was configured at the restart, from the restarted agent's own log: a
                # fast-start switch may confirm the cache before status.json is read.
                with open(agent_log, errors="replace") as f:
                    f.seek(restart_log_at)
                    restart_log = f.read()
                res["restart_lldp_sources"] = [
                    "cache" if f"interface '{n}': Port Description" in restart_log and "from the LLDP cache" in restart_log
                    .split(f"interface '{n}': Port Description", 1)[1].split("\n", 1)[0] else "frame" for n in nic_names]
                confirmed = None
                while time.monotonic() < end and agent.poll() is None:
                    if sources() == ["frame"] * len(nic_names):
                        confirmed = time.monotonic()
                        break
                    time.sleep(0.01)
                res["cache_confirmed_s"] = (confirmed - t_r) if confirmed else None
                res["restart_rccl_net"] = json.loads((tmp / "rccl-net.json").read_text())
        if flap_port is not None and t_ready:
            # Carrier loss on one switch port: the agent must withdraw the label, then restore
            # it (and the NIC's routes) once the port is back.
            sp = sw_ports[flap_port]
            t_down = time.monotonic()
            set_switch_port(pid, sp, False)
            gone = None
            end = t_down + 10
            while time.monotonic() < end:
                if not label.exists():
                    gone = time.monotonic()
                    break
                time.sleep(0.001)
            res["flap_withdraw_s"] = (gone - t_down) if gone else None
            t_up = time.monotonic()
            set_switch_port(pid, sp, True)
            back = _wait_for(label, 10, agent)
            res["flap_restore_s"] = (back - t_up) if back else None
            link = rt.link_by_name(nic_names[flap_port])
            res["flap_routes_after"] = [r for r in rt.route_list() if r["ifindex"] == link["index"]]
        if xgmi_link_flap is not None and t_ready:
            # A GPU's xGMI link drops after readiness (gpu_metrics): the label goes while it is
            # down, with the reason, and comes back with the link.
            bdf = fx["gpus"][xgmi_link_flap[0]]["bdf"]
            time.sleep(0.05)  # status.json follows the label
            t_down = time.monotonic()
            fakesysfs.set_xgmi_link(tmp / "sys", bdf, xgmi_link_flap[1], False)
            gone = None
            while time.monotonic() < t_down + 10 and agent.poll() is None:
                if not label.exists():
                    gone = time.monotonic()
                    break
                time.sleep(0.002)
            reason = tmp / "status.json.not-ready"
            why = reason.read_text() if reason.exists() else None
            t_up = time.monotonic()
            fakesysfs.set_xgmi_link(tmp / "sys", bdf, xgmi_link_flap[1], True)
            back = _wait_for(label, 10, agent)
            res["xgmi_flap"] = {"gpu": bdf, "withdraw_s": (gone - t_down) if gone else None,
                                "restore_s": (back - t_up) if back else None, "reason": why}
        if pcie_flap is not None and t_ready:
            bdf = fakesysfs.nic_pci_dir(tmp / "sys", nic_names[pcie_flap]).name
            time.sleep(0.05)  # status.json follows the label
            t_down = time.monotonic()
            fakesysfs.set_pcie_link(tmp / "sys", bdf, 16.0, 8)
            gone = None
            while time.monotonic() < t_down + 10 and agent.poll() is None:
                if not label.exists():
                    gone = time.monotonic()
                    break
                time.sleep(0.002)
            reason = tmp / "status.json.not-ready"
            why = reason.read_text() if reason.exists() else None
            t_up = time.monotonic()
            fakesysfs.set_pcie_link(tmp / "sys", bdf, 32.0, 16)
            back = _wait_for(label, 10, agent)
            res["pcie_flap"] = {"withdraw_s": (gone - t_down) if gone else None,
                                "restore_s": (back - t_up) if back else None, "reason": why}
        if flap_burst is not None and t_ready:
            # A flapping optic: the port goes down and up `count` times.  Every label transition
            # is recorded (polled every 0.5 ms); with a hold-down the label goes once and comes back
            # once, hold-down seconds after the last flap.
            import threading

            port, count, period = int(flap_burst[0]), int(flap_burst[1]), float(flap_burst[2])
            time.sleep(0.05)  # status.json follows the label
            edges, done = [], threading.Event()

            def watch():
                was = label.exists()
                while not done.is_set():
                    now = label.exists()
                    if now != was:
                        edges.append((time.monotonic(), now))
                        was = now
                    time.sleep(0.0005)
            w = threading.Thread(target=watch)
            w.start()
            t_first = time.monotonic()
            reasons = []
            for _ in range(count):
                set_switch_port(pid, sw_ports[port], False)
                time.sleep(period / 2)
                set_switch_port(pid, sw_ports[port], True)
                t_last_up = time.monotonic()
                time.sleep(period / 2)
                try:
                    reasons.append((tmp / "status.json.not-ready").read_text())
                except OSError:
                    pass
            back = None
            end = t_last_up + 30
            while time.monotonic() < end and agent.poll() is None:
                if edges and edges[-1][1]:
                    back = edges[-1][0]
                    break
                time.sleep(0.005)
            done.set()
            w.join()
            res["flap_burst"] = {"flaps": count, "burst_s": t_last_up - t_first,
                                 "withdrawals": sum(1 for _, up in edges if not up),
                                 "publishes": sum(1 for _, up in edges if up),
                                 "last_up_to_label_s": (back - t_last_up) if back else None,
                                 "reasons": sorted(set(reasons))}
            try:
                res["flap_burst"]["metrics_status"] = json.loads((tmp / "status.json").read_text()).get("ready")
            except (OSError, ValueError):
                pass
        if gpu_metrics_stall and t_ready:
            # A wedged SMU: GPU 0's gpu_metrics read never returns (a FIFO nobody writes).  The
            # monitor must keep handling link events at once; once the read times out it names the
            # GPU and withholds the label; when the SMU answers again, the label comes back.
            bdf = fx["gpus"][0]["bdf"]
            gm = tmp / "sys" / "bus" / "pci" / "devices" / bdf / "gpu_metrics"
            blob = gm.read_bytes()
            time.sleep(0.05)

            def withdraw_after_carrier_loss(port):
                # Timed from the carrier loss: set_switch_port returns once the switch end is down
                # (its netns hop, a fork, costs a few ms and is not the agent's).
                set_switch_port(pid, sw_ports[port], False)
                t = time.monotonic()
                while time.monotonic() < t + 10 and agent.poll() is None:
                    if not label.exists():
                        return time.monotonic() - t
                    time.sleep(0.0002)
                return None

            def flaps(n):  # carrier losses, each withdrawal timed; the port back up, the label back
                out = []
                for k in range(n):
                    out.append(withdraw_after_carrier_loss(k % 2))
                    set_switch_port(pid, sw_ports[k % 2], True)
                    _wait_for(label, 5, agent)
                    time.sleep(0.02)
                return out
            base = flaps(5)  # the same, with no read stalled
            gm.unlink()
            os.mkfifo(gm)
            t_stall = time.monotonic()
            time.sleep(0.3)  # several --xgmi-health-interval periods: a read is stuck by now
            during = flaps(5)  # all within the read timeout: the label is still up before each
            flaps_done = time.monotonic() - t_stall
            reason = tmp / "status.json.not-ready"
            t_why, why = None, None
            while time.monotonic() < t_stall + 30 and agent.poll() is None:
                try:
                    why = reason.read_text()
                    if "did not answer" in why:
                        t_why = time.monotonic()
                        break
                except OSError:
                    pass
                time.sleep(0.01)
            gone = _wait_gone(label, 1.0)  # the label follows the reason (write_status goes first)

            def med(xs):
                xs = [x for x in xs if x is not None]
                return _pct(xs, 0.5) if xs else None
            stall = {"withdraw_during_stall_s": during, "withdraw_during_stall_p50_s": med(during),
                     "withdraw_without_stall_s": base, "withdraw_without_stall_p50_s": med(base),
                     "flaps_done_s": flaps_done, "reason": why,
                     "stall_to_reason_s": (t_why - t_stall) if t_why else None, "label_while_stalled": not gone}
            # The SMU answers again: the blocked read gets its data, the file is a file again.
            try:  # ENXIO when no read is blocked on it
                fd = os.open(gm, os.O_WRONLY | os.O_NONBLOCK)
            except OSError:
                fd = -1
            if fd >= 0:
                try:
                    os.write(fd, blob)
                finally:
                    os.close(fd)
            tmpf = gm.with_name("gpu_metrics.tmp")
            tmpf.write_bytes(blob)
            tmpf.replace(gm)
            t_ans = time.monotonic()
            back = _wait_for(label, 15, agent)
            stall["answer_to_label_s"] = (back - t_ans) if back else None
            res["gpu_metrics_stall"] = stall
        if soak_cycles and t_ready:
            # Carrier loss on a random port, over and over, with the agent in monitor mode: every
            # cycle must withdraw and restore the label, and the agent must not leak descriptors,
            # threads or memory.  The baseline is taken after the first cycle (lazy allocations).
            def proc_stat():
                time.sleep(0.1)  # let the agent finish the status write that follows the label
                st = Path(f"/proc/{agent.pid}/status").read_text().splitlines()
                val = {x.split(":")[0]: x.split()[1] for x in st if x.startswith(("VmRSS:", "Threads:"))}
                return {"fds": len(os.listdir(f"/proc/{agent.pid}/fd")), "rss_kib": int(val["VmRSS"]),
                        "threads": int(val["Threads"])}
            withdraw, restore, base = [], [], None
            for k in range(soak_cycles):
                i = rng.randrange(len(nic_names))
                t_down = time.monotonic()
                set_switch_port(pid, sw_ports[i], False)
                gone = None
                end = t_down + 10
                while time.monotonic() < end and agent.poll() is None:
                    if not label.exists():
                        gone = time.monotonic()
                        break
                    time.sleep(0.0005)
                t_up = time.monotonic()
                set_switch_port(pid, sw_ports[i], True)
                back = _wait_for(label, 10, agent)
                if gone is None or back is None:
                    break
                withdraw.append(gone - t_down)
                restore.append(back - t_up)
                if k == 0:
                    base = proc_stat()
            fin = proc_stat() if agent.poll() is None else None
            addrs_ok = all(rt.addr_list(rt.link_by_name(n)["index"]) == [p["local"] + "/30"]
                           for n, p in zip(nic_names, plan)) if mode == "L3" else None
            res["soak"] = {"cycles": len(withdraw), "asked": soak_cycles, "first": base, "last": fin,
                           "withdraw_p50_s": _pct(withdraw, 0.5) if withdraw else None,
                           "withdraw_max_s": max(withdraw) if withdraw else None,
                           "restore_p50_s": _pct(restore, 0.5) if restore else None,
                           "restore_max_s": max(restore) if restore else None, "addrs_ok": addrs_ok}
        t_term = None
        if sigterm and agent.poll() is None:
            t_term = time.monotonic()
            agent.send_signal(signal.SIGTERM)
        try:
            agent.wait(timeout=20)
        except subprocess.TimeoutExpired:
            agent.kill()
            agent.wait()
        out = agent_log.read_text(errors="replace") if agent_log.exists() else ""
        res["sigterm_to_exit_s"] = (time.monotonic() - t_term) if t_term else None
        res["agent_rc"] = agent.returncode
        res["agent_log"] = out[-6000:]
        try:  # the agent's last word (a failed start never wrote a ready-time status)
            res["status_at_exit"] = json.loads((tmp / "status.json").read_text())
        except (OSError, ValueError):
            res["status_at_exit"] = None
        if res.get("status") is None:
            res["status"] = res["status_at_exit"]
        after = {}
        for node_if in nic_names:
            link = rt.link_by_name(node_if)
            after[node_if] = {"up": link["up"], "addrs": rt.addr_list(link["index"])}
        res["after_sigterm"] = after
        res["rules_after_sigterm"] = [r for r in rt.rule_list() if 0 < r["priority"] < 32766]
        res["label_after_sigterm"] = label.exists()
        res["link_state_left"] = (tmp / "link-state").exists()
        if nm is not None:
            res["nm_keyfile_after_sigterm"] = keyfile.exists()
            res["nm_managed_after_sigterm"] = dict(nm.devices)
            nm.stop()
            bus.stop()
        sw.stop()
        res["switch_start_offset_s"] = t0 - t_switch
        return res
    finally:
        if not keep_tmp:
            shutil.rmtree(tmp, ignore_errors=True)


def run_policy_routing_uplink() -> dict:
    """a rail NIC with its own source-routing table holding a default route
    (``from 192.168.50.0/24 lookup 1001``, ``default via 192.168.50.1 dev rail0 table 1001``)
    while the node's uplink is another NIC (main table).  The agent must take the rail (dry run:
    not refused; a real L2 start: configured, with a warning about the per-NIC route) and still
    refuse the uplink.  The table id is above 255 (RTA_TABLE).  Must run inside ``unshare -rn``."""
    from ..utils.paths import native_bin

    nat = _native()
    rt = nat.Rtnl()
    rt.link_set_up(rt.link_by_name("lo")["index"])
    tmp = Path(tempfile.mkdtemp(prefix="netop-polroute-"))
    try:
        for nif, peer in (("rail0", "rpeer0"), ("mgmt0", "mpeer0")):
            rt.veth_add(nif, peer)
            rt.link_set_up(rt.link_by_name(peer)["index"])
            rt.link_set_up(rt.link_by_name(nif)["index"])
        rail, mgmt = rt.link_by_name("rail0")["index"], rt.link_by_name("mgmt0")["index"]
        rt.addr_add(rail, "192.168.50.10/24")
        rt.addr_add(mgmt, "10.0.0.5/24")
        rt.rule_add("192.168.50.0/24", 1001, 1000)
        rt.route_append("0.0.0.0/0", "192.168.50.1", rail, 4, table=1001)  # RTPROT_STATIC
        rt.route_append("0.0.0.0/0", "10.0.0.1", mgmt, 4)
        res: dict = {"default_route_links": sorted(rt.default_route_links()), "rail": rail, "mgmt": mgmt,
                     "rules": rt.rule_list(), "table_1001": rt.route_list(1001)}
        base = [str(native_bin("discover")), "--mode=L2", "--nic-discovery=none", "--mtu=9000", "-v=2",
                f"--nfd-features-dir={tmp / 'features.d'}"]
        env = dict(os.environ, SYSFS_ROOT=str(tmp / "sys"))
        (tmp / "sys").mkdir()
        for name, ifs in (("dry_rail", "rail0"), ("dry_mgmt", "mgmt0")):
            st = tmp / f"{name}.json"
            r = subprocess.run([*base, "--dry-run", f"--interfaces={ifs}", f"--status-file={st}"], env=env,
                               capture_output=True, text=True, timeout=30)
            res[name] = {"rc": r.returncode, "stderr": r.stderr[-2000:],
                         "status": json.loads(st.read_text()) if st.exists() else None}
        # rail0 holds 192.168.50.10/24, the source its rule selects: the node reaches 192.168.50/24
        # through it: refused unless --allow-policy-routed.
        r = subprocess.run([*base, "--configure=true", "--interfaces=rail0", "--carrier-wait=2s"], env=env,
                           capture_output=True, text=True, timeout=30)
        res["configure_rail_refused"] = {"rc": r.returncode, "stderr": r.stderr[-3000:],
                                         "mtu": rt.link_by_name("rail0")["mtu"], "addrs": rt.addr_list(rail)}
        r = subprocess.run([*base, "--configure=true", "--interfaces=rail0", "--carrier-wait=2s", "--allow-policy-routed"],
                           env=env, capture_output=True, text=True, timeout=30)
        res["configure_rail"] = {"rc": r.returncode, "stderr": r.stderr[-3000:],
                                 "mtu": rt.link_by_name("rail0")["mtu"]}
        # rail1: its own policy table serves only a /30 of the agent's (an earlier --keep-config
        # run): configured without the opt-in, with the warning.
        rt.veth_add("rail1", "rpeer1")
        rt.link_set_up(rt.link_by_name("rpeer1")["index"])
        r1 = rt.link_by_name("rail1")["index"]
        rt.link_set_up(r1)
        rt.addr_add(r1, "10.77.1.1/30")
        rt.rule_add("10.99.0.0/16", 1002, 1001)
        rt.route_append("0.0.0.0/0", "10.77.1.2", r1, 4, table=1002)
        r = subprocess.run([*base, "--configure=true", "--interfaces=rail1", "--carrier-wait=2s"], env=env,
                           capture_output=True, text=True, timeout=30)
        res["configure_own_rail"] = {"rc": r.returncode, "stderr": r.stderr[-3000:], "mtu": rt.link_by_name("rail1")["mtu"]}
        r = subprocess.run([*base, "--configure=true", "--interfaces=mgmt0"], env=env, capture_output=True, text=True,
                           timeout=30)
        res["configure_mgmt"] = {"rc": r.returncode, "stderr": r.stderr[-2000:], "mtu": rt.link_by_name("mgmt0")["mtu"],
                                 "addrs": rt.addr_list(mgmt)}
        return res
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


MGMT_NIC, HOST_NIC = "ens9np0", "ens49np1"  # the fixture node's two NICs on their own root ports


def run_host_nic_ownership(mode: str = "L2", rails: int = 8, mgmt_bridge: bool = False,
                           include_gpu_rails: bool = False, host_nic_addr: str = "",
                           free_host_nic: bool = False) -> dict:
    """A default ``host-nic`` policy's agent (rdma discovery, the default driver list) on the
    captured MI355X node, where every NIC is mlx5 with an RDMA device:

    * the GPU rails already carry what an amd-so agent gave them (a /30 each, MTU 9000);
    * ``ens9np0`` is the node's management NIC: 192.168.77.10/24 and the default route;
    * ``ens49np1`` is a free host NIC (down, no address).

    Records the state before, while the agent is ready, and after SIGTERM; then starts an agent
    that names the management NIC explicitly (``--interfaces``), which must refuse.  Each veth's
    peer stays in this namespace (up: the NIC has carrier).  With ``mgmt_bridge`` the management
    address and the default route sit on a bridge ``br0`` and ``ens9np0`` is only its port (the
    kernel's IFLA_MASTER is all that links them here: this sysfs is a fake).  With
    ``include_gpu_rails`` the agent runs as ``hostNic.includeGpuRails`` makes it (a node without
    amd-so): it takes the rails too, never the management NIC.  With ``host_nic_addr`` the
    second NIC is the node's own too (e.g. its storage network, that address /24): nothing is
    left for the agent, which must stay up unlabelled and say why (``idle``).  With
    ``free_host_nic`` that address is then removed: the idle agent, looking again every 300 ms,
    must exit so that its restart configures the NIC.  Must run inside ``unshare -rn``."""
    from . import fakesysfs
    from ..utils.paths import native_bin

    nat = _native()
    rt = nat.Rtnl()
    rt.link_set_up(rt.link_by_name("lo")["index"])
    tmp = Path(tempfile.mkdtemp(prefix="netop-owner-"))
    try:
        fakesysfs.build_mi355x_node(tmp / "sys", n_gpus=8)
        rail_names = fakesysfs.real_nic_order()[:rails]
        for k, nif in enumerate(rail_names + [MGMT_NIC, HOST_NIC]):
            rt.veth_add(nif, f"peer{k}")
            rt.link_set_up(rt.link_by_name(f"peer{k}")["index"])
        for k, nif in enumerate(rail_names):
            idx = rt.link_by_name(nif)["index"]
            rt.link_set_mtu(idx, 9000)
            rt.link_set_up(idx)
            rt.addr_add(idx, f"10.77.{k}.1/30")
        m = rt.link_by_name(MGMT_NIC)["index"]
        rt.link_set_up(m)
        if mgmt_bridge:
            rt.link_add("br0", "bridge")
            br = rt.link_by_name("br0")["index"]
            rt.link_set_master(m, br)
            rt.link_set_up(br)
            m = br
        rt.addr_add(m, "192.168.77.10/24")
        rt.route_append("0.0.0.0/0", "192.168.77.1", m, 16)  # a DHCP lease's default route
        if host_nic_addr:
            h = rt.link_by_name(HOST_NIC)["index"]
            rt.link_set_up(h)
            rt.addr_add(h, host_nic_addr)

        def snapshot() -> dict:
            out = {}
            for nif in rail_names + [MGMT_NIC, HOST_NIC]:
                link = rt.link_by_name(nif)
                out[nif] = {"up": link["up"], "mtu": link["mtu"], "addrs": rt.addr_list(link["index"]),
                            "master": link["master"]}
            out["default_routes"] = [r for r in rt.route_list() if r["dst"] == "0.0.0.0/0"]
            return out

        feat = tmp / "features.d"
        feat.mkdir()
        label = feat / "host-nic-readiness.txt"
        base = [str(native_bin("discover")), "--configure=true", "--keep-running", f"--mode={mode}", "--mtu=9000",
                "--restore-mtu", f"--mtu-state={tmp / 'mtu-state'}", f"--nfd-features-dir={feat}",
                "--nfd-label-file=host-nic-readiness.txt",
                "--nfd-label=amd.feature.node.kubernetes.io/host-nic-ready", "--wait=3s", "-v=2"]
        env = dict(os.environ, SYSFS_ROOT=str(tmp / "sys"), NODE_NAME="mi355x-node-0")
        res: dict = {"rails": rail_names, "before": snapshot(),
                     "discovery": nat.discover(str(tmp / "sys"), mode="rdma")}
        log_path = tmp / "agent.log"
        with open(log_path, "w") as logf:
            extra = ["--rdma-include-gpu-rails"] if include_gpu_rails else []
            if host_nic_addr:
                extra.append("--rediscover-interval=300ms")
            agent = subprocess.Popen([*base, "--nic-discovery=rdma", *extra, f"--status-file={tmp / 'status.json'}"],
                                     env=env, stdout=logf, stderr=subprocess.STDOUT)
        if host_nic_addr:
            reason = tmp / "status.json.not-ready"
            t_why = _wait_for(reason, 15, agent)
            time.sleep(1.0)  # still running a second later: no exit, no restart
            res["idle"] = {"reason_s": t_why is not None, "running": agent.poll() is None,
                           "label": label.exists(), "reason": reason.read_text() if reason.exists() else None}
            pr = subprocess.run([str(native_bin("discover")), "--ready-check", f"--nfd-features-dir={feat}",
                                 "--nfd-label-file=host-nic-readiness.txt", f"--status-file={tmp / 'status.json'}"],
                                capture_output=True, text=True, timeout=10)
            res["idle"]["ready_check"] = {"rc": pr.returncode, "stdout": pr.stdout.strip()}
            if free_host_nic:
                # The node gives the storage NIC up: the idle agent must notice and exit (rc 0),
                # so that the kubelet's restart configures it.
                rt.addr_del(rt.link_by_name(HOST_NIC)["index"], host_nic_addr)
                t_free = time.monotonic()
                try:
                    agent.wait(timeout=5)
                except subprocess.TimeoutExpired:
                    pass
                res["idle"]["after_free"] = {"exited": agent.poll() is not None, "rc": agent.poll(),
                                             "seconds": round(time.monotonic() - t_free, 3)}
        t_ready = _wait_for(label, 0.0 if host_nic_addr else 15, agent)
        res["ready"] = t_ready is not None
        res["label"] = label.read_text() if label.exists() else None
        time.sleep(0.05)  # status.json follows the label
        res["while_ready"] = snapshot()
        try:
            res["status"] = json.loads((tmp / "status.json").read_text())
        except (OSError, ValueError):
            res["status"] = None
        if agent.poll() is None:
            agent.send_signal(signal.SIGTERM)
        try:
            agent.wait(timeout=20)
        except subprocess.TimeoutExpired:
            agent.kill()
            agent.wait()
        res["agent_rc"] = agent.returncode
        res["after_sigterm"] = snapshot()
        res["mtu_state_left"] = (tmp / "mtu-state").exists()
        res["agent_log"] = log_path.read_text(errors="replace")[-6000:]
        # The management NIC named explicitly: refused, nothing touched.
        r = subprocess.run([*base, "--nic-discovery=none", f"--interfaces={MGMT_NIC}"], env=env, capture_output=True,
                           text=True, timeout=30)
        res["named_mgmt"] = {"rc": r.returncode, "stderr": r.stderr[-2000:], "after": snapshot()[MGMT_NIC]}
        return res
    finally:
        shutil.rmtree(tmp, ignore_errors=True)


# ---------------------------------------------------------------------------
# From outside: spawn into a fresh namespace
# ---------------------------------------------------------------------------
def run_isolated(timeout: float = 300, **kw) -> dict:
    """Runs ``run_scenario(**kw)`` in a new user+net namespace and returns its result."""
    cmd = [*unshare_cmd(), sys.executable, "-m", "network_operator_amd.testing.netns", "--json", json.dumps(kw)]
    root = Path(__file__).resolve().parents[2]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=root,
                       env=dict(os.environ, PYTHONPATH=str(root)))
    if r.returncode != 0:
        raise RuntimeError(f"scenario failed rc={r.returncode}: {r.stderr[-3000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def _wait_gone(path: Path, timeout: float) -> bool:
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if not path.exists():
            return True
        time.sleep(0.0005)
    return not path.exists()


def _pct(xs, q):
    s = sorted(xs)
    return s[min(len(s) - 1, max(0, int(round(q * (len(s) - 1)))))]


def node_ready_bench(n_nics: int = 8, runs: int = 5, interval: str = "30s", seed: int = 1, legacy: bool = True,
                     mode: str = "L3") -> dict:
    """Node-ready latency over `runs` fresh bring-ups, with (and optionally without) switch fast start."""
    out = {"n_nics": n_nics, "runs": runs, "interval": interval, "mode": mode}
    for label, fs in (("fast_start_switch", True), ("legacy_switch", False))[: 2 if legacy else 1]:
        lat, ref = [], []
        for k in range(runs):
            r = run_isolated(n_nics=n_nics, seed=seed * 1000 + k, interval=interval, fast_start=fs, verbose=0,
                             mode=mode)
            if not r["ready"]:
                raise RuntimeError(f"run {k} did not become ready: {r['agent_log'][-2000:]}")
            lat.append(r["latency_s"])
            ref.append(r.get("reference_model_s"))
        refs = [x for x in ref if x is not None]
        out[label] = {"latency_s": lat, "p50_s": statistics.median(lat), "p95_s": _pct(lat, 0.95), "max_s": max(lat),
                      "reference_model_s": ref,
                      "reference_model_p50_s": statistics.median(refs) if refs else None}
    return out


def _main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="{}", help="run_scenario kwargs")
    a = ap.parse_args(argv)
    kw = json.loads(a.json)
    if kw.pop("policy_routing_uplink", False):
        res = run_policy_routing_uplink()
    else:
        res = run_host_nic_ownership(**kw) if kw.pop("host_nic_ownership", False) else run_scenario(**kw)
    print(json.dumps(res))
    return 0


if __name__ == "__main__":
    sys.exit(_main())
