"""End-to-end node bring-up in private network namespaces (veth "NICs" + synthetic switch).

Runs the real ``discover`` binary against a fake sysfs copy of an 8x MI355X node.  Needs
root or user namespaces (available in the build container; skipped elsewhere).
"""

import ipaddress
import os

import pytest

from network_operator_amd.testing import netns

pytestmark = pytest.mark.netns


def _check_configured(r, rdma_prefix="mlx5_"):
    assert r["ready"], r["agent_log"][-3000:]
    for nic, p in zip(r["nics"], r["plan"]):
        st = r["state"][nic]
        assert st["up"] and st["mtu"] == 9000
        assert st["addrs"] == [p["local"] + "/30"]
        routes = {(x["dst"], x["gateway"]) for x in st["routes"]}
        assert (p["p2p"], None) in routes, routes
        assert (p["routed"], p["peer"]) in routes, routes
        kernel = [x for x in st["routes"] if x["dst"] == p["p2p"]][0]
        assert kernel["prefsrc"] == p["local"] and kernel["scope"] == 253  # link scope
    entries = r["rccl_net"]["NIC_NET_CONFIG"]
    assert len(entries) == len(r["nics"])
    by_name = {e["NIC_NAME"]: e for e in entries}
    for nic, p in zip(r["nics"], r["plan"]):
        e = by_name[nic]
        assert e["NIC_IP"] == p["local"] and e["GATEWAY_IP"] == p["peer"]
        assert e["SUBNET_MASK"] == "255.255.255.252"
        assert e["GID_INDEX"] == 3 and e["RDMA_DEV"].startswith(rdma_prefix)
        assert e["PCIE_PATH"] == "PXB" and e["NUMA_NODE"] == (0 if e["GPU_INDEX"] < 4 else 1)
    # GPU order: entry i belongs to GPU i.
    assert [e["GPU_INDEX"] for e in entries] == list(range(len(entries)))


def test_l3_fast_start_switch_full_node():
    r = netns.run_isolated(n_nics=8, seed=11, interval="30s", fast_start=True)
    _check_configured(r)
    assert r["latency_s"] < 3.0, r["latency_s"]  # answered by fast start, not the 30 s timer
    assert r["label"].startswith("amd.feature.node.kubernetes.io/gpu-scale-out=true\n")
    assert "gpu-xgmi.pairs=28" in r["label"]
    assert "NCCL_IB_GID_INDEX=3" in r["rccl_env"]
    # RCCL-consumed topology: the file exists, rccl.env names it, and bootstrap goes over the
    # rails in GPU order (rail 0 first on every node).
    topo_line = [l for l in r["rccl_env"].splitlines() if l.startswith("NCCL_TOPO_FILE=")]
    assert len(topo_line) == 1 and topo_line[0].endswith("/rccl-topo.xml")
    assert "NCCL_SOCKET_IFNAME==" + ",".join(r["nics"]) + "\n" in r["rccl_env"]
    import xml.etree.ElementTree as ET

    topo = ET.fromstring(r["rccl_topo"])
    assert len([n for n in topo.iter("net")]) == 8 and len([p for p in topo.iter("pci") if p.get("class") == "0x120000"]) == 8
    assert len(r["networkd_files"]) == 8
    # CPU of the bring-up, for the DaemonSet's CPU limit (500m; discovery/__init__.py).  Sanitizer
    # builds (make test-netns-asan) run several times slower.
    assert 0 < float(r["status"]["cpu_ms_at_ready"]) < (50 if not os.environ.get("NETOP_BIN_DIR") else 500)
    # SIGTERM: label removed, addresses flushed, links back down.
    assert r["agent_rc"] == 0
    assert not r["label_after_sigterm"]
    for nic in r["nics"]:
        assert r["after_sigterm"][nic] == {"up": False, "addrs": []}
    st = r["status"]
    assert st["ready"] and all(i["configured"] for i in st["interfaces"])
    # Resource envelope: far inside the DaemonSet's 45Mi request (reference daemonset.yaml:37-43).
    if not os.environ.get("NETOP_BIN_DIR"):  # sanitizer builds (make test-netns-asan) carry shadow memory
        assert r["agent_rss_kib"] is not None and r["agent_rss_kib"] < 16 * 1024


def test_first_announce_waits_for_operstate_up():
    """Frames sent between admin-up and linkwatch's qdisc attach are dropped silently; the agent
    announces per NIC on operstate UP, so no bring-up falls back to the 1 s re-announce (before
    that fix, 2 of 10 runs on a fresh machine took ~1.03 s)."""
    lat = [netns.run_isolated(n_nics=8, seed=400 + k, interval="30s", fast_start=True, verbose=0)["latency_s"]
           for k in range(6)]
    # (the fallback this pins is the 1 s re-announce, ~1.03 s; a loaded machine adds tenths)
    assert all(x is not None and x < 0.9 for x in lat), lat


def test_l3_legacy_switch_periodic_only():
    r = netns.run_isolated(n_nics=4, seed=12, interval="1s", fast_start=False)
    _check_configured(r)
    assert r["latency_s"] < 1.0 + 1.5


def test_without_announce_waits_for_periodic_frames():
    r = netns.run_isolated(n_nics=2, seed=13, interval="1500ms", phase="zero", fast_start=True, announce=False)
    _check_configured(r)


def test_pipeline_off_barrier_mode():
    r = netns.run_isolated(n_nics=3, seed=14, interval="1s", fast_start=True, pipeline=False)
    _check_configured(r)


def test_bad_port_description_fails_without_label():
    r = netns.run_isolated(n_nics=3, seed=15, interval="1s", fast_start=True, bad_nics=1, wait="5s")
    assert not r["ready"]
    assert r["agent_rc"] == 1
    assert "Not all interfaces were configured (2/3)" in r["agent_log"]


def test_silent_switch_port_times_out():
    """The silent NIC is named with its driver (the fake node's rail NICs are mlx5_core) and what
    it heard meanwhile, in the exit error (-> policy status.errors) and the status file."""
    r = netns.run_isolated(n_nics=2, seed=16, interval="1s", fast_start=True, silent_nics=1, wait="2s")
    assert not r["ready"]
    assert r["agent_rc"] == 1
    assert "expired with 1 interface(s) silent" in r["agent_log"]
    silent = r["nics"][-1]
    err = [ln for ln in r["agent_log"].splitlines() if ln.startswith("Error: ")][-1]
    assert err.startswith("Error: Not all interfaces were configured (1/2). LLDP silent on 1 NIC(s): "
                          f"{silent} (mlx5_core: no LLDPDU in 2s, "), err
    assert "frame(s) arrived meanwhile" in err
    st = {i["name"]: i for i in r["status"]["interfaces"]}
    assert st[silent]["driver"] == "mlx5_core" and st[silent]["lldp_silent"].startswith("mlx5_core: no LLDPDU in 2s")
    assert "lldp_silent" not in st[r["nics"][0]]


def test_l2_mode_no_addresses():
    r = netns.run_isolated(n_nics=2, seed=17, mode="L2", interval="1s")
    assert r["ready"], r["agent_log"][-2000:]
    for nic in r["nics"]:
        assert r["state"][nic]["up"] and r["state"][nic]["addrs"] == []
    assert "gpu-scale-out.mode=L2" in r["label"]
    # MI355X L2: RCCL still gets the scale-out HCAs and the RoCE v2 link-local GID index.
    assert "NCCL_IB_GID_INDEX=1" in r["rccl_env"] and "NCCL_IB_HCA==mlx5_" in r["rccl_env"]


def test_incomplete_xgmi_mesh_blocks_readiness():
    r = netns.run_isolated(n_nics=8, seed=18, interval="1s", drop_xgmi=[[0, 5]], wait="5s")
    assert not r["ready"]
    assert "xGMI mesh incomplete: 27 of 28" in r["agent_log"]


def test_random_plans_are_valid():
    import random

    for s in range(20):
        plan = netns.random_plan(8, random.Random(s))
        nets = set()
        for p in plan:
            peer, local = ipaddress.ip_address(p["peer"]), ipaddress.ip_address(p["local"])
            net = ipaddress.ip_network(p["p2p"])
            assert peer in net and local in net and peer != local
            assert peer not in (net.network_address, net.broadcast_address)
            nets.add(net)
        assert len(nets) == 8


def test_carrier_loss_withdraws_and_restores_readiness():
    r = netns.run_isolated(n_nics=4, seed=19, interval="1s", fast_start=True, flap_port=2)
    _check_configured(r)
    assert r["flap_withdraw_s"] is not None and r["flap_withdraw_s"] < 1.0, r["agent_log"][-3000:]
    assert r["flap_restore_s"] is not None and r["flap_restore_s"] < 2.0, r["agent_log"][-3000:]
    p = r["plan"][2]
    routes = {(x["dst"], x["gateway"]) for x in r["flap_routes_after"]}
    assert (p["routed"], p["peer"]) in routes and (p["p2p"], None) in routes
    assert "lost link" in r["agent_log"] and "readiness label republished" in r["agent_log"]


def test_repeated_carrier_loss_soak_leaks_nothing():
    """40 carrier-loss cycles on random ports under the monitor: each withdraws and restores the
    label, and descriptors, threads and RSS after the last cycle equal those after the first."""
    r = netns.run_isolated(n_nics=8, seed=21, interval="1s", fast_start=True, soak_cycles=40)
    _check_configured(r)
    s = r["soak"]
    assert s["cycles"] == 40, r["agent_log"][-3000:]
    assert s["addrs_ok"]
    assert s["last"]["fds"] == s["first"]["fds"] and s["last"]["threads"] == s["first"]["threads"], s
    if "ASAN_OPTIONS" not in os.environ:  # ASan's quarantine holds freed memory; LSan checks at exit
        assert s["last"]["rss_kib"] - s["first"]["rss_kib"] <= 256, s  # page-granular noise only
    assert s["withdraw_max_s"] < 1.0 and s["restore_max_s"] < 2.0, s
    assert r["agent_rc"] == 0


def test_verify_peers_asks_every_switch_port_over_arp():
    """--verify-peers on real veths: every NIC's switch-side /30 answers a who-has from the NIC's
    address; the status records the answer (and the port's MAC) and the node is ready."""
    r = netns.run_isolated(n_nics=8, seed=23, interval="1s", fast_start=True, extra_args=["--verify-peers=2s"])
    _check_configured(r)
    assert "verify_peers" in r["status"]["phases_ms"]
    for i in r["status"]["interfaces"]:
        assert i["peer_verified"] is True and i["peer_arp_ms"] < 1000 and i["peer_arp_mac"], i


def test_verify_peers_refuses_a_port_that_does_not_answer():
    """A switch port with the right Port Description that does not answer on that /30: without
    the check the node would be labelled; with it the agent fails and names the NIC."""
    r = netns.run_isolated(n_nics=4, seed=23, interval="1s", fast_start=True, extra_args=["--verify-peers=300ms"],
                           arp_silent_ports=1)
    assert not r["ready"] and r["agent_rc"] == 1
    silent = r["nics"][-1]
    assert f"({silent}: peer {r['plan'][-1]['peer']} did not answer ARP within 300ms" in r["agent_log"]
    assert r["label"] is None  # (the kubelet restarts the agent, which flushes and starts over)


def test_disable_fw_lldp_on_real_veths():
    """Real SIOCETHTOOL on veths: no private flags -> nothing changed, node still ready."""
    r = netns.run_isolated(n_nics=2, seed=19, interval="1s", fast_start=True,
                           extra_args=["--disable-fw-lldp", "--fw-lldp-priv-flag=lldp-offload=off"])
    _check_configured(r)
    assert [i["fw_lldp"] for i in r["status"]["interfaces"]] == ["no firmware LLDP flag"] * 2


def test_crash_restart_reconfigures_in_fast_start_time():
    """SIGKILL after readiness, then restart: stale label removed, node ready again quickly even
    though the switch still lists the dead agent as a neighbour (shutdown LLDPDU first).  Phase
    "zero" + 30 s interval: the switch's next periodic frame is ~25 s away at restart."""
    r = netns.run_isolated(n_nics=4, seed=20, interval="30s", phase="zero", fast_start=True, crash_restart=True,
                           crash_after_s=5.0)
    _check_configured(r)
    assert r["stale_label_after_crash"]
    assert r["restart_latency_s"] is not None and r["restart_latency_s"] < 3.0, r["restart_latency_s"]
    assert r["agent_rc"] == 0 and not r["label_after_sigterm"]


def test_crash_restart_without_shutdown_first_is_not_fast_started():
    """Control: same run without the shutdown LLDPDU — the switch still knows the neighbour, so
    no fast start, and nothing arrives within the 3 s wait."""
    r = netns.run_isolated(n_nics=2, seed=21, interval="30s", phase="zero", fast_start=True, crash_restart=True,
                           crash_after_s=5.0, wait="3s", extra_args=["--lldp-restart-fast=false"])
    assert r["stale_label_after_crash"]
    assert r["restart_latency_s"] is None


def test_lldp_cache_restart_against_a_switch_without_fast_start():
    """A switch that only sends periodic LLDP (no fast start, 10 s interval): a restarted agent
    without the cache waits for the next periodic frame; with --lldp-cache it configures from the
    last confirmed Port Descriptions at once, and the next periodic frame confirms them."""
    kw = dict(n_nics=2, seed=22, interval="10s", phase="zero", fast_start=False, crash_restart=True,
              crash_after_s=1.0)
    cached = netns.run_isolated(lldp_cache=True, **kw)
    _check_configured(cached)
    assert cached["restart_latency_s"] is not None and cached["restart_latency_s"] < 1.0, cached["restart_latency_s"]
    assert cached["restart_lldp_sources"] == ["cache", "cache"], cached["agent_log"]
    assert cached["cache_confirmed_s"] is not None, cached["agent_log"]
    ips = lambda j: [n["NIC_IP"] for n in j["NIC_NET_CONFIG"]]  # noqa: E731
    assert ips(cached["restart_rccl_net"]) == ips(cached["rccl_net"])
    assert cached["agent_rc"] == 0 and not cached["label_after_sigterm"]
    control = netns.run_isolated(**kw)
    assert control["restart_latency_s"] is not None and control["restart_latency_s"] > 5.0, control["restart_latency_s"]
    # A fast-start switch: the restarted agent still announces itself as a new neighbour, so the
    # switch's answer confirms the cache within about a second, not at its next periodic frame.
    fast = netns.run_isolated(lldp_cache=True, **dict(kw, fast_start=True, interval="30s"))
    assert fast["restart_lldp_sources"] == ["cache", "cache"], fast["agent_log"]
    assert fast["cache_confirmed_s"] is not None and fast["cache_confirmed_s"] < 2.0, fast["cache_confirmed_s"]


def test_two_nodes_l3_fabric_carries_a_collective():
    """BASELINE config "L3 mode, 2 nodes": two agents configure their nodes from one routing
    switch; a gloo all-reduce then runs node A <-> node B over the scale-out /30s and /16 routes."""
    from network_operator_amd.testing import twonode

    r = twonode.run_isolated_two_nodes(n_nics=2, seed=7)
    b = r["B"]
    assert r["A_ready_s"] is not None and b["ready_s"] is not None, r.get("A_agent_log")
    assert r["A_worker_rc"] == 0 and b["worker_rc"] == 0, (r.get("A_worker"), b.get("worker"))
    assert r["A_worker"]["ok"] and b["worker"]["ok"]
    # /16 via the switch port of every NIC, on both nodes.
    for routes, plan in ((r["A_routes"], r["plan"][:2]), (b["routes"], r["plan"][2:])):
        assert sorted(x["gateway"] for x in routes if x["dst"].endswith("/16")) == sorted(p["peer"] for p in plan)
    assert r["A_agent_rc"] == 0 and b["agent_rc"] == 0


def test_late_rocev2_gids_are_waited_for():
    """GIDs appear 300 ms after the agent starts (the RDMA core populates them asynchronously):
    the agent waits for them instead of writing rccl.env without NCCL_IB_GID_INDEX."""
    r = netns.run_isolated(n_nics=2, seed=22, interval="1s", gid_delay_s=0.3)
    _check_configured(r)
    assert "NCCL_IB_GID_INDEX=3" in r["rccl_env"]


def test_rail_tables_in_the_kernel():
    """--rail-table-base: one routing table per NIC (its /30 and its /16 via the switch port) and
    a source rule per NIC address in the real kernel; all removed on SIGTERM."""
    r = netns.run_isolated(n_nics=3, seed=23, interval="1s", fast_start=True, extra_args=["--rail-table-base=100"],
                           egress_probe=True)
    _check_configured(r)
    # the kernel's routing decision: datagrams from NIC k's address leave through NIC k only
    for k, row in enumerate(r["egress"]):
        # (a few stray frames — LLDP announces, IPv6 ND — can land anywhere)
        assert row[k] >= 20 and max(x for j, x in enumerate(row) if j != k) <= 5, r["egress"]
    rules = sorted(r["rules"], key=lambda x: x["priority"])
    assert [x["priority"] for x in rules] == [100, 101, 102], rules
    # Tagged (FRA_PROTOCOL) so cleanup can tell the agent's rules and routes from the host's.
    assert {x["protocol"] for x in rules} == {0xa3}, rules
    assert all(x["protocol"] == 0xa3 for t in r["rail_tables"].values() for x in t), r["rail_tables"]
    by_src = {x["src"]: x["table"] for x in rules}
    for nic, p in zip(r["nics"], r["plan"]):
        table = by_src[p["local"] + "/32"]
        routes = r["rail_tables"][str(table)]  # JSON object keys
        assert sorted(x["dst"] for x in routes) == sorted([p["p2p"], p["routed"]]), routes
        gw = [x for x in routes if x["gateway"]]
        assert len(gw) == 1 and gw[0]["gateway"] == p["peer"], routes
        assert all(x["ifindex"] == routes[0]["ifindex"] for x in routes)
    assert r["rules_after_sigterm"] == []


def test_without_rail_tables_sources_share_one_egress():
    """The reference's main-table-only routing: every NIC's /16 route has the same prefix and
    metric, so the kernel sends all off-link traffic through one NIC whatever the source
    address — the case --rail-table-base exists for."""
    r = netns.run_isolated(n_nics=3, seed=23, interval="1s", fast_start=True, egress_probe=True)
    _check_configured(r)
    busiest = [max(range(len(row)), key=row.__getitem__) for row in r["egress"]]
    assert len(set(busiest)) == 1 and all(row[busiest[0]] >= 20 for row in r["egress"]), r["egress"]


def test_networkmanager_unmanaged_while_ready_and_handed_back_on_sigterm():
    """--disable-networkmanager --nm-restore through a real dbus-daemon: the NICs are unmanaged
    (runtime Managed=false + the persistent keyfile) while the node is ready; SIGTERM removes the
    keyfile and hands the NICs back (opt-in; the reference leaves Managed=false behind,
    reference cmd/discover/main.go:143-159)."""
    from network_operator_amd.testing.fakedbus import BusDaemon

    if not BusDaemon.available():
        pytest.skip("dbus-daemon not installed")
    r = netns.run_isolated(n_nics=4, seed=5, interval="30s", fast_start=True, nm_bus=True)
    assert r["label"] and r["agent_rc"] == 0
    assert "unmanaged-devices+=" + ";".join(f"interface-name:{n}" for n in r["nics"]) in r["nm_keyfile_while_ready"]
    assert r["nm_managed_while_ready"] == {**{n: False for n in r["nics"]}, "eth9": True}
    assert r["nm_keyfile_after_sigterm"] is False
    assert r["nm_managed_after_sigterm"] == {**{n: True for n in r["nics"]}, "eth9": True}


def test_networkmanager_stays_off_the_nics_across_an_ordinary_restart():
    """Default (the DaemonSet's args): SIGTERM from a rolling update, drain or reboot leaves the
    keyfile and Managed=false, so NetworkManager cannot reclaim the scale-out NICs (and start DHCP
    on them) before the next agent runs."""
    from network_operator_amd.testing.fakedbus import BusDaemon

    if not BusDaemon.available():
        pytest.skip("dbus-daemon not installed")
    r = netns.run_isolated(n_nics=2, seed=6, interval="30s", fast_start=True, nm_bus=True, nm_restore=False)
    assert r["label"] and r["agent_rc"] == 0
    assert r["nm_keyfile_after_sigterm"] is True
    assert r["nm_managed_after_sigterm"] == {**{n: False for n in r["nics"]}, "eth9": True}


def test_rail_cabling_check_names_a_nic_on_another_rails_leaf():
    """railSwitchPattern: every rail has its own leaf ("leaf-r<k>"), and the NIC of GPU k must
    reach leaf k.  Correct cabling labels the node; a NIC cabled to rail 3's leaf instead of rail
    2's is left unconfigured, and the error names it, the switch and its port."""
    ok = netns.run_isolated(n_nics=4, seed=31, interval="1s", fast_start=True, switch_name="leaf-r{port}",
                            extra_args=["--rail-switch-pattern=leaf-r{rail}"])
    _check_configured(ok)
    bad = netns.run_isolated(n_nics=4, seed=31, interval="1s", fast_start=True, switch_name="leaf-r{port}",
                             port_switch_names={"swp2": "leaf-r3"}, extra_args=["--rail-switch-pattern=leaf-r{rail}"])
    assert not bad["ready"] and bad["agent_rc"] == 1
    nic = bad["nics"][2]
    err = [ln for ln in bad["agent_log"].splitlines() if ln.startswith("Error: ")][-1]
    assert err.startswith("Error: Not all interfaces were configured (3/4). Not configured: "
                          f"{nic}: rail 2 is cabled to switch 'leaf-r3' port 'swp2', not to one matching 'leaf-r2'"), err
    assert bad["state"][nic]["addrs"] == [] and all(bad["state"][n]["addrs"] for n in bad["nics"] if n != nic)


def test_min_link_speed_names_a_nic_that_came_up_slow():
    """minLinkSpeedGbps: on a 400G fabric one NIC negotiated 200G.  It is left unconfigured and
    named, with its speed in status.json; at full speed the node is labelled."""
    fast = netns.run_isolated(n_nics=4, seed=32, interval="1s", fast_start=True, nic_speeds_mbps=[400000] * 4,
                              extra_args=["--min-link-speed-gbps=400"])
    _check_configured(fast)
    slow = netns.run_isolated(n_nics=4, seed=32, interval="1s", fast_start=True,
                              nic_speeds_mbps=[400000, 200000, 400000, 400000], extra_args=["--min-link-speed-gbps=400"])
    assert not slow["ready"] and slow["agent_rc"] == 1
    nic = slow["nics"][1]
    err = [ln for ln in slow["agent_log"].splitlines() if ln.startswith("Error: ")][-1]
    assert f"Not configured: {nic}: link negotiated at 200 Gb/s, below the required 400 Gb/s" in err, err
    st = {i["name"]: i for i in slow["status"]["interfaces"]}
    assert st[nic]["speed_mbps"] == 200000 and st[slow["nics"][0]]["speed_mbps"] == 400000


def test_switch_without_jumbo_frames_is_caught_before_jobs_hang():
    """The switch ports advertise (LLDP 802.3 Maximum Frame Size) 1518-byte frames while the
    policy asks for MTU 9000: jumbo RoCE frames would be dropped.  Every NIC is refused with the
    numbers; with 9216-byte ports the node comes up."""
    ok = netns.run_isolated(n_nics=2, seed=33, interval="1s", fast_start=True, mtu=9000, switch_max_frame=9216)
    _check_configured(ok)
    assert all(i["peer_max_frame"] == 9216 for i in ok["status"]["interfaces"])
    bad = netns.run_isolated(n_nics=2, seed=33, interval="1s", fast_start=True, mtu=9000, switch_max_frame=1518)
    assert not bad["ready"] and bad["agent_rc"] == 1
    err = [ln for ln in bad["agent_log"].splitlines() if ln.startswith("Error: ")][-1]
    assert err.startswith("Error: Not all interfaces were configured (0/2). Not configured: "), err
    assert "its switch port accepts frames up to 1518 bytes, but MTU 9000 needs 9018" in err


@pytest.mark.parametrize("mgmt_bridge", [False, True])
def test_default_host_nic_policy_leaves_the_management_nic_and_the_gpu_rails_alone(mgmt_bridge):
    """The captured MI355X node, every NIC mlx5 with an RDMA device: a host-nic agent with the
    default driver list takes only the free host NIC.  The management NIC (address + default
    route) and the eight GPU rails (an amd-so agent's /30s, MTU 9000) are untouched while it runs
    and after it exits; naming the management NIC explicitly is refused.  Second case: the
    management address and default route are on a bridge and the NIC is its port (a kernel
    bridge; the same holds for a bond)."""
    r = netns.run_isolated(host_nic_ownership=True, mgmt_bridge=mgmt_bridge)
    via = " via br0" if mgmt_bridge else ""
    assert r["ready"], r["agent_log"]
    assert "host-nic-ready.nics=1" in r["label"]
    rails = r["rails"]
    assert len(rails) == 8
    # The discovery view (no netlink): the rails are left out as the GPUs' NICs.
    assert sorted(r["discovery"]["ifnames"]) == [netns.HOST_NIC, netns.MGMT_NIC]
    assert sorted(r["discovery"]["excluded"]) == sorted(rails)
    assert all("scale-out rail of GPU" in why for why in r["discovery"]["excluded"].values())
    # The agent's view: the management NIC left out too, for its default route.
    assert [i["name"] for i in r["status"]["interfaces"]] == [netns.HOST_NIC]
    assert f"{netns.MGMT_NIC}: the node's own NIC: it carries the node's default route{via}" in r["status"]["excluded"]
    for phase in ("while_ready", "after_sigterm"):
        for nif in rails + [netns.MGMT_NIC]:
            assert r[phase][nif] == r["before"][nif], (phase, nif, r[phase][nif], r["before"][nif])
        assert r[phase]["default_routes"] == r["before"]["default_routes"]
    assert r["while_ready"][netns.HOST_NIC] == {"up": True, "mtu": 9000, "addrs": [], "master": 0}
    assert r["after_sigterm"][netns.HOST_NIC]["up"] is False  # restored to its original state
    assert r["after_sigterm"][netns.HOST_NIC]["mtu"] == 1500  # --restore-mtu (the operator passes it for host-nic)
    assert r["mtu_state_left"] is False  # every MTU went back: the record goes with the agent
    assert r["agent_rc"] == 0
    named = r["named_mgmt"]
    assert named["rc"] == 1 and f"Refusing to configure {netns.MGMT_NIC}{via}: the node's default route" in named["stderr"]
    assert (r["before"][netns.MGMT_NIC]["master"] != 0) == mgmt_bridge
    assert named["after"] == r["before"][netns.MGMT_NIC]


def test_host_nic_policy_with_include_gpu_rails_takes_the_rails_but_never_the_management_nic():
    """hostNic.includeGpuRails (a node without an amd-so policy): the host-nic agent takes the
    eight rails and the free host NIC; the management NIC (default route) is still the node's."""
    r = netns.run_isolated(host_nic_ownership=True, include_gpu_rails=True)
    assert r["ready"], r["agent_log"]
    rails = r["rails"]
    assert sorted(i["name"] for i in r["status"]["interfaces"]) == sorted(rails + [netns.HOST_NIC])
    assert "host-nic-ready.nics=9" in r["label"]
    assert f"{netns.MGMT_NIC}: the node's own NIC: it carries the node's default route" in r["status"]["excluded"]
    for nif in rails:
        assert r["while_ready"][nif]["mtu"] == 9000 and r["while_ready"][nif]["addrs"] == []  # L2: taken, flushed
    assert r["while_ready"][netns.MGMT_NIC] == r["before"][netns.MGMT_NIC]


def test_l2_waits_for_carrier_on_every_nic_before_the_label():
    """L2 on real veths with one switch port down (an unplugged cable): admin-up is not a link.
    No label; the reason names the NIC in status.json and the readiness probe's output; the port
    comes up and the monitor publishes the label (the reference labels right after link-up,
    reference cmd/discover/main.go:198-206,239-246)."""
    r = netns.run_isolated(n_nics=3, seed=41, mode="L2", interval="1s", dark_port=1,
                           extra_args=["--carrier-wait=300ms"])
    d = r["dark"]
    dark_nic = r["nics"][1]
    assert d["reason_s"] is not None, r["agent_log"]
    assert d["label_while_dark"] is False
    assert d["reason"] == f"{dark_nic}: no carrier (check the cable, the switch port and the optic)\n"
    assert d["status_ready"] is False and d["status_no_carrier"] == [dark_nic]
    assert d["ready_check"]["rc"] == 1 and dark_nic + ": no carrier" in d["ready_check"]["stdout"]
    assert r["ready"] and d["port_up_to_label_s"] is not None and d["port_up_to_label_s"] < 2.0, r["agent_log"]
    assert "gpu-scale-out.nics=3" in r["label"]
    assert f"Interface '{dark_nic}' has carrier now" in r["agent_log"]
    for nic in r["nics"]:
        assert r["state"][nic]["up"] and r["state"][nic]["addrs"] == []
    assert r["agent_rc"] == 0


def test_l2_link_still_training_is_start_up_not_no_carrier():
    """a 200/400G optic commonly trains for 5-15 s.  The switch port comes
    up 5 s after the agent started; with the default --carrier-wait (30 s) the agent reports
    "waiting for carrier" meanwhile (a start-up reason for the operator), never "no carrier",
    and publishes the label milliseconds after the carrier arrives.  (The 3 s --link-wait is the
    netlink echo wait, reference cmd/discover/network.go:242-283, not a carrier wait.)"""
    r = netns.run_isolated(n_nics=3, seed=43, mode="L2", interval="1s", dark_port=1, dark_port_up_after=5.0)
    d = r["dark"]
    dark_nic = r["nics"][1]
    assert d["port_up_s"] >= 5.0 and d["label_while_dark"] is False, r["agent_log"]
    assert d["reasons_seen"] == [f"{dark_nic}: waiting for carrier\n"], d["reasons_seen"]
    assert d["status_flags_seen"] == [f"{dark_nic}:awaiting_carrier"], d["status_flags_seen"]
    assert r["ready"] and d["port_up_to_label_s"] is not None and d["port_up_to_label_s"] < 0.5, r["agent_log"]
    assert "no carrier" not in r["agent_log"]
    assert f"Interface '{dark_nic}' has carrier after" in r["agent_log"]
    assert r["agent_rc"] == 0


def test_host_nic_policy_with_nothing_of_its_own_idles_with_one_reason():
    """a default host-nic policy on a node whose RDMA NICs are all taken --
    the rails by amd-so, the management NIC (default route) and the storage NIC (its /24) by the
    node.  The agent configures nothing, publishes no label, stays up (no crash loop) and says
    why in status.json and through --ready-check.  (The reference exits for "no interfaces",
    reference cmd/discover/main.go:171-179; for amd-so that stays a failure.)"""
    r = netns.run_isolated(host_nic_ownership=True, host_nic_addr="10.9.8.7/24")
    idle = r["idle"]
    assert idle["reason_s"] and idle["running"] and not idle["label"], r["agent_log"]
    assert idle["reason"].startswith("no host NIC of its own (left alone: "), idle["reason"]
    assert f"{netns.MGMT_NIC}: the node's own NIC: it carries the node's default route" in idle["reason"]
    assert f"{netns.HOST_NIC}: the node's own NIC" in idle["reason"]
    assert idle["ready_check"]["rc"] == 1 and "no host NIC of its own" in idle["ready_check"]["stdout"]
    assert r["ready"] is False and r["status"]["ready"] is False and r["status"]["interfaces"] == []
    assert f"{netns.MGMT_NIC}: the node's own NIC" in r["status"]["excluded"]
    for nif in r["rails"] + [netns.MGMT_NIC, netns.HOST_NIC]:  # nothing touched, before or after SIGTERM
        assert r["while_ready"][nif] == r["before"][nif] and r["after_sigterm"][nif] == r["before"][nif], nif
    assert r["agent_rc"] == 0  # SIGTERM ends the wait cleanly


def test_per_nic_policy_routing_default_is_not_the_node_uplink():
    """a default route in a per-NIC source-routing table (reached only by
    ``from <subnet> lookup 1001``) is not the main table's uplink.  ADVICE r5 (medium): but the NIC
    holding the address that rule selects (192.168.50.10/24) is how the node reaches that network:
    on a real kernel the agent refuses it (dry run: named as refused; real start: nothing touched)
    unless --allow-policy-routed, and takes a rail whose policy table serves only its own /30,
    with a warning.  The NIC with the main table's default route is refused either way."""
    r = netns.run_isolated(policy_routing_uplink=True)
    assert r["default_route_links"] == [r["mgmt"]], r
    assert any(x["table"] == 1001 and x["selective"] for x in r["rules"]), r["rules"]
    assert [x["table"] for x in r["table_1001"]] == [1001]  # table ids above 255 are kept
    assert r["dry_rail"]["rc"] == 0 and r["dry_rail"]["status"]["interfaces"][0]["name"] == "rail0", r["dry_rail"]
    assert ("rail0: carries a default route in policy-routing table 1001 and the node's address 192.168.50.10/24, the "
            "source its rule 'from 192.168.50.0/24 lookup 1001' selects (refused)") in r["dry_rail"]["status"]["excluded"]
    assert "mgmt0: carries the node's default route (refused)" in r["dry_mgmt"]["status"]["excluded"], r["dry_mgmt"]
    refused = r["configure_rail_refused"]
    assert refused["rc"] == 1 and "Refusing to configure rail0 (a default route in policy-routing table 1001" in \
        refused["stderr"], refused
    assert refused["mtu"] == 1500 and refused["addrs"] == ["192.168.50.10/24"], refused
    own = r["configure_own_rail"]
    assert own["rc"] == 0 and own["mtu"] == 9000, own
    assert "Interface 'rail1' has a default route in routing table 1002, which only selective rules reach" in own["stderr"]
    cr = r["configure_rail"]
    assert cr["rc"] == 0 and cr["mtu"] == 9000, cr
    assert "Interface 'rail0' has a default route in routing table 1001, which only selective rules reach" in cr["stderr"]
    cm = r["configure_mgmt"]
    assert cm["rc"] == 1 and "Refusing to configure mgmt0: the node's default route" in cm["stderr"]
    assert cm["mtu"] == 1500 and cm["addrs"] == ["10.0.0.5/24"], cm


def test_idle_host_nic_agent_exits_when_a_nic_of_its_own_appears():
    """The idle host-nic agent looks again every --rediscover-interval: once the node gives the
    storage NIC up (its address removed), the agent exits 0 within about one interval, so that
    its restart (restartPolicy Always) configures the NIC instead of idling forever."""
    r = netns.run_isolated(host_nic_ownership=True, host_nic_addr="10.9.8.7/24", free_host_nic=True)
    idle = r["idle"]
    assert idle["running"] and idle["reason"].startswith("no host NIC of its own"), r["agent_log"]
    after = idle["after_free"]
    assert after["exited"] and after["rc"] == 0 and after["seconds"] < 2.0, (after, r["agent_log"])
    assert f"Interface(s) of its own appeared: {netns.HOST_NIC}" in r["agent_log"]


def test_l3_reports_waiting_for_carrier_while_a_port_trains():
    """L3: a switch port that comes up 2 s after the agent started.  While it trains, the probe's
    reason for that NIC is "waiting for carrier" (no frame can come yet), a start-up reason like
    "waiting for LLDP"; once the carrier is there the switch answers and the label follows."""
    r = netns.run_isolated(n_nics=2, seed=44, mode="L3", interval="30s", dark_port=1, dark_port_up_after=2.0)
    d = r["dark"]
    dark_nic = r["nics"][1]
    assert any(f"{dark_nic}: waiting for carrier" in x for x in d["reasons_seen"]), (d["reasons_seen"], r["agent_log"])
    assert not any("no carrier" in x for x in d["reasons_seen"])
    assert r["ready"] and d["port_up_to_label_s"] is not None and d["port_up_to_label_s"] < 1.5, r["agent_log"]


def test_agent_killed_part_way_through_configuring_converges_on_restart():
    """SIGKILL (OOM kill, crash) after 1, 2, then 3 of 4 NICs are configured, rail tables on,
    each time restarted over what the dead agent left: the last start reaches exactly the state
    of a clean bring-up -- one address, one /30 and one /16 per NIC, one source rule and two
    table routes per rail, nothing doubled -- and SIGTERM still removes all of it, links included.  The switch
    sends periodic frames only, at a random phase per port, so the NICs configure one by one."""
    r = netns.run_isolated(n_nics=4, seed=31, interval="1s", phase="random", fast_start=False,
                           kill_mid_config=3, extra_args=["--rail-table-base=100"])
    _check_configured(r)
    kills = r["mid_config_kills"]
    assert [k["wanted"] for k in kills] == [1, 2, 3], kills
    assert not any(k["label"] for k in kills), kills
    assert any(0 < k["nics_with_address"] < 4 for k in kills), kills
    for nic in r["nics"]:
        keys = [(x["dst"], x["gateway"]) for x in r["state"][nic]["routes"]]
        assert len(keys) == len(set(keys)) == 2, keys
    rules = r["rules"]
    assert sorted(x["priority"] for x in rules) == [100, 101, 102, 103], rules
    assert sorted(x["src"] for x in rules) == sorted(p["local"] + "/32" for p in r["plan"]), rules
    for table, routes in r["rail_tables"].items():
        assert len(routes) == 2, (table, routes)
    assert r["agent_rc"] == 0 and not r["label_after_sigterm"] and r["rules_after_sigterm"] == []
    # Down again, as before the first agent: the restarted agent found them up, and only the
    # --link-state record (the operator passes it) says otherwise.  The record goes with them.
    for nic in r["nics"]:
        assert r["after_sigterm"][nic] == {"up": False, "addrs": []}
    assert not r["link_state_left"]


@pytest.mark.parametrize("driver,prefix", [("ionic", "ionic_"), ("bnxt_en", "bnxt_re")])
def test_pollara_and_thor_rails_configure_like_connectx(driver, prefix):
    """The scale-out NICs of MI355X platforms are often AMD Pollara 400 (ionic) or Broadcom Thor
    (bnxt_en) rather than ConnectX: the same L3 bring-up, with RCCL told about their RDMA devices
    (NCCL_IB_HCA in GPU order, RDMA_DEV per rail).  The host NICs stay mlx5 and are left alone."""
    r = netns.run_isolated(n_nics=4, seed=41, interval="30s", fast_start=True, rail_driver=driver)
    _check_configured(r, rdma_prefix=prefix)
    hca = [l for l in r["rccl_env"].splitlines() if l.startswith("NCCL_IB_HCA=")]
    by_gpu = sorted(r["rccl_net"]["NIC_NET_CONFIG"], key=lambda e: e["GPU_INDEX"])
    assert hca == ["NCCL_IB_HCA==" + ",".join(f"{e['RDMA_DEV']}:1" for e in by_gpu)], (hca, by_gpu)
    assert "mlx5_" not in hca[0]


def test_an_xgmi_link_down_keeps_the_node_unlabelled_and_a_drop_withdraws_the_label():
    """The xGMI check reads each GPU's trained link state from amdgpu's gpu_metrics (the layout
    captured on a live MI355X).  A link already down at start fails the check and names the GPU
    and the link; a link that drops after readiness withdraws the label with that reason until it
    is back.  (KFD's topology, the mesh check, lists the link either way.)"""
    # With the monitor (the DaemonSet's agent): configured, unlabelled with the reason, labelled
    # when the link is back.  Without it, the start fails and names the link.
    r = netns.run_isolated(n_nics=2, seed=43, interval="30s", fast_start=True, xgmi_down_at_start=(1, 3),
                           xgmi_up_after=1.0, extra_args=["--xgmi-health-interval=100ms"])
    _check_configured(r)
    d = r["dark"]
    assert not d["label_while_down"] and any("xGMI: GPU 0000:23:00.0: link 3 down" in w for w in d["reasons_seen"]), d
    assert d["link_up_to_label_s"] is not None and d["link_up_to_label_s"] < 3.0, d
    r = netns.run_isolated(n_nics=2, seed=43, interval="30s", fast_start=True, xgmi_down_at_start=(1, 3), wait="5s",
                           extra_args=["--monitor=false"])
    assert not r["ready"] and r["agent_rc"] != 0
    assert "xGMI: GPU 0000:23:00.0: link 3 down" in r["agent_log"], r["agent_log"][-2000:]
    r = netns.run_isolated(n_nics=2, seed=44, interval="30s", fast_start=True, xgmi_link_flap=(0, 5),
                           extra_args=["--xgmi-health-interval=100ms"])
    _check_configured(r)
    assert r["status"]["xgmi_links"] == "14 up, 0 down on 2 GPUs, x16 at 38 Gb/s (gpu_metrics)", r["status"]
    f = r["xgmi_flap"]
    assert f["withdraw_s"] is not None and f["withdraw_s"] < 3.0, f
    assert f["reason"] and "xGMI: GPU 0000:0a:00.0: link 5 down" in f["reason"], f
    assert f["restore_s"] is not None and f["restore_s"] < 3.0, f
    assert r["agent_rc"] == 0


def test_a_rail_whose_pcie_link_trained_narrow_is_reported_and_with_require_full_pcie_not_labelled():
    """A NIC (or its GPU) whose PCIe link trained below what it supports moves RDMA at a fraction
    of the rail's rate.  The agent reports the link of every NIC and its GPU (status.json
    ``pcie`` / ``gpu_pcie``, ``netop_agent_nic_pcie_degraded``); with --require-full-pcie such a
    rail is not configured and the node stays unlabelled, naming it.  A GPU's link speed alone
    may drop while the GPU idles, so only its width counts."""
    r = netns.run_isolated(n_nics=2, seed=45, interval="30s", fast_start=True,
                           pcie_degraded={1: (16.0, 8), "gpu0": (2.5, 16)})
    _check_configured(r)
    st = {i["name"]: i for i in r["status"]["interfaces"]}
    assert st[r["nics"][0]]["pcie"] == "32.0 GT/s x16" and st[r["nics"][1]]["pcie"] == "16.0 GT/s x8 of 32.0 GT/s x16"
    assert st[r["nics"][0]]["gpu_pcie"] == "2.5 GT/s x16 of 32.0 GT/s x16"
    r = netns.run_isolated(n_nics=2, seed=45, interval="30s", fast_start=True, wait="3s",
                           pcie_degraded={1: (16.0, 8), "gpu0": (2.5, 16)}, extra_args=["--require-full-pcie"])
    assert not r["ready"]
    why = r["status_at_exit"]["interfaces"]
    assert "its PCIe link trained at 16.0 GT/s x8 of 32.0 GT/s x16" in why[1].get("config_error", ""), why
    assert not why[0].get("config_error"), why  # the idle GPU's lower speed alone is not a fault
    # A rail that retrains narrower after readiness (PCIe errors, a reset): the monitor withdraws
    # the label with the reason and restores it when the link is back at x16.
    r = netns.run_isolated(n_nics=2, seed=46, interval="30s", fast_start=True, pcie_flap=0,
                           extra_args=["--require-full-pcie", "--xgmi-health-interval=100ms"])
    _check_configured(r)
    f = r["pcie_flap"]
    assert f["withdraw_s"] is not None and f["withdraw_s"] < 3.0, f
    assert f["reason"] and "its PCIe link trained at 16.0 GT/s x8 of 32.0 GT/s x16" in f["reason"], f
    assert f["restore_s"] is not None and f["restore_s"] < 3.0, f


def test_rails_without_rdma_devices_stay_unlabelled_until_the_rdma_driver_loads():
    """scale-out ready means RDMA ready.  Rails whose NIC has no RDMA device (the
    Pollara boxes of this pool: ionic without ionic_rdma) are configured, but the agent keeps the
    label and rccl.env back and says "waiting for RDMA device" (a start-up reason).  When the RDMA
    driver registers the devices (fakesysfs bind), the label follows within a second and rccl.env
    names every rail's HCA."""
    r = netns.run_isolated(n_nics=4, seed=51, interval="30s", fast_start=True, rail_driver="ionic",
                           rails_without_rdma=4, rdma_bind_after=2.0)  # --require-rdma: the operator's default
    d = r["dark"]
    assert d["running_while_missing"] and not d["label_while_missing"] and not d["rccl_env_while_missing"], d
    assert sorted(d["configured_while_missing"]) == sorted(r["nics"]), d
    want = "; ".join(f"{n}: waiting for RDMA device" for n in r["nics"]) + "\n"
    assert want in d["reasons_seen"], d["reasons_seen"]
    assert d["bind_to_label_s"] is not None and d["bind_to_label_s"] < 1.0, d
    _check_configured(r, rdma_prefix="ionic_")
    hca = [l for l in r["rccl_env"].splitlines() if l.startswith("NCCL_IB_HCA=")]
    assert len(hca) == 1 and hca[0].count("ionic_") == 4, r["rccl_env"]
    # Without --require-rdma (requireRdma: false): the reference's behaviour, labelled at once.
    r = netns.run_isolated(n_nics=2, seed=52, interval="30s", fast_start=True, rail_driver="ionic", rails_without_rdma=2,
                           require_rdma=False)
    assert r["ready"] and "NCCL_IB_HCA" not in r["rccl_env"], r["rccl_env"]


def test_a_flapping_port_withdraws_the_label_once_and_republishes_it_after_the_holddown():
    """ten flaps in five seconds withdraw the label once; it comes back once, the
    hold-down after the last flap (not ten withdrawals and republications)."""
    r = netns.run_isolated(n_nics=2, seed=53, interval="30s", fast_start=True, label_holddown="2s",
                           flap_burst=(0, 10, 0.5))
    assert r["ready"]
    f = r["flap_burst"]
    assert f["withdrawals"] == 1 and f["publishes"] == 1, f
    # (timed from when the harness's port-up call returned; the agent sees the carrier a little
    # earlier, so the 2 s hold-down can end a few ms before "2.0")
    assert 1.9 <= f["last_up_to_label_s"] < 3.0, f
    assert any("label hold-down" in x or "link down" in x for x in f["reasons"]), f


def test_a_stalled_gpu_metrics_read_neither_holds_back_link_events_nor_hides_its_reason():
    """the monitor reads gpu_metrics on a worker.  While GPU 0's read is stalled (a
    FIFO nobody writes: a wedged SMU), carrier losses still withdraw the label within milliseconds,
    as fast as with no read stalled; once the read times out the reason names the GPU and the
    label stays off; when the SMU answers again the label comes back."""
    r = netns.run_isolated(n_nics=2, seed=54, interval="30s", fast_start=True, gpu_metrics_stall=True,
                           sysfs_read_timeout="3s", extra_args=["--xgmi-health-interval=100ms"])
    assert r["ready"]
    s = r["gpu_metrics_stall"]
    # Under 10 ms on a quiet machine (~2 ms here); on a loaded one (the suite runs -n 8) no slower
    # than twice the same carrier losses with no read stalled.  A loop blocked behind the read
    # would take the whole 3 s timeout.
    assert None not in s["withdraw_during_stall_s"], s
    assert s["withdraw_during_stall_p50_s"] < max(0.010, 2 * s["withdraw_without_stall_p50_s"]), s
    assert s["stall_to_reason_s"] is not None and s["stall_to_reason_s"] > s["flaps_done_s"], s  # stalled throughout
    assert s["reason"] and "gpu_metrics of 0000:0a:00.0 did not answer in 3s" in s["reason"], s
    assert not s["label_while_stalled"], s
    assert s["answer_to_label_s"] is not None and s["answer_to_label_s"] < 3.0, s


def test_an_l2_rail_left_unconfigured_for_its_pcie_link_is_configured_when_the_link_retrains():
    """with --require-full-pcie, an L2 rail whose PCIe link trained at x8 is left
    unconfigured at start and the node unlabelled.  With the monitor the L2 agent never exits, so
    no restart would re-check it: the monitor's PCIe sample does, and once the link is back at
    32 GT/s x16 the NIC is configured and the node labelled.  (L3 fails the start instead, and the
    kubelet's restart re-checks.)"""
    r = netns.run_isolated(n_nics=2, seed=47, interval="30s", fast_start=True, mode="L2", wait="5s",
                           pcie_degraded={1: (16.0, 8)}, pcie_restored_after=1.5,
                           extra_args=["--require-full-pcie", "--xgmi-health-interval=100ms"])
    d = r["dark"]
    assert d["running_while_narrow"] and not d["label_while_narrow"], d
    assert any("its PCIe link trained at 16.0 GT/s x8 of 32.0 GT/s x16" in w for w in d["reasons_seen"]), d
    assert d["restore_to_label_s"] is not None and d["restore_to_label_s"] < 2.0, d
    assert r["ready"] and r["agent_rc"] == 0, r["agent_log"][-2000:]
