"""Whole-system run: operator + fake API server + simulated node + real agent + synthetic switch.

The chain a user starts with ``kubectl apply`` of a NetworkClusterPolicy, end to end, in one
private user+network namespace:

    policy created --(operator: watch, reconcile)--> DaemonSet --(fake API: DS controller)--> Pod
    --(nodesim kubelet)--> discover (real binary, veth NICs, fake MI355X sysfs) --LLDP--> switch
    --> NICs addressed, RCCL artifacts, features.d label --(nodesim NFD)--> Node label
    --(readinessProbe: discover --ready-check)--> Pod Ready --> DaemonSet numberReady
    --(operator)--> policy status "All good"

and back on deletion: policy deleted --(garbage collector)--> DaemonSet, Pod --> agent SIGTERM
--> addresses and label removed --> Node label gone.

``config_type="host-nic"`` runs BASELINE.json configs[4]: the node's two host NICs have no
driver bound until the policy's driver container (KMD install, an init container mapped to a
command that binds them in the fake sysfs) has run; the agent then discovers them as RDMA NICs
of the ``ionic`` driver and publishes the host-nic label.

Measured from the moment the policy is created: the DaemonSet, the agent's start, the Node
label (scale-out readiness as a job scheduler sees it), and the policy's ``All good``.  This
is the control-plane-inclusive version of the node-ready metric; ``netns.py`` measures the agent
alone.  BASELINE.json configs[0] ("L2 mode on kind/envtest with fake LLDP frames over veth
pairs") and the L3 equivalent.
"""

from __future__ import annotations

import argparse
import asyncio
import json
import os
import random
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path
from typing import Optional

from . import fakesysfs, netns

READY_LABEL = "amd.feature.node.kubernetes.io/gpu-scale-out"
HOST_NIC_READY_LABEL = "amd.feature.node.kubernetes.io/host-nic-ready"
# host-nic scenario: the two management-side NICs of the fixture node, driverless until the
# driver container (the KMD install of BASELINE.json configs[4]) binds them.
HOST_NICS = ("ens9np0", "ens49np1")
KMD_IMAGE = "example.com/amd/ionic-kmd:1.0"
# amd-so driverImage: the rails' RDMA driver (ionic_rdma on Pollara), simulated by fakesysfs bind-rdma
RDMA_KMD_IMAGE = "example.com/amd/ionic-rdma-kmd:1.0"
KMD_DRIVER = "ionic"
VALIDATED_LABEL = "amd.feature.node.kubernetes.io/gpu-fabric-validated"
# Stand-in for the validation image on a CPU-only harness: what validate.py does with its verdict
# (the label file through NFD on success, exit status = result).  validate.py itself runs on the
# MI355X box (tests/test_gpu_ops.py); here the Job plumbing around it is under test.
_VALIDATE_STUB = (
    "import sys, pathlib\n"
    "ok = sys.argv[1] == 'pass'\n"
    "d = [a.split('=', 1)[1] for a in sys.argv[2:] if a.startswith('--nfd-features-dir=')][0]\n"
    "if ok:\n"
    "    pathlib.Path(d, 'gpu-fabric-validation.txt').write_text("
    "'amd.feature.node.kubernetes.io/gpu-fabric-validated=true\\n')\n"
    "sys.exit(0 if ok else 1)\n")


async def _until(fn, timeout: float, poll: float = 0.001) -> Optional[float]:
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if fn():
            return time.monotonic()
        await asyncio.sleep(poll)
    return None


async def _edit(c, res, name: str, change, attempts: int = 50) -> dict:
    """kubectl edit: get, change, replace, again on a conflict (the operator writes the status
    and its finalizer concurrently)."""
    from ..operator.kube import ApiError

    for _ in range(attempts):
        cur = await c.get(res, name)
        change(cur)
        try:
            return await c.replace(res, cur)
        except ApiError as e:
            if e.status != 409:
                raise
            await asyncio.sleep(0.01)
    raise RuntimeError(f"edit of {name} kept conflicting")


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


async def _scrape(port: int, names) -> dict:
    """The operator's own /metrics (plain HTTP: no --metrics-secure here), selected series."""
    import aiohttp

    out: dict = {}
    async with aiohttp.ClientSession() as s:
        async with s.get(f"http://127.0.0.1:{port}/metrics") as r:
            text = await r.text()
    for line in text.splitlines():
        for n in names:
            if line.startswith(n + "{") or line.startswith(n + " "):
                out[line.rsplit(" ", 1)[0]] = float(line.rsplit(" ", 1)[1])
    return out


# HA run: lease timings short enough for a test (controller-runtime's are 15 s / 10 s / 2 s), with
# the stop margin the flag check requires (lease - renew > leader.STOP_BUDGET_S).
_LEASE_ARGS = ("--leader-elect-lease-duration=3", "--leader-elect-renew-deadline=1.5",
               "--leader-elect-retry-period=0.25")


def _port_open(port: int) -> bool:
    import socket

    with socket.socket() as s:
        s.settimeout(0.2)
        return s.connect_ex(("127.0.0.1", port)) == 0


def _lease_holder(fake, ns: str) -> str:
    from ..operator import kube
    from ..operator.leader import DEFAULT_LEASE_ID

    return ((fake.get_object(kube.LEASES, DEFAULT_LEASE_ID, ns) or {}).get("spec") or {}).get("holderIdentity") or ""


async def _start_replicas(tmp: Path, url: str, ns: str, n: int = 2) -> list:
    """The operator Deployment with ``replicas: n``: separate processes (so the leader can be
    SIGKILLed), ``--leader-elect``, webhooks on with one serving certificate (the Secret that
    cert-manager issues, mounted in every pod)."""
    from ..operator.servers import generate_self_signed

    generate_self_signed(tmp / "certs")
    root = Path(__file__).resolve().parents[2]
    out = []
    for i in range(n):
        r = {"name": f"operator-{chr(ord('a') + i)}", "webhook": _free_port(), "metrics": _free_port()}
        r["log"] = tmp / f"{r['name']}.log"
        env = dict(os.environ, ENABLE_WEBHOOKS="true", OPERATOR_NAMESPACE=ns, POD_NAME=r["name"],
                   PYTHONPATH=str(root))
        with open(r["log"], "wb") as logf:
            r["proc"] = await asyncio.create_subprocess_exec(
                sys.executable, "-m", "network_operator_amd.operator", "--master", url, "--leader-elect",
                *_LEASE_ARGS, f"--webhook-port={r['webhook']}", f"--webhook-cert-dir={tmp / 'certs'}",
                "--health-probe-bind-address=0", f"--metrics-bind-address=127.0.0.1:{r['metrics']}",
                "--dependency-check-interval=0", env=env, stdout=asyncio.subprocess.DEVNULL, stderr=logf)
        out.append(r)
    return out


async def _stop_replicas(replicas: list) -> list:
    rcs = []
    for r in replicas:
        p = r["proc"]
        if p.returncode is None:
            p.terminate()
            try:
                await asyncio.wait_for(p.wait(), 20)
            except asyncio.TimeoutError:  # pragma: no cover
                p.kill()
                await p.wait()
        rcs.append(p.returncode)
    return rcs


async def _register_webhooks(fake, c, tmp: Path, ns: str, replica: dict) -> dict:
    """What the kustomize tree installs for admission: the webhook Service and the two
    configurations exactly as packaged (service-routed, plural resource), the CA bundle filled
    in as cert-manager's CA injector does, and the Service's endpoint the first replica's pod
    (set once it serves, as the endpoints controller would)."""
    import base64

    from ..operator import kube
    from ..packaging import manifests as M

    ca = base64.b64encode((tmp / "certs" / "tls.crt").read_bytes()).decode()
    svc, names = "", []
    for o in M.finalize([M.webhook_service(), *M.webhook_configurations()], ns):
        if o["kind"] == "Service":
            await c.create(kube.SERVICES, o, namespace=ns)
            svc = o["metadata"]["name"]
            continue
        for wh in o["webhooks"]:
            wh["clientConfig"]["caBundle"] = ca
        await c.create(kube.MUTATINGWEBHOOKS if o["kind"].startswith("Mutating") else kube.VALIDATINGWEBHOOKS, o)
        names.append(o["metadata"]["name"])
    assert await _until(lambda: _port_open(replica["webhook"]), 30, poll=0.05), f"{replica['name']} not serving"
    fake.service_endpoints[(ns, svc)] = f"https://127.0.0.1:{replica['webhook']}"
    return {"service": svc, "configurations": names, "endpoint": replica["name"]}


async def _ha_checks(fake, c, rt, node, replicas: list, ns: str, name: str, mode: str, nic_names: list,
                     label_key: str, all_good, new_mtu: int) -> dict:
    """Admission and fail-over with the node already ready: the stored policy was defaulted by
    the mutating webhook, an invalid one is refused by the validating webhook; then the leader
    is SIGKILLed (no lease release), the policy is edited, and the standby must take the lease
    and roll the edit out to the node."""
    from ..api.v1alpha1 import types as T
    from ..operator import kube
    from ..operator.kube import ApiError
    from ..operator.leader import DEFAULT_LEASE_ID

    P = kube.NETWORKCLUSTERPOLICIES
    out: dict = {"admission_calls": len(fake.admission_calls)}
    out["defaulted_image"] = ((fake.get_object(P, name) or {}).get("spec") or {}).get("amdScaleOut", {}).get("image")
    try:
        await c.create(P, T.new_policy("bad", layer=mode, node_selector={"foo.com": "_bar"}).to_dict())
        out["bad_policy"] = "admitted"
    except ApiError as e:
        out["bad_policy"] = {"status": e.status, "message": e.message}
    holder = _lease_holder(fake, ns)
    leader = next(r for r in replicas if holder.startswith(r["name"] + "_"))
    standby = next(r for r in replicas if r is not leader)
    t1 = time.monotonic()
    leader["proc"].kill()
    await leader["proc"].wait()
    for k in list(fake.service_endpoints):  # the endpoints controller drops the dead pod
        fake.service_endpoints[k] = f"https://127.0.0.1:{standby['webhook']}"
    gen = (await _edit(c, P, name, lambda cur: cur["spec"]["amdScaleOut"].update(mtu=new_mtu)))["metadata"]["generation"]
    t_lead = await _until(lambda: _lease_holder(fake, ns).startswith(standby["name"] + "_"), 30)
    t_mtu = await _until(lambda: all(rt.link_by_name(n)["mtu"] == new_mtu for n in nic_names), 30)

    def rolled_out():
        st = (fake.get_object(P, name) or {}).get("status") or {}
        return (st.get("observedGeneration") == gen and all_good()
                and node.node_labels().get(label_key) == "true")
    t_ready = await _until(rolled_out, 30)
    rel = lambda t: round(t - t1, 6) if t else None  # noqa: E731
    lease = fake.get_object(kube.LEASES, DEFAULT_LEASE_ID, ns) or {}
    out["failover"] = {"killed": leader["name"], "new_leader": _lease_holder(fake, ns).split("_")[0],
                       "lease_transitions": (lease.get("spec") or {}).get("leaseTransitions"),
                       "kill_to_new_leader_s": rel(t_lead), "kill_to_mtu_applied_s": rel(t_mtu),
                       "kill_to_ready_again_s": rel(t_ready), "generation": gen,
                       "admission_calls": len(fake.admission_calls)}
    return out


async def _scenario(tmp: Path, n_nics: int, mode: str, seed: int, interval: str, fast_start: bool,
                    teardown: bool, node_name: str, policy_kw: dict, update_mtu: int, config_type: str,
                    flap: bool, validation: str, crash_agent: bool, driver_reload: bool, ha: bool,
                    silent_nics: int = 0, lldp_wait: str = "", duplicate_policy: bool = False,
                    dark_port_s: float = 0.0, host_nics_owned: bool = False, pcie_narrow_nic: int = -1,
                    xgmi_link_down: bool = False, rdma: str = "", flap_burst: int = 0) -> dict:
    from ..api.v1alpha1 import types as T
    from ..operator import kube, manager
    from ..operator.kube import ApiClient, KubeConfig
    from .fakeapi import FakeApiServer
    from .nodesim import SimNode

    rng = random.Random(seed)
    rt = netns._native().Rtnl()
    rt.link_set_up(rt.link_by_name("lo")["index"])
    fx = fakesysfs.build_mi355x_node(tmp / "sys", n_gpus=n_nics)
    nat = netns._native()
    host_nic = config_type == "host-nic"
    both = config_type == "both"  # an amd-so policy and a host-nic policy on the same node
    label_key = HOST_NIC_READY_LABEL if host_nic else READY_LABEL
    if host_nic:
        nic_names = list(HOST_NICS)
    else:
        nic_names = [p["nic"] for p in nat.discover(str(tmp / "sys"))["pairs"]][:n_nics]
    if both:
        nic_names += list(HOST_NICS)
    for nif in nic_names:
        if nif in HOST_NICS:
            fakesysfs.unbind_driver(tmp / "sys", nif)
    if xgmi_link_down:  # GPU 1's xGMI link 3 is down in its gpu_metrics when the agent starts
        fakesysfs.set_xgmi_link(tmp / "sys", fx["gpus"][1]["bdf"], 3, False)
    if pcie_narrow_nic >= 0:  # that rail's NIC trained its PCIe link at 16 GT/s x8 (a worn slot)
        fakesysfs.set_pcie_link(tmp / "sys", fakesysfs.nic_pci_dir(tmp / "sys", nic_names[pcie_narrow_nic]).name, 16.0, 8)
    # rdma: the rails have no RDMA device when the agent starts (ionic without ionic_rdma);
    # "driver-image": the policy's driverImage loads it (init container); "late": nothing does
    # until the harness registers the devices, with the agent running.
    rdma_removed = {nif: fakesysfs.remove_rdma(tmp / "sys", nif) for nif in (nic_names if rdma else [])}
    plan = netns.random_plan(len(nic_names), rng)
    for n in nat.discover(str(tmp / "sys"))["nics"]:  # RoCE v2 GIDs as the RDMA core adds them
        if n["ifname"] in nic_names and n["rdma_dev"]:
            fakesysfs.add_rocev2_gids(tmp / "sys", n["rdma_dev"], [plan[nic_names.index(n["ifname"])]["local"]])
    sw = netns.SyntheticSwitch(nic_names, plan, rng, interval=interval, phase="random", fast_start=fast_start,
                               silent_nics=silent_nics)
    sw.start(rt)
    if host_nics_owned:
        # Both host NICs are the node's own: the first carries its management address and
        # default route, the second its storage network.  A host-nic policy has nothing to do.
        for k, nif in enumerate(HOST_NICS):
            idx = rt.link_by_name(nif)["index"]
            rt.link_set_up(idx)
            rt.addr_add(idx, f"192.168.{70 + k}.10/24")
            if k == 0:
                rt.route_append("0.0.0.0/0", "192.168.70.1", idx, 16)
    if dark_port_s:
        # The first NIC's switch port comes up `dark_port_s` after the agent starts: an optic
        # still training its link (5-15 s on 200/400G).
        netns.set_switch_port(sw.pid, sw.ports[0], False)

    res: dict = {"n_nics": len(nic_names), "mode": mode, "plan": plan, "nics": nic_names, "fast_start": fast_start}
    fake = FakeApiServer(extra_groups=["nfd.k8s-sigs.io", "cert-manager.io"])
    url = await fake.start()
    os.environ["ENABLE_WEBHOOKS"] = "false"
    os.environ["OPERATOR_NAMESPACE"] = "amd-network-operator"
    stop = asyncio.Event()
    started = asyncio.Event()
    metrics_port = _free_port()
    replicas: list = []
    if ha:
        op = None
        replicas = await _start_replicas(tmp, url, "amd-network-operator")
    else:
        op = asyncio.ensure_future(manager.run(["--master", url, "--health-probe-bind-address=0",
                                                f"--metrics-bind-address=127.0.0.1:{metrics_port}",
                                                "--dependency-check-interval=0"],
                                               stop=stop, started=started))
    # "both": the host NICs come up as mlx5 like the rails (ConnectX everywhere), and the host-nic
    # policy keeps the default driver list, so ownership rests on discovery alone.
    kmd = [sys.executable, "-m", "network_operator_amd.testing.fakesysfs", "bind", "mlx5_core" if both else KMD_DRIVER,
           *[n for n in nic_names if n in HOST_NICS]]
    rdma_kmd = [sys.executable, "-m", "network_operator_amd.testing.fakesysfs", "bind-rdma",
                *[f"{nif}={dev}@{plan[nic_names.index(nif)]['local']}" for nif, dev in rdma_removed.items()]]
    from ..api.v1alpha1 import types as T0

    overrides = {**({"--wait": lldp_wait} if lldp_wait else {}), **({"--label-holddown": "2s"} if flap_burst else {})}
    node = SimNode(fake, node_name, {"amd.feature.node.kubernetes.io/gpu-ready": "true"}, tmp / "host",
                   sysfs_root=tmp / "sys", init_images={KMD_IMAGE: kmd, RDMA_KMD_IMAGE: rdma_kmd},
                   env={"PYTHONPATH": str(Path(__file__).resolve().parents[2])},
                   job_images={T0.DEFAULT_VALIDATION_IMAGE: [sys.executable, "-c", _VALIDATE_STUB, validation or "pass"]},
                   agent_arg_overrides=overrides or None)
    if rdma == "driver-image":
        policy_kw = dict(policy_kw, driverImage=RDMA_KMD_IMAGE)
    if validation and not host_nic:
        policy_kw = dict(policy_kw, validation={"enabled": True, "minBusbw": 300})
    P, DS = kube.NETWORKCLUSTERPOLICIES, kube.DAEMONSETS
    ns = "amd-network-operator"
    name = "scale-out"
    try:
        if ha:
            async with ApiClient(KubeConfig(host=url)) as c:
                res["webhook_registration"] = await _register_webhooks(fake, c, tmp, ns, replicas[0])
            leader = await _until(lambda: _lease_holder(fake, ns), 20)
            assert leader, "no operator replica took the lease"
            metrics_port = next(r for r in replicas if _lease_holder(fake, ns).startswith(r["name"] + "_"))["metrics"]
        else:
            await asyncio.wait_for(started.wait(), 20)
        await node.start()
        async with ApiClient(KubeConfig(host=url)) as c:
            if host_nic:
                pol = T.new_host_nic_policy(name, layer=mode, mtu=9000, nicDrivers=[KMD_DRIVER],
                                            driverImage=KMD_IMAGE, **policy_kw).to_dict()
            else:
                pol = T.new_policy(name, layer=mode, mtu=9000, **policy_kw).to_dict()
            t0 = time.monotonic()
            await c.create(P, pol)
            t_ds = await _until(lambda: fake.get_object(DS, name, ns) is not None, 10)
            t_agent = await _until(lambda: any(x.proc is not None for x in node.containers.values()), 10)
            if host_nics_owned:
                def idle_errors():
                    st = (fake.get_object(P, name) or {}).get("status") or {}
                    return [e for e in st.get("errors") or [] if "no host NIC of its own" in e]
                t_err = await _until(lambda: bool(idle_errors()), 20)
                await asyncio.sleep(7.0)  # more than one probe period: repeated probes, one report
                evs = [e for e in fake.list_objects(kube.EVENTS) if (e.get("involvedObject") or {}).get("kind") == T.KIND]
                res["idle"] = {
                    "policy_to_reason_s": round(t_err - t0, 6) if t_err else None,
                    "status_errors": idle_errors(),
                    "policy_events": [(e.get("reason"), e.get("count", 1), e.get("message", "")) for e in evs],
                    "probe_failures": sum(int(e.get("count", 1)) for e in fake.list_objects(kube.EVENTS)
                                          if e.get("reason") == "Unhealthy"),
                    "agent_restarts": sum(x.restarts for x in node.containers.values()),
                    "agent_running": any(x.proc is not None and x.proc.poll() is None for x in node.containers.values()),
                    "exited": len(node.exited), "label": node.node_labels().get(label_key)}
                res["policy_status"] = (fake.get_object(P, name) or {}).get("status")
                return res
            dark_watch = None
            if dark_port_s:
                seen: dict = {"degraded": [], "errors": []}

                async def watch_policy():  # every Degraded=True and every status error, however brief
                    while True:
                        st = (fake.get_object(P, name) or {}).get("status") or {}
                        for cnd in st.get("conditions") or []:
                            d = f"{cnd.get('reason')}: {cnd.get('message')}"
                            if cnd.get("type") == "Degraded" and cnd.get("status") == "True" and d not in seen["degraded"]:
                                seen["degraded"].append(d)
                        seen["errors"].extend(e for e in st.get("errors") or [] if e not in seen["errors"])
                        await asyncio.sleep(0.005)
                dark_watch = asyncio.ensure_future(watch_policy())
                await asyncio.sleep(max(0.0, t_agent + dark_port_s - time.monotonic()))
                netns.set_switch_port(sw.pid, sw.ports[0], True)
                t_port_up = time.monotonic()
            if pcie_narrow_nic >= 0 or xgmi_link_down:
                # The agent keeps the label off and says why; the operator puts it into
                # status.errors, naming the node (and records it on the Node).
                marker = "PCIe link trained" if pcie_narrow_nic >= 0 else "link 3 down"

                def marked_errors():
                    st = (fake.get_object(P, name) or {}).get("status") or {}
                    return [e for e in st.get("errors") or [] if marker in e]
                t_err = await _until(lambda: bool(marked_errors()), 30)
                res["policy_to_pcie_error_s" if pcie_narrow_nic >= 0 else "policy_to_xgmi_error_s"] = \
                    round(t_err - t0, 6) if t_err else None
                await _until(lambda: any((e.get("involvedObject") or {}).get("kind") == "Node"
                                         for e in fake.list_objects(kube.EVENTS)), 5)
                res["node_events"] = [{"reason": e.get("reason"), "message": e.get("message")}
                                      for e in fake.list_objects(kube.EVENTS)
                                      if (e.get("involvedObject") or {}).get("kind") == "Node"]
                res["agent_restarts"] = sum(x.restarts for x in node.containers.values())
                res["policy_status"] = (fake.get_object(P, name) or {}).get("status")
                res["node_labels"] = node.node_labels()
                return res
            if rdma == "late":
                # No RDMA driver yet: the agent configures the rails and waits, running and
                # unlabelled; "waiting for RDMA device" is a start-up reason, not an error.  Then
                # the driver is loaded (the devices appear) and the label follows.
                seen: dict = {"degraded": [], "errors": [], "reasons": []}

                async def watch_waiting():
                    while True:
                        st = (fake.get_object(P, name) or {}).get("status") or {}
                        for cnd in st.get("conditions") or []:
                            d = f"{cnd.get('reason')}: {cnd.get('message')}"
                            if cnd.get("type") == "Degraded" and cnd.get("status") == "True" and d not in seen["degraded"]:
                                seen["degraded"].append(d)
                        seen["errors"].extend(e for e in st.get("errors") or [] if e not in seen["errors"])
                        await asyncio.sleep(0.005)
                watcher = asyncio.ensure_future(watch_waiting())
                await asyncio.sleep(3.0)
                c0 = next(iter(node.containers.values()))
                pr = subprocess.run(c0.probe, capture_output=True, text=True, timeout=10)
                res["rdma_wait"] = {"probe": {"rc": pr.returncode, "stdout": pr.stdout.strip()},
                                    "label": node.node_labels().get(label_key),
                                    "agent_running": c0.proc is not None and c0.proc.poll() is None,
                                    "rccl_env": node.host_path("/etc/amd/scale-out/rccl.env").exists(),
                                    "addrs": {nif: rt.addr_list(rt.link_by_name(nif)["index"]) for nif in nic_names},
                                    "policy_status": (fake.get_object(P, name) or {}).get("status")}
                t_bind = time.monotonic()
                for nif, dev in rdma_removed.items():
                    fakesysfs.bind_rdma(tmp / "sys", nif, dev, [plan[nic_names.index(nif)]["local"]])
                t_lab = await _until(lambda: node.node_labels().get(label_key) == "true", 10)
                watcher.cancel()
                res["rdma_wait"].update(bind_to_label_s=round(t_lab - t_bind, 6) if t_lab else None,
                                        degraded_seen=seen["degraded"], errors_seen=seen["errors"],
                                        policy_events=sorted({e.get("reason") for e in fake.list_objects(kube.EVENTS)
                                                              if (e.get("involvedObject") or {}).get("kind") == T.KIND}))
            if silent_nics:
                # A switch port that never sends LLDP: the agent's exit error names the NIC, its
                # driver and what it heard, and the operator puts that into status.errors.
                def silent_errors():
                    st = (fake.get_object(P, name) or {}).get("status") or {}
                    return [e for e in st.get("errors") or [] if "LLDP silent" in e]
                t_err = await _until(lambda: bool(silent_errors()), 30)
                res["policy_to_silent_error_s"] = round(t_err - t0, 6) if t_err else None
                await _until(lambda: any(e.get("reason") == "AgentFailed" for e in fake.list_objects(kube.EVENTS)), 5)
                res["policy_status"] = (fake.get_object(P, name) or {}).get("status")
                res["node_labels"] = node.node_labels()
                res["events"] = [e.get("reason") + ": " + e.get("message", "") for e in fake.list_objects(kube.EVENTS)]
                return res
            t_label = await _until(lambda: node.node_labels().get(label_key) == "true", 30)

            if both:
                await c.create(P, T.new_host_nic_policy("host-nics", layer=mode, mtu=9000,
                                                        driverImage=KMD_IMAGE).to_dict())

                def host_good():
                    st = (fake.get_object(P, "host-nics") or {}).get("status") or {}
                    return st.get("state") == "All good" and node.node_labels().get(HOST_NIC_READY_LABEL) == "true"
                t_host = await _until(host_good, 30)
                res["host_nic_policy_all_good_s"] = round(t_host - t0, 6) if t_host else None
                res["host_nic_status"] = (fake.get_object(P, "host-nics") or {}).get("status")
                # What each agent took (its status file) and left alone: two disjoint NIC sets.
                res["agent_nic_sets"], res["agent_excluded"] = {}, {}
                for x in node.containers.values():
                    sf = next((a.split("=", 1)[1] for a in x.argv if a.startswith("--status-file=")), None)
                    try:
                        st = json.loads(Path(sf).read_text()) if sf else {}
                    except (OSError, ValueError):
                        st = {}
                    res["agent_nic_sets"][x.daemonset] = [i["name"] for i in st.get("interfaces", [])]
                    res["agent_excluded"][x.daemonset] = st.get("excluded", "")

            def all_good():
                st = (fake.get_object(P, name) or {}).get("status") or {}
                return st.get("state") == "All good" and st.get("ready") == 1

            t_good = await _until(all_good, 30)
            rel = lambda t: round(t - t0, 6) if t else None  # noqa: E731
            if dark_watch is not None:
                dark_watch.cancel()
                res["dark_port"] = {
                    "port_up_after_agent_s": round(t_port_up - t_agent, 6),
                    "port_up_to_label_s": round(t_label - t_port_up, 6) if t_label else None,
                    "degraded_seen": seen["degraded"], "errors_seen": seen["errors"],
                    "policy_events": sorted({e.get("reason") for e in fake.list_objects(kube.EVENTS)
                                             if (e.get("involvedObject") or {}).get("kind") == T.KIND}),
                    "probe_events": [e.get("message") for e in fake.list_objects(kube.EVENTS)
                                     if e.get("reason") == "Unhealthy"],
                    "agent_restarts": sum(x.restarts for x in node.containers.values())}
            res.update(policy_to_daemonset_s=rel(t_ds), policy_to_agent_start_s=rel(t_agent),
                       policy_to_node_label_s=rel(t_label), policy_to_all_good_s=rel(t_good))
            res["policy_status"] = (fake.get_object(P, name) or {}).get("status")
            if validation:
                def validated():
                    st = (fake.get_object(P, name) or {}).get("status") or {}
                    c = {x["type"]: x for x in st.get("conditions", [])}.get("FabricValidated") or {}
                    return c.get("status") in ("True", "False") and c
                t_val = await _until(validated, 30)
                res["policy_to_validated_s"] = rel(t_val)
                res["validation_condition"] = validated() or None
                res["validation_jobs"] = [{"node": (j["metadata"].get("annotations") or {}).get("amd.com/node"),
                                           "status": j.get("status")} for j in fake.list_objects(kube.JOBS)]
                res["job_runs"] = node.job_runs
                await _until(lambda: validation != "pass" or VALIDATED_LABEL in node.node_labels(), 5)
                res["node_labels"] = node.node_labels()
            res["operator_metrics"] = await _scrape(metrics_port, ("amd_network_operator_agent_ready_seconds_count",
                                                                   "amd_network_operator_agent_ready_seconds_sum",
                                                                   "amd_network_operator_policy_ready"))
            if duplicate_policy:
                # A second amd-so policy selecting the same node: its agent would flush and
                # re-address the same NICs.  The operator holds it off the node (node affinity):
                # no agent of it runs there, so nothing waits on the node lock or restarts.  Once
                # the older policy goes, the newer one takes the node.
                dup = "scale-out-dup"
                addrs_before = {nif: rt.addr_list(rt.link_by_name(nif)["index"]) for nif in nic_names}
                dup_pods_seen = []

                async def watch_dup():
                    while True:
                        dup_pods_seen.extend(x.pod[1] for x in node.containers.values()
                                             if x.daemonset == f"{ns}/{dup}" and x.pod[1] not in dup_pods_seen)
                        await asyncio.sleep(0.002)
                watcher = asyncio.ensure_future(watch_dup())
                await c.create(P, T.new_policy(dup, layer=mode, mtu=9000, **policy_kw).to_dict())

                def dup_error():
                    st = (fake.get_object(P, dup) or {}).get("status") or {}
                    return [e for e in st.get("errors") or [] if "held off" in e]
                await _until(lambda: bool(dup_error()), 20)
                await asyncio.sleep(2.0)  # long enough for a placed agent to show up
                res["duplicate_policy_errors"] = dup_error()
                res["duplicate_policy_status"] = (fake.get_object(P, dup) or {}).get("status")
                res["duplicate_daemonset_affinity"] = (fake.get_object(DS, dup, ns) or {}).get(
                    "spec", {}).get("template", {}).get("spec", {}).get("affinity")
                res["duplicate_agents_while_held"] = list(dup_pods_seen)
                res["first_policy_status_after_duplicate"] = (fake.get_object(P, name) or {}).get("status")
                res["addrs_unchanged_by_duplicate"] = addrs_before == {
                    nif: rt.addr_list(rt.link_by_name(nif)["index"]) for nif in nic_names}
                res["label_after_duplicate"] = node.node_labels().get(label_key)
                gen0 = fake.get_object(DS, dup, ns)["metadata"]["generation"]
                t1 = time.monotonic()
                await c.delete(P, name)
                t_release = await _until(lambda: not (fake.get_object(DS, dup, ns) or {}).get("spec", {}).get(
                    "template", {}).get("spec", {}).get("affinity"), 10)

                def dup_good():
                    st = (fake.get_object(P, dup) or {}).get("status") or {}
                    return st.get("state") == "All good" and st.get("errors") == [] and \
                        node.node_labels().get(label_key) == "true"
                t_dup_ready = await _until(dup_good, 60)
                watcher.cancel()
                dup_c = [x for x in node.containers.values() if x.daemonset == f"{ns}/{dup}"]
                res["takeover"] = {
                    "delete_to_hold_released_s": round(t_release - t1, 6) if t_release else None,
                    "daemonset_updates": fake.get_object(DS, dup, ns)["metadata"]["generation"] - gen0,
                    "delete_to_newer_ready_s": round(t_dup_ready - t1, 6) if t_dup_ready else None,
                    "newer_agent_restarts": sum(x.restarts for x in dup_c), "newer_agents": len(dup_c),
                    "newer_status": (fake.get_object(P, dup) or {}).get("status")}
                res["agent_exit_codes"] = [e["rc"] for e in node.exited]
                return res
            if ha:
                res.update(await _ha_checks(fake, c, rt, node, replicas, ns, name, mode, nic_names, label_key,
                                            all_good, update_mtu or 4200))
            res["init_runs"] = [dict(r, t_start=rel(r["t_start"]), t_end=rel(r["t_end"])) for r in node.init_runs]
            res["agent_started_s"] = [rel(t) for x in node.containers.values() for t in x.started_at]
            res["node_labels"] = node.node_labels()
            res["agent_argv"] = next(iter(node.containers.values())).argv if node.containers else None
            art = node.host_path("/etc/amd/scale-out")
            res["artifacts"] = sorted(os.listdir(art)) if art.exists() else []
            res["rccl_env"] = (art / "rccl.env").read_text() if (art / "rccl.env").exists() else None
            state = {}
            for nif in nic_names:
                link = rt.link_by_name(nif)
                state[nif] = {"up": link["up"], "mtu": link["mtu"], "addrs": rt.addr_list(link["index"])}
            res["state"] = state
            if driver_reload:
                # The first NIC's driver is reloaded: its netdev disappears and comes back with a new
                # ifindex.  The agent tears down and exits, the kubelet restarts it (it keeps failing
                # while the NIC is missing), and once the NIC is back the node is ready again.
                c0 = next(iter(node.containers.values()))
                nif, port = nic_names[0], sw.ports[0]
                t1 = time.monotonic()
                rt.link_del(rt.link_by_name(nif)["index"])  # takes the switch end with it
                t_unlabel = await _until(lambda: label_key not in node.node_labels(), 10)
                await asyncio.sleep(0.3)  # the driver takes a moment
                rt.veth_add(nif, port)
                rt.link_set_netns_pid(rt.link_by_name(port)["index"], sw.pid)
                t_back = await _until(lambda: all_good() and node.node_labels().get(label_key) == "true", 30)
                res["reload_to_unlabelled_s"] = round(t_unlabel - t1, 6) if t_unlabel else None
                res["reload_to_all_good_s"] = round(t_back - t1, 6) if t_back else None
                res["agent_starts_after_reload"] = len(c0.started_at)
                link = rt.link_by_name(nif)
                res["reloaded_nic_addrs"] = rt.addr_list(link["index"])
            if crash_agent:
                # The agent dies without cleaning up (OOM kill): the kubelet restarts the container,
                # the new agent removes the stale label, configures again and is ready again.
                c0 = next(iter(node.containers.values()))
                # The kubelet's first restart back-off is 10 s; 1 s here keeps the outage long enough
                # for the operator to report it on a loaded test machine (0.1 s sometimes was not).
                c0.backoff = 1.0

                def crash_errors():
                    return [e for e in ((fake.get_object(P, name) or {}).get("status") or {}).get("errors") or []
                            if "exited with code" in e]
                seen: list = []

                async def record():  # every crash entry the status carries, however briefly
                    while True:
                        seen.extend(e for e in crash_errors() if e not in seen)
                        await asyncio.sleep(0.001)
                recorder = asyncio.ensure_future(record())
                t1 = time.monotonic()
                c0.proc.kill()
                t_unready = await _until(lambda: not all_good(), 10)
                await _until(lambda: bool(seen), 10)
                t_back = await _until(lambda: len(c0.started_at) == 2 and c0.ready and all_good()
                                      and node.node_labels().get(label_key) == "true", 30)
                recorder.cancel()
                res["crash_status_errors"] = list(seen)
                res["crash_to_unready_s"] = round(t_unready - t1, 6) if t_unready else None
                res["crash_to_all_good_s"] = round(t_back - t1, 6) if t_back else None
                res["agent_restarts"] = c0.restarts
                res["operator_metrics_after_crash"] = await _scrape(metrics_port, (
                    "amd_network_operator_agent_unready_total", "amd_network_operator_agent_ready_seconds_count"))
            if flap:
                # Carrier loss on one switch port: the agent withdraws the label, the probe fails,
                # the operator reports the node; the port comes back and so does everything else.
                t1 = time.monotonic()
                netns.set_switch_port(sw.pid, sw.ports[0], False)

                def degraded():
                    st = (fake.get_object(P, name) or {}).get("status") or {}
                    return label_key not in node.node_labels() and st.get("state") != "All good" and st.get("errors")

                t_deg = await _until(degraded, 10)
                # The probe's reason reaches status.errors through the kubelet's event.
                t_why = await _until(lambda: any("link down" in e for e in (
                    (fake.get_object(P, name) or {}).get("status") or {}).get("errors") or []), 10)
                res["port_down_to_reason_in_status_s"] = round(t_why - t1, 6) if t_why else None
                await _until(lambda: any(e.get("reason") == "NodeDegraded" for e in fake.list_objects(kube.EVENTS)), 5)
                res["policy_events_after_flap"] = sorted({e.get("reason") for e in fake.list_objects(kube.EVENTS)
                                                          if (e.get("involvedObject") or {}).get("kind") == T.KIND})
                await _until(lambda: any((e.get("involvedObject") or {}).get("kind") == "Node"
                                         for e in fake.list_objects(kube.EVENTS)), 5)
                node_obj = fake.get_object(kube.NODES, node_name) or {}
                res["node_events_after_flap"] = [
                    {"reason": e.get("reason"), "message": e.get("message"), "namespace": e["metadata"].get("namespace"),
                     "uid_matches": (e.get("involvedObject") or {}).get("uid") == node_obj.get("metadata", {}).get("uid")}
                    for e in fake.list_objects(kube.EVENTS) if (e.get("involvedObject") or {}).get("kind") == "Node"]
                res["flap_status"] = (fake.get_object(P, name) or {}).get("status")
                # The readiness probe's output, which the kubelet puts in the Pod's events.
                c0 = next(iter(node.containers.values()))
                pr = subprocess.run(c0.probe, capture_output=True, text=True, timeout=10)
                res["probe_while_degraded"] = {"rc": pr.returncode, "stdout": pr.stdout.strip()}
                t2 = time.monotonic()
                netns.set_switch_port(sw.pid, sw.ports[0], True)
                # (the agent's default --label-holddown, 10 s, delays the republication)
                t_back = await _until(lambda: node.node_labels().get(label_key) == "true" and all_good(), 30)
                res["port_down_to_status_degraded_s"] = round(t_deg - t1, 6) if t_deg else None
                res["port_up_to_all_good_s"] = round(t_back - t2, 6) if t_back else None
            if flap_burst:
                # A flapping optic: port 0 goes down and up `flap_burst` times in a row.  With the
                # agent's label hold-down the node is withdrawn once and republished once, so the
                # policy goes Degraded once -- not once per flap.
                edges: dict = {"degraded": [], "label": []}

                async def watch_edges():
                    was_deg, was_lab = False, True
                    while True:
                        st = (fake.get_object(P, name) or {}).get("status") or {}
                        deg = any(x.get("type") == "Degraded" and x.get("status") == "True" for x in st.get("conditions") or [])
                        lab = node.node_labels().get(label_key) == "true"
                        if deg != was_deg:
                            edges["degraded"].append((round(time.monotonic() - t0, 4), deg))
                            was_deg = deg
                        if lab != was_lab:
                            edges["label"].append((round(time.monotonic() - t0, 4), lab))
                            was_lab = lab
                        await asyncio.sleep(0.002)
                w = asyncio.ensure_future(watch_edges())
                for _ in range(flap_burst):
                    netns.set_switch_port(sw.pid, sw.ports[0], False)
                    await asyncio.sleep(0.25)
                    netns.set_switch_port(sw.pid, sw.ports[0], True)
                    await asyncio.sleep(0.25)
                t_last = time.monotonic()
                t_back = await _until(lambda: node.node_labels().get(label_key) == "true" and all_good(), 30)
                await asyncio.sleep(0.5)
                w.cancel()
                res["flap_burst"] = {"flaps": flap_burst, "degraded_edges": edges["degraded"], "label_edges": edges["label"],
                                     "last_flap_to_all_good_s": round(t_back - t_last, 6) if t_back else None,
                                     "agent_restarts": sum(x.restarts for x in node.containers.values())}
            if update_mtu:
                # `kubectl edit`: new MTU -> DaemonSet template changes -> the kubelet replaces the
                # agent -> the new agent configures the NICs again and republishes the label.
                # Sampled every ~0.5 ms through the roll: how long a NIC was without its /30 (what
                # an RCCL job's RoCE QPs bound to it would have seen).
                want = {nif: [p["local"] + "/30"] for nif, p in zip(nic_names, plan)} if mode == "L3" else {}
                samples = {"n": 0, "missing": 0, "first": None, "last": None}
                sampling = asyncio.Event()

                async def sample():
                    idx = {nif: rt.link_by_name(nif)["index"] for nif in want}
                    while not sampling.is_set():
                        now = time.monotonic()
                        samples["n"] += 1
                        if any(rt.addr_list(i) != want[nif] for nif, i in idx.items()):
                            samples["missing"] += 1
                            samples["first"] = samples["first"] or now
                            samples["last"] = now
                        await asyncio.sleep(0.0005)
                sampler = asyncio.ensure_future(sample())
                t1 = time.monotonic()
                await _edit(c, P, name, lambda cur: cur["spec"]["amdScaleOut"].update(mtu=update_mtu))

                def mtu_applied():
                    return all(rt.link_by_name(nif)["mtu"] == update_mtu for nif in nic_names)

                t_mtu = await _until(mtu_applied, 30)
                t_relabel = await _until(lambda: node.node_labels().get(label_key) == "true" and all_good(), 30)
                sampling.set()
                await sampler
                res["roll_address_samples"] = samples["n"]
                res["roll_address_missing_samples"] = samples["missing"]
                res["roll_address_gap_s"] = round(samples["last"] - samples["first"], 6) if samples["first"] else 0.0
                res["update_to_mtu_applied_s"] = round(t_mtu - t1, 6) if t_mtu else None
                res["update_to_ready_again_s"] = round(t_relabel - t1, 6) if t_relabel else None
                res["agent_starts"] = sum(len(x.started_at) for x in node.containers.values()) + len(node.exited)
            if teardown:
                t1 = time.monotonic()
                await c.delete(P, name)
                t_gone = await _until(lambda: fake.get_object(DS, name, ns) is None and not any(
                    x.daemonset == f"{ns}/{name}" for x in node.containers.values()), 30)
                t_unlabel = await _until(lambda: label_key not in node.node_labels(), 10)
                res["delete_to_agent_stopped_s"] = round(t_gone - t1, 6) if t_gone else None
                res["delete_to_label_removed_s"] = round(t_unlabel - t1, 6) if t_unlabel else None
                if policy_kw.get("keepConfigOnRestart"):
                    # The agent left its addresses; the finalizer holds the policy until the
                    # cleanup Job (the agent with --cleanup) has removed them.
                    def cleaned():
                        return fake.get_object(P, name) is None and all(
                            rt.addr_list(rt.link_by_name(nif)["index"]) == [] for nif in nic_names)
                    t_clean = await _until(cleaned, 30)
                    res["delete_to_cleaned_and_policy_gone_s"] = round(t_clean - t1, 6) if t_clean else None
                    res["cleanup_job_runs"] = [dict(j, t_start=round(j["t_start"] - t1, 6), t_end=round(j["t_end"] - t1, 6))
                                               for j in node.job_runs]
                    art = node.host_path("/etc/amd/scale-out")
                    res["artifacts_after_cleanup"] = sorted(os.listdir(art)) if art.exists() else []
                res["after_delete"] = {nif: rt.addr_list(rt.link_by_name(nif)["index"]) for nif in nic_names}
                res["links_up_after_delete"] = {nif: rt.link_by_name(nif)["up"] for nif in nic_names}
                res["link_state_after_delete"] = node.host_path("/etc/amd/scale-out/link-state").exists()
                res["agent_exit_codes"] = [e["rc"] for e in node.exited]
                res["agent_sigterm_to_exit_s"] = [e["sigterm_to_exit_s"] for e in node.exited]
    finally:
        res["agent_log"] = "".join(e["log"] for e in node.exited)[-6000:]
        if not res["agent_log"]:
            for f in sorted((tmp / "pod-logs").glob("*.log")) if (tmp / "pod-logs").exists() else []:
                res["agent_log"] += f.read_text(errors="replace")[-6000:]
        await node.stop()
        stop.set()
        if op is not None:
            try:
                res["operator_rc"] = await asyncio.wait_for(op, 20)
            except Exception as e:  # pragma: no cover
                res["operator_rc"] = repr(e)
        if replicas:
            res["operator_rc"] = await _stop_replicas(replicas)
            res["operator_logs"] = {r["name"]: r["log"].read_text(errors="replace")[-3000:] for r in replicas}
        await fake.stop()
        sw.stop()
    return res


async def _fabric_scenario(tmp: Path, n_nodes: int, n_nics: int, seed: int, collective: bool) -> dict:
    """`n_nodes` nodes on one routing leaf switch, one policy: the operator's DaemonSet lands on
    every node, each node's agent addresses its NICs, the policy reports n/n, and (2 nodes) a
    gloo all-reduce runs between the nodes over the configured /16 routes."""
    from ..api.v1alpha1 import types as T
    from ..operator import kube, manager
    from ..operator.kube import ApiClient, KubeConfig
    from . import twonode
    from .fakeapi import FakeApiServer
    from .nodesim import SimNode

    rng = random.Random(seed)
    nat = netns._native()
    rt = nat.Rtnl()
    rt.link_set_up(rt.link_by_name("lo")["index"])
    holders = [None] + [netns.NetnsHolder() for _ in range(n_nodes - 1)]
    res: dict = {"n_nodes": n_nodes, "n_nics": n_nics}
    sw = None
    fake = nodes = op = None
    stop = asyncio.Event()
    try:
        for j, h in enumerate(holders):
            fakesysfs.build_mi355x_node(tmp / f"sys{j}", n_gpus=n_nics)
            if h is not None:
                h.run(lambda: nat.Rtnl().link_set_up(nat.Rtnl().link_by_name("lo")["index"]))
        nic_names = [p["nic"] for p in nat.discover(str(tmp / "sys0"))["pairs"]][:n_nics]
        plan = netns.random_plan(n_nodes * n_nics, rng)  # node j owns plan[j*n : (j+1)*n]
        for j in range(n_nodes):
            for n in nat.discover(str(tmp / f"sys{j}"))["nics"]:
                if n["ifname"] in nic_names and n["rdma_dev"]:
                    ip = plan[j * n_nics + nic_names.index(n["ifname"])]["local"]
                    fakesysfs.add_rocev2_gids(tmp / f"sys{j}", n["rdma_dev"], [ip])
        remote = [(h.pid, nif) for h in holders[1:] for nif in nic_names]
        sw = netns.SyntheticSwitch(nic_names, plan, rng, interval="30s", phase="random", fast_start=True,
                                   remote=remote, forward=True)
        sw.start(rt)
        res["plan"], res["nics"] = plan, nic_names

        fake = FakeApiServer(extra_groups=["nfd.k8s-sigs.io", "cert-manager.io"])
        url = await fake.start()
        os.environ["ENABLE_WEBHOOKS"] = "false"
        os.environ["OPERATOR_NAMESPACE"] = "amd-network-operator"
        started = asyncio.Event()
        op = asyncio.ensure_future(manager.run(["--master", url, "--health-probe-bind-address=0",
                                                "--metrics-bind-address=0", "--dependency-check-interval=0"],
                                               stop=stop, started=started))
        await asyncio.wait_for(started.wait(), 20)
        nodes = [SimNode(fake, f"mi355x-{j}", {"amd.feature.node.kubernetes.io/gpu-ready": "true"}, tmp / f"host{j}",
                         sysfs_root=tmp / f"sys{j}", netns=h) for j, h in enumerate(holders)]
        for nd in nodes:
            await nd.start()
        P = kube.NETWORKCLUSTERPOLICIES
        async with ApiClient(KubeConfig(host=url)) as c:
            t0 = time.monotonic()
            await c.create(P, T.new_policy("fabric", layer="L3", mtu=9000).to_dict())

            def all_labelled():
                return all(nd.node_labels().get(READY_LABEL) == "true" for nd in nodes)

            def all_good():
                st = (fake.get_object(P, "fabric") or {}).get("status") or {}
                return st.get("state") == "All good" and st.get("ready") == n_nodes

            t_lab = await _until(all_labelled, 30)
            t_good = await _until(all_good, 30)
            res["policy_to_all_nodes_labelled_s"] = round(t_lab - t0, 6) if t_lab else None
            res["policy_to_all_good_s"] = round(t_good - t0, 6) if t_good else None
            res["policy_status"] = (fake.get_object(P, "fabric") or {}).get("status")
            res["node_labels"] = {nd.name: nd.node_labels() for nd in nodes}
            addrs = []
            for j, h in enumerate(holders):
                out = tmp / f"addrs{j}.json"

                def dump(path=out):
                    r = nat.Rtnl()
                    path.write_text(json.dumps({nif: r.addr_list(r.link_by_name(nif)["index"]) for nif in nic_names}))
                if h is None:
                    dump()
                else:
                    h.run(dump)
                addrs.append(json.loads(out.read_text()))
            res["addrs"] = addrs
            if collective and t_good and n_nodes == 2:
                # One rank per node, bound to its first scale-out NIC, rendezvous on node 0's
                # first rail address: the bytes cross NIC, /16 route, the leaf's forwarding, NIC.
                port = 29500 + rng.randrange(0, 400)
                master = plan[0]["local"]
                procs = []
                for j, h in enumerate(holders):
                    procs.append(await asyncio.create_subprocess_exec(
                        sys.executable, "-c", twonode._WORKER, env=twonode._worker_env(j, nic_names[0], master, port),
                        stdout=asyncio.subprocess.PIPE, stderr=asyncio.subprocess.PIPE,
                        preexec_fn=h.enter if h else None))
                outs = [await asyncio.wait_for(p.communicate(), 180) for p in procs]
                res["collective"] = []
                for p, (o, e) in zip(procs, outs):
                    text = o.decode().strip().splitlines()
                    res["collective"].append(json.loads(text[-1]) if p.returncode == 0 and text else
                                             {"rc": p.returncode, "stderr": e.decode()[-2000:]})
            t1 = time.monotonic()
            await c.delete(P, "fabric")
            t_gone = await _until(lambda: all(not nd.containers for nd in nodes)
                                  and not any(READY_LABEL in nd.node_labels() for nd in nodes), 30)
            res["delete_to_all_nodes_clean_s"] = round(t_gone - t1, 6) if t_gone else None
            res["agent_exit_codes"] = [[e["rc"] for e in nd.exited] for nd in nodes]
    finally:
        if nodes:
            res["agent_logs"] = ["".join(e["log"] for e in nd.exited)[-3000:] for nd in nodes]
            for nd in nodes:
                await nd.stop()
        stop.set()
        if op is not None:
            try:
                res["operator_rc"] = await asyncio.wait_for(op, 20)
            except Exception as e:  # pragma: no cover
                res["operator_rc"] = repr(e)
        if fake is not None:
            await fake.stop()
        if sw is not None:
            sw.stop()
        for h in holders:
            if h is not None:
                h.stop()
    return res


def run_fabric(n_nodes: int = 2, n_nics: int = 2, seed: int = 1, collective: bool = True,
               keep_tmp: bool = False) -> dict:
    """Must already run inside a private user+net namespace (``run_isolated(fabric=True, ...)``)."""
    tmp = Path(tempfile.mkdtemp(prefix="netop-fabric-"))
    try:
        return asyncio.run(_fabric_scenario(tmp, n_nodes, n_nics, seed, collective))
    finally:
        if not keep_tmp:
            shutil.rmtree(tmp, ignore_errors=True)


def run_scenario(n_nics: int = 2, mode: str = "L3", seed: int = 1, interval: str = "30s", fast_start: bool = True,
                 teardown: bool = True, node_name: str = "mi355x-0", policy_kw: Optional[dict] = None,
                 update_mtu: int = 0, config_type: str = "amd-so", flap: bool = False, validation: str = "",
                 crash_agent: bool = False, driver_reload: bool = False, ha: bool = False,
                 silent_nics: int = 0, lldp_wait: str = "", keep_tmp: bool = False,
                 duplicate_policy: bool = False, dark_port_s: float = 0.0, host_nics_owned: bool = False,
                 pcie_narrow_nic: int = -1, xgmi_link_down: bool = False, rdma: str = "",
                 flap_burst: int = 0) -> dict:
    """Must already run inside a private user+net namespace (``run_isolated``)."""
    tmp = Path(tempfile.mkdtemp(prefix="netop-e2e-"))
    try:
        return asyncio.run(_scenario(tmp, n_nics, mode, seed, interval, fast_start, teardown, node_name,
                                     dict(policy_kw or {}), update_mtu, config_type, flap, validation,
                                     crash_agent, driver_reload, ha, silent_nics, lldp_wait, duplicate_policy,
                                     dark_port_s=dark_port_s, host_nics_owned=host_nics_owned,
                                     pcie_narrow_nic=pcie_narrow_nic, xgmi_link_down=xgmi_link_down, rdma=rdma,
                                     flap_burst=flap_burst))
    finally:
        if not keep_tmp:
            shutil.rmtree(tmp, ignore_errors=True)


def run_isolated(timeout: float = 300, **kw) -> dict:
    """``run_scenario(**kw)`` in a fresh user+net namespace."""
    import subprocess

    cmd = [*netns.unshare_cmd(), sys.executable, "-m", "network_operator_amd.testing.e2e", "--json", json.dumps(kw)]
    root = Path(__file__).resolve().parents[2]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, cwd=root,
                       env=dict(os.environ, PYTHONPATH=str(root)))
    if r.returncode != 0:
        raise RuntimeError(f"e2e scenario failed rc={r.returncode}: {r.stderr[-3000:]}")
    return json.loads(r.stdout.strip().splitlines()[-1])


def _main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--json", default="{}", help="run_scenario kwargs")
    a = ap.parse_args(argv)
    kw = json.loads(a.json)
    print(json.dumps(run_fabric(**kw) if kw.pop("fabric", False) else run_scenario(**kw)))
    return 0


if __name__ == "__main__":
    sys.exit(_main())
