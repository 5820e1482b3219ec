"""Control-plane tests against the in-process fake API server.

Mirrors the reference's envtest suite (reference internal/controller/networkconfiguration_controller_test.go)
and adds what envtest could not show: DaemonSet status -> policy status with node targeting,
ownerRef garbage collection, conflicts, watch recovery, leader election, metrics.
"""

import asyncio
import json
import contextlib

import pytest

from network_operator_amd.api.v1alpha1 import types as T
from network_operator_amd import discovery
from network_operator_amd.operator import kube
from network_operator_amd.operator.controller import PolicyController
from network_operator_amd.operator.kube import ApiClient, ApiError, KubeConfig
from network_operator_amd.operator.leader import LeaderElector
from network_operator_amd.operator.reconciler import agent_args
from network_operator_amd.testing.fakeapi import FakeApiServer

TOPO_ARGS = ["--rccl-topo=/host/etc/amd/scale-out/rccl-topo.xml", "--rccl-topo-env-path=/etc/amd/scale-out/rccl-topo.xml"]
STATUS_ARG = "--status-file=/run/amd-network-agent/status.json"  # the probe prints why a node is not ready
LINK_STATE_ARG = "--link-state=/host/etc/amd/scale-out/link-state"  # the NICs' up/down from before any agent
HOST_NIC_LINK_STATE_ARG = "--link-state=/host/etc/amd/scale-out/host-nic-link-state"

NS = "amd-network-operator"


def run(coro, timeout=60):
    return asyncio.run(asyncio.wait_for(coro, timeout))


async def eventually(fn, timeout=5.0, interval=0.02):
    end = asyncio.get_event_loop().time() + timeout
    last = None
    while True:
        try:
            r = fn()
            if asyncio.iscoroutine(r):
                r = await r
            if r is not False:
                return r
        except (AssertionError, KeyError, TypeError, ApiError) as e:
            last = e
        if asyncio.get_event_loop().time() > end:
            raise AssertionError(f"condition not met: {last!r}")
        await asyncio.sleep(interval)


async def value(fn, timeout=5.0):
    """Waits until fn() returns something other than None / False and returns it."""
    out = []

    def check():
        v = fn()
        assert v not in (None, False)
        out.append(v)
    await eventually(check, timeout)
    return out[-1]


OPERATOR_UA = "amd-network-operator/0.1"


@contextlib.asynccontextmanager
async def cluster(openshift=True, workers=2, user_client=None, **fake_kw):
    """A fake API server and a running controller.  The yielded client is the controller's own,
    or with ``user_client`` a separate one with that User-Agent (faults can then target the
    operator's requests alone)."""
    fake = FakeApiServer(openshift=openshift, **fake_kw)
    url = await fake.start()
    client = ApiClient(KubeConfig(host=url), user_agent=OPERATOR_UA)
    user = ApiClient(KubeConfig(host=url), user_agent=user_client) if user_client else client
    ctl = PolicyController(client, NS, is_openshift=openshift, workers=workers)
    await ctl.start()
    try:
        yield fake, user, ctl
    finally:
        await ctl.stop()
        if user is not client:
            await user.close()
        await client.close()
        await fake.stop()


async def edit(client, name, change, attempts=20):
    """kubectl edit: get, change, replace; a write of the operator's in between (status,
    finalizer) is a conflict, and the edit is retried on the new object, as a client does."""
    for _ in range(attempts):
        cur = await client.get(kube.NETWORKCLUSTERPOLICIES, name)
        change(cur)
        try:
            return await client.replace(kube.NETWORKCLUSTERPOLICIES, cur)
        except ApiError as e:
            if e.status != 409:
                raise
            await asyncio.sleep(0.01)
    raise AssertionError(f"edit of {name} kept conflicting")


# The CRD's (and the mutating webhook's) MI355X-first defaults: xgmiCheck and requireRdma on.
MI355X_DEFAULTS = ["--xgmi-expect=0", "--require-rdma"]


def policy(name="policy", layer="L3", **so):
    p = T.new_policy(name, layer=layer, node_selector={"foo": "bar"}, **so)
    return p.to_dict()


def test_reconcile_lifecycle_reference_parity():
    async def body():
        async with cluster(openshift=True) as (fake, client, ctl):
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy(image="amd/my-linkdiscovery:latest", mtu=8000))

            def status_ok():
                p = fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")
                assert p["spec"]["configurationType"] == "amd-so"
                assert p["status"]["targets"] == 0 and p["status"]["state"] == "No targets"
                assert p["status"]["errors"] == []
            await eventually(status_ok)

            def ds_ok():
                ds = fake.get_object(kube.DAEMONSETS, "policy", NS)
                pod = ds["spec"]["template"]["spec"]
                assert pod["serviceAccountName"] == "policy-sa"
                c = pod["containers"]
                assert len(c) == 1 and c[0]["image"] == "amd/my-linkdiscovery:latest"
                assert c[0]["args"] == ["--configure=true", "--keep-running", "--mode=L3", "--mtu=8000", "--wait=90s",
                                        "--rccl-net=/host/etc/amd/scale-out/rccl-net.json",
                                        "--rccl-env=/host/etc/amd/scale-out/rccl.env", *TOPO_ARGS, *MI355X_DEFAULTS,
                                        LINK_STATE_ARG, STATUS_ARG]
                assert [v["name"] for v in pod["volumes"]] == ["nfd-features", "agent-run", "rccl-artifacts"]
                assert [m["name"] for m in c[0]["volumeMounts"]] == ["nfd-features", "agent-run", "rccl-artifacts"]
                assert pod["nodeSelector"] == {"foo": "bar"}
                ref = ds["metadata"]["ownerReferences"][0]
                assert ref["kind"] == "NetworkClusterPolicy" and ref["controller"] is True
                sa = fake.get_object(kube.SERVICEACCOUNTS, "policy-sa", NS)
                rb = fake.get_object(kube.ROLEBINDINGS, "policy-sa-rb", NS)
                assert sa and rb["subjects"] == [{"kind": "ServiceAccount", "name": "policy-sa", "namespace": NS}]
                assert rb["roleRef"]["name"] == "system:openshift:scc:privileged"
            await eventually(ds_ok)

            # update to L2: the reference's 3 args (+ --v; controller_test.go:138-151), plus rccl.env:
            # on MI355X RCCL needs the scale-out HCAs and the link-local RoCE v2 GID in L2 too
            await edit(client, "policy", lambda cur: cur["spec"].update(
                amdScaleOut={"layer": "L2", "image": "amd/my-linkdiscovery:latest"}))

            def l2_ok():
                ds = fake.get_object(kube.DAEMONSETS, "policy", NS)
                c = ds["spec"]["template"]["spec"]["containers"][0]
                assert c["args"] == ["--configure=true", "--keep-running", "--mode=L2",
                                     "--rccl-env=/host/etc/amd/scale-out/rccl.env", *TOPO_ARGS, *MI355X_DEFAULTS,
                                     LINK_STATE_ARG, STATUS_ARG]
                assert [v["name"] for v in ds["spec"]["template"]["spec"]["volumes"]] == ["nfd-features", "agent-run",
                                                                                          "rccl-artifacts"]
            await eventually(l2_ok)

            # L3 + disableNetworkManager + mtu 0: volumes in stable order (controller_test.go:153-180)
            await edit(client, "policy", lambda cur: cur["spec"].update(
                amdScaleOut={"layer": "L3", "disableNetworkManager": True, "pullPolicy": "Always"}, logLevel=4))

            def l3nm_ok():
                ds = fake.get_object(kube.DAEMONSETS, "policy", NS)
                c = ds["spec"]["template"]["spec"]["containers"][0]
                assert c["args"][:6] == ["--configure=true", "--keep-running", "--mode=L3", "--v=4",
                                         "--disable-networkmanager", "--nm-keyfile-dir=/etc/NetworkManager/conf.d"]
                assert c["args"][6] == "--wait=90s"
                assert c["imagePullPolicy"] == "Always"  # fix: pullPolicy applied
                assert [v["name"] for v in ds["spec"]["template"]["spec"]["volumes"]] == \
                    ["nfd-features", "agent-run", "var-run-dbus", "networkmanager", "rccl-artifacts"]
                assert all(v["hostPath"]["type"] == "DirectoryOrCreate"
                           for v in ds["spec"]["template"]["spec"]["volumes"] if "hostPath" in v)
            await eventually(l3nm_ok)

            # delete: ownerRef GC removes DaemonSet, ServiceAccount, RoleBinding
            await client.delete(kube.NETWORKCLUSTERPOLICIES, "policy")

            def gone():
                assert fake.get_object(kube.DAEMONSETS, "policy", NS) is None
                assert fake.get_object(kube.SERVICEACCOUNTS, "policy-sa", NS) is None
                assert fake.get_object(kube.ROLEBINDINGS, "policy-sa-rb", NS) is None
            await eventually(gone)
    run(body())


def test_status_tracks_targets_and_agent_readiness():
    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            for i in range(4):
                fake.add_node(f"gpu-node-{i}", {"foo": "bar"} if i < 3 else {"foo": "other"})
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy())

            def working():
                st = fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]
                assert st["targets"] == 3 and st["ready"] == 0 and st["state"] == "Working on it.."
                # per-node explanation from the agent pods' Ready condition
                assert st["errors"] == [f"gpu-node-{i}: scale-out not ready (ContainersNotReady)" for i in range(3)]
            await eventually(working)
            assert "serviceAccountName" not in fake.get_object(kube.DAEMONSETS, "policy", NS)["spec"]["template"]["spec"]
            for i in range(3):
                fake.set_agent_ready(f"gpu-node-{i}")

            def good():
                st = fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]
                assert st["ready"] == 3 and st["state"] == "All good" and st["errors"] == []
            await eventually(good)
            # a node loses its label file (agent not ready) -> back to working, with the node named
            fake.set_agent_ready("gpu-node-1", False)

            def one_down():
                st = fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]
                assert st["ready"] == 2 and st["errors"] == ["gpu-node-1: scale-out not ready (ContainersNotReady)"]
            await eventually(one_down)
            # a new matching node joins
            fake.set_node_labels("gpu-node-3", {"foo": "bar"})
            await eventually(lambda: fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]["targets"] == 4)
            events = [e for e in fake.list_objects(kube.EVENTS)]
            assert any(e["reason"] == "DaemonSetCreated" for e in events)
            assert any(e["reason"] == "AllNodesReady" for e in events)
            # Node readiness as the operator measured it: three Pods went Ready, one went unready.
            reg = ctl.metrics.registry
            assert reg.get_sample_value("amd_network_operator_agent_ready_seconds_count", {"policy": "policy"}) == 3
            assert reg.get_sample_value("amd_network_operator_agent_ready_seconds_sum", {"policy": "policy"}) > 0
            assert reg.get_sample_value("amd_network_operator_agent_unready_total", {"policy": "policy"}) == 1
    run(body())


def test_manual_daemonset_drift_is_reverted():
    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy(mtu=9000))
            ds = await value(lambda: fake.get_object(kube.DAEMONSETS, "policy", NS))
            ds["spec"]["template"]["spec"]["containers"][0]["args"] = ["--hacked"]
            await client.replace(kube.DAEMONSETS, ds)
            await eventually(lambda: fake.get_object(kube.DAEMONSETS, "policy", NS)["spec"]["template"]["spec"]
                             ["containers"][0]["args"][0] == "--configure=true")
    run(body())


def test_status_conflict_is_retried_and_api_errors_back_off():
    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            fake.fail_next("PUT", r"/networkclusterpolicies/policy/status$", status=409, count=2, reason="Conflict")
            fake.fail_next("POST", r"/daemonsets$", status=500, count=2)
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy())
            await eventually(lambda: fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy").get("status", {})
                             .get("state") == "No targets", timeout=10)
            assert ctl.queue.retries_total >= 2
    run(body())


def test_watch_interruptions_and_compaction_recover():
    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy("a"))
            await value(lambda: fake.get_object(kube.DAEMONSETS, "a", NS))
            fake.drop_watches()
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy("b"))
            await value(lambda: fake.get_object(kube.DAEMONSETS, "b", NS))
            fake.compact()
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy("c"))
            await value(lambda: fake.get_object(kube.DAEMONSETS, "c", NS))
            assert ctl.policies.relists >= 2
    run(body())


def test_schema_validation_rejects_bad_specs():
    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        async with ApiClient(KubeConfig(host=url)) as client:
            bad = [
                ({"amdScaleOut": {"layer": "L4"}}, "Unsupported value"),
                ({"amdScaleOut": {"layer": "L3", "mtu": 100}}, "greater than or equal to 1500"),
                ({"amdScaleOut": {"layer": "L3", "mtu": 9001}}, "less than or equal to 9000"),
                ({"logLevel": 9}, "less than or equal to 8"),
                ({"amdScaleOut": {"layer": "L3", "pullPolicy": "Sometimes"}}, "Unsupported value"),
                ({"configurationType": "gaudi-so"}, "Unsupported value"),
            ]
            for i, (patch, msg) in enumerate(bad):
                p = policy(f"p{i}")
                for k, v in patch.items():
                    p["spec"][k] = v
                with pytest.raises(ApiError) as ei:
                    await client.create(kube.NETWORKCLUSTERPOLICIES, p)
                assert ei.value.status == 422 and msg in ei.value.message, ei.value.message
            p = policy("missing")
            del p["spec"]["configurationType"]
            with pytest.raises(ApiError):
                await client.create(kube.NETWORKCLUSTERPOLICIES, p)
            # unknown fields are pruned, not stored
            p = policy("pruned")
            p["spec"]["bogus"] = 1
            created = await client.create(kube.NETWORKCLUSTERPOLICIES, p)
            assert "bogus" not in created["spec"]
        await fake.stop()
    run(body())


def test_require_full_pcie_link_reaches_the_agent():
    from network_operator_amd.operator import reconciler as R

    hn = T.new_host_nic_policy("h", layer="L2", minLinkSpeedGbps=200, requireFullPcieLink=True)
    assert {"--require-full-pcie", "--min-link-speed-gbps=200"} <= set(R.host_nic_agent_args(hn))
    assert T.NetworkClusterPolicy.from_dict(hn.to_dict()).spec.hostNic.requireFullPcieLink is True
    p = T.new_policy("x", layer="L2", requireFullPcieLink=True)
    assert "--require-full-pcie" in agent_args(p)
    assert "--require-full-pcie" not in agent_args(T.new_policy("x", layer="L2"))
    assert T.NetworkClusterPolicy.from_dict(p.to_dict()).spec.amdScaleOut.requireFullPcieLink is True


def test_allow_policy_routed_reaches_the_agent_from_either_policy_type():
    """The agent's refusal of a policy-routed NIC that holds the node's address names its opt-in;
    the policy carries it (amdScaleOut / hostNic.allowPolicyRouted), off by default."""
    from network_operator_amd.operator import reconciler as R

    from network_operator_amd.api.v1alpha1 import webhook as W

    p = T.new_policy("x", layer="L3", allowPolicyRouted=True)
    assert "--allow-policy-routed" in agent_args(p)
    assert W.validate_create(p) == [W.ALLOW_POLICY_ROUTED_WARNING]  # said at kubectl apply
    assert T.NetworkClusterPolicy.from_dict(p.to_dict()).spec.amdScaleOut.allowPolicyRouted is True
    assert "--allow-policy-routed" not in agent_args(T.new_policy("x", layer="L3"))
    hn = T.new_host_nic_policy("h", layer="L3", allowPolicyRouted=True)
    assert "--allow-policy-routed" in R.host_nic_agent_args(hn)
    assert T.NetworkClusterPolicy.from_dict(hn.to_dict()).spec.hostNic.allowPolicyRouted is True
    assert "--allow-policy-routed" not in R.host_nic_agent_args(T.new_host_nic_policy("h", layer="L3"))


def test_agent_args_mi355x_options():
    p = T.new_policy("x", layer="L3", xgmiCheck=True, lldpAnnounce=False, interfaces=["ens1", "ens2"],
                     nicDrivers=["mlx5_core"])
    a = agent_args(p)
    assert a[-7:] == ["--xgmi-expect=0", "--require-rdma", "--lldp-announce=false", "--interfaces=ens1,ens2",
                      "--nic-drivers=mlx5_core", LINK_STATE_ARG, STATUS_ARG]


def test_xgmi_check_and_require_rdma_are_on_unless_the_policy_turns_them_off():
    """MI355X-first: unset means on -- a policy stored before the fields
    existed, or written without them, still verifies the mesh and waits for RDMA devices."""
    assert "--xgmi-expect=0" in agent_args(T.new_policy("x")) and "--require-rdma" in agent_args(T.new_policy("x"))
    off = agent_args(T.new_policy("x", xgmiCheck=False, requireRdma=False, rdmaWait="10m"))
    assert not any(a.startswith(("--xgmi-expect", "--require-rdma", "--rdma-wait")) for a in off), off
    assert "--rdma-wait=10m" in agent_args(T.new_policy("x", rdmaWait="10m"))


def test_leader_election_single_active_and_failover():
    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        c1, c2 = ApiClient(KubeConfig(host=url)), ApiClient(KubeConfig(host=url))
        e1 = LeaderElector(c1, NS, identity="one", lease_duration=0.6, renew_deadline=0.4, retry_period=0.1)
        e2 = LeaderElector(c2, NS, identity="two", lease_duration=0.6, renew_deadline=0.4, retry_period=0.1,
                           release_on_cancel=False)
        leading = []
        stop1 = asyncio.Event()

        async def work(name, stop):
            leading.append(name)
            await stop.wait()

        t1 = asyncio.ensure_future(e1.run(lambda: work("one", stop1)))
        await eventually(lambda: leading == ["one"])
        stop2 = asyncio.Event()
        t2 = asyncio.ensure_future(e2.run(lambda: work("two", stop2)))
        await asyncio.sleep(1.0)
        assert leading == ["one"]  # lease held and renewed
        lease = fake.get_object(kube.LEASES, "9a8a7ba6.amd.com", NS)
        assert lease["spec"]["holderIdentity"] == "one"
        # leader 1 stops voluntarily -> releases -> 2 takes over quickly
        stop1.set()
        await t1
        await eventually(lambda: leading == ["one", "two"], timeout=5)
        lease = fake.get_object(kube.LEASES, "9a8a7ba6.amd.com", NS)
        assert lease["spec"]["holderIdentity"] == "two" and lease["spec"]["leaseTransitions"] >= 1
        stop2.set()
        await t2
        await c1.close()
        await c2.close()
        await fake.stop()
    run(body())


def test_leader_election_timings_are_flags_and_checked(monkeypatch):
    """``--leader-elect-{lease-duration,renew-deadline,retry-period}`` reach the elector; an
    order that client-go would reject (lease <= renew deadline) stops the manager."""
    from network_operator_amd.operator import manager

    opts = manager.build_parser().parse_args(["--leader-elect-lease-duration=4", "--leader-elect-renew-deadline=3",
                                              "--leader-elect-retry-period=0.5"])
    assert (opts.leader_elect_lease_duration, opts.leader_elect_renew_deadline,
            opts.leader_elect_retry_period) == (4, 3, 0.5)
    monkeypatch.setenv("ENABLE_WEBHOOKS", "false")

    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        rc = await manager.run(["--master", url, "--health-probe-bind-address=0", "--dependency-check-interval=0",
                                "--leader-elect", "--leader-elect-lease-duration=2",
                                "--leader-elect-renew-deadline=2"])
        await fake.stop()
        return rc
    assert run(body()) == 1


def test_fake_api_server_semantics():
    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        async with ApiClient(KubeConfig(host=url)) as c:
            sa = {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": "x", "labels": {"a": "1"}}}
            o = await c.create(kube.SERVICEACCOUNTS, sa, namespace="ns1")
            with pytest.raises(ApiError) as ei:
                await c.create(kube.SERVICEACCOUNTS, sa, namespace="ns1")
            assert kube.is_already_exists(ei.value)
            stale = dict(o)
            o["metadata"]["labels"]["b"] = "2"
            o2 = await c.replace(kube.SERVICEACCOUNTS, o)
            assert int(o2["metadata"]["resourceVersion"]) > int(o["metadata"]["resourceVersion"])
            stale["metadata"] = dict(stale["metadata"], labels={"z": "9"}, resourceVersion=o["metadata"]["resourceVersion"])
            with pytest.raises(ApiError) as ei:
                await c.replace(kube.SERVICEACCOUNTS, stale)
            assert kube.is_conflict(ei.value)
            assert len((await c.list(kube.SERVICEACCOUNTS, "ns1", label_selector="a=1,b=2"))["items"]) == 1
            assert len((await c.list(kube.SERVICEACCOUNTS, "ns1", label_selector="a=2"))["items"]) == 0
            p = await c.patch(kube.SERVICEACCOUNTS, "x", {"metadata": {"labels": {"a": None}}}, namespace="ns1")
            assert p["metadata"]["labels"] == {"b": "2"}
            p = await c.patch(kube.SERVICEACCOUNTS, "x", [{"op": "add", "path": "/metadata/labels/c", "value": "3"}],
                              namespace="ns1", patch_type="json")
            assert p["metadata"]["labels"] == {"b": "2", "c": "3"}
            groups = await c.server_groups()
            assert "amd.com" in groups and "route.openshift.io" not in groups
            # watch replays from a resourceVersion
            seen = []
            async for typ, obj in c.watch(kube.SERVICEACCOUNTS, "ns1", resource_version="1", timeout_seconds=1):
                seen.append(typ)
            assert seen[:3] == ["ADDED", "MODIFIED", "MODIFIED"]
        await fake.stop()
    run(body())


def test_agent_args_fw_lldp_and_metrics_port():
    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.discovery import discovery_daemonset as daemonset
    from network_operator_amd.operator.reconciler import agent_args, update_amd_scale_out_daemonset

    p = T.new_policy("p", layer="L3")
    p.spec.amdScaleOut.disableFirmwareLldp = True
    p.spec.amdScaleOut.metricsPort = 9102
    args = agent_args(p)
    assert "--disable-fw-lldp" in args and "--metrics-bind-address=:9102" in args
    ds = daemonset()
    update_amd_scale_out_daemonset(ds, p, "ns")
    c = ds["spec"]["template"]["spec"]["containers"][0]
    assert c["ports"] == [{"name": "metrics", "containerPort": 9102, "protocol": "TCP"}]
    p.spec.amdScaleOut.metricsPort = 0
    p.spec.amdScaleOut.layer = "L2"
    update_amd_scale_out_daemonset(ds, p, "ns")
    assert "ports" not in c and "--disable-fw-lldp" not in c["args"]
    assert T.NetworkClusterPolicy.from_dict(p.to_dict()).spec.amdScaleOut.disableFirmwareLldp
    # keepConfigOnRestart: the firmware LLDP originals stay recorded on the node across restarts,
    # and the node's cleanup Job (same args, --cleanup) restores them.
    from network_operator_amd.operator.reconciler import cleanup_job

    p.spec.amdScaleOut.layer = "L3"
    state = "--fw-lldp-state=/host/etc/amd/scale-out/fw-lldp-state"
    assert state in agent_args(p)  # a record left by keepConfigOnRestart agents is restored on exit
    p.spec.amdScaleOut.keepConfigOnRestart = True
    assert state in agent_args(p)
    assert state in cleanup_job(p, "n1", "ns")["spec"]["template"]["spec"]["containers"][0]["args"]
    p.spec.amdScaleOut.disableFirmwareLldp = False
    assert not any(a.startswith("--fw-lldp-state") for a in agent_args(p))


def test_agent_args_gpudirect_rdma():
    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.operator.reconciler import agent_args

    p = T.new_policy("p", layer="L3")
    p.spec.amdScaleOut.gpuDirectRdma = "PeerMem"
    assert "--require-gdr=peermem" in agent_args(p)
    assert T.NetworkClusterPolicy.from_dict(p.to_dict()).spec.amdScaleOut.gpuDirectRdma == "PeerMem"


def test_host_nic_daemonset_branch():
    """configurationType host-nic (the reference's future-work branch): RDMA NIC discovery, its own
    label/file + readinessProbe, optional privileged KMD init container; switching back cleans up."""
    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.discovery import discovery_daemonset
    from network_operator_amd.operator.reconciler import update_daemonset_for

    p = T.new_host_nic_policy("storage", layer="L3", mtu=9000, nicDrivers=["mlx5_core"],
                              driverImage="registry/nic-kmd:6.8", pullPolicy="Always")
    ds = discovery_daemonset()
    update_daemonset_for(ds, p, "ns")
    pod = ds["spec"]["template"]["spec"]
    c = pod["containers"][0]
    assert c["args"][:6] == ["--configure=true", "--keep-running", "--mode=L3", "--nic-discovery=rdma",
                             "--nfd-label-file=host-nic-readiness.txt",
                             "--nfd-label=amd.feature.node.kubernetes.io/host-nic-ready"]
    assert "--mtu=9000" in c["args"] and "--nic-drivers=mlx5_core" in c["args"] and "--wait=90s" in c["args"]
    assert not any(a.startswith("--rccl-net") for a in c["args"])
    assert c["readinessProbe"]["exec"]["command"][1:] == ["--ready-check", "--nfd-label-file=host-nic-readiness.txt",
                                                          STATUS_ARG]
    init = pod["initContainers"][0]
    assert init["name"] == "nic-driver" and init["securityContext"]["privileged"] and init["imagePullPolicy"] == "Always"
    assert any(v["name"] == "host-lib-modules" for v in pod["volumes"])
    # Explicit interfaces: no discovery, just those.
    p.spec.hostNic.interfaces = ["ens1f0np0"]
    p.spec.hostNic.driverImage = ""
    update_daemonset_for(ds, p, "ns")
    assert "--nic-discovery=none" in c["args"] and "--interfaces=ens1f0np0" in c["args"]
    assert "initContainers" not in pod and all(v["name"] != "host-lib-modules" for v in pod["volumes"])
    # Back to amd-so: default probe, scale-out args.
    q = T.new_policy("storage", layer="L3")
    update_daemonset_for(ds, q, "ns")
    assert c["readinessProbe"]["exec"]["command"][1:] == ["--ready-check", STATUS_ARG]
    assert any(a.startswith("--rccl-net") for a in c["args"])


def test_host_nic_webhook_rules():
    import pytest

    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.api.v1alpha1 import webhook as W

    p = T.new_host_nic_policy("h", layer="L2")
    W.default(p)
    assert p.spec.hostNic.image == T.DEFAULT_AGENT_IMAGE
    assert W.validate_create(p)  # warning: no interfaces / drivers
    p.spec.hostNic = None
    with pytest.raises(W.MissingHostNicSpecError):
        W.validate_create(p)
    rt = T.NetworkClusterPolicy.from_dict(T.new_host_nic_policy("h", driverImage="x").to_dict())
    assert rt.spec.configurationType == "host-nic" and rt.spec.hostNic.driverImage == "x"


def test_rccl_env_extra_settings_validated_and_passed():
    import pytest

    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.api.v1alpha1 import webhook as W
    from network_operator_amd.operator.reconciler import agent_args

    p = T.new_policy("p", layer="L3")
    p.spec.amdScaleOut.rcclEnv = {"NCCL_IB_TC": "106", "NCCL_IB_QPS_PER_CONNECTION": "4"}
    assert W.validate_create(p) == []
    assert "--rccl-env-extra=NCCL_IB_QPS_PER_CONNECTION=4,NCCL_IB_TC=106" in agent_args(p)
    p.spec.amdScaleOut.rcclEnv = {"LD_PRELOAD": "/x.so"}
    with pytest.raises(W.InvalidRcclEnvError):
        W.validate_create(p)
    p.spec.amdScaleOut.rcclEnv = {"NCCL_DEBUG": "INFO,WARN"}
    with pytest.raises(W.InvalidRcclEnvError):
        W.validate_create(p)


def test_lldp_wait_validated_and_passed():
    """amdScaleOut.lldpWait / hostNic.lldpWait: the agent's --wait (the reference fixes 90s,
    controller.go:198); a Go duration, 1s..30m, checked by the CRD pattern and the webhook."""
    from network_operator_amd.api.v1alpha1 import crd as CRD
    from network_operator_amd.api.v1alpha1 import webhook as W
    from network_operator_amd.operator.reconciler import host_nic_agent_args

    p = T.new_policy("p", layer="L3")
    assert "--wait=90s" in agent_args(p)
    for value, secs in (("5s", 5), ("1m30s", 90), ("1.5s", 1.5), ("30m", 1800), ("1000ms", 1)):
        p.spec.amdScaleOut.lldpWait = value
        assert T.parse_go_duration(value) == pytest.approx(secs)
        assert W.validate_create(p) == [] and f"--wait={value}" in agent_args(p)
        d = p.to_dict()
        assert d["spec"]["amdScaleOut"]["lldpWait"] == value and CRD.validate(d) == []
        assert T.NetworkClusterPolicy.from_dict(d).spec.amdScaleOut.lldpWait == value
    for bad in ("500ms", "31m", "2h", "90", "1d", "-5s", " 5s"):
        p.spec.amdScaleOut.lldpWait = bad
        with pytest.raises(W.InvalidLldpWaitError):
            W.validate_create(p)
    p.spec.amdScaleOut.lldpWait = "90"
    assert CRD.validate(p.to_dict())  # the schema pattern refuses it too
    p.spec.amdScaleOut.lldpWait, p.spec.amdScaleOut.layer = "5s", "L2"
    assert W.validate_create(p) == ["lldpWait has no effect in L2 mode"]
    assert not any(a.startswith("--wait") for a in agent_args(p))
    # lldpAnnounce likewise (the agent announces only in L3), whatever xgmiCheck says
    p.spec.amdScaleOut.lldpWait = ""
    for xgmi in (None, True, False):
        p.spec.amdScaleOut.lldpAnnounce, p.spec.amdScaleOut.xgmiCheck = False, xgmi
        assert W.validate_create(p) == ["lldpAnnounce has no effect in L2 mode"]
    p.spec.amdScaleOut.layer = "L3"
    assert W.validate_create(p) == []
    h = T.new_host_nic_policy("h", layer="L3", lldpWait="20s")
    assert "--wait=20s" in host_nic_agent_args(h) and W.validate_create(h) == [
        "hostNic: no interfaces or nicDrivers given; every RDMA NIC of the default driver list that is neither a "
        "GPU's scale-out rail nor the node's own NIC (default route, non-/30 address) will be configured"]
    assert T.NetworkClusterPolicy.from_dict(h.to_dict()).spec.hostNic.lldpWait == "20s"
    h.spec.hostNic.lldpWait = "0s"
    with pytest.raises(W.InvalidLldpWaitError):
        W.validate_create(h)


def test_status_conditions_ready_degraded_and_observed_generation():
    """Additive status: Ready / Degraded conditions with stable lastTransitionTime, and
    observedGeneration following spec changes (the reference only has the state string)."""
    from network_operator_amd.operator.reconciler import policy_conditions

    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            for i in range(2):
                fake.add_node(f"gpu-node-{i}", {"foo": "bar"})
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy())

            def conds():
                st = fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]
                return st, {c["type"]: c for c in st.get("conditions", [])}

            def not_ready():
                st, c = conds()
                assert c["Ready"]["status"] == "False" and c["Ready"]["reason"] == "NodesNotReady"
                # agents running, not probed yet: nodes starting up, not a degradation
                assert c["Degraded"]["status"] == "False" and c["Degraded"]["reason"] == "AsExpected"
                assert st["observedGeneration"] == 1 and c["Ready"]["observedGeneration"] == 1
                assert len(st["errors"]) == 2
            await eventually(not_ready)
            fake.record_probe_failure(NS, "policy-gpu-node-1", "Readiness probe failed: not ready: ens1: waiting for carrier")
            await eventually(lambda: any("waiting for carrier" in e for e in conds()[0]["errors"]))
            assert conds()[1]["Degraded"]["status"] == "False"  # a start-up reason
            fake.record_probe_failure(NS, "policy-gpu-node-1", "Readiness probe failed: not ready: ens1: link down")

            def degraded():
                st, c = conds()
                assert c["Degraded"]["status"] == "True" and c["Degraded"]["reason"] == "AgentErrors"
                assert "ens1: link down" in c["Degraded"]["message"] and "gpu-node-0" not in c["Degraded"]["message"]
            await eventually(degraded)
            degraded_since = conds()[1]["Degraded"]["lastTransitionTime"]
            fake.set_agent_ready("gpu-node-0")

            def one_ready():
                st, c = conds()
                assert st["ready"] == 1 and c["Ready"]["message"] == "1/2 nodes configured"
            await eventually(one_ready)
            assert conds()[1]["Degraded"]["lastTransitionTime"] == degraded_since  # no flip, no move
            fake.set_agent_ready("gpu-node-1")

            def ready():
                st, c = conds()
                assert c["Ready"]["status"] == "True" and c["Ready"]["reason"] == "AllNodesReady"
                assert c["Degraded"]["status"] == "False" and c["Degraded"]["reason"] == "AsExpected"
            await eventually(ready)
            await edit(client, "policy", lambda cur: cur["spec"]["amdScaleOut"].update(mtu=4000))
            await eventually(lambda: conds()[0]["observedGeneration"] == 2)
    run(body())
    # No targets; a missing dependency is reported as such.
    c = {x["type"]: x for x in policy_conditions([], 0, 0, ["dependency missing: node-feature-discovery"], 3, "T0")}
    assert c["Ready"]["reason"] == "NoTargets" and c["Degraded"]["reason"] == "DependencyMissing"
    assert c["Ready"]["lastTransitionTime"] == "T0" and c["Ready"]["observedGeneration"] == 3


def test_agent_args_rail_tables_l3_only():
    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.operator.reconciler import agent_args

    p = T.new_policy("p", layer="L3")
    assert not any(a.startswith("--rail-table-base") for a in agent_args(p))
    p.spec.amdScaleOut.railTableBase = 100
    assert "--rail-table-base=100" in agent_args(p)
    assert T.NetworkClusterPolicy.from_dict(p.to_dict()).spec.amdScaleOut.railTableBase == 100
    p.spec.amdScaleOut.layer = "L2"  # no addresses in L2: nothing to route
    assert not any(a.startswith("--rail-table-base") for a in agent_args(p))


def test_agent_args_verify_peers_l3_only():
    from network_operator_amd.api.v1alpha1 import crd as CRD
    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.operator.reconciler import agent_args, host_nic_agent_args

    p = T.new_policy("p", layer="L3")
    assert not any(a.startswith("--verify-peers") for a in agent_args(p))
    p.spec.amdScaleOut.verifyPeers = True
    assert "--verify-peers=2s" in agent_args(p)
    d = p.to_dict()
    assert d["spec"]["amdScaleOut"]["verifyPeers"] is True and CRD.validate(d) == []
    assert T.NetworkClusterPolicy.from_dict(d).spec.amdScaleOut.verifyPeers is True
    p.spec.amdScaleOut.layer = "L2"  # no /30 in L2: no peer address to ask
    assert not any(a.startswith("--verify-peers") for a in agent_args(p))
    h = T.new_host_nic_policy("h", layer="L3", verifyPeers=True)
    assert "--verify-peers=2s" in host_nic_agent_args(h)
    assert T.NetworkClusterPolicy.from_dict(h.to_dict()).spec.hostNic.verifyPeers is True
    assert CRD.validate(h.to_dict()) == []


def test_fabric_validation_jobs_follow_ready_nodes_and_report_a_condition():
    """amdScaleOut.validation: one validation Job per node whose agent is ready, pinned to it, for
    the policy's current generation; the outcome is the FabricValidated condition."""
    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            for i in range(2):
                fake.add_node(f"gpu-node-{i}", {"foo": "bar"})
            await client.create(kube.NETWORKCLUSTERPOLICIES,
                                policy(validation={"enabled": True, "minBusbw": 300, "gpus": 8}))
            await eventually(lambda: fake.get_object(kube.DAEMONSETS, "policy", NS) is not None)
            fake.set_agent_ready("gpu-node-0")

            def jobs():
                return {j["metadata"]["annotations"]["amd.com/node"]: j for j in fake.list_objects(kube.JOBS)}

            await eventually(lambda: set(jobs()) == {"gpu-node-0"})  # only ready nodes are validated
            j = jobs()["gpu-node-0"]
            spec = j["spec"]["template"]["spec"]
            assert spec["nodeName"] == "gpu-node-0" and spec["restartPolicy"] == "Never"
            c = spec["containers"][0]
            assert c["command"] == ["python3", "-m", "network_operator_amd.validate"]
            assert "--min-busbw=300" in c["args"] and "--gpus=8" in c["args"]
            assert c["resources"]["limits"] == {"amd.com/gpu": 8}
            assert j["metadata"]["ownerReferences"][0]["kind"] == "NetworkClusterPolicy"

            def cond():
                st = fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy").get("status") or {}
                return {c["type"]: c for c in st.get("conditions", [])}.get("FabricValidated")

            await eventually(lambda: cond() and cond()["status"] == "Unknown")
            fake.set_agent_ready("gpu-node-1")
            await eventually(lambda: set(jobs()) == {"gpu-node-0", "gpu-node-1"})
            fake.set_job_result(jobs()["gpu-node-0"]["metadata"]["name"], NS, True)
            fake.set_job_result(jobs()["gpu-node-1"]["metadata"]["name"], NS, False)

            def failed():
                st = fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]
                c = cond()
                return c["status"] == "False" and c["reason"] == "ValidationFailed" and \
                    "gpu-node-1: fabric validation failed" in st["errors"]
            await eventually(failed)

            # A new spec (generation 2): the old results go, both nodes are validated again.
            old_names = {j["metadata"]["name"] for j in jobs().values()}
            await edit(client, "policy", lambda cur: cur["spec"]["amdScaleOut"].update(mtu=4200))
            await eventually(lambda: set(jobs()) == {"gpu-node-0", "gpu-node-1"}
                             and not old_names & {j["metadata"]["name"] for j in jobs().values()})
            for j in jobs().values():
                fake.set_job_result(j["metadata"]["name"], NS, True)
            await eventually(lambda: cond()["status"] == "True" and cond()["reason"] == "AllNodesValidated")
            st = fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]
            assert st["state"] == "All good" and st["errors"] == []

            # Validation off: no Jobs, no condition.
            await edit(client, "policy", lambda cur: cur["spec"]["amdScaleOut"].update(validation={"enabled": False}))
            await eventually(lambda: cond() is None and not fake.list_objects(kube.JOBS))
    run(body())


def test_validation_job_not_admitted_is_retried_and_a_new_agent_readiness_revalidates():
    """a validation Pod the kubelet refused (GPUs allocated to workloads:
    OutOfamd.com/gpu) is not a fabric verdict: reported as not admitted and re-created after a
    back-off.  A genuine failure stays until the node's agent becomes ready again (restart or
    cleared fault), which validates the node again.  A persisting failure does not rewrite the
    policy status on every reconcile."""
    from network_operator_amd.operator.reconciler import AGENT_EPOCH_ANN, ATTEMPT_ANN

    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            fake.add_node("gpu-node-0", {"foo": "bar"})
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy(validation={"enabled": True}))
            await eventually(lambda: fake.get_object(kube.DAEMONSETS, "policy", NS) is not None)
            fake.set_agent_ready("gpu-node-0")
            await eventually(lambda: len(fake.list_objects(kube.JOBS)) == 1)

            def cond():
                st = fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy").get("status") or {}
                return {c["type"]: c for c in st.get("conditions", [])}.get("FabricValidated") or {}

            # 1. Not admitted just now: reported, not a failure, retry pending.
            j0 = fake.list_objects(kube.JOBS)[0]
            fake.set_job_result(j0["metadata"]["name"], NS, False, pod_reason="OutOfamd.com/gpu",
                                pod_message="Node didn't have enough resource: amd.com/gpu")
            await eventually(lambda: cond().get("reason") == "ValidationNotAdmitted")
            st = fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]
            assert cond()["status"] == "Unknown" and "OutOfamd.com/gpu" in cond()["message"]
            assert "retrying in" in cond()["message"] and st["errors"] == []
            assert [j["metadata"]["name"] for j in fake.list_objects(kube.JOBS)] == [j0["metadata"]["name"]]
            # 2. Its back-off has passed (it failed long ago): a new attempt replaces it.
            fake.set_job_result(j0["metadata"]["name"], NS, False, pod_reason="OutOfamd.com/gpu",
                                finished="2000-01-01T00:00:00Z")
            await eventually(lambda: [j["metadata"]["annotations"][ATTEMPT_ANN] for j in fake.list_objects(kube.JOBS)]
                             == ["1"])
            j1 = fake.list_objects(kube.JOBS)[0]
            assert j1["metadata"]["name"] != j0["metadata"]["name"]
            assert j1["metadata"]["annotations"][AGENT_EPOCH_ANN] == j0["metadata"]["annotations"][AGENT_EPOCH_ANN]
            # 3. A genuine failure: reported, and the status is not rewritten while nothing changes.
            fake.set_job_result(j1["metadata"]["name"], NS, False)
            await eventually(lambda: cond().get("reason") == "ValidationFailed")
            assert fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]["errors"] == [
                "gpu-node-0: fabric validation failed"]
            # the controller's cache has the stored status (a reconcile on a stale cache would send
            # a write the API server refuses with a conflict, which still counts as a request)
            rv = fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["metadata"]["resourceVersion"]
            await eventually(lambda: ((ctl.policies.get("policy") or {}).get("metadata") or {}).get("resourceVersion")
                             == rv)
            await asyncio.sleep(0.2)
            writes = sum(1 for m, path in fake.requests if m == "PUT" and path.endswith("/status"))
            for _ in range(5):  # unrelated events: every one reconciles the policy
                await ctl.requeue_all()
                await asyncio.sleep(0.05)
            assert sum(1 for m, path in fake.requests if m == "PUT" and path.endswith("/status")) == writes
            # 4. The agent restarts (not ready, then ready again): the node is validated again.
            fake.set_agent_ready("gpu-node-0", False)
            await eventually(lambda: fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]["ready"] == 0)
            fake.set_agent_ready("gpu-node-0")
            await eventually(lambda: [j["metadata"]["name"] for j in fake.list_objects(kube.JOBS)] not in
                             ([], [j1["metadata"]["name"]]))
            j2 = fake.list_objects(kube.JOBS)[0]
            assert j2["metadata"]["annotations"][AGENT_EPOCH_ANN] != j1["metadata"]["annotations"][AGENT_EPOCH_ANN]
            await eventually(lambda: cond().get("reason") == "ValidationRunning")
            fake.set_job_result(j2["metadata"]["name"], NS, True)
            await eventually(lambda: cond().get("status") == "True")
            assert fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]["errors"] == []
    run(body())


def test_agent_exit_reason_quotes_the_agents_error_line():
    """The DaemonSet keeps a failed agent's log tail as its termination message
    (FallbackToLogsOnError); the policy's errors quote the agent's "Error: ..." line."""
    from network_operator_amd import discovery
    from network_operator_amd.operator.reconciler import agent_exit_reason

    c = discovery.discovery_daemonset()["spec"]["template"]["spec"]["containers"][0]
    assert c["terminationMessagePolicy"] == "FallbackToLogsOnError"
    msg = ("I1017 00:31:06.157259 3794 agent.cpp:1040] xGMI: 8 GPUs\n"
           "W1017 00:31:08.1 3794 agent.cpp:1407] interface 'ens2': peer 10.200.0.9 did not answer ARP\n"
           "Error: 1 of 8 switch-side peers did not answer ARP (ens2: peer 10.200.0.9 did not answer ARP)\n")
    pod = {"status": {"containerStatuses": [{"name": "configurator", "restartCount": 3, "lastState": {
        "terminated": {"exitCode": 1, "reason": "Error", "message": msg}}}]}}
    assert agent_exit_reason(pod) == "1 of 8 switch-side peers did not answer ARP (ens2: peer 10.200.0.9 did not answer ARP)"
    pod["status"]["containerStatuses"][0]["lastState"]["terminated"] = {"exitCode": 137, "reason": "OOMKilled"}
    assert agent_exit_reason(pod) == "agent exited with code 137 (OOMKilled)"
    assert agent_exit_reason({"status": {"containerStatuses": [{"name": "configurator", "ready": False}]}}) is None
    assert agent_exit_reason({"status": {}}) is None


def test_agent_exit_reason_reaches_status_and_events():
    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            fake.add_node("gpu-node-0", {"foo": "bar"})
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy())
            await eventually(lambda: fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]["targets"] == 1)
            fake.set_agent_ready("gpu-node-0", False, terminated={
                "exitCode": 1, "reason": "Error",
                "message": "E1017 agent.cpp:1283] boom\nError: No LLDP peers with a /30 Port Description were found\n"})
            want = ("gpu-node-0: scale-out not ready (ContainersNotReady): "
                    "No LLDP peers with a /30 Port Description were found")

            def reported():
                assert fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]["errors"] == [want]
                ev = [e for e in fake.list_objects(kube.EVENTS) if e["reason"] == "AgentFailed"]
                assert len(ev) == 1 and ev[0]["type"] == "Warning" and ev[0]["message"] == want
            await eventually(reported)
            pod = [p for p in fake.list_objects(kube.PODS)][0]
            assert pod["status"]["containerStatuses"][0]["restartCount"] == 0
            fake.set_agent_ready("gpu-node-0")
            await eventually(lambda: fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]["errors"] == [])
    run(body())


def test_keep_config_policy_cleans_nodes_through_jobs_on_deletion_and_departure(monkeypatch):
    """keepConfigOnRestart: agents run with --keep-config (and the LLDP cache that lets the next
    agent adopt the addresses).  The operator records the nodes it configured, and owes each a
    cleanup Job (the agent with --cleanup, pinned to the node): when the node leaves the policy,
    after a grace period, and when the policy is deleted, which its finalizer holds until then."""
    from network_operator_amd.operator import reconciler as R

    monkeypatch.setattr(R, "KEPT_ORPHAN_GRACE_S", 0.3)
    monkeypatch.setattr(R, "CLEANUP_POLL_S", 0.05)

    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            for i in range(3):
                fake.add_node(f"gpu-node-{i}", {"foo": "bar"})
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy(keepConfigOnRestart=True))
            plain = policy("plain")  # on other nodes: two amd-so policies never share one
            plain["spec"]["nodeSelector"] = {"foo": "elsewhere"}
            await client.create(kube.NETWORKCLUSTERPOLICIES, plain)
            await eventually(lambda: fake.get_object(kube.DAEMONSETS, "policy", NS) is not None)
            args = fake.get_object(kube.DAEMONSETS, "policy", NS)["spec"]["template"]["spec"]["containers"][0]["args"]
            assert "--keep-config" in args and "--lldp-cache=/host/etc/amd/scale-out/lldp-cache" in args
            for i in range(3):
                fake.set_agent_ready(f"gpu-node-{i}", daemonset=f"{NS}/policy")

            def pol(name="policy"):
                return fake.get_object(kube.NETWORKCLUSTERPOLICIES, name)
            await eventually(lambda: pol()["status"].get("keptNodes") == [f"gpu-node-{i}" for i in range(3)])
            assert pol()["metadata"]["finalizers"] == [R.FINALIZER]
            assert not pol("plain")["metadata"].get("finalizers") and "keptNodes" not in pol("plain")["status"]
            await eventually(lambda: ctl.metrics.registry.get_sample_value(
                "amd_network_operator_nodes_owing_cleanup", {"policy": "policy"}) == 3)

            # gpu-node-2 leaves the policy: its agent Pod goes; after the grace period, a cleanup Job
            fake.set_node_labels("gpu-node-2", {"foo": "other"})
            job = await value(lambda: next(iter(fake.list_objects(kube.JOBS)), None), timeout=5)
            spec = job["spec"]["template"]["spec"]
            c = spec["containers"][0]
            assert spec["nodeName"] == "gpu-node-2" and spec["restartPolicy"] == "Never" and spec["hostNetwork"]
            assert "--cleanup" in c["args"] and "--keep-running" not in c["args"] and "--keep-config" not in c["args"]
            assert "readinessProbe" not in c and "nodeSelector" not in spec
            assert job["metadata"]["ownerReferences"][0]["name"] == "policy"
            await asyncio.sleep(0.2)
            assert pol()["status"]["keptNodes"] == [f"gpu-node-{i}" for i in range(3)]  # owed until it ran
            fake.set_job_result(job["metadata"]["name"], NS, True)
            await eventually(lambda: pol()["status"].get("keptNodes") == ["gpu-node-0", "gpu-node-1"])
            await eventually(lambda: fake.list_objects(kube.JOBS) == [])

            # deletion: the finalizer holds the policy until both remaining nodes ran their cleanup
            await client.delete(kube.NETWORKCLUSTERPOLICIES, "policy")
            await eventually(lambda: fake.get_object(kube.DAEMONSETS, "policy", NS) is None)
            await eventually(lambda: sorted(j["spec"]["template"]["spec"]["nodeName"]
                                            for j in fake.list_objects(kube.JOBS)) == ["gpu-node-0", "gpu-node-1"])
            assert pol()["metadata"]["deletionTimestamp"]
            for j in fake.list_objects(kube.JOBS):
                fake.set_job_result(j["metadata"]["name"], NS, j["spec"]["template"]["spec"]["nodeName"] == "gpu-node-0")
            await eventually(lambda: pol() is None)
            ev = [e for e in fake.list_objects(kube.EVENTS) if e["reason"] == "NodeCleanupFailed"]
            assert len(ev) == 1 and ev[0]["message"].startswith("gpu-node-1: cleanup Job")
            reg = ctl.metrics.registry
            assert reg.get_sample_value("amd_network_operator_node_cleanups_total",
                                        {"policy": "policy", "outcome": "succeeded"}) == 2
            assert reg.get_sample_value("amd_network_operator_node_cleanups_total",
                                        {"policy": "policy", "outcome": "failed"}) == 1
            assert pol("plain") is not None
            await client.delete(kube.NETWORKCLUSTERPOLICIES, "plain")  # no finalizer: gone at once
            assert pol("plain") is None
    run(body())


def test_network_manager_is_handed_back_when_the_policy_goes():
    """disableNetworkManager keeps the NICs unmanaged across agent restarts: the
    hand-back happens once, when the policy is deleted: a cleanup Job with --nm-restore per node
    that ran the agent, held by the node-cleanup finalizer.  host-nic policies alike."""
    from network_operator_amd.operator import reconciler as R

    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            fake.add_node("gpu-node-0", {"foo": "bar"})
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy(disableNetworkManager=True))
            hn = T.new_host_nic_policy("hosts", layer="L2", node_selector={"foo": "bar"}, disableNetworkManager=True)
            await client.create(kube.NETWORKCLUSTERPOLICIES, hn.to_dict())
            for name in ("policy", "hosts"):
                await eventually(lambda: fake.get_object(kube.DAEMONSETS, name, NS) is not None)
                fake.set_agent_ready("gpu-node-0", daemonset=f"{NS}/{name}")
            for name in ("policy", "hosts"):
                await eventually(lambda: (fake.get_object(kube.NETWORKCLUSTERPOLICIES, name).get("status") or {})
                                 .get("keptNodes") == ["gpu-node-0"])
                assert fake.get_object(kube.NETWORKCLUSTERPOLICIES, name)["metadata"]["finalizers"] == [R.FINALIZER]
                await client.delete(kube.NETWORKCLUSTERPOLICIES, name)
                job = await value(lambda: next((j for j in fake.list_objects(kube.JOBS)
                                                if j["metadata"]["labels"]["amd.com/policy"] == name), None))
                args = job["spec"]["template"]["spec"]["containers"][0]["args"]
                assert "--cleanup" in args and "--nm-restore" in args and "--disable-networkmanager" in args
                if name == "hosts":  # its own label file, hence its own NetworkManager keyfile
                    assert "--nfd-label-file=host-nic-readiness.txt" in args
                fake.set_job_result(job["metadata"]["name"], NS, True)
                await eventually(lambda: fake.get_object(kube.NETWORKCLUSTERPOLICIES, name) is None)
    run(body())


def test_host_nic_keep_config_args_volume_and_cleanup():
    from network_operator_amd.operator import reconciler as R

    p = T.new_host_nic_policy("hosts", layer="L3", keepConfigOnRestart=True, nicDrivers=["mlx5_core"])
    args = R.host_nic_agent_args(p)
    assert args[-4:] == ["--lldp-cache=/host/etc/amd/scale-out/host-nic-lldp-cache", "--keep-config",
                         HOST_NIC_LINK_STATE_ARG, STATUS_ARG]
    assert R.keeps_config(p) and R.needs_node_cleanup(p)
    job = R.cleanup_job(p, "n0", NS)
    spec = job["spec"]["template"]["spec"]
    c = spec["containers"][0]
    assert "--cleanup" in c["args"] and "--keep-config" not in c["args"] and "--nm-restore" not in c["args"]
    assert "--nfd-label-file=host-nic-readiness.txt" in c["args"]  # its own lock, label and keyfile
    assert "rccl-artifacts" in [v["name"] for v in spec["volumes"]]
    assert HOST_NIC_LINK_STATE_ARG in c["args"]  # what no agent in memory saw goes back from the record
    l2 = T.new_host_nic_policy("hosts", layer="L2", keepConfigOnRestart=True)
    assert R.host_nic_agent_args(l2)[-3] == "--keep-config" and not any("lldp-cache" in a for a in R.host_nic_agent_args(l2))
    # The records live on the node whatever the policy says now: a policy that dropped mtu (or
    # keepConfigOnRestart) still mounts them for the next agent and the cleanup Job.
    ds = discovery.discovery_daemonset()
    R.update_daemonset_for(ds, T.new_host_nic_policy("hosts", layer="L2"), NS)
    assert "rccl-artifacts" in [v["name"] for v in ds["spec"]["template"]["spec"]["volumes"]]
    plain = T.new_host_nic_policy("hosts", layer="L3")
    assert not R.needs_node_cleanup(plain) and "--keep-config" not in R.host_nic_agent_args(plain)


def test_deleted_before_the_status_recorded_its_nodes_still_cleans_them():
    """A keepConfigOnRestart policy deleted before any status write listed its nodes: the
    finalizer first records every node with an agent Pod (ready or not), then removes the
    DaemonSet, so the cleanup Jobs cover nodes the status never mentioned."""
    from network_operator_amd.operator import reconciler as R

    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        try:
            for i in range(2):
                fake.add_node(f"gpu-node-{i}", {"foo": "bar"})
            async with ApiClient(KubeConfig(host=url)) as client:
                pol = policy(keepConfigOnRestart=True)
                pol["metadata"]["finalizers"] = [R.FINALIZER]
                raw = await client.create(kube.NETWORKCLUSTERPOLICIES, pol)
                ds = R.discovery.discovery_daemonset()
                R.update_daemonset_for(ds, T.NetworkClusterPolicy.from_dict(raw), NS)
                R.set_controller_reference(raw, ds)
                await client.create(kube.DAEMONSETS, ds, namespace=NS)
                pods = lambda name: [p for p in fake.list_objects(kube.PODS)  # noqa: E731
                                     if p["metadata"]["name"].startswith(name + "-")]
                assert len(pods("policy")) == 2  # not ready, status empty
                rec = R.NetworkClusterPolicyReconciler(
                    client, NS, False, get_policy=lambda n: fake.get_object(kube.NETWORKCLUSTERPOLICIES, n),
                    list_owned=lambda n: [d for d in [fake.get_object(kube.DAEMONSETS, n, NS)] if d],
                    list_pods=pods)
                await client.delete(kube.NETWORKCLUSTERPOLICIES, "policy")
                for _ in range(10):
                    await rec.reconcile("policy")
                    if fake.list_objects(kube.JOBS):
                        break
                assert fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]["keptNodes"] == [
                    "gpu-node-0", "gpu-node-1"]
                assert fake.get_object(kube.DAEMONSETS, "policy", NS) is None
                assert sorted(j["spec"]["template"]["spec"]["nodeName"] for j in fake.list_objects(kube.JOBS)) == [
                    "gpu-node-0", "gpu-node-1"]
        finally:
            await fake.stop()
    run(body())


def test_rail_switch_pattern_validated_and_passed():
    from network_operator_amd.api.v1alpha1 import webhook as W

    p = T.new_policy("p", layer="L3", railSwitchPattern="leaf-r{rail}-su[0-9]+")
    assert "--rail-switch-pattern=leaf-r{rail}-su[0-9]+" in agent_args(p)
    assert W.validate_create(p) == []
    assert not any("rail-switch" in a for a in agent_args(T.new_policy("p", layer="L2", railSwitchPattern="x")))
    assert W.validate_create(T.new_policy("p", layer="L2", railSwitchPattern="x")) == [
        "railSwitchPattern has no effect in L2 mode (no LLDP)"]
    with pytest.raises(W.InvalidRailSwitchPatternError, match="invalid railSwitchPattern"):
        W.validate_create(T.new_policy("p", layer="L3", railSwitchPattern="leaf-(r{rail}"))
    rt = T.NetworkClusterPolicy.from_dict(p.to_dict())
    assert rt.spec.amdScaleOut.railSwitchPattern == "leaf-r{rail}-su[0-9]+"


def test_max_unavailable_sets_the_rollout_width():
    from network_operator_amd.api.v1alpha1 import crd as CRD
    from network_operator_amd.api.v1alpha1 import webhook as W

    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy())

            def width():
                ds = fake.get_object(kube.DAEMONSETS, "policy", NS)
                return ds and ds["spec"]["updateStrategy"]["rollingUpdate"]
            await eventually(lambda: width() == {"maxSurge": 0, "maxUnavailable": 1})  # the reference's default
            await edit(client, "policy", lambda cur: cur["spec"].update(maxUnavailable="10%"))
            await eventually(lambda: width() == {"maxSurge": 0, "maxUnavailable": "10%"})
            await edit(client, "policy", lambda cur: cur["spec"].update(maxUnavailable=4))
            await eventually(lambda: width()["maxUnavailable"] == 4)
    run(body())
    for bad in (0, "0%", "150%", "ten", True):
        with pytest.raises(W.InvalidMaxUnavailableError):
            W.validate_max_unavailable(bad)
    pol = policy()
    pol["spec"]["maxUnavailable"] = "25%"
    assert CRD.validate(pol) == []
    pol["spec"]["maxUnavailable"] = "25 percent"
    assert CRD.validate(pol) and "should match" in CRD.validate(pol)[0]


def test_pod_informer_caches_only_what_the_operator_reads():
    """3000 nodes x 4 policies of whole Pods took the manager over its 128 MiB limit
    (profiles/r3_control_plane_3000n_4p.json); the informer keeps the fields the reconciler and
    the metrics read, and the exit-reason / readiness / admission logic still works on them."""
    from network_operator_amd.operator.informer import slim_pod
    from network_operator_amd.operator.reconciler import agent_epoch, agent_exit_reason, job_not_admitted

    pod = {"apiVersion": "v1", "kind": "Pod",
           "metadata": {"name": "p-n0", "namespace": NS, "uid": "u1", "resourceVersion": "7", "labels": {"app": "x"},
                        "ownerReferences": [{"kind": "DaemonSet", "name": "p", "uid": "d", "controller": True}],
                        "managedFields": [{"manager": "kubelet", "fieldsV1": {"f:status": {}}}] * 5},
           "spec": {"nodeName": "n0", "containers": [{"name": "c", "image": "i", "env": [{"name": "A", "value": "b"}]}],
                    "volumes": [{"name": "v", "hostPath": {"path": "/x"}}] * 4, "tolerations": [{"key": "k"}] * 7},
           "status": {"phase": "Running", "hostIP": "10.0.0.1", "podIP": "10.0.0.1",
                      "conditions": [{"type": "Initialized", "status": "True"},
                                     {"type": "Ready", "status": "False", "reason": "ContainersNotReady",
                                      "lastTransitionTime": "2026-01-01T00:00:01Z"}],
                      "containerStatuses": [{"name": "c", "ready": False, "restartCount": 2, "image": "i",
                                             "imageID": "sha256:abc", "containerID": "containerd://x",
                                             "lastState": {"terminated": {"exitCode": 1, "reason": "Error",
                                                                          "message": "Error: no LLDP peers"}}}]}}
    s = slim_pod(pod)
    assert set(s["metadata"]) == {"name", "namespace", "uid", "resourceVersion", "ownerReferences"}
    assert s["spec"] == {"nodeName": "n0"}
    assert [c["type"] for c in s["status"]["conditions"]] == ["Ready"]
    assert "imageID" not in s["status"]["containerStatuses"][0] and "podIP" not in s["status"]
    assert agent_exit_reason(s) == agent_exit_reason(pod) == "no LLDP peers"
    assert agent_epoch(s) == agent_epoch(pod)
    assert len(json.dumps(s)) < len(json.dumps(pod)) / 2
    refused = {"status": {"phase": "Failed", "reason": "OutOfamd.com/gpu", "message": "no GPUs"}, "metadata": {"name": "j"}}
    assert job_not_admitted([slim_pod(refused)]) == job_not_admitted([refused])


def test_min_link_speed_passed_in_both_layers():
    from network_operator_amd.api.v1alpha1 import crd as CRD

    for layer in ("L2", "L3"):
        assert "--min-link-speed-gbps=400" in agent_args(T.new_policy("p", layer=layer, minLinkSpeedGbps=400))
    assert not any("min-link-speed" in a for a in agent_args(T.new_policy("p")))
    bad = policy(minLinkSpeedGbps=5000)
    assert any("less than or equal to 3200" in e for e in CRD.validate(bad))


def test_probe_reason_takes_the_latest_kubelet_event():
    from network_operator_amd.operator.informer import slim_event
    from network_operator_amd.operator.reconciler import probe_reason

    old = {"metadata": {"name": "p.1", "namespace": NS}, "involvedObject": {"kind": "Pod", "name": "p"},
           "reason": "Unhealthy", "message": "Readiness probe failed: not ready: ens1: link down",
           "lastTimestamp": "2026-01-01T00:00:01Z", "count": 3, "source": {"component": "kubelet"}}
    new = dict(old, message="Readiness probe failed: not ready: ens2: waiting for LLDP", lastTimestamp="2026-01-01T00:00:09Z")
    assert probe_reason([slim_event(old), slim_event(new)]) == "ens2: waiting for LLDP"
    assert probe_reason([]) is None
    assert "source" not in slim_event(old) and slim_event(old)["involvedObject"] == {"kind": "Pod", "name": "p"}


def test_cleanup_survives_an_operator_restart_mid_deletion(monkeypatch):
    """The finalizer's progress lives in the API server (status.keptNodes and the cleanup Jobs),
    not in the operator's memory: a new leader picks the deletion up where the old one stopped,
    without cleaning a finished node twice."""
    from network_operator_amd.operator import reconciler as R

    monkeypatch.setattr(R, "CLEANUP_POLL_S", 0.05)

    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        client = ApiClient(KubeConfig(host=url))
        try:
            for i in range(3):
                fake.add_node(f"gpu-node-{i}", {"foo": "bar"})
            ctl = PolicyController(client, NS, is_openshift=False, workers=2)
            await ctl.start()
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy(keepConfigOnRestart=True))
            await eventually(lambda: (fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy").get("status") or {})
                             .get("keptNodes") == [f"gpu-node-{i}" for i in range(3)])
            await client.delete(kube.NETWORKCLUSTERPOLICIES, "policy")
            await eventually(lambda: len(fake.list_objects(kube.JOBS)) == 3)
            first = {j["metadata"]["name"] for j in fake.list_objects(kube.JOBS)}
            await ctl.stop()  # the leader goes away; one node's cleanup finishes meanwhile
            done = next(j for j in fake.list_objects(kube.JOBS) if j["spec"]["template"]["spec"]["nodeName"] == "gpu-node-0")
            fake.set_job_result(done["metadata"]["name"], NS, True)
            ctl2 = PolicyController(client, NS, is_openshift=False, workers=2)
            await ctl2.start()
            await eventually(lambda: (fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy").get("status") or {})
                             .get("keptNodes") == ["gpu-node-1", "gpu-node-2"])
            for j in fake.list_objects(kube.JOBS):
                if not (j.get("status") or {}).get("conditions"):
                    fake.set_job_result(j["metadata"]["name"], NS, True)
            await eventually(lambda: fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy") is None)
            created = [m for m, path in fake.requests if m == "POST" and path.endswith("/jobs")]
            assert len(created) == 3 and first  # no node was cleaned twice
            await ctl2.stop()
        finally:
            await client.close()
            await fake.stop()
    run(body())


def test_foreground_deletion_cleans_every_node_once_and_leaves_no_jobs(monkeypatch):
    """kubectl delete --cascade=foreground: while the policy carries foregroundDeletion the garbage
    collector deletes every new dependent of it.  Cleanup Jobs created during the deletion are
    therefore not owned by the policy (one owned by it would be collected mid-run and the node
    cleaned again); the finalizer deletes them itself once every node is clean."""
    from network_operator_amd.operator import reconciler as R

    monkeypatch.setattr(R, "CLEANUP_POLL_S", 0.05)

    async def body():
        fake = FakeApiServer(foreground_hold=3.0)  # the collector's latency covers the Jobs' creation
        url = await fake.start()
        client = ApiClient(KubeConfig(host=url))
        try:
            for i in range(3):
                fake.add_node(f"gpu-node-{i}", {"foo": "bar"})
            ctl = PolicyController(client, NS, is_openshift=False, workers=2)
            await ctl.start()
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy(keepConfigOnRestart=True))
            await eventually(lambda: (fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy").get("status") or {})
                             .get("keptNodes") == [f"gpu-node-{i}" for i in range(3)])
            await client.delete(kube.NETWORKCLUSTERPOLICIES, "policy", propagation="Foreground")
            await eventually(lambda: len(fake.list_objects(kube.JOBS)) == 3)
            jobs = fake.list_objects(kube.JOBS)
            assert all(not j["metadata"].get("ownerReferences") for j in jobs)
            await eventually(lambda: "foregroundDeletion" not in
                             fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["metadata"]["finalizers"], timeout=10)
            # The collector has released the policy: the Jobs were left alone.
            assert {j["metadata"]["name"] for j in fake.list_objects(kube.JOBS)} == {j["metadata"]["name"] for j in jobs}
            for j in jobs:
                fake.set_job_result(j["metadata"]["name"], NS, True)
            await eventually(lambda: fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy") is None)
            assert fake.list_objects(kube.JOBS) == []  # deleted by the finalizer, not left behind
            created = [m for m, path in fake.requests if m == "POST" and path.endswith("/jobs")]
            assert len(created) == 3  # every node cleaned exactly once
            await ctl.stop()
        finally:
            await client.close()
            await fake.stop()
    run(body())


def test_a_node_that_rejoins_during_its_cleanup_keeps_its_agent(monkeypatch):
    """A node leaves the policy, its cleanup Job starts, and it comes back before the Job ran:
    the Job is withdrawn (the node lock on the node keeps the two apart if it had started) and
    the node stays in keptNodes for its new agent."""
    from network_operator_amd.operator import reconciler as R

    monkeypatch.setattr(R, "KEPT_ORPHAN_GRACE_S", 0.2)
    monkeypatch.setattr(R, "CLEANUP_POLL_S", 0.05)

    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            fake.add_node("gpu-node-0", {"foo": "bar"})
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy(keepConfigOnRestart=True))
            await eventually(lambda: (fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy").get("status") or {})
                             .get("keptNodes") == ["gpu-node-0"])
            fake.set_node_labels("gpu-node-0", {"foo": "other"})
            await eventually(lambda: len(fake.list_objects(kube.JOBS)) == 1)
            fake.set_node_labels("gpu-node-0", {"foo": "bar"})  # back before the Job ran
            await eventually(lambda: fake.list_objects(kube.JOBS) == [])
            await asyncio.sleep(0.3)
            assert fake.list_objects(kube.JOBS) == []
            assert fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]["keptNodes"] == ["gpu-node-0"]
    run(body())


def test_a_starting_node_is_not_reported_as_degraded():
    from network_operator_amd.operator.reconciler import _starting_up

    assert _starting_up("ens0: waiting for LLDP; ens1: not configured yet")
    assert not _starting_up("ens0: waiting for LLDP; ens1: link down")
    # requireRdma: waiting for the RDMA devices is start-up until rdmaWait, then a fault; the
    # label hold-down after a flap is a degraded node recovering, not one starting.
    assert _starting_up("ens0: waiting for RDMA device; ens1: waiting for LLDP")
    assert not _starting_up("ens0: no RDMA device (load its RDMA driver); ens1: waiting for RDMA device")
    assert not _starting_up("label hold-down: healthy again after 1 withdrawal(s), republished in 7.5s without a flap")


def test_dcbx_hand_over_and_peer_mtu_check_are_policy_fields():
    """handing DCBX to the host (mlx5 firmware mode) is its own opt-in, off by default,
    so disableFirmwareLldp keeps meaning "private flags only" on upgrade; checkPeerMtu: false turns
    the jumbo-frame check off for switches that misreport the 802.3 TLV."""
    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.api.v1alpha1 import webhook as W
    from network_operator_amd.operator.reconciler import agent_args, host_nic_agent_args

    p = T.new_policy("p", layer="L3")
    p.spec.amdScaleOut.disableFirmwareLldp = True
    args = agent_args(p)
    assert "--disable-fw-lldp" in args and "--fw-lldp-dcbx-host" not in args
    assert "--check-peer-mtu=false" not in args  # the agent's default: on
    p.spec.amdScaleOut.handDcbxToHost = True
    p.spec.amdScaleOut.checkPeerMtu = False
    args = agent_args(p)
    assert args.index("--fw-lldp-dcbx-host") == args.index("--disable-fw-lldp") + 1
    assert "--check-peer-mtu=false" in args
    back = T.NetworkClusterPolicy.from_dict(p.to_dict()).spec.amdScaleOut
    assert back.handDcbxToHost is True and back.checkPeerMtu is False and not back.extra
    assert W.validate_create(p) == []
    p.spec.amdScaleOut.disableFirmwareLldp = False
    assert "--fw-lldp-dcbx-host" not in agent_args(p)
    assert W.validate_create(p) == ["handDcbxToHost has no effect without disableFirmwareLldp in L3 mode"]
    h = T.new_host_nic_policy("h", layer="L3", checkPeerMtu=False, nicDrivers=["mlx5_core"])
    assert "--check-peer-mtu=false" in host_nic_agent_args(h)
    assert T.NetworkClusterPolicy.from_dict(h.to_dict()).spec.hostNic.checkPeerMtu is False
    from network_operator_amd.api.v1alpha1 import crd as CRD

    assert not CRD.validate(p.to_dict()) and not CRD.validate(h.to_dict())


def test_host_nic_policy_can_take_the_gpu_rails_only_on_request():
    """host-nic discovery leaves the GPUs' scale-out NICs to amd-so; hostNic.includeGpuRails
    (nodes without an amd-so policy) hands the agent --rdma-include-gpu-rails.  Named interfaces
    are taken as named, so the field is then moot and the webhook says so."""
    from network_operator_amd.api.v1alpha1 import crd as CRD
    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.api.v1alpha1 import webhook as W
    from network_operator_amd.operator.reconciler import host_nic_agent_args

    h = T.new_host_nic_policy("h", layer="L2", nicDrivers=["mlx5_core"])
    assert "--rdma-include-gpu-rails" not in host_nic_agent_args(h)
    h.spec.hostNic.includeGpuRails = True
    args = host_nic_agent_args(h)
    assert "--nic-discovery=rdma" in args and "--rdma-include-gpu-rails" in args
    assert T.NetworkClusterPolicy.from_dict(h.to_dict()).spec.hostNic.includeGpuRails is True
    assert not CRD.validate(h.to_dict())
    assert any("amd-so policy on the same nodes" in w for w in W.validate_create(h))
    h.spec.hostNic.interfaces = ["ens9np0"]
    assert "--rdma-include-gpu-rails" not in host_nic_agent_args(h)
    assert any("no effect with interfaces" in w for w in W.validate_create(h))


def test_policy_tolerations_and_priority_reach_the_agent_pods_and_their_jobs():
    """GPU nodes are often tainted (amd.com/gpu:NoSchedule): spec.tolerations goes to the agent
    DaemonSet's Pod template, the cleanup Job (a copy of that template) and the validation Job;
    removing it from the policy removes it from the template.  Admission applies the API
    server's toleration rules, so a bad one fails at kubectl apply instead of at the DaemonSet."""
    from network_operator_amd import discovery
    from network_operator_amd.api.v1alpha1 import crd as CRD
    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.api.v1alpha1 import webhook as W
    from network_operator_amd.operator import reconciler as R

    tol = [{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"},
           {"key": "node.kubernetes.io/unreachable", "operator": "Exists", "effect": "NoExecute",
            "tolerationSeconds": 300}]
    for p in (T.new_policy("p", layer="L3"), T.new_host_nic_policy("h", layer="L2", nicDrivers=["mlx5_core"])):
        p.spec.tolerations = tol
        assert T.NetworkClusterPolicy.from_dict(p.to_dict()).spec.tolerations == tol
        assert not CRD.validate(p.to_dict())
        W.validate_create(p)
        ds = discovery.discovery_daemonset()
        R.update_daemonset_for(ds, p, "ns")
        assert ds["spec"]["template"]["spec"]["tolerations"] == tol
        assert R.cleanup_job(p, "n0", "ns")["spec"]["template"]["spec"]["tolerations"] == tol
        p.spec.priorityClassName = "system-node-critical"
        R.update_daemonset_for(ds, p, "ns")
        assert ds["spec"]["template"]["spec"]["priorityClassName"] == "system-node-critical"
        assert R.cleanup_job(p, "n0", "ns")["spec"]["template"]["spec"]["priorityClassName"] == "system-node-critical"
        assert T.NetworkClusterPolicy.from_dict(p.to_dict()).spec.priorityClassName == "system-node-critical"
        assert not CRD.validate(p.to_dict())
        p.spec.tolerations, p.spec.priorityClassName = [], ""
        R.update_daemonset_for(ds, p, "ns")
        assert "tolerations" not in ds["spec"]["template"]["spec"]
        assert "priorityClassName" not in ds["spec"]["template"]["spec"]
    v = T.new_policy("v", layer="L3")
    v.spec.tolerations = tol[:1]
    assert R.validation_job(v, "n0", 1, "ns")["spec"]["template"]["spec"]["tolerations"] == tol[:1]
    assert "tolerations" not in R.validation_job(T.new_policy("w", layer="L3"), "n0", 1, "ns")["spec"]["template"][
        "spec"]
    for bad in ({"operator": "Exists", "value": "x"}, {"value": "x"}, {"key": "a b"},
                {"key": "k", "effect": "NoSchedule", "tolerationSeconds": 5}):
        v.spec.tolerations = [bad]
        with pytest.raises(W.ValidationError):
            W.validate_create(v)


def test_tainted_gpu_nodes_are_targeted_once_the_policy_tolerates_the_taint():
    """Through the controller loop: two of three selected nodes carry amd.com/gpu:NoSchedule.
    Without tolerations the DaemonSet places agents on the untainted node only (targets 1); the
    policy gains the toleration, the DaemonSet template follows, and all three are targeted."""
    async def body():
        async with cluster(openshift=False) as (fake, client, ctl):
            taint = [{"key": "amd.com/gpu", "value": "present", "effect": "NoSchedule"}]
            for i in range(3):
                fake.add_node(f"gpu-node-{i}", {"foo": "bar"}, taints=taint if i else None)
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy())

            def targets(n):
                def check():
                    assert fake.get_object(kube.NETWORKCLUSTERPOLICIES, "policy")["status"]["targets"] == n
                return check
            await eventually(targets(1))
            cur = await client.get(kube.NETWORKCLUSTERPOLICIES, "policy")
            cur["spec"]["tolerations"] = [{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}]
            await client.replace(kube.NETWORKCLUSTERPOLICIES, cur)
            await eventually(targets(3))
            ds = fake.get_object(kube.DAEMONSETS, "policy", NS)
            assert ds["spec"]["template"]["spec"]["tolerations"] == cur["spec"]["tolerations"]

    asyncio.run(asyncio.wait_for(body(), 60))


def test_stalled_lease_renewal_stops_the_leader_before_anyone_else_can_lead():
    """the leader's Lease PUTs stall for 20 s (a wedged API path).  Its renewal
    attempts are bounded by the renew deadline, so it cancels its work within renew_deadline of
    its last renewal -- before the lease (lease_duration) can expire for the standby -- and the two
    replicas' work never overlaps.  (Unbounded, each stalled PUT ran to the client's 30 s timeout
    while the stalled leader kept reconciling.)"""
    lease_duration, renew_deadline, retry = 1.5, 1.0, 0.25

    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        c1 = ApiClient(KubeConfig(host=url), user_agent="replica-one")
        c2 = ApiClient(KubeConfig(host=url), user_agent="replica-two")
        kw = dict(lease_duration=lease_duration, renew_deadline=renew_deadline, retry_period=retry)
        e1 = LeaderElector(c1, NS, identity="one", **kw)
        e2 = LeaderElector(c2, NS, identity="two", release_on_cancel=False, **kw)
        loop = asyncio.get_event_loop()
        ticks = {"one": [], "two": []}

        async def work(name):
            while True:  # "reconciling": a tick every 10 ms while this replica leads
                ticks[name].append(loop.time())
                await asyncio.sleep(0.01)

        t1 = asyncio.ensure_future(e1.run(lambda: work("one")))
        await eventually(lambda: bool(ticks["one"]))
        t2 = asyncio.ensure_future(e2.run(lambda: work("two")))
        await asyncio.sleep(3 * retry)
        last_renew = fake.get_object(kube.LEASES, "9a8a7ba6.amd.com", NS)["spec"]["renewTime"]
        fake.stall("PUT", r"/leases/", 20.0, user_agent="replica-one")
        t_stall = loop.time()
        await asyncio.wait_for(t1, renew_deadline + 2 * retry + 1.0)  # replica one gives up leading
        assert e1.lost_at is not None and e1.lost_at - t_stall <= renew_deadline + retry + 0.1, e1.lost_at - t_stall
        await eventually(lambda: bool(ticks["two"]), timeout=lease_duration + 3)
        stop_one, start_two = max(ticks["one"]), min(ticks["two"])
        assert stop_one < start_two, (stop_one, start_two)  # never both reconciling
        assert stop_one - t_stall <= renew_deadline + retry + 0.1
        lease = fake.get_object(kube.LEASES, "9a8a7ba6.amd.com", NS)
        assert lease["spec"]["holderIdentity"] == "two" and lease["spec"]["renewTime"] != last_renew
        fake.clear_stalls()
        t2.cancel()
        try:
            await t2
        except asyncio.CancelledError:
            pass
        await c1.close()
        await c2.close()
        await fake.stop()
    run(body())


# One corpus through both engines: what admission accepts must compile in the agent's ECMAScript
# std::regex (via the pybind module) and Python's re, and match the same System Names.
RAIL_PATTERN_CORPUS = [
    # (pattern, admitted)
    ("leaf-r{rail}-.*", True), ("leaf-r{rail}", True), (r"leaf-r{rail}-\d+", True), ("(?:spine|leaf)-{rail}", True),
    ("^leaf-r{rail}$", True), (r"leaf\.r{rail}", True), ("leaf-[a-z]{2,3}-{rail}", True), ("x{2,}y?", True),
    ("leaf(?=-r{rail})-r{rail}", True), ("leaf(?!-spine).*", True), (r"[\w.-]+-{rail}", True), ("a+?b*?", True),
    (r"leaf\x2dr{rail}", True), (r"lea", True), (r"(l)eaf\1?", True), ("[^ ]+", True), (r"\s*leaf\b", True),
    ("(?i)leaf-r{rail}", False), ("(?<=x)leaf", False), ("(?<!x)leaf", False), ("(?P<r>leaf)", False),
    ("(?<r>leaf)", False), ("(?>leaf)", False), ("(?#c)leaf", False), ("(?P=r)", False),
    (r"leaf\Z", False), (r"\Aleaf", False), (r"leaf\z", False), (r"\Gleaf", False), (r"\Qa.b\E", False),
    (r"\p{L}+", False), (r"\k<r>", False), (r"\h", False), (r"\cJ", False), (r"\012", False),
    ("a*+", False), ("a++", False), ("a?+", False), ("a{2}+", False), ("a{,3}", False),
    ("[[:alpha:]]+", False), ("[[=a=]]", False), ("[]a]", False), ("leaf(", False), ("leaf)", False),
    ("[a-", False), ("*leaf", False), ("a{3,1}", False), ("a{{rail},3}", False), (r"(a)\12", False),
    ("x{", False), ("x}", False), ("\\", False),
]


@pytest.mark.parametrize("pattern,admitted", RAIL_PATTERN_CORPUS)
def test_rail_switch_pattern_admission_agrees_with_the_agents_regex_engine(native, pattern, admitted):
    """the webhook and the agent used different regex dialects, so a pattern
    admission accepted ((?i), lookbehind, (?P<n>)) crash-looped the agents.  Admitted now means:
    compiles in std::regex ECMAScript for every rail index, compiles in Python, and both engines
    match the same names."""
    import re

    from network_operator_amd.api.v1alpha1 import webhook as W

    try:
        W.validate_rail_switch_pattern(pattern)
        ok = True
    except W.InvalidRailSwitchPatternError:
        ok = False
    assert ok == admitted, (pattern, ok)
    if ok:
        assert native.rail_pattern_error(pattern) == ""
        names = ["leaf-r0-sw1", "leaf-r3", "spine-3", "Leaf-R0", "leaf.r0", "leaf-abc-0", "xxy", "aab", "a",
                 "leaf", "leaf-spine", "l", "", "leaf-r10", " leaf", "leaf--r0", "lea", "leafleaf"]
        for k in (0, 3):
            p = pattern.replace("{rail}", str(k))
            for name in names:
                assert native.ecmascript_full_match(p, name) == bool(re.fullmatch(p, name)), (p, name)


def test_rail_switch_pattern_random_corpus_never_admits_what_the_agent_rejects(native):
    """Random patterns from regex tokens: whatever admission lets through, the agent compiles and
    both engines agree on a set of names (fixed seed; the sweep that shaped the grammar ran 10^6
    patterns and found \\B on an empty name, quantified and nested assertions, set syntax)."""
    import random
    import re

    from network_operator_amd.api.v1alpha1 import webhook as W

    import warnings

    tokens = ["a", "b", "-", ".", "*", "+", "?", "{2}", "{1,3}", "{,2}", "(", ")", "(?:", "(?=", "(?!", "(?i)",
              "(?<=", "[", "]", "[^", "^", "$", "|", r"\d", r"\w", r"\s", r"\b", r"\B", r"\Z", r"\1", r"\2",
              r"\x41", "{rail}", "0", "[[:digit:]]", "*+", r"\-", r"\.", "leaf", r"\]", r"\[", "a-z", "[a-", "/",
              ",", "}", "{", r"\t", r"\0", r"\u0041", "--", "&&", r"\D", r"\S", r"\W", "(?=a)", "(?!b)"]
    rng = random.Random(4)
    names = ["a", "ab", "leaf0", "b-a", "", "aaa", "leafA", "0", "a.b", "leaf-0", "A", "-", "]", "a b", "[", "0a"]
    admitted = 0
    for _ in range(20000):
        p = "".join(rng.choice(tokens) for _ in range(rng.randint(1, 8)))
        try:
            with warnings.catch_warnings():
                warnings.simplefilter("error")  # Python's FutureWarnings (nested sets) are refusals too
                W.validate_rail_switch_pattern(p)
        except W.InvalidRailSwitchPatternError:
            continue
        admitted += 1
        assert native.rail_pattern_error(p) == "", p
        q = p.replace("{rail}", "0")
        for name in names:
            assert native.ecmascript_full_match(q, name) == bool(re.fullmatch(q, name)), (p, name)
    assert admitted > 2000  # the sweep exercised the accepting side too (1M patterns: 0 disagreements)


def test_hold_off_terms_select_exactly_the_nodes_no_older_selector_matches():
    """hold_off_terms against brute force: over random selectors and random node labels, a node
    passes (the newer selector AND the terms, as the DaemonSet controller evaluates them) exactly
    when the newer selector matches it and no older selector does."""
    import random

    from network_operator_amd.operator.reconciler import HELD_EVERYWHERE_KEY, hold_off_terms
    from network_operator_amd.testing.fakeapi import _node_affinity_ok

    assert hold_off_terms({"a": "1"}, []) is None
    assert hold_off_terms({"a": "1"}, [{"a": "2"}]) is None  # disjoint
    assert hold_off_terms({"a": "1"}, [{"a": "1"}]) == [
        {"matchExpressions": [{"key": HELD_EVERYWHERE_KEY, "operator": "Exists"}]}]
    assert hold_off_terms({"a": "1"}, [{"a": "1", "b": "x"}, {"c": "y"}]) == [
        {"matchExpressions": [{"key": "b", "operator": "NotIn", "values": ["x"]},
                              {"key": "c", "operator": "NotIn", "values": ["y"]}]}]
    rng = random.Random(7)
    keys, vals = ["a", "b", "c", "d"], ["0", "1"]

    def sel():
        return {k: rng.choice(vals) for k in rng.sample(keys, rng.randint(1, 3))}
    checked = 0
    for _ in range(400):
        mine, older = sel(), [sel() for _ in range(rng.randint(0, 4))]
        terms = hold_off_terms(mine, older)
        spec = {"affinity": {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
            "nodeSelectorTerms": terms}}}} if terms else {}
        for _ in range(30):
            labels = {k: rng.choice(vals) for k in keys if rng.random() < 0.8}
            node = {"metadata": {"name": "n", "labels": labels}}
            matches = lambda s: all(labels.get(k) == v for k, v in s.items())  # noqa: E731
            want = matches(mine) and not any(matches(q) for q in older)
            assert (matches(mine) and _node_affinity_ok(node, spec)) == want, (mine, older, labels, terms)
            checked += 1
    assert checked == 12000


def test_two_policies_of_one_type_on_the_same_nodes_are_reported_on_both():
    """Two amd-so policies select the same nodes: the newer one's status names the older one and
    the shared nodes at once (Degraded/PolicyConflict, a Warning Event) instead of its agents
    failing on the node lock a minute later; the older one's status is its agents' own.  A
    host-nic policy on the same nodes is no conflict.  Narrowing a selector clears it, and so does
    deleting the older policy."""
    async def body():
        async with cluster(openshift=False, agent_ready_delay=0.01) as (fake, client, ctl):
            for i in range(3):
                fake.add_node(f"n{i}", {"foo": "bar", "rack": "a" if i < 2 else "b"})
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy("one"))
            await client.create(kube.NETWORKCLUSTERPOLICIES, policy("two"))
            hn = T.new_host_nic_policy("hosts", node_selector={"foo": "bar"}).to_dict()
            await client.create(kube.NETWORKCLUSTERPOLICIES, hn)

            def st(name):
                return fake.get_object(kube.NETWORKCLUSTERPOLICIES, name)["status"]

            def conflicted(name, other, nodes):
                def check():
                    s = st(name)
                    assert len(s["errors"]) == 1 and s["errors"][0].startswith(f"{nodes}: also selected by policy {other} "), s
                    c = {x["type"]: x for x in s["conditions"]}
                    assert c["Degraded"]["status"] == "True" and c["Degraded"]["reason"] == "PolicyConflict"
                    assert s["ready"] == s["targets"]  # the conflict is not a readiness verdict
                return check

            def clean(name, targets):
                def check():
                    s = st(name)
                    assert s["errors"] == [] and s["targets"] == targets, s
                    assert {x["type"]: x for x in s["conditions"]}["Degraded"]["reason"] == "AsExpected"
                return check
            await eventually(conflicted("two", "one", "n0, n1, n2"))
            await eventually(clean("one", 3))
            await eventually(clean("hosts", 3))
            events = [e for e in fake.list_objects(kube.EVENTS) if e.get("reason") == "PolicyConflict"]
            assert {e["involvedObject"]["name"] for e in events} == {"two"}

            def conflicts(name):
                return ctl.metrics.registry.get_sample_value("amd_network_operator_policy_conflicts", {"policy": name})
            await eventually(lambda: conflicts("two") == 1 and conflicts("one") == 0)

            await edit(client, "two", lambda cur: cur["spec"].update(nodeSelector={"rack": "b"}))
            await eventually(conflicted("two", "one", "n2"))
            await edit(client, "one", lambda cur: cur["spec"].update(nodeSelector={"rack": "a"}))
            await eventually(clean("two", 1))
            await eventually(clean("one", 2))
            await eventually(lambda: conflicts("two") == 0)

            await edit(client, "two", lambda cur: cur["spec"].update(nodeSelector={"foo": "bar"}))
            await eventually(conflicted("two", "one", "n0, n1"))
            await client.delete(kube.NETWORKCLUSTERPOLICIES, "one")
            await eventually(clean("two", 3))
            await eventually(clean("hosts", 3))

    run(body())


@pytest.mark.parametrize("seed,gc_delay", [(s, d) for s in range(1, 7) for d in (0.0, 0.05)])
def test_random_edits_converge_to_the_policies_the_cluster_asks_for(seed, gc_delay):
    """Model check through the controller loop: a random sequence of policy creates / edits /
    deletes (both types, both layers, selectors, tolerations), node relabels and DaemonSet
    deletions, applied with and without pauses between them, with and without a garbage collector
    that lags.  Once it settles, every live policy has exactly its DaemonSet (selector,
    tolerations, --mode) and a status that matches a model of the cluster: targets, ready, and a
    PolicyConflict entry for each older same-type policy it shares nodes with -- nothing left over
    from the states it passed through."""
    _model_check(seed, gc_delay)


@pytest.mark.parametrize("seed", [11, 12, 13, 14])
def test_random_edits_converge_through_api_faults_and_lost_watches(seed):
    """The same model check with a hostile API server: the operator's requests (only its own --
    the user's edits go through) randomly fail with 500 / 503 / 429 / 409 on DaemonSet writes,
    status writes, Events, policy writes and reads; its watches are dropped, and the API server's
    event history is compacted so the informers' resume gets 410 Gone and must relist.  Once the
    faults stop, the cluster converges to the same model."""
    _model_check(seed, 0.0, chaos=True)


@pytest.mark.parametrize("seed", [21, 22, 23, 24])
def test_random_edits_converge_across_operator_restarts(seed, monkeypatch):
    """The same model check with the operator stopped at random points -- often mid-reconcile,
    with writes half done -- and a new one started from nothing but the API server's state (no
    queue, no hold-off or cleanup memory, fresh informers).  Together with API faults, and with
    keepConfigOnRestart policies, whose deletion (and whose nodes leaving the selector) runs
    cleanup Jobs behind a finalizer.  Whatever the old process left, the new one converges to the
    same model, every deleted policy is gone and no cleanup Job is left unfinished."""
    from network_operator_amd.operator import reconciler as R

    monkeypatch.setattr(R, "KEPT_ORPHAN_GRACE_S", 0.2)
    monkeypatch.setattr(R, "CLEANUP_POLL_S", 0.05)
    _model_check(seed, 0.0, chaos=True, restarts=True, keep_config=True)


def _model_check(seed, gc_delay, chaos=False, restarts=False, keep_config=False):
    import random

    rng = random.Random(seed)
    chaos_stats = {}
    taint = [{"key": "amd.com/gpu", "value": "present", "effect": "NoSchedule"}]
    tol = [{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}]
    selectors = [{"rack": "a"}, {"rack": "b"}, {"gpu": "yes"}, {"rack": "a", "gpu": "yes"}]

    async def body():
        # agents turn ready 20 ms after their Pod is placed, on every DaemonSet the run makes
        async with cluster(openshift=False, workers=3, gc_delay=gc_delay, agent_ready_delay=0.02,
                           user_client="kubectl" if chaos else None) as (fake, client, ctl):
            live = {"ctl": ctl, "client": None}  # the running operator (restarts replace it)

            async def restart():
                await live["ctl"].stop()
                if live["client"] is not None:
                    await live["client"].close()
                live["client"] = ApiClient(KubeConfig(host=fake.url), user_agent=OPERATOR_UA)
                live["ctl"] = PolicyController(live["client"], NS, is_openshift=False, workers=3)
                await live["ctl"].start()
                chaos_stats["restarts"] = chaos_stats.get("restarts", 0) + 1
            nodes = {}
            for i in range(6):
                labels = {"rack": rng.choice("ab"), **({"gpu": "yes"} if rng.random() < 0.5 else {})}
                nodes[f"n{i}"] = (labels, i == 5)  # n5 is tainted
                fake.add_node(f"n{i}", labels, taints=taint if i == 5 else None)
            model = {}  # name -> (type, layer, selector, tolerates)

            def spec_of(name, ctype):
                sel, layer, tols = rng.choice(selectors), rng.choice(["L2", "L3"]), rng.random() < 0.5
                if ctype == "amd-so":
                    d = T.new_policy(name, layer=layer, node_selector=sel).to_dict()
                else:
                    d = T.new_host_nic_policy(name, layer=layer, node_selector=sel).to_dict()
                if tols:
                    d["spec"]["tolerations"] = tol
                if keep_config and rng.random() < 0.4:
                    d["spec"]["amdScaleOut" if ctype == "amd-so" else "hostNic"]["keepConfigOnRestart"] = True
                return d, (ctype, layer, sel, tols)

            async def job_controller():
                # The cleanup Jobs' Pods run on their nodes and finish a little later.
                while True:
                    for j in fake.list_objects(kube.JOBS):
                        if not (j.get("status") or {}).get("conditions"):
                            with contextlib.suppress(KeyError):
                                fake.set_job_result(j["metadata"]["name"], j["metadata"]["namespace"], True)
                    await asyncio.sleep(0.01)
            jobs_task = asyncio.ensure_future(job_controller()) if keep_config else None

            for _ in range(40):
                op = rng.random()
                names = sorted(model)
                if op < 0.3 or not names:
                    name = rng.choice([n for n in ("p0", "p1", "p2", "p3", "p4") if n not in model] or ["p0"])
                    if name in model:
                        continue
                    body_, m = spec_of(name, rng.choice(["amd-so", "amd-so", "host-nic"]))
                    try:
                        await client.create(kube.NETWORKCLUSTERPOLICIES, body_)
                    except ApiError as e:  # still finalizing after its deletion (keepConfigOnRestart)
                        if e.status != 409:
                            raise
                        continue
                    model[name] = m
                elif op < 0.55:
                    name = rng.choice(names)
                    ctype = model[name][0]
                    new, m = spec_of(name, ctype)
                    await edit(client, name, lambda cur: cur.__setitem__("spec", new["spec"]))
                    model[name] = m
                elif op < 0.7:
                    name = rng.choice(names)
                    await client.delete(kube.NETWORKCLUSTERPOLICIES, name)
                    del model[name]
                elif op < 0.85:
                    n = rng.choice(sorted(nodes))
                    labels = {"rack": rng.choice("ab"), **({"gpu": "yes"} if rng.random() < 0.5 else {})}
                    nodes[n] = (labels, nodes[n][1])
                    fake.set_node_labels(n, labels)
                else:
                    name = rng.choice(names)
                    if fake.get_object(kube.DAEMONSETS, name, NS) is not None:
                        with contextlib.suppress(ApiError):
                            await client.delete(kube.DAEMONSETS, name, NS)
                if restarts and rng.random() < 0.2:
                    # A crash or a rollout of the operator: whatever the old process was doing
                    # stops at its next await; the new one starts from the API server alone.
                    await asyncio.sleep(rng.choice([0.0, 0.001, 0.005, 0.02]))
                    await restart()
                if chaos and rng.random() < 0.35:
                    c = rng.random()
                    if c < 0.7:  # the operator's next requests of one kind fail
                        method, path = rng.choice([("PUT", r"/daemonsets/"), ("POST", r"/daemonsets"),
                                                   ("PUT", r"/networkclusterpolicies/[^/]+/status"),
                                                   ("POST", r"/events"), ("PUT", r"/networkclusterpolicies/[^/]+$"),
                                                   ("GET", r"/nodes"), ("DELETE", r"/")])
                        status, reason = rng.choice([(500, "InternalError"), (503, "ServiceUnavailable"),
                                                     (429, "TooManyRequests"), (409, "Conflict")])
                        fake.fail_next(method, path, status=status, count=rng.randint(1, 3), reason=reason,
                                       user_agent=OPERATOR_UA)
                    elif c < 0.85:
                        fake.drop_watches()  # connection loss: the informers re-watch
                    else:
                        fake.compact()  # etcd compaction: resuming gets 410 Gone, the informers relist
                if rng.random() < 0.5:
                    await asyncio.sleep(rng.choice([0.0, 0.01, 0.05]))
            if chaos:
                await asyncio.sleep(0.2)  # let the queued faults meet the operator's requests
                assert fake.faults_fired > 0
                chaos_stats["fired"] = fake.faults_fired
            fake.faults.clear()
            if keep_config:
                # Whatever the random run left to finalize, one deletion certainly does: a kept
                # node of its own, the operator restarted right after the delete.
                nodes["n6"] = ({"pk": "yes"}, False)
                fake.add_node("n6", {"pk": "yes"})
                pk = T.new_policy("pk", layer="L3", node_selector={"pk": "yes"}, keepConfigOnRestart=True).to_dict()
                await client.create(kube.NETWORKCLUSTERPOLICIES, pk)
                await eventually(lambda: (fake.get_object(kube.NETWORKCLUSTERPOLICIES, "pk").get("status") or {})
                                 .get("keptNodes") == ["n6"], timeout=10)
                await client.delete(kube.NETWORKCLUSTERPOLICIES, "pk")
                await asyncio.sleep(rng.choice([0.0, 0.005, 0.02]))
                await restart()

            def placed(m):
                _, _, sel, tols = m
                return sorted(n for n, (labels, tainted) in nodes.items()
                              if all(labels.get(k) == v for k, v in sel.items()) and (tols or not tainted))

            def converged():
                dss = {d["metadata"]["name"] for d in fake.list_objects(kube.DAEMONSETS)}
                assert dss == set(model), (dss, model)
                names = {q["metadata"]["name"] for q in fake.list_objects(kube.NETWORKCLUSTERPOLICIES)}
                assert names == set(model), (names, model)  # finalizers released
                assert all((j.get("status") or {}).get("conditions") for j in fake.list_objects(kube.JOBS))
                if keep_config:  # pk's node was cleaned by a Job before its finalizer went
                    assert any(w[2] == "POST" and w[3].endswith("/jobs") for w in fake.writes)
                for name, m in model.items():
                    ctype, layer, sel, tols = m
                    ds = fake.get_object(kube.DAEMONSETS, name, NS)
                    pod = ds["spec"]["template"]["spec"]
                    assert pod["nodeSelector"] == sel
                    assert (pod.get("tolerations") == tol) if tols else not pod.get("tolerations")
                    assert f"--mode={layer}" in pod["containers"][0]["args"]
                    assert ds["metadata"]["ownerReferences"][0]["name"] == name
                    s = fake.get_object(kube.NETWORKCLUSTERPOLICIES, name)["status"]

                    def age(n):
                        return (fake.get_object(kube.NETWORKCLUSTERPOLICIES, n)["metadata"]["creationTimestamp"], n)

                    def selects(sel_, n):
                        return all(nodes[n][0].get(k) == v for k, v in sel_.items())
                    older = [o for o, om in model.items() if o != name and om[0] == ctype and age(o) < age(name)]
                    # a node belongs to the oldest policy of the type whose selector matches it
                    held = {n for n in nodes for o in older if selects(model[o][2], n)}
                    mine = sorted(set(placed(m)) - held)
                    assert s["targets"] == len(mine) and s["ready"] == len(mine), (name, s, mine, held)
                    # invariant: no agent Pod of a newer policy on a node an older one of its type holds
                    pods = [q["spec"]["nodeName"] for q in fake.list_objects(kube.PODS)
                            if (q["metadata"].get("ownerReferences") or [{}])[0].get("uid") == ds["metadata"]["uid"]]
                    assert sorted(pods) == mine, (name, pods, mine, held)
                    others = sorted(o for o in older if any(selects(model[o][2], n) and selects(sel, n) for n in nodes))
                    got = sorted(e.split(" also selected by policy ")[1].split(" ")[0] for e in s["errors"])
                    assert got == others and len(s["errors"]) == len(others), (name, s["errors"], others)
                return True
            try:
                await eventually(converged, timeout=30 if chaos else 20)
            finally:
                if jobs_task is not None:
                    jobs_task.cancel()
                if live["client"] is not None:
                    await live["ctl"].stop()
                    await live["client"].close()
        if restarts:
            assert chaos_stats.get("restarts", 0) >= 3, chaos_stats

    run(body(), timeout=150)


def test_a_node_taken_over_by_a_same_nic_policy_owes_no_cleanup(monkeypatch):
    """A keepConfigOnRestart policy leaves a node, and another amd-so policy taking the same NICs
    now runs its agent there (it was held off the node until then): that agent holds the node
    lock and replaces the old configuration, so no cleanup Job is owed -- one would only wait for
    the lock and fail.  A node nobody took still gets its Job."""
    from network_operator_amd.operator import reconciler as R

    monkeypatch.setattr(R, "KEPT_ORPHAN_GRACE_S", 0.3)
    monkeypatch.setattr(R, "CLEANUP_POLL_S", 0.05)

    async def body():
        async with cluster(openshift=False, agent_ready_delay=0.01) as (fake, client, ctl):
            fake.add_node("n0", {"foo": "bar", "rack": "a"})
            fake.add_node("n1", {"foo": "bar", "rack": "b"})
            fake.add_node("n2", {"foo": "bar", "rack": "c"})
            keep = T.new_policy("a-keep", layer="L3", node_selector={"foo": "bar"}, keepConfigOnRestart=True).to_dict()
            await client.create(kube.NETWORKCLUSTERPOLICIES, keep)
            await client.create(kube.NETWORKCLUSTERPOLICIES,
                                T.new_policy("b-plain", layer="L3", node_selector={"rack": "a"}).to_dict())

            def pol(name):
                return fake.get_object(kube.NETWORKCLUSTERPOLICIES, name)
            await eventually(lambda: pol("a-keep")["status"].get("keptNodes") == ["n0", "n1", "n2"])
            await eventually(lambda: pol("b-plain")["status"]["targets"] == 0)  # held off n0
            # a-keep leaves n0 (b-plain takes it) and n2 (nobody does)
            await edit(client, "a-keep", lambda cur: cur["spec"].update(nodeSelector={"foo": "bar", "rack": "b"}))
            await eventually(lambda: pol("b-plain")["status"]["targets"] == 1)
            job = await value(lambda: next(iter(fake.list_objects(kube.JOBS)), None), timeout=5)
            assert job["spec"]["template"]["spec"]["nodeName"] == "n2"
            await eventually(lambda: pol("a-keep")["status"].get("keptNodes") == ["n1", "n2"])
            await asyncio.sleep(0.5)  # past the grace period: still no Job for n0
            assert [j["spec"]["template"]["spec"]["nodeName"] for j in fake.list_objects(kube.JOBS)] == ["n2"]
    run(body())
