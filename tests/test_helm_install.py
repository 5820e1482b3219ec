"""``helm install --set config.amd.enabled=true`` on a fresh cluster, end to end in the fake API
server: every object of the rendered chart is applied in Helm's install order, then the operator
pod "starts" (its webhook certificate issued, its Service gaining an endpoint after it serves).

The fake API server resolves service-referenced webhooks (round 1 skipped them), so it now has
the race a real cluster has. A NetworkClusterPolicy created in the same release, as the
reference chart does (reference charts/network-operator/templates/gaudi.yaml:1-22,
README.md:22-26), is rejected by the Fail-policy webhook while no operator pod serves. The chart
therefore ships its policies in a ConfigMap, and the operator applies them itself once its
webhook is up (operator/seeder.py). This test drives install, upgrade, disable and uninstall.
"""

import asyncio
import base64
import socket
from pathlib import Path

import pytest
import yaml

from network_operator_amd.operator import kube, manager
from network_operator_amd.operator.kube import ApiClient, ApiError, KubeConfig, Resource
from network_operator_amd.operator.servers import generate_self_signed
from network_operator_amd.packaging import manifests as M
from network_operator_amd.testing.fakeapi import FakeApiServer
from network_operator_amd.testing.render import helm_template

ROOT = Path(__file__).resolve().parent.parent
CHART = ROOT / "charts" / "network-operator"
NS = "amd-network-operator"
P = kube.NETWORKCLUSTERPOLICIES

# Add-on kinds the chart uses (cert-manager, NFD): served by the fake like installed CRDs.
ISSUERS = Resource("cert-manager.io", "v1", "issuers", "Issuer", True)
CERTIFICATES = Resource("cert-manager.io", "v1", "certificates", "Certificate", True)
NODEFEATURERULES = Resource("nfd.k8s-sigs.io", "v1alpha1", "nodefeaturerules", "NodeFeatureRule", False)
BY_KIND = {r.kind: r for r in kube.ALL_RESOURCES + [ISSUERS, CERTIFICATES, NODEFEATURERULES]}

# Helm's InstallOrder (pkg/releaseutil/kind_sorter.go); kinds it does not list go last.
HELM_ORDER = ["Namespace", "NetworkPolicy", "ResourceQuota", "LimitRange", "PodSecurityPolicy", "PodDisruptionBudget",
              "ServiceAccount", "Secret", "SecretList", "ConfigMap", "StorageClass", "PersistentVolume",
              "PersistentVolumeClaim", "CustomResourceDefinition", "ClusterRole", "ClusterRoleList",
              "ClusterRoleBinding", "ClusterRoleBindingList", "Role", "RoleList", "RoleBinding", "RoleBindingList",
              "Service", "DaemonSet", "Pod", "ReplicationController", "ReplicaSet", "Deployment",
              "HorizontalPodAutoscaler", "StatefulSet", "Job", "CronJob", "IngressClass", "Ingress", "APIService",
              "MutatingWebhookConfiguration", "ValidatingWebhookConfiguration"]


def helm_install_order(docs):
    rank = {k: i for i, k in enumerate(HELM_ORDER)}
    return sorted(docs, key=lambda d: rank.get(d["kind"], len(HELM_ORDER)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


async def _until(fn, timeout=15.0):
    end = asyncio.get_event_loop().time() + timeout
    last = None
    while asyncio.get_event_loop().time() < end:
        try:
            if fn():
                return
        except (KeyError, TypeError, IndexError) as e:
            last = e
        await asyncio.sleep(0.02)
    raise AssertionError(f"timeout ({last!r})")


def _policies_file(docs, path: Path) -> None:
    """What the kubelet projects from the ConfigMap volume into the operator container."""
    cm = [d for d in docs if d["kind"] == "ConfigMap" and d["metadata"]["name"] == M.POLICIES_CONFIGMAP][0]
    tmp = path.with_suffix(".tmp")
    tmp.write_text(cm["data"]["policies.yaml"])
    tmp.replace(path)


def _dep_args(docs):
    dep = [d for d in docs if d["kind"] == "Deployment"][0]
    return dep["spec"]["template"]["spec"]["containers"][0]["args"]


def test_reference_style_policy_in_the_release_fails_while_the_operator_is_down():
    """The bug class the fake could not see in round 1: Fail-policy webhooks registered in the
    same release as the CR, no operator endpoint yet -> the API server refuses the CR."""
    async def body():
        fake = FakeApiServer(extra_groups=["cert-manager.io", "nfd.k8s-sigs.io"])
        fake.resources += [ISSUERS, CERTIFICATES, NODEFEATURERULES]
        url = await fake.start()
        try:
            docs = helm_install_order(helm_template(CHART, {"config": {"amd": {"enabled": True}}}, NS))
            async with ApiClient(KubeConfig(host=url)) as c:
                for d in docs:
                    await c.create(BY_KIND[d["kind"]], d, d["metadata"].get("namespace"))
                policy = yaml.safe_load(_configmap_text(docs))["policies"][0]
                with pytest.raises(ApiError) as e:
                    await c.create(P, policy)
                assert e.value.status == 500 and "no endpoints available" in str(e.value)
        finally:
            await fake.stop()

    asyncio.run(asyncio.wait_for(body(), 60))


def _configmap_text(docs):
    return [d for d in docs if d["kind"] == "ConfigMap" and d["metadata"]["name"] == M.POLICIES_CONFIGMAP][0][
        "data"]["policies.yaml"]


def test_one_release_helm_install_upgrade_and_uninstall(tmp_path, monkeypatch):
    monkeypatch.setenv("OPERATOR_NAMESPACE", NS)
    hook_port = _free_port()

    async def body():
        fake = FakeApiServer(extra_groups=["cert-manager.io", "nfd.k8s-sigs.io"])
        fake.resources += [ISSUERS, CERTIFICATES, NODEFEATURERULES]
        url = await fake.start()
        fake.add_node("mi355x-0", {"amd.feature.node.kubernetes.io/gpu-ready": "true"})
        stop, started = asyncio.Event(), asyncio.Event()
        task = None
        try:
            docs = helm_install_order(helm_template(CHART, {"config": {"amd": {"enabled": True, "mtu": 9000}}}, NS))
            assert not [d for d in docs if d["kind"] == "NetworkClusterPolicy"]
            async with ApiClient(KubeConfig(host=url)) as c:
                # 1. `helm install`: every release object, Helm's order, nothing else running.
                for d in docs:
                    await c.create(BY_KIND[d["kind"]], d, d["metadata"].get("namespace"))
                assert not fake.list_objects(P)

                # 2. cert-manager issues the serving certificate and injects its CA.
                certs = tmp_path / "certs"
                crt, _ = generate_self_signed(certs, cn=f"amd-network-webhook.{NS}.svc")
                ca = base64.b64encode(crt.read_bytes()).decode()
                for res in (kube.MUTATINGWEBHOOKS, kube.VALIDATINGWEBHOOKS):
                    for cfg in fake.list_objects(res):
                        for wh in cfg["webhooks"]:
                            wh["clientConfig"]["caBundle"] = ca
                        await c.replace(res, cfg)

                # 3. The operator pod starts with the Deployment's own args (the ConfigMap volume
                #    projected to a file); the Service gets its endpoint a moment after it serves.
                pfile = tmp_path / "policies.yaml"
                _policies_file(docs, pfile)
                args = [a for a in _dep_args(docs) if not a.startswith(("--policies-file", "--webhook-port",
                                                                         "--webhook-cert-dir", "--metrics-bind",
                                                                         "--health-probe"))]
                assert "--policies-owner=ClusterRole/amd-network-operator" in args
                task = asyncio.ensure_future(manager.run(
                    args + ["--master", url, f"--policies-file={pfile}", "--policies-interval=0.2",
                            f"--webhook-port={hook_port}", f"--webhook-cert-dir={certs}",
                            "--health-probe-bind-address=0", "--dependency-check-interval=0"],
                    stop=stop, started=started))
                await asyncio.wait_for(started.wait(), 10)
                await asyncio.sleep(0.3)  # readiness probe period: creates before this fail and retry
                fake.service_endpoints[(NS, "amd-network-webhook")] = f"https://127.0.0.1:{hook_port}"

                # The policy exists, went through both webhooks, and is reconciled.
                await _until(lambda: fake.get_object(P, "netconf-amd-scale-out") is not None)
                assert ("default.networkclusterpolicies.amd.com", "CREATE") in fake.admission_calls
                assert ("validate.networkclusterpolicies.amd.com", "CREATE") in fake.admission_calls
                await _until(lambda: fake.get_object(kube.DAEMONSETS, "netconf-amd-scale-out", NS) is not None)
                pol = fake.get_object(P, "netconf-amd-scale-out")
                role = fake.get_object(kube.CLUSTERROLES, "amd-network-operator")
                assert pol["metadata"]["ownerReferences"] == [{"apiVersion": "rbac.authorization.k8s.io/v1",
                                                               "kind": "ClusterRole", "name": "amd-network-operator",
                                                               "uid": role["metadata"]["uid"]}]
                assert pol["spec"]["amdScaleOut"]["mtu"] == 9000
                # Steady state: the seeder (0.2 s interval) rewrites nothing.
                replaces = sum(1 for m, path in fake.requests if m == "PUT" and "/networkclusterpolicies/" in path
                               and not path.endswith("/status"))
                await asyncio.sleep(1.0)
                assert sum(1 for m, path in fake.requests if m == "PUT" and "/networkclusterpolicies/" in path
                           and not path.endswith("/status")) == replaces
                assert fake.get_object(P, "netconf-amd-scale-out")["metadata"]["generation"] == 1

                # 4. `helm upgrade --set config.amd.mtu=4200`: the projected file changes.
                up = helm_template(CHART, {"config": {"amd": {"enabled": True, "mtu": 4200}}}, NS)
                _policies_file(up, pfile)
                await _until(lambda: "--mtu=4200" in fake.get_object(kube.DAEMONSETS, "netconf-amd-scale-out", NS)
                             ["spec"]["template"]["spec"]["containers"][0]["args"])

                # A user's own policy is never touched by the seeder.
                mine = yaml.safe_load(_configmap_text(up))["policies"][0]
                mine["metadata"] = {"name": "user-policy"}
                await c.create(P, mine)

                # 5. `helm upgrade --set config.amd.enabled=false`: the policy and its DaemonSet go.
                _policies_file(helm_template(CHART, {}, NS), pfile)
                await _until(lambda: fake.get_object(P, "netconf-amd-scale-out") is None)
                await _until(lambda: fake.get_object(kube.DAEMONSETS, "netconf-amd-scale-out", NS) is None)
                assert fake.get_object(P, "user-policy") is not None

                # 6. Re-enable, then `helm uninstall`: the release's ClusterRole goes, and the
                #    garbage collector takes the seeded policy and its DaemonSet with it.
                _policies_file(docs, pfile)
                await _until(lambda: fake.get_object(kube.DAEMONSETS, "netconf-amd-scale-out", NS) is not None)
                stop.set()
                assert await asyncio.wait_for(task, 10) == 0
                task = None
                for d in reversed(docs):
                    if d["kind"] != "CustomResourceDefinition":  # Helm keeps crds/ on uninstall
                        await c.delete(BY_KIND[d["kind"]], d["metadata"]["name"], d["metadata"].get("namespace"))
                assert fake.get_object(P, "netconf-amd-scale-out") is None
                assert fake.get_object(kube.DAEMONSETS, "netconf-amd-scale-out", NS) is None
                assert fake.get_object(P, "user-policy") is not None
        finally:
            stop.set()
            if task is not None:
                await asyncio.wait_for(task, 10)
            await fake.stop()

    asyncio.run(asyncio.wait_for(body(), 90))


def _policy(name, mtu=9000):
    return {"apiVersion": "amd.com/v1alpha1", "kind": "NetworkClusterPolicy", "metadata": {"name": name},
            "spec": {"configurationType": "amd-so", "nodeSelector": {"amd.feature.node.kubernetes.io/gpu-ready": "true"},
                     "amdScaleOut": {"layer": "L3", "mtu": mtu}}}


def test_seeder_ownership_is_release_scoped(tmp_path):
    """ownership is decided by the release's anchor (ownerReference uid), or
    by a release-unique seeder id without one — never by the generic managed-by label.  A user's
    copy of a seeded policy (labels included) survives; a second operator instance with another
    owner leaves the first one's policies alone, and vice versa."""
    from network_operator_amd.operator.seeder import MANAGED_BY, MANAGED_BY_KEY, SEEDER_KEY, PolicySeeder

    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        try:
            async with ApiClient(KubeConfig(host=url)) as c:
                for role in ("release-a", "release-b"):
                    await c.create(kube.CLUSTERROLES, {"apiVersion": "rbac.authorization.k8s.io/v1",
                                                       "kind": "ClusterRole", "metadata": {"name": role}, "rules": []})
                fa, fb = tmp_path / "a.yaml", tmp_path / "b.yaml"
                fa.write_text(yaml.safe_dump({"policies": [_policy("pol-a")]}))
                fb.write_text(yaml.safe_dump({"policies": [_policy("pol-b", 4200)]}))
                a = PolicySeeder(c, str(fa), owner="ClusterRole/release-a", interval=0.1)
                b = PolicySeeder(c, str(fb), owner="ClusterRole/release-b", interval=0.1)
                await a.sync_once()
                seeded = fake.get_object(P, "pol-a")
                assert seeded["metadata"]["labels"][MANAGED_BY_KEY] == MANAGED_BY
                # The user copies the seeded YAML, labels included, under another name.
                copy_ = {"apiVersion": seeded["apiVersion"], "kind": seeded["kind"],
                         "metadata": {"name": "user-copy", "labels": dict(seeded["metadata"]["labels"])},
                         "spec": seeded["spec"]}
                await c.create(P, copy_)
                await a.sync_once()
                assert fake.get_object(P, "user-copy") is not None
                # A second operator instance (another release) on the same cluster.
                await b.sync_once()
                await a.sync_once()
                await b.sync_once()
                assert fake.get_object(P, "pol-a") is not None and fake.get_object(P, "pol-b") is not None
                assert fake.get_object(P, "pol-b")["spec"]["amdScaleOut"]["mtu"] == 4200
                # B may not take over A's policy of the same name either.
                fb.write_text(yaml.safe_dump({"policies": [_policy("pol-b", 4200), _policy("pol-a", 1500)]}))
                await b.sync_once()
                assert fake.get_object(P, "pol-a")["spec"]["amdScaleOut"]["mtu"] == 9000
                # A disabled: only A's own policy goes.
                fa.write_text(yaml.safe_dump({"policies": []}))
                await a.sync_once()
                assert fake.get_object(P, "pol-a") is None
                assert fake.get_object(P, "pol-b") is not None and fake.get_object(P, "user-copy") is not None
                # B's anchor gone (uninstall in progress): B writes nothing, deletes nothing.
                await c.delete(kube.CLUSTERROLES, "release-b")
                fb.write_text(yaml.safe_dump({"policies": []}))
                writes = b.writes
                await b.sync_once()
                assert b.writes == writes

                # Without an owner: a release-unique seeder id decides.
                fx, fy = tmp_path / "x.yaml", tmp_path / "y.yaml"
                fx.write_text(yaml.safe_dump({"policies": [_policy("pol-x")]}))
                fy.write_text(yaml.safe_dump({"policies": []}))
                x = PolicySeeder(c, str(fx), seed_id="ns-x.lease")
                y = PolicySeeder(c, str(fy), seed_id="ns-y.lease")
                await x.sync_once()
                assert fake.get_object(P, "pol-x")["metadata"]["labels"][SEEDER_KEY] == "ns-x.lease"
                await y.sync_once()  # lists nothing of its own: pol-x stays
                assert fake.get_object(P, "pol-x") is not None
                fx.write_text(yaml.safe_dump({"policies": []}))
                await x.sync_once()
                assert fake.get_object(P, "pol-x") is None and fake.get_object(P, "user-copy") is not None
        finally:
            await fake.stop()

    asyncio.run(asyncio.wait_for(body(), 60))


def test_seeder_leaves_a_policy_that_is_being_deleted_alone(tmp_path):
    """A seeded policy under deletion (its finalizer is cleaning nodes) is not edited back to the
    file's spec, which would roll agents on nodes being cleaned; it is seeded anew once gone."""
    from network_operator_amd.operator.seeder import PolicySeeder

    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        try:
            async with ApiClient(KubeConfig(host=url)) as c:
                f = tmp_path / "p.yaml"
                f.write_text(yaml.safe_dump({"policies": [_policy("pol", 9000)]}))
                s = PolicySeeder(c, str(f), seed_id="ns.lease")
                await s.sync_once()
                cur = fake.get_object(P, "pol")
                cur["metadata"]["finalizers"] = ["amd.com/node-cleanup"]
                await c.replace(P, cur)
                await c.delete(P, "pol")
                f.write_text(yaml.safe_dump({"policies": [_policy("pol", 4200)]}))
                writes = s.writes
                await s.sync_once()
                held = fake.get_object(P, "pol")
                assert held["metadata"]["deletionTimestamp"] and held["spec"]["amdScaleOut"]["mtu"] == 9000
                assert s.writes == writes
                await c.replace(P, dict(held, metadata=dict(held["metadata"], finalizers=[])))  # finalized
                assert fake.get_object(P, "pol") is None
                await s.sync_once()
                assert fake.get_object(P, "pol")["spec"]["amdScaleOut"]["mtu"] == 4200
        finally:
            await fake.stop()

    asyncio.run(asyncio.wait_for(body(), 60))


def test_seed_id_label_is_a_valid_distinct_label_value():
    from network_operator_amd.operator.seeder import seed_id_label

    assert seed_id_label("amd-network-operator.9a8a7ba6.amd.com") == "amd-network-operator.9a8a7ba6.amd.com"
    long_a, long_b = "n" * 70 + "a", "n" * 70 + "b"
    la, lb = seed_id_label(long_a), seed_id_label(long_b)
    assert la != lb and len(la) <= 63 and len(lb) <= 63
    odd = seed_id_label("ns/with spaces")
    import re

    assert re.fullmatch(r"[A-Za-z0-9]([A-Za-z0-9._-]*[A-Za-z0-9])?", odd) and odd != seed_id_label("ns/with-spaces")


@pytest.mark.parametrize("which", ["amd", "hostNic"])
def test_uninstall_with_keep_config_policies_runs_the_predelete_hook_first(tmp_path, which):
    """config.<amd|hostNic>.keepConfigOnRestart: the seeded policy carries the node-cleanup
    finalizer.  An uninstall that removed the operator first would leave it Terminating for good
    (nobody to clean the nodes and release it); the chart's pre-delete hook deletes the release's
    policies while the operator runs and returns once they are finalized.  A user's policy is left
    alone."""
    from network_operator_amd.operator import reconciler as R
    from network_operator_amd.operator.controller import PolicyController
    from network_operator_amd.operator.predelete import drain
    from network_operator_amd.operator.seeder import PolicySeeder

    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        fake.add_node("mi355x-0", {"amd.feature.node.kubernetes.io/gpu-ready": "true"})
        docs = helm_template(CHART, {"config": {which: {"enabled": True, "keepConfigOnRestart": True}}}, NS)
        seeded = "netconf-amd-scale-out" if which == "amd" else "netconf-amd-host-nic"
        hook = [d for d in docs if d["kind"] == "Job"][0]
        owner = next(a.split("=", 1)[1] for a in hook["spec"]["template"]["spec"]["containers"][0]["args"]
                     if a.startswith("--owner="))
        async with ApiClient(KubeConfig(host=url)) as c:
            await c.create(kube.CLUSTERROLES, [d for d in docs if d["kind"] == "ClusterRole"
                                               and d["metadata"]["name"] == "amd-network-operator"][0])
            pfile = tmp_path / "policies.yaml"
            _policies_file(docs, pfile)
            await PolicySeeder(c, str(pfile), owner=owner).sync_once()
            await c.create(P, dict(_policy("user-policy"), spec=dict(_policy("user-policy")["spec"],
                                                                      amdScaleOut={"layer": "L3",
                                                                                   "keepConfigOnRestart": True})))
            ctl = PolicyController(c, NS, is_openshift=False, workers=2)
            await ctl.start()
            try:
                await _until(lambda: fake.get_object(kube.DAEMONSETS, seeded, NS) is not None)
                fake.set_agent_ready("mi355x-0", daemonset=f"{NS}/{seeded}")
                await _until(lambda: (fake.get_object(P, seeded).get("status") or {})
                             .get("keptNodes") == ["mi355x-0"])

                async def kubelet():  # the node runs each cleanup Job to success
                    while True:
                        for j in fake.list_objects(kube.JOBS):
                            if j["metadata"]["labels"].get("app") == R.CLEANUP_APP and not j.get("status"):
                                fake.set_job_result(j["metadata"]["name"], NS, True)
                        await asyncio.sleep(0.02)
                k = asyncio.ensure_future(kubelet())
                assert await asyncio.wait_for(drain(c, owner, timeout=20, poll=0.05), 30) == 0
                k.cancel()
                assert fake.get_object(P, seeded) is None
                assert fake.get_object(kube.DAEMONSETS, seeded, NS) is None
                assert fake.get_object(P, "user-policy") is not None
            finally:
                await ctl.stop()
            # Without the hook: the operator is gone when the policy is deleted -> stuck.
            await c.delete(P, "user-policy")
            await asyncio.sleep(0.2)
            stuck = fake.get_object(P, "user-policy")
            assert stuck["metadata"]["deletionTimestamp"] and stuck["metadata"]["finalizers"] == [R.FINALIZER]
        await fake.stop()

    asyncio.run(asyncio.wait_for(body(), 60))


@pytest.mark.parametrize("keep,nm", [(False, False), (True, False), (False, True), (True, True)])
@pytest.mark.parametrize("which", ["amd", "hostNic"])
def test_predelete_hook_is_rendered_whenever_the_seeded_policy_gets_the_finalizer(keep, nm, which):
    """a release with config.amd.disableNetworkManager=true seeds a policy that
    carries the node-cleanup finalizer (the NICs are handed back to NetworkManager by cleanup
    Jobs), so it needs the pre-delete hook as much as keepConfigOnRestart does; without it
    `helm uninstall` leaves the policy Terminating and its agents running with no operator."""
    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.operator import reconciler as R

    # (the chart exposes the same two fields for the host-nic policy: the same finalizer, the same hook)
    docs = helm_template(CHART, {"config": {which: {"enabled": True, "keepConfigOnRestart": keep,
                                                    "disableNetworkManager": nm}}}, NS)
    hooks = [d for d in docs if d["kind"] == "Job" and
             (d["metadata"].get("annotations") or {}).get("helm.sh/hook") == "pre-delete"]
    cm = [d for d in docs if d["kind"] == "ConfigMap" and d["metadata"]["name"] == M.POLICIES_CONFIGMAP][0]
    seeded = [T.NetworkClusterPolicy.from_dict(x) for x in yaml.safe_load(cm["data"]["policies.yaml"])["policies"]]
    assert [p.name for p in seeded] == ["netconf-amd-scale-out" if which == "amd" else "netconf-amd-host-nic"]
    assert bool(hooks) == R.needs_node_cleanup(seeded[0]) == (keep or nm)


# Non-default chart values for every field of the two policy specs, and what the seeded policy
# must then carry.  image / pullPolicy come from config.amd.image; layer from `mode`.
_AMD_VALUES = {
    "mode": "L3", "mtu": 4200, "disableNetworkManager": True, "xgmiCheck": False, "lldpAnnounce": False,
    "interfaces": ["ens1np0", "ens2np0"], "nicDrivers": ["mlx5_core", "bnxt_en"], "disableFirmwareLldp": True,
    "metricsPort": 9501, "gpuDirectRdma": "DmaBuf", "rcclEnv": {"NCCL_IB_TC": "106"}, "railTableBase": 100,
    "rcclSocketIfname": "eno1", "lldpCache": True, "verifyPeers": True, "lldpWait": "2m", "carrierWait": "45s",
    "keepConfigOnRestart": True, "railSwitchPattern": "leaf-r{rail}-.*", "minLinkSpeedGbps": 400, "requireFullPcieLink": True,
    "checkPeerMtu": False, "handDcbxToHost": True, "maxUnavailable": "25%", "requireRdma": True, "rdmaWait": "7m",
    "driverImage": "reg/rdma-kmd:1", "allowPolicyRouted": True,
    "validation": {"enabled": True, "minBusbw": 300, "minLink": 40, "gpus": 4, "image": "reg/val:1"},
    "tolerations": [{"key": "amd.com/gpu", "operator": "Exists", "effect": "NoSchedule"}],
    "priorityClassName": "system-node-critical",
    "image": {"repository": "reg/agent", "tag": "9.9", "imagePullPolicy": "Always"},
}
_HOST_NIC_VALUES = {
    "enabled": True, "mode": "L3", "mtu": 4000, "nicDrivers": ["bnxt_en"], "driverImage": "reg/kmd:1",
    "interfaces": ["ens9np0"], "disableNetworkManager": True, "verifyPeers": True, "lldpWait": "45s", "carrierWait": "1m",
    "checkPeerMtu": False, "keepConfigOnRestart": True, "includeGpuRails": True, "minLinkSpeedGbps": 200,
    "requireFullPcieLink": True, "allowPolicyRouted": True,
}


def test_every_policy_field_is_settable_from_the_chart_and_documented():
    """A user of the chart reaches every field of the CRD's amdScaleOut and hostNic specs from
    values.yaml (round 4 added checkPeerMtu and handDcbxToHost to the CRD; the chart exposed only
    some fields), the rendered policies pass admission without warnings, and the chart README
    lists every config value."""
    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.api.v1alpha1 import webhook as W

    # (two releases: includeGpuRails next to an enabled config.amd is refused at render time)
    seeded = {}
    for values in ({"amd": dict(_AMD_VALUES, enabled=True)},
                   {"amd": {"image": _AMD_VALUES["image"]}, "hostNic": _HOST_NIC_VALUES}):
        docs = helm_template(CHART, {"config": values}, NS)
        seeded.update({p["metadata"]["name"]: T.NetworkClusterPolicy.from_dict(p)
                       for p in yaml.safe_load(_configmap_text(docs))["policies"]})
    so = seeded["netconf-amd-scale-out"].spec.amdScaleOut
    want = {k: v for k, v in _AMD_VALUES.items() if k not in ("mode", "image", "validation", "maxUnavailable",
                                                               "tolerations", "priorityClassName")}
    want.update(layer="L3", image="reg/agent:9.9", pullPolicy="Always")
    assert set(want) | {"validation"} == set(T.AmdScaleOutSpec._FIELDS), "a new amdScaleOut field needs a chart value"
    for k, v in want.items():
        assert getattr(so, k) == v, k
    assert so.validation.to_dict() == _AMD_VALUES["validation"]
    assert seeded["netconf-amd-scale-out"].spec.maxUnavailable == "25%"
    assert seeded["netconf-amd-scale-out"].spec.tolerations == _AMD_VALUES["tolerations"]
    assert seeded["netconf-amd-scale-out"].spec.priorityClassName == "system-node-critical"
    assert not so.extra

    hn = seeded["netconf-amd-host-nic"].spec.hostNic
    fields = {f for f in T.HostNicSpec.__dataclass_fields__ if f != "extra"}
    want = {k: v for k, v in _HOST_NIC_VALUES.items() if k not in ("enabled", "mode")}
    want.update(layer="L3", image="reg/agent:9.9", pullPolicy="Always")
    assert set(want) == fields, "a new hostNic field needs a chart value"
    for k, v in want.items():
        assert getattr(hn, k) == v, k
    assert not hn.extra

    # (carrierWait is an L2 setting; these values are an L3 policy)
    # (and the pinned agent tag 9.9 draws the older-agent warning)
    # (and allowPolicyRouted draws its safety warning)
    assert [w for w in W.validate_create(seeded["netconf-amd-scale-out"])
            if "carrierWait" not in w and "pins agent tag '9.9'" not in w and "allowPolicyRouted" not in w] == []
    # (includeGpuRails next to interfaces only draws the "no effect" warning)
    assert [w for w in W.validate_create(seeded["netconf-amd-host-nic"])
            if "includeGpuRails" not in w and "carrierWait" not in w and "allowPolicyRouted" not in w] == []

    # Defaults render the policy the CRD defaults describe: no optional field forced on.
    plain = yaml.safe_load(_configmap_text(helm_template(CHART, {"config": {"amd": {"enabled": True},
                                                                            "hostNic": {"enabled": True}}}, NS)))
    so = plain["policies"][0]["spec"]["amdScaleOut"]
    for k in ("checkPeerMtu", "handDcbxToHost", "lldpAnnounce", "interfaces", "nicDrivers", "gpuDirectRdma",
              "rcclEnv", "rcclSocketIfname"):
        assert k not in so, k
    hn = plain["policies"][1]["spec"]["hostNic"]
    for k in ("interfaces", "disableNetworkManager", "verifyPeers", "lldpWait", "checkPeerMtu",
              "keepConfigOnRestart", "includeGpuRails"):
        assert k not in hn, k

    readme = (CHART / "README.md").read_text()
    values = yaml.safe_load((CHART / "values.yaml").read_text())["config"]
    for section in ("amd", "hostNic"):
        for k in values[section]:
            documented = (f"`config.{section}.{k}`" in readme or f"`config.{section}.{k}." in readme
                          or f"/ `{k}`" in readme)
            assert documented, f"config.{section}.{k} undocumented"


def test_chart_refuses_to_give_the_gpu_rails_to_two_policies():
    """config.hostNic.includeGpuRails next to config.amd.enabled (same node selector): both
    policies' agents would want the rails, and one would fail on every node on its NIC locks.
    The render fails instead, naming the two values."""
    from network_operator_amd.testing.render import RenderError

    with pytest.raises(RenderError) as e:
        helm_template(CHART, {"config": {"amd": {"enabled": True},
                                         "hostNic": {"enabled": True, "includeGpuRails": True}}}, NS)
    assert "includeGpuRails" in str(e.value) and "config.amd" in str(e.value)
    helm_template(CHART, {"config": {"hostNic": {"enabled": True, "includeGpuRails": True}}}, NS)  # alone: fine



def test_monitoring_objects_render_only_when_enabled_and_keep_prometheus_templates():
    """`monitoring.enabled` renders the kustomize tree's prometheus/ objects for Helm users: the
    operator's ServiceMonitor, the agents' PodMonitor and the alert rules, named and placed like
    the release's other objects.  The alerts' own {{ $labels.x }} / {{ $value }} templates reach
    Prometheus as written (Helm raw strings), and the rules are the generator's."""
    kinds = {"ServiceMonitor", "PodMonitor", "PrometheusRule"}
    plain = helm_template(CHART, {}, NS)
    assert not [d for d in plain if d["kind"] in kinds]
    docs = [d for d in helm_template(CHART, {"monitoring": {"enabled": True}}, NS) if d["kind"] in kinds]
    assert sorted(d["kind"] for d in docs) == sorted(kinds)
    for d in docs:
        assert d["metadata"]["name"].startswith(M.PREFIX) and d["metadata"]["namespace"] == NS
    rules = next(d for d in docs if d["kind"] == "PrometheusRule")
    assert rules["spec"] == M.prometheus_rules()["spec"]  # every alert, its {{ $labels.x }} text intact
    summaries = [r["annotations"]["summary"] for g in rules["spec"]["groups"] for r in g["rules"]]
    assert any("{{ $labels.nic }}" in s for s in summaries) and any("{{ $value }}" in s for s in summaries)
    dash = [d for d in helm_template(CHART, {"monitoring": {"enabled": True}}, NS)
            if d["kind"] == "ConfigMap" and d["metadata"]["name"] == M.PREFIX + "dashboard"]
    assert len(dash) == 1 and dash[0]["data"] == M.grafana_dashboard_configmap()["data"]  # the JSON survives Helm
    svc = next(d for d in helm_template(CHART, {}, NS) if d["kind"] == "Service" and d["metadata"]["name"].endswith("metrics"))
    monitor = next(d for d in docs if d["kind"] == "ServiceMonitor")
    assert monitor["spec"]["endpoints"][0]["port"] in [p["name"] for p in svc["spec"]["ports"]]
    assert monitor["spec"]["selector"]["matchLabels"].items() <= svc["metadata"]["labels"].items()
