"""v1alpha1 API: types, deep copy, CRD manifest drift, defaulting / validation webhooks,
AdmissionReview protocol and an end-to-end admission path through the fake API server."""

import asyncio
import base64
import copy
from pathlib import Path

import pytest
import yaml

from network_operator_amd.api.v1alpha1 import crd as CRD
from network_operator_amd.api.v1alpha1 import types as T
from network_operator_amd.api.v1alpha1 import webhook as W

ROOT = Path(__file__).resolve().parent.parent


def _p(ns=None, layer="L3", ctype=T.CONFIG_AMD_SCALE_OUT):
    p = T.new_policy("test", layer=layer, node_selector=ns if ns is not None else {"foo": "bar"})
    p.spec.configurationType = ctype
    return p


# --- types ---------------------------------------------------------------------------------
def test_roundtrip_and_unknown_fields_preserved():
    d = {"apiVersion": "amd.com/v1alpha1", "kind": "NetworkClusterPolicy", "metadata": {"name": "x"},
         "spec": {"configurationType": "amd-so", "nodeSelector": {"a": "b"}, "logLevel": 3,
                  "amdScaleOut": {"layer": "L3", "mtu": 9000, "disableNetworkManager": True, "future": 1},
                  "futureTop": {"k": "v"}},
         "status": {"targets": 2, "ready": 1, "state": "Working on it..", "errors": []}}
    p = T.NetworkClusterPolicy.from_dict(d)
    assert p.spec.amdScaleOut.mtu == 9000 and p.status.ready == 1
    assert p.to_dict() == d


def test_deepcopy_does_not_share_maps_or_slices():
    p = _p({"a": "b"})
    p.status.errors = ["x"]
    q = p.deepcopy()
    q.spec.nodeSelector["a"] = "z"
    q.status.errors.append("y")
    assert p.spec.nodeSelector == {"a": "b"} and p.status.errors == ["x"]


# --- CRD -----------------------------------------------------------------------------------
def test_crd_checked_in_matches_generator():
    text = CRD.render_yaml()
    for f in ("config/operator/crd/bases/amd.com_networkclusterpolicies.yaml",
              "charts/network-operator/crds/networkclusterpolicy-crd.yaml"):
        assert (ROOT / f).read_text() == text, f"{f} is stale: run python -m network_operator_amd.api.v1alpha1.crd"


def test_crd_shape():
    c = yaml.safe_load(CRD.render_yaml())
    assert c["metadata"]["name"] == "networkclusterpolicies.amd.com"
    assert c["spec"]["scope"] == "Cluster"
    v = c["spec"]["versions"][0]
    assert v["name"] == "v1alpha1" and v["subresources"] == {"status": {}}
    s = v["schema"]["openAPIV3Schema"]["properties"]
    assert s["spec"]["required"] == ["configurationType"]
    so = s["spec"]["properties"]["amdScaleOut"]["properties"]
    assert so["layer"]["enum"] == ["L2", "L3"] and so["mtu"]["minimum"] == 1500 and so["mtu"]["maximum"] == 9000
    assert so["pullPolicy"]["enum"] == ["Never", "Always", "IfNotPresent"]
    assert s["status"]["required"] == ["errors", "ready", "state", "targets"]


@pytest.mark.parametrize("spec,ok", [
    ({"configurationType": "amd-so", "amdScaleOut": {"layer": "L3", "mtu": 9000}}, True),
    ({"configurationType": "amd-so", "amdScaleOut": {"layer": "L3BGP"}}, False),
    ({"configurationType": "amd-so", "logLevel": -1}, False),
    ({"configurationType": "amd-so", "nodeSelector": {"a": 1}}, False),
    ({"configurationType": "amd-so", "amdScaleOut": {"interfaces": ["a" * 16]}}, False),
    ({"amdScaleOut": {"layer": "L3"}}, False),
])
def test_schema_validation(spec, ok):
    errs = CRD.validate({"apiVersion": T.API_VERSION, "kind": T.KIND, "metadata": {"name": "x"}, "spec": spec})
    assert (errs == []) == ok, errs


# --- webhook logic (reference networkconfiguration_webhook_test.go) -------------------------
def test_default_image():
    p = _p()
    W.default(p)
    assert p.spec.amdScaleOut.image == T.DEFAULT_AGENT_IMAGE
    p.spec.amdScaleOut.image = "mine:1"
    W.default(p)
    assert p.spec.amdScaleOut.image == "mine:1"
    other = _p(ctype="host-nic")
    W.default(other)
    assert other.spec.amdScaleOut.image == ""


def test_empty_and_unknown():
    with pytest.raises(W.EmptyNodeSelectorError):
        W.validate_create(_p({}))
    with pytest.raises(W.UnknownConfigurationError) as ei:
        W.validate_create(_p(ctype="gaudi-so"))
    assert str(ei.value) == "unknown error"
    # host-nic (reserved in the reference) is implemented here and needs spec.hostNic.
    with pytest.raises(W.MissingHostNicSpecError):
        W.validate_create(_p(ctype="host-nic"))


@pytest.mark.parametrize("sel", [
    {"amd.feature.node.kubernetes.io/gpu-ready": "true"},
    {"gpu.amd.com": "mi355x"},
    {"foo": ""},
])
def test_good_node_selectors(sel):
    assert W.validate_create(_p(sel)) == []


@pytest.mark.parametrize("sel", [
    {"foobar.com?foo": "bar"},
    {"__.com/foo": "bar"},
    {"foo.com_": "bar"},
    {"foo.com": "_bar"},
    {"foo.com": "???foo"},
    {"foo.com": "foo_"},
    {"foo.com": "0123456789012345678901234567890123456789012345678901234567890123"},
    {"foo.com/bar/plaaplaa_": "ok"},
    {"foo.com_/bar": "ok"},
    {"a" * 254: "x"},
    # reference quirk kept: the key *prefix* regex rejects '-'
    {"node-feature.example.com/x": "y"},
])
def test_bad_node_selectors(sel):
    with pytest.raises(W.InvalidNodeSelectorError):
        W.validate_create(_p(sel))


def test_update_and_delete():
    nc = _p()
    nc2 = nc.deepcopy()
    assert W.validate_update(nc2, nc) == []
    nc2.spec.nodeSelector = {"foobar.com?foo": "bar"}
    with pytest.raises(W.ValidationError):
        W.validate_update(nc2, nc)
    bad = _p(layer="L3BGP")
    assert W.validate_delete(bad) == []


def test_interface_names_validated():
    p = _p()
    p.spec.amdScaleOut.interfaces = ["ens1", "bad,name"]
    with pytest.raises(W.InvalidInterfaceError):
        W.validate_create(p)


# --- AdmissionReview --------------------------------------------------------------------------
def test_admission_review_mutate_and_validate():
    obj = _p().to_dict()
    review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview",
              "request": {"uid": "u1", "operation": "CREATE", "object": obj}}
    out = W.admission_review(review, mutate=True)
    assert out["response"]["uid"] == "u1" and out["response"]["allowed"]
    ptype, ops = W.decode_patch(out)
    assert ptype == "JSONPatch"
    assert {"op": "add", "path": "/spec/amdScaleOut/image", "value": T.DEFAULT_AGENT_IMAGE} in ops
    out = W.admission_review(review, mutate=False)
    assert out["response"]["allowed"]
    bad = copy.deepcopy(review)
    bad["request"]["object"]["spec"]["nodeSelector"] = {}
    out = W.admission_review(bad, mutate=False)
    assert not out["response"]["allowed"] and out["response"]["status"]["message"] == "empty node-selector"
    delete = {"request": {"uid": "u2", "operation": "DELETE", "oldObject": bad["request"]["object"]}}
    assert W.admission_review(delete, mutate=False)["response"]["allowed"]


def test_json_patch_roundtrip():
    from network_operator_amd.testing.fakeapi import json_patch_apply

    a = {"x": {"y": 1, "z": [1, 2]}, "k/~": 1}
    b = {"x": {"y": 2, "w": 3, "z": [1, 2]}, "n": None}
    assert json_patch_apply(a, W.json_patch(a, b)) == b


# --- end-to-end admission through the fake API server -------------------------------------------
def _webhook_config(kind, url, ca, resource):
    name = "mpolicy.amd.com" if kind == "Mutating" else "vpolicy.amd.com"
    path = W.MUTATE_PATH if kind == "Mutating" else W.VALIDATE_PATH
    return {"apiVersion": "admissionregistration.k8s.io/v1", "kind": f"{kind}WebhookConfiguration",
            "metadata": {"name": f"amd-network-{kind.lower()}-webhook-configuration"},
            "webhooks": [{"name": name, "admissionReviewVersions": ["v1"], "sideEffects": "None",
                          "failurePolicy": "Fail",
                          "clientConfig": {"url": url + path, "caBundle": base64.b64encode(ca).decode()},
                          "rules": [{"apiGroups": ["amd.com"], "apiVersions": ["v1alpha1"],
                                     "operations": ["CREATE", "UPDATE"], "resources": [resource]}]}]}


@pytest.mark.parametrize("resource,called", [("networkclusterpolicies", True), ("networkclusterpolicy", False)])
def test_webhooks_end_to_end(tmp_path, resource, called):
    """With the plural resource the API server calls the webhooks (defaulting + validation);
    with the singular — what the reference registers — it never does."""
    from network_operator_amd.operator import kube
    from network_operator_amd.operator.kube import ApiClient, ApiError, KubeConfig
    from network_operator_amd.operator.metrics import OperatorMetrics
    from network_operator_amd.operator.servers import Servers, generate_self_signed
    from network_operator_amd.testing.fakeapi import FakeApiServer

    crt, key = generate_self_signed(tmp_path / "certs")

    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        srv = Servers(OperatorMetrics())
        await srv.start(probe_addr="127.0.0.1:0", webhook_port=0, cert_dir=str(tmp_path / "certs"))
        wurl = f"https://127.0.0.1:{srv.ports['webhook']}"
        async with ApiClient(KubeConfig(host=url)) as c:
            await c.create(kube.MUTATINGWEBHOOKS, _webhook_config("Mutating", wurl, crt.read_bytes(), resource))
            await c.create(kube.VALIDATINGWEBHOOKS, _webhook_config("Validating", wurl, crt.read_bytes(), resource))
            created = await c.create(kube.NETWORKCLUSTERPOLICIES, _p().to_dict())
            bad = _p({"foo.com": "_bar"}).to_dict()
            bad["metadata"]["name"] = "bad"
            if called:
                assert created["spec"]["amdScaleOut"]["image"] == T.DEFAULT_AGENT_IMAGE
                with pytest.raises(ApiError) as ei:
                    await c.create(kube.NETWORKCLUSTERPOLICIES, bad)
                assert ei.value.status == 403 and "invalid node selector" in ei.value.message
                assert len(fake.admission_calls) >= 3
            else:
                assert "image" not in created["spec"]["amdScaleOut"]
                await c.create(kube.NETWORKCLUSTERPOLICIES, bad)  # nothing stops it
                assert fake.admission_calls == []
        await srv.stop()
        await fake.stop()

    asyncio.run(asyncio.wait_for(body(), 60))


def test_rccl_socket_ifname_field_validated_and_passed_to_the_agent():
    from network_operator_amd.api.v1alpha1 import crd as CRD2
    from network_operator_amd.operator.reconciler import agent_args

    def pol(v):
        p = T.new_policy("p", rcclSocketIfname=v).to_dict()
        return p, CRD2.validate(p)

    for ok in ("auto", "none", "enp8s0np0", "enp8s0np0,enp33s0np0"):
        p, errs = pol(ok)
        assert errs == [], (ok, errs)
        assert f"--rccl-socket-ifname={ok}" in agent_args(T.NetworkClusterPolicy.from_dict(p))
    for bad in ("", "a b", "x,", "waytoolonginterfacename0", "eth0;rm -rf"):
        if bad == "":
            assert "--rccl-socket-ifname" not in " ".join(agent_args(T.new_policy("p")))
            continue
        assert pol(bad)[1], bad


def test_lldp_cache_field_passed_to_the_agent_in_l3_only():
    from network_operator_amd.api.v1alpha1 import crd as CRD2
    from network_operator_amd.operator.reconciler import agent_args

    p = T.new_policy("p", lldpCache=True).to_dict()
    assert CRD2.validate(p) == [] and p["spec"]["amdScaleOut"]["lldpCache"] is True
    assert "--lldp-cache=/host/etc/amd/scale-out/lldp-cache" in agent_args(T.NetworkClusterPolicy.from_dict(p))
    assert "--lldp-cache" not in " ".join(agent_args(T.new_policy("p")))
    l2 = T.new_policy("p", lldpCache=True, layer="L2")
    assert "--lldp-cache" not in " ".join(agent_args(l2))
    assert CRD2.validate(dict(p, spec=dict(p["spec"], amdScaleOut={"lldpCache": "yes"})))


@pytest.mark.parametrize("resource", ["networkclusterpolicies", "networkclusterpolicy"])
def test_a_minimal_amd_so_policy_verifies_the_xgmi_mesh_and_rdma_by_default(tmp_path, resource):
    """MI355X-first defaults: a policy written with kubectl as just a type and a
    selector -- no amdScaleOut at all -- comes back with xgmiCheck and requireRdma true, from the
    real webhook server (plural registration) and, with the webhooks never called (the singular),
    from the CRD schema's defaults alone; its DaemonSet's agent checks the mesh and the RDMA devices."""
    from network_operator_amd import discovery
    from network_operator_amd.operator import kube
    from network_operator_amd.operator.kube import ApiClient, KubeConfig
    from network_operator_amd.operator.metrics import OperatorMetrics
    from network_operator_amd.operator.servers import Servers, generate_self_signed
    from network_operator_amd.operator.templates import update_daemonset_for
    from network_operator_amd.testing.fakeapi import FakeApiServer

    crt, _ = generate_self_signed(tmp_path / "certs")
    minimal = {"apiVersion": T.API_VERSION, "kind": T.KIND, "metadata": {"name": "minimal"},
               "spec": {"configurationType": "amd-so", "nodeSelector": {"amd.feature.node.kubernetes.io/gpu-ready": "true"}}}

    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        srv = Servers(OperatorMetrics())
        await srv.start(probe_addr="127.0.0.1:0", webhook_port=0, cert_dir=str(tmp_path / "certs"))
        wurl = f"https://127.0.0.1:{srv.ports['webhook']}"
        async with ApiClient(KubeConfig(host=url)) as c:
            await c.create(kube.MUTATINGWEBHOOKS, _webhook_config("Mutating", wurl, crt.read_bytes(), resource))
            await c.create(kube.VALIDATINGWEBHOOKS, _webhook_config("Validating", wurl, crt.read_bytes(), resource))
            created = await c.create(kube.NETWORKCLUSTERPOLICIES, copy.deepcopy(minimal))
        await srv.stop()
        await fake.stop()
        return created

    created = asyncio.run(asyncio.wait_for(body(), 60))
    so = created["spec"]["amdScaleOut"]
    assert so["xgmiCheck"] is True and so["requireRdma"] is True, so
    ds = discovery.discovery_daemonset()
    update_daemonset_for(ds, T.NetworkClusterPolicy.from_dict(created), "amd-network-operator")
    args = ds["spec"]["template"]["spec"]["containers"][0]["args"]
    assert "--xgmi-expect=0" in args and "--require-rdma" in args, args
    # Turned off explicitly, they stay off (the defaults fill only what is absent).
    off = copy.deepcopy(minimal)
    off["spec"]["amdScaleOut"] = {"xgmiCheck": False, "requireRdma": False}
    CRD.apply_defaults(off, CRD.openapi_schema())
    assert off["spec"]["amdScaleOut"] == {"xgmiCheck": False, "requireRdma": False}


def test_every_sample_policy_is_admitted_and_renders_its_agent():
    """config/operator/samples/*.yaml: each passes the CRD schema and the webhooks, and its
    DaemonSet passes what the sample asks for (the Pollara sample: the RDMA driver container and
    --require-rdma / --rdma-wait)."""
    from network_operator_amd import discovery
    from network_operator_amd.operator.templates import update_daemonset_for

    root = Path(__file__).resolve().parent.parent / "config" / "operator" / "samples"
    seen = {}
    for f in sorted(root.glob("*.yaml")):
        if f.name == "kustomization.yaml":
            continue
        obj = yaml.safe_load(f.read_text())
        assert CRD.validate(obj) == [], (f.name, CRD.validate(obj))
        pol = W.default(T.NetworkClusterPolicy.from_dict(obj))
        assert [w for w in W.validate_create(pol) if "no interfaces or nicDrivers" not in w] == [], f.name
        ds = discovery.discovery_daemonset()
        update_daemonset_for(ds, pol, "amd-network-operator")
        seen[f.name] = ds["spec"]["template"]["spec"]
    pollara = seen["amd-l3-pollara.yaml"]
    args = pollara["containers"][0]["args"]
    assert "--require-rdma" in args and "--rdma-wait=10m" in args and "--nic-drivers=ionic" in args, args
    assert [c["name"] for c in pollara["initContainers"]] == ["nic-driver"]
    assert pollara["initContainers"][0]["securityContext"] == {"privileged": True}
