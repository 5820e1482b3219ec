"""Migration from the Gaudi network operator (``api/v1alpha1/migrate.py``): its policies and
Helm values are converted into objects this operator's CRD schema and webhook admit, with every
change named.  The reference's own samples and chart values are converted too when the reference
tree is present (they are read with ``yaml.safe_load``, nothing else)."""

import asyncio
import subprocess
import sys
from pathlib import Path

import pytest
import yaml

from network_operator_amd.api.v1alpha1 import migrate as M
from network_operator_amd.api.v1alpha1 import types as T
from network_operator_amd.operator import kube
from network_operator_amd.operator.kube import ApiClient, KubeConfig
from network_operator_amd.packaging import manifests as PM
from network_operator_amd.testing.fakeapi import FakeApiServer
from network_operator_amd.testing.render import helm_template

ROOT = Path(__file__).resolve().parent.parent
REFERENCE = Path("/root/reference")

# The shape of the reference's samples (config/operator/samples/gaudi-l3.yaml), as a cluster
# returns it: server-written metadata, a last-applied annotation, a status.
GAUDI_L3 = """
apiVersion: intel.com/v1alpha1
kind: NetworkClusterPolicy
metadata:
  name: netconf-gaudi-scale-out-l3
  uid: 0b5c6e2a-1111-2222-3333-444455556666
  resourceVersion: "81234"
  generation: 3
  creationTimestamp: "2025-01-02T03:04:05Z"
  finalizers: [intel.com/something]
  labels: {team: infra}
  annotations:
    kubectl.kubernetes.io/last-applied-configuration: '{"apiVersion":"intel.com/v1alpha1"}'
    owner: platform
spec:
  configurationType: gaudi-so
  gaudiScaleOut:
    layer: L3
    image: intel/intel-network-linkdiscovery:1.0.0
    pullPolicy: IfNotPresent
    mtu: 8000
    disableNetworkManager: true
  logLevel: 1
  nodeSelector:
    intel.feature.node.kubernetes.io/gaudi-ready: "true"
    rack: a
status: {targets: 4, ready: 4, state: All good, errors: []}
"""


def test_a_gaudi_policy_becomes_an_amd_so_policy_that_is_admitted():
    objs, notes, errors = M.convert_policies(GAUDI_L3)
    assert errors == []
    assert objs == [{
        "apiVersion": "amd.com/v1alpha1", "kind": "NetworkClusterPolicy",
        "metadata": {"name": "netconf-gaudi-scale-out-l3", "labels": {"team": "infra"},
                     "annotations": {"owner": "platform"}},
        "spec": {"configurationType": "amd-so",
                 "amdScaleOut": {"disableNetworkManager": True, "layer": "L3", "pullPolicy": "IfNotPresent", "mtu": 8000,
                                 "xgmiCheck": True, "requireRdma": True},
                 "nodeSelector": {"amd.feature.node.kubernetes.io/gpu-ready": "true", "rack": "a"},
                 "logLevel": 1}}]
    text = "\n".join(notes)
    assert "is the Gaudi agent -> amd/amd-network-linkdiscovery" in text
    assert "gaudi-ready -> amd.feature.node.kubernetes.io/gpu-ready" in text
    assert "last-applied-configuration" in text and "gpu-scale-out=true" in text and "rccl.env" in text
    assert "xgmiCheck and requireRdma set true" in text
    assert M.admission_errors(objs[0]) == []
    # An explicit image wins; a non-Gaudi image is kept, with a note to check it.
    objs, notes, _ = M.convert_policies(GAUDI_L3, image="reg/agent:2")
    assert objs[0]["spec"]["amdScaleOut"]["image"] == "reg/agent:2"
    mine = GAUDI_L3.replace("intel/intel-network-linkdiscovery:1.0.0", "reg.local:5000/agent:3")
    objs, notes, _ = M.convert_policies(mine)
    assert objs[0]["spec"]["amdScaleOut"]["image"] == "reg.local:5000/agent:3"
    assert any("kept: make sure" in n for n in notes)


def test_the_converted_policy_is_created_and_reconciled_like_any_other():
    """Through the fake API server's schema check and the operator: the migrated policy gets its
    DaemonSet with the AMD agent image and selector."""
    from network_operator_amd.operator.controller import PolicyController

    async def body():
        fake = FakeApiServer()
        url = await fake.start()
        client = ApiClient(KubeConfig(host=url))
        ctl = PolicyController(client, "amd-network-operator", workers=1)
        await ctl.start()
        try:
            obj = M.convert_policies(GAUDI_L3)[0][0]
            obj["spec"]["amdScaleOut"]["image"] = T.DEFAULT_AGENT_IMAGE  # what the mutating webhook adds
            await client.create(kube.NETWORKCLUSTERPOLICIES, obj)
            for _ in range(250):
                ds = fake.get_object(kube.DAEMONSETS, "netconf-gaudi-scale-out-l3", "amd-network-operator")
                if ds:
                    break
                await asyncio.sleep(0.02)
            pod = ds["spec"]["template"]["spec"]
            assert pod["nodeSelector"] == {"amd.feature.node.kubernetes.io/gpu-ready": "true", "rack": "a"}
            assert pod["containers"][0]["image"] == T.DEFAULT_AGENT_IMAGE
            assert "--mtu=8000" in pod["containers"][0]["args"]
        finally:
            await ctl.stop()
            await client.close()
            await fake.stop()

    asyncio.run(asyncio.wait_for(body(), 30))


def test_lists_several_documents_and_what_cannot_be_converted():
    doc2 = GAUDI_L3.replace("netconf-gaudi-scale-out-l3", "second").replace("layer: L3", "layer: L2")
    listed = yaml.safe_dump({"apiVersion": "v1", "kind": "List", "items": [yaml.safe_load(GAUDI_L3),
                                                                          yaml.safe_load(doc2)]})
    objs, _, errors = M.convert_policies(listed + "---\n" + doc2.replace("name: second", "name: third"))
    assert [o["metadata"]["name"] for o in objs] == ["netconf-gaudi-scale-out-l3", "second", "third"] and not errors
    # Out of range for the CRD (the reference's own bounds: mtu 1500..9000): converted, but an error.
    objs, _, errors = M.convert_policies(GAUDI_L3.replace("mtu: 8000", "mtu: 900"))
    assert len(objs) == 1 and len(errors) == 1 and "would not be admitted" in errors[0] and "mtu" in errors[0]
    # A type without a counterpart, a foreign group, another kind: named, nothing emitted.
    bad = GAUDI_L3.replace("gaudi-so", "host-nic") + "---\n" + GAUDI_L3.replace("intel.com", "example.com") + \
        "---\napiVersion: v1\nkind: ConfigMap\nmetadata: {name: x}\n"
    objs, _, errors = M.convert_policies(bad)
    assert objs == [] and len(errors) == 3
    # Unknown fields are dropped by name.
    extra = GAUDI_L3.replace("  logLevel: 1", "  logLevel: 1\n  futureField: 1").replace(
        "    mtu: 8000", "    mtu: 8000\n    gaudiOnly: x")
    _, notes, errors = M.convert_policies(extra)
    assert not errors and any("spec.futureField" in n for n in notes) and any("gaudiScaleOut.gaudiOnly" in n for n in notes)
    # Already converted: passed through.
    objs, notes, _ = M.convert_policies(yaml.safe_dump(T.new_policy("mine").to_dict()))
    assert objs[0]["metadata"]["name"] == "mine" and "unchanged" in notes[0]


def test_command_line_exit_status_and_streams(tmp_path):
    f = tmp_path / "p.yaml"
    f.write_text(GAUDI_L3)
    r = subprocess.run([sys.executable, "-m", "network_operator_amd.api.v1alpha1.migrate", str(f)],
                       capture_output=True, text=True, cwd=ROOT, timeout=60)
    assert r.returncode == 0, r.stderr
    assert list(yaml.safe_load_all(r.stdout))[0]["spec"]["configurationType"] == "amd-so"
    assert "note:" in r.stderr
    f.write_text(GAUDI_L3.replace("mtu: 8000", "mtu: 100000"))
    r = subprocess.run([sys.executable, "-m", "network_operator_amd.api.v1alpha1.migrate", str(f)],
                       capture_output=True, text=True, cwd=ROOT, timeout=60)
    assert r.returncode == 1 and "error:" in r.stderr


REFERENCE_VALUES = {
    "logLevel": 2,
    "operator": {"image": {"repository": "intel/intel-network-operator", "tag": "1.0.0",
                           "imagePullPolicy": "IfNotPresent"},
                 "resources": {"limits": {"cpu": "500m", "memory": "128Mi"},
                               "requests": {"cpu": "10m", "memory": "64Mi"}}},
    "nfd": {"install": False, "gaudiRule": True},
    "config": {"gaudi": {"enabled": True, "mode": "L3", "mtu": 8000,
                         "image": {"repository": "intel/intel-network-linkdiscovery", "tag": "1.0.0",
                                   "imagePullPolicy": "IfNotPresent"},
                         "nodeSelector": {"intel.feature.node.kubernetes.io/gaudi-ready": "true"}}},
}


def _render(values):
    docs = helm_template(ROOT / "charts" / "network-operator", values, "amd-network-operator")
    cm = [d for d in docs if d["kind"] == "ConfigMap" and d["metadata"]["name"] == PM.POLICIES_CONFIGMAP][0]
    dep = [d for d in docs if d["kind"] == "Deployment"][0]
    return yaml.safe_load(cm["data"]["policies.yaml"])["policies"], dep


def test_reference_chart_values_render_an_amd_release():
    values, notes = M.convert_values(REFERENCE_VALUES)
    assert values["nfd"] == {"install": False, "amdGpuRule": True}
    assert values["operator"]["image"] == {"repository": "amd/amd-network-operator", "imagePullPolicy": "IfNotPresent"}
    assert "tag" not in values["config"]["amd"]["image"]
    assert any("config.gaudi -> config.amd" in n for n in notes)
    policies, dep = _render(values)
    assert len(policies) == 1
    p = policies[0]
    assert p["spec"]["configurationType"] == "amd-so"
    assert p["spec"]["nodeSelector"] == {"amd.feature.node.kubernetes.io/gpu-ready": "true"}
    assert p["spec"]["amdScaleOut"]["layer"] == "L3" and p["spec"]["amdScaleOut"]["mtu"] == 8000
    assert p["spec"]["amdScaleOut"]["image"].startswith("amd/amd-network-linkdiscovery:")
    assert M.admission_errors(p) == []
    image = dep["spec"]["template"]["spec"]["containers"][0]["image"]
    assert image.startswith("amd/amd-network-operator:") and not image.endswith(":1.0.0")


@pytest.mark.skipif(not (REFERENCE / "config/operator/samples").is_dir(), reason="reference tree not present")
def test_the_reference_samples_and_chart_values_convert_and_are_admitted():
    """Parity pinned on the reference's own files: both samples and the chart's values."""
    for sample in sorted((REFERENCE / "config/operator/samples").glob("*.yaml")):
        objs, _, errors = M.convert_policies(sample.read_text())
        assert errors == [] and len(objs) == 1, (sample.name, errors)
        assert objs[0]["spec"]["nodeSelector"] == {"amd.feature.node.kubernetes.io/gpu-ready": "true"}
    values, _ = M.convert_values(yaml.safe_load((REFERENCE / "charts/network-operator/values.yaml").read_text()))
    values["config"]["amd"]["enabled"] = True  # the reference ships it disabled
    policies, _ = _render(values)
    assert [M.admission_errors(p) for p in policies] == [[]]
