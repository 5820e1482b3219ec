"""Deployment artefacts: Helm chart, kustomize tree, samples, NFD rule, Dockerfiles.

Rendered with the offline renderers in ``network_operator_amd.testing.render`` (no helm /
kustomize binaries in this environment)."""

import json
from pathlib import Path

import pytest
import yaml

from network_operator_amd.api.v1alpha1 import crd as CRD
from network_operator_amd.api.v1alpha1 import types as T
from network_operator_amd.api.v1alpha1 import webhook as W
from network_operator_amd.packaging import manifests as M
from network_operator_amd.testing.render import RenderError, helm_template, kustomize_build, render_template

ROOT = Path(__file__).resolve().parent.parent
CHART = ROOT / "charts" / "network-operator"


def _by_kind(docs, kind):
    return [d for d in docs if d["kind"] == kind]


def _chart_policies(docs):
    """The policies a Helm release asks for: the ConfigMap the operator seeds them from."""
    cm = [d for d in docs if d["kind"] == "ConfigMap" and d["metadata"]["name"] == M.POLICIES_CONFIGMAP]
    assert len(cm) == 1
    return (yaml.safe_load(cm[0]["data"]["policies.yaml"]) or {}).get("policies") or []


HELM_SEED_ARGS = [f"--policies-file={M.POLICIES_DIR}/policies.yaml", "--policies-owner=ClusterRole/amd-network-operator"]


def _rules_allow(roles, group, resource, verb):
    for r in roles:
        for rule in r.get("rules", []):
            if group in rule.get("apiGroups", []) and resource in rule.get("resources", []) and verb in rule.get("verbs", []):
                return True
    return False


def test_render_template_subset():
    src = '{{- $v := list "a" "b" }}x: {{ .Values.k | default "d" | quote }}\n{{- if has .Values.m $v }}\nok: {{ .Values.n }}\n{{- else }}\nno\n{{- end }}'
    assert render_template(src, {"k": "", "m": "a", "n": 3}) == 'x: "d"\nok: 3'
    assert render_template(src, {"k": "z", "m": "q"}) == 'x: "z"\nno'


def test_helm_defaults():
    docs = helm_template(CHART, namespace="amd-net")
    kinds = {d["kind"] for d in docs}
    assert {"Deployment", "ClusterRole", "Role", "RoleBinding", "ClusterRoleBinding", "Service", "Certificate", "Issuer",
            "ServiceAccount", "MutatingWebhookConfiguration", "ValidatingWebhookConfiguration",
            "CustomResourceDefinition", "NodeFeatureRule"} <= kinds
    assert not _by_kind(docs, "NetworkClusterPolicy")  # never a release object (see operator/seeder.py)
    assert _chart_policies(docs) == []  # config.amd.enabled defaults to false
    dep = _by_kind(docs, "Deployment")[0]
    assert dep["metadata"]["namespace"] == "amd-net"
    c = dep["spec"]["template"]["spec"]["containers"][0]
    assert c["args"] == M.operator_args(metrics=True) + HELM_SEED_ARGS
    assert {"name": "policies", "configMap": {"name": M.POLICIES_CONFIGMAP, "optional": True}} in \
        dep["spec"]["template"]["spec"]["volumes"]
    assert "--metrics-bind-address=:8443" in c["args"] and "--leader-elect" in c["args"]
    assert c["image"] == "amd/amd-network-operator:0.1.0"
    assert dep["spec"]["replicas"] == 1
    assert {"name": "POD_NAME", "valueFrom": {"fieldRef": {"fieldPath": "metadata.name"}}} in c["env"]
    two = _by_kind(helm_template(CHART, {"operator": {"replicas": 2}}, "amd-net"), "Deployment")[0]
    assert two["spec"]["replicas"] == 2  # an integer, not the string "2"
    assert c["resources"] == M.RESOURCES and c["imagePullPolicy"] == "IfNotPresent"
    cert = _by_kind(docs, "Certificate")[0]
    assert cert["spec"]["dnsNames"][0] == "amd-network-webhook.amd-net.svc"
    assert dep["spec"]["template"]["spec"]["volumes"][0]["secret"]["secretName"] == cert["spec"]["secretName"]
    for wh in _by_kind(docs, "MutatingWebhookConfiguration") + _by_kind(docs, "ValidatingWebhookConfiguration"):
        rule = wh["webhooks"][0]["rules"][0]
        assert rule["resources"] == [T.PLURAL]  # fixed: the reference registers the singular
        path = wh["webhooks"][0]["clientConfig"]["service"]["path"]
        assert path in (W.MUTATE_PATH, W.VALIDATE_PATH)
    roles = _by_kind(docs, "ClusterRole") + _by_kind(docs, "Role")
    for res, verb in (("daemonsets", "create"), ("daemonsets", "update"), ("serviceaccounts", "create"),
                      ("events", "create"), ("networkclusterpolicies", "watch")):
        grp = {"daemonsets": "apps", "networkclusterpolicies": "amd.com"}.get(res, "")
        assert _rules_allow(roles, grp, res, verb), (res, verb)
    assert _rules_allow(roles, "amd.com", "networkclusterpolicies/status", "update")
    assert _rules_allow(roles, "rbac.authorization.k8s.io", "rolebindings", "create")
    assert _rules_allow(roles, "coordination.k8s.io", "leases", "update")
    assert _rules_allow(roles, "authentication.k8s.io", "tokenreviews", "create")


def test_helm_policy_rendering_and_validation():
    docs = helm_template(CHART, {"config": {"amd": {"enabled": True, "mode": "L3", "mtu": 9000}}})
    assert not _by_kind(docs, "NetworkClusterPolicy")
    cr = _chart_policies(docs)[0]
    assert CRD.validate(cr) == []
    assert W.validate_create(T.NetworkClusterPolicy.from_dict(cr)) == []
    assert cr["spec"]["amdScaleOut"]["image"] == "amd/amd-network-linkdiscovery:0.1.0"
    assert cr["spec"]["nodeSelector"] == {"amd.feature.node.kubernetes.io/gpu-ready": "true"}
    assert cr["spec"]["amdScaleOut"]["xgmiCheck"] is True
    assert "lldpWait" not in cr["spec"]["amdScaleOut"]  # the agent's 90s
    waited = _chart_policies(helm_template(CHART, {"config": {"amd": {"enabled": True, "lldpWait": "15s"}}}))[0]
    assert waited["spec"]["amdScaleOut"]["lldpWait"] == "15s" and CRD.validate(waited) == []
    assert "keepConfigOnRestart" not in cr["spec"]["amdScaleOut"] and not [
        d for d in docs if d["kind"] == "Job"]  # no pre-delete hook without keepConfigOnRestart
    keep_docs = helm_template(CHART, {"config": {"amd": {"enabled": True, "keepConfigOnRestart": True}}})
    kept = _chart_policies(keep_docs)[0]
    assert kept["spec"]["amdScaleOut"]["keepConfigOnRestart"] is True and CRD.validate(kept) == []
    hook = _by_kind(keep_docs, "Job")
    assert len(hook) == 1 and hook[0]["metadata"]["annotations"]["helm.sh/hook"] == "pre-delete"
    c = hook[0]["spec"]["template"]["spec"]["containers"][0]
    assert c["command"] == ["python3", "-m", "network_operator_amd.operator.predelete"]
    assert "--owner=ClusterRole/amd-network-operator" in c["args"]
    assert hook[0]["spec"]["template"]["spec"]["serviceAccountName"] == "amd-network-operator"
    with pytest.raises(RenderError, match="Invalid layer mode"):
        helm_template(CHART, {"config": {"amd": {"enabled": True, "mode": "L4"}}})
    for mtu in (1499, 9001):
        with pytest.raises(RenderError, match="MTU must be between 1500 and 9000"):
            helm_template(CHART, {"config": {"amd": {"enabled": True, "mtu": mtu}}})


def test_kustomize_default_build():
    docs = kustomize_build(ROOT / "config/operator/default")
    dep = _by_kind(docs, "Deployment")[0]
    assert dep["metadata"]["name"] == "amd-network-operator"
    assert dep["metadata"]["namespace"] == "amd-network-operator"
    pod = dep["spec"]["template"]["spec"]
    c = pod["containers"][0]
    assert c["image"] == "amd/amd-network-operator:0.1.0"
    assert c["args"] == M.operator_args(metrics=True)  # the default overlay's metrics patch
    assert {"containerPort": 9443, "name": "webhook", "protocol": "TCP"} in c["ports"]
    assert {"containerPort": 8443, "name": "metrics", "protocol": "TCP"} in c["ports"]
    assert pod["volumes"][0]["secret"]["secretName"] == "amd-network-webhook-tls"
    assert c["volumeMounts"][0]["mountPath"] == M.CERT_DIR
    assert pod["serviceAccountName"] == "amd-network-operator"
    cert = _by_kind(docs, "Certificate")[0]
    assert cert["spec"]["secretName"] == "amd-network-webhook-tls"
    assert cert["spec"]["issuerRef"]["name"] in {d["metadata"]["name"] for d in _by_kind(docs, "Issuer")}
    svc_names = {d["metadata"]["name"] for d in _by_kind(docs, "Service")}
    assert cert["spec"]["dnsNames"][0].split(".")[0] in svc_names
    ns = _by_kind(docs, "Namespace")[0]
    assert ns["metadata"]["name"] == "amd-network-operator"
    for crb in _by_kind(docs, "ClusterRoleBinding") + _by_kind(docs, "RoleBinding"):
        for s in crb["subjects"]:
            assert s["namespace"] == "amd-network-operator"
        if crb["roleRef"]["kind"] != "ClusterRole" or not crb["roleRef"]["name"].startswith("system:"):
            assert crb["roleRef"]["name"].startswith("amd-network-")
    for wh in _by_kind(docs, "MutatingWebhookConfiguration"):
        svc = wh["webhooks"][0]["clientConfig"]["service"]
        assert svc == {"name": "amd-network-webhook", "namespace": "amd-network-operator",
                       "path": W.MUTATE_PATH}
        assert wh["webhooks"][0]["rules"][0]["resources"] == [T.PLURAL]
        assert wh["metadata"]["annotations"]["cert-manager.io/inject-ca-from"] == \
            "amd-network-operator/" + cert["metadata"]["name"]
    crd = _by_kind(docs, "CustomResourceDefinition")[0]
    assert crd == yaml.safe_load(CRD.render_yaml())
    names = {d["metadata"]["name"] for d in docs}
    assert "amd-network-operator-metrics" in names


def test_generated_manifests_up_to_date():
    """Every generated kustomize / Helm file matches the generator (`make manifests`), and no
    stale file from an earlier layout is left in a generated directory."""
    assert M.check() == []


def test_kustomize_and_helm_install_the_same_operator():
    """The two install paths come from one description: same RBAC rules, same Deployment pod
    apart from the Helm placeholders, same webhook registrations."""
    kz = kustomize_build(ROOT / "config/operator/default")
    hm = helm_template(CHART, namespace="amd-network-operator")

    def rules(docs):
        # The Helm operator's one extra rule: reading its own ClusterRole (the seeded policies' owner).
        seed = M.rbac.policy_owner_rule("amd-network-operator")
        return sorted((r["metadata"]["name"], yaml.safe_dump([x for x in r["rules"] if x != seed]))
                      for r in _by_kind(docs, "ClusterRole"))

    assert rules(kz) == rules(hm)
    kp = _by_kind(kz, "Deployment")[0]["spec"]["template"]["spec"]
    hp = _by_kind(hm, "Deployment")[0]["spec"]["template"]["spec"]
    kc, hc = kp["containers"][0], hp["containers"][0]
    # Helm alone seeds the release's policies (kustomize users apply config/operator/samples).
    assert kc["args"] + HELM_SEED_ARGS == hc["args"] and kc["ports"] == hc["ports"] and kc["resources"] == hc["resources"]
    assert kp["volumes"] == [v for v in hp["volumes"] if v["name"] != "policies"]
    assert kp["serviceAccountName"] == hp["serviceAccountName"]
    for kind in ("MutatingWebhookConfiguration", "ValidatingWebhookConfiguration"):
        assert _by_kind(kz, kind)[0]["webhooks"] == _by_kind(hm, kind)[0]["webhooks"]
        assert _by_kind(kz, kind)[0]["metadata"]["annotations"] == _by_kind(hm, kind)[0]["metadata"]["annotations"]


def test_kustomize_manifests_and_samples_validate():
    docs = kustomize_build(ROOT / "config/operator/manifests")
    crs = _by_kind(docs, "NetworkClusterPolicy")
    assert {c["spec"].get("amdScaleOut", c["spec"].get("hostNic", {}))["layer"] for c in crs} == {"L2", "L3"}
    assert {c["spec"]["configurationType"] for c in crs} == {"amd-so", "host-nic"}
    for c in crs:
        assert CRD.validate(c) == []
        assert W.validate_create(T.NetworkClusterPolicy.from_dict(c)) == []


def test_nfd_rules_consistent():
    kz = yaml.safe_load((ROOT / "config/nfd/amd-gpu-device-rule.yaml").read_text())
    helm = [d for d in helm_template(CHART) if d["kind"] == "NodeFeatureRule"][0]
    assert kz["spec"] == helm["spec"]
    devs = kz["spec"]["rules"][0]["matchFeatures"][0]["matchExpressions"]["device"]["value"]
    assert "75a3" in devs  # MI355X, verified on hardware (tests/fixtures/mi355x_node_topology.json)
    ready = kz["spec"]["rules"][1]
    assert ready["labels"] == {"amd.feature.node.kubernetes.io/gpu-ready": "true"}


def test_dockerfiles_build_the_native_agent():
    op = (ROOT / "build/Dockerfile.operator").read_text()
    agent = (ROOT / "build/Dockerfile.linkdiscovery").read_text()
    assert "network_operator_amd.operator" in op and "USER 65532" in op
    assert "discover" in agent and "cmake" in agent
    assert "setcap" not in agent  # capabilities come from the DaemonSet, not file caps in the image


def test_build_installer_single_file(tmp_path):
    from network_operator_amd import packaging

    docs = packaging.installer(img="registry.local/op:1.2")
    kinds = [d["kind"] for d in docs]
    assert kinds.count("CustomResourceDefinition") == 1 and "Deployment" in kinds
    assert "MutatingWebhookConfiguration" in kinds and "ValidatingWebhookConfiguration" in kinds
    dep = [d for d in docs if d["kind"] == "Deployment"][0]
    assert dep["spec"]["template"]["spec"]["containers"][0]["image"] == "registry.local/op:1.2"
    assert packaging.main(["installer", "--out", str(tmp_path / "install.yaml")]) == 0
    assert len(list(yaml.safe_load_all((tmp_path / "install.yaml").read_text()))) == len(docs)


def test_olm_bundle_matches_installer(tmp_path):
    from network_operator_amd import packaging

    b = packaging.bundle(version="0.2.0", img="x/op:0.2.0")
    csv = b["manifests"]["amd-network-operator.clusterserviceversion.yaml"]
    assert csv["metadata"]["name"] == "amd-network-operator.v0.2.0" and csv["spec"]["version"] == "0.2.0"
    assert csv["spec"]["customresourcedefinitions"]["owned"][0]["name"] == "networkclusterpolicies.amd.com"
    perms = csv["spec"]["install"]["spec"]
    rules = perms["clusterPermissions"][0]["rules"]
    assert any("daemonsets" in r.get("resources", []) for r in rules)
    assert any("networkclusterpolicies/status" in r.get("resources", []) for r in rules)
    assert any("leases" in r.get("resources", []) for r in perms["permissions"][0]["rules"])
    dep = perms["deployments"][0]
    assert dep["spec"]["template"]["spec"]["containers"][0]["image"] == "x/op:0.2.0"
    assert all(v["name"] != "cert" for v in dep["spec"]["template"]["spec"].get("volumes", []))
    hooks = csv["spec"]["webhookdefinitions"]
    assert {h["type"] for h in hooks} == {"MutatingAdmissionWebhook", "ValidatingAdmissionWebhook"}
    assert all(h["rules"][0]["resources"] == ["networkclusterpolicies"] for h in hooks)  # plural (fix)
    examples = json.loads(csv["metadata"]["annotations"]["alm-examples"])
    assert {e["spec"]["configurationType"] for e in examples} == {"amd-so", "host-nic"}
    ann = b["metadata"]["annotations.yaml"]["annotations"]
    assert ann["operators.operatorframework.io.bundle.package.v1"] == "amd-network-operator"
    files = packaging.write_bundle(tmp_path / "bundle")
    assert (tmp_path / "bundle.Dockerfile").read_text().startswith("FROM scratch")
    assert len(files) == 5


def test_helm_package_archive(tmp_path):
    import tarfile

    from network_operator_amd import packaging

    out = packaging.helm_package(tmp_path)
    assert out.name == "amd-network-operator-0.1.0.tgz"
    with tarfile.open(out) as t:
        names = t.getnames()
    assert "amd-network-operator/Chart.yaml" in names and "amd-network-operator/templates/policies.yaml" in names
    again = packaging.helm_package(tmp_path / "again")
    assert again.read_bytes() == out.read_bytes()  # deterministic


def test_ci_workflows_parse_and_cover_reference_jobs():
    wf = Path(__file__).resolve().parent.parent / ".github" / "workflows"
    docs = {p.name: yaml.safe_load(p.read_text()) for p in wf.glob("*.y*ml")}
    assert {"ci.yaml", "codeql.yml", "scorecard.yml", "helm-publish.yaml"} <= set(docs)
    ci = docs["ci.yaml"]["jobs"]
    assert {"build-test", "netns", "trivy"} <= set(ci)
    steps = " ".join(str(s.get("run", "")) for s in ci["build-test"]["steps"])
    for target in ("sanitize", "vet", "build-installer", "bundle", "helm-package-chart"):
        assert target in steps, target


def test_helm_host_nic_policy():
    docs = helm_template(ROOT / "charts" / "network-operator",
                         {"config": {"hostNic": {"enabled": True, "mode": "L3", "driverImage": "r/kmd:1"}}})
    hn = _chart_policies(docs)
    assert len(hn) == 1 and hn[0]["spec"]["configurationType"] == "host-nic"
    assert hn[0]["spec"]["hostNic"]["layer"] == "L3" and hn[0]["spec"]["hostNic"]["driverImage"] == "r/kmd:1"
    from network_operator_amd.api.v1alpha1 import crd as CRD_

    assert CRD_.validate(hn[0]) == []
    with pytest.raises(RenderError):
        helm_template(ROOT / "charts" / "network-operator", {"config": {"hostNic": {"enabled": True, "mode": "L4"}}})


def test_validation_job_manifest():
    job = yaml.safe_load((ROOT / "config" / "validation" / "validation-job.yaml").read_text())
    c = job["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 8
    assert c["command"][:3] == ["python3", "-m", "network_operator_amd.validate"]
    assert job["spec"]["template"]["spec"]["nodeSelector"] == {"amd.feature.node.kubernetes.io/gpu-scale-out": "true"}


def test_project_metadata_matches_crd():
    """PROJECT (kubebuilder-style layout metadata) names the same API as the generated CRD."""
    proj = yaml.safe_load((ROOT / "PROJECT").read_text())
    crd = CRD.crd_manifest()
    (res,) = proj["resources"]
    assert res["group"] == crd["spec"]["group"] == proj["domain"]
    assert res["kind"] == crd["spec"]["names"]["kind"]
    assert res["plural"] == crd["spec"]["names"]["plural"]
    assert res["scope"] == crd["spec"]["scope"]
    assert [v["name"] for v in crd["spec"]["versions"]] == [res["version"]]


def test_trivy_ignores_reference_rendered_files():
    """Every path the Trivy ignore file names exists (rendered by `make deployments` or in-tree),
    and the renderer for the agent DaemonSet produces the objects those entries are about."""
    from network_operator_amd.testing.render import discovery_for

    ign = yaml.safe_load((ROOT / ".trivyignore.yaml").read_text())
    paths = {p for m in ign["misconfigurations"] for p in m.get("paths", [])}
    rendered = {"deployments/operator.yaml", "deployments/helm-default.yaml", "deployments/discovery.yaml",
                "deployments/discovery-host-nic.yaml"}
    assert paths - rendered == {"build/Dockerfile.linkdiscovery", "build/Dockerfile.rdma-driver"}
    assert all((ROOT / p).exists() for p in paths - rendered)
    docs = discovery_for(ROOT / "config/operator/samples/amd-l3.yaml")
    ds = _by_kind(docs, "DaemonSet")[0]
    pod = ds["spec"]["template"]["spec"]
    assert pod["hostNetwork"] is True
    caps = pod["containers"][0]["securityContext"]["capabilities"]
    assert sorted(caps["add"]) == ["NET_ADMIN", "NET_RAW"] and caps["drop"] == ["ALL"]
    hn = _by_kind(discovery_for(ROOT / "config/operator/samples/amd-host-nic.yaml"), "DaemonSet")[0]
    assert hn["spec"]["template"]["spec"]["containers"][0]["args"]


# The developer-facing targets of the reference Makefile (Makefile:100-351), under the same names.
# Tool-download targets (controller-gen, kustomize, envtest, golangci-lint, operator-sdk, opm) have
# no counterpart: the manifests are generated by Python and the renderers are in-tree.
REFERENCE_MAKE_TARGETS = ("manifests", "generate", "fmt", "vet", "test", "test-e2e", "lint", "lint-fix", "fuzz",
                          "deployments", "build", "run", "operator-image", "operator-push", "discover-image",
                          "docker-buildx", "build-installer", "install", "uninstall", "bundle", "bundle-build",
                          "bundle-push", "catalog-build", "catalog-push", "helm-update-dependencies",
                          "helm-package-chart", "helm-push-chart")


def test_makefile_has_the_reference_targets():
    """Every reference target exists and expands (make -n: nothing runs)."""
    import shutil
    import subprocess

    if not shutil.which("make"):
        pytest.skip("make not installed")
    for t in REFERENCE_MAKE_TARGETS:
        r = subprocess.run(["make", "-n", "-C", str(ROOT), t], capture_output=True, text=True)
        assert r.returncode == 0, f"make -n {t}: {r.stderr}"
        assert r.stdout.strip(), t


def test_validation_direct_check_without_pytorch(monkeypatch):
    """The validation image has no PyTorch: check 5 runs the native harness instead of failing."""
    from network_operator_amd import validate as V
    from network_operator_amd.parallel import xgmi_allreduce as XA

    calls = []

    def fake_run(**kw):
        calls.append(kw)
        return [{"mode": "pull", "bytes": 1 << 20, "time_us": 10.0, "busbw_GBps": 150.0, "wrong": 0},
                {"mode": "push", "bytes": 1 << 30, "time_us": 9000.0, "busbw_GBps": 260.0, "wrong": 0}]

    monkeypatch.setattr(V, "_have_torch", lambda: False)
    monkeypatch.setattr(XA, "run", fake_run)
    c = V.direct_all_reduce_check(8, 1 << 30, 300)
    assert c["ok"] and c["peak_busbw_GBps"] == 260.0 and "no PyTorch" in c["runner"]
    assert calls[0]["ranks"] == 8 and calls[0]["max_bytes"] == 1 << 30 and calls[0]["timeout"] == 300
    monkeypatch.setattr(XA, "run", lambda **kw: [dict(fake_run(**kw)[0], wrong=5)])
    c = V.direct_all_reduce_check(8, 1 << 30, 300)
    assert not c["ok"] and c["wrong"] == 5
    monkeypatch.setattr(XA, "run", lambda **kw: [])
    assert not V.direct_all_reduce_check(8, 1 << 30, 300)["ok"]


def test_validation_image_file_set_runs_without_pytorch(tmp_path):
    """build/Dockerfile.validation copies the whole package onto a ROCm image without PyTorch or
    any other third-party Python package: the entrypoint and every module a validation run
    imports must load with those unimportable."""
    import subprocess
    import sys

    df = (ROOT / "build" / "Dockerfile.validation").read_text()
    final = df.rsplit("\nFROM ", 1)[1]
    assert "pytorch" not in final.splitlines()[0].lower()
    assert 'ENTRYPOINT ["python3", "-m", "network_operator_amd.validate"]' in final
    block = ("import sys, runpy\n"
             "for m in ('torch', 'numpy', 'yaml', 'aiohttp', 'prometheus_client'): sys.modules[m] = None\n"
             "import network_operator_amd.models.topology, network_operator_amd.ops.smi, network_operator_amd.ops.hip\n"
             "import network_operator_amd.parallel.rccl_bench, network_operator_amd.parallel.xgmi_allreduce\n"
             "sys.argv = ['validate', '--help']\n"
             "runpy.run_module('network_operator_amd.validate', run_name='__main__')")
    r = subprocess.run([sys.executable, "-c", block], cwd=str(tmp_path), env={"PYTHONPATH": str(ROOT), "PATH": "/usr/bin:/bin"},
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and "--tune-rccl" in r.stdout, r.stderr[-2000:]


def test_validation_rccl_sweep_sources_the_agents_artifacts(monkeypatch, tmp_path):
    """validate.py check 3 runs RCCL the way jobs on the node do: with <artifact-dir>/rccl.env
    (and rccl-tuned.env) in its environment, NCCL_TOPO_FILE included, and reads RCCL's dump of that
    run back (rccl_xgmi_links).  RCCL is faked here: it writes a dump with the given xGMI links."""
    from network_operator_amd import validate as V
    from network_operator_amd.parallel import rccl_bench

    art = tmp_path / "scale-out"
    art.mkdir()
    topo = '<system version="2"><cpu numaid="0"><pci busid="0000:01:00.0"><pci busid="0000:0a:00.0"/></pci>' \
           '<pci busid="0000:1c:00.0"><pci busid="0000:23:00.0"/></pci></cpu></system>'
    (art / "rccl-topo.xml").write_text(topo)
    (art / "rccl.env").write_text(f"NCCL_TOPO_FILE={art}/rccl-topo.xml\n")
    (art / "rccl-tuned.env").write_text("NCCL_MIN_NCHANNELS=64\n")
    seen = []

    def dump(links):  # links: True (to the peer), False (none), "elsewhere" (only to a GPU outside the job)
        def g(b, p, t):
            x = {True: f'<xgmi target="{t}" count="1"/>', False: "",
                 "elsewhere": '<xgmi target="0000:99:00.0" count="1"/>'}[links]
            return f'<pci busid="{p}"><pci busid="{b}"><gpu dev="0" rank="0">{x}</gpu></pci></pci>'

        return (f'<system version="2"><cpu numaid="0">{g("0000:0a:00.0", "0000:01:00.0", "0000:23:00.0")}'
                f'{g("0000:23:00.0", "0000:1c:00.0", "0000:0a:00.0")}</cpu></system>')

    def fake_run(timeout=300, env=None, **kw):
        seen.append(dict(env))
        with open(env["NCCL_TOPO_DUMP_FILE"], "w") as f:
            f.write(dump(links=True))
        return [rccl_bench.Row("all_reduce", 1 << 30, 1 << 29, 2, 5000.0, 200.0, 200.0, 0, True, False, False)]

    monkeypatch.setattr(rccl_bench, "run", fake_run)
    monkeypatch.setattr(V, "direct_all_reduce_check", lambda *a, **k: V._check("xgmi_direct_all_reduce", True))
    monkeypatch.setattr(V.subprocess, "run", lambda *a, **k: (_ for _ in ()).throw(FileNotFoundError("no probe")))
    rep = V.run(gpus=2, min_busbw=0, min_link_GBps=0, max_bytes=1 << 30, sysfs_root=str(tmp_path / "nosys") + "/",
                artifact_dir=str(art))
    by = {c["check"]: c for c in rep["checks"]}
    assert seen[0]["NCCL_TOPO_FILE"] == f"{art}/rccl-topo.xml" and seen[0]["NCCL_MIN_NCHANNELS"] == "64"
    assert by["rccl_all_reduce"]["ok"] and by["rccl_all_reduce"]["artifacts_applied"]
    assert by["rccl_xgmi_links"]["ok"] and by["rccl_xgmi_links"]["status"] == "ok"
    assert by["rccl_xgmi_links"]["rccl_dump"]["gpu_ancestry_equal"] is True

    # RCCL under the file sees no peer of the job: the check fails.  No <xgmi> element at all, and
    # no defaults run to compare with: reported as unverifiable, not failed.
    def run_with(links):
        def run(timeout=300, env=None, **kw):
            with open(env["NCCL_TOPO_DUMP_FILE"], "w") as f:
                f.write(dump(links=links))
            return [rccl_bench.Row("all_reduce", 1 << 30, 1 << 29, 2, 5000.0, 200.0, 200.0, 0, True, False, False)]
        return run

    monkeypatch.setattr(rccl_bench, "run", run_with(False))
    rep = V.run(gpus=2, min_busbw=0, min_link_GBps=0, max_bytes=1 << 30, sysfs_root=str(tmp_path / "nosys") + "/",
                artifact_dir=str(art))
    c = {x["check"]: x for x in rep["checks"]}["rccl_xgmi_links"]
    assert c["ok"] and c["status"] == "unverifiable"
    monkeypatch.setattr(rccl_bench, "run", run_with("elsewhere"))
    rep = V.run(gpus=2, min_busbw=0, min_link_GBps=0, max_bytes=1 << 30, sysfs_root=str(tmp_path / "nosys") + "/",
                artifact_dir=str(art))
    by = {c["check"]: c for c in rep["checks"]}
    assert not by["rccl_xgmi_links"]["ok"] and by["rccl_xgmi_links"]["status"] == "failed" and not rep["ok"]


def test_helm_rail_switch_pattern_renders_quoted():
    docs = helm_template(CHART, {"config": {"amd": {"enabled": True, "railSwitchPattern": "leaf-r{rail}-.*"}}})
    cr = _chart_policies(docs)[0]
    assert cr["spec"]["amdScaleOut"]["railSwitchPattern"] == "leaf-r{rail}-.*" and CRD.validate(cr) == []


def test_helm_max_unavailable_renders():
    docs = helm_template(CHART, {"config": {"amd": {"enabled": True, "maxUnavailable": "10%"}}})
    cr = _chart_policies(docs)[0]
    assert cr["spec"]["maxUnavailable"] == "10%" and CRD.validate(cr) == []
    assert "maxUnavailable" not in _chart_policies(helm_template(CHART, {"config": {"amd": {"enabled": True}}}))[0]["spec"]


def test_rendered_deployments_are_up_to_date():
    """deployments/ is what `make deployments` renders (kustomize, the chart, the agent
    DaemonSets of the samples); a CRD or template change must be re-rendered."""
    import subprocess
    import sys

    from network_operator_amd.testing.render import dump_all

    want = {
        "operator.yaml": dump_all(kustomize_build(ROOT / "config/operator/default")),
        "helm-default.yaml": dump_all(helm_template(CHART, {"config": {"amd": {"enabled": True}}}, "amd-network-operator")),
    }
    for name, sample in (("discovery.yaml", "amd-l3.yaml"), ("discovery-host-nic.yaml", "amd-host-nic.yaml")):
        want[name] = subprocess.run([sys.executable, "-m", "network_operator_amd.testing.render", "--discovery",
                                     str(ROOT / "config/operator/samples" / sample)], capture_output=True, text=True,
                                    check=True, cwd=ROOT).stdout
    stale = [n for n, text in want.items() if (ROOT / "deployments" / n).read_text() != text]
    assert not stale, f"run `make deployments`: {stale}"


def test_prometheus_overlay_scrapes_the_operator_and_the_agents():
    docs = kustomize_build(ROOT / "config/operator/prometheus")
    kinds = sorted(d["kind"] for d in docs)
    assert kinds == ["ConfigMap", "PodMonitor", "PrometheusRule", "ServiceMonitor"]  # (the ConfigMap: the dashboard)
    pm = next(d for d in docs if d["kind"] == "PodMonitor")
    assert pm["spec"]["selector"]["matchLabels"] == {"app": "amd-network-tools"}
    assert pm["spec"]["podMetricsEndpoints"][0]["port"] == "metrics"  # the container port metricsPort opens


def test_alert_rules_use_only_metrics_that_exist():
    """Every metric an alert of config/operator/prometheus/alert-rules.yaml reads is exported: the
    operator's from its registry, the agents' from the agent's /metrics writer (agent_status.cpp); each
    alert has a severity and a summary."""
    import re

    import yaml

    from network_operator_amd.operator.metrics import OperatorMetrics

    doc = yaml.safe_load((ROOT / "config/operator/prometheus/alert-rules.yaml").read_text())
    assert doc["kind"] == "PrometheusRule"
    operator_names = set()
    for fam in OperatorMetrics().registry.collect():
        operator_names.add(fam.name + ("_total" if fam.type == "counter" else ""))
        operator_names.update(s.name for s in fam.samples)
    agent_src = (ROOT / "native/src/agent_status.cpp").read_text()
    rules = [r for g in doc["spec"]["groups"] for r in g["rules"]]
    assert len(rules) >= 6
    for r in rules:
        assert r["labels"]["severity"] in ("warning", "critical") and r["annotations"]["summary"]
        for name in re.findall(r"\b((?:amd_network_operator|netop_agent)_[a-z_]+)", r["expr"]):
            if name.startswith("netop_agent_"):
                assert f'metric("{name}"' in agent_src, (r["alert"], name)
            else:
                assert name in operator_names, (r["alert"], name)
    kust = yaml.safe_load((ROOT / "config/operator/prometheus/kustomization.yaml").read_text())
    assert "alert-rules.yaml" in kust["resources"]


def test_grafana_dashboard_reads_only_metrics_that_exist():
    """The dashboard ConfigMap (config/operator/prometheus/dashboard.yaml, and the chart's with
    monitoring.enabled): valid Grafana JSON whose every panel queries exported series, labelled
    for the Grafana sidecar."""
    import re

    from network_operator_amd.operator.metrics import OperatorMetrics

    cm = yaml.safe_load((ROOT / "config/operator/prometheus/dashboard.yaml").read_text())
    assert cm["kind"] == "ConfigMap" and cm["metadata"]["labels"]["grafana_dashboard"] == "1"
    dash = json.loads(cm["data"]["amd-network-operator.json"])
    assert dash["uid"] == "amd-network-operator"
    operator_names = set()
    for fam in OperatorMetrics().registry.collect():
        operator_names.add(fam.name + ("_total" if fam.type == "counter" else ""))
        if fam.type == "histogram":  # (labelled: no samples before the first observation)
            operator_names.update(fam.name + x for x in ("_bucket", "_sum", "_count"))
        operator_names.update(s.name for s in fam.samples)
    agent_src = (ROOT / "native/src/agent_status.cpp").read_text()
    panels = [p for p in dash["panels"] if p["type"] == "timeseries"]
    assert len(panels) >= 12 and len({p["id"] for p in dash["panels"]}) == len(dash["panels"])
    for p in panels:
        for name in re.findall(r"\b((?:amd_network_operator|netop_agent)_[a-z_]+)", p["targets"][0]["expr"]):
            if name.startswith("netop_agent_"):
                assert f'metric("{name}"' in agent_src, (p["title"], name)
            else:
                assert name in operator_names, (p["title"], name)
    kust = yaml.safe_load((ROOT / "config/operator/prometheus/kustomization.yaml").read_text())
    assert "dashboard.yaml" in kust["resources"]


def test_ci_builds_and_scans_every_image():
    """the reference CI builds its operator and agent images and runs Trivy on them
    (reference .github/workflows/validate-common.yaml:49-65).  The images job builds the operator,
    link-discovery, validation and RDMA-driver images (their in-build gates run there) and scans
    each; every Dockerfile in build/ is in the matrix."""
    ci = yaml.safe_load((ROOT / ".github" / "workflows" / "ci.yaml").read_text())["jobs"]["images"]
    images = ci["strategy"]["matrix"]["image"]
    assert sorted(images) == ["linkdiscovery", "operator", "rdma-driver", "validation"]
    assert sorted(images) == sorted(p.name.split(".", 1)[1] for p in (ROOT / "build").glob("Dockerfile.*"))
    for img in images:
        assert (ROOT / "build" / f"Dockerfile.{img}").exists(), img
    build = [s for s in ci["steps"] if str(s.get("uses", "")).startswith("docker/build-push-action")]
    scan = [s for s in ci["steps"] if str(s.get("uses", "")).startswith("aquasecurity/trivy-action")]
    assert len(build) == 1 and build[0]["with"]["file"] == "build/Dockerfile.${{ matrix.image }}"
    assert build[0]["with"]["load"] is True and build[0]["with"]["push"] is False
    assert len(scan) == 1 and scan[0]["with"]["scan-type"] == "image"
    assert scan[0]["with"]["image-ref"] == build[0]["with"]["tags"]
    assert scan[0]["with"]["exit-code"] == "1" and scan[0]["with"]["severity"] == "HIGH,CRITICAL"


def test_operator_image_dependencies_are_pinned_exactly():
    """the operator image installs from a file of exact pins (no floating
    ``==N.*``), with --no-deps, so two builds of one tag are the same; the pins cover every
    module the operator imports and match the versions this suite runs with."""
    import importlib.metadata as md
    import re as _re

    dockerfiles = {p.name: p.read_text() for p in (ROOT / "build").glob("Dockerfile.*")}
    for name, text in dockerfiles.items():
        assert not _re.search(r"==\d+\.\*", text), name
    op = dockerfiles["Dockerfile.operator"]
    assert "COPY build/requirements-operator.txt" in op and "--no-deps" in op and "-r /tmp/requirements.txt" in op
    pins = {}
    for line in (ROOT / "build" / "requirements-operator.txt").read_text().splitlines():
        line = line.split("#", 1)[0].strip()
        if line:
            name, _, ver = line.partition("==")
            assert ver and _re.fullmatch(r"[0-9][0-9A-Za-z.]*", ver), line
            pins[name.lower().replace("_", "-")] = ver
    assert {"aiohttp", "pyyaml", "prometheus-client"} <= set(pins)
    for req in md.requires("aiohttp") or []:  # aiohttp's own unconditional dependencies are pinned too
        if "extra ==" in req or "python_version" in req:
            continue
        dep = _re.split(r"[<>=!~; \[]", req, 1)[0].lower().replace("_", "-")
        assert dep in pins, dep
    for name, ver in pins.items():
        assert md.version(name) == ver, (name, md.version(name), ver)


def test_rdma_driver_container_loads_the_rdma_driver_of_each_bound_nic_driver(tmp_path):
    """build/Dockerfile.rdma-driver's entrypoint (the driverImage init container): the RDMA
    module of every RoCE NIC driver bound on the node, each once, none already loaded; arguments
    override; a module modprobe cannot load fails the container naming it."""
    import os
    import subprocess

    script = ROOT / "build" / "rdma-driver" / "load-rdma-modules.sh"
    sysfs = tmp_path / "sys"
    drivers = sysfs / "bus" / "pci" / "drivers"
    for nic, drv in (("enp8s0np0", "ionic"), ("enp33s0np0", "ionic"), ("ens1np0", "mlx5_core"), ("eno1", "igb")):
        (drivers / drv).mkdir(parents=True, exist_ok=True)
        dev = sysfs / "devices" / nic
        dev.mkdir(parents=True)
        (dev / "driver").symlink_to(drivers / drv)
        (sysfs / "class" / "net" / nic).mkdir(parents=True)
        (sysfs / "class" / "net" / nic / "device").symlink_to(dev)
    (sysfs / "module" / "mlx5_ib").mkdir(parents=True)  # already loaded
    bin_dir = tmp_path / "bin"
    bin_dir.mkdir()
    log = tmp_path / "modprobe.log"
    (bin_dir / "modprobe").write_text(f'#!/bin/sh\necho "$@" >> {log}\n[ "$1" != broken_rdma ]\n')
    (bin_dir / "modprobe").chmod(0o755)
    env = dict(os.environ, SYSFS_ROOT=str(sysfs), PATH=f"{bin_dir}:{os.environ['PATH']}")
    r = subprocess.run(["sh", str(script)], capture_output=True, text=True, env=env, timeout=30)
    assert r.returncode == 0, r.stderr
    assert log.read_text() == "ionic_rdma\n"  # once for both ionic NICs; mlx5_ib is there; igb is no RoCE NIC
    assert "ionic_rdma: loaded" in r.stdout and "mlx5_ib: already loaded" in r.stdout
    r = subprocess.run(["sh", str(script), "broken_rdma"], capture_output=True, text=True, env=env, timeout=30)
    assert r.returncode == 1 and "broken_rdma: modprobe failed" in r.stderr
    dockerfile = (ROOT / "build" / "Dockerfile.rdma-driver").read_text()
    assert "load-rdma-modules.sh /usr/local/bin/load-rdma-modules" in dockerfile and "kmod" in dockerfile
    sample = yaml.safe_load((ROOT / "config" / "operator" / "samples" / "amd-l3-pollara.yaml").read_text())
    assert sample["spec"]["amdScaleOut"]["driverImage"] == "amd/amd-network-rdma-driver:0.1.0"
