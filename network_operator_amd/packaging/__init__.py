"""Release packaging, offline: single-file installer, OLM bundle, Helm chart archive.

Reference counterparts (Makefile): ``build-installer`` (kustomize build > dist/install.yaml),
``bundle`` (operator-sdk generate kustomize manifests + generate bundle, :281-286),
``helm-package-chart`` (:341-346).  The reference shells out to kustomize / operator-sdk /
helm, which are downloaded at build time; here the same artefacts are produced by the in-repo
kustomize and Helm renderers (``testing/render.py``), so release packaging works in an
air-gapped build and is covered by tests.

    python -m network_operator_amd.packaging installer   [--out dist/install.yaml] [--img IMG]
    python -m network_operator_amd.packaging bundle      [--out bundle] [--version V] [--img IMG]
    python -m network_operator_amd.packaging helm        [--out .charts]
"""

from __future__ import annotations

import argparse
import copy
import io
import json
import tarfile
from pathlib import Path
from typing import List, Optional

import yaml

from ..testing.render import dump_all, kustomize_build
from ..utils.paths import REPO_ROOT

PACKAGE = "amd-network-operator"
DEFAULT_VERSION = "0.1.0"
DEFAULT_IMG = f"amd/amd-network-operator:{DEFAULT_VERSION}"
CHANNEL = "alpha"


def _set_manager_image(docs: List[dict], img: Optional[str]) -> None:
    if not img:
        return
    for d in docs:
        if d.get("kind") == "Deployment":
            for c in d["spec"]["template"]["spec"]["containers"]:
                if c.get("name") == "manager":
                    c["image"] = img


def installer(img: Optional[str] = None) -> List[dict]:
    """Everything needed to install the operator (CRD, RBAC, webhooks, cert-manager objects,
    Deployment) as one document list — ``make build-installer``."""
    docs = kustomize_build(REPO_ROOT / "config" / "operator" / "default")
    _set_manager_image(docs, img)
    return docs


def _by_kind(docs: List[dict], kind: str) -> List[dict]:
    return [d for d in docs if d.get("kind") == kind]


def _samples() -> List[dict]:
    out = []
    for f in sorted((REPO_ROOT / "config" / "operator" / "samples").glob("*.yaml")):
        if f.name == "kustomization.yaml":
            continue
        out += [d for d in yaml.safe_load_all(f.read_text()) if d]
    return out


def _webhook_definitions(docs: List[dict], deployment: str) -> List[dict]:
    """OLM ``webhookdefinitions`` from the rendered (Mutating|Validating)WebhookConfigurations."""
    out = []
    for kind, typ in (("MutatingWebhookConfiguration", "MutatingAdmissionWebhook"),
                      ("ValidatingWebhookConfiguration", "ValidatingAdmissionWebhook")):
        for cfg in _by_kind(docs, kind):
            for w in cfg.get("webhooks", []):
                svc = w.get("clientConfig", {}).get("service", {})
                out.append({
                    "type": typ, "generateName": w["name"], "deploymentName": deployment,
                    "containerPort": 443, "targetPort": 9443, "webhookPath": svc.get("path", "/"),
                    "admissionReviewVersions": w.get("admissionReviewVersions", ["v1"]),
                    "sideEffects": w.get("sideEffects", "None"), "failurePolicy": w.get("failurePolicy", "Fail"),
                    "rules": w.get("rules", []),
                })
    return out


def bundle(version: str = DEFAULT_VERSION, img: str = DEFAULT_IMG) -> dict:
    """OLM bundle: ``{"manifests": {file: doc}, "metadata": {file: doc}, "bundle.Dockerfile": str}``.

    The ClusterServiceVersion is assembled from the same kustomize output as the installer, so
    RBAC, the manager Deployment and the webhooks can never drift from the plain install.
    Cert-manager objects are dropped: OLM provisions webhook certificates itself.
    """
    docs = installer(img)
    deploy = _by_kind(docs, "Deployment")[0]
    sa = deploy["spec"]["template"]["spec"].get("serviceAccountName", "default")
    cluster_rules, ns_rules = [], []
    for rb in _by_kind(docs, "ClusterRoleBinding"):
        role = next((r for r in _by_kind(docs, "ClusterRole") if r["metadata"]["name"] == rb["roleRef"]["name"]), None)
        if role and any(s.get("name") == sa for s in rb.get("subjects", [])):
            cluster_rules += role.get("rules", [])
    for rb in _by_kind(docs, "RoleBinding"):
        role = next((r for r in _by_kind(docs, "Role") if r["metadata"]["name"] == rb["roleRef"]["name"]), None)
        if role and any(s.get("name") == sa for s in rb.get("subjects", [])):
            ns_rules += role.get("rules", [])
    crd = _by_kind(docs, "CustomResourceDefinition")[0]
    kind = crd["spec"]["names"]["kind"]
    owned = [{"name": crd["metadata"]["name"], "version": v["name"], "kind": kind, "displayName": "Network Cluster Policy",
              "description": "Scale-out network configuration of the GPU nodes selected by nodeSelector."}
             for v in crd["spec"]["versions"] if v.get("served")]
    dspec = copy.deepcopy(deploy["spec"])
    # OLM mounts the webhook certificate itself (apiservice-cert); drop the cert-manager volume.
    pod = dspec["template"]["spec"]
    pod["volumes"] = [v for v in pod.get("volumes", []) if v.get("name") != "cert"]
    for c in pod["containers"]:
        c["volumeMounts"] = [m for m in c.get("volumeMounts", []) if m.get("name") != "cert"]
        if not c["volumeMounts"]:
            c.pop("volumeMounts")
    name = f"{PACKAGE}.v{version}"
    csv = {
        "apiVersion": "operators.coreos.com/v1alpha1",
        "kind": "ClusterServiceVersion",
        "metadata": {
            "name": name,
            "namespace": "placeholder",
            "annotations": {
                "alm-examples": json.dumps(_samples(), indent=2),
                "capabilities": "Basic Install",
                "categories": "Networking",
                "containerImage": img,
                "description": "Configures the scale-out NICs of AMD Instinct MI355X nodes for RCCL",
                "operators.operatorframework.io/builder": "network_operator_amd.packaging",
            },
        },
        "spec": {
            "displayName": "AMD Network Operator",
            "description": ("Discovers the RoCE NICs next to each MI355X GPU, assigns point-to-point L3 addresses "
                            "learnt over LLDP (or brings them up in L2), verifies the xGMI mesh, writes RCCL "
                            "configuration files and labels the node scale-out ready."),
            "version": version,
            "maturity": CHANNEL,
            "minKubeVersion": "1.28.0",
            "keywords": ["networking", "rdma", "roce", "rccl", "amd", "instinct", "mi355x"],
            "provider": {"name": "AMD network operator authors"},
            "maintainers": [{"name": "AMD network operator authors", "email": "noreply@example.com"}],
            "installModes": [{"type": "OwnNamespace", "supported": False},
                             {"type": "SingleNamespace", "supported": False},
                             {"type": "MultiNamespace", "supported": False},
                             {"type": "AllNamespaces", "supported": True}],
            "customresourcedefinitions": {"owned": owned},
            "install": {
                "strategy": "deployment",
                "spec": {
                    "clusterPermissions": [{"serviceAccountName": sa, "rules": cluster_rules}],
                    "permissions": [{"serviceAccountName": sa, "rules": ns_rules}],
                    "deployments": [{"name": deploy["metadata"]["name"], "label": deploy["metadata"].get("labels", {}),
                                     "spec": dspec}],
                },
            },
            "webhookdefinitions": _webhook_definitions(docs, deploy["metadata"]["name"]),
        },
    }
    crd_out = copy.deepcopy(crd)
    crd_out["metadata"].get("annotations", {}).pop("cert-manager.io/inject-ca-from", None)
    crd_out["spec"].pop("conversion", None)
    manifests = {f"{PACKAGE}.clusterserviceversion.yaml": csv, f"{crd['metadata']['name']}.yaml": crd_out}
    for svc in _by_kind(docs, "Service"):
        if "metrics" in svc["metadata"]["name"]:
            manifests[f"{svc['metadata']['name']}_v1_service.yaml"] = svc
    annotations = {"annotations": {
        "operators.operatorframework.io.bundle.mediatype.v1": "registry+v1",
        "operators.operatorframework.io.bundle.manifests.v1": "manifests/",
        "operators.operatorframework.io.bundle.metadata.v1": "metadata/",
        "operators.operatorframework.io.bundle.package.v1": PACKAGE,
        "operators.operatorframework.io.bundle.channels.v1": CHANNEL,
        "operators.operatorframework.io.bundle.channel.default.v1": CHANNEL,
    }}
    dockerfile = "FROM scratch\n" + "".join(
        f"LABEL {k}={v}\n" for k, v in annotations["annotations"].items()) + (
        "COPY bundle/manifests /manifests/\nCOPY bundle/metadata /metadata/\n")
    return {"manifests": manifests, "metadata": {"annotations.yaml": annotations}, "bundle.Dockerfile": dockerfile}


def write_bundle(out: Path, version: str = DEFAULT_VERSION, img: str = DEFAULT_IMG) -> List[Path]:
    b = bundle(version, img)
    written = []
    for sub in ("manifests", "metadata"):
        (out / sub).mkdir(parents=True, exist_ok=True)
        for fname, doc in b[sub].items():
            p = out / sub / fname
            p.write_text(yaml.safe_dump(doc, sort_keys=False))
            written.append(p)
    p = out.parent / "bundle.Dockerfile"
    p.write_text(b["bundle.Dockerfile"])
    written.append(p)
    return written


def helm_package(out_dir: Path, chart_dir: Optional[Path] = None) -> Path:
    """``helm package``: ``<name>-<version>.tgz`` with the chart under ``<name>/``, deterministic."""
    chart_dir = Path(chart_dir or REPO_ROOT / "charts" / "network-operator")
    meta = yaml.safe_load((chart_dir / "Chart.yaml").read_text())
    name, version = meta["name"], str(meta["version"])
    out_dir.mkdir(parents=True, exist_ok=True)
    out = out_dir / f"{name}-{version}.tgz"
    import gzip

    # The gzip header carries a timestamp too ("w:gz" writes the current time): mtime 0, no name.
    with open(out, "wb") as raw, gzip.GzipFile(filename="", mode="wb", fileobj=raw, mtime=0) as gz, \
            tarfile.open(fileobj=gz, mode="w", format=tarfile.PAX_FORMAT) as tar:
        for f in sorted(p for p in chart_dir.rglob("*") if p.is_file()):
            data = f.read_bytes()
            ti = tarfile.TarInfo(f"{name}/{f.relative_to(chart_dir).as_posix()}")
            ti.size, ti.mode, ti.mtime = len(data), 0o644, 0
            tar.addfile(ti, io.BytesIO(data))
    return out


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m network_operator_amd.packaging")
    sub = ap.add_subparsers(dest="cmd", required=True)
    a = sub.add_parser("installer")
    a.add_argument("--out", default="dist/install.yaml")
    a.add_argument("--img", default=None)
    b = sub.add_parser("bundle")
    b.add_argument("--out", default="bundle")
    b.add_argument("--version", default=DEFAULT_VERSION)
    b.add_argument("--img", default=DEFAULT_IMG)
    h = sub.add_parser("helm")
    h.add_argument("--out", default=".charts")
    args = ap.parse_args(argv)
    if args.cmd == "installer":
        out = Path(args.out)
        out.parent.mkdir(parents=True, exist_ok=True)
        out.write_text(dump_all(installer(args.img)))
        print(out)
    elif args.cmd == "bundle":
        for p in write_bundle(Path(args.out), args.version, args.img):
            print(p)
    else:
        print(helm_package(Path(args.out)))
    return 0
