"""Move a cluster from the Gaudi network operator to this one: its NetworkClusterPolicy objects
and its Helm values, converted and checked against this operator's CRD schema and webhook.

Input is YAML: NetworkClusterPolicy objects of the reference, alone, as several documents or as a
``List`` (``intel.com/v1alpha1``, ``configurationType: gaudi-so``, ``spec.gaudiScaleOut``;
reference api/v1alpha1/networkconfiguration_types.go:24-68, samples config/operator/samples/),
or, with ``--values``, the reference chart's values (reference charts/network-operator/values.yaml).
The result goes to stdout.  Every field that changed meaning or was dropped is named on stderr.
The exit status is 1 when an object would not be admitted.

    python -m network_operator_amd.api.v1alpha1.migrate gaudi-l3.yaml > amd-l3.yaml
    python -m network_operator_amd.api.v1alpha1.migrate --values old-values.yaml > values.yaml

What changes (docs/USER_GUIDE.md section 7):
- ``intel.com`` becomes ``amd.com``, ``gaudi-so`` becomes ``amd-so`` and ``gaudiScaleOut`` becomes ``amdScaleOut``.
  ``disableNetworkManager``, ``layer``, ``pullPolicy``, ``mtu``, ``logLevel`` and ``nodeSelector`` carry over.
- The Gaudi agent image cannot configure MI355X nodes: an ``intel/`` or Habana image is replaced
  by this operator's agent image (``--image`` names another).
- The NFD labels the reference selects on (``intel.feature.node.kubernetes.io/gaudi-ready``,
  ``.../gaudi``) become the AMD rule's (``amd.feature.node.kubernetes.io/gpu-ready``, ``.../gpu``).
  Other selector keys are kept as they are.
- ``xgmiCheck`` and ``requireRdma`` are written out as true, this operator's defaults: the label
  also waits for the xGMI mesh and for an RDMA device on every scale-out NIC.
- Server-written metadata (uid, resourceVersion, status, managedFields, finalizers, the last-applied
  annotation) is dropped: the result is something to apply, not a copy of the old object.
"""

from __future__ import annotations

import argparse
import copy
import sys
from typing import Any, Dict, List, Optional, Tuple

import yaml

from . import crd
from . import types as T
from . import webhook

REFERENCE_GROUP = "intel.com"
REFERENCE_TYPE = "gaudi-so"
# NFD labels of the reference's rule (reference config/nfd/gaudi-device-rule.yaml) -> the AMD rule's
# (config/nfd/amd-gpu-device-rule.yaml).
LABEL_MAP = {
    "intel.feature.node.kubernetes.io/gaudi-ready": "amd.feature.node.kubernetes.io/gpu-ready",
    "intel.feature.node.kubernetes.io/gaudi": "amd.feature.node.kubernetes.io/gpu",
}
# The reference's readiness label and artifact, for the notes about their consumers.
REFERENCE_READY_LABEL = "intel.feature.node.kubernetes.io/gaudi-scale-out"
READY_LABEL = "amd.feature.node.kubernetes.io/gpu-scale-out"
CARRIED_SO_FIELDS = ("disableNetworkManager", "layer", "pullPolicy", "mtu")
SERVER_METADATA = ("uid", "resourceVersion", "generation", "creationTimestamp", "deletionTimestamp",
                   "deletionGracePeriodSeconds", "managedFields", "finalizers", "ownerReferences", "selfLink")
LAST_APPLIED = "kubectl.kubernetes.io/last-applied-configuration"


class MigrationError(ValueError):
    pass


def _gaudi_image(image: str) -> bool:
    repo = image.split("@")[0]
    if ":" in repo.rsplit("/", 1)[-1]:  # a tag, not a registry port
        repo = repo[:repo.rfind(":")]
    return repo.startswith(("intel/", "docker.io/intel/")) or "habana" in repo or "gaudi" in repo


def _selector(sel: Dict[str, Any], where: str, notes: List[str]) -> Dict[str, Any]:
    out = {}
    for k, v in (sel or {}).items():
        if k in LABEL_MAP:
            out[LABEL_MAP[k]] = v
            notes.append(f"{where}: nodeSelector {k} -> {LABEL_MAP[k]}")
        else:
            out[k] = v
            if k.startswith("intel.feature.node.kubernetes.io/"):
                notes.append(f"{where}: nodeSelector {k} kept as is: no AMD counterpart, check that your nodes carry it")
    return out


def convert_policy(obj: dict, image: Optional[str] = None) -> Tuple[dict, List[str]]:
    """One reference NetworkClusterPolicy -> (this operator's policy as a dict, notes)."""
    if not isinstance(obj, dict) or obj.get("kind") != T.KIND:
        raise MigrationError(f"not a {T.KIND}: kind {obj.get('kind') if isinstance(obj, dict) else type(obj).__name__!r}")
    meta = obj.get("metadata") or {}
    name = meta.get("name") or "<unnamed>"
    where = f"{T.KIND} {name}"
    group = str(obj.get("apiVersion", "")).split("/")[0]
    if group == T.GROUP:
        return copy.deepcopy(obj), [f"{where}: already {T.API_VERSION}, unchanged"]
    if group != REFERENCE_GROUP:
        raise MigrationError(f"{where}: apiVersion {obj.get('apiVersion')!r} is neither {REFERENCE_GROUP} nor {T.GROUP}")
    notes: List[str] = []
    spec = dict(obj.get("spec") or {})
    ctype = spec.pop("configurationType", None)
    if ctype != REFERENCE_TYPE:
        raise MigrationError(f"{where}: configurationType {ctype!r}: only {REFERENCE_TYPE!r} has a counterpart ({T.CONFIG_AMD_SCALE_OUT})")
    gso = dict(spec.pop("gaudiScaleOut", None) or {})
    so: Dict[str, Any] = {k: gso.pop(k) for k in CARRIED_SO_FIELDS if k in gso}
    old_image = gso.pop("image", "")
    if image:
        so["image"] = image
        notes.append(f"{where}: image {old_image or '(default)'} -> {image}")
    elif old_image and not _gaudi_image(old_image):
        so["image"] = old_image
        notes.append(f"{where}: image {old_image} kept: make sure it is this operator's agent, not the Gaudi one")
    elif old_image:
        notes.append(f"{where}: image {old_image} is the Gaudi agent -> {T.DEFAULT_AGENT_IMAGE} (the webhook's default)")
    for k in sorted(gso):
        notes.append(f"{where}: gaudiScaleOut.{k} has no counterpart and was dropped")
    # Written out, so the converted object says what it does: the MI355X defaults (the CRD's and
    # the webhook's).  requireRdma keeps the reference's meaning of the label -- its NICs are RDMA
    # NICs by construction (reference cmd/discover/network.go:34) -- on nodes whose RoCE NICs need
    # an RDMA driver loaded.
    so["xgmiCheck"] = True
    so["requireRdma"] = True
    notes.append(f"{where}: amdScaleOut.xgmiCheck and requireRdma set true (this operator's defaults): the readiness "
                 "label also waits for a complete xGMI mesh and an RDMA device on every scale-out NIC")
    new_spec: Dict[str, Any] = {"configurationType": T.CONFIG_AMD_SCALE_OUT, "amdScaleOut": so}
    if "nodeSelector" in spec:
        new_spec["nodeSelector"] = _selector(spec.pop("nodeSelector"), where, notes)
    if "logLevel" in spec:
        new_spec["logLevel"] = spec.pop("logLevel")
    for k in sorted(spec):
        notes.append(f"{where}: spec.{k} has no counterpart and was dropped")
    new_meta = {k: copy.deepcopy(v) for k, v in meta.items() if k not in SERVER_METADATA and k != "namespace"}
    ann = dict(new_meta.get("annotations") or {})
    if ann.pop(LAST_APPLIED, None) is not None:
        notes.append(f"{where}: dropped the {LAST_APPLIED} annotation (it describes the old object)")
    if ann:
        new_meta["annotations"] = ann
    else:
        new_meta.pop("annotations", None)
    out = {"apiVersion": T.API_VERSION, "kind": T.KIND, "metadata": new_meta, "spec": new_spec}
    return out, notes


def admission_errors(obj: dict) -> List[str]:
    """What the API server (CRD schema) and the validating webhook would refuse."""
    errs = crd.validate(obj)
    if errs:
        return errs
    try:
        pol = webhook.default(T.NetworkClusterPolicy.from_dict(copy.deepcopy(obj)))
        webhook.validate_create(pol)
    except webhook.ValidationError as e:
        return [getattr(e, "message", None) or str(e)]
    return []


def _documents(text: str) -> List[dict]:
    out = []
    for doc in yaml.safe_load_all(text):
        if doc is None:
            continue
        if isinstance(doc, dict) and doc.get("kind", "").endswith("List") and isinstance(doc.get("items"), list):
            out.extend(doc["items"])
        else:
            out.append(doc)
    return out


def convert_policies(text: str, image: Optional[str] = None) -> Tuple[List[dict], List[str], List[str]]:
    """(converted objects, notes, errors) for a YAML stream of policies."""
    objs, notes, errors = [], [], []
    for doc in _documents(text):
        try:
            new, n = convert_policy(doc, image)
        except MigrationError as e:
            errors.append(str(e))
            continue
        notes += n
        errors += [f"{T.KIND} {new['metadata'].get('name')}: would not be admitted: {e}" for e in admission_errors(new)]
        objs.append(new)
    if objs:
        notes.append(f"workloads selecting nodes by {REFERENCE_READY_LABEL}=true must select {READY_LABEL}=true; "
                     "jobs read /etc/amd/scale-out/rccl.env (NCCL_TOPO_FILE and the HCA list) instead of "
                     "/etc/habanalabs/gaudinet.json")
    return objs, notes, errors


def _swap_repo(img: dict, old: str, new: str, where: str, notes: List[str]) -> dict:
    img = dict(img or {})
    repo = img.get("repository", "")
    if repo.endswith(old) or _gaudi_image(repo):
        img["repository"] = new
        img.pop("tag", None)  # the Gaudi release's tag means nothing here: the chart's default
        notes.append(f"{where}.image: {repo} -> {new} (tag: the chart's)")
    return img


def convert_values(values: dict) -> Tuple[dict, List[str]]:
    """The reference chart's values -> this chart's (only what the reference chart has; every
    MI355X option keeps this chart's default)."""
    notes: List[str] = []
    out: Dict[str, Any] = {}
    v = copy.deepcopy(values or {})
    if "logLevel" in v:
        out["logLevel"] = v.pop("logLevel")
    op = v.pop("operator", None)
    if op is not None:
        o = dict(op)
        if "image" in o:
            o["image"] = _swap_repo(o["image"], "intel-network-operator", "amd/amd-network-operator", "operator", notes)
            if not o["image"]:
                del o["image"]
        out["operator"] = o
    nfd = v.pop("nfd", None)
    if nfd is not None:
        n = dict(nfd)
        if "gaudiRule" in n:
            n["amdGpuRule"] = n.pop("gaudiRule")
            notes.append("nfd.gaudiRule -> nfd.amdGpuRule")
        out["nfd"] = n
    cfg = dict(v.pop("config", None) or {})
    g = cfg.pop("gaudi", None)
    if g is not None:
        a = dict(g)
        if "image" in a:
            a["image"] = _swap_repo(a["image"], "intel-network-linkdiscovery", "amd/amd-network-linkdiscovery",
                                    "config.amd", notes)
        if "nodeSelector" in a:
            a["nodeSelector"] = _selector(a["nodeSelector"], "config.amd", notes)
        out["config"] = {"amd": a}
        notes.append("config.gaudi -> config.amd (an amd-so policy; see the chart's README for the MI355X options)")
    for k in sorted(cfg):
        out.setdefault("config", {})[k] = cfg[k]
    for k in sorted(v):
        notes.append(f"{k}: not a value of the reference chart; kept as is")
        out[k] = v[k]
    return out, notes


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m network_operator_amd.api.v1alpha1.migrate",
                                 description=__doc__.split("\n\n")[0])
    ap.add_argument("file", nargs="?", default="-", help="YAML file; - or nothing = stdin")
    ap.add_argument("--values", action="store_true", help="the input is the reference chart's values.yaml")
    ap.add_argument("--image", default=None, help="agent image for the converted policies")
    a = ap.parse_args(argv)
    text = sys.stdin.read() if a.file == "-" else open(a.file, encoding="utf-8").read()
    if a.values:
        out, notes = convert_values(yaml.safe_load(text) or {})
        sys.stdout.write(yaml.safe_dump(out, sort_keys=False))
        errors: List[str] = []
    else:
        objs, notes, errors = convert_policies(text, a.image)
        sys.stdout.write(yaml.safe_dump_all(objs, sort_keys=False, explicit_start=True) if objs else "")
    for n in notes:
        print(f"note: {n}", file=sys.stderr)
    for e in errors:
        print(f"error: {e}", file=sys.stderr)
    return 1 if errors else 0


if __name__ == "__main__":
    sys.exit(main())
