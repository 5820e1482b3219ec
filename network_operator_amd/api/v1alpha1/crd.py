"""CRD manifest for ``networkclusterpolicies.amd.com`` and a structural-schema validator.

The schema is the single source of truth: ``python -m network_operator_amd.api.v1alpha1.crd``
regenerates ``config/operator/crd/bases/amd.com_networkclusterpolicies.yaml`` and the Helm
chart copy (both are checked for drift by the test-suite, the job controller-gen does for
the reference: reference config/operator/crd/bases/intel.com_networkclusterpolicies.yaml).

``validate(obj)`` applies the same OpenAPI v3 rules the API server enforces (types, enums,
minimum/maximum, required, additionalProperties) — the fake API server uses it so tests see
the same 422 Invalid answers a real cluster would give.
"""

from __future__ import annotations

import re

import sys
from pathlib import Path
from typing import Any, List

import yaml

from . import types as T

LLDP_WAIT_SCHEMA = {
    "description": "L3: how long the agent waits for every NIC's first LLDPDU (a Go duration, 1s..30m;\n"
                   "default 90s, the reference's fixed value).  Shorter with fast-start switches, so a\n"
                   "silent NIC is diagnosed sooner; longer for switches with a long transmit interval.",
    "pattern": T.LLDP_WAIT_PATTERN, "type": "string"}
CARRIER_WAIT_SCHEMA = {
    "description": "L2: how long each NIC may take to get a carrier after it is set up (a Go duration,\n"
                   "1s..10m; default 30s).  200/400G optics commonly train for 5-15 s; meanwhile the\n"
                   "node reports \"waiting for carrier\" (start-up, not Degraded), afterwards \"no carrier\".",
    "pattern": T.LLDP_WAIT_PATTERN, "type": "string"}

_API_VERSION_DESC = (
    "APIVersion defines the versioned schema of this representation of an object.\n"
    "Servers should convert recognized schemas to the latest internal value, and\n"
    "may reject unrecognized values.\n"
    "More info: https://git.k8s.io/community/contributors/devel/sig-architecture/api-conventions.md#resources")
_KIND_DESC = (
    "Kind is a string value representing the REST resource this object represents.\n"
    "Servers may infer this from the endpoint the client submits requests to.\n"
    "Cannot be updated.\n"
    "In CamelCase.\n"
    "More info: https://git.k8s.io/community/contributors/devel/sig-architecture/api-conventions.md#types-kinds")


def openapi_schema() -> dict:
    amd_so = {
        "description": "AMD MI355X scale-out specific settings. Only valid when configuration type is 'amd-so'",
        "default": {},
        "type": "object",
        "properties": {
            "disableNetworkManager": {
                "description": "Take the scale-out interfaces away from NetworkManager on nodes where it would\n"
                               "otherwise try to configure them.",
                "type": "boolean"},
            "image": {"description": "Container image of the link-discovery agent on the worker nodes.", "type": "string"},
            "layer": {"description": "Layer where the configuration should occur. Possible options: L2 and L3.",
                      "enum": list(T.LAYERS), "type": "string"},
            "mtu": {"description": "MTU for the scale-out interfaces.", "maximum": T.MTU_MAX, "minimum": T.MTU_MIN,
                    "type": "integer"},
            "pullPolicy": {"description": "Image pull policy used in the resulting daemonset.",
                           "enum": list(T.PULL_POLICIES), "type": "string"},
            "xgmiCheck": {"description": "Publish the readiness label only when the node's xGMI mesh is complete\n"
                                         "(every GPU pair linked, read from the KFD topology) and every link is up\n"
                                         "(amdgpu gpu_metrics).  Default true; false for nodes without an xGMI mesh.",
                          "default": True, "type": "boolean"},
            "requireRdma": {"description": "Scale-out ready means RDMA ready: publish the readiness label (and write\n"
                                           "rccl.env) only once every scale-out NIC has an RDMA device, i.e. its RDMA\n"
                                           "driver (ionic_rdma, mlx5_ib, bnxt_re) is loaded.  Meanwhile the NICs are\n"
                                           "configured and the node reports \"waiting for RDMA device\"; it is labelled\n"
                                           "as soon as the devices appear.  Default true; false labels nodes whose rails\n"
                                           "RCCL could use only over TCP sockets.",
                            "default": True, "type": "boolean"},
            "rdmaWait": {"description": "With requireRdma: how long a missing RDMA device counts as start-up (a Go\n"
                                        "duration, 1s..1h; default 5m).  Afterwards the node reports \"no RDMA device\n"
                                        "(load its RDMA driver)\" and the policy is Degraded.",
                         "pattern": T.LLDP_WAIT_PATTERN, "type": "string"},
            "driverImage": {"description": "Optional NIC RDMA-driver (KMD) container, run as a privileged init container\n"
                                           "before the agent with the host's /lib/modules; it must load the driver\n"
                                           "(e.g. ionic_rdma for AMD Pollara) and exit 0.",
                            "type": "string"},
            "lldpAnnounce": {"description": "Transmit an LLDPDU from every scale-out NIC so IEEE 802.1AB-2009 switches\n"
                                            "answer with fast transmission (default true).",
                             "type": "boolean"},
            "interfaces": {"description": "Additional interfaces to configure besides the GPU-affine NICs.",
                           "items": {"type": "string", "maxLength": 15}, "type": "array"},
            "nicDrivers": {"description": "NIC driver allow-list for GPU-affinity discovery (default: common RoCE drivers).",
                           "items": {"type": "string"}, "type": "array"},
            "disableFirmwareLldp": {"description": "L3: turn off NIC-firmware LLDP agents (ethtool private flags, e.g. i40e\n"
                                                   "disable-fw-lldp, ice fw-lldp-agent) while the agent runs, so switch\n"
                                                   "LLDPDUs reach the host.",
                                    "type": "boolean"},
            "handDcbxToHost": {"description": "With disableFirmwareLldp, on DCB NICs without a firmware-LLDP flag whose\n"
                                              "DCBX an embedded agent runs (mlx5_core firmware mode): hand DCBX to the\n"
                                              "host.  The firmware then stops negotiating PFC/ETS with the switch, so\n"
                                              "only for hosts that run DCBX themselves.  Restored when the agent exits.",
                               "type": "boolean"},
            "checkPeerMtu": {"description": "L3: refuse a NIC whose switch port advertises (LLDP 802.3 Maximum Frame\n"
                                            "Size) frames smaller than the NIC's own (MTU + 18, + 4 on a VLAN NIC).\n"
                                            "Default true; false for switches that misreport the TLV.",
                             "type": "boolean"},
            "gpuDirectRdma": {"description": "Require GPUDirect RDMA before labelling the node: Any, PeerMem (amdkfd\n"
                                             "peer-memory client) or DmaBuf (RDMA dma-buf MRs).  Empty: report only.",
                              "enum": ["Any", "PeerMem", "DmaBuf"], "type": "string"},
            "rcclEnv": {"description": "Site settings appended to rccl.env (e.g. NCCL_IB_TC for the fabric's RoCE\n"
                                       "traffic class).  Keys: NCCL_*, RCCL_*, HSA_*.",
                        "additionalProperties": {"type": "string"}, "type": "object"},
            "metricsPort": {"description": "Serve agent metrics (/metrics, /healthz, /readyz) on this host port (0 = off).",
                            "maximum": 65535, "minimum": 0, "type": "integer"},
            "railTableBase": {"description": "L3: per-rail source routing.  The NIC of GPU k gets routing table and rule\n"
                                             "priority railTableBase+k (its /30 and its /16 via the switch), so traffic\n"
                                             "from a rail's address leaves through that rail.  0 = off.",
                              "maximum": 200, "minimum": 0, "type": "integer"},
            "rcclSocketIfname": {"description": "NCCL_SOCKET_IFNAME written into rccl.env: auto (L3: the configured\n"
                                                "scale-out NICs in GPU order, so bootstrap meets on rail 0; L2: not set),\n"
                                                "none (not set: RCCL picks, usually the management network), or a\n"
                                                "comma-separated interface list.  Empty = auto.",
                                 "pattern": r"^(auto|none|[A-Za-z0-9_.:@-]{1,15}(,[A-Za-z0-9_.:@-]{1,15})*)$",
                                 "type": "string"},
            "validation": {"description": "Post-configuration fabric validation: once a node's agent is ready, run the\n"
                                          "validation Job there (exact all-reduce, busbw and xGMI link floors, RCCL loading\n"
                                          "the topology file) and report it in the FabricValidated condition.",
                           "type": "object",
                           "properties": {
                               "enabled": {"type": "boolean"},
                               "image": {"description": "Validation image (default amd/amd-network-validation).",
                                         "type": "string"},
                               "gpus": {"description": "GPUs to validate per node (default 8).", "minimum": 1,
                                        "maximum": 8, "type": "integer"},
                               "minBusbw": {"description": "Required 1 GiB all-reduce busbw in GB/s (0: correctness only).",
                                            "minimum": 0, "type": "integer"},
                               "minLink": {"description": "Required per-link xGMI pull bandwidth in GB/s (0: not checked).",
                                           "minimum": 0, "type": "integer"},
                           },
                           "required": ["enabled"]},
            "lldpCache": {"description": "L3: remember each NIC's last confirmed Port Description on the node, so a\n"
                                         "restarted agent configures at once instead of waiting for the switch's next\n"
                                         "periodic LLDPDU (switches without fast start).  The switch must confirm it\n"
                                         "within 95 s, else the readiness label is withdrawn until it does.",
                          "type": "boolean"},
            "verifyPeers": {"description": "L3: before labelling the node, require every NIC's switch-side /30 address\n"
                                           "to answer ARP (within 2 s).  Catches a switch port whose Port Description\n"
                                           "and interface address disagree, which LLDP alone cannot.",
                            "type": "boolean"},
            "lldpWait": LLDP_WAIT_SCHEMA,
            "carrierWait": CARRIER_WAIT_SCHEMA,
            "keepConfigOnRestart": {
                "description": "Keep addresses, routes and links when an agent exits (rolling update, drain,\n"
                               "crash), so RCCL jobs keep their RoCE connections; the next agent adopts them\n"
                               "(L3: from the LLDP cache, which this turns on).  The operator removes the\n"
                               "configuration with a cleanup Job per node when the policy is deleted or a\n"
                               "node leaves it (finalizer amd.com/node-cleanup).",
                "type": "boolean"},
            "railSwitchPattern": {
                "description": "L3 rail cabling check: the NIC of GPU k must be cabled to a switch whose LLDP System\n"
                               "Name matches this regular expression with {rail} replaced by k, e.g.\n"
                               "'leaf-r{rail}-.*' on a rail-optimized fabric.  A NIC on another rail's leaf is\n"
                               "left unconfigured and named in status.errors.",
                "maxLength": 253, "type": "string"},
            "minLinkSpeedGbps": {
                "description": "Minimum negotiated link speed of every scale-out NIC in Gb/s (e.g. 400).  A NIC that\n"
                               "came up slower (a marginal cable or optic, a port renegotiated down) is left\n"
                               "unconfigured and named in status.errors.  0 = not checked.",
                "minimum": 0, "maximum": 3200, "type": "integer"},
            "requireFullPcieLink": {
                "description": "Configure a scale-out NIC only if its PCIe link trained at the speed and width it\n"
                               "supports, and its GPU's at full width: a card in a worn slot or riser (x8, or a\n"
                               "lower generation) moves RDMA at a fraction of the rail's rate.  Such a NIC is left\n"
                               "unconfigured and named in status.errors.  Reported in the agent's status either way.",
                "type": "boolean"},
            "allowPolicyRouted": {
                "description": "Configure a selected NIC that has a default route in a per-NIC policy-routing table\n"
                               "even when it holds the node's own address (the source its rule selects, or any\n"
                               "address that is not a /30).  Such a NIC is how the node reaches a network, so by\n"
                               "default it is refused like the node's uplink.",
                "type": "boolean"},
        },
    }
    host_nic = {
        "description": "HostNic configures the node's own RDMA NICs (not paired with a GPU); used with\n"
                       "configurationType host-nic.",
        "type": "object",
        "properties": {
            "layer": {"description": "L2: links up only; L3: LLDP-driven /30 addressing.", "enum": list(T.LAYERS),
                      "type": "string"},
            "mtu": {"description": "MTU for the host NICs.", "maximum": T.MTU_MAX, "minimum": T.MTU_MIN,
                    "type": "integer"},
            "image": {"description": "Container image of the link-discovery agent.", "type": "string"},
            "pullPolicy": {"description": "Image pull policy of the agent and driver containers.",
                           "enum": list(T.PULL_POLICIES), "type": "string"},
            "disableNetworkManager": {"description": "Take the host NICs away from NetworkManager.",
                                      "type": "boolean"},
            "interfaces": {"description": "Host NICs to configure (default: every RDMA NIC of nicDrivers that is\n"
                                          "neither a GPU's scale-out rail nor the node's own NIC: default route,\n"
                                          "a non-/30 address, a route the agent does not install).",
                           "items": {"type": "string", "maxLength": 15}, "type": "array"},
            "nicDrivers": {"description": "NIC driver allow-list for RDMA NIC discovery.",
                           "items": {"type": "string"}, "type": "array"},
            "driverImage": {"description": "Optional NIC kernel-driver (KMD) container, run as a privileged init\n"
                                           "container before the agent; it must load the driver and exit 0.",
                            "type": "string"},
            "verifyPeers": {"description": "L3: label only once every NIC's switch-side /30 address answers ARP.",
                            "type": "boolean"},
            "lldpWait": LLDP_WAIT_SCHEMA,
            "carrierWait": CARRIER_WAIT_SCHEMA,
            "keepConfigOnRestart": {"description": "As amdScaleOut.keepConfigOnRestart, for the host NICs.",
                                    "type": "boolean"},
            "checkPeerMtu": {"description": "As amdScaleOut.checkPeerMtu, for the host NICs.", "type": "boolean"},
            "includeGpuRails": {"description": "Let discovery take the NICs next to the GPUs (within a PCIe switch of an\n"
                                               "amdgpu function), which an amd-so policy owns; only for nodes that run\n"
                                               "no amd-so policy.",
                                "type": "boolean"},
            "minLinkSpeedGbps": {"description": "As amdScaleOut.minLinkSpeedGbps, for the host NICs.",
                                 "minimum": 0, "maximum": 3200, "type": "integer"},
            "requireFullPcieLink": {"description": "As amdScaleOut.requireFullPcieLink, for the host NICs (their own\n"
                                                   "PCIe link; they have no GPU).",
                                    "type": "boolean"},
            "allowPolicyRouted": {"description": "As amdScaleOut.allowPolicyRouted, for the host NICs.", "type": "boolean"},
        },
        "required": ["layer"],
    }
    spec = {
        "description": "NetworkClusterPolicySpec defines the desired state of NetworkClusterPolicy",
        "type": "object",
        "properties": {
            "configurationType": {
                "description": "Configuration type that the operator will configure to the nodes. Possible options:\n"
                               "amd-so (GPU scale-out NICs), host-nic (the node's own RDMA NICs)",
                "enum": list(T.CONFIGURATION_TYPES), "type": "string"},
            "amdScaleOut": amd_so,
            "hostNic": host_nic,
            "maxUnavailable": {
                "description": "Agent Pods the DaemonSet may replace at once during a rolling update: a number or\n"
                               "a percentage of the targeted nodes (default 1, as in the reference).  Larger\n"
                               "values roll big clusters faster; with keepConfigOnRestart the roll does not\n"
                               "disturb running jobs.",
                "anyOf": [{"type": "integer"}, {"type": "string"}], "pattern": "^(100|[1-9][0-9]?)%$",
                "x-kubernetes-int-or-string": True},
            "logLevel": {"description": "LogLevel sets the agent's log level.", "maximum": T.LOG_LEVEL_MAX,
                         "minimum": T.LOG_LEVEL_MIN, "type": "integer"},
            "nodeSelector": {"additionalProperties": {"type": "string"},
                             "description": "Select which nodes the operator should target. Align with labels created by NFD.",
                             "type": "object"},
            "priorityClassName": {
                "description": "PriorityClass of the agent Pods (e.g. system-node-critical); empty = the cluster's\n"
                               "default priority.",
                "type": "string", "maxLength": 253,
                "pattern": "^[a-z0-9]([-a-z0-9]*[a-z0-9])?(\\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*$"},
            "tolerations": {
                "description": "Tolerations of the agent Pods (and of their cleanup and validation Jobs), so that\n"
                               "they run on tainted GPU nodes (e.g. amd.com/gpu:NoSchedule).",
                "type": "array",
                "items": {
                    "type": "object",
                    "properties": {
                        "key": {"type": "string"},
                        "operator": {"type": "string", "enum": ["Exists", "Equal"]},
                        "value": {"type": "string"},
                        "effect": {"type": "string", "enum": ["NoSchedule", "PreferNoSchedule", "NoExecute"]},
                        "tolerationSeconds": {"type": "integer", "format": "int64"},
                    },
                },
            },
        },
        "required": ["configurationType"],
    }
    status = {
        "description": "NetworkClusterPolicyStatus defines the observed state of NetworkClusterPolicy",
        "type": "object",
        "properties": {
            "conditions": {
                "description": ("Standard conditions: Ready (every targeted node is configured and "
                                "labelled) and Degraded (node or dependency errors; see errors)."),
                "type": "array",
                "x-kubernetes-list-type": "map",
                "x-kubernetes-list-map-keys": ["type"],
                "items": {
                    "type": "object",
                    "properties": {
                        "type": {"type": "string", "maxLength": 316},
                        "status": {"type": "string", "enum": ["True", "False", "Unknown"]},
                        "observedGeneration": {"type": "integer", "format": "int64", "minimum": 0},
                        "lastTransitionTime": {"type": "string", "format": "date-time"},
                        "reason": {"type": "string", "maxLength": 1024},
                        "message": {"type": "string", "maxLength": 32768},
                    },
                    "required": ["type", "status", "lastTransitionTime", "reason", "message"],
                },
            },
            "errors": {"items": {"type": "string"}, "type": "array"},
            "keptNodes": {"description": "Nodes whose agents left configuration behind (keepConfigOnRestart: addresses\n"
                                         "and routes; disableNetworkManager: NICs unmanaged) that a cleanup Job still\n"
                                         "has to remove when the policy is deleted or the node leaves it.",
                          "items": {"type": "string"}, "type": "array"},
            "observedGeneration": {"description": "The spec generation the status describes.",
                                   "format": "int64", "type": "integer"},
            "ready": {"format": "int32", "type": "integer"},
            "state": {"type": "string"},
            "targets": {"format": "int32", "type": "integer"},
        },
        "required": ["errors", "ready", "state", "targets"],
    }
    return {
        "description": "NetworkClusterPolicy is the Schema for the networkclusterpolicies API",
        "type": "object",
        "properties": {
            "apiVersion": {"description": _API_VERSION_DESC, "type": "string"},
            "kind": {"description": _KIND_DESC, "type": "string"},
            "metadata": {"type": "object"},
            "spec": spec,
            "status": status,
        },
    }


def crd_manifest() -> dict:
    return {
        "apiVersion": "apiextensions.k8s.io/v1",
        "kind": "CustomResourceDefinition",
        "metadata": {"name": f"{T.PLURAL}.{T.GROUP}",
                     "annotations": {"amd.com/generated-by": "network_operator_amd.api.v1alpha1.crd"}},
        "spec": {
            "group": T.GROUP,
            "names": {"kind": T.KIND, "listKind": T.LIST_KIND, "plural": T.PLURAL, "singular": T.SINGULAR,
                      "shortNames": ["ncp"]},
            "scope": "Cluster",
            "versions": [{
                "name": T.VERSION,
                "served": True,
                "storage": True,
                "schema": {"openAPIV3Schema": openapi_schema()},
                "subresources": {"status": {}},
                "additionalPrinterColumns": [
                    # amd-so and host-nic policies side by side: the type, and the layer of each.
                    {"name": "Type", "type": "string", "jsonPath": ".spec.configurationType"},
                    {"name": "Layer", "type": "string", "jsonPath": ".spec.amdScaleOut.layer"},
                    {"name": "Host-NIC-Layer", "type": "string", "priority": 1, "jsonPath": ".spec.hostNic.layer"},
                    {"name": "Targets", "type": "integer", "jsonPath": ".status.targets"},
                    {"name": "Ready", "type": "integer", "jsonPath": ".status.ready"},
                    {"name": "State", "type": "string", "jsonPath": ".status.state"},
                    {"name": "Degraded", "type": "string", "priority": 1,
                     "jsonPath": '.status.conditions[?(@.type=="Degraded")].status'},
                    {"name": "Age", "type": "date", "jsonPath": ".metadata.creationTimestamp"},
                ],
            }],
        },
    }


def render_yaml() -> str:
    return "---\n" + yaml.safe_dump(crd_manifest(), sort_keys=True, width=100)


# ---------------------------------------------------------------------------
# Structural-schema validation (subset of OpenAPI v3 used by CRDs)
# ---------------------------------------------------------------------------
_PY_TYPES = {"string": (str,), "integer": (int,), "boolean": (bool,), "object": (dict,), "array": (list,),
             "number": (int, float)}


def _validate(value: Any, schema: dict, path: str, errs: List[str]) -> None:
    if schema.get("x-kubernetes-int-or-string"):
        if isinstance(value, bool) or not isinstance(value, (int, str)):
            errs.append(f"{path}: Invalid value: {value!r}: {path} in body must be of type integer or string")
            return
        if isinstance(value, str) and "pattern" in schema and not re.search(schema["pattern"], value):
            errs.append(f'{path}: Invalid value: "{value}": {path} in body should match \'{schema["pattern"]}\'')
        return
    t = schema.get("type")
    if t:
        ok = isinstance(value, _PY_TYPES[t]) and not (t in ("integer", "number") and isinstance(value, bool))
        if not ok:
            errs.append(f"{path}: Invalid value: {value!r}: {path} in body must be of type {t}")
            return
    if "enum" in schema and value not in schema["enum"]:
        allowed = ", ".join(f'"{x}"' for x in schema["enum"])
        errs.append(f"{path}: Unsupported value: {value!r}: supported values: {allowed}")
    if "minimum" in schema and isinstance(value, (int, float)) and value < schema["minimum"]:
        errs.append(f"{path}: Invalid value: {value}: {path} in body should be greater than or equal to {schema['minimum']}")
    if "maximum" in schema and isinstance(value, (int, float)) and value > schema["maximum"]:
        errs.append(f"{path}: Invalid value: {value}: {path} in body should be less than or equal to {schema['maximum']}")
    if "maxLength" in schema and isinstance(value, str) and len(value) > schema["maxLength"]:
        errs.append(f"{path}: Too long: may not be longer than {schema['maxLength']}")
    if "pattern" in schema and isinstance(value, str) and not re.search(schema["pattern"], value):
        errs.append(f'{path}: Invalid value: "{value}": {path} in body should match \'{schema["pattern"]}\'')
    if isinstance(value, dict):
        for r in schema.get("required", []):
            if r not in value:
                errs.append(f"{path}.{r}: Required value")
        props = schema.get("properties", {})
        addl = schema.get("additionalProperties")
        for k, v in value.items():
            if k in props:
                _validate(v, props[k], f"{path}.{k}", errs)
            elif isinstance(addl, dict):
                _validate(v, addl, f"{path}.{k}", errs)
    if isinstance(value, list) and "items" in schema:
        for i, v in enumerate(value):
            _validate(v, schema["items"], f"{path}[{i}]", errs)


def prune(value: Any, schema: dict) -> Any:
    """Drops fields unknown to a structural schema (what the API server does on write)."""
    if isinstance(value, dict) and schema.get("type") == "object":
        props = schema.get("properties")
        addl = schema.get("additionalProperties")
        if props is None and addl is None:
            return value  # e.g. metadata: opaque
        out = {}
        for k, v in value.items():
            if props and k in props:
                out[k] = prune(v, props[k])
            elif isinstance(addl, dict):
                out[k] = prune(v, addl)
        return out
    if isinstance(value, list) and "items" in schema:
        return [prune(v, schema["items"]) for v in value]
    return value


def apply_defaults(value: Any, schema: dict) -> Any:
    """Fills the schema's ``default`` values into objects that lack the field, in place -- what
    the API server does for a structural schema, on every read and write, before mutating
    admission (so a minimal policy written with kubectl gets them even with webhooks off)."""
    if isinstance(value, dict) and schema.get("type") == "object":
        for k, ps in (schema.get("properties") or {}).items():
            if k not in value and "default" in ps:
                value[k] = ps["default"]
            if k in value:
                apply_defaults(value[k], ps)
    elif isinstance(value, list) and isinstance(schema.get("items"), dict):
        for v in value:
            apply_defaults(v, schema["items"])
    return value


def validate(obj: dict) -> List[str]:
    """Returns the API-server style field errors for a NetworkClusterPolicy object."""
    errs: List[str] = []
    schema = openapi_schema()
    body = {k: v for k, v in obj.items() if k in ("apiVersion", "kind", "metadata", "spec", "status")}
    # status is validated through the status subresource only
    body.pop("status", None)
    _validate(body, schema, "", errs)
    return [e[1:] if e.startswith(".") else e for e in errs]


def missing_fields(installed: dict) -> List[str]:
    """Property paths of this release's schema that an installed CRD object lacks, e.g.
    ``spec.amdScaleOut.carrierWait``.  Helm installs ``crds/`` once and never upgrades it, so
    after ``helm upgrade`` the API server keeps the old schema and silently drops every new field
    a user sets (structural pruning, before any webhook sees the object)."""
    want = openapi_schema()
    have = next((v.get("schema", {}).get("openAPIV3Schema") for v in (installed.get("spec") or {}).get("versions") or []
                 if v.get("name") == T.VERSION), None)
    if have is None:
        return [f"version {T.VERSION}"]
    out: List[str] = []

    def walk(w: dict, h: dict, path: str) -> None:
        if h.get("x-kubernetes-preserve-unknown-fields"):
            return  # the installed schema keeps anything here
        for k, ws in (w.get("properties") or {}).items():
            hs = (h.get("properties") or {}).get(k)
            if hs is None:
                out.append(path + k)
            else:
                walk(ws, hs, path + k + ".")
        for key in ("items", "additionalProperties"):
            if isinstance(w.get(key), dict) and isinstance(h.get(key), dict):
                walk(w[key], h[key], path + ("[]." if key == "items" else "*."))
    walk(want, have, "")
    return out


def main(argv=None) -> int:
    root = Path(__file__).resolve().parents[3]
    text = render_yaml()
    targets = [root / "config/operator/crd/bases/amd.com_networkclusterpolicies.yaml",
               root / "charts/network-operator/crds/networkclusterpolicy-crd.yaml"]
    if argv and argv[0] == "--stdout":
        sys.stdout.write(text)
        return 0
    for t in targets:
        t.parent.mkdir(parents=True, exist_ok=True)
        t.write_text(text)
        print(f"wrote {t}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
