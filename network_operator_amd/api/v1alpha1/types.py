"""v1alpha1 ``NetworkClusterPolicy`` — cluster-scoped, group ``amd.com``.

Field-for-field counterpart of the reference's CRD types
(reference api/v1alpha1/networkconfiguration_types.go:24-100) with the Gaudi specifics
renamed for MI355X:

=====================================  ==============================================
reference                              this API
=====================================  ==============================================
configurationType enum ``gaudi-so``    ``amd-so``; ``host-nic`` (the reference's TODO, types.go:26,
                                       README "Future work") implemented as spec.hostNic
spec.gaudiScaleOut                     spec.amdScaleOut (same sub-fields)
status {targets, ready, state, errors} identical
=====================================  ==============================================

``amdScaleOut`` adds optional MI355X fields (all additive): ``xgmiCheck`` (gate readiness on the
xGMI mesh; on unless set false), ``requireRdma`` (gate it on every rail's RDMA device; on unless
set false), ``driverImage`` (the NICs' RDMA driver container), ``lldpAnnounce`` (self-announce to
trigger switch fast start), ``interfaces`` (extra NICs) and ``nicDrivers`` (affinity allow-list).

Objects are plain dataclasses with lossless ``to_dict`` / ``from_dict`` (unknown fields are
preserved in ``extra`` so a round trip never drops data written by a newer client).
"""

from __future__ import annotations

import copy
from dataclasses import dataclass, field
from typing import Any, Dict, List, Optional, Union

GROUP = "amd.com"
VERSION = "v1alpha1"
API_VERSION = f"{GROUP}/{VERSION}"
KIND = "NetworkClusterPolicy"
LIST_KIND = "NetworkClusterPolicyList"
PLURAL = "networkclusterpolicies"
SINGULAR = "networkclusterpolicy"

CONFIG_AMD_SCALE_OUT = "amd-so"
CONFIG_HOST_NIC = "host-nic"
CONFIGURATION_TYPES = (CONFIG_AMD_SCALE_OUT, CONFIG_HOST_NIC)
LAYERS = ("L2", "L3")
# lldpWait: a Go duration the agent's --wait accepts (units h, m, s, ms), checked 1s..30m by the webhook
LLDP_WAIT_PATTERN = r"^([0-9]+(\.[0-9]+)?(h|m|s|ms))+$"
LLDP_WAIT_MIN_S, LLDP_WAIT_MAX_S = 1.0, 1800.0
# carrierWait: the same duration grammar; L2, how long NICs may train their links (agent default 30s)
CARRIER_WAIT_MIN_S, CARRIER_WAIT_MAX_S = 1.0, 600.0
# rdmaWait: the same grammar; how long a missing RDMA device is start-up (agent default 5m)
RDMA_WAIT_MIN_S, RDMA_WAIT_MAX_S = 1.0, 3600.0


def parse_go_duration(s: str) -> float:
    """Seconds of a Go duration string limited to h/m/s/ms units ("90s", "1m30s", "1.5s");
    raises ValueError otherwise."""
    import re

    if not re.fullmatch(LLDP_WAIT_PATTERN, s or ""):
        raise ValueError(f"not a duration: {s!r}")
    unit = {"h": 3600.0, "m": 60.0, "s": 1.0, "ms": 1e-3}
    return sum(float(v) * unit[u] for v, u in re.findall(r"([0-9]+(?:\.[0-9]+)?)(ms|h|m|s)", s))
PULL_POLICIES = ("Never", "Always", "IfNotPresent")
MTU_MIN, MTU_MAX = 1500, 9000
LOG_LEVEL_MIN, LOG_LEVEL_MAX = 0, 8
DEFAULT_AGENT_IMAGE = "amd/amd-network-linkdiscovery:latest"
OPERATOR_VERSION = "0.1.0"  # the agent release whose flags the operator passes (Makefile VERSION)


DEFAULT_VALIDATION_IMAGE = "amd/amd-network-validation:0.1.0"


@dataclass
class ValidationSpec:
    """Post-configuration fabric validation (MI355X addition): once a node's agent is ready, the
    operator runs ``python -m network_operator_amd.validate`` there as a Job (all-reduce checked
    exactly, busbw and xGMI link floors, NCCL_TOPO_FILE loaded by RCCL) and reports the result in
    the policy's ``FabricValidated`` condition; a passing node gets the
    ``gpu-fabric-validated`` label."""
    enabled: bool = False
    image: str = ""
    gpus: int = 0           # 0 = 8 (the whole node)
    minBusbw: int = 0       # GB/s, large-message all-reduce; 0 = correctness only
    minLink: int = 0        # GB/s per xGMI link (pull); 0 = not checked

    def to_dict(self) -> dict:
        d: dict = {"enabled": self.enabled}
        for k in ("image", "gpus", "minBusbw", "minLink"):
            if getattr(self, k):
                d[k] = getattr(self, k)
        return d

    @classmethod
    def from_dict(cls, d: Optional[dict]) -> Optional["ValidationSpec"]:
        if d is None:
            return None
        return cls(enabled=bool(d.get("enabled", False)), image=d.get("image", "") or "", gpus=int(d.get("gpus", 0) or 0),
                   minBusbw=int(d.get("minBusbw", 0) or 0), minLink=int(d.get("minLink", 0) or 0))


@dataclass
class AmdScaleOutSpec:
    disableNetworkManager: bool = False
    layer: str = ""
    image: str = ""
    pullPolicy: str = ""
    mtu: int = 0
    # MI355X additions
    xgmiCheck: Optional[bool] = None  # None = on (the CRD default, the mutating webhook): verify the mesh
    lldpAnnounce: Optional[bool] = None
    interfaces: List[str] = field(default_factory=list)
    nicDrivers: List[str] = field(default_factory=list)
    disableFirmwareLldp: bool = False
    metricsPort: int = 0
    gpuDirectRdma: str = ""
    rcclEnv: Dict[str, str] = field(default_factory=dict)
    railTableBase: int = 0
    rcclSocketIfname: str = ""
    lldpCache: bool = False
    verifyPeers: bool = False
    lldpWait: str = ""  # L3 LLDP wait (Go duration); "" = the reference's 90s
    carrierWait: str = ""  # L2 link-training allowance (Go duration); "" = the agent's 30s
    # Hitless agent restarts: addresses / routes stay when an agent exits; the operator cleans the
    # nodes up (cleanup Jobs) when the policy is deleted or a node leaves it.
    keepConfigOnRestart: bool = False
    # L3 rail cabling check: regex over the LLDP System Name, "{rail}" = GPU index ("" = off)
    railSwitchPattern: str = ""
    # Minimum negotiated link speed of every scale-out NIC, Gb/s (0 = off)
    minLinkSpeedGbps: int = 0
    # Every scale-out NIC's PCIe link trained at the speed and width it supports, its GPU's at full width
    requireFullPcieLink: bool = False
    # L3 jumbo-frame check against the switch port's LLDP 802.3 Maximum Frame Size (None = on)
    checkPeerMtu: Optional[bool] = None
    # With disableFirmwareLldp: hand DCBX to the host on DCB NICs without a firmware-LLDP flag
    handDcbxToHost: bool = False
    # Scale-out ready means RDMA ready: every rail needs an RDMA device before the label and
    # rccl.env (None = on, like xgmiCheck).  rdmaWait: how long that is start-up (Go duration).
    requireRdma: Optional[bool] = None
    rdmaWait: str = ""
    # The NICs' RDMA driver (KMD) container, a privileged init container as for hostNic.driverImage
    driverImage: str = ""
    # Configure a NIC whose default route lives in a per-NIC policy-routing table even when it
    # holds the node's own address (refused by default, like the node's uplink)
    allowPolicyRouted: bool = False
    validation: Optional[ValidationSpec] = None
    extra: Dict[str, Any] = field(default_factory=dict)

    def __post_init__(self):
        if isinstance(self.validation, dict):  # new_policy(validation={...})
            self.validation = ValidationSpec.from_dict(self.validation)

    _FIELDS = ("disableNetworkManager", "layer", "image", "pullPolicy", "mtu", "xgmiCheck", "lldpAnnounce",
               "interfaces", "nicDrivers", "disableFirmwareLldp", "metricsPort", "gpuDirectRdma", "rcclEnv",
               "railTableBase", "rcclSocketIfname", "lldpCache", "verifyPeers", "lldpWait", "carrierWait", "keepConfigOnRestart",
               "railSwitchPattern", "minLinkSpeedGbps", "requireFullPcieLink", "checkPeerMtu", "handDcbxToHost",
               "requireRdma", "rdmaWait", "driverImage", "allowPolicyRouted", "validation")

    def to_dict(self) -> dict:
        d: dict = {}
        # omitempty semantics, like the Go struct tags
        if self.disableNetworkManager:
            d["disableNetworkManager"] = True
        for k in ("layer", "image", "pullPolicy"):
            if getattr(self, k):
                d[k] = getattr(self, k)
        if self.mtu:
            d["mtu"] = self.mtu
        if self.xgmiCheck is not None:
            d["xgmiCheck"] = self.xgmiCheck
        if self.lldpAnnounce is not None:
            d["lldpAnnounce"] = self.lldpAnnounce
        if self.interfaces:
            d["interfaces"] = list(self.interfaces)
        if self.nicDrivers:
            d["nicDrivers"] = list(self.nicDrivers)
        if self.disableFirmwareLldp:
            d["disableFirmwareLldp"] = True
        if self.metricsPort:
            d["metricsPort"] = self.metricsPort
        if self.gpuDirectRdma:
            d["gpuDirectRdma"] = self.gpuDirectRdma
        if self.rcclEnv:
            d["rcclEnv"] = dict(self.rcclEnv)
        if self.railTableBase:
            d["railTableBase"] = self.railTableBase
        if self.rcclSocketIfname:
            d["rcclSocketIfname"] = self.rcclSocketIfname
        if self.lldpCache:
            d["lldpCache"] = True
        if self.verifyPeers:
            d["verifyPeers"] = True
        if self.lldpWait:
            d["lldpWait"] = self.lldpWait
        if self.carrierWait:
            d["carrierWait"] = self.carrierWait
        if self.keepConfigOnRestart:
            d["keepConfigOnRestart"] = True
        if self.railSwitchPattern:
            d["railSwitchPattern"] = self.railSwitchPattern
        if self.minLinkSpeedGbps:
            d["minLinkSpeedGbps"] = self.minLinkSpeedGbps
        if self.requireFullPcieLink:
            d["requireFullPcieLink"] = True
        if self.checkPeerMtu is not None:
            d["checkPeerMtu"] = self.checkPeerMtu
        if self.handDcbxToHost:
            d["handDcbxToHost"] = True
        if self.requireRdma is not None:
            d["requireRdma"] = self.requireRdma
        if self.rdmaWait:
            d["rdmaWait"] = self.rdmaWait
        if self.driverImage:
            d["driverImage"] = self.driverImage
        if self.allowPolicyRouted:
            d["allowPolicyRouted"] = True
        if self.validation is not None:
            d["validation"] = self.validation.to_dict()
        d.update(copy.deepcopy(self.extra))
        return d

    @classmethod
    def from_dict(cls, d: Optional[dict]) -> "AmdScaleOutSpec":
        d = dict(d or {})
        s = cls(
            disableNetworkManager=bool(d.pop("disableNetworkManager", False)),
            layer=d.pop("layer", "") or "",
            image=d.pop("image", "") or "",
            pullPolicy=d.pop("pullPolicy", "") or "",
            mtu=int(d.pop("mtu", 0) or 0),
            xgmiCheck=d.pop("xgmiCheck", None),
            lldpAnnounce=d.pop("lldpAnnounce", None),
            interfaces=list(d.pop("interfaces", []) or []),
            nicDrivers=list(d.pop("nicDrivers", []) or []),
            disableFirmwareLldp=bool(d.pop("disableFirmwareLldp", False)),
            metricsPort=int(d.pop("metricsPort", 0) or 0),
            gpuDirectRdma=d.pop("gpuDirectRdma", "") or "",
            rcclEnv=dict(d.pop("rcclEnv", {}) or {}),
            railTableBase=int(d.pop("railTableBase", 0) or 0),
            rcclSocketIfname=d.pop("rcclSocketIfname", "") or "",
            lldpCache=bool(d.pop("lldpCache", False)),
            keepConfigOnRestart=bool(d.pop("keepConfigOnRestart", False)),
            railSwitchPattern=d.pop("railSwitchPattern", "") or "",
            minLinkSpeedGbps=int(d.pop("minLinkSpeedGbps", 0) or 0),
            requireFullPcieLink=bool(d.pop("requireFullPcieLink", False)),
            checkPeerMtu=d.pop("checkPeerMtu", None),
            handDcbxToHost=bool(d.pop("handDcbxToHost", False)),
            requireRdma=d.pop("requireRdma", None),
            rdmaWait=d.pop("rdmaWait", "") or "",
            driverImage=d.pop("driverImage", "") or "",
            allowPolicyRouted=bool(d.pop("allowPolicyRouted", False)),
            verifyPeers=bool(d.pop("verifyPeers", False)),
            lldpWait=d.pop("lldpWait", "") or "",
            carrierWait=d.pop("carrierWait", "") or "",
            validation=ValidationSpec.from_dict(d.pop("validation", None)),
        )
        s.extra = d
        return s


@dataclass
class HostNicSpec:
    """``host-nic``: the node's own RDMA NICs (frontend / storage / scale-out NICs not paired
    with a GPU), configured by the same agent in ``--nic-discovery=rdma`` mode, optionally after
    a driver container installed the NIC's kernel driver (KMD)."""
    layer: str = ""
    mtu: int = 0
    image: str = ""
    pullPolicy: str = ""
    disableNetworkManager: bool = False
    interfaces: List[str] = field(default_factory=list)
    nicDrivers: List[str] = field(default_factory=list)
    driverImage: str = ""
    verifyPeers: bool = False
    lldpWait: str = ""
    carrierWait: str = ""
    keepConfigOnRestart: bool = False
    checkPeerMtu: Optional[bool] = None
    includeGpuRails: bool = False  # discovery may take the NICs next to the GPUs (no amd-so policy)
    minLinkSpeedGbps: int = 0  # as amdScaleOut's, for the host NICs
    requireFullPcieLink: bool = False  # as amdScaleOut's (host NICs have no GPU: the NIC's link)
    allowPolicyRouted: bool = False  # as amdScaleOut's
    extra: Dict[str, Any] = field(default_factory=dict)

    def to_dict(self) -> dict:
        d: dict = {}
        for k in ("layer", "image", "pullPolicy", "driverImage", "lldpWait", "carrierWait"):
            if getattr(self, k):
                d[k] = getattr(self, k)
        if self.mtu:
            d["mtu"] = self.mtu
        if self.disableNetworkManager:
            d["disableNetworkManager"] = True
        if self.interfaces:
            d["interfaces"] = list(self.interfaces)
        if self.nicDrivers:
            d["nicDrivers"] = list(self.nicDrivers)
        if self.verifyPeers:
            d["verifyPeers"] = True
        if self.keepConfigOnRestart:
            d["keepConfigOnRestart"] = True
        if self.checkPeerMtu is not None:
            d["checkPeerMtu"] = self.checkPeerMtu
        if self.includeGpuRails:
            d["includeGpuRails"] = True
        if self.minLinkSpeedGbps:
            d["minLinkSpeedGbps"] = self.minLinkSpeedGbps
        if self.requireFullPcieLink:
            d["requireFullPcieLink"] = True
        if self.allowPolicyRouted:
            d["allowPolicyRouted"] = True
        d.update(copy.deepcopy(self.extra))
        return d

    @classmethod
    def from_dict(cls, d: Optional[dict]) -> "HostNicSpec":
        d = dict(d or {})
        s = cls(layer=d.pop("layer", "") or "", mtu=int(d.pop("mtu", 0) or 0), image=d.pop("image", "") or "",
                pullPolicy=d.pop("pullPolicy", "") or "", disableNetworkManager=bool(d.pop("disableNetworkManager", False)),
                interfaces=list(d.pop("interfaces", []) or []), nicDrivers=list(d.pop("nicDrivers", []) or []),
                driverImage=d.pop("driverImage", "") or "", verifyPeers=bool(d.pop("verifyPeers", False)),
                lldpWait=d.pop("lldpWait", "") or "",
                carrierWait=d.pop("carrierWait", "") or "",
                keepConfigOnRestart=bool(d.pop("keepConfigOnRestart", False)),
                checkPeerMtu=d.pop("checkPeerMtu", None),
                includeGpuRails=bool(d.pop("includeGpuRails", False)),
                minLinkSpeedGbps=int(d.pop("minLinkSpeedGbps", 0) or 0),
                requireFullPcieLink=bool(d.pop("requireFullPcieLink", False)),
                allowPolicyRouted=bool(d.pop("allowPolicyRouted", False)))
        s.extra = d
        return s


@dataclass
class NetworkClusterPolicySpec:
    configurationType: str = ""
    nodeSelector: Dict[str, str] = field(default_factory=dict)
    amdScaleOut: AmdScaleOutSpec = field(default_factory=AmdScaleOutSpec)
    hostNic: Optional[HostNicSpec] = None
    logLevel: int = 0
    # DaemonSet rollingUpdate.maxUnavailable: int >= 1 or "N%" (None = 1, the reference's default)
    maxUnavailable: Optional[Union[int, str]] = None
    # Pod tolerations of the agent DaemonSet (and of its cleanup / validation Jobs): GPU nodes are
    # often tainted (amd.com/gpu:NoSchedule) and the agent has to run on every one of them.
    tolerations: List[Dict[str, Any]] = field(default_factory=list)
    # PriorityClass of the agent Pods (e.g. system-node-critical: a node's network agent should not
    # be the first Pod evicted under memory pressure).  "" = the cluster default.
    priorityClassName: str = ""
    extra: Dict[str, Any] = field(default_factory=dict)

    def to_dict(self) -> dict:
        d: dict = {"configurationType": self.configurationType}
        if self.nodeSelector:
            d["nodeSelector"] = dict(self.nodeSelector)
        so = self.amdScaleOut.to_dict()
        d["amdScaleOut"] = so  # struct without omitempty pointer: always serialised
        if self.hostNic is not None:
            d["hostNic"] = self.hostNic.to_dict()
        if self.logLevel:
            d["logLevel"] = self.logLevel
        if self.maxUnavailable is not None:
            d["maxUnavailable"] = self.maxUnavailable
        if self.tolerations:
            d["tolerations"] = copy.deepcopy(self.tolerations)
        if self.priorityClassName:
            d["priorityClassName"] = self.priorityClassName
        d.update(copy.deepcopy(self.extra))
        return d

    @classmethod
    def from_dict(cls, d: Optional[dict]) -> "NetworkClusterPolicySpec":
        d = dict(d or {})
        s = cls(
            configurationType=d.pop("configurationType", "") or "",
            nodeSelector=dict(d.pop("nodeSelector", {}) or {}),
            amdScaleOut=AmdScaleOutSpec.from_dict(d.pop("amdScaleOut", None)),
            hostNic=HostNicSpec.from_dict(d.pop("hostNic")) if d.get("hostNic") is not None else None,
            logLevel=int(d.pop("logLevel", 0) or 0),
            maxUnavailable=d.pop("maxUnavailable", None),
            tolerations=copy.deepcopy(list(d.pop("tolerations", []) or [])),
            priorityClassName=d.pop("priorityClassName", "") or "",
        )
        s.extra = d
        return s


@dataclass
class NetworkClusterPolicyStatus:
    targets: int = 0
    ready: int = 0
    state: str = ""
    errors: List[str] = field(default_factory=list)
    # Additive (not in the reference): standard conditions and the generation they describe.
    conditions: List[dict] = field(default_factory=list)
    observedGeneration: int = 0
    # Nodes whose agents left configuration behind (keepConfigOnRestart, disableNetworkManager):
    # a cleanup Job is owed to each (reconciler.needs_node_cleanup).
    keptNodes: List[str] = field(default_factory=list)

    def to_dict(self) -> dict:
        d = {"targets": self.targets, "ready": self.ready, "state": self.state, "errors": list(self.errors)}
        if self.conditions:
            d["conditions"] = [dict(c) for c in self.conditions]
        if self.observedGeneration:
            d["observedGeneration"] = self.observedGeneration
        if self.keptNodes:
            d["keptNodes"] = list(self.keptNodes)
        return d

    @classmethod
    def from_dict(cls, d: Optional[dict]) -> "NetworkClusterPolicyStatus":
        d = d or {}
        return cls(targets=int(d.get("targets", 0) or 0), ready=int(d.get("ready", 0) or 0),
                   state=d.get("state", "") or "", errors=list(d.get("errors") or []),
                   conditions=[dict(c) for c in d.get("conditions") or []],
                   observedGeneration=int(d.get("observedGeneration", 0) or 0),
                   keptNodes=list(d.get("keptNodes") or []))

    def condition(self, type_: str) -> Optional[dict]:
        return next((c for c in self.conditions if c.get("type") == type_), None)


@dataclass
class NetworkClusterPolicy:
    metadata: Dict[str, Any] = field(default_factory=dict)
    spec: NetworkClusterPolicySpec = field(default_factory=NetworkClusterPolicySpec)
    status: NetworkClusterPolicyStatus = field(default_factory=NetworkClusterPolicyStatus)
    has_status: bool = False

    apiVersion = API_VERSION
    kind = KIND

    @property
    def name(self) -> str:
        return self.metadata.get("name", "")

    @property
    def uid(self) -> str:
        return self.metadata.get("uid", "")

    def to_dict(self) -> dict:
        d = {"apiVersion": API_VERSION, "kind": KIND, "metadata": copy.deepcopy(self.metadata),
             "spec": self.spec.to_dict()}
        if self.has_status or self.status.state or self.status.targets or self.status.ready:
            d["status"] = self.status.to_dict()
        return d

    @classmethod
    def from_dict(cls, d: dict) -> "NetworkClusterPolicy":
        return cls(metadata=copy.deepcopy(d.get("metadata", {})), spec=NetworkClusterPolicySpec.from_dict(d.get("spec")),
                   status=NetworkClusterPolicyStatus.from_dict(d.get("status")), has_status="status" in d)

    def deepcopy(self) -> "NetworkClusterPolicy":
        """DeepCopy (reference zz_generated.deepcopy.go): maps and slices are copied, not shared."""
        return copy.deepcopy(self)


def new_policy(name: str, layer: str = "L3", node_selector: Optional[dict] = None, **so) -> NetworkClusterPolicy:
    """Convenience constructor used by samples, the Helm renderer and tests."""
    return NetworkClusterPolicy(
        metadata={"name": name},
        spec=NetworkClusterPolicySpec(configurationType=CONFIG_AMD_SCALE_OUT,
                                      nodeSelector=dict({"amd.feature.node.kubernetes.io/gpu-ready": "true"}
                                                        if node_selector is None else node_selector),
                                      amdScaleOut=AmdScaleOutSpec(layer=layer, **so)))


def new_host_nic_policy(name: str, layer: str = "L3", node_selector: Optional[dict] = None,
                        **hn) -> NetworkClusterPolicy:
    return NetworkClusterPolicy(
        metadata={"name": name},
        spec=NetworkClusterPolicySpec(configurationType=CONFIG_HOST_NIC,
                                      nodeSelector=dict({"amd.feature.node.kubernetes.io/gpu-ready": "true"}
                                                        if node_selector is None else node_selector),
                                      hostNic=HostNicSpec(layer=layer, **hn)))
