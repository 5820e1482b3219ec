"""``NetworkClusterPolicy`` reconciler.

Behavioural counterpart of the reference controller
(reference internal/controller/networkconfiguration_controller.go):

* one DaemonSet per policy, named after the policy, in the operator namespace, owned by the
  policy (controller ownerReference -> garbage-collected with it);
* agent arguments are fully recomputed from the spec on every reconcile, in the reference
  order ``--configure=true --keep-running --mode=<L> [--v=N] [--mtu=N]
  [--disable-networkmanager] [L3: --wait=90s --rccl-net=... ]`` (:164-204), followed by the
  MI355X options;
* hostPath volumes are added by name with type DirectoryOrCreate in the reference order
  (nfd-features, [var-run-dbus, networkmanager], [artifact dir]) (:69-107);
* status mirrors the DaemonSet: targets = desiredNumberScheduled, ready = numberReady,
  state "No targets" / "Working on it.." / "All good", errors [] (:267-307); a status
  write conflict requeues;
* OpenShift: ServiceAccount ``<name>-sa`` + RoleBinding ``<name>-sa-rb`` to
  ``system:openshift:scc:privileged`` (:109-162).

Deliberate fixes (SURVEY.md §7.6 "fix" list): ``pullPolicy`` is applied; volumes that are no
longer wanted are removed; the agent has a readinessProbe (in the template) so ``ready``
counts *configured* nodes; ``AlreadyExists`` on create falls back to the update path; and
Kubernetes Events are emitted (RBAC for them was granted but unused by the reference).
"""

from __future__ import annotations

import asyncio
import copy
import time
import logging
from dataclasses import dataclass
from typing import Callable, Dict, List, Optional, Set, Tuple

from .. import discovery
from ..api.v1alpha1 import types as T
from . import kube
from .kube import ApiClient, ApiError, is_already_exists, is_conflict, is_not_found

log = logging.getLogger("controller")

OWNER_KEY = ".metadata.controller"
ARTIFACT_DIR_HOST = "/etc/amd/scale-out"
ARTIFACT_DIR_CONTAINER = "/host" + ARTIFACT_DIR_HOST
RCCL_NET_FILE = "rccl-net.json"
RCCL_ENV_FILE = "rccl.env"
RCCL_TOPO_FILE = "rccl-topo.xml"
# --verify-peers: a switch answers ARP in well under a millisecond; 2 s covers a port that is
# still coming up, and stays far below the kubelet's restart back-off.
VERIFY_PEERS_TIMEOUT = "2s"
FW_LLDP_STATE_FILE = "fw-lldp-state"  # --fw-lldp-state: firmware LLDP originals kept by --keep-config agents
LLDP_CACHE_FILE = "lldp-cache"  # --lldp-cache, beside the artifacts so it survives pod restarts
L3_WAIT = "90s"

STATE_NO_TARGETS = "No targets"
STATE_WORKING = "Working on it.."
STATE_ALL_GOOD = "All good"
COND_READY = "Ready"
COND_DEGRADED = "Degraded"
COND_VALIDATED = "FabricValidated"
VALIDATION_APP = "amd-gpu-fabric-validation"  # Job label; the operator's Job informer selects on it

# Volumes the reconciler manages (the template's nfd-features is never touched).
MANAGED_VOLUMES = ("var-run-dbus", "networkmanager", "rccl-artifacts")


@dataclass
class Result:
    requeue: bool = False
    requeue_after: float = 0.0


def owner_reference(owner: dict) -> dict:
    md = owner["metadata"]
    return {"apiVersion": owner.get("apiVersion", T.API_VERSION), "kind": owner.get("kind", T.KIND), "name": md["name"],
            "uid": md.get("uid", ""), "controller": True, "blockOwnerDeletion": True}


def set_controller_reference(owner: dict, obj: dict) -> None:
    """ctrl.SetControllerReference: replace any existing controller reference."""
    refs = [r for r in obj.setdefault("metadata", {}).get("ownerReferences", []) or [] if not r.get("controller")]
    refs.append(owner_reference(owner))
    obj["metadata"]["ownerReferences"] = refs


def policy_owner_index(obj: dict) -> List[str]:
    """indexDaemonSets (:364-383): DaemonSets -> name of the owning NetworkClusterPolicy."""
    for ref in obj.get("metadata", {}).get("ownerReferences", []) or []:
        if ref.get("controller") and ref.get("apiVersion") == T.API_VERSION and ref.get("kind") == T.KIND:
            return [ref["name"]]
    return []


def job_owner_index(obj: dict) -> List[str]:
    """Pods -> name of the owning Job (the validation Jobs' Pods)."""
    for ref in obj.get("metadata", {}).get("ownerReferences", []) or []:
        if ref.get("controller") and ref.get("apiVersion") == "batch/v1" and ref.get("kind") == "Job":
            return [ref["name"]]
    return []


def daemonset_owner_index(obj: dict) -> List[str]:
    """indexPods (:385-404): Pods -> name of the owning DaemonSet."""
    for ref in obj.get("metadata", {}).get("ownerReferences", []) or []:
        if ref.get("controller") and ref.get("apiVersion") == "apps/v1" and ref.get("kind") == "DaemonSet":
            return [ref["name"]]
    return []


def add_host_volume(ds: dict, name: str, host_path: str, container_path: str,
                    volume_type: str = "DirectoryOrCreate") -> None:
    spec = ds["spec"]["template"]["spec"]
    vols = spec.setdefault("volumes", [])
    if any(v.get("name") == name for v in vols):
        return
    vols.append({"name": name, "hostPath": {"path": host_path, "type": volume_type}})
    containers = spec.get("containers") or []
    if containers:
        containers[0].setdefault("volumeMounts", []).append({"name": name, "mountPath": container_path})


def remove_volume(ds: dict, name: str) -> None:
    spec = ds["spec"]["template"]["spec"]
    spec["volumes"] = [v for v in spec.get("volumes", []) if v.get("name") != name]
    for c in spec.get("containers") or []:
        if "volumeMounts" in c:
            c["volumeMounts"] = [m for m in c["volumeMounts"] if m.get("name") != name]


def order_managed_volumes(ds: dict) -> None:
    """Volumes (and the agent's mounts) in one canonical order: the template's own first, then
    NetworkManager, then artifacts, then the driver container's -- the order the reference
    produces from scratch (controller_test.go:170-179), kept stable however the spec evolves."""
    rank = {n: i for i, n in enumerate(MANAGED_VOLUMES + ("host-lib-modules",))}
    key = lambda x: (x.get("name") in rank, rank.get(x.get("name"), 0))  # noqa: E731 (stable sort)
    pod = ds["spec"]["template"]["spec"]
    if "volumes" in pod:
        pod["volumes"] = sorted(pod["volumes"], key=key)
    for c in pod.get("containers") or []:
        if "volumeMounts" in c:
            c["volumeMounts"] = sorted(c["volumeMounts"], key=key)


def agent_args(p: T.NetworkClusterPolicy) -> List[str]:
    so = p.spec.amdScaleOut
    args = ["--configure=true", "--keep-running", f"--mode={so.layer}"]
    if p.spec.logLevel > 0:
        args.append(f"--v={p.spec.logLevel}")
    if so.mtu > 0:
        args.append(f"--mtu={so.mtu}")
    if so.disableNetworkManager:
        args += ["--disable-networkmanager", "--nm-keyfile-dir=/etc/NetworkManager/conf.d"]
    if so.layer == "L3":
        args += [f"--wait={so.lldpWait or L3_WAIT}", f"--rccl-net={ARTIFACT_DIR_CONTAINER}/{RCCL_NET_FILE}",
                 f"--rccl-env={ARTIFACT_DIR_CONTAINER}/{RCCL_ENV_FILE}"]
    else:
        # MI355X: RCCL needs the HCA list and the link-local RoCE v2 GID in L2 as well (Gaudi's
        # firmware did not, so the reference passes nothing in L2).
        args.append(f"--rccl-env={ARTIFACT_DIR_CONTAINER}/{RCCL_ENV_FILE}")
        if so.carrierWait:
            args.append(f"--carrier-wait={so.carrierWait}")
    # NCCL_TOPO_FILE: written through the agent's mount, named in rccl.env by the host path jobs
    # mount (the reference's HCCL contract is gaudinet.json, controller.go:198-200).
    args += [f"--rccl-topo={ARTIFACT_DIR_CONTAINER}/{RCCL_TOPO_FILE}",
             f"--rccl-topo-env-path={ARTIFACT_DIR_HOST}/{RCCL_TOPO_FILE}"]
    # MI355X options
    if so.xgmiCheck:
        args.append("--xgmi-expect=0")
    if so.lldpAnnounce is False:
        args.append("--lldp-announce=false")
    if so.interfaces:
        args.append("--interfaces=" + ",".join(so.interfaces))
    if so.nicDrivers:
        args.append("--nic-drivers=" + ",".join(so.nicDrivers))
    if so.disableFirmwareLldp and so.layer == "L3":
        args.append("--disable-fw-lldp")
        if so.handDcbxToHost:  # opt-in: the NIC firmware stops negotiating PFC/ETS
            args.append("--fw-lldp-dcbx-host")
    if so.metricsPort:
        args.append(f"--metrics-bind-address=:{so.metricsPort}")
    if so.railTableBase and so.layer == "L3":
        args.append(f"--rail-table-base={so.railTableBase}")
    if so.rcclSocketIfname:
        args.append(f"--rccl-socket-ifname={so.rcclSocketIfname}")
    if (so.lldpCache or so.keepConfigOnRestart) and so.layer == "L3":
        # keepConfigOnRestart: the cache is what lets the next agent adopt the addresses it finds
        args.append(f"--lldp-cache={ARTIFACT_DIR_CONTAINER}/{LLDP_CACHE_FILE}")
    if so.keepConfigOnRestart:
        args.append("--keep-config")
    if so.disableFirmwareLldp and so.layer == "L3":
        # The originals of what --disable-fw-lldp changes, on the node: with --keep-config they stay
        # changed across restarts and the cleanup Job restores them; without, they outlive an agent
        # that fails and the next clean exit restores them.
        args.append(f"--fw-lldp-state={ARTIFACT_DIR_CONTAINER}/{FW_LLDP_STATE_FILE}")
    if so.railSwitchPattern and so.layer == "L3":
        args.append(f"--rail-switch-pattern={so.railSwitchPattern}")
    if so.minLinkSpeedGbps:
        args.append(f"--min-link-speed-gbps={so.minLinkSpeedGbps}")
    if so.checkPeerMtu is False and so.layer == "L3":
        args.append("--check-peer-mtu=false")
    args.append(f"--status-file={discovery.AGENT_STATUS_FILE}")
    if so.verifyPeers and so.layer == "L3":
        args.append(f"--verify-peers={VERIFY_PEERS_TIMEOUT}")
    if so.rcclEnv:
        args.append("--rccl-env-extra=" + ",".join(f"{k}={v}" for k, v in sorted(so.rcclEnv.items())))
    if so.gpuDirectRdma:
        args.append("--require-gdr=" + {"Any": "any", "PeerMem": "peermem", "DmaBuf": "dmabuf"}[so.gpuDirectRdma])
    return args


def update_amd_scale_out_daemonset(ds: dict, p: T.NetworkClusterPolicy, namespace: str) -> None:
    """updateGaudiScaleOutDaemonSet (:164-204) for amd-so."""
    md = ds.setdefault("metadata", {})
    md["name"] = p.name
    md["namespace"] = namespace
    pod = ds["spec"]["template"]["spec"]
    if p.spec.nodeSelector:
        pod["nodeSelector"] = dict(p.spec.nodeSelector)
    c = pod["containers"][0]
    so = p.spec.amdScaleOut
    if so.image:
        c["image"] = so.image
    if so.pullPolicy:
        c["imagePullPolicy"] = so.pullPolicy
    wanted = set()
    if so.disableNetworkManager:
        add_host_volume(ds, "var-run-dbus", "/var/run/dbus", "/var/run/dbus")
        add_host_volume(ds, "networkmanager", "/etc/NetworkManager", "/etc/NetworkManager")
        wanted |= {"var-run-dbus", "networkmanager"}
    add_host_volume(ds, "rccl-artifacts", ARTIFACT_DIR_HOST, ARTIFACT_DIR_CONTAINER)  # L2 too (rccl.env)
    wanted.add("rccl-artifacts")
    for v in MANAGED_VOLUMES + ("host-lib-modules",):
        if v not in wanted:
            remove_volume(ds, v)
    order_managed_volumes(ds)
    # A policy that switched from host-nic: no driver container, default readiness probe.
    inits = [x for x in pod.get("initContainers", []) if x.get("name") != "nic-driver"]
    if inits:
        pod["initContainers"] = inits
    else:
        pod.pop("initContainers", None)
    probe = c.get("readinessProbe", {}).get("exec")
    if probe:
        probe["command"] = probe["command"][:1] + ["--ready-check", f"--status-file={discovery.AGENT_STATUS_FILE}"]
    # Agent metrics port (hostNetwork: the container port is the node port).
    ports = [x for x in c.get("ports", []) if x.get("name") != "metrics"]
    if so.metricsPort:
        ports.append({"name": "metrics", "containerPort": so.metricsPort, "protocol": "TCP"})
    if ports:
        c["ports"] = ports
    else:
        c.pop("ports", None)
    c["args"] = agent_args(p)


HOST_NIC_LABEL = "amd.feature.node.kubernetes.io/host-nic-ready"
HOST_NIC_LABEL_FILE = "host-nic-readiness.txt"
HOST_NIC_LLDP_CACHE_FILE = "host-nic-lldp-cache"
HOST_NIC_MTU_STATE_FILE = "host-nic-mtu-state"  # --mtu-state: the host NICs' own MTUs
DRIVER_CONTAINER = "nic-driver"


def host_nic_agent_args(p: T.NetworkClusterPolicy) -> List[str]:
    """Agent flags for ``host-nic``: RDMA NIC discovery instead of GPU affinity, its own readiness
    label and file (so it can coexist with an ``amd-so`` policy on the same node)."""
    hn = p.spec.hostNic or T.HostNicSpec()
    args = ["--configure=true", "--keep-running", f"--mode={hn.layer}",
            "--nic-discovery=" + ("none" if hn.interfaces else "rdma"),
            f"--nfd-label-file={HOST_NIC_LABEL_FILE}", f"--nfd-label={HOST_NIC_LABEL}"]
    if p.spec.logLevel > 0:
        args.append(f"--v={p.spec.logLevel}")
    if hn.mtu > 0:
        args.append(f"--mtu={hn.mtu}")
    # The node's own NICs get their MTU back when the agent goes for good: on a clean exit, or
    # (keepConfigOnRestart) from the record the cleanup Job reads.  Always, not only while mtu is
    # set: the agent applies its default MTU otherwise, and a policy that dropped mtu must still
    # let the next agent and the cleanup Job find and restore the record.
    args += ["--restore-mtu", f"--mtu-state={ARTIFACT_DIR_CONTAINER}/{HOST_NIC_MTU_STATE_FILE}"]
    if hn.disableNetworkManager:
        args += ["--disable-networkmanager", "--nm-keyfile-dir=/etc/NetworkManager/conf.d"]
    if hn.layer == "L3":
        args.append(f"--wait={hn.lldpWait or L3_WAIT}")
        if hn.verifyPeers:
            args.append(f"--verify-peers={VERIFY_PEERS_TIMEOUT}")
    elif hn.carrierWait:
        args.append(f"--carrier-wait={hn.carrierWait}")
    if hn.interfaces:
        args.append("--interfaces=" + ",".join(hn.interfaces))
    if hn.nicDrivers:
        args.append("--nic-drivers=" + ",".join(hn.nicDrivers))
    if hn.includeGpuRails and not hn.interfaces:
        args.append("--rdma-include-gpu-rails")
    if hn.checkPeerMtu is False and hn.layer == "L3":
        args.append("--check-peer-mtu=false")
    if hn.keepConfigOnRestart:
        if hn.layer == "L3":  # its own cache beside the scale-out agent's
            args.append(f"--lldp-cache={ARTIFACT_DIR_CONTAINER}/{HOST_NIC_LLDP_CACHE_FILE}")
        args.append("--keep-config")
    args.append(f"--status-file={discovery.AGENT_STATUS_FILE}")
    return args


def update_host_nic_daemonset(ds: dict, p: T.NetworkClusterPolicy, namespace: str) -> None:
    """The ``host-nic`` branch (the reference's "Future work": Host-NIC use + KMD install)."""
    hn = p.spec.hostNic or T.HostNicSpec()
    md = ds.setdefault("metadata", {})
    md["name"] = p.name
    md["namespace"] = namespace
    pod = ds["spec"]["template"]["spec"]
    if p.spec.nodeSelector:
        pod["nodeSelector"] = dict(p.spec.nodeSelector)
    c = pod["containers"][0]
    if hn.image:
        c["image"] = hn.image
    if hn.pullPolicy:
        c["imagePullPolicy"] = hn.pullPolicy
    wanted = set()
    if hn.disableNetworkManager:
        add_host_volume(ds, "var-run-dbus", "/var/run/dbus", "/var/run/dbus")
        add_host_volume(ds, "networkmanager", "/etc/NetworkManager", "/etc/NetworkManager")
        wanted |= {"var-run-dbus", "networkmanager"}
    if (hn.keepConfigOnRestart and hn.layer == "L3") or hn.mtu > 0:  # the LLDP cache / MTU record outlive the Pod
        add_host_volume(ds, "rccl-artifacts", ARTIFACT_DIR_HOST, ARTIFACT_DIR_CONTAINER)
        wanted.add("rccl-artifacts")
    # Optional kernel-driver container: privileged, sees the host's modules, runs to completion
    # before the agent starts (init container), so the NICs exist when discovery runs.
    inits = [x for x in pod.get("initContainers", []) if x.get("name") != DRIVER_CONTAINER]
    if hn.driverImage:
        spec_vols = pod.setdefault("volumes", [])
        if not any(v.get("name") == "host-lib-modules" for v in spec_vols):
            spec_vols.append({"name": "host-lib-modules", "hostPath": {"path": "/lib/modules", "type": "Directory"}})
        wanted.add("host-lib-modules")
        inits.append({"name": DRIVER_CONTAINER, "image": hn.driverImage,
                      "imagePullPolicy": hn.pullPolicy or "IfNotPresent",
                      "securityContext": {"privileged": True},
                      "volumeMounts": [{"name": "host-lib-modules", "mountPath": "/lib/modules"}]})
    if inits:
        pod["initContainers"] = inits
    else:
        pod.pop("initContainers", None)
    for v in MANAGED_VOLUMES + ("host-lib-modules",):
        if v not in wanted:
            remove_volume(ds, v)
    order_managed_volumes(ds)
    probe = c.get("readinessProbe", {}).get("exec")
    if probe:
        probe["command"] = [probe["command"][0], "--ready-check", f"--nfd-label-file={HOST_NIC_LABEL_FILE}",
                            f"--status-file={discovery.AGENT_STATUS_FILE}"]
    c["args"] = host_nic_agent_args(p)


def update_daemonset_for(ds: dict, p: T.NetworkClusterPolicy, namespace: str,
                         hold_off: Optional[List[dict]] = None) -> None:
    """createDaemonSet / updateDaemonSet dispatch on configurationType (:243-265).  Also the
    rolling-update width (spec.maxUnavailable; 1 when unset, like the reference's DaemonSet) and
    the node affinity that holds the agents off nodes an older policy of the type selects."""
    ds["spec"].setdefault("updateStrategy", {"type": "RollingUpdate"}).setdefault("rollingUpdate", {})[
        "maxUnavailable"] = p.spec.maxUnavailable if p.spec.maxUnavailable is not None else 1
    if p.spec.configurationType == T.CONFIG_AMD_SCALE_OUT:
        update_amd_scale_out_daemonset(ds, p, namespace)
    elif p.spec.configurationType == T.CONFIG_HOST_NIC:
        update_host_nic_daemonset(ds, p, namespace)
    else:
        raise ValueError(f"unknown configuration type {p.spec.configurationType!r}")
    # Tainted GPU nodes (amd.com/gpu:NoSchedule, ...): the policy's tolerations, exactly (a
    # toleration removed from the policy leaves the template; the cleanup Job copies this spec).
    pod = ds["spec"]["template"]["spec"]
    if p.spec.tolerations:
        pod["tolerations"] = copy.deepcopy(p.spec.tolerations)
    else:
        pod.pop("tolerations", None)
    if p.spec.priorityClassName:
        pod["priorityClassName"] = p.spec.priorityClassName
    else:
        pod.pop("priorityClassName", None)
    set_hold_off(pod, hold_off)


def status_for(targets: int, ready: int) -> str:
    if targets == 0:
        return STATE_NO_TARGETS
    if ready < targets:
        return STATE_WORKING
    return STATE_ALL_GOOD


def _now_rfc3339() -> str:
    import datetime

    return datetime.datetime.now(datetime.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def _set_condition(conds: List[dict], type_: str, status: str, reason: str, message: str, generation: int,
                   now: str) -> None:
    """meta.SetStatusCondition: lastTransitionTime moves only when the status flips."""
    for c in conds:
        if c["type"] == type_:
            if c.get("status") != status:
                c["lastTransitionTime"] = now
            c.update(status=status, reason=reason, message=message, observedGeneration=generation)
            return
    conds.append({"type": type_, "status": status, "observedGeneration": generation, "lastTransitionTime": now,
                  "reason": reason, "message": message})


def agent_exit_reason(pod: dict, limit: int = 1500) -> Optional[str]:
    """Why the agent container last exited, from the Pod's container status: the agent's own
    one-line "Error: ..." from the termination message (the DaemonSet sets
    FallbackToLogsOnError, so that is the log tail of a failed start), else the exit code."""
    for cs in (pod.get("status", {}) or {}).get("containerStatuses") or []:
        t = (cs.get("state") or {}).get("terminated") or (cs.get("lastState") or {}).get("terminated")
        if not t:
            continue
        lines = [ln.strip() for ln in (t.get("message") or "").splitlines() if ln.strip()]
        fatal = [ln[len("Error: "):] for ln in lines if ln.startswith("Error: ")]
        if fatal:
            return fatal[-1][:limit]
        code = t.get("exitCode")
        if code:
            return f"agent exited with code {code}" + (f" ({t['reason']})" if t.get("reason") not in (None, "Error") else "")
    return None


PROBE_PREFIXES = ("Readiness probe failed: ", "not ready: ")


def probe_reason(events: List[dict], limit: int = 1500) -> Optional[str]:
    """Why the running agent's readiness probe fails: the latest kubelet "Unhealthy" event on its
    Pod carries the probe's output (the agent's per-NIC reason, e.g. "enp30s0np0: link down")."""
    if not events:
        return None
    ev = max(events, key=lambda e: (e.get("lastTimestamp") or e.get("eventTime") or "", int(e.get("count", 0) or 0)))
    msg = (ev.get("message") or "").strip()
    for p in PROBE_PREFIXES:
        if msg.startswith(p):
            msg = msg[len(p):]
    return msg[:limit] or None


# What an agent says while its node is still coming up.  "waiting for carrier": L2, a NIC whose
# optic / switch port is still training its link, within the agent's --carrier-wait.
# "agent starting": probed before the agent wrote its status file (discover --ready-check).
STARTUP_REASONS = ("waiting for LLDP", "not configured yet", "waiting for carrier", "agent starting")


def _starting_up(reason: str) -> bool:
    """Every NIC of the probe's reason is still coming up (no Event for a node that starts)."""
    return all(part.split(": ", 1)[-1] in STARTUP_REASONS for part in reason.split("; "))


def _container_running(pod: dict) -> bool:
    return any("running" in (cs.get("state") or {}) for cs in (pod.get("status") or {}).get("containerStatuses") or [])


# Two policies of one configurationType that select the same node would run two agents there;
# they share the node lock (named after the type's NFD label), so the later one would wait and
# then fail, restarting forever.  Instead a node belongs to the OLDEST live policy of the type
# whose nodeSelector matches it: every newer one's DaemonSet carries a required node-affinity
# term that excludes the nodes the older selectors match, so its agents are never placed there.
# The term is built from the selectors, not from a node list: it does not change when nodes come,
# go or get relabelled (a DaemonSet template change rolls every agent of the policy), only when
# an older policy's selector does.  The newer policy's status names the held-off nodes
# (Degraded/PolicyConflict, a Warning Event); once the older policy goes, the term goes with it
# and the newer policy's agents take those nodes.  (The reference has no guard at all,
# internal/controller/networkconfiguration_controller.go:164-204,313-362.)
CONFLICT_MARK = ": also selected by policy "
# A node-selector term no node matches (no node carries this label): a newer policy whose
# every node an older one selects.
HELD_EVERYWHERE_KEY = "network.amd.com/held-off-by-an-older-policy"
MAX_HOLD_OFF_TERMS = 64  # required terms are ORed: the hold-off expands to at most this many
# While an older selector overlaps, the held-off nodes are read again this often: a node
# relabelled into or out of the overlap moves no Pod of this policy, so no event would.
HELD_OFF_REFRESH_S = 30.0


def hold_off_terms(mine: Dict[str, str], older: List[Dict[str, str]]) -> Optional[List[dict]]:
    """nodeSelectorTerms (ORed) of the nodes ``mine`` (a nodeSelector) selects that no selector in
    ``older`` matches, to AND with ``mine``; None when nothing is held off.

    Not matching {k1: v1, k2: v2} is (k1 NotIn [v1]) OR (k2 NotIn [v2]) (NotIn also matches a node
    without the label).  Over several older selectors that is a conjunction of such clauses,
    expanded here into a disjunction of terms.  A clause whose pairs all sit in ``mine`` already
    excludes every node: nothing is left.  An older selector with a key ``mine`` requires at
    another value is disjoint: no clause.  Raises ValueError past MAX_HOLD_OFF_TERMS."""
    clauses = set()
    for q in older:
        if any(k in mine and mine[k] != v for k, v in q.items()):
            continue  # disjoint selections
        clause = tuple(sorted((k, v) for k, v in q.items() if mine.get(k) != v))
        if not clause:
            return [{"matchExpressions": [{"key": HELD_EVERYWHERE_KEY, "operator": "Exists"}]}]
        clauses.add(clause)
    if not clauses:
        return None
    kept: List[tuple] = []  # absorption: a clause implied by a shorter one adds nothing
    for c in sorted(clauses, key=lambda c: (len(c), c)):
        if not any(set(k) <= set(c) for k in kept):
            kept.append(c)
    terms: List[frozenset] = [frozenset()]
    for c in kept:
        terms = sorted({t | {lit} for t in terms for lit in c}, key=sorted)
        if len(terms) > MAX_HOLD_OFF_TERMS:
            raise ValueError(f"{len(kept)} overlapping older selectors expand to more than {MAX_HOLD_OFF_TERMS} "
                             "node-affinity terms")
    terms = [t for t in terms if not any(o < t for o in terms)]  # a term implied by a smaller one
    out = []
    for t in terms:
        by_key: Dict[str, List[str]] = {}
        for k, v in sorted(t):
            by_key.setdefault(k, []).append(v)
        out.append({"matchExpressions": [{"key": k, "operator": "NotIn", "values": vs} for k, vs in by_key.items()]})
    return out


def set_hold_off(pod: dict, terms: Optional[List[dict]]) -> None:
    """The agent Pod template's required node affinity: the hold-off terms, or none.  (The policy
    has no affinity field of its own, so the operator owns this one.)"""
    if terms:
        pod["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
            "nodeSelectorTerms": copy.deepcopy(terms)}}}
    else:
        pod.pop("affinity", None)


def held_off_error(ctype: str, nodes: List[str], more: bool, other: str) -> str:
    """status.errors entry for the nodes this policy is kept off because ``other`` (older, same
    configurationType) selects them too."""
    shown = ", ".join(nodes) + (" and more" if more else "")
    return (f"{shown}{CONFLICT_MARK}{other} ({ctype} too, created earlier): one agent per node and type "
            f"configures the NICs, so this policy's agents are held off these nodes while {other} selects them; "
            f"narrow a nodeSelector")


def policy_conditions(current: List[dict], targets: int, ready: int, errors: List[str], generation: int,
                      now: Optional[str] = None) -> List[dict]:
    """The policy's Ready / Degraded conditions (additive to the reference's state string,
    which stays as it is for parity, reference networkconfiguration_controller.go:289-295)."""
    now = now or _now_rfc3339()
    conds = [dict(c) for c in current if c.get("type") in (COND_READY, COND_DEGRADED)]
    if targets == 0:
        _set_condition(conds, COND_READY, "False", "NoTargets", "no node matches the nodeSelector", generation, now)
    elif ready < targets:
        _set_condition(conds, COND_READY, "False", "NodesNotReady", f"{ready}/{targets} nodes configured",
                       generation, now)
    else:
        _set_condition(conds, COND_READY, "True", "AllNodesReady", f"{ready}/{targets} nodes configured",
                       generation, now)
    if any(e.startswith("dependency missing") for e in errors):
        _set_condition(conds, COND_DEGRADED, "True", "DependencyMissing", "; ".join(errors)[:1024], generation, now)
    elif any(CONFLICT_MARK in e for e in errors):
        _set_condition(conds, COND_DEGRADED, "True", "PolicyConflict", "; ".join(errors)[:1024], generation, now)
    elif errors:
        _set_condition(conds, COND_DEGRADED, "True", "AgentErrors", "; ".join(errors)[:1024], generation, now)
    else:
        _set_condition(conds, COND_DEGRADED, "False", "AsExpected", "", generation, now)
    conds.sort(key=lambda c: c["type"] != COND_READY)
    return conds


# ---------------------------------------------------------------------------------------------
# Fabric validation Jobs (amdScaleOut.validation, MI355X addition)
# ---------------------------------------------------------------------------------------------
AGENT_EPOCH_ANN = "amd.com/agent-ready-since"  # the agent readiness the Job validates
ATTEMPT_ANN = "amd.com/attempt"                # re-runs of a Job the kubelet did not admit
# Pod status reasons of a validation Pod the kubelet refused to run (it never validated
# anything): the GPUs are allocated to workloads (OutOfamd.com/gpu), a device plugin error
# (UnexpectedAdmissionError), the node no longer fits, or it was evicted / preempted.
NOT_ADMITTED_REASONS = ("OutOf", "UnexpectedAdmissionError", "NodeAffinity", "NodeName", "NodePorts", "Evicted",
                        "Preempting", "Terminated", "Shutdown")
NOT_ADMITTED_RETRY_S = (30.0, 600.0)  # back-off base and cap of re-running a Job that was not admitted


def validation_job_name(policy: str, node: str, generation: int, epoch: str = "", attempt: int = 0) -> str:
    """DNS-1123, <= 63 characters, unique per (policy, node, policy generation, agent readiness,
    attempt): a re-run never collides with the Job it replaces while that one is being deleted."""
    import hashlib

    h = hashlib.sha256(f"{policy}/{node}".encode()).hexdigest()[:10]
    name = f"{policy[:30].rstrip('-')}-val-{h}-g{generation}"
    if epoch or attempt:
        name += "-" + hashlib.sha256(f"{epoch}/{attempt}".encode()).hexdigest()[:6]
    return name


def agent_epoch(pod: dict) -> str:
    """When the node's agent last became Ready: the Pod uid and its Ready condition's
    lastTransitionTime.  A new value (agent restarted, fault cleared, Pod replaced) means the
    node's fabric may differ from what an earlier validation saw."""
    ready = next((c for c in (pod.get("status") or {}).get("conditions") or [] if c.get("type") == "Ready"), {})
    return f"{pod.get('metadata', {}).get('uid', '')}@{ready.get('lastTransitionTime', '')}"


def job_not_admitted(pods: List[dict]) -> Optional[str]:
    """The kubelet's reason when it refused the Job's Pod (not a validation verdict), else None."""
    for pod in pods:
        st = pod.get("status") or {}
        reason = st.get("reason") or ""
        if st.get("phase") == "Failed" and reason.startswith(NOT_ADMITTED_REASONS):
            msg = st.get("message") or ""
            return f"{reason}: {msg}"[:200] if msg else reason
    return None


# keepConfigOnRestart: agents leave their configuration in place when they exit, so the operator
# owes each node it ever configured a cleanup (the agent in --cleanup mode, as a Job pinned to the
# node) when the policy is deleted (finalizer) or the node leaves the policy (its agent Pod has
# been gone for KEPT_ORPHAN_GRACE_S: longer than any DaemonSet roll, drain or reboot).
FINALIZER = "amd.com/node-cleanup"
CLEANUP_APP = "amd-network-cleanup"
KEPT_ORPHAN_GRACE_S = 600.0
CLEANUP_TIMEOUT_S = 600.0  # a cleanup Job not finished by then (node gone, image missing) is given up
CLEANUP_POLL_S = 2.0       # cleanup Jobs are not watched: poll while some are running
CLEANUP_CREATE_CONCURRENCY = 32
CLEANUP_LIST_PAGE = 500


def keeps_config(p: T.NetworkClusterPolicy) -> bool:
    if p.spec.configurationType == T.CONFIG_AMD_SCALE_OUT:
        return p.spec.amdScaleOut.keepConfigOnRestart
    return p.spec.configurationType == T.CONFIG_HOST_NIC and bool(p.spec.hostNic and p.spec.hostNic.keepConfigOnRestart)


def disables_nm(p: T.NetworkClusterPolicy) -> bool:
    if p.spec.configurationType == T.CONFIG_AMD_SCALE_OUT:
        return p.spec.amdScaleOut.disableNetworkManager
    return p.spec.configurationType == T.CONFIG_HOST_NIC and bool(p.spec.hostNic and p.spec.hostNic.disableNetworkManager)


def needs_node_cleanup(p: T.NetworkClusterPolicy) -> bool:
    """The agents leave something on the node that only a cleanup Job removes: the data plane
    (keepConfigOnRestart) or NetworkManager's hands off the NICs (disableNetworkManager: kept
    across agent restarts on purpose, handed back once the policy no longer covers the node)."""
    return keeps_config(p) or disables_nm(p)


def same_nics(p: T.NetworkClusterPolicy, q: T.NetworkClusterPolicy) -> bool:
    """Whether q's agents take exactly the NICs p's agents configured on a node, and leave
    NetworkManager as p's would (so q's agent, replacing p's config there, settles p's debt)."""
    if p.spec.configurationType != q.spec.configurationType or (disables_nm(p) and not disables_nm(q)):
        return False
    if p.spec.configurationType == T.CONFIG_AMD_SCALE_OUT:
        a, b = p.spec.amdScaleOut, q.spec.amdScaleOut
        return (a.interfaces, a.nicDrivers) == (b.interfaces, b.nicDrivers)
    a, b = p.spec.hostNic, q.spec.hostNic
    return bool(a and b) and (a.interfaces, a.nicDrivers, a.includeGpuRails) == (b.interfaces, b.nicDrivers,
                                                                                 b.includeGpuRails)


def cleanup_job_name(policy: str, node: str) -> str:
    import hashlib

    return f"{policy[:30].rstrip('-')}-clean-{hashlib.sha256(f'{policy}/{node}'.encode()).hexdigest()[:10]}"


def cleanup_job(p: T.NetworkClusterPolicy, node: str, namespace: str) -> dict:
    """The agent's own Pod template (image, privileges, host paths, discovery flags) run once on
    ``node`` with ``--cleanup``: it removes what --keep-config agents left there (addresses of
    the NICs it discovers, its tagged rail rules and routes, label, artifacts, LLDP cache)."""
    ds = discovery.discovery_daemonset()
    update_daemonset_for(ds, p, namespace)
    pod = copy.deepcopy(ds["spec"]["template"]["spec"])
    pod.pop("initContainers", None)  # the NIC driver is loaded already, or there is nothing to clean
    pod["restartPolicy"] = "Never"
    pod["nodeName"] = node
    pod.pop("nodeSelector", None)  # the node may have left the policy's selector
    pod.pop("affinity", None)      # ... or be held off now
    c = pod["containers"][0]
    for k in ("readinessProbe", "livenessProbe", "startupProbe"):
        c.pop(k, None)
    c["args"] = [a for a in c.get("args") or [] if a not in ("--keep-running", "--keep-config")] + \
        ["--cleanup", f"--nfd-features-dir={discovery.LABEL_FEATURES_DIR}"] + (["--nm-restore"] if disables_nm(p) else [])
    labels = {"app": CLEANUP_APP, "amd.com/policy": p.name[:63]}
    return {
        "apiVersion": "batch/v1", "kind": "Job",
        "metadata": {"name": cleanup_job_name(p.name, node), "namespace": namespace, "labels": dict(labels),
                     "annotations": {"amd.com/node": node}},
        "spec": {"backoffLimit": 2, "activeDeadlineSeconds": int(CLEANUP_TIMEOUT_S),
                 "template": {"metadata": {"labels": dict(labels)}, "spec": pod}},
    }


def _rfc3339_to_unix(ts: str) -> Optional[float]:
    import datetime

    try:
        return datetime.datetime.strptime(ts, "%Y-%m-%dT%H:%M:%SZ").replace(tzinfo=datetime.timezone.utc).timestamp()
    except (TypeError, ValueError):
        return None


def _job_finished_at(job: dict) -> Optional[float]:
    import datetime

    for c in (job.get("status") or {}).get("conditions") or []:
        if c.get("type") in ("Failed", "Complete") and c.get("status") == "True" and c.get("lastTransitionTime"):
            try:
                return datetime.datetime.strptime(c["lastTransitionTime"], "%Y-%m-%dT%H:%M:%SZ").replace(
                    tzinfo=datetime.timezone.utc).timestamp()
            except ValueError:
                return None
    return None


def validation_job(p: T.NetworkClusterPolicy, node: str, generation: int, namespace: str, epoch: str = "",
                   attempt: int = 0) -> dict:
    """``python -m network_operator_amd.validate`` on one node, all its GPUs, the agent's artifacts
    read-only, the label through NFD (config/validation/validation-job.yaml, pinned to a node)."""
    v = p.spec.amdScaleOut.validation or T.ValidationSpec()
    gpus = v.gpus or 8
    args = [f"--gpus={gpus}", f"--min-busbw={v.minBusbw}", f"--min-link={v.minLink}",
            f"--nfd-features-dir={discovery.LABEL_FEATURES_DIR}", f"--artifact-dir={ARTIFACT_DIR_HOST}"]
    labels = {"app": VALIDATION_APP, "amd.com/policy": p.name[:63]}
    return {
        "apiVersion": "batch/v1", "kind": "Job",
        "metadata": {"name": validation_job_name(p.name, node, generation, epoch, attempt), "namespace": namespace,
                     "labels": dict(labels),
                     "annotations": {"amd.com/node": node, "amd.com/policy-generation": str(generation),
                                     AGENT_EPOCH_ANN: epoch, ATTEMPT_ANN: str(attempt)}},
        "spec": {
            "backoffLimit": 0,  # kept (no TTL) while the policy generation is current: its result is the status
            "template": {
                "metadata": {"labels": dict(labels)},
                "spec": {
                    "restartPolicy": "Never",
                    "nodeName": node,
                    **({"tolerations": copy.deepcopy(p.spec.tolerations)} if p.spec.tolerations else {}),
                    "containers": [{
                        "name": "validate",
                        "image": v.image or T.DEFAULT_VALIDATION_IMAGE,
                        "imagePullPolicy": p.spec.amdScaleOut.pullPolicy or "IfNotPresent",
                        "command": ["python3", "-m", "network_operator_amd.validate"],
                        "args": args,
                        "resources": {"limits": {"amd.com/gpu": gpus}},
                        "volumeMounts": [
                            {"name": "nfd-features", "mountPath": discovery.LABEL_FEATURES_DIR},
                            {"name": "rccl-artifacts", "mountPath": ARTIFACT_DIR_HOST, "readOnly": True},
                        ],
                    }],
                    "volumes": [
                        {"name": "nfd-features",
                         "hostPath": {"path": discovery.LABEL_FEATURES_DIR, "type": "DirectoryOrCreate"}},
                        {"name": "rccl-artifacts", "hostPath": {"path": ARTIFACT_DIR_HOST, "type": "DirectoryOrCreate"}},
                    ],
                },
            },
        },
    }


def job_outcome(job: dict) -> str:
    """"succeeded", "failed" or "running"."""
    st = job.get("status") or {}
    if int(st.get("succeeded", 0) or 0) > 0:
        return "succeeded"
    if int(st.get("failed", 0) or 0) > 0:
        return "failed"
    for c in st.get("conditions") or []:
        if c.get("status") == "True" and c.get("type") in ("Complete", "Failed"):
            return "succeeded" if c["type"] == "Complete" else "failed"
    return "running"


class EventRecorder:
    """Best-effort core/v1 Events on the policy (failures are only logged)."""

    def __init__(self, client: ApiClient, namespace: str, component: str = "amd-network-operator"):
        self.client, self.namespace, self.component = client, namespace, component
        self.sent = 0

    async def event(self, obj: dict, type_: str, reason: str, message: str) -> None:
        md = obj.get("metadata", {})
        body = {
            "apiVersion": "v1", "kind": "Event",
            "metadata": {"generateName": f"{md.get('name', 'obj')}.", "namespace": self.namespace},
            "involvedObject": {"apiVersion": obj.get("apiVersion"), "kind": obj.get("kind"), "name": md.get("name"),
                               "uid": md.get("uid")},
            "type": type_, "reason": reason, "message": message, "source": {"component": self.component},
            "count": 1,
        }
        try:
            await self.client.create(kube.EVENTS, body, namespace=self.namespace)
            self.sent += 1
        except Exception as e:  # events must never fail a reconcile
            log.debug("event not recorded: %s", e)


class NetworkClusterPolicyReconciler:
    def __init__(self, client: ApiClient, namespace: str, is_openshift: bool,
                 get_policy: Callable[[str], Optional[dict]], list_owned: Callable[[str], List[dict]],
                 recorder: Optional[EventRecorder] = None,
                 list_pods: Optional[Callable[[str], List[dict]]] = None,
                 list_jobs: Optional[Callable[[str], List[dict]]] = None,
                 list_job_pods: Optional[Callable[[str], List[dict]]] = None,
                 clock: Callable[[], float] = time.time,
                 list_probe_events: Optional[Callable[[str], List[dict]]] = None,
                 list_policies: Optional[Callable[[], List[dict]]] = None):
        self.client = client
        self.namespace = namespace
        self.is_openshift = is_openshift
        # Cluster add-ons the policy cannot work without (set by the manager's dependency check;
        # the reference only lists them in its README).
        self.missing_dependencies: List[str] = []
        self._get_policy = get_policy
        self._list_owned = list_owned
        self._list_pods = list_pods
        self._list_jobs = list_jobs  # validation Jobs of a policy (by its name)
        self._list_job_pods = list_job_pods  # the Pods of a validation Job (by its name)
        self._list_probe_events = list_probe_events  # kubelet "Unhealthy" events of an agent Pod (by its name)
        self._list_policies = list_policies  # every policy (the informer cache): conflicting selections
        self._clock = clock
        self.recorder = recorder
        # keepConfigOnRestart: (policy, node) -> when the node's agent Pod was first seen missing
        self._missing_since: dict = {}
        self.on_cleanup: Optional[Callable[[str, str], None]] = None  # (policy, outcome): metrics
        self._cleanups_reported: set = set()  # finished cleanup Jobs already counted / reported
        self._cleanup_jobs_exist: set = set()  # policies with cleanup Jobs left to finish or delete

    def _node_errors(self, ds_name: str, limit: int = 16) -> Tuple[List[str], Set[str], Set[str]]:
        """Per-node agent problems from the agent Pods' Ready condition (the reference indexes
        Pods by owner but never reads them and always reports ``errors: []``).  Also returns
        which entries are a running node that degraded (its probe, not an exit) and which are a
        node still starting up (a start-up reason, or a running agent not probed yet): those
        do not make the policy Degraded.  Returned, not kept on the reconciler: two workers
        reconcile two policies at once."""
        degraded: Set[str] = set()
        starting: Set[str] = set()
        if self._list_pods is None:
            return [], degraded, starting
        errs = []
        for pod in sorted(self._list_pods(ds_name), key=lambda p: p.get("spec", {}).get("nodeName", "")):
            conds = {c.get("type"): c for c in (pod.get("status", {}) or {}).get("conditions", []) or []}
            ready = conds.get("Ready", {})
            if ready.get("status") == "True":
                continue
            node = pod.get("spec", {}).get("nodeName") or pod["metadata"]["name"]
            err = f"{node}: scale-out not ready ({ready.get('reason') or pod.get('status', {}).get('phase', 'Pending')})"
            # A running agent that withdrew its label says why through its probe (kubelet event);
            # an agent that exited, through its termination message.
            running = _container_running(pod)
            probed = probe_reason(self._list_probe_events(pod["metadata"]["name"])) \
                if self._list_probe_events is not None and (running or not agent_exit_reason(pod)) \
                else None
            why = probed or agent_exit_reason(pod)
            entry = f"{err}: {why}" if why else err
            if probed and not _starting_up(probed):
                degraded.add(entry)
            elif (probed and _starting_up(probed)) or (why is None and running):
                starting.add(entry)
            errs.append(entry)
        if len(errs) > limit:
            errs = errs[:limit] + [f"... and {len(errs) - limit} more"]
        return errs, degraded, starting

    async def _hold_off(self, p: T.NetworkClusterPolicy) -> Tuple[Optional[List[dict]], List[str], bool]:
        """(node-affinity terms that keep this policy's agents off the nodes older live policies of
        its type select, status.errors naming those nodes, whether an older selector overlaps).  Older: earlier creationTimestamp, the
        name breaking a tie (the timestamps have seconds).  The nodes are read with one LIST per
        overlapping older policy, by the two selectors together, three names at most."""
        if self._list_policies is None:
            return None, [], False
        me = (p.metadata.get("creationTimestamp") or "", p.name)
        older: Dict[str, Dict[str, str]] = {}
        for q in self._list_policies():
            md = q.get("metadata") or {}
            if md.get("name") == p.name or md.get("deletionTimestamp") or \
                    (md.get("creationTimestamp") or "", md.get("name", "")) > me:
                continue
            if (q.get("spec") or {}).get("configurationType", "") != p.spec.configurationType:
                continue
            older[md["name"]] = dict((q.get("spec") or {}).get("nodeSelector") or {})
        mine = dict(p.spec.nodeSelector)
        errors: List[str] = []
        try:
            terms = hold_off_terms(mine, list(older.values()))
        except ValueError as e:
            terms = None
            errors.append(f"shared nodes{CONFLICT_MARK}{', '.join(sorted(older))} ({p.spec.configurationType} too, "
                          f"created earlier) are not held off: {e}; this policy's agents there wait for the node lock "
                          f"and fail; narrow a nodeSelector")
        overlapping = False
        for other in sorted(older):
            sel = older[other]
            if any(k in mine and mine[k] != v for k, v in sel.items()):
                continue
            overlapping = True
            both = ",".join(f"{k}={v}" for k, v in sorted({**sel, **mine}.items()))
            try:
                lst = await self.client.list(kube.NODES, label_selector=both or None, limit=3)
            except ApiError as e:
                log.warning("unable to list the nodes %s shares with %s: %s", p.name, other, e)
                continue
            names = sorted(n["metadata"]["name"] for n in lst.get("items") or [])
            if names:
                errors.append(held_off_error(p.spec.configurationType, names,
                                             bool((lst.get("metadata") or {}).get("continue")), other))
        return terms, errors, overlapping

    async def _delete_job(self, j: dict) -> None:
        try:
            await self.client.delete(kube.JOBS, j["metadata"]["name"], self.namespace)
        except ApiError as e:
            if not is_not_found(e):
                raise

    async def _cleanup_jobs(self, policy: str) -> dict:
        """node -> the policy's cleanup Job, reduced to what is used (name, creation time,
        status), read in pages: a thousand-node policy's Jobs in one LIST would be megabytes
        of JSON parsed at once, against the operator's 128 MiB limit."""
        out, cont = {}, ""
        while True:
            lst = await self.client.list(kube.JOBS, self.namespace, limit=CLEANUP_LIST_PAGE, continue_=cont,
                                         label_selector=f"app={CLEANUP_APP},amd.com/policy={policy[:63]}")
            for j in lst.get("items") or []:
                md = j["metadata"]
                out[(md.get("annotations") or {}).get("amd.com/node", "")] = {
                    "metadata": {"name": md["name"], "creationTimestamp": md.get("creationTimestamp", "")},
                    "status": j.get("status") or {}}
            cont = (lst.get("metadata") or {}).get("continue") or ""
            if not cont:
                return out

    async def _run_cleanups(self, raw: dict, p: T.NetworkClusterPolicy, nodes: List[str]) -> List[str]:
        """Cleanup Jobs for ``nodes``: created when missing; a node whose Job finished (or ran
        past CLEANUP_TIMEOUT_S) is done.  Returns the nodes still in progress.  A finished Job is
        kept until a later pass finds its node no longer asked for, i.e. until the caller has
        recorded the node as done: deleting it at once would make the next pass, reading a
        status written before, take the node for one without a Job and clean it again."""
        jobs = await self._cleanup_jobs(p.name)
        now = self._clock()
        want = set(nodes)
        stale = [j for node, j in jobs.items() if node not in want]
        pending = [node for node in nodes if node not in jobs]
        if pending:
            # One template for all of them (only the node differs); CLEANUP_CREATE_CONCURRENCY
            # creates in flight, so a thousand-node policy is cleaned in seconds, not minutes.
            template = cleanup_job(p, "", self.namespace)
            if not raw["metadata"].get("deletionTimestamp"):
                # Owned, so the garbage collector removes what is left with the policy.  Not once
                # the policy is being deleted: under foreground deletion the collector deletes
                # every new dependent, a cleanup Job mid-run included (_finalize deletes these).
                set_controller_reference(raw, template)
            sem = asyncio.Semaphore(CLEANUP_CREATE_CONCURRENCY)

            async def create(node: str) -> None:
                async with sem:  # built inside: at most CLEANUP_CREATE_CONCURRENCY bodies exist at once
                    job = copy.deepcopy(template)
                    job["metadata"]["name"] = cleanup_job_name(p.name, node)
                    job["metadata"]["annotations"]["amd.com/node"] = node
                    job["spec"]["template"]["spec"]["nodeName"] = node
                    try:
                        await self.client.create(kube.JOBS, job, namespace=self.namespace)
                    except ApiError as e:
                        if not is_already_exists(e):
                            raise
            await asyncio.gather(*(create(n) for n in pending))
            log.info("Created %d node cleanup Job(s) for policy %s", len(pending), p.name)
        done = 0
        for node in nodes:
            j = jobs.get(node)
            if j is None:
                continue
            outcome = job_outcome(j)
            created = _rfc3339_to_unix(j["metadata"].get("creationTimestamp", "")) or now
            if outcome == "running" and now - created < CLEANUP_TIMEOUT_S:
                pending.append(node)
                continue
            done += 1
            if j["metadata"]["name"] in self._cleanups_reported:
                continue
            self._cleanups_reported.add(j["metadata"]["name"])
            if self.on_cleanup is not None:
                self.on_cleanup(p.name, "timed_out" if outcome == "running" else outcome)
            if outcome != "succeeded":
                why = "timed out" if outcome == "running" else "failed"
                await self._event(raw, "Warning", "NodeCleanupFailed",
                                  f"{node}: cleanup Job {j['metadata']['name']} {why}; addresses and routes the agent "
                                  "left may remain (run the agent with --cleanup on the node)")
        if done:
            log.info("Policy %s: %d node cleanup(s) finished, %d in progress", p.name, done, len(pending))
        if stale:
            sem = asyncio.Semaphore(CLEANUP_CREATE_CONCURRENCY)

            async def delete(j: dict) -> None:
                async with sem:
                    await self._delete_job(j)
                self._cleanups_reported.discard(j["metadata"]["name"])
            await asyncio.gather(*(delete(j) for j in stale))
        if len(jobs) - len(stale) + (len(nodes) - len([n for n in nodes if n in jobs])):
            self._cleanup_jobs_exist.add(p.name)
        else:
            self._cleanup_jobs_exist.discard(p.name)
        return pending

    def _taken_over(self, p: T.NetworkClusterPolicy) -> Dict[str, str]:
        """node -> another live policy of p's type whose agent runs there and takes the same NICs
        (same_nics): it holds the node lock and replaces whatever p's agents left, so p owes that
        node no cleanup Job (which would only wait for that lock and fail)."""
        if self._list_policies is None or self._list_pods is None:
            return {}
        out: Dict[str, str] = {}
        for q in self._list_policies():
            md = q.get("metadata") or {}
            if md.get("name") == p.name or md.get("deletionTimestamp"):
                continue
            try:
                qp = T.NetworkClusterPolicy.from_dict(q)
            except Exception:
                continue
            if not same_nics(p, qp):
                continue
            for pod in self._list_pods(md["name"]):
                node = (pod.get("spec") or {}).get("nodeName")
                if node:
                    out.setdefault(node, md["name"])
        return out

    async def _kept_nodes(self, raw: dict, p: T.NetworkClusterPolicy, ds: dict) -> tuple:
        """keepConfigOnRestart / disableNetworkManager bookkeeping: (status.keptNodes,
        requeue_after).  A node joins when an agent Pod runs there (ready or not: an agent that
        failed half-way may have configured some NICs); it leaves after its cleanup Job, which runs
        once its agent Pod has been gone for KEPT_ORPHAN_GRACE_S."""
        cur = list(p.status.keptNodes)
        if not needs_node_cleanup(p) and not cur:
            return [], 0.0
        pods = self._list_pods(ds["metadata"]["name"]) if self._list_pods is not None else []
        with_pod = {pod.get("spec", {}).get("nodeName", "") for pod in pods}
        kept = set(cur) | ((with_pod - {""}) if needs_node_cleanup(p) else set())
        now = self._clock()
        due, requeue_after = [], 0.0
        taken = self._taken_over(p) if kept - with_pod else {}
        for node in sorted(kept):
            key = (p.name, node)
            if node in with_pod:
                self._missing_since.pop(key, None)
                continue
            if node in taken:  # handed over (e.g. an older policy of the type holds it now)
                log.info("Policy %s: node %s is taken over by policy %s; no cleanup owed", p.name, node, taken[node])
                kept.discard(node)
                self._missing_since.pop(key, None)
                continue
            left = self._missing_since.setdefault(key, now) + KEPT_ORPHAN_GRACE_S - now
            if left <= 0:
                due.append(node)
            else:
                requeue_after = min(requeue_after, left) if requeue_after else left
        if due or p.name in self._cleanup_jobs_exist:  # (finished Jobs of done nodes are deleted here)
            pending = set(await self._run_cleanups(raw, p, due))
            for node in due:
                if node not in pending:
                    kept.discard(node)
                    self._missing_since.pop((p.name, node), None)
            if pending:
                requeue_after = min(requeue_after, CLEANUP_POLL_S) if requeue_after else CLEANUP_POLL_S
        return sorted(kept), requeue_after

    async def _finalize(self, raw: dict, p: T.NetworkClusterPolicy) -> Result:
        """The policy is being deleted and carries FINALIZER: stop the agents (delete the
        DaemonSet and wait for its Pods to go), clean every kept node, then release the policy."""
        fins = list(raw["metadata"].get("finalizers") or [])
        if FINALIZER not in fins:
            return Result()
        owned = self._list_owned(p.name)
        if owned and self._list_pods is not None:
            # Every node with an agent Pod now owes a cleanup, whether or not the status has
            # recorded it yet: record them before the Pods (the only other trace) go.
            nodes = {pod.get("spec", {}).get("nodeName", "") for pod in self._list_pods(owned[0]["metadata"]["name"])}
            kept = sorted((nodes - {""}) | set(p.status.keptNodes))
            if kept != sorted(p.status.keptNodes):
                body = copy.deepcopy(raw)
                body["status"] = dict(raw.get("status") or {}, keptNodes=kept)
                try:
                    await self.client.replace_status(kube.NETWORKCLUSTERPOLICIES, body)
                except ApiError as e:
                    if is_conflict(e):
                        return Result(requeue=True)
                    if is_not_found(e):
                        return Result()
                    raise
                return Result(requeue=True)  # continue from the stored status
        for ds in owned:
            try:
                await self.client.delete(kube.DAEMONSETS, ds["metadata"]["name"], self.namespace)
                log.info("Policy %s is being deleted: removed DaemonSet %s", p.name, ds["metadata"]["name"])
            except ApiError as e:
                if not is_not_found(e):
                    raise
        if self._list_pods is not None and self._list_pods(p.name):
            return Result(requeue_after=1.0)  # agents still exiting: a cleanup must not race them
        taken = self._taken_over(p)
        pending = await self._run_cleanups(raw, p, [n for n in p.status.keptNodes if n not in taken])
        if pending:
            if sorted(pending) != sorted(p.status.keptNodes):
                # Nodes whose cleanup finished leave the list now; the next pass deletes their
                # Jobs (see _run_cleanups) instead of taking them for nodes without a Job.
                body = copy.deepcopy(raw)
                body["status"] = dict(raw.get("status") or {}, keptNodes=sorted(pending))
                try:
                    await self.client.replace_status(kube.NETWORKCLUSTERPOLICIES, body)
                except ApiError as e:
                    if not (is_conflict(e) or is_not_found(e)):
                        raise
            return Result(requeue_after=CLEANUP_POLL_S)
        if p.status.keptNodes:
            # Every node is clean: record that before the Jobs go (a pass reading keptNodes with
            # no Jobs would clean the nodes again), then delete them on the next pass.
            body = copy.deepcopy(raw)
            body["status"] = dict(raw.get("status") or {}, keptNodes=[])
            try:
                await self.client.replace_status(kube.NETWORKCLUSTERPOLICIES, body)
            except ApiError as e:
                if is_not_found(e):
                    return Result()
                if not is_conflict(e):
                    raise
            return Result(requeue=True)
        # The finished Jobs: those created during the deletion have no owner to take them along.
        await self._run_cleanups(raw, p, [])
        body = copy.deepcopy(raw)
        body["metadata"]["finalizers"] = [f for f in fins if f != FINALIZER]
        try:
            await self.client.replace(kube.NETWORKCLUSTERPOLICIES, body)
        except ApiError as e:
            if is_conflict(e):
                return Result(requeue=True)
            if not is_not_found(e):
                raise
        for k in [k for k in self._missing_since if k[0] == p.name]:
            del self._missing_since[k]
        self._cleanup_jobs_exist.discard(p.name)
        prefix = cleanup_job_name(p.name, "")[:-10]
        self._cleanups_reported = {n for n in self._cleanups_reported if not n.startswith(prefix)}
        log.info("Policy %s: every node cleaned up, finalizer removed", p.name)
        return Result()

    async def _reconcile_validation(self, raw: dict, p: T.NetworkClusterPolicy, ds: dict, generation: int,
                                    errors: List[str]) -> Optional[tuple]:
        """One validation Job per node whose agent is ready, for the policy's current generation
        and the agent's current readiness (``agent_epoch``): a Job that validated an earlier
        readiness of the node (agent restarted, fault cleared, Pod replaced) is replaced, so a
        failure is never stuck until the next spec change.  A Job whose Pod the kubelet refused
        (GPUs allocated to workloads, device-plugin error) is not a verdict: it is re-created
        after a back-off (``NOT_ADMITTED_RETRY_S``) and reported as not admitted.  Jobs of older
        generations are removed.  Returns ((status, reason, message), requeue_after) or None
        when validation is off; failed nodes are added to `errors`."""
        v = p.spec.amdScaleOut.validation
        if self._list_jobs is None or self._list_pods is None:
            return None
        enabled = p.spec.configurationType == T.CONFIG_AMD_SCALE_OUT and v is not None and v.enabled
        ready_pods = {pod.get("spec", {}).get("nodeName", ""): pod for pod in self._list_pods(ds["metadata"]["name"])
                      if any(c.get("type") == "Ready" and c.get("status") == "True"
                             for c in (pod.get("status") or {}).get("conditions") or [])}
        ready_pods.pop("", None)
        jobs = {}
        for j in self._list_jobs(p.name):
            ann = j["metadata"].get("annotations") or {}
            node = ann.get("amd.com/node", "")
            if not enabled or ann.get("amd.com/policy-generation") != str(generation):
                await self._delete_job(j)  # a result for a spec that no longer exists
                continue
            if node in ready_pods and ann.get(AGENT_EPOCH_ANN, "") != agent_epoch(ready_pods[node]) \
                    and job_outcome(j) != "running":  # a running one finishes first: no kill/restart loop on flaps
                log.info("Agent on %s became ready again since validation Job %s: validating again", node,
                         j["metadata"]["name"])
                await self._delete_job(j)
                continue
            if node in jobs:  # keep the newest attempt
                if int(ann.get(ATTEMPT_ANN, 0) or 0) <= int((jobs[node]["metadata"].get("annotations") or {})
                                                             .get(ATTEMPT_ANN, 0) or 0):
                    continue
            jobs[node] = j
        if not enabled:
            return None
        ready_nodes = sorted(ready_pods)
        requeue_after = 0.0
        not_admitted = {}
        now = self._clock()
        to_create = []
        for node in ready_nodes:
            j = jobs.get(node)
            attempt = 0
            if j is not None and job_outcome(j) == "failed" and self._list_job_pods is not None:
                why = job_not_admitted(self._list_job_pods(j["metadata"]["name"]))
                if why:
                    attempt = int((j["metadata"].get("annotations") or {}).get(ATTEMPT_ANN, 0) or 0)
                    base, cap = NOT_ADMITTED_RETRY_S
                    wait = min(base * 2 ** attempt, cap)
                    left = (_job_finished_at(j) or now) + wait - now
                    if left > 0:
                        not_admitted[node] = f"{why}; retrying in {int(left + 0.999)}s"
                        requeue_after = min(requeue_after, left) if requeue_after else left
                        continue
                    log.info("Validation Job %s on %s was not admitted (%s): re-creating it", j["metadata"]["name"],
                             node, why)
                    await self._delete_job(j)
                    del jobs[node]
                    attempt += 1
            if node not in jobs:
                to_create.append((node, attempt))
        if to_create:
            # CLEANUP_CREATE_CONCURRENCY creates in flight: a cluster that comes up at once gets
            # its thousands of validation Jobs in seconds.
            sem = asyncio.Semaphore(CLEANUP_CREATE_CONCURRENCY)

            async def create(node: str, attempt: int) -> None:
                async with sem:
                    job = validation_job(p, node, generation, self.namespace, agent_epoch(ready_pods[node]), attempt)
                    set_controller_reference(raw, job)
                    try:
                        await self.client.create(kube.JOBS, job, namespace=self.namespace)
                        log.debug("Created fabric validation Job %s for node %s", job["metadata"]["name"], node)
                    except ApiError as e:
                        if not is_already_exists(e):
                            raise
            await asyncio.gather(*(create(n, a) for n, a in to_create))
            log.info("Created %d fabric validation Job(s) for policy %s", len(to_create), p.name)
        # Judged over the nodes ready now: a node that left keeps its Job (and result) until the
        # next generation, but no longer counts either way.
        outcome = {n: job_outcome(jobs[n]) for n in ready_nodes if n in jobs and n not in not_admitted}
        failed = sorted(n for n, o in outcome.items() if o == "failed")
        passed = sum(1 for o in outcome.values() if o == "succeeded")
        errors += [f"{n}: fabric validation failed" for n in failed]
        if failed:
            return ("False", "ValidationFailed", f"{len(failed)} node(s) failed: {', '.join(failed)[:900]}"), requeue_after
        if ready_nodes and passed >= len(ready_nodes):
            return ("True", "AllNodesValidated", f"{passed}/{len(ready_nodes)} nodes validated"), requeue_after
        if not_admitted:
            msg = "; ".join(f"{n}: {w}" for n, w in sorted(not_admitted.items()))
            return ("Unknown", "ValidationNotAdmitted",
                    f"{passed}/{len(ready_nodes)} ready nodes validated; not admitted: {msg}"[:1024]), requeue_after
        return ("Unknown", "ValidationRunning", f"{passed}/{len(ready_nodes)} ready nodes validated"), requeue_after

    async def _event(self, obj: dict, type_: str, reason: str, msg: str) -> None:
        if self.recorder:
            await self.recorder.event(obj, type_, reason, msg)

    # -- create ----------------------------------------------------------------------------------
    async def _create_openshift_collateral(self, parent: dict, sa_name: str) -> None:
        sa = discovery.linkdiscovery_service_account()
        sa["metadata"]["name"] = sa_name
        sa["metadata"]["namespace"] = self.namespace
        set_controller_reference(parent, sa)
        try:
            await self.client.create(kube.SERVICEACCOUNTS, sa, namespace=self.namespace)
        except ApiError as e:
            if not is_already_exists(e):
                log.error("unable to create service account: %s", e)
                return
        rb = discovery.openshift_role_binding()
        rb["metadata"]["name"] = sa_name + "-rb"
        rb["metadata"]["namespace"] = self.namespace
        rb["subjects"] = [{"kind": "ServiceAccount", "name": sa_name, "namespace": self.namespace}]
        set_controller_reference(parent, rb)
        try:
            await self.client.create(kube.ROLEBINDINGS, rb, namespace=self.namespace)
        except ApiError as e:
            if not is_already_exists(e):
                log.error("unable to create role binding: %s", e)

    async def _create_daemonset(self, raw: dict, p: T.NetworkClusterPolicy, hold: tuple = (None, [], False)) -> Result:
        if p.spec.configurationType not in T.CONFIGURATION_TYPES:
            log.info("Unknown configuration type, this shouldn't happen! type=%s", p.spec.configurationType)
            raise ValueError(f"unknown configuration type {p.spec.configurationType!r}")
        ds = discovery.discovery_daemonset()
        sa_name = p.name + "-sa" if self.is_openshift else ""
        if sa_name:
            ds["spec"]["template"]["spec"]["serviceAccountName"] = sa_name
        update_daemonset_for(ds, p, self.namespace, hold[0])
        set_controller_reference(raw, ds)
        log.info("Creating %s DaemonSet name=%s", p.spec.configurationType, p.name)
        try:
            created = await self.client.create(kube.DAEMONSETS, ds, namespace=self.namespace)
        except ApiError as e:
            if not is_already_exists(e):
                raise
            # Our cache has not seen it yet: continue on the update path with the live object.
            created = await self.client.get(kube.DAEMONSETS, p.name, self.namespace)
            return await self._update(raw, p, created, hold)
        await self._event(raw, "Normal", "DaemonSetCreated", f"Created DaemonSet {self.namespace}/{p.name}")
        if sa_name:
            await self._create_openshift_collateral(raw, sa_name)
        return await self._update_status(raw, p, created, hold[1], hold[2])

    # -- update ----------------------------------------------------------------------------------
    async def _update(self, raw: dict, p: T.NetworkClusterPolicy, ds: dict, hold: tuple = (None, [], False)) -> Result:
        original = copy.deepcopy(ds)
        update_daemonset_for(ds, p, self.namespace, hold[0])
        if original["spec"]["template"]["spec"] != ds["spec"]["template"]["spec"] or \
                original["spec"].get("updateStrategy") != ds["spec"].get("updateStrategy"):
            log.info("DS difference for %s", p.name)
            ds = await self.client.replace(kube.DAEMONSETS, ds)
            await self._event(raw, "Normal", "DaemonSetUpdated", f"Updated DaemonSet {self.namespace}/{p.name}")
        return await self._update_status(raw, p, ds, hold[1], hold[2])

    async def _update_status(self, raw: dict, p: T.NetworkClusterPolicy, ds: dict,
                             held_off: Optional[List[str]] = None, overlapping: bool = False) -> Result:
        st = ds.get("status", {}) or {}
        targets = int(st.get("desiredNumberScheduled", 0) or 0)
        ready = int(st.get("numberReady", 0) or 0)
        cur = p.status
        updated = not p.has_status or not cur.state
        if cur.targets != targets or cur.ready != ready:
            updated = True
        new_state = status_for(targets, ready)
        errors = [f"dependency missing: {d}" for d in self.missing_dependencies]
        errors += held_off or []
        node_errs, degraded, starting = self._node_errors(ds["metadata"]["name"]) if targets and ready < targets \
            else ([], set(), set())
        errors += node_errs
        generation = int(raw.get("metadata", {}).get("generation", 0) or 0)
        # Validation first: it adds its failed nodes to `errors`, and the comparison with the stored
        # status must see the whole list (else every reconcile rewrites an unchanged status).
        v = await self._reconcile_validation(raw, p, ds, generation, errors)
        validated, requeue_after = v if v is not None else (None, 0.0)
        kept, kept_requeue = await self._kept_nodes(raw, p, ds)
        if kept_requeue:
            requeue_after = min(requeue_after, kept_requeue) if requeue_after else kept_requeue
        if overlapping:
            requeue_after = min(requeue_after, HELD_OFF_REFRESH_S) if requeue_after else HELD_OFF_REFRESH_S
        if cur.state != new_state or cur.errors != errors or cur.keptNodes != kept:
            updated = True
        # Nodes still starting up are in status.errors (with their reason) and keep Ready False,
        # but they are not a degradation.
        conditions = policy_conditions(cur.conditions, targets, ready, [e for e in errors if e not in starting],
                                       generation)
        if validated is not None:
            now = _now_rfc3339()
            old_v = [dict(c) for c in cur.conditions if c.get("type") == COND_VALIDATED]
            _set_condition(old_v, COND_VALIDATED, *validated, generation, now)
            conditions = conditions + old_v
        if conditions != cur.conditions or cur.observedGeneration != generation:
            updated = True
        if not updated:
            return Result(requeue_after=requeue_after)
        body = copy.deepcopy(raw)
        body["status"] = {"targets": targets, "ready": ready, "state": new_state, "errors": errors,
                          "conditions": conditions, "observedGeneration": generation}
        if kept:
            body["status"]["keptNodes"] = kept
        try:
            await self.client.replace_status(kube.NETWORKCLUSTERPOLICIES, body)
        except ApiError as e:
            if is_conflict(e):
                return Result(requeue=True)
            if is_not_found(e):
                return Result()
            log.error("unable to update network conf status: %s", e)
            raise
        if cur.state != new_state and new_state == STATE_ALL_GOOD:
            await self._event(raw, "Normal", "AllNodesReady", f"{ready}/{targets} nodes configured")
        for e in errors:  # an agent that exited / a node that degraded, with its reason: once per new message
            if e not in cur.errors and CONFLICT_MARK in e:
                await self._event(raw, "Warning", "PolicyConflict", e[:1024])
            elif e not in cur.errors and "scale-out not ready (" in e and "): " in e:
                if e in degraded:
                    await self._event(raw, "Warning", "NodeDegraded", e[:1024])
                elif not e.endswith(tuple(STARTUP_REASONS)):
                    await self._event(raw, "Warning", "AgentFailed", e[:1024])
        return Result(requeue_after=requeue_after)

    # -- entry point -------------------------------------------------------------------------------
    async def reconcile(self, name: str) -> Result:
        raw = self._get_policy(name)
        if raw is None:
            return Result()  # deleted; ownerRef GC removes the DaemonSet
        p = T.NetworkClusterPolicy.from_dict(raw)
        if raw["metadata"].get("deletionTimestamp"):
            return await self._finalize(raw, p)
        fins = list(raw["metadata"].get("finalizers") or [])
        want = needs_node_cleanup(p) or bool(p.status.keptNodes)  # released only once every kept node is clean
        if want != (FINALIZER in fins):
            body = copy.deepcopy(raw)
            body["metadata"]["finalizers"] = fins + [FINALIZER] if want else [f for f in fins if f != FINALIZER]
            try:
                raw = await self.client.replace(kube.NETWORKCLUSTERPOLICIES, body)
            except ApiError as e:
                if is_conflict(e):
                    return Result(requeue=True)
                if is_not_found(e):
                    return Result()
                raise
        owned = self._list_owned(name)
        hold = await self._hold_off(p)
        if not owned:
            return await self._create_daemonset(raw, p, hold)
        return await self._update(raw, p, copy.deepcopy(owned[0]), hold)
