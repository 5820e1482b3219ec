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

The DaemonSet template is built in ``templates.py`` and the same-type hold-off in ``holdoff.py``;
this module reads the cluster and writes what they build.

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
from .holdoff import (CONFLICT_MARK, HELD_EVERYWHERE_KEY, HELD_OFF_REFRESH_S, MAX_HOLD_OFF_TERMS,  # noqa: F401
                      held_off_error, hold_off_terms, set_hold_off)
from .templates import (ARTIFACT_DIR_CONTAINER, ARTIFACT_DIR_HOST, DRIVER_CONTAINER, FW_LLDP_STATE_FILE,  # noqa: F401
                        HOST_NIC_LABEL, HOST_NIC_LABEL_FILE, HOST_NIC_LINK_STATE_FILE, HOST_NIC_LLDP_CACHE_FILE,
                        HOST_NIC_MTU_STATE_FILE, L3_WAIT, LINK_STATE_FILE, LLDP_CACHE_FILE, MANAGED_VOLUMES, RCCL_ENV_FILE, RCCL_NET_FILE, RCCL_TOPO_FILE,
                        VERIFY_PEERS_TIMEOUT, add_host_volume, agent_args, host_nic_agent_args, order_managed_volumes,
                        remove_volume, update_amd_scale_out_daemonset, update_daemonset_for, update_host_nic_daemonset)

log = logging.getLogger("controller")

OWNER_KEY = ".metadata.controller"

STATE_NO_TARGETS = "No targets"
STATE_WORKING = "Working on it.."
STATE_ALL_GOOD = "All good"
COND_READY = "Ready"
COND_DEGRADED = "Degraded"
COND_VALIDATED = "FabricValidated"
VALIDATION_APP = "amd-gpu-fabric-validation"  # Job label; the operator's Job informer selects on it


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
STARTUP_REASONS = ("waiting for LLDP", "not configured yet", "waiting for carrier", "agent starting",
                   "waiting for RDMA device")


def _starting_up(reason: str) -> bool:
    """Every NIC of the probe's reason is still coming up (no Event for a node that starts)."""
    return all(part.split(": ", 1)[-1] in STARTUP_REASONS for part in reason.split("; "))


def _container_running(pod: dict) -> bool:
    return any("running" in (cs.get("state") or {}) for cs in (pod.get("status") or {}).get("containerStatuses") or [])


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
EVENT_CONCURRENCY = 16  # Events (and the Node GETs behind Node events) in flight per status update
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

    async def event(self, obj: dict, type_: str, reason: str, message: str, namespace: Optional[str] = None) -> None:
        md = obj.get("metadata", {})
        ns = namespace or self.namespace
        body = {
            "apiVersion": "v1", "kind": "Event",
            "metadata": {"generateName": f"{md.get('name', 'obj')}.", "namespace": ns},
            "involvedObject": {"apiVersion": obj.get("apiVersion"), "kind": obj.get("kind"), "name": md.get("name"),
                               "uid": md.get("uid")},
            "type": type_, "reason": reason, "message": message, "source": {"component": self.component},
            "count": 1,
        }
        try:
            await self.client.create(kube.EVENTS, body, namespace=ns)
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
        sends = []
        for e in errors:  # an agent that exited / a node that degraded, with its reason: once per new message
            if e not in cur.errors and CONFLICT_MARK in e:
                sends.append(lambda e=e: self._event(raw, "Warning", "PolicyConflict", e[:1024]))
            elif e not in cur.errors and "scale-out not ready (" in e and "): " in e:
                if e in degraded:
                    sends.append(lambda e=e: self._event(raw, "Warning", "NodeDegraded", e[:1024]))
                    sends.append(lambda e=e: self._node_event(e, "ScaleOutDegraded", p.name))
                elif not e.endswith(tuple(STARTUP_REASONS)):
                    sends.append(lambda e=e: self._event(raw, "Warning", "AgentFailed", e[:1024]))
                    sends.append(lambda e=e: self._node_event(e, "ScaleOutAgentFailed", p.name))
        if sends:  # a switch reboot degrades every node at once: not thousands of round trips in a row
            gate = asyncio.Semaphore(EVENT_CONCURRENCY)

            async def send(make):  # (coroutines made only when sent: none left un-awaited on a cancel)
                async with gate:
                    await make()
            await asyncio.gather(*(send(c) for c in sends))
        return Result(requeue_after=requeue_after)

    async def _node_event(self, error: str, reason: str, policy: str) -> None:
        """The same news on the Node itself, so ``kubectl describe node`` shows why its scale-out
        label went or never came.  Events of cluster-scoped objects live in "default"; describe
        matches them by the Node's uid, hence the GET (rare: once per new message)."""
        if not self.recorder:
            return
        node = error.split(": scale-out not ready (", 1)[0]
        try:
            obj = await self.client.get(kube.NODES, node)
        except ApiError as e:
            log.debug("node %s for its event: %s", node, e)
            return
        why = error.split("): ", 1)[1] if "): " in error else error
        await self.recorder.event({"apiVersion": "v1", "kind": "Node", "metadata": obj.get("metadata", {})},
                                  "Warning", reason, f"{why} (policy {policy})"[:1024], namespace="default")

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
