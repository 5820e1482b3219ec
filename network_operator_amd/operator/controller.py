"""Controller: informers + work queue + workers around the reconciler.

The reference builds this with ``ctrl.NewControllerManagedBy(mgr).For(&NetworkClusterPolicy{})
.Owns(&apps.DaemonSet{})`` (reference internal/controller/networkconfiguration_controller.go:407-429):
events on a policy enqueue the policy; events on a DaemonSet enqueue the policy that controls
it.  Reconcile errors are retried with per-item exponential backoff, ``Result.requeue`` is
rate-limited, ``Result.requeue_after`` is delayed, success forgets the item's backoff.
"""

from __future__ import annotations

import asyncio
import logging
import time
from typing import Dict, List, Optional

from ..api.v1alpha1 import types as T
from . import kube
from .informer import Informer, controller_of, slim_event, slim_job, slim_pod
from .kube import ApiClient
from .metrics import OperatorMetrics
from .reconciler import (CONFLICT_MARK, OWNER_KEY, VALIDATION_APP, EventRecorder, NetworkClusterPolicyReconciler,
                         daemonset_owner_index, job_owner_index, policy_owner_index)
from .workqueue import RateLimitingQueue

log = logging.getLogger("controller")

CONTROLLER_NAME = "networkclusterpolicy"
PROBE_EVENT_KEY = "involvedObject.name"


def pod_ready(pod: Optional[dict]) -> bool:
    conds = ((pod or {}).get("status") or {}).get("conditions") or []
    return any(c.get("type") == "Ready" and c.get("status") == "True" for c in conds)


class PolicyController:
    def __init__(self, client: ApiClient, namespace: str, is_openshift: bool = False, workers: int = 2,
                 metrics: Optional[OperatorMetrics] = None, record_events: bool = True):
        self.client = client
        self.namespace = namespace
        self.workers = workers
        self.metrics = metrics or OperatorMetrics()
        self.policies = Informer(client, kube.NETWORKCLUSTERPOLICIES)
        self.daemonsets = Informer(client, kube.DAEMONSETS, namespace=namespace)
        self.daemonsets.add_index(OWNER_KEY, policy_owner_index)
        # Agent pods (indexPods in the reference, :385-404): their Ready condition explains
        # which nodes are not configured yet (status.errors).
        self.pods = Informer(client, kube.PODS, namespace=namespace, label_selector="app=amd-network-tools",
                             transform=slim_pod)
        self.pods.add_index(OWNER_KEY, daemonset_owner_index)
        # Fabric validation Jobs (amdScaleOut.validation): their outcome is the FabricValidated condition.
        self.jobs = Informer(client, kube.JOBS, namespace=namespace, label_selector=f"app={VALIDATION_APP}",
                             transform=slim_job)
        self.jobs.add_index(OWNER_KEY, policy_owner_index)
        # Their Pods: a Pod the kubelet refused to run is not a validation verdict.
        self.job_pods = Informer(client, kube.PODS, namespace=namespace, label_selector=f"app={VALIDATION_APP}",
                                 transform=slim_pod,
                                 keep=lambda p: (p.get("status") or {}).get("phase") == "Failed")
        self.job_pods.add_index(OWNER_KEY, job_owner_index)
        # The kubelet's readiness-probe failures on agent Pods: the probe prints the agent's
        # reason, so status.errors can say why a running node withdrew its label.
        self.probe_events = Informer(client, kube.EVENTS, namespace=namespace, transform=slim_event,
                                     field_selector="involvedObject.kind=Pod,reason=Unhealthy")
        self.probe_events.add_index(PROBE_EVENT_KEY, lambda e: [(e.get("involvedObject") or {}).get("name", "")])
        self.queue = RateLimitingQueue(CONTROLLER_NAME)
        self.reconciler = NetworkClusterPolicyReconciler(
            client, namespace, is_openshift,
            get_policy=lambda name: self.policies.get(name),
            list_owned=lambda name: self.daemonsets.by_index(OWNER_KEY, name),
            recorder=EventRecorder(client, namespace) if record_events else None,
            list_pods=lambda ds: self.pods.by_index(OWNER_KEY, ds),
            list_jobs=lambda name: self.jobs.by_index(OWNER_KEY, name),
            list_job_pods=lambda job: self.job_pods.by_index(OWNER_KEY, job),
            list_probe_events=lambda pod: self.probe_events.by_index(PROBE_EVENT_KEY, pod),
            list_policies=self.policies.list)
        self.reconciler.on_cleanup = lambda policy, outcome: self.metrics.node_cleanups.labels(policy, outcome).inc()
        self.policies.add_handler(self._on_policy)
        self.daemonsets.add_handler(self._on_daemonset)
        self.pods.add_handler(self._on_pod)
        self.jobs.add_handler(self._on_job)
        self.job_pods.add_handler(self._on_job_pod)
        self.probe_events.add_handler(self._on_probe_event)
        self._tasks: List[asyncio.Task] = []
        self.reconciles = 0
        self._pod_seen: Dict[str, float] = {}  # agent Pod uid -> monotonic time first seen, until Ready

    async def _on_policy(self, ev: str, obj: dict, old: Optional[dict]) -> None:
        await self._enqueue(obj["metadata"]["name"])
        # Which nodes a policy holds depends on the older policies of its type: one that comes,
        # goes (or starts deleting) or changes its selector or type moves the others' hold-off.
        def placement(o: Optional[dict]) -> tuple:
            spec = (o or {}).get("spec") or {}
            return (spec.get("configurationType", ""), spec.get("nodeSelector") or {},
                    bool(((o or {}).get("metadata") or {}).get("deletionTimestamp")))
        if ev != "MODIFIED" or placement(old) != placement(obj):
            for ctype in {placement(obj)[0], placement(old)[0]} if old else {placement(obj)[0]}:
                await self._enqueue_type(obj["metadata"]["name"], ctype)

    async def _enqueue_type(self, name: str, ctype: str) -> None:
        for p in self.policies.list():
            if p["metadata"]["name"] != name and (p.get("spec") or {}).get("configurationType", "") == ctype:
                await self._enqueue(p["metadata"]["name"])

    async def _on_daemonset(self, ev: str, obj: dict, old: Optional[dict]) -> None:
        ref = controller_of(obj)
        if ref and ref.get("kind") == T.KIND and ref.get("apiVersion") == T.API_VERSION:
            await self._enqueue(ref["name"])

    async def _on_pod(self, ev: str, obj: dict, old: Optional[dict]) -> None:
        ref = controller_of(obj)
        if ref and ref.get("kind") == "DaemonSet":
            ds = self.daemonsets.get(ref["name"], self.namespace)
            owner = controller_of(ds) if ds else None
            if owner and owner.get("kind") == T.KIND:
                self._observe_readiness(owner["name"], ev, obj, old)
                await self._enqueue(owner["name"])
                if ev in ("ADDED", "DELETED"):
                    await self._enqueue_others(owner["name"])
            elif ds is None and ev in ("ADDED", "DELETED"):
                # The DaemonSet is not in the cache (yet: the watches are separate streams; or any
                # more: its policy is gone): every policy may share, or no longer share, this node.
                await self._enqueue_others(None)

    async def _enqueue_others(self, name: Optional[str]) -> None:
        """An agent Pod came or went: the nodes the other policies of its type are held off may
        have changed, and their status names them (reconciler._hold_off).  Without a known owner,
        every policy."""
        me = self.policies.get(name) if name else None
        ctype = ((me or {}).get("spec") or {}).get("configurationType", "") if me else None
        for p in self.policies.list():
            if p["metadata"]["name"] != name and (ctype is None or (p.get("spec") or {}).get("configurationType", "") == ctype):
                await self._enqueue(p["metadata"]["name"])

    async def _on_job(self, ev: str, obj: dict, old: Optional[dict]) -> None:
        ref = controller_of(obj)
        if ref and ref.get("kind") == T.KIND:
            await self._enqueue(ref["name"])

    async def _on_probe_event(self, ev: str, obj: dict, old: Optional[dict]) -> None:
        io = obj.get("involvedObject") or {}
        pod = self.pods.get(io.get("name", ""), io.get("namespace") or self.namespace)
        ref = controller_of(pod) if pod else None
        if ref and ref.get("kind") == "DaemonSet":
            ds = self.daemonsets.get(ref["name"], self.namespace)
            owner = controller_of(ds) if ds else None
            if owner and owner.get("kind") == T.KIND:
                await self._enqueue(owner["name"])

    async def _on_job_pod(self, ev: str, obj: dict, old: Optional[dict]) -> None:
        ref = controller_of(obj)
        if ref and ref.get("kind") == "Job":
            job = self.jobs.get(ref["name"], self.namespace)
            owner = controller_of(job) if job else None
            if owner and owner.get("kind") == T.KIND:
                await self._enqueue(owner["name"])

    def _observe_readiness(self, policy: str, ev: str, obj: dict, old: Optional[dict]) -> None:
        uid = obj.get("metadata", {}).get("uid", "")
        if ev == "DELETED":
            self._pod_seen.pop(uid, None)
            return
        now, was = time.monotonic(), pod_ready(old) if old else False
        ready = pod_ready(obj)
        if not ready:
            self._pod_seen.setdefault(uid, now)
            if was:
                self.metrics.agent_unready.labels(policy).inc()
        elif not was and uid in self._pod_seen:
            self.metrics.agent_ready_time.labels(policy).observe(now - self._pod_seen.pop(uid))

    async def requeue_all(self) -> None:
        """Reconcile every policy again (e.g. after a cluster dependency appeared or vanished)."""
        for p in self.policies.list():
            await self.queue.add(p["metadata"]["name"])

    async def _enqueue(self, name: str) -> None:
        await self.queue.add(name)
        self.metrics.queue_adds.labels(CONTROLLER_NAME).inc()
        self.metrics.queue_depth.labels(CONTROLLER_NAME).set(self.queue.depth)

    async def _worker(self) -> None:
        while True:
            name = await self.queue.get()
            if name is None:
                return
            self.metrics.queue_depth.labels(CONTROLLER_NAME).set(self.queue.depth)
            t0 = time.perf_counter()
            try:
                res = await self.reconciler.reconcile(name)
            except asyncio.CancelledError:
                await self.queue.done(name)
                raise
            except Exception as e:
                log.error("Reconciler error for %s: %s", name, e)
                self.metrics.reconcile_errors.labels(CONTROLLER_NAME).inc()
                self.metrics.reconcile_total.labels(CONTROLLER_NAME, "error").inc()
                self.metrics.queue_retries.labels(CONTROLLER_NAME).inc()
                await self.queue.add_rate_limited(name)
            else:
                if res.requeue_after > 0:
                    self.queue.forget(name)
                    await self.queue.add_after(name, res.requeue_after)
                    self.metrics.reconcile_total.labels(CONTROLLER_NAME, "requeue_after").inc()
                elif res.requeue:
                    await self.queue.add_rate_limited(name)
                    self.metrics.queue_retries.labels(CONTROLLER_NAME).inc()
                    self.metrics.reconcile_total.labels(CONTROLLER_NAME, "requeue").inc()
                else:
                    self.queue.forget(name)
                    self.metrics.reconcile_total.labels(CONTROLLER_NAME, "success").inc()
                self._export_policy(name)
            finally:
                self.reconciles += 1
                self.metrics.reconcile_time.labels(CONTROLLER_NAME).observe(time.perf_counter() - t0)
            await self.queue.done(name)

    def _export_policy(self, name: str) -> None:
        p = self.policies.get(name)
        if p is None:
            for g in (self.metrics.policy_targets, self.metrics.policy_ready, self.metrics.nodes_owing_cleanup,
                      self.metrics.policy_conflicts):
                try:
                    g.remove(name)
                except KeyError:
                    pass
            return
        st = p.get("status") or {}
        self.metrics.policy_targets.labels(name).set(st.get("targets", 0) or 0)
        self.metrics.policy_ready.labels(name).set(st.get("ready", 0) or 0)
        self.metrics.nodes_owing_cleanup.labels(name).set(len(st.get("keptNodes") or []))
        self.metrics.policy_conflicts.labels(name).set(sum(CONFLICT_MARK in e for e in st.get("errors") or []))

    async def start(self) -> None:
        self._tasks.append(self.policies.start())
        self._tasks.append(self.daemonsets.start())
        self._tasks.append(self.pods.start())
        self._tasks.append(self.jobs.start())
        self._tasks.append(self.job_pods.start())
        self._tasks.append(self.probe_events.start())
        await asyncio.gather(self.policies.synced.wait(), self.daemonsets.synced.wait(), self.pods.synced.wait(),
                             self.jobs.synced.wait(), self.job_pods.synced.wait(), self.probe_events.synced.wait())
        for _ in range(self.workers):
            self._tasks.append(asyncio.ensure_future(self._worker()))

    def has_synced(self) -> bool:
        return all(i.synced.is_set() for i in (self.policies, self.daemonsets, self.pods, self.jobs, self.job_pods,
                                               self.probe_events))

    async def stop(self) -> None:
        await self.queue.shutdown()
        for t in self._tasks:
            t.cancel()
        for t in self._tasks:
            try:
                await t
            except (asyncio.CancelledError, Exception):
                pass
        self._tasks.clear()
