"""In-process fake Kubernetes API server (aiohttp) for control-plane tests.

The reference tests its controller against envtest — a real etcd + kube-apiserver without
controllers (reference internal/controller/suite_test.go:61-102).  Neither is available
here, so this server implements the API-server behaviour the operator depends on:

* discovery (``/api``, ``/apis``, group/version resource lists; optional OpenShift groups);
* CRUD on any registered resource, cluster-scoped and namespaced, ``generateName``;
* ``metadata.resourceVersion`` optimistic concurrency (409 Conflict), ``uid``,
  ``generation`` bumped on spec changes, no-op updates do not bump the version;
* the ``status`` subresource (main writes keep status, status writes keep spec);
* JSON merge patch and RFC 6902 JSON patch;
* LIST with label / field selectors; WATCH with replay from a resourceVersion, BOOKMARK
  events, ``410 Gone`` for compacted history, ``timeoutSeconds``;
* CRD structural-schema validation of NetworkClusterPolicies (422 Invalid) and pruning;
* admission: calls Mutating/ValidatingWebhookConfigurations registered in the store — by
  ``clientConfig.url``, or by ``clientConfig.service`` resolved through the stored Service and a
  test-set ready endpoint (``service_endpoints``), failing per ``failurePolicy`` while the
  Service or its endpoint is missing, as a real API server does before the operator pod
  serves — and applies the returned JSONPatch, including the *rules* match on the resource
  plural, so a webhook registered for a wrong resource is never called;
* background garbage collection of dependents through ``ownerReferences``;
* a DaemonSet controller simulation: ``desiredNumberScheduled`` from Nodes matching the pod
  template's nodeSelector, ``numberReady`` from per-node agent readiness set by the test;
* TokenReview / SubjectAccessReview answers from a token table (metrics authn/authz);
* fault injection: fail the next N matching requests, stall matching requests (a wedged API
  server or network path, optionally for one client by its User-Agent), drop all watch
  streams, compact.
"""

from __future__ import annotations

import asyncio
import base64
import copy
import datetime as dt
import json
import re
import ssl
import tempfile
import uuid
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import aiohttp
from aiohttp import web

from ..api.v1alpha1 import crd as CRD
from ..api.v1alpha1 import types as T
from ..operator import kube
from ..operator.kube import Resource


def _now() -> str:
    return dt.datetime.now(dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%SZ")


def _status(code: int, reason: str, message: str, details: Optional[dict] = None) -> web.Response:
    body = {"kind": "Status", "apiVersion": "v1", "status": "Failure", "message": message, "reason": reason,
            "code": code}
    if details:
        body["details"] = details
    return web.json_response(body, status=code)


def merge_patch(target, patch):
    """RFC 7386."""
    if not isinstance(patch, dict):
        return copy.deepcopy(patch)
    out = copy.deepcopy(target) if isinstance(target, dict) else {}
    for k, v in patch.items():
        if v is None:
            out.pop(k, None)
        else:
            out[k] = merge_patch(out.get(k), v)
    return out


def _ptr(doc, path: str):
    parts = [p.replace("~1", "/").replace("~0", "~") for p in path.lstrip("/").split("/")] if path not in ("", "/") else []
    parent = None
    cur = doc
    for p in parts:
        parent = cur
        if isinstance(cur, list):
            cur = None if p == "-" else cur[int(p)]  # "-": one past the end (RFC 6902 add)
        else:
            cur = cur.get(p) if isinstance(cur, dict) else None
    return parent, (parts[-1] if parts else None), cur


def json_patch_apply(doc, ops):
    """RFC 6902 subset: add, replace, remove, test."""
    doc = copy.deepcopy(doc)
    for op in ops:
        parent, key, cur = _ptr(doc, op["path"])
        kind = op["op"]
        if kind == "test":
            if cur != op["value"]:
                raise ValueError(f"test failed at {op['path']}")
            continue
        if parent is None:
            if kind in ("add", "replace"):
                doc = copy.deepcopy(op["value"])
                continue
            raise ValueError("cannot remove the root")
        if isinstance(parent, list):
            idx = len(parent) if key == "-" else int(key)
            if kind == "add":
                parent.insert(idx, copy.deepcopy(op["value"]))
            elif kind == "replace":
                parent[idx] = copy.deepcopy(op["value"])
            elif kind == "remove":
                parent.pop(idx)
        else:
            if kind in ("add", "replace"):
                if kind == "replace" and key not in parent:
                    raise ValueError(f"replace of missing path {op['path']}")
                parent[key] = copy.deepcopy(op["value"])
            elif kind == "remove":
                if key not in parent:
                    raise ValueError(f"remove of missing path {op['path']}")
                del parent[key]
    return doc


def match_labels(labels: dict, selector: str) -> bool:
    for term in [t.strip() for t in selector.split(",") if t.strip()]:
        if "!=" in term:
            k, v = term.split("!=", 1)
            if labels.get(k) == v:
                return False
        elif "==" in term or "=" in term:
            k, v = re.split("==?", term, maxsplit=1)
            if labels.get(k) != v:
                return False
        elif term.startswith("!"):
            if term[1:] in labels:
                return False
        elif term not in labels:
            return False
    return True


def _match_fields(obj: dict, selector: str) -> bool:
    """Field selectors as the API server serves them for the fields used here: dotted paths
    (metadata.name, spec.nodeName, status.phase, involvedObject.kind, reason, ...)."""
    for term in [t.strip() for t in selector.split(",") if t.strip()]:
        neg = "!=" in term
        k, v = re.split("!=|==|=", term, maxsplit=1)
        actual = obj
        for part in k.split("."):
            actual = actual.get(part) if isinstance(actual, dict) else None
        if (str(actual) if actual is not None else None) == v or (actual is None and v == ""):
            if neg:
                return False
        elif not neg:
            return False
    return True


@dataclass
class _Watch:
    res: Resource
    namespace: Optional[str]
    label_selector: Optional[str]
    field_selector: Optional[str] = None
    queue: asyncio.Queue = field(default_factory=asyncio.Queue)


@dataclass
class _Fault:
    method: str
    pattern: re.Pattern
    status: int
    count: int
    reason: str = "InternalError"
    user_agent: Optional[str] = None  # only this client's requests (None: everyone's)


FOREGROUND_DELETION = "foregroundDeletion"


def _node_affinity_ok(node: dict, pod_spec: dict) -> bool:
    """The template's requiredDuringSchedulingIgnoredDuringExecution node affinity, as the
    DaemonSet controller evaluates it: terms ORed, expressions within a term ANDed (In, NotIn,
    Exists, DoesNotExist, Gt, Lt on labels; matchFields on metadata.name); a term with no
    expression matches nothing."""
    terms = ((((pod_spec.get("affinity") or {}).get("nodeAffinity") or {})
              .get("requiredDuringSchedulingIgnoredDuringExecution") or {}).get("nodeSelectorTerms"))
    if not terms:
        return True
    labels = node["metadata"].get("labels") or {}

    def ok(e: dict, value) -> bool:
        op, vals = e.get("operator"), e.get("values") or []
        if op == "In":
            return value is not None and value in vals
        if op == "NotIn":
            return value is None or value not in vals
        if op == "Exists":
            return value is not None
        if op == "DoesNotExist":
            return value is None
        if op in ("Gt", "Lt") and value is not None and vals:
            try:
                return int(value) > int(vals[0]) if op == "Gt" else int(value) < int(vals[0])
            except ValueError:
                return False
        return False
    name = node["metadata"]["name"]
    return any((t.get("matchExpressions") or t.get("matchFields"))
               and all(ok(e, labels.get(e.get("key"))) for e in t.get("matchExpressions") or [])
               and all(ok(e, name if e.get("key") == "metadata.name" else None) for e in t.get("matchFields") or [])
               for t in terms)


class FakeApiServer:
    STATUS_SUBRESOURCE = {kube.NETWORKCLUSTERPOLICIES, kube.DAEMONSETS}

    def __init__(self, openshift: bool = False, history: int = 10000, bookmark_interval: float = 1.0,
                 gc_delay: float = 0.0, agent_ready_delay: Optional[float] = None,
                 extra_groups: Optional[List[str]] = None, foreground_hold: float = 0.0):
        self.resources: List[Resource] = list(kube.ALL_RESOURCES)
        self.openshift = openshift
        self.objects: Dict[Tuple[str, str, str], Dict[Tuple[str, str], dict]] = {}
        self._owned: Dict[str, set] = {}  # owner uid -> {(resource, namespace, name)} (garbage collector)
        self._live_uids: set = set()  # uids of the stored objects: a dependent of none of them is collected
        self.rv = 100
        self.events: List[Tuple[int, Resource, str, dict]] = []
        self.history = history
        self.compacted_before = 0
        self.watches: List[_Watch] = []
        self.bookmark_interval = bookmark_interval
        self.gc_delay = gc_delay
        # Foreground cascading deletion: owner uid -> (resource, namespace, name) of owners that
        # carry the foregroundDeletion finalizer.  The garbage collector deletes their dependents,
        # deletes any dependent created meanwhile, and releases the owner `foreground_hold`
        # seconds after it last found no dependent (the real GC's processing latency).
        self._foreground: Dict[str, Tuple[Resource, str, str]] = {}
        self.foreground_hold = foreground_hold
        self.agent_ready_delay = agent_ready_delay
        # API groups of add-ons installed in the fake cluster (e.g. "nfd.k8s-sigs.io").
        self.extra_groups: List[str] = list(extra_groups or [])
        self.node_ready: Dict[Tuple[str, str], bool] = {}   # (ds ns/name, node) -> ready
        # (ds ns/name, node) -> the agent container's restartCount and lastState.terminated
        self.node_last_exit: Dict[Tuple[str, str], dict] = {}
        self.tokens: Dict[str, dict] = {}                    # bearer -> {"username", "groups", "allowed"}
        self.faults: List[_Fault] = []
        self.faults_fired = 0  # injected failures actually served
        # (method, path pattern, User-Agent or None, seconds): matching requests wait that long
        # before they are served (the client usually gives up first)
        self.stalls: List[tuple] = []
        self._unstall: Optional[asyncio.Event] = None
        self.requests: List[Tuple[str, str]] = []
        self.writes: List[Tuple[float, str, str, str]] = []  # (loop time, User-Agent, method, path)
        self.accesses: set = set()                           # (verb, group, resource[/sub])
        self.admission_calls: List[Tuple[str, str]] = []
        # (namespace, service) -> "https://host:port" of a ready endpoint (service-referenced webhooks)
        self.service_endpoints: Dict[Tuple[str, str], str] = {}
        self._runner: Optional[web.AppRunner] = None
        self.url = ""
        self._bg: List[asyncio.Task] = []
        self._closing = False

    # ------------------------------------------------------------------------------------------
    # lifecycle
    # ------------------------------------------------------------------------------------------
    async def start(self, host: str = "127.0.0.1", port: int = 0) -> str:
        app = web.Application(client_max_size=8 << 20)
        app.router.add_route("*", "/{tail:.*}", self._dispatch)
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, host, port)
        await site.start()
        sock = site._server.sockets[0]  # type: ignore[union-attr]
        self.url = f"http://{host}:{sock.getsockname()[1]}"
        return self.url

    async def stop(self) -> None:
        self._closing = True
        self.drop_watches()
        for t in self._bg:
            t.cancel()
        if self._runner:
            await self._runner.cleanup()

    # ------------------------------------------------------------------------------------------
    # test helpers
    # ------------------------------------------------------------------------------------------
    @staticmethod
    def _rkey(res: Resource) -> Tuple[str, str, str]:
        return (res.group, res.version, res.plural)

    def _table(self, res: Resource) -> Dict[Tuple[str, str], dict]:
        return self.objects.setdefault(self._rkey(res), {})

    def get_object(self, res: Resource, name: str, namespace: Optional[str] = None) -> Optional[dict]:
        o = self._table(res).get((namespace or "", name))
        return copy.deepcopy(o) if o else None

    def list_objects(self, res: Resource) -> List[dict]:
        return [copy.deepcopy(o) for o in self._table(res).values()]

    def add_node(self, name: str, labels: Optional[dict] = None, taints: Optional[List[dict]] = None) -> dict:
        node = {"apiVersion": "v1", "kind": "Node", "metadata": {"name": name, "labels": dict(labels or {})}}
        if taints:
            node["spec"] = {"taints": [dict(t) for t in taints]}
        obj = self._create(kube.NODES, node, None)
        self._sync_daemonsets()
        return obj

    def set_node_labels(self, name: str, labels: dict) -> None:
        o = self._table(kube.NODES)[("", name)]
        new = copy.deepcopy(o)
        new["metadata"]["labels"] = dict(labels)
        self._store(kube.NODES, new, "MODIFIED")
        self._sync_daemonsets()

    def set_agent_ready(self, node: str, ready: bool = True, daemonset: Optional[str] = None,
                        terminated: Optional[dict] = None) -> None:
        """Simulates the agent pod's readinessProbe on `node` (all DaemonSets if none given).
        `terminated` ({exitCode, reason, message}) is what the kubelet records when the agent
        container exits: it becomes the container's ``lastState.terminated`` and the restart
        count goes up."""
        for (ns, name), _ in self._table(kube.DAEMONSETS).items():
            if daemonset is None or daemonset in (name, f"{ns}/{name}"):
                self.node_ready[(f"{ns}/{name}", node)] = ready
                if terminated is not None:
                    prev = self.node_last_exit.get((f"{ns}/{name}", node), {})
                    self.node_last_exit[(f"{ns}/{name}", node)] = {
                        "restartCount": prev.get("restartCount", -1) + 1, "terminated": dict(terminated)}
        self._sync_daemonsets()

    def record_probe_failure(self, namespace: str, pod: str, message: str) -> None:
        """The kubelet's Event for a failed probe: reason Unhealthy, type Warning, on the Pod;
        a repeat of the same message bumps its count (the kubelet's event aggregation)."""
        name = f"{pod}.unhealthy"
        cur = self._table(kube.EVENTS).get((namespace, name))
        now = _now()
        if cur is not None and cur.get("message") == message:
            new = copy.deepcopy(cur)
            new["count"] = int(cur.get("count", 1)) + 1
            new["lastTimestamp"] = now
            self._store(kube.EVENTS, new, "MODIFIED")
            return
        body = {"apiVersion": "v1", "kind": "Event", "type": "Warning", "reason": "Unhealthy", "message": message,
                "metadata": {"name": name, "namespace": namespace},
                "involvedObject": {"apiVersion": "v1", "kind": "Pod", "name": pod, "namespace": namespace,
                                   "fieldPath": "spec.containers{configurator}"},
                "source": {"component": "kubelet"}, "count": 1, "firstTimestamp": now, "lastTimestamp": now}
        if cur is not None:
            body["metadata"] = copy.deepcopy(cur["metadata"])
            self._store(kube.EVENTS, body, "MODIFIED")
        else:
            self._create(kube.EVENTS, body, namespace)

    def set_job_result(self, name: str, namespace: str, succeeded: bool, pod_reason: Optional[str] = None,
                       pod_message: str = "", finished: Optional[str] = None) -> None:
        """What the Job controller records when the Job's only Pod ends (backoffLimit 0).  With
        `pod_reason` the Pod also exists, Failed with that kubelet reason (e.g. the admission
        rejection "OutOfamd.com/gpu"); `finished` overrides the condition's time (RFC 3339)."""
        o = self._table(kube.JOBS)[(namespace, name)]
        if pod_reason is not None:
            labels = dict((o["spec"]["template"].get("metadata") or {}).get("labels") or {})
            pod = {"apiVersion": "v1", "kind": "Pod",
                   "metadata": {"name": f"{name}-pod", "namespace": namespace, "labels": labels,
                                "ownerReferences": [{"apiVersion": "batch/v1", "kind": "Job", "name": name,
                                                     "uid": o["metadata"]["uid"], "controller": True}]},
                   "spec": {"nodeName": (o["spec"]["template"].get("spec") or {}).get("nodeName", "")},
                   "status": {"phase": "Failed", "reason": pod_reason, "message": pod_message}}
            cur = self._table(kube.PODS).get((namespace, pod["metadata"]["name"]))
            if cur is None:
                self._create(kube.PODS, pod, namespace)
            else:
                self._store(kube.PODS, dict(copy.deepcopy(cur), status=pod["status"]), "MODIFIED")
        new = copy.deepcopy(o)
        cond = "Complete" if succeeded else "Failed"
        new["status"] = {"succeeded" if succeeded else "failed": 1,
                         "conditions": [{"type": cond, "status": "True", "lastTransitionTime": finished or _now()}]}
        self._store(kube.JOBS, new, "MODIFIED")

    def fail_next(self, method: str, path_regex: str, status: int = 500, count: int = 1,
                  reason: str = "InternalError", user_agent: Optional[str] = None) -> None:
        self.faults.append(_Fault(method.upper(), re.compile(path_regex), status, count, reason, user_agent))

    def stall(self, method: str, path_regex: str, seconds: float, user_agent: Optional[str] = None) -> None:
        """Hold every matching request `seconds` before serving it, until clear_stalls()."""
        self.stalls.append((method.upper(), re.compile(path_regex), user_agent, seconds))

    def clear_stalls(self) -> None:
        """Ends the stalls, releasing requests that are being held."""
        self.stalls.clear()
        if self._unstall is not None:
            self._unstall.set()
            self._unstall = None

    def drop_watches(self) -> None:
        for w in self.watches:
            w.queue.put_nowait(None)
        self.watches.clear()

    def compact(self) -> None:
        """Forget event history (etcd compaction + API-server restart): every watch resuming
        from any resourceVersion issued so far gets 410 Gone and must relist."""
        self.compacted_before = self.rv + 2
        self.events.clear()
        self.drop_watches()

    # ------------------------------------------------------------------------------------------
    # storage core
    # ------------------------------------------------------------------------------------------
    def _next_rv(self) -> str:
        self.rv += 1
        return str(self.rv)

    def _emit(self, res: Resource, typ: str, obj: dict) -> None:
        rv = int(obj["metadata"]["resourceVersion"]) if typ != "DELETED" else self.rv
        # One snapshot, shared by the history and every watcher (they only serialise it).
        snap = json.loads(json.dumps(obj))
        self.events.append((rv, res, typ, snap))
        if len(self.events) > self.history:
            drop = len(self.events) - self.history
            self.compacted_before = self.events[drop - 1][0] + 1
            del self.events[:drop]
        for w in list(self.watches):
            if w.res == res and self._visible(w, obj):
                w.queue.put_nowait((typ, snap))

    @staticmethod
    def _visible(w: _Watch, obj: dict) -> bool:
        md = obj.get("metadata", {})
        if w.namespace and md.get("namespace") != w.namespace:
            return False
        if w.label_selector and not match_labels(md.get("labels", {}) or {}, w.label_selector):
            return False
        if w.field_selector and not _match_fields(obj, w.field_selector):
            return False
        return True

    def _store(self, res: Resource, obj: dict, typ: str) -> dict:
        # Owner index for the garbage collector (a scan of every object per deletion is
        # quadratic at thousands of Pods and Jobs); entries are re-checked when used.
        for r in obj["metadata"].get("ownerReferences") or []:
            if r.get("uid"):
                self._owned.setdefault(r["uid"], set()).add(
                    (res, obj["metadata"].get("namespace", "") if res.namespaced else "", obj["metadata"]["name"]))
        obj["metadata"]["resourceVersion"] = self._next_rv()
        self._table(res)[(obj["metadata"].get("namespace", "") if res.namespaced else "", obj["metadata"]["name"])] = obj
        self._emit(res, typ, obj)
        return obj

    def _create(self, res: Resource, obj: dict, namespace: Optional[str]) -> dict:
        obj = copy.deepcopy(obj)
        md = obj.setdefault("metadata", {})
        if not md.get("name"):
            if md.get("generateName"):
                md["name"] = md["generateName"] + uuid.uuid4().hex[:5]
            else:
                raise web.HTTPUnprocessableEntity(text="name or generateName is required")
        if res.namespaced:
            md["namespace"] = namespace or md.get("namespace") or "default"
        else:
            md.pop("namespace", None)
        key = (md.get("namespace", "") if res.namespaced else "", md["name"])
        if key in self._table(res):
            raise _Conflict(409, "AlreadyExists", f'{res.plural}.{res.group or "core"} "{md["name"]}" already exists',
                            {"name": md["name"], "kind": res.plural})
        md["uid"] = str(uuid.uuid4())
        md["creationTimestamp"] = _now()
        md["generation"] = 1
        obj.setdefault("apiVersion", res.api_version)
        obj.setdefault("kind", res.kind)
        if res in self.STATUS_SUBRESOURCE:
            obj.pop("status", None)
        if res == kube.DAEMONSETS:
            obj["status"] = {"currentNumberScheduled": 0, "desiredNumberScheduled": 0, "numberMisscheduled": 0,
                             "numberReady": 0, "observedGeneration": 1}
        self._store(res, obj, "ADDED")
        self._live_uids.add(md["uid"])
        if res in (kube.DAEMONSETS, kube.NODES):
            self._sync_daemonsets()
        created = self._table(res)[key]
        refs = [r.get("uid") for r in md.get("ownerReferences") or []]
        if any(u in self._foreground for u in refs):
            # A dependent of an owner in foreground deletion: the garbage collector deletes it.
            self._delete_or_mark(res, md["name"], key[0])
        elif refs and not any(u in self._live_uids for u in refs):
            # Every owner is gone already (a controller acting on a stale cache): the collector
            # finds the dangling references and deletes the dependent, as it does with any other.
            uid = md["uid"]
            if self.gc_delay <= 0:
                self._collect_dangling(res, key[0], md["name"], uid)
            else:
                self._bg.append(asyncio.ensure_future(self._collect_dangling_later(res, key[0], md["name"], uid)))
        return created

    def _collect_dangling(self, res: Resource, ns: str, name: str, uid: str) -> None:
        o = self._table(res).get((ns, name))
        if o is not None and o["metadata"].get("uid") == uid:
            self._delete_or_mark(res, name, ns)

    async def _collect_dangling_later(self, res: Resource, ns: str, name: str, uid: str) -> None:
        await asyncio.sleep(self.gc_delay)
        self._collect_dangling(res, ns, name, uid)

    def _delete(self, res: Resource, name: str, namespace: str) -> dict:
        key = (namespace if res.namespaced else "", name)
        obj = self._table(res).pop(key)
        obj = copy.deepcopy(obj)
        self._next_rv()
        obj["metadata"]["resourceVersion"] = str(self.rv)
        self._emit(res, "DELETED", obj)
        uid = obj["metadata"].get("uid")
        self._live_uids.discard(uid)
        if self.gc_delay <= 0:
            self._collect(uid)
        else:
            self._bg.append(asyncio.ensure_future(self._collect_later(uid)))
        if res == kube.DAEMONSETS:
            self.node_ready = {k: v for k, v in self.node_ready.items() if k[0] != f"{namespace}/{name}"}
            self.node_last_exit = {k: v for k, v in self.node_last_exit.items() if k[0] != f"{namespace}/{name}"}
        self._foreground.pop(uid, None)
        for r in obj["metadata"].get("ownerReferences") or []:
            if r.get("uid") in self._foreground:
                self._foreground_check(r["uid"])
        return obj

    def _dependents(self, uid: str) -> list:
        out = []
        for res, ns, name in sorted(self._owned.get(uid, ()), key=lambda k: (k[0].plural, k[1], k[2])):
            o = self._table(res).get((ns, name))
            if o is not None and any(r.get("uid") == uid for r in o.get("metadata", {}).get("ownerReferences") or []):
                out.append((res, ns, name))
        return out

    def _foreground_check(self, uid: str) -> None:
        """Releases an owner in foreground deletion once it has no dependents left."""
        if uid not in self._foreground or self._dependents(uid):
            return
        if self.foreground_hold > 0:
            self._bg.append(asyncio.ensure_future(self._foreground_release_later(uid)))
        else:
            self._foreground_release(uid)

    async def _foreground_release_later(self, uid: str) -> None:
        await asyncio.sleep(self.foreground_hold)
        if uid in self._foreground and not self._dependents(uid):
            self._foreground_release(uid)

    def _foreground_release(self, uid: str) -> None:
        res, ns, name = self._foreground.pop(uid)
        cur = self._table(res).get((ns, name))
        if cur is None:
            return
        new = copy.deepcopy(cur)
        new["metadata"]["finalizers"] = [f for f in cur["metadata"].get("finalizers") or [] if f != FOREGROUND_DELETION]
        if new["metadata"]["finalizers"]:
            self._store(res, new, "MODIFIED")
        else:
            self._store(res, new, "MODIFIED")
            self._delete(res, name, ns)

    def _delete_or_mark(self, res: Resource, name: str, namespace: str, propagation: str = "Background") -> dict:
        """DELETE as the API server does it: an object with finalizers is only marked
        (deletionTimestamp) and goes once its last finalizer is removed (see _update).
        ``propagationPolicy: Foreground`` adds the foregroundDeletion finalizer: the object stays
        until the garbage collector has deleted every dependent (including ones created after)."""
        key = (namespace if res.namespaced else "", name)
        cur = self._table(res)[key]
        if propagation == "Foreground" and not cur["metadata"].get("deletionTimestamp"):
            new = copy.deepcopy(cur)
            new["metadata"]["finalizers"] = list(cur["metadata"].get("finalizers") or []) + [FOREGROUND_DELETION]
            new["metadata"]["deletionTimestamp"] = _now()
            new["metadata"]["deletionGracePeriodSeconds"] = 0
            self._store(res, new, "MODIFIED")
            uid = new["metadata"]["uid"]
            self._foreground[uid] = (res, key[0], name)
            for dres, dns, dname in self._dependents(uid):
                if (dns, dname) in self._table(dres):
                    self._delete_or_mark(dres, dname, dns)
            self._foreground_check(uid)
            return self._table(res).get(key) or new
        if not cur["metadata"].get("finalizers"):
            return self._delete(res, name, namespace)
        if not cur["metadata"].get("deletionTimestamp"):
            new = copy.deepcopy(cur)
            new["metadata"]["deletionTimestamp"] = _now()
            new["metadata"]["deletionGracePeriodSeconds"] = 0
            self._store(res, new, "MODIFIED")
        return self._table(res)[key]

    async def _collect_later(self, uid: str) -> None:
        await asyncio.sleep(self.gc_delay)
        self._collect(uid)

    def _collect(self, uid: str) -> None:
        """Background cascading deletion of dependents (garbage collector)."""
        for res, ns, name in sorted(self._owned.pop(uid, ()), key=lambda k: (k[0].plural, k[1], k[2])):
            o = self._table(res).get((ns, name))
            if o is not None and any(r.get("uid") == uid for r in o.get("metadata", {}).get("ownerReferences") or []):
                self._delete_or_mark(res, name, ns)

    # ------------------------------------------------------------------------------------------
    # DaemonSet controller simulation
    # ------------------------------------------------------------------------------------------
    @staticmethod
    def _tolerated(taint: dict, tolerations: List[dict]) -> bool:
        """Kubernetes' toleration match: the effect (empty = any), then Exists (an empty key
        tolerates every taint) or Equal (the default) on key and value."""
        for t in tolerations:
            if t.get("effect") and t["effect"] != taint.get("effect"):
                continue
            if (t.get("operator") or "Equal") == "Exists":
                if not t.get("key") or t["key"] == taint.get("key"):
                    return True
            elif t.get("key") == taint.get("key") and (t.get("value") or "") == (taint.get("value") or ""):
                return True
        return False

    def _sync_daemonsets(self) -> None:
        nodes = list(self._table(kube.NODES).values())
        for (ns, name), ds in list(self._table(kube.DAEMONSETS).items()):
            pod_spec = ds["spec"]["template"]["spec"]
            sel = pod_spec.get("nodeSelector") or {}
            tols = pod_spec.get("tolerations") or []
            # The DaemonSet controller places a Pod where the selector matches and every
            # NoSchedule / NoExecute taint of the node is tolerated (PreferNoSchedule never blocks).
            matching = [n["metadata"]["name"] for n in nodes
                        if all((n["metadata"].get("labels") or {}).get(k) == v for k, v in sel.items())
                        and all(self._tolerated(t, tols) for t in (n.get("spec") or {}).get("taints") or []
                                if t.get("effect") in ("NoSchedule", "NoExecute"))
                        and _node_affinity_ok(n, pod_spec)]
            ready = sum(1 for n in matching if self.node_ready.get((f"{ns}/{name}", n)))
            st = {"currentNumberScheduled": len(matching), "desiredNumberScheduled": len(matching),
                  "numberMisscheduled": 0, "numberReady": ready,
                  "numberAvailable": ready, "observedGeneration": ds["metadata"].get("generation", 1)}
            if ds.get("status") != st:
                new = copy.deepcopy(ds)
                new["status"] = st
                self._store(kube.DAEMONSETS, new, "MODIFIED")
            self._sync_pods(ns, name, ds, matching)
            if self.agent_ready_delay is not None:
                for n in matching:
                    if (f"{ns}/{name}", n) not in self.node_ready:
                        self.node_ready[(f"{ns}/{name}", n)] = False
                        self._bg.append(asyncio.ensure_future(self._auto_ready(f"{ns}/{name}", n)))

    def _sync_pods(self, ns: str, name: str, ds: dict, nodes: List[str]) -> None:
        """One agent Pod per targeted node, owned by the DaemonSet, with a Ready condition that
        mirrors the agent's readinessProbe."""
        pods = self._table(kube.PODS)
        want = {f"{name}-{n}": n for n in nodes}
        for (pns, pname), p in list(pods.items()):
            refs = p["metadata"].get("ownerReferences") or []
            if pns == ns and any(r.get("uid") == ds["metadata"]["uid"] for r in refs) and pname not in want:
                self._delete(kube.PODS, pname, pns)
        for pname, node in want.items():
            ready = bool(self.node_ready.get((f"{ns}/{name}", node)))
            cur = pods.get((ns, pname))
            if cur is not None and not any(r.get("uid") == ds["metadata"]["uid"]
                                           for r in cur["metadata"].get("ownerReferences") or []):
                # The Pod of an earlier DaemonSet of this name that the collector has not reached
                # yet (Pod names here are <daemonset>-<node>, not random): it goes, ours comes.
                self._delete(kube.PODS, pname, ns)
                cur = None
            # lastTransitionTime moves only when the condition flips (the kubelet's status manager)
            old_ready = next((c for c in ((cur or {}).get("status") or {}).get("conditions") or []
                              if c.get("type") == "Ready"), None)
            since = old_ready.get("lastTransitionTime") if old_ready and \
                (old_ready.get("status") == "True") == ready else self._transition_time()
            cond = [{"type": "Ready", "status": "True" if ready else "False", "lastTransitionTime": since,
                     **({} if ready else {"reason": "ContainersNotReady",
                                          "message": "containers with unready status: [configurator]"})}]
            status = {"phase": "Running", "conditions": cond}
            last = self.node_last_exit.get((f"{ns}/{name}", node))
            cname = ((ds["spec"]["template"].get("spec") or {}).get("containers") or [{}])[0].get("name", "agent")
            if last:
                status["containerStatuses"] = [{"name": cname, "ready": ready, "restartCount": last["restartCount"],
                                                "lastState": {"terminated": last["terminated"]}}]
            else:  # the agent container started and has not exited (what the kubelet reports)
                status["containerStatuses"] = [{"name": cname, "ready": ready, "restartCount": 0,
                                                "state": {"running": {}}}]
            labels = dict((ds["spec"]["template"].get("metadata") or {}).get("labels") or {})
            if cur is None:
                pod = {"apiVersion": "v1", "kind": "Pod",
                       "metadata": {"name": pname, "namespace": ns, "labels": labels,
                                    "ownerReferences": [{"apiVersion": "apps/v1", "kind": "DaemonSet", "name": name,
                                                         "uid": ds["metadata"]["uid"], "controller": True}]},
                       "spec": self._pod_spec(ds, node), "status": status}
                self._create(kube.PODS, pod, ns)
            elif cur.get("status") != status:
                new = copy.deepcopy(cur)
                new["status"] = status
                self._store(kube.PODS, new, "MODIFIED")

    _DS_TOLERATIONS = [{"key": k, "operator": "Exists", "effect": e} for k, e in (
        ("node.kubernetes.io/not-ready", "NoExecute"), ("node.kubernetes.io/unreachable", "NoExecute"),
        ("node.kubernetes.io/disk-pressure", "NoSchedule"), ("node.kubernetes.io/memory-pressure", "NoSchedule"),
        ("node.kubernetes.io/pid-pressure", "NoSchedule"), ("node.kubernetes.io/unschedulable", "NoSchedule"),
        ("node.kubernetes.io/network-unavailable", "NoSchedule"))]

    def _pod_spec(self, ds: dict, node: str) -> dict:
        """What the DaemonSet controller and the API server put in a Pod: the template, the node
        affinity pin, the DaemonSet tolerations and the service-account token volume.  Real Pods
        are kilobytes each, and an operator caching them whole feels it at scale.  The template
        part is built once per DaemonSet generation and shared (stored objects are copied before
        any change, never mutated in place)."""
        key = (ds["metadata"].get("uid"), ds["metadata"].get("generation"))
        cache = self.__dict__.setdefault("_pod_spec_cache", {})
        if key not in cache:
            if len(cache) > 64:
                cache.clear()
            cache[key] = self._pod_spec_base(ds)
        spec = dict(cache[key])
        spec["nodeName"] = node
        spec["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {"nodeSelectorTerms": [
            {"matchFields": [{"key": "metadata.name", "operator": "In", "values": [node]}]}]}}}
        return spec

    @classmethod
    def _pod_spec_base(cls, ds: dict) -> dict:
        spec = copy.deepcopy(ds["spec"]["template"].get("spec") or {})
        spec["tolerations"] = list(spec.get("tolerations") or []) + [dict(t) for t in cls._DS_TOLERATIONS]
        spec.setdefault("volumes", []).append(
            {"name": "kube-api-access-x7k2p", "projected": {"defaultMode": 420, "sources": [
                {"serviceAccountToken": {"expirationSeconds": 3607, "path": "token"}},
                {"configMap": {"name": "kube-root-ca.crt", "items": [{"key": "ca.crt", "path": "ca.crt"}]}},
                {"downwardAPI": {"items": [{"path": "namespace", "fieldRef": {"apiVersion": "v1",
                                                                              "fieldPath": "metadata.namespace"}}]}}]}})
        spec.update(dnsPolicy="ClusterFirstWithHostNet", restartPolicy="Always", schedulerName="default-scheduler",
                    serviceAccountName=spec.get("serviceAccountName", "default"), enableServiceLinks=True,
                    preemptionPolicy="PreemptLowerPriority", priority=0)
        return spec

    def _transition_time(self) -> str:
        """RFC 3339 seconds like the API server, made unique per transition (a real cluster's
        transitions of one Pod are seconds apart; the tests' are milliseconds)."""
        import datetime

        self._transitions = getattr(self, "_transitions", 0) + 1
        t = datetime.datetime(2026, 1, 1, tzinfo=datetime.timezone.utc) + datetime.timedelta(seconds=self._transitions)
        return t.strftime("%Y-%m-%dT%H:%M:%SZ")

    async def _auto_ready(self, ds_key: str, node: str) -> None:
        await asyncio.sleep(self.agent_ready_delay or 0)
        if (ds_key, node) in self.node_ready:
            self.node_ready[(ds_key, node)] = True
            self._sync_daemonsets()

    # ------------------------------------------------------------------------------------------
    # HTTP routing
    # ------------------------------------------------------------------------------------------
    def _parse(self, path: str) -> Tuple[Optional[Resource], Optional[str], Optional[str], Optional[str]]:
        parts = [p for p in path.split("/") if p]
        if parts[:2] == ["api", "v1"]:
            group, version, rest = "", "v1", parts[2:]
        elif len(parts) >= 3 and parts[0] == "apis":
            group, version, rest = parts[1], parts[2], parts[3:]
        else:
            return None, None, None, None
        by_plural = {(r.group, r.version, r.plural): r for r in self.resources}
        ns = None
        if len(rest) >= 3 and rest[0] == "namespaces" and (group, version, rest[2]) in by_plural:
            ns, rest = rest[1], rest[2:]
        if not rest:
            return None, None, None, None
        res = by_plural.get((group, version, rest[0]))
        name = rest[1] if len(rest) > 1 else None
        sub = rest[2] if len(rest) > 2 else None
        return res, ns, name, sub

    async def _dispatch(self, req: web.Request) -> web.StreamResponse:
        resp = await self._serve(req)
        if req.method in ("POST", "PUT", "PATCH", "DELETE") and resp.status < 300:
            # When each write took effect, and whose it was: e.g. "no write of the old leader
            # lands after the new leader's first" (two-replica leader-election tests).
            self.writes.append((asyncio.get_event_loop().time(), req.headers.get("User-Agent", ""),
                                req.method, req.path))
        return resp

    async def _serve(self, req: web.Request) -> web.StreamResponse:
        path = req.path
        self.requests.append((req.method, path))
        for method, pattern, ua, seconds in list(self.stalls):
            if method in (req.method, "*") and pattern.search(path) and ua in (None, req.headers.get("User-Agent")):
                if self._unstall is None:
                    self._unstall = asyncio.Event()
                try:
                    await asyncio.wait_for(self._unstall.wait(), seconds)
                except asyncio.TimeoutError:
                    pass
        for f in list(self.faults):
            if f.method in (req.method, "*") and f.pattern.search(path) and \
                    f.user_agent in (None, req.headers.get("User-Agent")):
                f.count -= 1
                if f.count <= 0:
                    self.faults.remove(f)
                self.faults_fired += 1
                return _status(f.status, f.reason, "injected fault")
        try:
            if path == "/api":
                return web.json_response({"kind": "APIVersions", "versions": ["v1"]})
            if path == "/apis":
                return web.json_response(self._group_list())
            if path == "/version":
                return web.json_response({"major": "1", "minor": "31", "gitVersion": "v1.31.0-fake"})
            res, ns, name, sub = self._parse(path)
            if res is None:
                return self._discovery(path)
            verb = {"POST": "create", "PUT": "update", "PATCH": "patch", "DELETE": "delete"}.get(req.method)
            if verb is None:
                verb = "get" if name else ("watch" if req.query.get("watch") in ("true", "1") else "list")
            # RBAC audit: what a ServiceAccount making these requests would need.
            self.accesses.add((verb, res.group, res.plural + (f"/{sub}" if sub else "")))
            if res.namespaced and ns is None and req.method not in ("GET",):
                ns = None
            m = req.method
            if m == "GET" and name is None:
                if req.query.get("watch") in ("true", "1"):
                    return await self._watch(req, res, ns)
                return self._list(req, res, ns)
            if m == "GET":
                o = self._table(res).get((ns or "", name))
                if o is None:
                    return _status(404, "NotFound", f'{res.plural} "{name}" not found', {"name": name, "kind": res.plural})
                return web.json_response(o)
            if m == "POST":
                return await self._post(req, res, ns)
            if m == "PUT":
                return await self._put(req, res, ns, name, sub)
            if m == "PATCH":
                return await self._patch(req, res, ns, name, sub)
            if m == "DELETE":
                if (ns or "", name) not in self._table(res):
                    return _status(404, "NotFound", f'{res.plural} "{name}" not found')
                opts = {}
                if req.can_read_body:
                    try:
                        opts = json.loads(await req.text() or "{}")
                    except ValueError:
                        return _status(400, "BadRequest", "DeleteOptions are not JSON")
                propagation = (opts or {}).get("propagationPolicy") or req.query.get("propagationPolicy") or "Background"
                return web.json_response(self._delete_or_mark(res, name, ns or "", propagation))
            return _status(405, "MethodNotAllowed", m)
        except _Conflict as c:
            return _status(c.code, c.reason, c.message, c.details)
        except web.HTTPException as e:
            return _status(e.status, "Invalid" if e.status == 422 else "BadRequest", e.text or "")

    def _group_list(self) -> dict:
        groups: Dict[str, List[str]] = {}
        for r in self.resources:
            if r.group:
                groups.setdefault(r.group, [])
                if r.version not in groups[r.group]:
                    groups[r.group].append(r.version)
        for g in self.extra_groups:
            groups.setdefault(g, ["v1"])
        if self.openshift:
            groups.setdefault("route.openshift.io", ["v1"])
            groups.setdefault("security.openshift.io", ["v1"])
        return {"kind": "APIGroupList", "apiVersion": "v1", "groups": [
            {"name": g, "versions": [{"groupVersion": f"{g}/{v}", "version": v} for v in vs],
             "preferredVersion": {"groupVersion": f"{g}/{vs[0]}", "version": vs[0]}} for g, vs in sorted(groups.items())]}

    def _discovery(self, path: str) -> web.Response:
        parts = [p for p in path.split("/") if p]
        if parts == ["api", "v1"]:
            g, v = "", "v1"
        elif len(parts) == 3 and parts[0] == "apis":
            g, v = parts[1], parts[2]
        else:
            return _status(404, "NotFound", f"the server could not find the requested resource {path}")
        rs = [r for r in self.resources if r.group == g and r.version == v]
        if not rs:
            return _status(404, "NotFound", path)
        return web.json_response({"kind": "APIResourceList", "groupVersion": f"{g}/{v}" if g else v, "resources": [
            {"name": r.plural, "namespaced": r.namespaced, "kind": r.kind,
             "verbs": ["create", "delete", "get", "list", "patch", "update", "watch"]} for r in rs]})

    # -- LIST / WATCH ---------------------------------------------------------------------------
    def _list(self, req: web.Request, res: Resource, ns: Optional[str]) -> web.Response:
        """LIST, with the API server's chunking: ``limit`` items per page and an opaque
        ``continue`` token (here: the last key served) in ``metadata.continue``."""
        items = []
        limit = int(req.query.get("limit") or 0)
        after = None
        if req.query.get("continue"):
            after = tuple(json.loads(base64.urlsafe_b64decode(req.query["continue"].encode())))
        more = ""
        for key, o in sorted(self._table(res).items()):
            (ons, _) = key
            if after is not None and key <= after:
                continue
            if res.namespaced and ns and ons != ns:
                continue
            if req.query.get("labelSelector") and not match_labels(o["metadata"].get("labels") or {},
                                                                    req.query["labelSelector"]):
                continue
            if req.query.get("fieldSelector") and not _match_fields(o, req.query["fieldSelector"]):
                continue
            if limit and len(items) == limit:
                more = base64.urlsafe_b64encode(json.dumps(list(last)).encode()).decode()
                break
            items.append(o)
            last = key
        md = {"resourceVersion": str(self.rv)}
        if more:
            md["continue"] = more
        return web.json_response({"kind": res.kind + "List", "apiVersion": res.api_version, "metadata": md,
                                  "items": items})

    async def _watch(self, req: web.Request, res: Resource, ns: Optional[str]) -> web.StreamResponse:
        since = int(req.query.get("resourceVersion") or 0)
        timeout = float(req.query.get("timeoutSeconds") or 300)
        bookmarks = req.query.get("allowWatchBookmarks") in ("true", "1")
        resp = web.StreamResponse(headers={"Content-Type": "application/json"})
        await resp.prepare(req)
        if since and since < self.compacted_before - 1:
            err = {"type": "ERROR", "object": {"kind": "Status", "apiVersion": "v1", "status": "Failure", "code": 410,
                                                "reason": "Expired", "message": f"too old resource version: {since}"}}
            await resp.write((json.dumps(err) + "\n").encode())
            return resp
        w = _Watch(res, ns, req.query.get("labelSelector"), req.query.get("fieldSelector"))
        for rv, r, typ, obj in self.events:
            if r == res and rv > since and self._visible(w, obj):
                w.queue.put_nowait((typ, obj))
        self.watches.append(w)
        loop = asyncio.get_event_loop()
        end = loop.time() + timeout
        try:
            while not self._closing:
                remaining = end - loop.time()
                if remaining <= 0:
                    break
                try:
                    item = await asyncio.wait_for(w.queue.get(), timeout=min(remaining, self.bookmark_interval))
                except asyncio.TimeoutError:
                    if bookmarks:
                        bm = {"type": "BOOKMARK", "object": {"kind": res.kind, "apiVersion": res.api_version,
                                                             "metadata": {"resourceVersion": str(self.rv)}}}
                        await resp.write((json.dumps(bm) + "\n").encode())
                    continue
                if item is None:
                    break
                typ, obj = item
                await resp.write((json.dumps({"type": typ, "object": obj}) + "\n").encode())
        except (ConnectionResetError, asyncio.CancelledError):
            pass
        finally:
            if w in self.watches:
                self.watches.remove(w)
        return resp

    # -- admission ------------------------------------------------------------------------------
    async def _admit(self, res: Resource, op: str, obj: dict, old: Optional[dict]) -> dict:
        for cfg_res, mutating in ((kube.MUTATINGWEBHOOKS, True), (kube.VALIDATINGWEBHOOKS, False)):
            for cfg in list(self._table(cfg_res).values()):
                for wh in cfg.get("webhooks", []) or []:
                    if not any(self._rule_matches(rule, res, op) for rule in wh.get("rules", []) or []):
                        continue
                    cc = wh.get("clientConfig") or {}
                    url, unreachable = cc.get("url"), None
                    if not url:
                        url, unreachable = self._service_url(cc.get("service") or {})
                    self.admission_calls.append((wh.get("name", ""), op))
                    if unreachable:
                        if wh.get("failurePolicy", "Fail") == "Ignore":
                            continue
                        raise _Conflict(500, "InternalError", f'Internal error occurred: failed calling webhook '
                                                              f'"{wh.get("name")}": failed to call webhook: {unreachable}')
                    review = {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "request": {
                        "uid": str(uuid.uuid4()), "kind": {"group": res.group, "version": res.version, "kind": res.kind},
                        "resource": {"group": res.group, "version": res.version, "resource": res.plural},
                        "operation": op, "object": obj, "oldObject": old, "name": obj.get("metadata", {}).get("name")}}
                    ctx: Optional[ssl.SSLContext] = None
                    ca = cc.get("caBundle")
                    if url.startswith("https"):
                        ctx = ssl.create_default_context()
                        if cc.get("service"):
                            ctx.check_hostname = False  # endpoints are 127.0.0.1 here, not <svc>.<ns>.svc
                        if ca:
                            with tempfile.NamedTemporaryFile("wb", suffix=".pem", delete=False) as f:
                                f.write(base64.b64decode(ca))
                            ctx.load_verify_locations(f.name)
                    try:
                        async with aiohttp.ClientSession() as s:
                            async with s.post(url, json=review, ssl=ctx if ctx else False,
                                              timeout=aiohttp.ClientTimeout(total=10)) as r:
                                out = await r.json()
                    except Exception as e:
                        if wh.get("failurePolicy", "Fail") == "Ignore":
                            continue
                        raise _Conflict(500, "InternalError", f'failed calling webhook "{wh.get("name")}": {e}')
                    resp = out.get("response", {})
                    if not resp.get("allowed", False):
                        msg = (resp.get("status") or {}).get("message", "denied")
                        raise _Conflict(403, "Forbidden",
                                        f'admission webhook "{wh.get("name")}" denied the request: {msg}')
                    if mutating and resp.get("patch"):
                        obj = json_patch_apply(obj, json.loads(base64.b64decode(resp["patch"])))
        return obj

    def _service_url(self, svc: dict) -> Tuple[str, Optional[str]]:
        """A service-referenced webhook, the way the API server reaches it: the Service must exist
        and have a ready endpoint (``service_endpoints``, set by the test when the operator pod
        is serving); otherwise the call fails and ``failurePolicy`` decides."""
        ns, name, path = svc.get("namespace", ""), svc.get("name", ""), svc.get("path", "/")
        port = svc.get("port", 443)
        shown = f'Post "https://{name}.{ns}.svc:{port}{path}?timeout=10s"'
        if (ns, name) not in self._table(kube.SERVICES):
            return "", f'{shown}: service "{name}" not found'
        base = self.service_endpoints.get((ns, name))
        if not base:
            return "", f'{shown}: no endpoints available for service "{name}"'
        return base.rstrip("/") + path, None

    @staticmethod
    def _rule_matches(rule: dict, res: Resource, op: str) -> bool:
        def ok(vals, v):
            return "*" in (vals or []) or v in (vals or [])
        return (ok(rule.get("apiGroups"), res.group) and ok(rule.get("apiVersions"), res.version)
                and ok(rule.get("operations"), op) and ok(rule.get("resources"), res.plural))

    def _validate_schema(self, res: Resource, obj: dict) -> dict:
        if res != kube.NETWORKCLUSTERPOLICIES:
            return obj
        errs = CRD.validate(obj)
        if errs:
            raise _Conflict(422, "Invalid", f'{T.KIND} "{obj.get("metadata", {}).get("name")}" is invalid: '
                            + "; ".join(errs), {"causes": [{"message": e} for e in errs]})
        schema = CRD.openapi_schema()
        pruned = CRD.apply_defaults(CRD.prune(obj, schema), schema)
        pruned["metadata"] = obj["metadata"]
        return pruned

    # -- writes ---------------------------------------------------------------------------------
    async def _body(self, req: web.Request) -> dict:
        try:
            return await req.json()
        except json.JSONDecodeError:
            raise web.HTTPBadRequest(text="invalid JSON body")

    async def _post(self, req: web.Request, res: Resource, ns: Optional[str]) -> web.Response:
        obj = await self._body(req)
        if res == kube.TOKENREVIEWS:
            info = self.tokens.get(obj.get("spec", {}).get("token", ""))
            obj["status"] = ({"authenticated": True, "user": {"username": info["username"], "groups": info.get("groups", [])}}
                             if info else {"authenticated": False})
            return web.json_response(obj, status=201)
        if res == kube.SUBJECTACCESSREVIEWS:
            user = obj.get("spec", {}).get("user")
            allowed = any(i["username"] == user and i.get("allowed") for i in self.tokens.values())
            obj["status"] = {"allowed": allowed}
            return web.json_response(obj, status=201)
        obj = self._validate_schema(res, obj)
        obj = await self._admit(res, "CREATE", obj, None)
        obj = self._validate_schema(res, obj)
        created = self._create(res, obj, ns)
        return web.json_response(created, status=201)

    def _update(self, res: Resource, ns: Optional[str], name: str, sub: Optional[str], new: dict) -> dict:
        key = (ns or "" if res.namespaced else "", name)
        cur = self._table(res).get(key)
        if cur is None:
            raise _Conflict(404, "NotFound", f'{res.plural} "{name}" not found')
        want_rv = new.get("metadata", {}).get("resourceVersion")
        if want_rv and want_rv != cur["metadata"]["resourceVersion"]:
            raise _Conflict(409, "Conflict", f'Operation cannot be fulfilled on {res.plural} "{name}": the object has '
                                             "been modified; please apply your changes to the latest version and try again")
        out = copy.deepcopy(cur)
        if sub == "status":
            out["status"] = copy.deepcopy(new.get("status"))
        else:
            for k, v in new.items():
                if k in ("metadata", "status"):
                    continue
                out[k] = copy.deepcopy(v)
            for k in list(out):
                if k not in new and k not in ("metadata", "status", "apiVersion", "kind"):
                    del out[k]
            md_new = new.get("metadata", {})
            for k in ("labels", "annotations", "ownerReferences", "finalizers"):
                if k in md_new:
                    out["metadata"][k] = copy.deepcopy(md_new[k])
                else:
                    out["metadata"].pop(k, None)
            if res not in self.STATUS_SUBRESOURCE and "status" in new:
                out["status"] = copy.deepcopy(new["status"])
            if out.get("spec") != cur.get("spec"):
                out["metadata"]["generation"] = cur["metadata"].get("generation", 1) + 1
        if out == cur:
            return cur  # no-op: resourceVersion unchanged, no event
        if cur["metadata"].get("deletionTimestamp") and not out["metadata"].get("finalizers"):
            self._store(res, out, "MODIFIED")
            return self._delete(res, name, key[0])  # the last finalizer is gone
        self._store(res, out, "MODIFIED")
        if res in (kube.DAEMONSETS, kube.NODES) and sub != "status":
            self._sync_daemonsets()
        return self._table(res)[key]

    async def _put(self, req: web.Request, res: Resource, ns: Optional[str], name: str, sub: Optional[str]) -> web.Response:
        new = await self._body(req)
        if sub is None:
            new = self._validate_schema(res, new)
            cur = self._table(res).get((ns or "" if res.namespaced else "", name))
            if cur is not None and res == kube.NETWORKCLUSTERPOLICIES:
                new = await self._admit(res, "UPDATE", new, cur)
                new = self._validate_schema(res, new)
        return web.json_response(self._update(res, ns, name, sub, new))

    async def _patch(self, req: web.Request, res: Resource, ns: Optional[str], name: str, sub: Optional[str]) -> web.Response:
        cur = self._table(res).get((ns or "" if res.namespaced else "", name))
        if cur is None:
            return _status(404, "NotFound", f'{res.plural} "{name}" not found')
        patch = await self._body(req)
        ct = req.headers.get("Content-Type", "")
        try:
            if "json-patch" in ct:
                new = json_patch_apply(cur, patch)
            else:
                new = merge_patch(cur, patch)
        except (ValueError, KeyError, IndexError) as e:
            return _status(422, "Invalid", f"patch failed: {e}")
        new.setdefault("metadata", {})["resourceVersion"] = cur["metadata"]["resourceVersion"]
        if sub is None:
            new = self._validate_schema(res, new)
        return web.json_response(self._update(res, ns, name, sub, new))


class _Conflict(Exception):
    def __init__(self, code: int, reason: str, message: str, details: Optional[dict] = None):
        super().__init__(message)
        self.code, self.reason, self.message, self.details = code, reason, message, details
