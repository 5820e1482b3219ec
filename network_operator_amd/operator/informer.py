"""List-and-watch informer with a local cache and field indexes.

controller-runtime's cache, reduced to what the reconciler needs (reference
internal/controller/networkconfiguration_controller.go:364-404 registers a field index
``.metadata.controller`` on DaemonSets and reads through the cache):

* initial LIST, then WATCH from the list's resourceVersion; bookmarks advance it;
* 410 Gone (compacted history) -> relist and emit synthetic adds/updates/deletes for the diff;
* any other stream end -> reconnect with jittered backoff;
* ``add_index(name, fn)`` / ``by_index(name, value)`` for owner lookups;
* ``transform``: what is cached (client-go's SetTransform), e.g. ``slim_pod``: one agent Pod per
  node and policy is tens of thousands of Pods on a large cluster, and a full Pod object
  (containers, volumes, tolerations, managedFields) costs kilobytes of Python heap each.
"""

from __future__ import annotations

import asyncio
import logging
import random
import sys
from typing import Awaitable, Callable, Dict, List, Optional

from .kube import ApiClient, ApiError, Resource, is_gone

log = logging.getLogger("informer")

Handler = Callable[[str, dict, Optional[dict]], Awaitable[None]]  # (event, obj, old)


def obj_key(obj: dict) -> str:
    md = obj.get("metadata", {})
    ns = md.get("namespace")
    return f"{ns}/{md['name']}" if ns else md["name"]


# (labels: the informers select on them server-side; nothing reads them from the cache)
_POD_META = ("name", "namespace", "uid", "resourceVersion", "ownerReferences", "deletionTimestamp")
_CONTAINER_STATUS = ("name", "ready", "restartCount", "state", "lastState")


def _shared(v):
    """Interns the keys and short string values of a slimmed object: tens of thousands of cached
    Pods and Jobs repeat the same namespace, owner uid, kind, annotation keys and condition
    types, and each JSON decode makes its own copies."""
    if isinstance(v, str):
        return sys.intern(v) if len(v) <= 96 else v
    if isinstance(v, dict):
        return {sys.intern(k): _shared(x) for k, x in v.items()}
    if isinstance(v, list):
        return [_shared(x) for x in v]
    return v


def _slim_meta(md: dict, keys) -> dict:
    out = {k: md[k] for k in keys if k in md}
    if "ownerReferences" in out:
        out["ownerReferences"] = [{k: r[k] for k in ("apiVersion", "kind", "name", "uid", "controller") if k in r}
                                  for r in out["ownerReferences"]]
    return out


def slim_pod(pod: dict) -> dict:
    """The fields the operator reads from a Pod (node, Ready condition, phase / admission reason,
    container exit records, owner), nothing else."""
    md = pod.get("metadata") or {}
    st = pod.get("status") or {}
    out_st = {k: st[k] for k in ("phase", "reason", "message") if k in st}
    conds = [c for c in st.get("conditions") or [] if c.get("type") == "Ready"]
    if conds:
        out_st["conditions"] = conds
    cs = [{k: c[k] for k in _CONTAINER_STATUS if k in c} for c in st.get("containerStatuses") or []]
    if cs:
        out_st["containerStatuses"] = cs
    return _shared({"apiVersion": pod.get("apiVersion", "v1"), "kind": pod.get("kind", "Pod"),
                    "metadata": _slim_meta(md, _POD_META),
                    "spec": {"nodeName": (pod.get("spec") or {}).get("nodeName", "")}, "status": out_st})


_JOB_META = _POD_META + ("annotations",)


def slim_job(job: dict) -> dict:
    """A Job as the reconciler reads it: identity, owner, its node / generation / epoch
    annotations and the outcome (succeeded / failed counts, Complete / Failed conditions)."""
    md = job.get("metadata") or {}
    st = job.get("status") or {}
    return _shared({"apiVersion": job.get("apiVersion", "batch/v1"), "kind": job.get("kind", "Job"),
            "metadata": _slim_meta(md, _JOB_META),
            "status": {k: st[k] for k in ("succeeded", "failed", "active") if k in st} |
            ({"conditions": [{k: c[k] for k in ("type", "status", "lastTransitionTime") if k in c}
                             for c in st["conditions"]]} if st.get("conditions") else {})})


def slim_event(ev: dict) -> dict:
    """A kubelet probe Event: what it is about, its message and when."""
    io = ev.get("involvedObject") or {}
    return _shared({"apiVersion": "v1", "kind": "Event",
                    "metadata": _slim_meta(ev.get("metadata") or {}, ("name", "namespace", "uid", "resourceVersion")),
                    "involvedObject": {k: io[k] for k in ("kind", "name", "namespace") if k in io},
                    "reason": ev.get("reason", ""), "message": ev.get("message", ""),
                    "lastTimestamp": ev.get("lastTimestamp") or ev.get("eventTime") or "",
                    "count": ev.get("count", 1)})


def controller_of(obj: dict) -> Optional[dict]:
    """metav1.GetControllerOf."""
    for ref in obj.get("metadata", {}).get("ownerReferences", []) or []:
        if ref.get("controller"):
            return ref
    return None


class Informer:
    def __init__(self, client: ApiClient, res: Resource, namespace: Optional[str] = None,
                 label_selector: Optional[str] = None, resync_timeout: int = 300,
                 transform: Optional[Callable[[dict], dict]] = None,
                 keep: Optional[Callable[[dict], bool]] = None, field_selector: Optional[str] = None):
        self.client = client
        self.transform = transform
        # Objects failing `keep` are not cached (as if deleted): e.g. only the failed Pods of the
        # validation Jobs, the ones whose admission reason matters.
        self.keep = keep
        self.res = res
        self.namespace = namespace
        self.label_selector = label_selector
        self.field_selector = field_selector
        self.resync_timeout = resync_timeout
        self.store: Dict[str, dict] = {}
        self.resource_version: Optional[str] = None
        self.handlers: List[Handler] = []
        self.synced = asyncio.Event()
        self._indexers: Dict[str, Callable[[dict], List[str]]] = {}
        self._indexes: Dict[str, Dict[str, set]] = {}
        self._task: Optional[asyncio.Task] = None
        self.relists = 0
        self.watch_restarts = 0

    # -- indexes ---------------------------------------------------------------------------------
    def add_index(self, name: str, fn: Callable[[dict], List[str]]) -> None:
        self._indexers[name] = fn
        idx: Dict[str, set] = {}
        for k, o in self.store.items():
            for v in fn(o) or []:
                idx.setdefault(v, set()).add(k)
        self._indexes[name] = idx

    def by_index(self, name: str, value: str) -> List[dict]:
        return [self.store[k] for k in sorted(self._indexes.get(name, {}).get(value, ())) if k in self.store]

    def _index_remove(self, key: str, obj: dict) -> None:
        for name, fn in self._indexers.items():
            for v in fn(obj) or []:
                s = self._indexes[name].get(v)
                if s:
                    s.discard(key)
                    if not s:
                        del self._indexes[name][v]

    def _index_add(self, key: str, obj: dict) -> None:
        for name, fn in self._indexers.items():
            for v in fn(obj) or []:
                self._indexes[name].setdefault(v, set()).add(key)

    # -- store -----------------------------------------------------------------------------------
    def get(self, name: str, namespace: Optional[str] = None) -> Optional[dict]:
        return self.store.get(f"{namespace}/{name}" if namespace else name)

    def list(self) -> List[dict]:
        return list(self.store.values())

    def add_handler(self, h: Handler) -> None:
        self.handlers.append(h)

    async def _emit(self, ev: str, obj: dict, old: Optional[dict] = None) -> None:
        for h in self.handlers:
            try:
                await h(ev, obj, old)
            except Exception:  # a handler must never kill the informer
                log.exception("informer handler failed")

    async def _apply(self, ev: str, obj: dict) -> None:
        if self.keep is not None and ev != "DELETED" and not self.keep(obj):
            if obj_key(obj) not in self.store:
                return
            ev = "DELETED"
        if self.transform is not None:
            obj = self.transform(obj)
        key = obj_key(obj)
        old = self.store.get(key)
        if ev == "DELETED":
            if old is not None:
                self._index_remove(key, old)
                del self.store[key]
            await self._emit("DELETED", obj, old)
            return
        if old is not None:
            self._index_remove(key, old)
        self.store[key] = obj
        self._index_add(key, obj)
        await self._emit("ADDED" if old is None else "MODIFIED", obj, old)

    async def _relist(self) -> None:
        lst = await self.client.list(self.res, self.namespace, label_selector=self.label_selector,
                                     field_selector=self.field_selector)
        self.relists += 1
        fresh = {obj_key(o): o for o in lst.get("items", [])}
        for key in list(self.store):
            if key not in fresh:
                await self._apply("DELETED", self.store[key])
        for key, o in fresh.items():
            o.setdefault("apiVersion", self.res.api_version)
            o.setdefault("kind", self.res.kind)
            old = self.store.get(key)
            if old is None or old.get("metadata", {}).get("resourceVersion") != o["metadata"].get("resourceVersion"):
                await self._apply("MODIFIED" if old else "ADDED", o)
        self.resource_version = lst.get("metadata", {}).get("resourceVersion")
        self.synced.set()

    async def run(self) -> None:
        backoff = 0.05
        need_list = True
        while True:
            try:
                if need_list:
                    await self._relist()
                    need_list = False
                async for ev, obj in self.client.watch(self.res, self.namespace, self.resource_version,
                                                       timeout_seconds=self.resync_timeout,
                                                       label_selector=self.label_selector,
                                                       field_selector=self.field_selector):
                    rv = obj.get("metadata", {}).get("resourceVersion")
                    if ev == "BOOKMARK":
                        self.resource_version = rv
                        continue
                    await self._apply(ev, obj)
                    if rv:
                        self.resource_version = rv
                backoff = 0.05
                self.watch_restarts += 1
            except asyncio.CancelledError:
                raise
            except ApiError as e:
                if is_gone(e):
                    need_list = True
                    continue
                log.warning("watch %s failed: %s", self.res.plural, e)
                await asyncio.sleep(backoff * (1 + random.random()))
                backoff = min(backoff * 2, 5.0)
                need_list = True
            except Exception as e:  # connection errors
                log.warning("watch %s interrupted: %s", self.res.plural, e)
                await asyncio.sleep(backoff * (1 + random.random()))
                backoff = min(backoff * 2, 5.0)

    def start(self) -> asyncio.Task:
        if self._task is None or self._task.done():
            self._task = asyncio.ensure_future(self.run())
        return self._task

    async def stop(self) -> None:
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except (asyncio.CancelledError, Exception):
                pass
