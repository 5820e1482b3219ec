"""Policies from the Helm release, created by the operator once its own webhook serves.

The reference chart renders its NetworkClusterPolicy as a plain release object
(reference charts/network-operator/templates/gaudi.yaml:1-22, installed with
``helm install ... --set config.gaudi.enabled=true``, README.md:22-26).  That only works because
the reference registers its admission webhooks for the singular resource, so the API server never
calls them (reference charts/network-operator/templates/webhooks.yaml:26,54).  This operator's
webhooks match the real plural and fail closed.  A policy applied in the same release would
therefore reach the API server before the operator pod and its cert-manager certificate exist,
and ``helm install`` would fail with "failed calling webhook".

So the chart renders its policies into a ConfigMap mounted into the operator
(``--policies-file``).  The leader applies them through the API server, which admits them
through the operator's own webhooks, once that server is up.  The seeder repeats this every
``interval`` so a ``helm upgrade`` converges.  A create that fails before the webhook Service has
endpoints is retried with backoff.  The seeder:

* creates missing policies and brings changed ones back to the file's spec, labels and
  annotations; it only touches policies carrying ``app.kubernetes.io/managed-by: amd-network-
  operator`` (a user's policy of the same name is left alone, with a warning);
* deletes managed policies that left the file (``config.amd.enabled=false`` on upgrade);
* makes each policy a dependent of a release-owned, cluster-scoped anchor (``--policies-owner``,
  the chart's operator ClusterRole), so ``helm uninstall`` garbage-collects the policies and
  then their DaemonSets, as uninstalling the reference's release deletes its CR.
"""

from __future__ import annotations

import asyncio
import copy
import logging
from pathlib import Path
from typing import List, Optional

import yaml

from ..api.v1alpha1 import types as T
from ..api.v1alpha1 import webhook as W
from . import kube
from .kube import ApiClient, ApiError, is_not_found

log = logging.getLogger("seeder")

MANAGED_BY_KEY = "app.kubernetes.io/managed-by"
MANAGED_BY = "amd-network-operator"
OWNER_KINDS = {"ClusterRole": kube.CLUSTERROLES}


def load_policies(path: str) -> Optional[List[dict]]:
    """The file's policies; None when the file is absent (seeding not configured / ConfigMap not
    yet projected), [] when it lists none.  Raises ValueError on a malformed file."""
    p = Path(path)
    if not p.exists():
        return None
    doc = yaml.safe_load(p.read_text()) or {}
    items = doc.get("policies") if isinstance(doc, dict) else None
    if items is None:
        return []
    if not isinstance(items, list):
        raise ValueError(f"{path}: 'policies' must be a list")
    out = []
    for i, item in enumerate(items):
        if not isinstance(item, dict) or not (item.get("metadata") or {}).get("name"):
            raise ValueError(f"{path}: policies[{i}] has no metadata.name")
        # Normalised and defaulted exactly as the mutating webhook will (unknown fields kept), so
        # the stored object compares equal and a steady state issues no updates.
        pol = W.default(T.NetworkClusterPolicy.from_dict(item)).to_dict()
        pol["apiVersion"], pol["kind"] = T.API_VERSION, T.KIND
        md = pol.setdefault("metadata", {})
        md["labels"] = dict(md.get("labels") or {}, **{MANAGED_BY_KEY: MANAGED_BY})
        out.append(pol)
    return out


class PolicySeeder:
    def __init__(self, client: ApiClient, path: str, owner: str = "", interval: float = 10.0,
                 max_backoff: float = 10.0, metrics=None):
        self.client, self.path, self.interval, self.max_backoff = client, path, interval, max_backoff
        self.owner = owner  # "ClusterRole/<name>" or ""
        self.metrics = metrics
        self.applied = 0    # successful sync passes (tests, metrics)
        self.writes = 0     # creates + updates + deletes issued
        self.last_error = ""

    async def _owner_reference(self) -> Optional[dict]:
        if not self.owner:
            return None
        kind, _, name = self.owner.partition("/")
        res = OWNER_KINDS.get(kind)
        if res is None or not name:
            raise ValueError(f"--policies-owner {self.owner!r}: want ClusterRole/<name>")
        try:
            o = await self.client.get(res, name)
        except ApiError as e:
            if is_not_found(e):  # uninstall in progress: no new links to a vanishing anchor
                return None
            raise
        return {"apiVersion": res.api_version, "kind": res.kind, "name": name, "uid": o["metadata"]["uid"]}

    @staticmethod
    def _managed(obj: dict) -> bool:
        return (obj.get("metadata", {}).get("labels") or {}).get(MANAGED_BY_KEY) == MANAGED_BY

    async def sync_once(self) -> bool:
        """One pass; True when the cluster matches the file (or there is no file)."""
        want = load_policies(self.path)
        if want is None:
            return True
        ref = await self._owner_reference()
        P = kube.NETWORKCLUSTERPOLICIES
        names = set()
        for pol in want:
            name = pol["metadata"]["name"]
            names.add(name)
            desired = copy.deepcopy(pol)
            if ref:
                desired["metadata"]["ownerReferences"] = [ref]
            try:
                cur = await self.client.get(P, name)
            except ApiError as e:
                if not is_not_found(e):
                    raise
                await self.client.create(P, desired)
                self.writes += 1
                log.info("created policy %s from %s", name, self.path)
                continue
            if not self._managed(cur):
                log.warning("policy %s exists and is not managed by the operator: left as it is", name)
                continue
            new = copy.deepcopy(cur)
            new["spec"] = desired.get("spec", {})
            md = new["metadata"]
            md["labels"] = dict(md.get("labels") or {}, **desired["metadata"]["labels"])
            if desired["metadata"].get("annotations"):
                md["annotations"] = dict(md.get("annotations") or {}, **desired["metadata"]["annotations"])
            if ref:
                others = [r for r in md.get("ownerReferences") or [] if r.get("kind") != ref["kind"]
                          or r.get("name") != ref["name"]]
                md["ownerReferences"] = others + [ref]
            if new != cur:
                await self.client.replace(P, new)
                self.writes += 1
                log.info("updated policy %s from %s", name, self.path)
        listed = await self.client.list(P, label_selector=f"{MANAGED_BY_KEY}={MANAGED_BY}")
        for cur in listed.get("items") or []:
            name = cur["metadata"]["name"]
            if name not in names:
                try:
                    await self.client.delete(P, name)
                    self.writes += 1
                    log.info("deleted policy %s (no longer in %s)", name, self.path)
                except ApiError as e:
                    if not is_not_found(e):
                        raise
        return True

    async def run(self, stop: asyncio.Event) -> None:
        backoff = 0.2
        while not stop.is_set():
            try:
                await self.sync_once()
                self.applied += 1
                self.last_error = ""
                if self.metrics is not None:
                    self.metrics.seed_in_sync.set(1)
                backoff = 0.2
                delay = self.interval
            except Exception as e:  # webhook endpoint not up yet, API hiccup, bad file
                msg = str(e)
                if self.metrics is not None:
                    self.metrics.seed_in_sync.set(0)
                    self.metrics.seed_errors.inc()
                if msg != self.last_error:
                    log.warning("applying %s failed (retrying): %s", self.path, msg)
                self.last_error = msg
                delay, backoff = backoff, min(backoff * 2, self.max_backoff)
            try:
                await asyncio.wait_for(stop.wait(), timeout=delay)
            except asyncio.TimeoutError:
                pass
