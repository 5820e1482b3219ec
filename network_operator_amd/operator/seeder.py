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
  annotations;
* deletes its own policies that left the file (``config.amd.enabled=false`` on upgrade);
* makes each policy a dependent of a release-owned, cluster-scoped anchor (``--policies-owner``,
  the chart's operator ClusterRole), so ``helm uninstall`` garbage-collects the policies and
  then their DaemonSets, as uninstalling the reference's release deletes its CR.

Ownership is release-scoped, never decided by the generic ``app.kubernetes.io/managed-by``
label (a user who copies a seeded policy's YAML copies that label too, and a second release or a
dev operator on the same cluster carries the same one).  A policy is this seeder's when

* with ``--policies-owner``: its ownerReferences hold *this* anchor's uid (a ClusterRole of
  another release has another uid; a copied policy has no reference, or a stale one);
* without an owner: it carries ``amd.com/policy-seeder: <seed id>`` with this operator's id
  (``--policies-seed-id``, default ``<namespace>.<leader election id>``).

Anything else of the same name is left alone, with a warning.  While the anchor is missing
(an uninstall in progress) the seeder writes nothing: it could neither prove ownership nor give
a new policy an owner the garbage collector will honour.
"""

from __future__ import annotations

import asyncio
import copy
import hashlib
import logging
import re
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
SEEDER_KEY = "amd.com/policy-seeder"


def seed_id_label(seed_id: str) -> str:
    """A label value (<= 63 chars of [A-Za-z0-9._-], alphanumeric at both ends) naming one
    operator instance; long or odd ids are shortened with a hash, so distinct ids stay distinct."""
    v = re.sub(r"[^A-Za-z0-9._-]", "-", seed_id).strip("-._")
    if v != seed_id or len(v) > 63:
        h = hashlib.sha256(seed_id.encode()).hexdigest()[:10]
        v = (v[:52].strip("-._") + "-" + h).strip("-._")
    return v or "default"
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
                 max_backoff: float = 10.0, metrics=None, seed_id: str = "default"):
        self.client, self.path, self.interval, self.max_backoff = client, path, interval, max_backoff
        self.owner = owner  # "ClusterRole/<name>" or ""
        self.seed_id = seed_id_label(seed_id)
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

    def _ours(self, obj: dict, ref: Optional[dict]) -> bool:
        """Release-scoped ownership (module docstring): the anchor's uid when there is an owner,
        this operator's seeder id otherwise.  The generic managed-by label never decides."""
        md = obj.get("metadata", {})
        if self.owner:
            return ref is not None and any(r.get("uid") == ref["uid"] for r in md.get("ownerReferences") or [])
        return (md.get("labels") or {}).get(SEEDER_KEY) == self.seed_id

    async def sync_once(self) -> bool:
        """One pass; True when the cluster matches the file (or there is no file)."""
        want = load_policies(self.path)
        if want is None:
            return True
        ref = await self._owner_reference()
        if self.owner and ref is None:
            log.info("policies owner %s not found (uninstall in progress?): nothing seeded this pass", self.owner)
            return True
        P = kube.NETWORKCLUSTERPOLICIES
        names = set()
        for pol in want:
            name = pol["metadata"]["name"]
            names.add(name)
            desired = copy.deepcopy(pol)
            desired["metadata"]["labels"][SEEDER_KEY] = self.seed_id
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
            if not self._ours(cur, ref):
                log.warning("policy %s exists and is not this operator's (%s): left as it is", name,
                            f"owner {self.owner}" if self.owner else f"{SEEDER_KEY}={self.seed_id}")
                continue
            if cur["metadata"].get("deletionTimestamp"):
                # Being deleted (by hand, or its nodes are being cleaned): editing its spec would
                # restart agents on nodes the finalizer is cleaning.  It is created anew once gone.
                log.info("policy %s is being deleted: it is seeded again once it is gone", name)
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
        listed = await self.client.list(P, label_selector=None if self.owner else f"{SEEDER_KEY}={self.seed_id}")
        for cur in listed.get("items") or []:
            name = cur["metadata"]["name"]
            if name not in names and self._ours(cur, ref):
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
