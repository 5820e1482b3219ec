"""Lease-based leader election (coordination.k8s.io/v1), client-go ``leaderelection`` semantics.

The reference manager enables it with ``--leader-elect`` and ID ``9a8a7ba6.intel.com``
(reference cmd/operator/main.go:98-100,174-175).  Here: ID ``9a8a7ba6.amd.com``, lease
duration 15 s, renew deadline 10 s, retry period 2 s (controller-runtime defaults).
Expiry is judged on the *locally observed* time of the last record change, as client-go
does, so clock skew between replicas does not matter.

Safety of the renew loop (client-go's ``renew``: ``PollImmediateUntil(retryPeriod, ...,
timeoutCtx(renewDeadline))``): another replica may take the lease ``lease_duration`` after it
last saw it change, i.e. no earlier than our last successful renewal + ``lease_duration``.  So
every renewal attempt -- and every API request inside it -- is bounded by what is left of
``renew_deadline`` since that renewal (each request by at most ``retry_period`` as well), and
when the deadline passes the leader's work is cancelled at once.  A replica whose API calls
stall therefore stops reconciling ``lease_duration - renew_deadline`` (5 s by default) before
anyone else can legally lead.

Order on loss: the leader's work -- which owns the reconcile workers --
is cancelled and awaited first, then ``on_stopped_leading`` runs, and only then is the lease
released, with ONE attempt bounded by ``retry_period`` (a stalled API cannot hold the stop up
behind GET + PUT round trips).  The time from the deadline to the last worker gone is kept in
``stop_latency``; ``STOP_BUDGET_S`` is what the manager's flag check reserves for it out of
``lease_duration - renew_deadline``.  (client-go releases in ``renew()`` before its
``OnStoppedLeading``; controller-runtime then exits 1 -- reference cmd/operator/main.go:229-232.)
"""

from __future__ import annotations

import asyncio
import datetime as dt
import logging
import math
import os
import socket
import uuid
from typing import Awaitable, Callable, Optional

from . import kube
from .kube import ApiClient, ApiError, is_already_exists, is_conflict, is_not_found

log = logging.getLogger("leaderelection")

DEFAULT_LEASE_ID = "9a8a7ba6.amd.com"
# Seconds reserved between the renew deadline and the lease's expiry for the leader's work to be
# cancelled (workers, seeder) and for a write already on the wire to land.  Cancelling is
# immediate in asyncio; the measured stop is milliseconds (``LeaderElector.stop_latency``).
STOP_BUDGET_S = 1.0


def unsafe_timings(lease_duration: float, renew_deadline: float, retry_period: float) -> str:
    """Why these leader-election timings are unsafe, or "" when they are safe: the order
    client-go requires, plus a margin of more than STOP_BUDGET_S between the renew deadline
    (when a stalled leader stops) and the lease duration (when a standby may take over)."""
    if not (lease_duration > renew_deadline > retry_period > 0):
        return "leader election needs lease duration > renew deadline > retry period > 0"
    if lease_duration - renew_deadline <= STOP_BUDGET_S:
        return (f"lease duration - renew deadline = {lease_duration - renew_deadline:g}s leaves no room for the "
                f"leader to stop ({STOP_BUDGET_S:g}s) before a standby may take over")
    return ""


def _now_str() -> str:
    return dt.datetime.now(dt.timezone.utc).strftime("%Y-%m-%dT%H:%M:%S.%fZ")


def default_identity() -> str:
    """``<pod>_<uuid>`` as controller-runtime builds it: the pod name (``POD_NAME`` from the
    downward API, else the hostname, which is the pod name in a pod)."""
    return f"{os.environ.get('POD_NAME') or socket.gethostname()}_{uuid.uuid4()}"


class LeaderElector:
    def __init__(self, client: ApiClient, namespace: str, name: str = DEFAULT_LEASE_ID,
                 identity: Optional[str] = None, lease_duration: float = 15.0, renew_deadline: float = 10.0,
                 retry_period: float = 2.0, release_on_cancel: bool = True, clock=None):
        self.client = client
        self.namespace = namespace
        self.name = name
        self.identity = identity or default_identity()
        self.lease_duration = lease_duration
        self.renew_deadline = renew_deadline
        self.retry_period = retry_period
        self.release_on_cancel = release_on_cancel
        self._loop_time = clock or (lambda: asyncio.get_event_loop().time())
        self._observed_record: Optional[dict] = None
        self._observed_time = 0.0
        self.is_leader = False
        self.transitions = 0
        self.lost_at: Optional[float] = None  # loop time at which leadership was given up
        self.stop_latency: Optional[float] = None  # seconds from lost_at until the work had ended
        self.work_stopped = True  # the leader's work ended within STOP_BUDGET_S of the stop

    def _lease_body(self, prev: Optional[dict]) -> dict:
        spec_prev = (prev or {}).get("spec", {}) or {}
        same_holder = spec_prev.get("holderIdentity") == self.identity
        transitions = int(spec_prev.get("leaseTransitions", 0) or 0) + (0 if same_holder or not prev else 1)
        body = {
            "apiVersion": "coordination.k8s.io/v1", "kind": "Lease",
            "metadata": {"name": self.name, "namespace": self.namespace},
            "spec": {"holderIdentity": self.identity, "leaseDurationSeconds": max(1, math.ceil(self.lease_duration)),
                     "acquireTime": spec_prev.get("acquireTime") if same_holder else _now_str(),
                     "renewTime": _now_str(), "leaseTransitions": transitions},
        }
        if prev:
            body["metadata"]["resourceVersion"] = prev["metadata"].get("resourceVersion")
        return body

    def _request_timeout(self) -> float:
        return self.retry_period

    async def try_acquire_or_renew(self) -> bool:
        t = self._request_timeout()
        try:
            lease = await self.client.get(kube.LEASES, self.name, self.namespace, timeout=t)
        except ApiError as e:
            if not is_not_found(e):
                log.warning("error retrieving lease %s: %s", self.name, e)
                return False
            try:
                await self.client.create(kube.LEASES, self._lease_body(None), namespace=self.namespace, timeout=t)
            except ApiError as ce:
                if is_already_exists(ce):
                    return False
                raise
            self._observe(None)
            return True
        spec = lease.get("spec", {}) or {}
        if self._observed_record != spec:
            self._observed_record = dict(spec)
            self._observed_time = self._loop_time()
        holder = spec.get("holderIdentity") or ""
        duration = float(spec.get("leaseDurationSeconds") or self.lease_duration)
        if holder and holder != self.identity and self._observed_time + duration > self._loop_time():
            return False  # held by someone else and not expired
        try:
            updated = await self.client.replace(kube.LEASES, self._lease_body(lease), timeout=t)
        except ApiError as e:
            if is_conflict(e):
                return False
            raise
        if holder != self.identity:
            self.transitions += 1
        self._observe(updated)
        return True

    def _observe(self, lease: Optional[dict]) -> None:
        self._observed_record = dict((lease or {}).get("spec", {}) or {}) if lease else None
        self._observed_time = self._loop_time()

    async def release(self) -> None:
        """Best effort, one attempt: hand the lease back so a standby need not wait out its
        duration.  Bounded by ``retry_period`` in total (GET and PUT together)."""
        async def once() -> None:
            lease = await self.client.get(kube.LEASES, self.name, self.namespace, timeout=self.retry_period)
            if (lease.get("spec", {}) or {}).get("holderIdentity") != self.identity:
                return
            lease["spec"]["holderIdentity"] = ""
            lease["spec"]["leaseDurationSeconds"] = 1
            await self.client.replace(kube.LEASES, lease, timeout=self.retry_period)
        try:
            await asyncio.wait_for(once(), timeout=self.retry_period)
        except Exception as e:
            log.info("lease release failed: %s", e or type(e).__name__)

    async def run(self, on_started_leading: Callable[[], Awaitable[None]],
                  on_stopped_leading: Optional[Callable[[], Awaitable[None]]] = None) -> None:
        """Blocks: acquire, run ``on_started_leading`` concurrently while renewing; returns when
        leadership is lost (the caller then exits, like controller-runtime)."""
        while True:
            try:
                if await self.try_acquire_or_renew():
                    break
            except Exception as e:
                log.warning("acquire failed: %s", e)
            await asyncio.sleep(self.retry_period)
        self.is_leader = True
        log.info("successfully acquired lease %s/%s as %s", self.namespace, self.name, self.identity)
        work = asyncio.ensure_future(on_started_leading())
        try:
            last_ok = self._loop_time()
            while True:
                if work.done():
                    await work  # propagate errors from the leader's work
                    return
                # Sleep until the next renewal, or until the leader's work ends -- never past the
                # renew deadline, or a stall found late would eat into the standby's margin.
                left = self.renew_deadline - (self._loop_time() - last_ok)
                await asyncio.wait({work}, timeout=max(0.0, min(self.retry_period, left)))
                if work.done():
                    continue
                left = self.renew_deadline - (self._loop_time() - last_ok)
                ok = False
                if left > 0:
                    try:
                        ok = await asyncio.wait_for(self.try_acquire_or_renew(), timeout=left)
                    except asyncio.TimeoutError:
                        log.warning("lease renewal still unanswered at the renew deadline")
                    except Exception as e:
                        log.warning("renew failed: %s", e)
                if ok:
                    last_ok = self._loop_time()
                elif self._loop_time() - last_ok >= self.renew_deadline:
                    log.error("leader election lost: no renewal within the %.1fs renew deadline", self.renew_deadline)
                    self.lost_at = self._loop_time()
                    return
        finally:
            self.is_leader = False
            # 1. the work (and with it every reconcile worker) ends first ...
            work.cancel()
            done, _ = await asyncio.wait({work}, timeout=STOP_BUDGET_S)
            self.work_stopped = bool(done)
            if not done:
                log.error("the leader's work did not stop within %.1fs of losing the lease: the lease is not "
                          "released, a standby takes it only once it has expired", STOP_BUDGET_S)
            elif not work.cancelled() and work.exception() is not None:
                log.info("leader's work ended with %r", work.exception())
            if on_stopped_leading:
                await on_stopped_leading()
            if self.lost_at is not None:
                self.stop_latency = self._loop_time() - self.lost_at
                log.info("stopped leading %.3fs after the renew deadline", self.stop_latency)
            # 2. ... and only then is the lease handed back (one bounded attempt).  Work still
            # running (a worker that swallowed its cancellation) may still write: then the lease
            # is left to expire on its own (lease_duration), so the margin unsafe_timings() checks
            # between this replica's writes and a standby's still holds.
            if self.release_on_cancel and self.work_stopped:
                await self.release()
