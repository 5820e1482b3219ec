"""Rate-limited, de-duplicating work queue (client-go ``workqueue`` semantics).

* an item added while queued is not queued twice (``dirty`` set);
* an item added while being processed is re-queued only after ``done`` (``processing``
  set), so one key is never reconciled by two workers at once;
* ``add_rate_limited`` backs off per item exponentially (5 ms * 2^n, capped at 1000 s —
  controller-runtime's default ItemExponentialFailureRateLimiter) combined with an overall
  token bucket (10 qps, burst 100), taking the larger delay; ``forget`` resets an item.
"""

from __future__ import annotations

import asyncio
import heapq
import itertools
import time
from typing import Dict, Hashable, List, Optional, Set, Tuple


class ExponentialRateLimiter:
    def __init__(self, base: float = 0.005, cap: float = 1000.0):
        self.base, self.cap = base, cap
        self.failures: Dict[Hashable, int] = {}

    def when(self, item: Hashable) -> float:
        n = self.failures.get(item, 0)
        self.failures[item] = n + 1
        return min(self.base * (2 ** n), self.cap)

    def forget(self, item: Hashable) -> None:
        self.failures.pop(item, None)

    def retries(self, item: Hashable) -> int:
        return self.failures.get(item, 0)


class BucketRateLimiter:
    def __init__(self, qps: float = 10.0, burst: int = 100):
        self.qps, self.burst = qps, burst
        self.tokens = float(burst)
        self.last = time.monotonic()

    def when(self, item: Hashable) -> float:
        now = time.monotonic()
        self.tokens = min(self.burst, self.tokens + (now - self.last) * self.qps)
        self.last = now
        self.tokens -= 1
        return 0.0 if self.tokens >= 0 else -self.tokens / self.qps

    def forget(self, item: Hashable) -> None:
        pass


class RateLimitingQueue:
    def __init__(self, name: str = "queue", item_limiter: Optional[ExponentialRateLimiter] = None,
                 bucket: Optional[BucketRateLimiter] = None):
        self.name = name
        self._queue: List[Hashable] = []
        self._dirty: Set[Hashable] = set()
        self._processing: Set[Hashable] = set()
        self._cond = asyncio.Condition()
        self._delayed: List[Tuple[float, int, Hashable]] = []
        self._seq = itertools.count()
        self._limiter = item_limiter or ExponentialRateLimiter()
        self._bucket = bucket or BucketRateLimiter()
        self._shutdown = False
        self._timer: Optional[asyncio.Task] = None
        self._wake = asyncio.Event()
        self.adds = 0
        self.retries_total = 0

    # -- basic queue ---------------------------------------------------------------------------
    async def add(self, item: Hashable) -> None:
        async with self._cond:
            self._add_locked(item)

    def _add_locked(self, item: Hashable) -> None:
        if self._shutdown or item in self._dirty:
            return
        self.adds += 1
        self._dirty.add(item)
        if item in self._processing:
            return
        self._queue.append(item)
        self._cond.notify()

    async def get(self) -> Optional[Hashable]:
        """Next item, or None after shutdown."""
        async with self._cond:
            while not self._queue and not self._shutdown:
                await self._cond.wait()
            if not self._queue:
                return None
            item = self._queue.pop(0)
            self._processing.add(item)
            self._dirty.discard(item)
            return item

    async def done(self, item: Hashable) -> None:
        async with self._cond:
            self._processing.discard(item)
            if item in self._dirty:
                self._queue.append(item)
                self._cond.notify()

    def __len__(self) -> int:
        return len(self._queue)

    @property
    def depth(self) -> int:
        return len(self._queue)

    # -- delays / rate limiting ---------------------------------------------------------------------
    async def add_after(self, item: Hashable, delay: float) -> None:
        if delay <= 0:
            await self.add(item)
            return
        async with self._cond:
            heapq.heappush(self._delayed, (time.monotonic() + delay, next(self._seq), item))
            self._wake.set()
            self._ensure_timer()

    async def add_rate_limited(self, item: Hashable) -> None:
        self.retries_total += 1
        await self.add_after(item, max(self._limiter.when(item), self._bucket.when(item)))

    def forget(self, item: Hashable) -> None:
        self._limiter.forget(item)

    def num_requeues(self, item: Hashable) -> int:
        return self._limiter.retries(item)

    def _ensure_timer(self) -> None:
        if self._timer is None or self._timer.done():
            self._timer = asyncio.ensure_future(self._run_timer())

    async def _run_timer(self) -> None:
        while True:
            async with self._cond:
                if self._shutdown or not self._delayed:
                    return
                due, _, item = self._delayed[0]
                now = time.monotonic()
                if due <= now:
                    heapq.heappop(self._delayed)
                    self._add_locked(item)
                    continue
                wait = due - now
                self._wake.clear()
            try:
                # An earlier item pushed meanwhile sets _wake and shortens the sleep.
                await asyncio.wait_for(self._wake.wait(), timeout=wait)
            except asyncio.TimeoutError:
                pass
            except asyncio.CancelledError:
                return

    async def shutdown(self) -> None:
        async with self._cond:
            self._shutdown = True
            self._cond.notify_all()
        if self._timer:
            self._timer.cancel()
