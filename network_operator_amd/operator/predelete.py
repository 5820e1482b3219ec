"""``helm uninstall`` pre-delete hook: delete this release's policies while the operator still runs.

A policy with ``amdScaleOut.keepConfigOnRestart`` carries the ``amd.com/node-cleanup`` finalizer:
its agents leave addresses and routes in place, and only the operator can remove them (cleanup
Jobs) and release the policy.  Uninstalling deletes the operator together with the policies'
owner (the ClusterRole anchor, ``seeder.py``), so without this hook such a policy would stay in
Terminating with nobody to finalize it.  The hook deletes the release's policies first and waits
until they are gone (the operator has cleaned every node), then helm removes the rest.

``python -m network_operator_amd.operator.predelete --owner ClusterRole/<name> [--timeout 600]``
exits 0 when the release's policies are gone, 1 when some remain at the timeout (their
``status.keptNodes`` is logged), 2 on a usage error.
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import sys
import time
from typing import List, Optional

from . import kube
from .kube import ApiClient, ApiError, is_not_found, load_config
from .seeder import PolicySeeder

log = logging.getLogger("predelete")
P = kube.NETWORKCLUSTERPOLICIES


async def _ours(client: ApiClient, seeder: PolicySeeder, ref: dict) -> List[dict]:
    lst = await client.list(P)
    return [p for p in lst.get("items") or [] if seeder._ours(p, ref)]


async def drain(client: ApiClient, owner: str, timeout: float, poll: float = 1.0) -> int:
    seeder = PolicySeeder(client, path="", owner=owner)
    ref = await seeder._owner_reference()
    if ref is None:
        log.info("owner %s not found: no policies of this release", owner)
        return 0
    ours = await _ours(client, seeder, ref)
    for p in ours:
        name = p["metadata"]["name"]
        try:
            await client.delete(P, name)
            log.info("deleted policy %s", name)
        except ApiError as e:
            if not is_not_found(e):
                raise
    end = time.monotonic() + timeout
    left: List[dict] = ours
    while left:
        left = await _ours(client, seeder, ref)
        if not left:
            break
        if time.monotonic() >= end:
            for p in left:
                log.error("policy %s still present (finalizers %s, nodes owing a cleanup: %s)", p["metadata"]["name"],
                          p["metadata"].get("finalizers"), ((p.get("status") or {}).get("keptNodes")))
            return 1
        await asyncio.sleep(poll)
    log.info("%d policy(ies) of this release deleted and finalized", len(ours))
    return 0


def main(argv: Optional[List[str]] = None) -> int:
    ap = argparse.ArgumentParser(prog="predelete", description=__doc__.split("\n\n")[0])
    ap.add_argument("--owner", required=True, help="ClusterRole/<name>: the anchor owning the release's policies")
    ap.add_argument("--timeout", type=float, default=600.0)
    ap.add_argument("--kubeconfig")
    ap.add_argument("--master")
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")

    async def go() -> int:
        async with ApiClient(load_config(a.kubeconfig, a.master)) as c:
            return await drain(c, a.owner, a.timeout)
    try:
        return asyncio.run(go())
    except ValueError as e:
        log.error("%s", e)
        return 2


if __name__ == "__main__":
    sys.exit(main())
