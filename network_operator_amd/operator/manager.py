"""``manager`` — the operator process (Deployment, one active replica via leader election).

Reference entrypoint: cmd/operator/main.go.  Same flags (:95-112):
``--metrics-bind-address`` (default "0" = off), ``--health-probe-bind-address`` (":8081"),
``--leader-elect``, ``--metrics-secure``, ``--enable-http2`` plus zap logging flags; same
environment: ``OPERATOR_NAMESPACE`` (default ``amd-network-operator``), ``ENABLE_WEBHOOKS``
("false" disables the webhook server).  OpenShift is detected from the API server's groups
(``route.openshift.io`` / ``security.openshift.io``, :64-87) — through the same client
configuration as everything else, so detection also works out of cluster.
"""

from __future__ import annotations

import argparse
import asyncio
import logging
import os
import signal
import sys
from typing import Dict, List, Optional

from . import kube, rbac
from .controller import PolicyController
from .kube import ApiClient, ApiError, load_config
from .leader import DEFAULT_LEASE_ID, LeaderElector, unsafe_timings
from .metrics import OperatorMetrics
from .seeder import PolicySeeder
from .servers import DEFAULT_CERT_DIR, Servers

log = logging.getLogger("setup")

DEFAULT_OPERATOR_NAMESPACE = "amd-network-operator"
OPENSHIFT_GROUPS = ("route.openshift.io", "security.openshift.io")


# Add-ons the operator depends on (reference README "Dependencies"), by API group.
#   node-feature-discovery: the default nodeSelector label (gpu-ready) and the readiness label
#                           (local feature files) are both NFD's; without it no node is ever
#                           selected or reported ready.
#   cert-manager:           serving certificates of the admission webhooks (kustomize / chart).
DEPENDENCIES = {"node-feature-discovery": "nfd.k8s-sigs.io", "cert-manager": "cert-manager.io"}
# Missing dependencies that break policies (surface in status.errors); the others are logged.
POLICY_DEPENDENCIES = ("node-feature-discovery",)


async def check_dependencies(client: ApiClient) -> Dict[str, bool]:
    groups = set(await client.server_groups())
    return {name: group in groups for name, group in DEPENDENCIES.items()}


async def check_crd(client: ApiClient) -> Optional[List[str]]:
    """Fields of this release's schema the installed CRD lacks (crd.missing_fields), or None when
    the CRD cannot be read (RBAC of an older release, not installed)."""
    from ..api.v1alpha1 import crd as crd_schema

    try:
        installed = await client.get(kube.CRDS, rbac.CRD_NAME, timeout=5.0)
    except ApiError as e:
        log.debug("cannot read CRD %s: %s", rbac.CRD_NAME, e)
        return None
    return crd_schema.missing_fields(installed)


async def watch_dependencies(client: ApiClient, controller, metrics, stop: asyncio.Event, interval: float,
                             webhooks: bool) -> None:
    """Checks the cluster add-ons now and every `interval` seconds; on a change the policies are
    reconciled again so their status reflects it.  Also whether the installed CRD is as new as
    the operator: Helm never upgrades a chart's crds/."""
    last: Optional[Dict[str, bool]] = None
    last_missing: Optional[List[str]] = None
    while not stop.is_set():
        try:
            missing = await check_crd(client)
            if missing is not None:
                metrics.crd_missing_fields.set(len(missing))
                if missing and missing != last_missing:
                    log.error("the installed CRD %s predates this operator: the API server drops %s from every "
                              "policy; apply the CRD of this release (kubectl apply -f charts/network-operator/crds/ or "
                              "config/operator/crd/bases/): helm upgrade never updates crds/",
                              rbac.CRD_NAME, ", ".join(missing[:10]) + (" ..." if len(missing) > 10 else ""))
                last_missing = missing
        except Exception as e:
            log.debug("CRD check failed: %s", e)
        try:
            present = await check_dependencies(client)
            for name, ok in present.items():
                metrics.dependency.labels(name).set(1 if ok else 0)
            if present != last:
                for name, ok in present.items():
                    if not ok and (name != "cert-manager" or webhooks):
                        log.warning("dependency missing: %s (API group %s not served)", name, DEPENDENCIES[name])
                controller.reconciler.missing_dependencies = [n for n in POLICY_DEPENDENCIES if not present.get(n, True)]
                if last is not None:
                    await controller.requeue_all()
                last = present
        except Exception as e:  # discovery hiccups must not stop the manager
            log.debug("dependency check failed: %s", e)
        try:
            await asyncio.wait_for(stop.wait(), timeout=interval)
        except asyncio.TimeoutError:
            pass


async def is_openshift(client: ApiClient) -> bool:
    groups = await client.server_groups()
    return any(g in OPENSHIFT_GROUPS for g in groups)


def build_parser() -> argparse.ArgumentParser:
    ap = argparse.ArgumentParser(prog="manager", description="AMD MI355X network operator")
    ap.add_argument("--metrics-bind-address", default="0",
                    help="The address the metrics endpoint binds to. Use :8443 for HTTPS or :8080 for HTTP, "
                         "or leave as 0 to disable the metrics service.")
    ap.add_argument("--health-probe-bind-address", default=":8081", help="The address the probe endpoint binds to.")
    ap.add_argument("--leader-elect", action="store_true",
                    help="Enable leader election for controller manager.")
    ap.add_argument("--metrics-secure", action="store_true", help="If set the metrics endpoint is served securely")
    ap.add_argument("--enable-http2", action="store_true",
                    help="If set, HTTP/2 would be enabled for the metrics and webhook servers (HTTP/1.1 only here)")
    ap.add_argument("--kubeconfig", default=None, help="kubeconfig file (default: the in-cluster service account)")
    ap.add_argument("--master", default=None, help="API server URL (overrides kubeconfig; tests)")
    ap.add_argument("--webhook-port", type=int, default=9443, help="HTTPS port of the admission webhooks")
    ap.add_argument("--webhook-cert-dir", default=DEFAULT_CERT_DIR,
                    help="directory with tls.crt / tls.key (cert-manager's Secret); reloaded when they change")
    ap.add_argument("--workers", type=int, default=2, help="concurrent reconciles")
    ap.add_argument("--dependency-check-interval", type=float, default=60.0,
                    help="seconds between checks for Node Feature Discovery / cert-manager (0 = off)")
    ap.add_argument("--leader-election-id", default=DEFAULT_LEASE_ID, help="name of the Lease the replicas elect through")
    # kube-controller-manager's names for client-go's LeaderElectionConfig timings; the defaults
    # are controller-runtime's (the reference does not expose them, main.go:174-175).
    ap.add_argument("--leader-elect-lease-duration", type=float, default=15.0,
                    help="seconds a standby waits after the last observed renewal before taking over")
    ap.add_argument("--leader-elect-renew-deadline", type=float, default=10.0,
                    help="seconds the leader keeps trying to renew before it gives up leading")
    ap.add_argument("--leader-elect-retry-period", type=float, default=2.0,
                    help="seconds between acquire / renew attempts")
    ap.add_argument("--policies-file", default="",
                    help="YAML file ({policies: [NetworkClusterPolicy, ...]}, the Helm chart's ConfigMap) whose "
                         "policies the leader creates / updates / deletes through the API server")
    ap.add_argument("--policies-owner", default="",
                    help="ClusterRole/<name>: cluster-scoped owner of the seeded policies (uninstalling it "
                         "garbage-collects them)")
    ap.add_argument("--policies-interval", type=float, default=10.0, help="seconds between --policies-file passes")
    ap.add_argument("--policies-seed-id", default="",
                    help="without --policies-owner: the id (label amd.com/policy-seeder) marking this operator's "
                         "seeded policies (default <namespace>.<leader election id>)")
    ap.add_argument("--zap-devel", action="store_true", default=True, help="development logging defaults (controller-runtime's flag)")
    ap.add_argument("--zap-log-level", default="info", help="debug, info, warn or error")
    ap.add_argument("--zap-encoder", default="console", choices=["console", "json"], help="log line format")
    return ap


def setup_logging(level: str, encoder: str) -> None:
    lvl = {"debug": logging.DEBUG, "info": logging.INFO, "error": logging.ERROR}.get(level, logging.INFO)
    if level.isdigit():
        lvl = max(1, logging.INFO - int(level))
    fmt = ('{"ts":"%(asctime)s","level":"%(levelname)s","logger":"%(name)s","msg":"%(message)s"}'
           if encoder == "json" else "%(asctime)s\t%(levelname)s\t%(name)s\t%(message)s")
    logging.basicConfig(level=lvl, format=fmt, stream=sys.stderr, force=True)


async def run(argv: Optional[List[str]] = None, stop: Optional[asyncio.Event] = None,
              started: Optional[asyncio.Event] = None, user_agent: Optional[str] = None,
              identity: Optional[str] = None) -> int:
    """The manager.  Returns 0 after a stop signal and 1 on a start-up failure or when leadership
    was lost (controller-runtime's manager exits 1 with "leader election lost", reference
    cmd/operator/main.go:229-232).  `stop`, `started`, `user_agent` and `identity` (the Lease
    holder; default ``<pod>_<uuid>``) let tests run several replicas in one process."""
    opts = build_parser().parse_args(argv)
    setup_logging(opts.zap_log_level, opts.zap_encoder)
    ns = os.environ.get("OPERATOR_NAMESPACE") or DEFAULT_OPERATOR_NAMESPACE
    log.info("Using namespace: %s", ns)
    stop = stop or asyncio.Event()
    loop = asyncio.get_event_loop()
    for sig in (signal.SIGTERM, signal.SIGINT):
        try:
            loop.add_signal_handler(sig, stop.set)
        except (NotImplementedError, RuntimeError):  # not the main thread (tests)
            pass

    if opts.leader_elect:
        why = unsafe_timings(opts.leader_elect_lease_duration, opts.leader_elect_renew_deadline,
                             opts.leader_elect_retry_period)
        if why:
            log.error("%s", why)
            return 1
    client = ApiClient(load_config(opts.kubeconfig, opts.master),
                       **({"user_agent": user_agent} if user_agent else {}))
    try:
        try:
            openshift = await is_openshift(client)
        except Exception as e:
            log.error("unable to check if running in OpenShift: %s", e)
            return 1
        if openshift:
            log.info("Detected OpenShift environment")
        metrics = OperatorMetrics()
        controller = PolicyController(client, ns, openshift, workers=opts.workers, metrics=metrics)
        servers = Servers(metrics, ready_check=lambda: True, client=client)
        webhooks = os.environ.get("ENABLE_WEBHOOKS", "") != "false"
        await servers.start(opts.health_probe_bind_address, opts.metrics_bind_address, opts.metrics_secure,
                            opts.webhook_port if webhooks else None, opts.webhook_cert_dir)

        dep_task = None
        exit_code = 0
        if opts.dependency_check_interval > 0:
            # First result before the controller starts, so the first status already has it.
            try:
                present = await check_dependencies(client)
                controller.reconciler.missing_dependencies = [n for n in POLICY_DEPENDENCIES
                                                             if not present.get(n, True)]
            except Exception as e:
                log.debug("dependency check failed: %s", e)
            dep_task = asyncio.ensure_future(watch_dependencies(client, controller, metrics, stop,
                                                                opts.dependency_check_interval, webhooks))

        async def lead() -> None:
            # The leader's work owns every writer: when the elector cancels it at the renew
            # deadline, the reconcile workers and the seeder are gone before the lease is
            # released (leader.py) -- not after, as when they outlived a cancelled wait.
            seed = None
            try:
                await controller.start()
                if opts.policies_file:
                    # Only the leader writes policies; the webhook server is already serving, so the
                    # API server can admit them (see seeder.py for why the chart does not create them).
                    seeder = PolicySeeder(client, opts.policies_file, opts.policies_owner, opts.policies_interval,
                                          metrics=metrics,
                                          seed_id=opts.policies_seed_id or f"{ns}.{opts.leader_election_id}")
                    seed = asyncio.ensure_future(seeder.run(stop))
                if started:
                    started.set()
                log.info("starting manager")
                await stop.wait()
            finally:
                if seed is not None:
                    seed.cancel()
                    try:
                        await seed
                    except (asyncio.CancelledError, Exception):
                        pass
                await controller.stop()

        try:
            if opts.leader_elect:
                elector = LeaderElector(client, ns, opts.leader_election_id, identity=identity,
                                        lease_duration=opts.leader_elect_lease_duration,
                                        renew_deadline=opts.leader_elect_renew_deadline,
                                        retry_period=opts.leader_elect_retry_period)
                metrics.leader.labels(opts.leader_election_id).set(0)

                async def lead_with_metric() -> None:
                    metrics.leader.labels(opts.leader_election_id).set(1)
                    await lead()

                async def stopped_leading() -> None:
                    metrics.leader.labels(opts.leader_election_id).set(0)
                    await controller.stop()

                runner = asyncio.ensure_future(elector.run(lead_with_metric, on_stopped_leading=stopped_leading))
                stopper = asyncio.ensure_future(stop.wait())
                done, _ = await asyncio.wait({runner, stopper}, return_when=asyncio.FIRST_COMPLETED)
                stopper.cancel()
                if runner not in done:
                    runner.cancel()
                    try:
                        await runner
                    except (asyncio.CancelledError, Exception):
                        pass
                elif elector.lost_at is not None or runner.exception() is not None:
                    log.error("problem running manager: %s",
                              "leader election lost" if elector.lost_at is not None else runner.exception())
                    exit_code = 1
            else:
                await lead()
        finally:
            if dep_task is not None:
                dep_task.cancel()
            await controller.stop()
            await servers.stop()
        return exit_code
    finally:
        await client.close()


def main(argv: Optional[List[str]] = None) -> int:
    return asyncio.run(run(argv))


if __name__ == "__main__":
    sys.exit(main())
