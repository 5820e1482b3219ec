"""HTTP(S) endpoints of the manager: health probes, Prometheus metrics, admission webhooks.

Reference wiring (reference cmd/operator/main.go:117-167,219-226):
* probes ``/healthz`` and ``/readyz`` on ``--health-probe-bind-address`` (":8081");
* metrics on ``--metrics-bind-address`` ("0" = disabled), HTTPS with authentication
  (TokenReview) and authorization (SubjectAccessReview on nonResourceURL /metrics) when
  ``--metrics-secure``;
* webhook server on :9443 with the serving certificate from
  ``/tmp/k8s-webhook-server/serving-certs/tls.{crt,key}``;
* TLS 1.2 only with two ECDHE AES-256-GCM suites; HTTP/2 is not offered (the reference
  disables it unless ``--enable-http2``; aiohttp only speaks HTTP/1.1).
"""

from __future__ import annotations

import asyncio
import json
import logging
import os
import ssl
import time
from pathlib import Path
from typing import Callable, Dict, List, Optional, Tuple

from aiohttp import web

from ..api.v1alpha1 import types as T
from ..api.v1alpha1 import webhook as W
from . import kube, selfsigned
from .kube import ApiClient
from .metrics import OperatorMetrics

log = logging.getLogger("servers")

TLS_CIPHERS = "ECDHE-RSA-AES256-GCM-SHA384:ECDHE-ECDSA-AES256-GCM-SHA384"
DEFAULT_CERT_DIR = "/tmp/k8s-webhook-server/serving-certs"


def _tls_context() -> ssl.SSLContext:
    """TLS 1.2 only, two ciphers, HTTP/1.1 (reference cmd/operator/main.go:122-147)."""
    ctx = ssl.SSLContext(ssl.PROTOCOL_TLS_SERVER)
    ctx.minimum_version = ssl.TLSVersion.TLSv1_2
    ctx.maximum_version = ssl.TLSVersion.TLSv1_2
    ctx.set_ciphers(TLS_CIPHERS)
    ctx.set_alpn_protocols(["http/1.1"])
    return ctx


def server_tls_context(cert_file: str, key_file: str) -> ssl.SSLContext:
    ctx = _tls_context()
    ctx.load_cert_chain(cert_file, key_file)
    return ctx


def self_signed_tls_context(cn: str = "amd-network-operator-metrics",
                            sans=("DNS:localhost", "IP:127.0.0.1")) -> ssl.SSLContext:
    """A serving context with a certificate made in memory (selfsigned.py), as controller-runtime
    self-signs the metrics certificate when none is mounted (reference cmd/operator/main.go:157-167).
    Nothing touches the filesystem (the operator's root filesystem is read-only): the PEM pair goes
    through an anonymous memfd that ``load_cert_chain`` reads by its /proc path."""
    ctx = _tls_context()
    cert, key = selfsigned.make_certificate(cn, sans)
    pem = (selfsigned.pem("CERTIFICATE", cert) + selfsigned.pem("EC PRIVATE KEY", key)).encode()
    fd = os.memfd_create("netop-self-signed", os.MFD_CLOEXEC)
    try:
        os.write(fd, pem)
        ctx.load_cert_chain(f"/proc/self/fd/{fd}")
    finally:
        os.close(fd)
    return ctx


class CertWatcher:
    """Reloads a serving certificate into a live SSLContext when its files change
    (controller-runtime's certwatcher): cert-manager rotates the webhook certificate in place,
    and an operator that kept the old one would start failing admission once it expires.
    New handshakes use the new pair; established connections keep theirs."""

    def __init__(self, ctx: ssl.SSLContext, cert_file: str, key_file: str, interval: float = 10.0):
        self.ctx, self.cert_file, self.key_file, self.interval = ctx, cert_file, key_file, interval
        self.reloads = 0
        self._stamp = self._read_stamp()
        self._task: Optional[asyncio.Task] = None

    def _read_stamp(self):
        try:
            return tuple((os.stat(f).st_mtime_ns, os.stat(f).st_size, os.stat(f).st_ino)
                         for f in (self.cert_file, self.key_file))
        except OSError:
            return None

    def check(self) -> bool:
        """Reloads if the files changed since the last successful load; True when reloaded."""
        stamp = self._read_stamp()
        if stamp is None or stamp == self._stamp:
            return False
        try:
            self.ctx.load_cert_chain(self.cert_file, self.key_file)
        except (ssl.SSLError, OSError) as e:  # half-written pair: retry at the next tick
            log.warning("certificate reload failed (will retry): %s", e)
            return False
        self._stamp = stamp
        self.reloads += 1
        log.info("reloaded serving certificate %s", self.cert_file)
        return True

    def start(self) -> None:
        async def loop():
            while True:
                await asyncio.sleep(self.interval)
                self.check()
        self._task = asyncio.ensure_future(loop())

    async def stop(self) -> None:
        if self._task:
            self._task.cancel()
            try:
                await self._task
            except asyncio.CancelledError:
                pass


def generate_self_signed(cert_dir: Path, cn: str = "localhost", sans=("DNS:localhost", "IP:127.0.0.1")) -> Tuple[Path, Path]:
    """Self-signed serving certificate files tls.crt / tls.key (tests / local runs; in clusters
    cert-manager issues it).  Made in process (selfsigned.py): no openssl binary needed."""
    return selfsigned.write_self_signed(Path(cert_dir), cn, sans, days=2)


def parse_bind(addr: str) -> Optional[Tuple[str, int]]:
    """":8081" -> ("0.0.0.0", 8081); "0" -> None (disabled)."""
    if addr in ("", "0"):
        return None
    host, _, port = addr.rpartition(":")
    return (host or "0.0.0.0", int(port))


class TokenAuthorizer:
    """controller-runtime's WithAuthenticationAndAuthorization filter for /metrics."""

    def __init__(self, client: ApiClient, ttl: float = 30.0):
        self.client = client
        self.ttl = ttl
        self._cache: Dict[str, Tuple[float, bool]] = {}

    async def allowed(self, token: str, path: str) -> bool:
        hit = self._cache.get(token)
        if hit and hit[0] > time.monotonic():
            return hit[1]
        ok = False
        try:
            tr = await self.client.create(kube.TOKENREVIEWS, {"apiVersion": "authentication.k8s.io/v1",
                                                             "kind": "TokenReview", "spec": {"token": token}})
            st = tr.get("status", {})
            if st.get("authenticated"):
                user = st.get("user", {})
                sar = await self.client.create(kube.SUBJECTACCESSREVIEWS, {
                    "apiVersion": "authorization.k8s.io/v1", "kind": "SubjectAccessReview",
                    "spec": {"user": user.get("username"), "groups": user.get("groups", []), "uid": user.get("uid"),
                             "nonResourceAttributes": {"path": path, "verb": "get"}}})
                ok = bool(sar.get("status", {}).get("allowed"))
        except Exception as e:
            log.warning("metrics authn/authz failed: %s", e)
        self._cache[token] = (time.monotonic() + self.ttl, ok)
        return ok


class Servers:
    def __init__(self, metrics: OperatorMetrics, ready_check: Callable[[], bool] = lambda: True,
                 client: Optional[ApiClient] = None):
        self.metrics = metrics
        self.ready_check = ready_check
        self.client = client
        self.runners: list = []
        self.ports: Dict[str, int] = {}
        self.cert_watcher: Optional[CertWatcher] = None  # the webhook's
        self.watchers: list = []
        self.cert_reload_interval = 10.0

    # -- apps ------------------------------------------------------------------------------------
    def probes_app(self) -> web.Application:
        app = web.Application()

        async def healthz(_):
            return web.Response(text="ok")

        async def readyz(_):
            return web.Response(text="ok") if self.ready_check() else web.Response(status=500, text="not ready")

        app.router.add_get("/healthz", healthz)
        app.router.add_get("/readyz", readyz)
        return app

    def metrics_app(self, secure: bool) -> web.Application:
        app = web.Application()
        authz = TokenAuthorizer(self.client) if secure and self.client else None

        async def metrics(req: web.Request):
            if authz is not None:
                auth = req.headers.get("Authorization", "")
                if not auth.startswith("Bearer "):
                    return web.Response(status=401, text="Unauthorized")
                if not await authz.allowed(auth[7:], req.path):
                    return web.Response(status=403, text="Forbidden")
            return web.Response(body=self.metrics.render(), headers={"Content-Type": self.metrics.content_type})

        app.router.add_get("/metrics", metrics)
        return app

    OVERLAP_LIST_TIMEOUT_S = 2.0  # inside the API server's webhook timeout (10 s); warnings only

    async def overlap_warnings(self, review: dict) -> List[str]:
        """An admitted CREATE / UPDATE of a policy whose selector overlaps another live policy of
        its type gets a warning naming it (kubectl prints it).  Best effort: without a client, or
        if the LIST fails or is slow, no warning -- admission never depends on it."""
        req = review.get("request") or {}
        if self.client is None or req.get("operation") not in ("CREATE", "UPDATE"):
            return []
        try:
            pol = T.NetworkClusterPolicy.from_dict(req.get("object") or {})
            lst = await self.client.list(kube.NETWORKCLUSTERPOLICIES, timeout=self.OVERLAP_LIST_TIMEOUT_S)
        except Exception as e:
            log.debug("overlap check skipped: %s", e)
            return []
        return W.overlap_warnings(pol, lst.get("items") or [])

    def webhook_app(self) -> web.Application:
        app = web.Application()

        def handler(mutate: bool):
            async def h(req: web.Request):
                try:
                    review = await req.json()
                except json.JSONDecodeError:
                    return web.Response(status=400, text="bad AdmissionReview")
                out = W.admission_review(review, mutate)
                resp = out.get("response") or {}
                if not mutate and resp.get("allowed"):
                    extra = await self.overlap_warnings(review)
                    if extra:
                        resp["warnings"] = list(resp.get("warnings") or []) + extra
                return web.json_response(out)
            return h

        app.router.add_post(W.MUTATE_PATH, handler(True))
        app.router.add_post(W.VALIDATE_PATH, handler(False))
        return app

    # -- lifecycle -------------------------------------------------------------------------------
    async def _serve(self, name: str, app: web.Application, host: str, port: int,
                     ssl_ctx: Optional[ssl.SSLContext] = None) -> int:
        runner = web.AppRunner(app, access_log=None)
        await runner.setup()
        site = web.TCPSite(runner, host, port, ssl_context=ssl_ctx)
        await site.start()
        self.runners.append(runner)
        sock = site._server.sockets[0]  # type: ignore[union-attr]
        self.ports[name] = sock.getsockname()[1]
        log.info("serving %s on %s:%d%s", name, host, self.ports[name], " (TLS)" if ssl_ctx else "")
        return self.ports[name]

    async def start(self, probe_addr: str = ":8081", metrics_addr: str = "0", metrics_secure: bool = False,
                    webhook_port: Optional[int] = None, cert_dir: str = DEFAULT_CERT_DIR) -> None:
        b = parse_bind(probe_addr)
        if b:
            await self._serve("probes", self.probes_app(), *b)
        b = parse_bind(metrics_addr)
        if b:
            ctx = None
            if metrics_secure:
                cd = Path(cert_dir)
                if (cd / "tls.crt").exists() and (cd / "tls.key").exists():
                    ctx = server_tls_context(str(cd / "tls.crt"), str(cd / "tls.key"))
                else:
                    # controller-runtime self-signs the metrics certificate too; the watcher below
                    # switches to a mounted pair as soon as one appears.
                    log.info("no serving certificate in %s: /metrics uses a self-signed one made in memory", cd)
                    ctx = self_signed_tls_context()
                self._watch(ctx, cd)
            await self._serve("metrics", self.metrics_app(metrics_secure), *b, ssl_ctx=ctx)
        if webhook_port is not None:
            cd = Path(cert_dir)
            ctx = server_tls_context(str(cd / "tls.crt"), str(cd / "tls.key"))
            await self._serve("webhook", self.webhook_app(), "0.0.0.0", webhook_port, ssl_ctx=ctx)
            self.cert_watcher = self._watch(ctx, cd)

    def _watch(self, ctx: ssl.SSLContext, cert_dir: Path) -> CertWatcher:
        w = CertWatcher(ctx, str(cert_dir / "tls.crt"), str(cert_dir / "tls.key"), self.cert_reload_interval)
        w.start()
        self.watchers.append(w)
        return w

    async def stop(self) -> None:
        for w in self.watchers:
            await w.stop()
        self.watchers.clear()
        for r in self.runners:
            await r.cleanup()
        self.runners.clear()
