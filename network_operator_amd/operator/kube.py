"""Asynchronous Kubernetes REST client (aiohttp) — the operator's only way to the API server.

Replaces what client-go / controller-runtime give the reference manager
(reference cmd/operator/main.go:169-187): typed resource paths, CRUD + status subresource,
merge / JSON patches, streaming watches with bookmarks, discovery (server groups), in-cluster
and kubeconfig credentials.  Service-account tokens are re-read from disk so projected
(rotating) tokens keep working.
"""

from __future__ import annotations

import base64
import json
import os
import ssl
import tempfile
from dataclasses import dataclass, field
from pathlib import Path
from typing import Any, AsyncIterator, Dict, List, Optional, Tuple

import aiohttp
import yaml


# ---------------------------------------------------------------------------
# Resources
# ---------------------------------------------------------------------------
@dataclass(frozen=True)
class Resource:
    group: str
    version: str
    plural: str
    kind: str
    namespaced: bool

    @property
    def api_version(self) -> str:
        return self.version if not self.group else f"{self.group}/{self.version}"

    def base(self) -> str:
        return "/api/v1" if not self.group else f"/apis/{self.group}/{self.version}"

    def path(self, namespace: Optional[str] = None, name: Optional[str] = None, sub: Optional[str] = None) -> str:
        p = self.base()
        if self.namespaced and namespace:
            p += f"/namespaces/{namespace}"
        p += f"/{self.plural}"
        if name:
            p += f"/{name}"
            if sub:
                p += f"/{sub}"
        return p


NETWORKCLUSTERPOLICIES = Resource("amd.com", "v1alpha1", "networkclusterpolicies", "NetworkClusterPolicy", False)
DAEMONSETS = Resource("apps", "v1", "daemonsets", "DaemonSet", True)
PODS = Resource("", "v1", "pods", "Pod", True)
NODES = Resource("", "v1", "nodes", "Node", False)
NAMESPACES = Resource("", "v1", "namespaces", "Namespace", False)
SERVICEACCOUNTS = Resource("", "v1", "serviceaccounts", "ServiceAccount", True)
EVENTS = Resource("", "v1", "events", "Event", True)
ROLEBINDINGS = Resource("rbac.authorization.k8s.io", "v1", "rolebindings", "RoleBinding", True)
LEASES = Resource("coordination.k8s.io", "v1", "leases", "Lease", True)
TOKENREVIEWS = Resource("authentication.k8s.io", "v1", "tokenreviews", "TokenReview", False)
SUBJECTACCESSREVIEWS = Resource("authorization.k8s.io", "v1", "subjectaccessreviews", "SubjectAccessReview", False)
MUTATINGWEBHOOKS = Resource("admissionregistration.k8s.io", "v1", "mutatingwebhookconfigurations",
                            "MutatingWebhookConfiguration", False)
VALIDATINGWEBHOOKS = Resource("admissionregistration.k8s.io", "v1", "validatingwebhookconfigurations",
                              "ValidatingWebhookConfiguration", False)
CRDS = Resource("apiextensions.k8s.io", "v1", "customresourcedefinitions", "CustomResourceDefinition", False)
CLUSTERROLES = Resource("rbac.authorization.k8s.io", "v1", "clusterroles", "ClusterRole", False)
CLUSTERROLEBINDINGS = Resource("rbac.authorization.k8s.io", "v1", "clusterrolebindings", "ClusterRoleBinding", False)
ROLES = Resource("rbac.authorization.k8s.io", "v1", "roles", "Role", True)
SERVICES = Resource("", "v1", "services", "Service", True)
CONFIGMAPS = Resource("", "v1", "configmaps", "ConfigMap", True)
DEPLOYMENTS = Resource("apps", "v1", "deployments", "Deployment", True)
JOBS = Resource("batch", "v1", "jobs", "Job", True)

ALL_RESOURCES = [NETWORKCLUSTERPOLICIES, DAEMONSETS, PODS, NODES, NAMESPACES, SERVICEACCOUNTS, EVENTS, ROLEBINDINGS,
                 LEASES, TOKENREVIEWS, SUBJECTACCESSREVIEWS, MUTATINGWEBHOOKS, VALIDATINGWEBHOOKS, CRDS,
                 CLUSTERROLES, CLUSTERROLEBINDINGS, ROLES, SERVICES, CONFIGMAPS, DEPLOYMENTS, JOBS]


# ---------------------------------------------------------------------------
# Errors
# ---------------------------------------------------------------------------
class ApiError(Exception):
    def __init__(self, status: int, reason: str = "", message: str = "", body: Optional[dict] = None):
        super().__init__(f"{status} {reason}: {message}")
        self.status = status
        self.reason = reason
        self.message = message
        self.body = body or {}


def is_not_found(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.status == 404


def is_conflict(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.status == 409 and e.reason != "AlreadyExists"


def is_already_exists(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.status == 409 and e.reason == "AlreadyExists"


def is_gone(e: BaseException) -> bool:
    return isinstance(e, ApiError) and e.status == 410


# ---------------------------------------------------------------------------
# Credentials
# ---------------------------------------------------------------------------
SA_DIR = Path("/var/run/secrets/kubernetes.io/serviceaccount")


@dataclass
class KubeConfig:
    host: str
    token: Optional[str] = None
    token_file: Optional[str] = None
    ca_file: Optional[str] = None
    client_cert: Optional[str] = None
    client_key: Optional[str] = None
    insecure: bool = False
    namespace: Optional[str] = None
    _tmpfiles: List[str] = field(default_factory=list, repr=False)

    def bearer(self) -> Optional[str]:
        if self.token_file:
            try:
                return Path(self.token_file).read_text().strip()
            except OSError:
                pass
        return self.token

    def ssl_context(self) -> Optional[ssl.SSLContext]:
        if not self.host.startswith("https"):
            return None
        ctx = ssl.create_default_context(cafile=self.ca_file) if self.ca_file else ssl.create_default_context()
        if self.insecure:
            ctx.check_hostname = False
            ctx.verify_mode = ssl.CERT_NONE
        if self.client_cert:
            ctx.load_cert_chain(self.client_cert, self.client_key)
        return ctx


def load_incluster() -> KubeConfig:
    host, port = os.environ.get("KUBERNETES_SERVICE_HOST"), os.environ.get("KUBERNETES_SERVICE_PORT")
    if not host or not port:
        raise RuntimeError("not running in a cluster (KUBERNETES_SERVICE_HOST/PORT unset)")
    if ":" in host:
        host = f"[{host}]"
    ns = (SA_DIR / "namespace").read_text().strip() if (SA_DIR / "namespace").exists() else None
    return KubeConfig(host=f"https://{host}:{port}", token_file=str(SA_DIR / "token"), ca_file=str(SA_DIR / "ca.crt"),
                      namespace=ns)


def _materialize(data_b64: Optional[str], cfg: KubeConfig) -> Optional[str]:
    if not data_b64:
        return None
    fd, path = tempfile.mkstemp(prefix="netop-kube-")
    with os.fdopen(fd, "wb") as f:
        f.write(base64.b64decode(data_b64))
    cfg._tmpfiles.append(path)
    return path


def load_kubeconfig(path: Optional[str] = None, context: Optional[str] = None) -> KubeConfig:
    path = path or os.environ.get("KUBECONFIG", "").split(os.pathsep)[0] or str(Path.home() / ".kube" / "config")
    doc = yaml.safe_load(Path(path).read_text())
    ctx_name = context or doc.get("current-context")
    ctx = next(c["context"] for c in doc.get("contexts", []) if c["name"] == ctx_name)
    cluster = next(c["cluster"] for c in doc.get("clusters", []) if c["name"] == ctx["cluster"])
    user = next((u["user"] for u in doc.get("users", []) if u["name"] == ctx.get("user")), {}) or {}
    cfg = KubeConfig(host=cluster["server"], insecure=bool(cluster.get("insecure-skip-tls-verify")),
                     namespace=ctx.get("namespace"))
    cfg.ca_file = cluster.get("certificate-authority") or _materialize(cluster.get("certificate-authority-data"), cfg)
    cfg.token = user.get("token")
    cfg.token_file = user.get("tokenFile")
    cfg.client_cert = user.get("client-certificate") or _materialize(user.get("client-certificate-data"), cfg)
    cfg.client_key = user.get("client-key") or _materialize(user.get("client-key-data"), cfg)
    return cfg


def load_config(kubeconfig: Optional[str] = None, master: Optional[str] = None) -> KubeConfig:
    """controller-runtime's GetConfigOrDie order: --kubeconfig, $KUBECONFIG, in-cluster, ~/.kube/config."""
    if master:
        return KubeConfig(host=master)
    if kubeconfig or os.environ.get("KUBECONFIG"):
        return load_kubeconfig(kubeconfig)
    try:
        return load_incluster()
    except RuntimeError:
        return load_kubeconfig()


# ---------------------------------------------------------------------------
# Client
# ---------------------------------------------------------------------------
class ApiClient:
    def __init__(self, cfg: KubeConfig, timeout: float = 30.0, user_agent: str = "amd-network-operator/0.1"):
        self.cfg = cfg
        self._timeout = aiohttp.ClientTimeout(total=timeout)
        self._ua = user_agent
        self._session: Optional[aiohttp.ClientSession] = None
        self.requests = 0

    async def _sess(self) -> aiohttp.ClientSession:
        if self._session is None or self._session.closed:
            conn = aiohttp.TCPConnector(ssl=self.cfg.ssl_context() or False, limit=32)
            self._session = aiohttp.ClientSession(connector=conn, headers={"User-Agent": self._ua})
        return self._session

    async def close(self) -> None:
        if self._session is not None:
            await self._session.close()
            self._session = None

    async def __aenter__(self) -> "ApiClient":
        return self

    async def __aexit__(self, *exc) -> None:
        await self.close()

    def _headers(self, content_type: Optional[str] = None) -> Dict[str, str]:
        h = {"Accept": "application/json"}
        tok = self.cfg.bearer()
        if tok:
            h["Authorization"] = f"Bearer {tok}"
        if content_type:
            h["Content-Type"] = content_type
        return h

    @staticmethod
    async def _error(resp: aiohttp.ClientResponse) -> ApiError:
        try:
            body = await resp.json(content_type=None)
        except Exception:
            body = {"message": (await resp.text())[:500]}
        if not isinstance(body, dict):
            body = {"message": str(body)}
        return ApiError(resp.status, body.get("reason", ""), body.get("message", ""), body)

    async def request(self, method: str, path: str, params: Optional[dict] = None, body: Any = None,
                      content_type: str = "application/json", timeout: Optional[float] = None) -> dict:
        """`timeout`: total seconds for this request (default: the client's), e.g. the lease
        renewals, which must never outlast the leader-election renew deadline."""
        s = await self._sess()
        self.requests += 1
        data = json.dumps(body) if body is not None else None
        async with s.request(method, self.cfg.host + path, params=params, data=data,
                             headers=self._headers(content_type if data is not None else None),
                             timeout=aiohttp.ClientTimeout(total=timeout) if timeout else self._timeout) as resp:
            if resp.status >= 400:
                raise await self._error(resp)
            if resp.status == 204:
                return {}
            return await resp.json(content_type=None)

    # -- CRUD --------------------------------------------------------------------------------------
    async def get(self, res: Resource, name: str, namespace: Optional[str] = None,
                  timeout: Optional[float] = None) -> dict:
        return await self.request("GET", res.path(namespace, name), timeout=timeout)

    async def list(self, res: Resource, namespace: Optional[str] = None, label_selector: Optional[str] = None,
                   field_selector: Optional[str] = None, resource_version: Optional[str] = None,
                   limit: int = 0, continue_: str = "", timeout: Optional[float] = None) -> dict:
        params = {}
        if limit:
            params["limit"] = str(limit)
        if continue_:
            params["continue"] = continue_
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        if resource_version is not None:
            params["resourceVersion"] = resource_version
        return await self.request("GET", res.path(namespace), params=params or None, timeout=timeout)

    async def create(self, res: Resource, obj: dict, namespace: Optional[str] = None,
                     timeout: Optional[float] = None) -> dict:
        ns = namespace or obj.get("metadata", {}).get("namespace")
        return await self.request("POST", res.path(ns), body=obj, timeout=timeout)

    async def replace(self, res: Resource, obj: dict, timeout: Optional[float] = None) -> dict:
        md = obj["metadata"]
        return await self.request("PUT", res.path(md.get("namespace"), md["name"]), body=obj, timeout=timeout)

    async def replace_status(self, res: Resource, obj: dict) -> dict:
        md = obj["metadata"]
        return await self.request("PUT", res.path(md.get("namespace"), md["name"], "status"), body=obj)

    async def patch(self, res: Resource, name: str, patch: Any, namespace: Optional[str] = None,
                    patch_type: str = "merge", sub: Optional[str] = None) -> dict:
        ct = {"merge": "application/merge-patch+json", "json": "application/json-patch+json",
              "strategic": "application/strategic-merge-patch+json"}[patch_type]
        return await self.request("PATCH", res.path(namespace, name, sub), body=patch, content_type=ct)

    async def delete(self, res: Resource, name: str, namespace: Optional[str] = None,
                     propagation: str = "Background") -> dict:
        return await self.request("DELETE", res.path(namespace, name),
                                  body={"kind": "DeleteOptions", "apiVersion": "v1", "propagationPolicy": propagation})

    # -- watch -------------------------------------------------------------------------------------
    async def watch(self, res: Resource, namespace: Optional[str] = None, resource_version: Optional[str] = None,
                    timeout_seconds: int = 300, label_selector: Optional[str] = None,
                    bookmarks: bool = True, field_selector: Optional[str] = None) -> AsyncIterator[Tuple[str, dict]]:
        """Yields (type, object) until the server closes the stream.  Raises ApiError(410) when
        ``resource_version`` is too old (an ERROR event with code 410 is translated too)."""
        params = {"watch": "true", "timeoutSeconds": str(timeout_seconds)}
        if resource_version:
            params["resourceVersion"] = resource_version
        if bookmarks:
            params["allowWatchBookmarks"] = "true"
        if label_selector:
            params["labelSelector"] = label_selector
        if field_selector:
            params["fieldSelector"] = field_selector
        s = await self._sess()
        self.requests += 1
        async with s.get(self.cfg.host + res.path(namespace), params=params, headers=self._headers(),
                         timeout=aiohttp.ClientTimeout(total=None, sock_read=timeout_seconds + 30)) as resp:
            if resp.status >= 400:
                raise await self._error(resp)
            buf = b""
            async for chunk in resp.content.iter_any():
                buf += chunk
                while b"\n" in buf:
                    line, buf = buf.split(b"\n", 1)
                    if not line.strip():
                        continue
                    ev = json.loads(line)
                    if ev.get("type") == "ERROR":
                        st = ev.get("object", {})
                        raise ApiError(int(st.get("code", 500)), st.get("reason", ""), st.get("message", ""), st)
                    yield ev["type"], ev["object"]

    # -- discovery ---------------------------------------------------------------------------------
    async def server_groups(self) -> List[str]:
        r = await self.request("GET", "/apis")
        return [g["name"] for g in r.get("groups", [])]


