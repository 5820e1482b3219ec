"""Workload objects of the link-discovery agent, built in code.

The reference embeds YAML templates with ``go:embed`` and panics if one does not parse
(reference config/discovery/discovery.go:26-81, config/discovery/base/daemonset.yaml).  Here
the objects are constructed from the constants below, so there is nothing to parse at run
time; the reconciler specialises a fresh copy per policy
(``operator/templates.py::update_daemonset_for``).

What the agent pod needs, and why:

* ``hostNetwork`` — it configures the node's own NICs and exchanges LLDP on them;
* ``NET_ADMIN`` (rtnetlink) and ``NET_RAW`` (AF_PACKET), every other capability dropped,
  read-only root filesystem, no privilege escalation;
* the NFD ``features.d`` directory of the host, where the readiness label file goes;
* a readiness probe (``discover --ready-check``) so ``status.ready`` counts nodes that are
  actually configured, not pods that merely started (the reference's agent has no probe);
* the reference DaemonSet's requests (40m / 45Mi) and memory limit (90Mi), which the agent's
  measured 5 MiB peak RSS sits far inside.  The CPU limit is 500m, not the reference's 100m:
  a bring-up costs the agent ~10 ms of CPU (8 NICs, getrusage at readiness, topology file
  included), which is the whole 10 ms per 100 ms CFS period that 100m allows.  At 100m the
  node's readiness would wait out the rest of a throttled period.  After bring-up the agent is
  idle (epoll), so the higher limit costs nothing in steady state.
"""

from __future__ import annotations

from typing import Dict, List

AGENT_APP_LABEL = "amd-network-tools"  # pod label; the operator's pod informer selects on it
AGENT_CONTAINER = "configurator"
AGENT_IMAGE = "amd/amd-network-linkdiscovery:latest"
AGENT_BINARY = "/usr/local/bin/discover"
AGENT_SERVICE_ACCOUNT = "linkdiscovery-sa"
OPENSHIFT_PRIVILEGED_SCC = "system:openshift:scc:privileged"

LABEL_FEATURES_DIR = "/etc/kubernetes/node-feature-discovery/features.d/"
# The agent's status file, in a per-Pod emptyDir: the readiness probe prints the reason the node
# is not ready from beside it, and the kubelet keeps that output in the Pod's events.
AGENT_RUN_DIR = "/run/amd-network-agent"
AGENT_STATUS_FILE = AGENT_RUN_DIR + "/status.json"

AGENT_REQUESTS = {"cpu": "40m", "memory": "45Mi"}
AGENT_LIMITS = {"cpu": "500m", "memory": "90Mi"}
AGENT_CAPABILITIES = ["NET_ADMIN", "NET_RAW"]
TERMINATION_GRACE_S = 10


def _host_dir(name: str, path: str) -> Dict:
    return {"name": name, "hostPath": {"path": path, "type": "DirectoryOrCreate"}}


def _agent_container() -> Dict:
    return {
        "name": AGENT_CONTAINER,
        "image": AGENT_IMAGE,
        "imagePullPolicy": "IfNotPresent",
        # NODE_NAME names the node in the agent's status file and logs (unused by the reference).
        "env": [{"name": "NODE_NAME",
                 "valueFrom": {"fieldRef": {"apiVersion": "v1", "fieldPath": "spec.nodeName"}}}],
        "readinessProbe": {"exec": {"command": [AGENT_BINARY, "--ready-check", f"--status-file={AGENT_STATUS_FILE}"]},
                           "initialDelaySeconds": 1, "periodSeconds": 5, "failureThreshold": 1},
        "resources": {"limits": dict(AGENT_LIMITS), "requests": dict(AGENT_REQUESTS)},
        "volumeMounts": [{"mountPath": LABEL_FEATURES_DIR, "name": "nfd-features"},
                         {"mountPath": AGENT_RUN_DIR, "name": "agent-run"}],
        # A failed start ends with the agent's one-line "Error: ..." on stderr; with this policy the
        # kubelet keeps the log tail as the container's termination message, and the operator
        # quotes it in the policy's status.errors (not in the reference).
        "terminationMessagePolicy": "FallbackToLogsOnError",
        "securityContext": {"allowPrivilegeEscalation": False, "readOnlyRootFilesystem": True,
                            "capabilities": {"drop": ["ALL"], "add": list(AGENT_CAPABILITIES)}},
    }


def discovery_daemonset() -> Dict:
    """The agent DaemonSet before specialisation (reference GaudiDiscoveryDaemonSet,
    discovery.go:35).  One node at a time is updated (maxUnavailable 1, no surge: two agents
    must never configure the same NICs at once)."""
    labels = {"app": AGENT_APP_LABEL}
    return {
        "apiVersion": "apps/v1",
        "kind": "DaemonSet",
        "metadata": {"name": AGENT_APP_LABEL, "labels": dict(labels)},
        "spec": {
            "selector": {"matchLabels": dict(labels)},
            "updateStrategy": {"type": "RollingUpdate", "rollingUpdate": {"maxSurge": 0, "maxUnavailable": 1}},
            "template": {
                "metadata": {"labels": dict(labels)},
                "spec": {
                    "hostNetwork": True,
                    "volumes": [_host_dir("nfd-features", LABEL_FEATURES_DIR),
                                {"name": "agent-run", "emptyDir": {"medium": "Memory", "sizeLimit": "1Mi"}}],
                    "containers": [_agent_container()],
                    "terminationGracePeriodSeconds": TERMINATION_GRACE_S,
                },
            },
        },
    }


def linkdiscovery_service_account() -> Dict:
    """ServiceAccount of the agent pods (reference GaudiLinkDiscoveryServiceAccount, discovery.go:39)."""
    return {"apiVersion": "v1", "kind": "ServiceAccount", "metadata": {"name": AGENT_SERVICE_ACCOUNT}}


def openshift_role_binding(namespace: str = "") -> Dict:
    """Binds the agent ServiceAccount to OpenShift's privileged SCC (reference
    OpenShiftRoleBinding, discovery.go:43); the reconciler names it ``<policy>-sa-rb``."""
    subject: Dict[str, str] = {"kind": "ServiceAccount", "name": AGENT_SERVICE_ACCOUNT}
    if namespace:
        subject["namespace"] = namespace
    return {
        "apiVersion": "rbac.authorization.k8s.io/v1",
        "kind": "RoleBinding",
        "metadata": {"name": "linkdiscovery-openshift-privileged"},
        "roleRef": {"apiGroup": "rbac.authorization.k8s.io", "kind": "ClusterRole", "name": OPENSHIFT_PRIVILEGED_SCC},
        "subjects": [subject],
    }


__all__: List[str] = ["AGENT_APP_LABEL", "LABEL_FEATURES_DIR", "discovery_daemonset", "linkdiscovery_service_account",
                      "openshift_role_binding"]
