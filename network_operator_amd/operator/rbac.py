"""The operator's Kubernetes permissions, as data.

This table is the single source of the RBAC the deploy manifests grant
(``network_operator_amd.packaging.manifests`` renders it into the kustomize tree, the Helm
chart and the OLM bundle).  The reference declares the same thing as kubebuilder markers on
the reconciler (reference internal/controller/networkconfiguration_controller.go:40-47) and
lets controller-gen write role.yaml; here the table is checked the other way round as well:
``tests/test_manager.py::test_operator_requests_stay_within_generated_rbac`` records every
request the running operator makes against the fake API server and fails on any request the
table does not allow.

Rules are grouped by API group and verb set, not one rule per resource.
"""

from __future__ import annotations

from typing import Dict, Iterable, List, Sequence, Tuple

READ = ("get", "list", "watch")
WRITE = ("create", "update", "patch", "delete")

# (apiGroup, resources, verbs): cluster-wide, bound to the operator's ServiceAccount.
OPERATOR_CLUSTER_RULES: Tuple[Tuple[str, Tuple[str, ...], Tuple[str, ...]], ...] = (
    # The policies it reconciles, their status subresource and finalizers.
    ("amd.com", ("networkclusterpolicies",), READ + WRITE),
    ("amd.com", ("networkclusterpolicies/status",), ("get", "update", "patch")),
    ("amd.com", ("networkclusterpolicies/finalizers",), ("update",)),
    # Agent DaemonSets (owned) and their pods (per-node readiness errors in status.errors).
    ("apps", ("daemonsets",), READ + WRITE),
    ("", ("pods",), READ),
    # Which nodes a newer policy of one type is held off (the ones an older policy selects too):
    # a LIST by label selector, three names at most, and only while two policies overlap.  GET:
    # the uid of a node an Event is recorded on (kubectl describe node matches events by it).
    ("", ("nodes",), ("get", "list")),
    # Agent ServiceAccount + OpenShift SCC RoleBinding (created on OpenShift only).
    ("", ("serviceaccounts",), ("get", "list", "create", "update", "delete")),
    ("rbac.authorization.k8s.io", ("rolebindings",), ("get", "list", "create", "update", "delete")),
    # Fabric validation Jobs (amdScaleOut.validation), one per ready node, owned by the policy.
    ("batch", ("jobs",), READ + ("create", "delete")),
    # Events on the policies (the reference grants read only and never emits any).
    ("", ("events",), ("create", "patch") + READ),
)

# Namespaced (the operator namespace): leader election.
LEADER_ELECTION_RULES = (
    ("coordination.k8s.io", ("leases",), READ + WRITE),
    ("", ("events",), ("create", "patch")),
)

# --metrics-secure: authenticate and authorise scrapers with TokenReview / SubjectAccessReview.
METRICS_AUTH_RULES = (
    ("authentication.k8s.io", ("tokenreviews",), ("create",)),
    ("authorization.k8s.io", ("subjectaccessreviews",), ("create",)),
)

# Helm install only: the policy seeder (operator/seeder.py) reads its own ClusterRole, the owner it
# makes the chart's policies dependents of.  Scoped to that one object by resourceNames.
def policy_owner_rule(cluster_role: str) -> dict:
    return {"apiGroups": ["rbac.authorization.k8s.io"], "resources": ["clusterroles"], "verbs": ["get"],
            "resourceNames": [cluster_role]}


# The installed NetworkClusterPolicy CRD, read to tell when it is older than the operator (Helm
# never upgrades crds/; manager.py::check_crd).  Scoped to that one object by resourceNames.
CRD_NAME = "networkclusterpolicies.amd.com"


def crd_read_rule() -> dict:
    return {"apiGroups": ["apiextensions.k8s.io"], "resources": ["customresourcedefinitions"], "verbs": ["get"],
            "resourceNames": [CRD_NAME]}


# Aggregated user-facing roles for NetworkClusterPolicy.
POLICY_EDITOR_RULES = (
    ("amd.com", ("networkclusterpolicies",), READ + WRITE),
    ("amd.com", ("networkclusterpolicies/status",), ("get",)),
)
POLICY_VIEWER_RULES = (
    ("amd.com", ("networkclusterpolicies",), READ),
    ("amd.com", ("networkclusterpolicies/status",), ("get",)),
)


def rules(table: Iterable[Tuple[str, Sequence[str], Sequence[str]]]) -> List[Dict[str, List[str]]]:
    """Kubernetes PolicyRule list for a table."""
    return [{"apiGroups": [g], "resources": list(r), "verbs": list(v)} for g, r, v in table]


def allows(policy_rules: Iterable[dict], verb: str, group: str, resource: str) -> bool:
    """Whether ``policy_rules`` grant ``verb`` on ``group/resource`` (``resource`` may carry a
    ``/subresource``); ``*`` wildcards honoured."""
    for r in policy_rules:
        if ("*" in r.get("apiGroups", []) or group in r.get("apiGroups", [])) and \
                ("*" in r.get("resources", []) or resource in r.get("resources", [])) and \
                ("*" in r.get("verbs", []) or verb in r.get("verbs", [])):
            return True
    return False
