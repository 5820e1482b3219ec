"""Prometheus metrics of the control plane.

controller-runtime exports reconcile counters / latency and work-queue gauges on the
metrics endpoint (reference cmd/operator/main.go:157-167); the same metric
names are used here so existing dashboards keep working, plus per-policy readiness gauges.
"""

from __future__ import annotations

from prometheus_client import CollectorRegistry, Counter, Gauge, Histogram, generate_latest
from prometheus_client.exposition import CONTENT_TYPE_LATEST


class OperatorMetrics:
    def __init__(self, registry: CollectorRegistry | None = None):
        self.registry = registry or CollectorRegistry()
        r = self.registry
        self.reconcile_total = Counter("controller_runtime_reconcile_total", "Total number of reconciliations per controller",
                                       ["controller", "result"], registry=r)
        self.reconcile_errors = Counter("controller_runtime_reconcile_errors_total",
                                        "Total number of reconciliation errors per controller", ["controller"], registry=r)
        self.reconcile_time = Histogram("controller_runtime_reconcile_time_seconds",
                                        "Length of time per reconciliation per controller", ["controller"],
                                        buckets=(0.001, 0.0025, 0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10),
                                        registry=r)
        self.queue_depth = Gauge("workqueue_depth", "Current depth of workqueue", ["name"], registry=r)
        self.queue_adds = Counter("workqueue_adds_total", "Total number of adds handled by workqueue", ["name"], registry=r)
        self.queue_retries = Counter("workqueue_retries_total", "Total number of retries handled by workqueue", ["name"],
                                     registry=r)
        self.dependency = Gauge("amd_network_operator_dependency_present",
                                "1 if a cluster add-on the operator relies on is installed", ["dependency"], registry=r)
        self.leader = Gauge("leader_election_master_status", "1 if this instance is the leader", ["name"], registry=r)
        self.policy_targets = Gauge("amd_network_operator_policy_targets", "Nodes targeted by a NetworkClusterPolicy",
                                    ["policy"], registry=r)
        self.policy_ready = Gauge("amd_network_operator_policy_ready",
                                  "Nodes whose agent published the scale-out readiness label", ["policy"], registry=r)
        # Node readiness as the operator sees it: the agent Pod's Ready condition (the readiness
        # probe checks the scale-out label), per policy.
        self.agent_ready_time = Histogram(
            "amd_network_operator_agent_ready_seconds",
            "Time from the operator first seeing an agent Pod to its Ready condition (node scale-out ready)",
            ["policy"], buckets=(0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 15, 30, 60, 120, 300, 600), registry=r)
        self.agent_unready = Counter("amd_network_operator_agent_unready_total",
                                     "Agent Pods that went from Ready to not Ready (link loss, lost peer, ...)",
                                     ["policy"], registry=r)
        # keepConfigOnRestart / disableNetworkManager: nodes owing a cleanup and how cleanups ended.
        self.nodes_owing_cleanup = Gauge("amd_network_operator_nodes_owing_cleanup",
                                         "Nodes whose agents left configuration a cleanup Job still has to remove",
                                         ["policy"], registry=r)
        self.policy_conflicts = Gauge("amd_network_operator_policy_conflicts",
                                      "Older policies of the same configurationType whose agents share nodes with this "
                                      "policy's (status.errors, Degraded reason PolicyConflict)",
                                      ["policy"], registry=r)
        self.node_cleanups = Counter("amd_network_operator_node_cleanups_total",
                                     "Node cleanup Jobs that ended, by outcome (succeeded, failed, timed_out)",
                                     ["policy", "outcome"], registry=r)
        self.crd_missing_fields = Gauge("amd_network_operator_crd_missing_fields",
                                        "Fields of this release's NetworkClusterPolicy schema the installed CRD lacks "
                                        "(helm upgrade never updates crds/: apply the release's CRD)", registry=r)
        self.seed_in_sync = Gauge("amd_network_operator_policies_file_in_sync",
                                  "1 when the policies of --policies-file (the Helm release's) match the cluster",
                                  registry=r)
        self.seed_errors = Counter("amd_network_operator_policies_file_errors_total",
                                   "Failed passes applying --policies-file (webhook not serving yet, rejected spec, ...)",
                                   registry=r)

    def render(self) -> bytes:
        return generate_latest(self.registry)

    content_type = CONTENT_TYPE_LATEST
