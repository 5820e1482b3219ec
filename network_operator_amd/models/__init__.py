"""Data models of the operator.

* the ``NetworkClusterPolicy`` object model, re-exported here from ``api.v1alpha1.types`` (no module
  of its own);
* ``topology`` — the node scale-out topology model: GPUs, NICs, GPU<->NIC PCIe pairing and the
  xGMI mesh, built from the native agent's sysfs / KFD discovery.
"""

from ..api.v1alpha1.types import (AmdScaleOutSpec, NetworkClusterPolicy, NetworkClusterPolicySpec,
                                  NetworkClusterPolicyStatus, new_policy)
from .topology import GpuNicPair, NodeTopology, XgmiMesh

__all__ = ["AmdScaleOutSpec", "NetworkClusterPolicy", "NetworkClusterPolicySpec", "NetworkClusterPolicyStatus",
           "new_policy", "GpuNicPair", "NodeTopology", "XgmiMesh"]
