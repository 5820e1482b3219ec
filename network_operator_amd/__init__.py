"""MI355X-native Kubernetes network operator.

A from-scratch, AMD Instinct MI355X-first re-design of the capabilities of the Intel Gaudi
network operator (tkatila/network-operator):

* ``network_operator_amd.api``        v1alpha1 ``NetworkClusterPolicy`` API (types, defaulting,
                                       validation, CRD schema)            — reference ``api/v1alpha1``
* ``network_operator_amd.operator``   control plane: reconciler, informers, work queue, leader
                                       election, webhooks, metrics       — reference ``cmd/operator``,
                                                                            ``internal/controller``
* ``network_operator_amd.discovery``  embedded DaemonSet / ServiceAccount / RoleBinding templates
                                                                          — reference ``config/discovery``
* ``network_operator_amd.agent``      Python view of the native C++ node agent (``discover``):
                                       LLDP, rtnetlink, D-Bus, sysfs/xGMI topology
                                                                          — reference ``cmd/discover``,
                                                                            ``pkg/lldp``, ``internal/nm``
* ``network_operator_amd.ops``        HIP/gfx950 validation kernels (ctypes over libnetop_hip.so)
* ``network_operator_amd.parallel``   RCCL-over-xGMI validation (all-reduce busbw, rccl-tests math)
* ``network_operator_amd.testing``    fake Kubernetes API server, netns/veth synthetic-switch harness
* ``network_operator_amd.utils``      paths, logging, shared helpers
"""

__version__ = "0.1.0"

GROUP = "amd.com"
VERSION = "v1alpha1"
KIND = "NetworkClusterPolicy"
PLURAL = "networkclusterpolicies"
