"""Embedded workload templates for the link-discovery agent.

Counterpart of the reference's ``go:embed`` templates (reference config/discovery/discovery.go:26-81):
the YAML files next to this module are parsed once at import time — a malformed template
raises immediately, the equivalent of the reference's panic — and every accessor returns a
fresh deep copy so callers can mutate freely.
"""

from __future__ import annotations

import copy
from pathlib import Path

import yaml

_DIR = Path(__file__).resolve().parent


def _load(rel: str, kind: str) -> dict:
    obj = yaml.safe_load((_DIR / rel).read_text())
    if not isinstance(obj, dict) or obj.get("kind") != kind:
        raise RuntimeError(f"embedded template {rel} is not a {kind}")
    return obj


_DAEMONSET = _load("base/daemonset.yaml", "DaemonSet")
_SERVICE_ACCOUNT = _load("generic/linkdiscovery-serviceaccount.yaml", "ServiceAccount")
_OPENSHIFT_ROLEBINDING = _load("openshift/rolebinding.yaml", "RoleBinding")

LABEL_FEATURES_DIR = "/etc/kubernetes/node-feature-discovery/features.d/"


def discovery_daemonset() -> dict:
    """The agent DaemonSet (reference GaudiDiscoveryDaemonSet, discovery.go:35)."""
    return copy.deepcopy(_DAEMONSET)


def linkdiscovery_service_account() -> dict:
    """reference GaudiLinkDiscoveryServiceAccount (discovery.go:39)."""
    return copy.deepcopy(_SERVICE_ACCOUNT)


def openshift_role_binding() -> dict:
    """reference OpenShiftRoleBinding (discovery.go:43)."""
    return copy.deepcopy(_OPENSHIFT_ROLEBINDING)


__all__ = ["LABEL_FEATURES_DIR", "discovery_daemonset", "linkdiscovery_service_account", "openshift_role_binding"]
