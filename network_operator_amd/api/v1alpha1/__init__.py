"""``amd.com/v1alpha1`` API (reference api/v1alpha1)."""

from .types import (API_VERSION, CONFIG_AMD_SCALE_OUT, DEFAULT_AGENT_IMAGE, GROUP, KIND, LIST_KIND, PLURAL, SINGULAR,
                    VERSION, AmdScaleOutSpec, NetworkClusterPolicy, NetworkClusterPolicySpec,
                    NetworkClusterPolicyStatus, new_policy)

__all__ = ["API_VERSION", "CONFIG_AMD_SCALE_OUT", "DEFAULT_AGENT_IMAGE", "GROUP", "KIND", "LIST_KIND", "PLURAL",
           "SINGULAR", "VERSION", "AmdScaleOutSpec", "NetworkClusterPolicy", "NetworkClusterPolicySpec",
           "NetworkClusterPolicyStatus", "new_policy"]
