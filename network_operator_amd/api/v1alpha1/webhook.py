"""Defaulting and validating admission logic for ``NetworkClusterPolicy``.

Mirrors the reference webhook (reference api/v1alpha1/networkconfiguration_webhook.go):

* ``default``: for ``amd-so`` with an empty image, set the default agent image (:65-74).
* ``validate_create`` / ``validate_update``: nodeSelector must be non-empty; every key
  <= 253 and value <= 63 characters; key prefix / name / value must match the same regular
  expressions (:83-85,91-119) — including the reference's quirk that the *prefix* regex
  does not accept ``-``; unknown ``configurationType`` -> ``UnknownConfigurationError``
  (:121-132).  ``validate_delete`` always allows (:149-153).
* ``admission_review``: the wire protocol (admission.k8s.io/v1 AdmissionReview) for the
  HTTPS server in ``network_operator_amd.operator.webhook_server``.  The mutating reply is
  an RFC 6902 JSONPatch.

The webhooks are registered for the *plural* resource ``networkclusterpolicies`` (the
reference registers the singular, so the API server never calls them — SURVEY.md §3.6).
"""

from __future__ import annotations

import base64
import copy
import json
import logging
import re
from typing import List, Optional, Tuple

from . import types as T

log = logging.getLogger("networkclusterpolicy-resource")

MUTATE_PATH = "/mutate-amd-com-v1alpha1-networkclusterpolicy"
VALIDATE_PATH = "/validate-amd-com-v1alpha1-networkclusterpolicy"

LABEL_HOST_RE = re.compile(r"^([A-Za-z0-9][A-Za-z0-9_\.]*)?[A-Za-z0-9]$")
LABEL_PATH_RE = re.compile(r"^([A-Za-z0-9][A-Za-z0-9-\._\/]*)?[A-Za-z0-9]$")
LABEL_VALUE_RE = re.compile(r"^(([A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?$")


class ValidationError(ValueError):
    message = "validation error"

    def __str__(self) -> str:  # same texts as the reference error types (:35-51)
        return self.message


class EmptyNodeSelectorError(ValidationError):
    message = "empty node-selector"


class InvalidNodeSelectorError(ValidationError):
    message = "invalid node selector"


class UnknownConfigurationError(ValidationError):
    message = "unknown error"


class InvalidInterfaceError(ValidationError):
    def __init__(self, name: str):
        super().__init__(name)
        self.message = f"invalid interface name {name!r}"


def default(policy: T.NetworkClusterPolicy) -> T.NetworkClusterPolicy:
    """The reference's Default (:65-74): the agent image.  MI355X-first defaults as well (the CRD
    schema carries them too, for webhooks-off installs): an amd-so policy verifies the node's
    xGMI mesh and requires every rail's RDMA device unless it says otherwise."""
    log.info("default name=%s", policy.name)
    so = policy.spec.amdScaleOut
    if policy.spec.configurationType == T.CONFIG_AMD_SCALE_OUT:
        if not so.image:
            so.image = T.DEFAULT_AGENT_IMAGE
        if so.xgmiCheck is None:
            so.xgmiCheck = True
        if so.requireRdma is None:
            so.requireRdma = True
    if policy.spec.configurationType == T.CONFIG_HOST_NIC and policy.spec.hostNic is not None \
            and not policy.spec.hostNic.image:
        policy.spec.hostNic.image = T.DEFAULT_AGENT_IMAGE
    return policy


def validate_node_selector(ns: dict) -> None:
    if not ns:
        raise EmptyNodeSelectorError()
    for k, v in ns.items():
        if not isinstance(k, str) or not isinstance(v, str):
            raise InvalidNodeSelectorError()
        if len(k) > 253 or len(v) > 63:
            raise InvalidNodeSelectorError()
        if not LABEL_VALUE_RE.match(v):
            raise InvalidNodeSelectorError()
        parts = k.split("/", 1)
        if len(parts) == 1:
            if not LABEL_HOST_RE.match(parts[0]):
                raise InvalidNodeSelectorError()
        else:
            if not LABEL_HOST_RE.match(parts[0]) or not LABEL_PATH_RE.match(parts[1]):
                raise InvalidNodeSelectorError()


RCCL_ENV_KEY_RE = re.compile(r"^(NCCL|RCCL|HSA)_[A-Z0-9_]+$")
# A Kubernetes qualified name (taint / toleration key): an optional DNS-subdomain prefix and "/",
# then a name of at most 63 characters.  (Not the reference's labelHostRegex quirk: taint keys
# such as node-role.kubernetes.io/... carry "-".)
QUALIFIED_NAME_RE = re.compile(r"^([a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*/)?"
                               r"[A-Za-z0-9]([-A-Za-z0-9_.]{0,61}[A-Za-z0-9])?$")


class InvalidRcclEnvError(ValidationError):
    def __init__(self, key: str):
        super().__init__(key)
        self.message = f"invalid rcclEnv entry {key!r}: keys must be NCCL_*, RCCL_* or HSA_*, values one line " \
                       "without ','"


class InvalidLldpWaitError(ValidationError):
    def __init__(self, value: str):
        super().__init__()
        self.message = (f"invalid lldpWait {value!r}: a duration such as 90s or 2m, between "
                        f"{int(T.LLDP_WAIT_MIN_S)}s and {int(T.LLDP_WAIT_MAX_S // 60)}m")


class InvalidCarrierWaitError(ValidationError):
    def __init__(self, value: str):
        super().__init__()
        self.message = (f"invalid carrierWait {value!r}: a duration such as 30s or 1m, between "
                        f"{int(T.CARRIER_WAIT_MIN_S)}s and {int(T.CARRIER_WAIT_MAX_S // 60)}m")


class InvalidRdmaWaitError(ValidationError):
    def __init__(self, value: str):
        super().__init__()
        self.message = (f"invalid rdmaWait {value!r}: a duration such as 5m or 10m, between "
                        f"{int(T.RDMA_WAIT_MIN_S)}s and {int(T.RDMA_WAIT_MAX_S // 60)}m")


class InvalidRailSwitchPatternError(ValidationError):
    def __init__(self, value: str, why: str):
        super().__init__()
        self.message = f"invalid railSwitchPattern {value!r}: {why}"


# Escapes both engines read the same way: ECMAScript's character-class and control escapes
# (std::regex, the agent) and Python's re (admission).  Any other letter or digit escape is either
# unknown to one of them (\A \Z \z \G \Q \E \h \R \K \p \P \N \k ...) or means something
# else (\0 followed by digits is an octal escape in Python).
_ESCAPE_LETTERS = set("dDwWsSbfnrtv")  # not \B: on an empty name Python says no, ECMAScript yes
_SYNTAX = set("^$\\.*+?()[]{}|/-")
MAX_RAILS = 16  # the agent's kMaxRails: {rail} is checked for every index 0..15


def ecmascript_subset_error(pattern: str) -> Optional[str]:
    """None when `pattern` stays inside the regular-expression subset that ECMAScript std::regex
    (the agent) and Python's re (this webhook) both accept and read alike; else why not.

    Refused: ``(?`` groups other than ``(?:``, ``(?=``, ``(?!`` -- inline flags ``(?i)``,
    lookbehind ``(?<=``, named groups ``(?P<n>``/``(?<n>``, atomic ``(?>``, comments ``(?#``;
    the escapes above; possessive quantifiers (``*+``, ``++``, ``?+``, ``}+``); ``{,n}``;
    quantified assertions; POSIX bracket expressions (``[[:alpha:]]``, an ordinary set in
    Python) and Python's reserved set syntax in classes; multi-digit back-references.  Found by
    sweeping random patterns through both engines (tests/test_operator.py)."""
    i, n = 0, len(pattern)
    in_class = False
    prev_quant = False  # the previous token was a quantifier (for possessive detection)
    prev_assert = False  # ... an assertion (^ $ \b \B (?= (?!): ECMAScript refuses to quantify it
    groups: List[bool] = []  # open groups: True for lookaheads
    while i < n:
        c = pattern[i]
        if not in_class and c in "*+?{" and prev_assert:
            return "quantified assertion (^, $, \\b, \\B or a lookahead)"
        prev_assert = False
        if c == "\\":
            if i + 1 >= n:
                return "trailing backslash"
            e = pattern[i + 1]
            if e.isdigit():
                if e == "0":
                    if i + 2 < n and pattern[i + 2].isdigit():
                        return f"octal escape \\0{pattern[i + 2]} (Python reads it as octal, ECMAScript as NUL then a digit)"
                elif not in_class and i + 2 < n and pattern[i + 2].isdigit():
                    return "multi-digit back-reference"
                elif in_class:
                    return f"back-reference \\{e} inside a character class"
                i += 2
            elif e == "x":
                if not re.fullmatch(r"[0-9A-Fa-f]{2}", pattern[i + 2:i + 4]):
                    return "\\x needs two hex digits"
                i += 4
            elif e == "u":
                if not re.fullmatch(r"[0-9A-Fa-f]{4}", pattern[i + 2:i + 6]):
                    return "\\u needs four hex digits"
                i += 6
            elif e == "c":
                return "control escape \\c (not in Python's re)"
            elif e.isalpha():
                if e not in _ESCAPE_LETTERS:
                    return f"escape \\{e} (not the same in ECMAScript and Python)"
                prev_assert = e == "b" and not in_class
                if prev_assert and any(groups):
                    return "\\b inside a lookahead (the engines disagree at the end of the name)"
                i += 2
            elif e in _SYNTAX or not e.isalnum():
                i += 2
            else:
                return f"escape \\{e}"
            prev_quant = False
            continue
        if in_class:
            if c == "[" and i + 1 < n and pattern[i + 1] in ":=.":
                return "POSIX bracket expression (e.g. [[:alpha:]]) inside a character class"
            if c == "[":  # a literal in both today; Python reserves it for nested sets (FutureWarning)
                return "unescaped '[' inside a character class (write \\[)"
            if pattern.startswith(("--", "&&", "~~", "||"), i):
                return f"{pattern[i:i + 2]!r} inside a character class (reserved for set operations in Python)"
            if c == "]":
                in_class = False
            i += 1
            continue
        if c == "[":
            in_class = True
            i += 1
            if i < n and pattern[i] == "^":
                i += 1
            if i < n and pattern[i] == "]":  # a literal ']' first: Python only ('[]' is empty in ECMAScript)
                return "']' first in a character class (a literal in Python, an empty class in ECMAScript)"
            prev_quant = False
            continue
        if c == "(":
            if pattern.startswith("(?", i):
                if not pattern.startswith(("(?:", "(?=", "(?!"), i):
                    return f"group construct {pattern[i:i + 4]!r} (only (?: (?= (?! are read alike)"
                groups.append(pattern[i + 2] != ":")
                i += 3
            else:
                groups.append(False)
                i += 1
            prev_quant = False
            continue
        if c == ")":
            prev_assert = bool(groups) and groups.pop()
            prev_quant = False
            i += 1
            continue
        if c in "^$":
            if any(groups):
                return f"{c!r} inside a lookahead"
            prev_assert = True
            prev_quant = False
            i += 1
            continue
        if c in "*+?":
            if prev_quant and c == "+":
                return "possessive quantifier (not in ECMAScript or this Python)"
            if prev_quant and c == "?":
                prev_quant = False  # lazy: fine in both
                i += 1
                continue
            prev_quant = True
            i += 1
            continue
        if c == "{":
            m = re.match(r"\{(\d*)(,?)(\d*)\}", pattern[i:])
            if m:
                if m.group(1) == "":
                    return "quantifier {,n} (ECMAScript needs a lower bound)"
                prev_quant = True
                i += m.end()
                continue
            return "'{' not starting a quantifier (escape it as \\{)"
        if c == "}":
            return "unbalanced '}' (escape it as \\})"
        prev_quant = False
        i += 1
    if in_class:
        return "unterminated character class"
    return None


def validate_rail_switch_pattern(value: str) -> None:
    """A regular expression over the switch's LLDP System Name, "{rail}" standing for the GPU
    index.  The agent matches with ECMAScript std::regex; admission accepts only what both that
    and Python's re compile and read alike (ecmascript_subset_error), for every rail index the
    agent substitutes, so a policy it admits never fails on the nodes (tests/test_operator.py
    feeds one corpus to both engines)."""
    if not value:
        return
    if len(value) > 253 or any(c in value for c in "\n\r"):
        raise InvalidRailSwitchPatternError(value, "at most 253 characters on one line")
    for k in range(MAX_RAILS):
        p = value.replace("{rail}", str(k))
        why = ecmascript_subset_error(p)
        if why is None:
            try:
                re.compile(p)
            except re.error as e:
                why = str(e)
        if why is not None:
            raise InvalidRailSwitchPatternError(value, why + ("" if k == 0 else f" (with {{rail}} = {k})")) from None


class InvalidMaxUnavailableError(ValidationError):
    def __init__(self, value):
        super().__init__()
        self.message = f"invalid maxUnavailable {value!r}: a number >= 1 or a percentage 1%..100%"


def validate_max_unavailable(value) -> None:
    import re

    if value is None:
        return
    if isinstance(value, bool) or not (isinstance(value, int) and value >= 1 or
                                       isinstance(value, str) and re.fullmatch(r"(100|[1-9][0-9]?)%", value)):
        raise InvalidMaxUnavailableError(value)


def validate_lldp_wait(value: str) -> None:
    if not value:
        return
    try:
        secs = T.parse_go_duration(value)
    except ValueError:
        raise InvalidLldpWaitError(value) from None
    if not T.LLDP_WAIT_MIN_S <= secs <= T.LLDP_WAIT_MAX_S:
        raise InvalidLldpWaitError(value)


def validate_carrier_wait(value: str) -> None:
    if not value:
        return
    try:
        secs = T.parse_go_duration(value)
    except ValueError:
        raise InvalidCarrierWaitError(value) from None
    if not T.CARRIER_WAIT_MIN_S <= secs <= T.CARRIER_WAIT_MAX_S:
        raise InvalidCarrierWaitError(value)


def validate_rdma_wait(value: str) -> None:
    if not value:
        return
    try:
        secs = T.parse_go_duration(value)
    except ValueError:
        raise InvalidRdmaWaitError(value) from None
    if not T.RDMA_WAIT_MIN_S <= secs <= T.RDMA_WAIT_MAX_S:
        raise InvalidRdmaWaitError(value)


def image_tag(image: str) -> str:
    """The tag of an image reference ("" for a digest or no tag)."""
    if "@" in image:
        return ""
    name = image.rsplit("/", 1)[-1]
    return name.split(":", 1)[1] if ":" in name else ""


ALLOW_POLICY_ROUTED_WARNING = ("allowPolicyRouted: the agent flushes and re-MTUs a selected NIC even when its default route in a "
                               "policy-routing table carries the node's own address; if the node reaches a network through "
                               "it, configuring it can cut the node off")


def validate_amd_so_spec(s: T.AmdScaleOutSpec) -> List[str]:
    """Returns admission warnings.  (The reference's validateGaudiSoSpec is a no-op, :87-89.)"""
    warnings = []
    if s.layer == "L2" and s.lldpAnnounce is not None:  # the agent announces only in L3 (agent_monitor.cpp)
        warnings.append("lldpAnnounce has no effect in L2 mode")
    for i in s.interfaces:
        if not i or len(i) > 15 or "/" in i or " " in i or "," in i:
            raise InvalidInterfaceError(i)
    for k, v in s.rcclEnv.items():
        if not RCCL_ENV_KEY_RE.match(str(k)) or not isinstance(v, str) or any(c in v for c in "\n\r,"):
            raise InvalidRcclEnvError(str(k))
    validate_lldp_wait(s.lldpWait)
    if s.lldpWait and s.layer == "L2":
        warnings.append("lldpWait has no effect in L2 mode")
    validate_carrier_wait(s.carrierWait)
    if s.carrierWait and s.layer == "L3":
        warnings.append("carrierWait has no effect in L3 mode (the LLDP wait covers link training)")
    validate_rail_switch_pattern(s.railSwitchPattern)
    if s.railSwitchPattern and s.layer == "L2":
        warnings.append("railSwitchPattern has no effect in L2 mode (no LLDP)")
    if s.handDcbxToHost and not (s.disableFirmwareLldp and s.layer == "L3"):
        warnings.append("handDcbxToHost has no effect without disableFirmwareLldp in L3 mode")
    if s.checkPeerMtu is not None and s.layer == "L2":
        warnings.append("checkPeerMtu has no effect in L2 mode (no LLDP)")
    validate_rdma_wait(s.rdmaWait)
    if s.rdmaWait and s.requireRdma is False:
        warnings.append("rdmaWait has no effect with requireRdma false")
    if s.requireRdma is False:
        warnings.append("requireRdma false: nodes whose scale-out NICs have no RDMA device are labelled scale-out "
                        "ready, and RCCL falls back to TCP sockets on those rails")
    if s.allowPolicyRouted:
        warnings.append(ALLOW_POLICY_ROUTED_WARNING)
    tag = image_tag(s.image)
    if s.image and tag not in ("", "latest", T.OPERATOR_VERSION):
        # the operator passes the flags of its own agent release; an older agent binary
        # exits on the first flag it does not know, on every selected node.
        warnings.append(f"image pins agent tag {tag!r}: this operator ({T.OPERATOR_VERSION}) passes flags of its own agent "
                        "release (e.g. --link-state, --require-rdma, --label-holddown); an older agent exits on a flag "
                        "it does not know")
    return warnings


class MissingHostNicSpecError(ValidationError):
    message = "configurationType host-nic needs spec.hostNic with a layer"


def validate_host_nic_spec(s: Optional[T.HostNicSpec]) -> List[str]:
    if s is None or s.layer not in T.LAYERS:
        raise MissingHostNicSpecError()
    for i in s.interfaces:
        if not i or len(i) > 15 or "/" in i or " " in i or "," in i:
            raise InvalidInterfaceError(i)
    validate_lldp_wait(s.lldpWait)
    validate_carrier_wait(s.carrierWait)
    warnings = []
    if s.carrierWait and s.layer == "L3":
        warnings.append("hostNic: carrierWait has no effect in L3 mode (the LLDP wait covers link training)")
    if not s.interfaces and not s.nicDrivers:
        warnings.append("hostNic: no interfaces or nicDrivers given; every RDMA NIC of the default driver list "
                        "that is neither a GPU's scale-out rail nor the node's own NIC (default route, non-/30 "
                        "address) will be configured")
    if s.allowPolicyRouted:
        warnings.append("hostNic." + ALLOW_POLICY_ROUTED_WARNING)
    if s.includeGpuRails and s.interfaces:
        warnings.append("hostNic.includeGpuRails has no effect with interfaces (the named NICs are taken as named)")
    elif s.includeGpuRails:
        warnings.append("hostNic.includeGpuRails: the GPUs' scale-out NICs are configured by this policy; an amd-so "
                        "policy on the same nodes would find them taken (its agent waits for their NIC locks)")
    return warnings


class InvalidTolerationError(ValidationError):
    def __init__(self, why: str):
        super().__init__(why)
        self.message = f"invalid toleration: {why}"


def validate_tolerations(tolerations: List[dict]) -> None:
    """The API server's own rules for a Pod toleration (the DaemonSet would be refused with them
    otherwise, long after admission): Exists takes no value; Equal (the default) needs a key; a
    tolerationSeconds only with NoExecute; a key is a qualified name."""
    for t in tolerations:
        if not isinstance(t, dict):
            raise InvalidTolerationError(f"{t!r} is not an object")
        op = t.get("operator") or "Equal"
        key, value, effect = t.get("key") or "", t.get("value") or "", t.get("effect") or ""
        if op == "Exists" and value:
            raise InvalidTolerationError(f"{key or '<any key>'}: operator Exists takes no value")
        if op == "Equal" and not key:
            raise InvalidTolerationError("operator Equal (the default) needs a key")
        if t.get("tolerationSeconds") is not None and effect != "NoExecute":
            raise InvalidTolerationError(f"{key}: tolerationSeconds only applies to effect NoExecute")
        if key and not QUALIFIED_NAME_RE.fullmatch(key):
            raise InvalidTolerationError(f"{key!r} is not a qualified name")


def validate_spec(spec: T.NetworkClusterPolicySpec) -> List[str]:
    validate_node_selector(spec.nodeSelector)
    validate_max_unavailable(spec.maxUnavailable)
    validate_tolerations(spec.tolerations)
    if spec.configurationType == T.CONFIG_AMD_SCALE_OUT:
        return validate_amd_so_spec(spec.amdScaleOut)
    if spec.configurationType == T.CONFIG_HOST_NIC:
        return validate_host_nic_spec(spec.hostNic)
    raise UnknownConfigurationError()


def validate_create(policy: T.NetworkClusterPolicy) -> List[str]:
    log.info("validate create name=%s", policy.name)
    return validate_spec(policy.spec)


def validate_update(policy: T.NetworkClusterPolicy, old: Optional[T.NetworkClusterPolicy] = None) -> List[str]:
    log.info("validate update name=%s", policy.name)
    return validate_spec(policy.spec)


def overlap_warnings(policy: T.NetworkClusterPolicy, others: List[dict]) -> List[str]:
    """Admission warnings for the live policies of ``policy``'s configurationType whose
    nodeSelector can match a node ``policy``'s matches too (no key required at two values).  A
    node belongs to the older policy of a type (operator/holdoff.py hold_off_terms): the newer
    one's agents are held off it.  ``policy`` without a creationTimestamp is being created, so it
    is the newest.  Which nodes actually match both is the operator's to say (status.errors)."""
    mine = dict(policy.spec.nodeSelector)
    me = (policy.metadata.get("creationTimestamp") or "\uffff", policy.name)
    out = []
    for q in sorted(others, key=lambda o: (o.get("metadata") or {}).get("name", "")):
        md = q.get("metadata") or {}
        spec = q.get("spec") or {}
        if md.get("name") == policy.name or md.get("deletionTimestamp") or \
                spec.get("configurationType", "") != policy.spec.configurationType:
            continue
        sel = dict(spec.get("nodeSelector") or {})
        if any(k in mine and mine[k] != v for k, v in sel.items()):
            continue  # disjoint selections
        older = (md.get("creationTimestamp") or "", md.get("name", "")) < me
        if older:
            out.append(f"policy {md['name']} ({policy.spec.configurationType} too, created earlier) can select the same "
                       f"nodes: those stay with it, and this policy's agents are held off them")
        else:
            out.append(f"policy {md['name']} ({policy.spec.configurationType} too, created later) can select the same "
                       f"nodes: they belong to this policy, and its agents are held off them")
    return out


def validate_delete(policy: T.NetworkClusterPolicy) -> List[str]:
    log.info("validate delete name=%s", policy.name)
    return []


# ---------------------------------------------------------------------------
# AdmissionReview wire protocol
# ---------------------------------------------------------------------------
def json_patch(before, after, path: str = "") -> list:
    """Minimal RFC 6902 diff (add / replace / remove) between two JSON documents."""
    ops = []
    if isinstance(before, dict) and isinstance(after, dict):
        for k in before:
            p = f"{path}/{_esc(k)}"
            if k not in after:
                ops.append({"op": "remove", "path": p})
            else:
                ops.extend(json_patch(before[k], after[k], p))
        for k in after:
            if k not in before:
                ops.append({"op": "add", "path": f"{path}/{_esc(k)}", "value": after[k]})
        return ops
    if before != after:
        ops.append({"op": "replace", "path": path or "/", "value": after})
    return ops


def _esc(k: str) -> str:
    return str(k).replace("~", "~0").replace("/", "~1")


def admission_review(review: dict, mutate: bool) -> dict:
    """Handles one admission.k8s.io/v1 AdmissionReview request and returns the response review."""
    req = review.get("request") or {}
    uid = req.get("uid", "")
    resp: dict = {"uid": uid, "allowed": True}
    op = req.get("operation", "")
    try:
        if mutate:
            obj = req.get("object") or {}
            before = copy.deepcopy(obj)
            pol = default(T.NetworkClusterPolicy.from_dict(obj))
            after = copy.deepcopy(obj)
            after["spec"] = pol.spec.to_dict()
            ops = json_patch(before, after)
            if ops:
                resp["patchType"] = "JSONPatch"
                resp["patch"] = base64.b64encode(json.dumps(ops).encode()).decode()
        else:
            warnings: List[str] = []
            if op == "CREATE":
                warnings = validate_create(T.NetworkClusterPolicy.from_dict(req.get("object") or {}))
            elif op == "UPDATE":
                warnings = validate_update(T.NetworkClusterPolicy.from_dict(req.get("object") or {}),
                                           T.NetworkClusterPolicy.from_dict(req.get("oldObject") or {}))
            elif op == "DELETE":
                warnings = validate_delete(T.NetworkClusterPolicy.from_dict(req.get("oldObject") or {}))
            if warnings:
                resp["warnings"] = warnings
    except ValueError as e:
        resp = {"uid": uid, "allowed": False, "status": {"code": 403, "message": str(e), "reason": "Forbidden"}}
    return {"apiVersion": "admission.k8s.io/v1", "kind": "AdmissionReview", "response": resp}


def decode_patch(resp_review: dict) -> Tuple[Optional[str], list]:
    r = resp_review.get("response", {})
    if "patch" not in r:
        return None, []
    return r.get("patchType"), json.loads(base64.b64decode(r["patch"]))
