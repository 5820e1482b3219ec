"""One node, one agent per configurationType: which policy a node belongs to when two of a type
select it, and how the others are kept off it (node affinity built from the older selectors).
See the comment below and docs/ARCHITECTURE.md "Two policies of one type".
"""

from __future__ import annotations

import copy
from typing import Dict, List, Optional

# Two policies of one configurationType that select the same node would run two agents there;
# they share the node lock (named after the type's NFD label), so the later one would wait and
# then fail, restarting forever.  Instead a node belongs to the OLDEST live policy of the type
# whose nodeSelector matches it: every newer one's DaemonSet carries a required node-affinity
# term that excludes the nodes the older selectors match, so its agents are never placed there.
# The term is built from the selectors, not from a node list: it does not change when nodes come,
# go or get relabelled (a DaemonSet template change rolls every agent of the policy), only when
# an older policy's selector does.  The newer policy's status names the held-off nodes
# (Degraded/PolicyConflict, a Warning Event); once the older policy goes, the term goes with it
# and the newer policy's agents take those nodes.  (The reference has no guard at all,
# internal/controller/networkconfiguration_controller.go:164-204,313-362.)
CONFLICT_MARK = ": also selected by policy "
# A node-selector term no node matches (no node carries this label): a newer policy whose
# every node an older one selects.
HELD_EVERYWHERE_KEY = "network.amd.com/held-off-by-an-older-policy"
MAX_HOLD_OFF_TERMS = 64  # required terms are ORed: the hold-off expands to at most this many
# While an older selector overlaps, the held-off nodes are read again this often: a node
# relabelled into or out of the overlap moves no Pod of this policy, so no event would.
HELD_OFF_REFRESH_S = 30.0


def hold_off_terms(mine: Dict[str, str], older: List[Dict[str, str]]) -> Optional[List[dict]]:
    """nodeSelectorTerms (ORed) of the nodes ``mine`` (a nodeSelector) selects that no selector in
    ``older`` matches, to AND with ``mine``; None when nothing is held off.

    Not matching {k1: v1, k2: v2} is (k1 NotIn [v1]) OR (k2 NotIn [v2]) (NotIn also matches a node
    without the label).  Over several older selectors that is a conjunction of such clauses,
    expanded here into a disjunction of terms.  A clause whose pairs all sit in ``mine`` already
    excludes every node: nothing is left.  An older selector with a key ``mine`` requires at
    another value is disjoint: no clause.  Raises ValueError past MAX_HOLD_OFF_TERMS."""
    clauses = set()
    for q in older:
        if any(k in mine and mine[k] != v for k, v in q.items()):
            continue  # disjoint selections
        clause = tuple(sorted((k, v) for k, v in q.items() if mine.get(k) != v))
        if not clause:
            return [{"matchExpressions": [{"key": HELD_EVERYWHERE_KEY, "operator": "Exists"}]}]
        clauses.add(clause)
    if not clauses:
        return None
    kept: List[tuple] = []  # absorption: a clause implied by a shorter one adds nothing
    for c in sorted(clauses, key=lambda c: (len(c), c)):
        if not any(set(k) <= set(c) for k in kept):
            kept.append(c)
    terms: List[frozenset] = [frozenset()]
    for c in kept:
        terms = sorted({t | {lit} for t in terms for lit in c}, key=sorted)
        if len(terms) > MAX_HOLD_OFF_TERMS:
            raise ValueError(f"{len(kept)} overlapping older selectors expand to more than {MAX_HOLD_OFF_TERMS} "
                             "node-affinity terms")
    terms = [t for t in terms if not any(o < t for o in terms)]  # a term implied by a smaller one
    out = []
    for t in terms:
        by_key: Dict[str, List[str]] = {}
        for k, v in sorted(t):
            by_key.setdefault(k, []).append(v)
        out.append({"matchExpressions": [{"key": k, "operator": "NotIn", "values": vs} for k, vs in by_key.items()]})
    return out


def set_hold_off(pod: dict, terms: Optional[List[dict]]) -> None:
    """The agent Pod template's required node affinity: the hold-off terms, or none.  (The policy
    has no affinity field of its own, so the operator owns this one.)"""
    if terms:
        pod["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
            "nodeSelectorTerms": copy.deepcopy(terms)}}}
    else:
        pod.pop("affinity", None)


def held_off_error(ctype: str, nodes: List[str], more: bool, other: str) -> str:
    """status.errors entry for the nodes this policy is kept off because ``other`` (older, same
    configurationType) selects them too."""
    shown = ", ".join(nodes) + (" and more" if more else "")
    return (f"{shown}{CONFLICT_MARK}{other} ({ctype} too, created earlier): one agent per node and type "
            f"configures the NICs, so this policy's agents are held off these nodes while {other} selects them; "
            f"narrow a nodeSelector")
