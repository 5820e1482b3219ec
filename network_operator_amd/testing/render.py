"""Offline renderers for the deployment manifests (no helm / kustomize binaries here).

* ``helm_template(chart_dir, values, namespace)`` — a Go-template subset sufficient for the
  chart in ``charts/network-operator``: ``{{- / -}}`` trimming, ``.Values`` / ``.Release``,
  ``if / else / end``, ``$v := ...``, pipelines, and the Sprig functions the chart uses
  (list, has, not, or, and, eq, ne, lt, gt, int, fail, toYaml, nindent, indent, default, quote).
* ``kustomize_build(dir)`` — resources (files / kustomization dirs, recursive), ``namespace``,
  ``namePrefix`` with the name references the tree relies on, ``images``, strategic-merge
  patches and JSON6902 patches with a target.

Used by the packaging tests and ``make deployments``; both fail loudly on anything outside
the supported subset instead of guessing.
"""

from __future__ import annotations

import copy
import re
import shlex
from pathlib import Path
from typing import Any, Dict, List, Optional

import yaml


class RenderError(Exception):
    pass


# ---------------------------------------------------------------------------
# Helm (Go template subset)
# ---------------------------------------------------------------------------
# An action may hold a raw string (`...`), whose text may itself contain "{{" / "}}" (how a chart
# writes Prometheus' own {{ $labels.x }} templates).
_ACTION = re.compile(r"{{(-?)\s*((?:`[^`]*`|.)*?)\s*(-?)}}", re.S)


def _tokenize(src: str):
    out, pos = [], 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip()
        out.append(("text", text))
        out.append(("action", m.group(2), bool(m.group(3))))
        pos = m.end()
    out.append(("text", src[pos:]))
    # right-trim markers eat the whitespace of the following text
    for i, t in enumerate(out):
        if t[0] == "action" and t[2] and i + 1 < len(out) and out[i + 1][0] == "text":
            out[i + 1] = ("text", out[i + 1][1].lstrip())
    return out


def _parse(tokens, i=0, stop=("end",)):
    nodes = []
    while i < len(tokens):
        t = tokens[i]
        if t[0] == "text":
            nodes.append(("text", t[1]))
            i += 1
            continue
        act = t[1]
        word = act.split(None, 1)[0] if act else ""
        if word in ("end", "else") and word in stop:
            return nodes, i
        if act.startswith("/*"):
            i += 1
            continue
        if word == "if":
            body, i = _parse(tokens, i + 1, stop=("end", "else"))
            other = []
            if tokens[i][1].startswith("else"):
                other, i = _parse(tokens, i + 1, stop=("end",))
            nodes.append(("if", act[2:].strip(), body, other))
            i += 1
            continue
        nodes.append(("expr", act))
        i += 1
    return nodes, i


def _to_yaml(v) -> str:
    return yaml.safe_dump(v, sort_keys=True, default_flow_style=False).rstrip("\n")


def _fail(msg):
    raise RenderError(str(msg))


_FUNCS = {
    "list": lambda *a: list(a),
    "has": lambda needle, lst: needle in (lst or []),
    "not": lambda v: not v,
    "or": lambda *a: next((x for x in a if x), a[-1] if a else None),
    "and": lambda *a: next((x for x in a if not x), a[-1] if a else None),
    "eq": lambda a, b: a == b,
    "ne": lambda a, b: a != b,
    "lt": lambda a, b: a < b,
    "gt": lambda a, b: a > b,
    "int": lambda v: int(v),
    "fail": _fail,
    "toYaml": _to_yaml,
    "nindent": lambda n, s: "\n" + "\n".join(" " * int(n) + line if line else line for line in str(s).split("\n")),
    "indent": lambda n, s: "\n".join(" " * int(n) + line for line in str(s).split("\n")),
    "default": lambda d, v=None: v if v not in (None, "", [], {}, 0, False) else d,
    "quote": lambda v: '"' + str(v).replace('"', '\\"') + '"',
}


class _Ctx:
    def __init__(self, root: dict):
        self.root = root
        self.vars: Dict[str, Any] = {}

    def lookup(self, path: str):
        cur: Any = self.root
        for part in path.lstrip(".").split("."):
            if part == "":
                continue
            if not isinstance(cur, dict):
                return None
            cur = cur.get(part)
        return cur


def _split_pipeline(expr: str) -> List[str]:
    parts, depth, cur, q = [], 0, "", None
    for ch in expr:
        if q:
            cur += ch
            if ch == q:
                q = None
            continue
        if ch in "\"'`":
            q = ch
        elif ch == "(":
            depth += 1
        elif ch == ")":
            depth -= 1
        if ch == "|" and depth == 0:
            parts.append(cur.strip())
            cur = ""
        else:
            cur += ch
    parts.append(cur.strip())
    return parts


def _terms(cmd: str) -> List[str]:
    out, depth, cur, q = [], 0, "", None
    for ch in cmd:
        if q:
            cur += ch
            if ch == q:
                q = None
            continue
        if ch in "\"'`":
            q = ch
            cur += ch
            continue
        if ch == "(":
            depth += 1
        if ch == ")":
            depth -= 1
        if ch.isspace() and depth == 0:
            if cur:
                out.append(cur)
            cur = ""
        else:
            cur += ch
    if cur:
        out.append(cur)
    return out


def _eval_term(t: str, ctx: _Ctx):
    if t.startswith("(") and t.endswith(")"):
        return _eval_pipeline(t[1:-1], ctx)
    if t[0] == "`" and t.endswith("`") and len(t) >= 2:  # a raw string: its text as it is
        return t[1:-1]
    if t[0] in "\"'":
        return shlex.split(t)[0]
    if re.fullmatch(r"-?\d+", t):
        return int(t)
    if t in ("true", "false"):
        return t == "true"
    if t.startswith("$"):
        return ctx.vars[t]
    if t.startswith("."):
        return ctx.lookup(t)
    raise RenderError(f"unsupported term {t!r}")


def _eval_command(cmd: str, ctx: _Ctx, piped=None, has_piped=False):
    terms = _terms(cmd)
    if terms and terms[0] in _FUNCS:
        args = [_eval_term(t, ctx) for t in terms[1:]]
        if has_piped:
            args.append(piped)
        return _FUNCS[terms[0]](*args)
    if has_piped:
        raise RenderError(f"cannot pipe into {cmd!r}")
    if len(terms) != 1:
        raise RenderError(f"unsupported command {cmd!r}")
    return _eval_term(terms[0], ctx)


def _eval_pipeline(expr: str, ctx: _Ctx):
    cmds = _split_pipeline(expr)
    val = _eval_command(cmds[0], ctx)
    for c in cmds[1:]:
        val = _eval_command(c, ctx, val, True)
    return val


def _render_nodes(nodes, ctx: _Ctx) -> str:
    out = []
    for n in nodes:
        if n[0] == "text":
            out.append(n[1])
        elif n[0] == "if":
            out.append(_render_nodes(n[2] if _eval_pipeline(n[1], ctx) else n[3], ctx))
        else:
            expr = n[1]
            m = re.match(r"(\$\w+)\s*:=\s*(.*)", expr, re.S)
            if m:
                ctx.vars[m.group(1)] = _eval_pipeline(m.group(2), ctx)
                continue
            v = _eval_pipeline(expr, ctx)
            out.append("" if v is None else (str(v).lower() if isinstance(v, bool) else str(v)))
    return "".join(out)


def render_template(src: str, values: dict, namespace: str = "default", release: str = "release") -> str:
    nodes, _ = _parse(_tokenize(src))
    ctx = _Ctx({"Values": values, "Release": {"Namespace": namespace, "Name": release}})
    return _render_nodes(nodes, ctx)


def _deep_merge(base, over):
    if isinstance(base, dict) and isinstance(over, dict):
        out = dict(base)
        for k, v in over.items():
            out[k] = _deep_merge(base.get(k), v) if k in base else copy.deepcopy(v)
        return out
    return copy.deepcopy(over)


def helm_template(chart_dir, values: Optional[dict] = None, namespace: str = "default") -> List[dict]:
    chart_dir = Path(chart_dir)
    vals = _deep_merge(yaml.safe_load((chart_dir / "values.yaml").read_text()) or {}, values or {})
    docs: List[dict] = []
    for crd in sorted((chart_dir / "crds").glob("*.yaml")):
        docs += [d for d in yaml.safe_load_all(crd.read_text()) if d]
    for t in sorted((chart_dir / "templates").glob("*.yaml")):
        text = render_template(t.read_text(), vals, namespace)
        docs += [d for d in yaml.safe_load_all(text) if d]
    return docs


# ---------------------------------------------------------------------------
# kustomize (subset)
# ---------------------------------------------------------------------------
CLUSTER_SCOPED = {"Namespace", "ClusterRole", "ClusterRoleBinding", "CustomResourceDefinition",
                  "MutatingWebhookConfiguration", "ValidatingWebhookConfiguration", "NetworkClusterPolicy",
                  "NodeFeatureRule"}


def _sm_merge(base, patch):
    """Strategic merge for the shapes used here: dicts merge, named lists merge by name."""
    if isinstance(base, dict) and isinstance(patch, dict):
        out = dict(base)
        for k, v in patch.items():
            out[k] = _sm_merge(base[k], v) if k in base else copy.deepcopy(v)
        return out
    if isinstance(base, list) and isinstance(patch, list) and all(isinstance(x, dict) and "name" in x for x in base + patch):
        out = [copy.deepcopy(x) for x in base]
        for p in patch:
            for i, b in enumerate(out):
                if b["name"] == p["name"]:
                    out[i] = _sm_merge(b, p)
                    break
            else:
                out.append(copy.deepcopy(p))
        return out
    if isinstance(base, list) and isinstance(patch, list):
        return base + [x for x in patch if x not in base]
    return copy.deepcopy(patch)


def _load_dir(d: Path) -> List[dict]:
    k = yaml.safe_load((d / "kustomization.yaml").read_text()) or {}
    docs: List[dict] = []
    for r in k.get("resources", []) or []:
        p = (d / r).resolve()
        docs += _load_dir(p) if p.is_dir() else [x for x in yaml.safe_load_all(p.read_text()) if x]
    for img in k.get("images", []) or []:
        for doc in docs:
            for c in (doc.get("spec", {}).get("template", {}).get("spec", {}).get("containers", []) or []):
                name = c.get("image", "").split(":")[0]
                if name == img["name"]:
                    c["image"] = f"{img.get('newName', name)}:{img.get('newTag', 'latest')}"
    for p in k.get("patches", []) or []:
        patch = yaml.safe_load((d / p["path"]).read_text())
        if isinstance(patch, list):  # JSON6902
            from .fakeapi import json_patch_apply

            tgt = p.get("target") or {}
            for i, doc in enumerate(docs):
                if all(doc.get(f) == tgt[f] or doc.get("metadata", {}).get(f) == tgt[f] for f in tgt):
                    docs[i] = json_patch_apply(doc, patch)
        else:
            hit = False
            for i, doc in enumerate(docs):
                if doc.get("kind") == patch.get("kind") and doc["metadata"]["name"] == patch["metadata"]["name"]:
                    docs[i] = _sm_merge(doc, patch)
                    hit = True
            if not hit:
                raise RenderError(f"patch {p['path']} matches no resource")
    ns, prefix = k.get("namespace"), k.get("namePrefix", "")
    if ns or prefix:
        names = {(doc["kind"], doc["metadata"]["name"]) for doc in docs}
        for doc in docs:
            md = doc["metadata"]
            kind = doc["kind"]
            if kind == "Namespace":
                if ns:
                    md["name"] = ns
                continue
            if kind != "CustomResourceDefinition":
                md["name"] = prefix + md["name"]
            if ns and kind not in CLUSTER_SCOPED:
                md["namespace"] = ns
            spec = doc.get("spec", {}) or {}
            pod = spec.get("template", {}).get("spec", {}) if isinstance(spec, dict) else {}
            if pod.get("serviceAccountName") and ("ServiceAccount", pod["serviceAccountName"]) in names:
                pod["serviceAccountName"] = prefix + pod["serviceAccountName"]
            if "roleRef" in doc and (doc["roleRef"]["kind"], doc["roleRef"]["name"]) in names:
                doc["roleRef"]["name"] = prefix + doc["roleRef"]["name"]
            for s in doc.get("subjects", []) or []:
                if s.get("kind") == "ServiceAccount":
                    if ("ServiceAccount", s["name"]) in names:
                        s["name"] = prefix + s["name"]
                    if ns:
                        s["namespace"] = ns
            for wh in doc.get("webhooks", []) or []:
                svc = (wh.get("clientConfig") or {}).get("service")
                if svc:
                    if ("Service", svc["name"]) in names:
                        svc["name"] = prefix + svc["name"]
                    if ns:
                        svc["namespace"] = ns
    return docs


def kustomize_build(d) -> List[dict]:
    return _load_dir(Path(d).resolve())


def dump_all(docs: List[dict]) -> str:
    return "---\n".join(yaml.safe_dump(d, sort_keys=False) for d in docs)


def discovery_for(policy_file, namespace: str = "amd-network-operator") -> List[dict]:
    """The agent DaemonSet (+ ServiceAccount) the reconciler would create for a policy file —
    what `make deployments` writes to deployments/discovery*.yaml for the Trivy config scan
    (reference trivy.yaml scans its discovery.yaml the same way)."""
    from network_operator_amd import discovery
    from network_operator_amd.api.v1alpha1 import types as T
    from network_operator_amd.operator import reconciler as R

    p = T.NetworkClusterPolicy.from_dict(yaml.safe_load(Path(policy_file).read_text()))
    ds = discovery.discovery_daemonset()
    R.update_daemonset_for(ds, p, namespace)
    sa = discovery.linkdiscovery_service_account()
    sa.setdefault("metadata", {})["namespace"] = namespace
    return [sa, ds]


if __name__ == "__main__":
    import argparse
    import sys

    ap = argparse.ArgumentParser(description="offline renderers")
    ap.add_argument("--discovery", metavar="POLICY_YAML", help="agent DaemonSet for a NetworkClusterPolicy")
    a = ap.parse_args()
    if a.discovery:
        sys.stdout.write(dump_all(discovery_for(a.discovery)))
