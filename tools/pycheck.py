#!/usr/bin/env python3
"""Static checks of the repository's Python that need nothing beyond the standard library: the
part of the reference's golangci-lint set (reference .golangci.yml: unused, ineffassign,
goimports) that maps onto Python.

- an import never used in its module (re-exports: listed in ``__all__``, a package
  ``__init__``, or a line marked ``# noqa``);
- a name imported twice in one scope;
- a local variable assigned and never read in its function (ineffassign);
- ``except:`` without a class (it also catches KeyboardInterrupt and the asyncio cancellation).

    python tools/pycheck.py [paths...]     # default: the package, bench/, tests/, tools/, top-level .py
Exit status 1 when something is found; one ``path:line: message`` per finding.
"""

from __future__ import annotations

import ast
import sys
from pathlib import Path
from typing import Dict, Iterable, List, Set

ROOT = Path(__file__).resolve().parent.parent
DEFAULT = ["network_operator_amd", "bench", "tests", "tools", "bench.py", "__graft_entry__.py"]
SKIP_DIRS = {"__pycache__", "_lib", "_build", ".hypothesis"}


def _files(paths: Iterable[str]) -> List[Path]:
    out = []
    for p in paths:
        q = (ROOT / p) if not Path(p).is_absolute() else Path(p)
        if q.is_file() and q.suffix == ".py":
            out.append(q)
        elif q.is_dir():
            out += [f for f in sorted(q.rglob("*.py")) if not SKIP_DIRS & set(f.relative_to(q).parts)]
    return out


class _Names(ast.NodeVisitor):
    """Every name read anywhere in the module (attribute roots, string annotations too)."""

    def __init__(self) -> None:
        self.used: Set[str] = set()

    def visit_Name(self, node: ast.Name) -> None:
        if isinstance(node.ctx, (ast.Load, ast.Del)):
            self.used.add(node.id)

    def visit_Constant(self, node: ast.Constant) -> None:
        # "T.Foo" in a string annotation or a forward reference
        if isinstance(node.value, str) and node.value.replace(".", "").replace("_", "").isalnum():
            self.used.add(node.value.split(".")[0])


def _all(tree: ast.Module) -> Set[str]:
    for node in tree.body:
        if isinstance(node, ast.Assign) and any(isinstance(t, ast.Name) and t.id == "__all__" for t in node.targets):
            if isinstance(node.value, (ast.List, ast.Tuple)):
                return {e.value for e in node.value.elts if isinstance(e, ast.Constant)}
    return set()


def _unused_locals(fn: ast.AST) -> List[ast.Name]:
    """Names only ever stored in this function (not in nested ones, not global / nonlocal).  As
    pyflakes: names bound by tuple unpacking (``a, b = f()``, ``for k, v in ...``) are exempt."""
    stored: Dict[str, ast.Name] = {}
    loaded: Set[str] = set()
    declared: Set[str] = set()
    unpacked: Set[str] = set()

    def walk(node: ast.AST) -> None:
        for child in ast.iter_child_nodes(node):
            if isinstance(child, (ast.FunctionDef, ast.AsyncFunctionDef, ast.Lambda, ast.ClassDef)):
                # a nested scope may read the enclosing one's names: count its reads, not its stores
                for n in ast.walk(child):
                    if isinstance(n, ast.Name) and isinstance(n.ctx, ast.Load):
                        loaded.add(n.id)
                continue
            if isinstance(child, (ast.Global, ast.Nonlocal)):
                declared.update(child.names)
            if isinstance(child, (ast.Tuple, ast.List)) and isinstance(child.ctx, ast.Store):
                unpacked.update(n.id for n in ast.walk(child) if isinstance(n, ast.Name))
            if isinstance(child, ast.AugAssign) and isinstance(child.target, ast.Name):
                loaded.add(child.target.id)  # x += ... reads x (and extends a list argument in place)
            if isinstance(child, ast.Name):
                if isinstance(child.ctx, ast.Store):
                    stored.setdefault(child.id, child)
                else:
                    loaded.add(child.id)
            walk(child)
    walk(fn)
    return [n for k, n in stored.items()
            if k not in loaded and k not in declared and k not in unpacked and not k.startswith("_")]


def check_file(path: Path) -> List[str]:
    src = path.read_text()
    try:
        tree = ast.parse(src, str(path))
    except SyntaxError as e:
        return [f"{path}:{e.lineno}: syntax error: {e.msg}"]
    lines = src.splitlines()
    rel = path.relative_to(ROOT) if path.is_relative_to(ROOT) else path
    out: List[str] = []

    def noqa(lineno: int) -> bool:
        return "noqa" in lines[lineno - 1] if 0 < lineno <= len(lines) else False

    names = _Names()
    names.visit(tree)
    exported = _all(tree)
    package_init = path.name == "__init__.py"
    seen: Dict[str, int] = {}
    for node in tree.body:
        if not isinstance(node, (ast.Import, ast.ImportFrom)):
            continue
        if isinstance(node, ast.ImportFrom) and node.module == "__future__":
            continue
        for a in node.names:
            name = (a.asname or a.name).split(".")[0]
            submodule = isinstance(node, ast.Import) and not a.asname and "." in a.name  # import a; import a.b
            if name in seen and not noqa(node.lineno) and not submodule:
                out.append(f"{rel}:{node.lineno}: {name!r} imported again (first at line {seen[name]})")
            seen.setdefault(name, node.lineno)
            if name in names.used or name in exported or package_init or noqa(node.lineno) or name == "*":
                continue
            out.append(f"{rel}:{node.lineno}: {name!r} imported but unused")
    for node in ast.walk(tree):
        if isinstance(node, (ast.FunctionDef, ast.AsyncFunctionDef)):
            for n in _unused_locals(node):
                if not noqa(n.lineno):
                    out.append(f"{rel}:{n.lineno}: local {n.id!r} assigned but never used")
        if isinstance(node, ast.ExceptHandler) and node.type is None and not noqa(node.lineno):
            out.append(f"{rel}:{node.lineno}: bare 'except:' (catches KeyboardInterrupt and CancelledError too)")
    return out


def main(argv=None) -> int:
    paths = (argv if argv is not None else sys.argv[1:]) or DEFAULT
    found = []
    for f in _files(paths):
        found += check_file(f)
    for line in found:
        print(line)
    return 1 if found else 0


if __name__ == "__main__":
    sys.exit(main())
