"""The documentation's evidence pointers resolve: every repository path a document names in
backticks exists, and every test it cites (`test_x.py::name`, `test_agent.cpp::name`, and the
`::name` shorthand that follows one) is defined in that file.  Paths that follow the word
"reference" are the upstream project's, not this repository's."""

import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
DOCS = sorted(p for p in (ROOT / "docs").glob("*.md") if p.name != "ROUND3.md") + [
    ROOT / "README.md", ROOT / "profiles" / "README.md", ROOT / "charts" / "network-operator" / "README.md"]
PREFIXES = ("profiles", "tests", "native", "tools", "network_operator_amd", "bench", "docs", "charts", "config")


def _sources():
    out = {}
    for p in list((ROOT / "tests").glob("*.py")) + list((ROOT / "native" / "tests").glob("*.cpp")):
        out[p.name] = p.read_text()
    return out


@pytest.mark.parametrize("doc", DOCS, ids=lambda p: str(p.relative_to(ROOT)))
def test_paths_named_in_the_docs_exist(doc):
    text = doc.read_text()
    missing = []
    for m in re.finditer(r"`((?:%s)/[A-Za-z0-9_./-]+)`" % "|".join(PREFIXES), text):
        path = m.group(1).rstrip(".")
        if "*" in path or "<" in path or "reference" in text[max(0, m.start() - 12):m.start()]:
            continue
        if not (ROOT / path).exists():
            missing.append(path)
    assert not missing, missing


@pytest.mark.parametrize("doc", DOCS, ids=lambda p: str(p.relative_to(ROOT)))
def test_tests_cited_in_the_docs_exist(doc):
    src = _sources()
    bad, cur = [], None
    for span in re.findall(r"`([^`]+)`", doc.read_text()):
        m = re.match(r"(?:tests/|native/tests/)?(test_[a-z_0-9]+\.(?:py|cpp))::([A-Za-z_0-9]+)", span)
        if m:
            cur, name = m.group(1), m.group(2)
        elif span.startswith("::") and cur:
            name = re.match(r"::([A-Za-z_0-9]+)", span).group(1)
        else:
            cur = None
            continue
        name = name.rstrip("_")  # `test_x.py::test_prefix_*` names a family
        if cur not in src or name not in src[cur]:
            bad.append(f"{cur}::{name}")
    assert not bad, bad


def test_every_agent_flag_is_in_the_user_guide():
    """`discover --help` against USER_GUIDE.md §4: a new agent flag needs its row (or a mention)."""
    import subprocess

    from network_operator_amd.utils.paths import native_bin

    out = subprocess.run([str(native_bin("discover")), "--help"], capture_output=True, text=True, timeout=30)
    flags = sorted(set(re.findall(r"^\s+(--[a-z0-9_-]+)", out.stdout + out.stderr, re.M)))
    assert len(flags) > 50, out.stdout[:500]
    guide = (ROOT / "docs" / "USER_GUIDE.md").read_text()
    missing = [f for f in flags if f != "--help" and not re.search(r"`" + re.escape(f) + r"(`|[ =,])", guide)]
    assert not missing, missing


def test_every_operator_flag_is_in_the_user_guide():
    """The manager's argparse flags against USER_GUIDE.md's operator flag table."""
    from network_operator_amd.operator import manager

    flags = sorted({o for a in manager.build_parser()._actions for o in a.option_strings
                    if o.startswith("--") and o != "--help"})
    assert len(flags) > 15
    guide = (ROOT / "docs" / "USER_GUIDE.md").read_text()
    missing = [f for f in flags if not re.search(r"`" + re.escape(f) + r"(`|[ =,])", guide)]
    assert not missing, missing


def test_every_policy_field_is_in_the_user_guide():
    """Every field of the NetworkClusterPolicy spec (amdScaleOut, hostNic, validation included)
    is named in USER_GUIDE.md."""
    from network_operator_amd.api.v1alpha1 import types as T

    fields = set(T.AmdScaleOutSpec._FIELDS)
    for cls in (T.HostNicSpec, T.NetworkClusterPolicySpec, T.ValidationSpec):
        fields |= {f for f in cls.__dataclass_fields__ if f != "extra"}
    guide = (ROOT / "docs" / "USER_GUIDE.md").read_text()
    missing = sorted(f for f in fields if not re.search(r"\b" + f + r"\b", guide))
    assert not missing, missing
