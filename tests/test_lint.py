"""``make vet``'s Python half on every run: tools/pycheck.py (unused imports, duplicate imports,
locals assigned and never read, bare ``except:``) finds nothing in the repository, and finds each
of those in a file that has them."""

import importlib.util
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def _pycheck():
    spec = importlib.util.spec_from_file_location("pycheck", ROOT / "tools" / "pycheck.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_repository_python_is_clean():
    pc = _pycheck()
    found = [line for f in pc._files(pc.DEFAULT) for line in pc.check_file(f)]
    assert found == []


def test_checker_finds_what_it_is_for(tmp_path):
    pc = _pycheck()
    f = tmp_path / "m.py"
    f.write_text("import os\nimport sys\nimport sys\nimport json  # noqa: F401\nimport xml.dom\nimport xml.sax\n"
                 "from typing import List\n\n\ndef g(errors):\n    errors += ['x']\n    a, b = 1, 2\n"
                 "    unused = 3\n    try:\n        pass\n    except:\n        pass\n    return sys.argv, xml\n")
    found = [line.split(": ", 1)[1] for line in pc.check_file(f)]
    assert len(found) == 5, found
    assert "'os' imported but unused" in found
    assert "'sys' imported again (first at line 2)" in found
    assert "'List' imported but unused" in found
    assert "local 'unused' assigned but never used" in found
    assert any(x.startswith("bare 'except:'") for x in found)
    assert not any("json" in x or "xml" in x or "'errors'" in x or "'a'" in x for x in found), found
