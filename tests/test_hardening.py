"""Binary hardening of the agent's executables (tools/check_hardening.py), the counterpart of the
reference's checksec gate (reference build/Dockerfile.linkdiscovery:36-41,
build/Dockerfile.operator:36-41), and the images' use of it."""

import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
import check_hardening as H  # noqa: E402

BIN = ROOT / "network_operator_amd" / "_lib" / "bin"


@pytest.mark.parametrize("name", ["discover", "netop-topo", "netop-lldp-tx"])
def test_agent_binaries_are_hardened(name):
    path = BIN / name
    if not path.exists():
        pytest.fail(f"{path} not built (run __graft_entry__.build())")
    r = H.inspect(str(path))
    assert H.failures(r) == [], r
    assert "__memcpy_chk" in r["fortify"] or "__snprintf_chk" in r["fortify"]


def test_gate_rejects_an_unhardened_binary(tmp_path):
    cc = shutil.which("gcc") or shutil.which("cc")
    if not cc:
        pytest.skip("no C compiler")
    src = tmp_path / "weak.c"
    src.write_text("#include <stdio.h>\n#include <string.h>\nint main(int c, char** v) { char b[8]; "
                   "strcpy(b, v[0]); printf(\"%s\\n\", b); return 0; }\n")
    weak = tmp_path / "weak"
    subprocess.run([cc, "-O2", "-U_FORTIFY_SOURCE", "-fno-stack-protector", "-no-pie", "-Wl,-z,norelro",
                    "-Wl,-z,lazy", "-Wl,-z,execstack", str(src), "-o", str(weak)], check=True, capture_output=True)
    r = H.inspect(str(weak))
    assert set(H.failures(r)) == {"pie", "relro", "bind_now", "nx_stack", "stack_protector", "fortify"}, r
    assert H.main([str(weak)]) == 1
    strong = tmp_path / "strong"
    subprocess.run([cc, "-O2", "-D_FORTIFY_SOURCE=2", "-fstack-protector-strong", "-fPIE", "-pie", "-Wl,-z,relro,-z,now",
                    str(src), "-o", str(strong)], check=True, capture_output=True)
    assert H.failures(H.inspect(str(strong))) == []
    assert H.main([str(strong)]) == 0
    (tmp_path / "text").write_text("not elf")
    assert H.main([str(tmp_path / "text")]) == 1


def test_images_gate_on_hardening_and_run_without_pip():
    agent = (ROOT / "build" / "Dockerfile.linkdiscovery").read_text()
    assert "check_hardening.py /out/bin/discover /out/bin/netop-topo" in agent
    op = (ROOT / "build" / "Dockerfile.operator").read_text()
    final = op.rsplit("FROM ", 1)[1]  # the runtime stage
    assert "distroless" in final.splitlines()[0] and "nonroot" in final.splitlines()[0]
    assert "pip" not in final and "USER 65532" in final


def test_operator_image_file_set_is_self_contained(tmp_path):
    """The operator image copies only some packages (build/Dockerfile.operator).  The manager
    must import and parse its flags from exactly that file set, which is what the image's
    build-time import check does, here without docker."""
    import re

    df = (ROOT / "build" / "Dockerfile.operator").read_text()
    copies = re.findall(r"^COPY (network_operator_amd\S*) (\S+)$", df, re.M)
    assert copies, df
    app = tmp_path / "app"
    for src, dst in copies:
        s, d = ROOT / src, app / dst
        if s.is_dir():
            shutil.copytree(s, d, ignore=shutil.ignore_patterns("__pycache__", "*.so"))
        else:
            d.parent.mkdir(parents=True, exist_ok=True)
            shutil.copy(s, d)
    r = subprocess.run([sys.executable, "-c", "import network_operator_amd.operator.manager as m; "
                        "m.build_parser().parse_args(['--policies-file=/x', '--leader-elect'])"],
                       cwd=str(tmp_path), env={"PYTHONPATH": str(app), "PATH": "/usr/bin:/bin"},
                       capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    r = subprocess.run([sys.executable, "-m", "network_operator_amd.operator", "--help"], cwd=str(tmp_path),
                       env={"PYTHONPATH": str(app), "PATH": "/usr/bin:/bin"}, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "--policies-file" in r.stdout, r.stderr[-2000:]
