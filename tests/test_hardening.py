"""Binary hardening of the agent's executables (tools/check_hardening.py), the counterpart of the
reference's checksec gate (reference build/Dockerfile.linkdiscovery:36-41,
build/Dockerfile.operator:36-41), and the images' use of it."""

import json
import os
import shutil
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT / "tools"))
import check_hardening as H  # noqa: E402

from network_operator_amd.utils.paths import native_bin  # noqa: E402

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
    # The chart's pre-delete hook runs the same image with another module.
    r = subprocess.run([sys.executable, "-m", "network_operator_amd.operator.predelete", "--help"], cwd=str(tmp_path),
                       env={"PYTHONPATH": str(app), "PATH": "/usr/bin:/bin"}, capture_output=True, text=True,
                       timeout=120)
    assert r.returncode == 0 and "--owner" in r.stdout, r.stderr[-2000:]


# What the agent image's runtime base (ubuntu:22.04) ships as shared libraries without any
# apt install: libc6, libgcc-s1 and libstdc++6 are all in the minimal image (apt needs them).
UBUNTU_BASE_LIBS = {"libc.so.6", "libm.so.6", "libstdc++.so.6", "libgcc_s.so.1", "ld-linux-x86-64.so.2",
                    "libpthread.so.0", "libdl.so.2", "librt.so.1"}


def _ldd(path):
    """soname -> resolved path of every shared library `path` loads (ldd, transitive)."""
    out = subprocess.run(["ldd", str(path)], capture_output=True, text=True, check=True).stdout
    libs = {}
    for line in out.splitlines():
        parts = line.split()
        if "=>" in parts and len(parts) >= 3 and parts[2].startswith("/"):
            libs[parts[0]] = parts[2]
        elif parts and parts[0].startswith("/"):  # the interpreter
            libs[os.path.basename(parts[0])] = parts[0]
    return libs


@pytest.mark.skipif(not hasattr(os, "geteuid") or os.geteuid() != 0, reason="chroot needs root")
def test_agent_image_runtime_stage_runs_in_its_own_rootfs(tmp_path):
    """The agent image, without docker: a root filesystem holding exactly what the runtime stage
    of build/Dockerfile.linkdiscovery copies, plus only the libraries its ubuntu:22.04 base ships.
    The ENTRYPOINT must start there (--version) and do a real dry run (netlink link dump, sysfs
    discovery, topology and status files) inside the chroot."""
    import re

    df = (ROOT / "build" / "Dockerfile.linkdiscovery").read_text()
    final = df.rsplit("\nFROM ", 1)[1]
    assert final.splitlines()[0].strip() == "ubuntu:22.04"
    (copy,) = re.findall(r"^COPY --from=builder (.+)$", final, re.M)
    *srcs, dest = copy.split()
    entry = json.loads(re.search(r"^ENTRYPOINT (\[.*\])$", final, re.M).group(1))
    root = tmp_path / "rootfs"
    for s in srcs:
        assert s.startswith("/out/bin/"), s
        binary = native_bin(os.path.basename(s))
        d = root / dest.lstrip("/")
        d.mkdir(parents=True, exist_ok=True)
        shutil.copy2(binary, d / binary.name)
        libs = _ldd(binary)
        assert set(libs) <= UBUNTU_BASE_LIBS, f"{binary.name} needs libraries the base image lacks: " \
                                              f"{sorted(set(libs) - UBUNTU_BASE_LIBS)}"
        for lib in libs.values():
            t = root / lib.lstrip("/")
            t.parent.mkdir(parents=True, exist_ok=True)
            shutil.copy2(os.path.realpath(lib), t)
    for lib64 in ("lib64",):  # the interpreter path the ELF names
        if (Path("/") / lib64).is_symlink() and not (root / lib64).exists():
            (root / lib64).symlink_to(os.readlink(Path("/") / lib64))
    for d in ("tmp", "sys-empty", "var/lib/amd-network"):
        (root / d).mkdir(parents=True, exist_ok=True)
    env = {"PATH": "/usr/local/bin:/usr/bin:/bin", "SYSFS_ROOT": "/sys-empty/"}

    def enter():  # in the child, before exec: the image's filesystem is all it can see
        os.chroot(str(root))
        os.chdir("/")

    r = subprocess.run(entry + ["--version"], capture_output=True, text=True, timeout=30, env=env, preexec_fn=enter)
    assert r.returncode == 0 and "0.1.0" in r.stdout, r.stderr
    r = subprocess.run([*entry, "--dry-run", "--interfaces=lo", "--mode=L3", "--xgmi-expect=0",
                        "--status-file=/var/lib/amd-network/status.json", "--rccl-topo=/var/lib/amd-network/topo.xml"],
                       capture_output=True, text=True, timeout=60, env=env, preexec_fn=enter)
    assert r.returncode == 0, r.stderr[-2000:]
    st = json.loads((root / "var/lib/amd-network/status.json").read_text())
    assert st["dry_run"] == "true" and [i["name"] for i in st["interfaces"]] == ["lo"]
    assert (root / "var/lib/amd-network/topo.xml").read_text().startswith("<system")


@pytest.mark.skipif(not hasattr(os, "geteuid") or os.geteuid() != 0, reason="chroot needs root")
def test_validation_image_file_set_runs_in_its_own_rootfs(tmp_path):
    """The validation image (build/Dockerfile.validation), without docker: a root filesystem
    holding the Python interpreter and its standard library only (the ROCm base image has no
    PyTorch, PyYAML or pip packages) plus exactly what the runtime stage copies.  The
    ENTRYPOINT must answer --help there, and check 1's topology discovery must run on a fake
    node through the in-tree native module."""
    import re

    from network_operator_amd.testing import fakesysfs

    df = (ROOT / "build" / "Dockerfile.validation").read_text()
    final = df.rsplit("\nFROM ", 1)[1]
    copies = re.findall(r"^COPY --from=builder /src/(\S+) (\S+)$", final, re.M)
    assert copies == [("network_operator_amd", "/opt/netop/network_operator_amd")], copies
    pypath = re.search(r"^ENV PYTHONPATH=(\S+)$", final, re.M).group(1)
    entry = json.loads(re.search(r"^ENTRYPOINT (\[.*\])$", final, re.M).group(1))
    assert entry[:3] == ["python3", "-m", "network_operator_amd.validate"]
    root = tmp_path / "rootfs"
    for src, dst in copies:
        shutil.copytree(ROOT / src, root / dst.lstrip("/"), symlinks=True,
                        ignore=shutil.ignore_patterns("__pycache__"))
    # the interpreter, its stdlib (no site / dist-packages) and the libraries they load
    py = os.path.realpath(shutil.which("python3"))
    stdlib = Path(os.path.dirname(os.__file__))
    shutil.copytree(stdlib, root / str(stdlib).lstrip("/"), symlinks=True,
                    ignore=shutil.ignore_patterns("__pycache__", "dist-packages", "site-packages", "test", "idlelib",
                                                  "tkinter", "turtledemo"))
    (root / "usr/bin").mkdir(parents=True, exist_ok=True)
    shutil.copy2(py, root / "usr/bin/python3")
    elfs = [Path(py)] + sorted((stdlib / "lib-dynload").glob("*.so")) + [
        p for p in (root / "opt/netop/network_operator_amd/_lib").glob("*.so")]
    for e in elfs:
        for lib in _ldd(e).values():
            t = root / lib.lstrip("/")
            if not t.exists():
                t.parent.mkdir(parents=True, exist_ok=True)
                shutil.copy2(os.path.realpath(lib), t)
    if Path("/lib64").is_symlink() and not (root / "lib64").exists():
        (root / "lib64").symlink_to(os.readlink("/lib64"))
    fakesysfs.build_mi355x_node(root / "sys-fake")
    (root / "tmp").mkdir(exist_ok=True)
    env = {"PATH": "/usr/bin:/bin", "PYTHONPATH": pypath, "PYTHONNOUSERSITE": "1"}

    def enter():
        os.chroot(str(root))
        os.chdir("/")

    r = subprocess.run([*entry, "--help"], capture_output=True, text=True, timeout=60, env=env, preexec_fn=enter)
    assert r.returncode == 0 and "--artifact-dir" in r.stdout, r.stderr[-2000:]
    code = ("import sys; from network_operator_amd.models.topology import NodeTopology; "
            "t = NodeTopology.discover('/sys-fake/'); print(len(t.gpus), len(t.pairs), t.xgmi.pairs_connected); "
            "assert 'torch' not in sys.modules and 'yaml' not in sys.modules")
    r = subprocess.run(["python3", "-c", code], capture_output=True, text=True, timeout=60, env=env, preexec_fn=enter)
    assert r.returncode == 0 and r.stdout.split() == ["8", "8", "28"], (r.stdout, r.stderr[-2000:])
