"""The agent binary itself on a real MI355X node (``-m gpu``: runs on the GPU box).

The box gives no NET_ADMIN / NET_RAW and no user namespaces, so the agent runs with
``--dry-run``: the real discovery, xGMI and GPUDirect checks and topology writer against the
box's own /sys, with no link, address or label change.  The pieces that need privileges run in
the netns harness (tests/test_netns_integration.py, tests/test_e2e.py).
"""

import json
import os
import re
import subprocess
from pathlib import Path

import pytest

from network_operator_amd.agent import native
from network_operator_amd.utils.paths import native_bin

pytestmark = pytest.mark.gpu


def test_agent_dry_run_on_this_node(tmp_path):
    topo, status = tmp_path / "rccl-topo.xml", tmp_path / "status.json"
    r = subprocess.run([str(native_bin("discover")), "--dry-run", "--mode=L3", "--mtu=9000", "--xgmi-expect=0",
                        f"--rccl-topo={topo}", f"--status-file={status}", "-v=2"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr[-3000:]
    st = json.loads(status.read_text())
    root = os.environ.get("SYSFS_ROOT", "/sys/")
    want = native().discover(root, "affine")
    index = {g["bdf"]: g["index"] for g in want["gpus"]}
    pairs = re.findall(r"GPU (\d+) \((\S+)\) <-> NIC (\S+) \((\S+), ", r.stderr)
    assert [(g, b, n) for g, b, n, _ in pairs] == [(str(index[p["gpu"]]), p["gpu"], p["nic"]) for p in want["pairs"]]
    x = native().read_xgmi(root)
    assert st["xgmi_pairs"] == f"{x['pairs_connected']}/{x['pairs_expected']}"
    assert st["dry_run"] == "true" and st["ready"] is False
    xml = topo.read_text()
    assert xml.startswith('<system version="2">') and xml.count("<net ") == len(want["pairs"])
    out = Path(os.environ.get("GRAFT_REPO_ROOT", ".")) / "gpurun_out"
    if out.is_dir():  # evidence for profiles/ when run through gpurun
        (out / "agent_dry_run_box.json").write_text(json.dumps({"status": st, "pairs": pairs,
                                                                "log_tail": r.stderr[-4000:]}, indent=1))
