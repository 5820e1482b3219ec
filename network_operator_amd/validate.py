"""Post-configuration fabric validation of one MI355X node (``python -m network_operator_amd.validate``).

The agent configures the node and checks what it can see without touching a GPU: the KFD
xGMI topology, GPUDirect RDMA support and LLDP peers.  This is the GPU-side counterpart.  It
runs where the GPUs are (a Job with ``amd.com/gpu: 8``, see ``config/validation/``) and
answers one question: do the links actually carry collectives at the expected speed?  It runs
these checks:

1. **Topology.**  KFD: every GPU pair is xGMI-linked; every GPU has its own scale-out NIC
   within one PCIe switch (the agent's pairing, ``models.topology.NodeTopology``); and, when
   the agent wrote one, its ``NCCL_TOPO_FILE`` places each pair under the same switch the live
   PCIe tree does.
2. **xGMI probe** (``netop-xgmi-probe``).  Per-link pull bandwidth, all-peers pull and push
   aggregates, all byte-exact.
3. **RCCL** (``netop-rccl-bench``) with the agent's artifacts applied: ``<artifact-dir>/rccl.env``
   (its ``NCCL_TOPO_FILE`` included) and ``rccl-tuned.env`` are sourced, as a job on the node
   sources them.  An all-reduce size sweep, every result checked exactly; with n > 1 the
   large-message busbw must reach ``--min-busbw``.  RCCL's topology dump of that run must show
   >= n-1 xGMI links per GPU and place every GPU / NIC where the file does
   (``parallel/fabric_artifacts.py``).
4. **Counters** (amd-smi).  Every up xGMI link moved data during the RCCL run.  This is the
   "RCCL sees every link" check from BASELINE.json.
5. **Direct xGMI all-reduce** (``parallel/xgmi_comm.py``).  The one-process-per-GPU
   all-reduce over HIP IPC buffers that jobs can use, every size checked exactly (after the
   counter window, so check 4 still sees RCCL traffic only).  Without PyTorch (the validation
   image) the native single-process harness runs the same algorithm instead.
6. **Optionally, RCCL tuning** (``--tune-rccl``, n > 1).  The 1 GiB all-reduce under the
   knob variants of ``parallel/rccl_bench.ENV_PROBES``, each in a fresh process.  A variant
   that beats RCCL's defaults by at least 3 % is written to ``<artifact-dir>/rccl-tuned.env``,
   for jobs to source after the agent's ``rccl.env``.  ``bench.py`` does the same before its
   timed run.
7. **Optionally, the label.**  If everything passed, the NFD label
   ``amd.feature.node.kubernetes.io/gpu-fabric-validated=true`` is written, along with the
   measured busbw.

The reference has no equivalent; its README only says the fabric is validated "with the
vendor's tests".  Prints one JSON report and exits 0 only if every check passed.
"""

from __future__ import annotations

import argparse
import json
import os
import shutil
import subprocess
import sys
import tempfile
import time
from pathlib import Path
from typing import List, Optional

from .utils.paths import native_bin

LABEL = "amd.feature.node.kubernetes.io/gpu-fabric-validated"
LABEL_FILE = "gpu-fabric-validation.txt"


def _check(name: str, ok: bool, **detail) -> dict:
    return {"check": name, "ok": bool(ok), **detail}


def _have_torch() -> bool:
    import importlib.util

    return importlib.util.find_spec("torch") is not None


def direct_all_reduce_check(gpus: int, max_bytes: int, timeout: float) -> dict:
    """Check 5.  With PyTorch present it runs the way jobs run it (``parallel/xgmi_comm.py``: one
    process per GPU, torch.distributed rendezvous, HIP IPC buffers).  The validation image is a
    plain ROCm image without PyTorch; there the same two-shot algorithm runs from the native
    single-process harness (``netop-xgmi-allreduce``: every GPU in one process, peer access),
    still checked exactly, instead of failing the node for a missing Python package."""
    try:
        if _have_torch():
            from .parallel import xgmi_comm

            d = xgmi_comm.run(gpus, nbytes=max_bytes, min_bytes=1 << 20, iters=5, warmup=2, timeout=timeout)
            return _check("xgmi_direct_all_reduce", d["wrong"] == 0, runner="xgmi_comm (one process per GPU)",
                          peak_busbw_GBps=d["peak_busbw_GBps"], wrong=d["wrong"],
                          sizes=[{k: r[k] for k in ("algo", "bytes", "time_us", "busbw_GBps")} for r in d["rows"]])
        from .parallel import xgmi_allreduce as XA

        rows = XA.run(ranks=gpus, min_bytes=min(1 << 20, max_bytes), max_bytes=max_bytes, factor=32, iters=5, warmup=2,
                      timeout=timeout)
        if not rows:
            return _check("xgmi_direct_all_reduce", False, runner="netop-xgmi-allreduce", error="no result rows")
        wrong = sum(int(r["wrong"]) for r in rows)
        return _check("xgmi_direct_all_reduce", wrong == 0, runner="netop-xgmi-allreduce (one process, no PyTorch)",
                      peak_busbw_GBps=max(float(r["busbw_GBps"]) for r in rows), wrong=wrong,
                      sizes=[{"algo": r["mode"], "bytes": r["bytes"], "time_us": r["time_us"],
                              "busbw_GBps": r["busbw_GBps"]} for r in rows])
    except Exception as e:
        return _check("xgmi_direct_all_reduce", False, error=str(e)[-500:])


def topo_file_agrees(xml_text: str, topo) -> dict:
    """Whether an RCCL topology file (the agent's rccl-topo.xml) nests each GPU and its paired
    NIC under the same outermost switch as the live PCIe tree, and lists every GPU."""
    import xml.etree.ElementTree as ET

    root = ET.fromstring(xml_text)
    top_of: dict = {}
    for cpu in root.findall("cpu"):
        for top in cpu.findall("pci"):
            for p in top.iter("pci"):
                top_of[p.get("busid")] = top.get("busid")
            for net in top.iter("net"):
                top_of["net:" + net.get("name", "")] = top.get("busid")
    missing = [g for g in topo.gpus if g not in top_of]
    split = []
    for p in topo.pairs:
        name = topo.rdma.get(p.nic) or p.nic
        if top_of.get(p.gpu_bdf) != top_of.get("net:" + name):
            split.append((p.gpu_bdf, name))
    return {"ok": not missing and not split, "gpus_missing": missing, "pairs_split": split}


def rccl_links_check(gpus: int, dump: str, art_env: dict, scratch: str, timeout: float) -> dict:
    """RCCL sees >= n-1 xGMI links per GPU under the agent's NCCL_TOPO_FILE, and its dump places
    every GPU (and NIC) where the file does.  Only when that fails is RCCL initialised once more
    without the artifacts, to tell "the file costs links" from "RCCL does not record them"."""
    from .parallel import fabric_artifacts as FA
    from .parallel import rccl_bench

    view = FA.read_view(dump, art_env.get("NCCL_TOPO_FILE"))
    verdict = FA.links_verdict(gpus, view, None)
    base = None
    if verdict["status"] == "failed" and gpus > 1:
        bdump = os.path.join(scratch, "rccl-topo-dump-defaults.xml")
        env = {k: v for k, v in os.environ.items() if k not in art_env}
        env["NCCL_TOPO_DUMP_FILE"] = bdump
        try:
            subprocess.run(rccl_bench.command(op="all_reduce", gpus=gpus, min_bytes=1 << 20, max_bytes=1 << 20,
                                              iters=2, warmup=1, check=False),
                           env=env, capture_output=True, text=True, timeout=timeout)
            base = FA.read_view(bdump)
        except Exception as e:
            base = {"error": str(e)[-300:]}
        verdict = FA.links_verdict(gpus, view, base)
    ok = verdict["status"] != "failed" and bool(view) and "error" not in view \
        and view.get("gpu_ancestry_equal", True) and view.get("nic_ancestry_equal") is not False
    return _check("rccl_xgmi_links", ok, **verdict,
                  rccl_dump={k: view.get(k) for k in ("gpus", "xgmi_links_per_gpu", "gpu_ancestry_equal",
                                                      "nic_ancestry_equal", "gpu_ancestry_diff", "nic_ancestry_diff",
                                                      "error")} if view else None,
                  rccl_dump_defaults={k: base.get(k) for k in ("gpus", "min_xgmi_links", "xgmi_elements", "error")}
                  if base else None)


def rail_pcie_check(topo, sysfs_root: str) -> Optional[dict]:
    """Each rail's PCIe links as trained, judged as the agent's --require-full-pcie judges them:
    the NIC at the speed and width both ends support, the GPU at full width (its speed drops while
    idle).  A rail at x8 or Gen4 moves RDMA at half rate whatever the busbw test saw.  None on a
    node without rails."""
    from .agent import native

    n = native()
    bdf = {nic["ifname"]: nic["bdf"] for nic in n.discover(sysfs_root)["nics"]}
    rails, slow = {}, []
    for pr in topo.pairs:
        nl, gl = n.read_pcie_link(sysfs_root, bdf.get(pr.nic, "")), n.read_pcie_link(sysfs_root, pr.gpu_bdf)
        rails[pr.nic] = {"nic": nl["str"], "gpu": gl["str"]}
        if nl["degraded"] or (gl["known"] and gl["width"] < gl["max_width"]):
            slow.append(pr.nic)
    return _check("rail_pcie_links", not slow, degraded=slow, links=rails) if rails else None


def run(gpus: int, min_busbw: float, min_link_GBps: float, max_bytes: int, sysfs_root: str = "/sys/",
        nfd_dir: Optional[str] = None, timeout: float = 600, artifact_dir: str = "/etc/amd/scale-out",
        tune_rccl: bool = False) -> dict:
    checks: List[dict] = []
    report: dict = {"gpus": gpus, "started": time.time()}

    # 1. topology (no GPU needed)
    try:
        from .models.topology import NodeTopology

        topo = NodeTopology.discover(sysfs_root)
        x = topo.xgmi
        need = x.pairs_expected if gpus == len(x.gpus) else gpus * (gpus - 1) // 2
        checks.append(_check("xgmi_topology", x.pairs_connected >= need, pairs=x.pairs_connected,
                             expected=need, per_gpu_bw_mbs=x.per_gpu_bw_mbs))
        checks.append(_check("gpu_nic_affinity", bool(topo.pairs) and not topo.unpaired_gpus,
                             pairs={p.gpu_bdf: f"{p.nic} ({p.path})" for p in topo.pairs},
                             unpaired_gpus=topo.unpaired_gpus))
        # The links' trained state (amdgpu gpu_metrics), as the agent reads it: none down.
        from .agent import native

        health = native().read_xgmi_health(sysfs_root, list(topo.gpus), 5000)  # bounded: a wedged SMU fails, never hangs
        known = [h for h in health if h["known"]]
        late = [h["bdf"] for h in health if h.get("late")]
        if late:
            checks.append(_check("gpu_metrics_answers", False, late=late, why="gpu_metrics did not answer in 5s"))
        if known:
            down = {h["bdf"]: [i for i, st in enumerate(h["status"]) if st == 0] for h in known}
            checks.append(_check("xgmi_link_state", not any(down.values()),
                                 links_up=sum(st == 1 for h in known for st in h["status"]),
                                 down={b: v for b, v in down.items() if v},
                                 width=min(h["width"] for h in known), speed_gbps=min(h["speed_gbps"] for h in known)))
        else:
            # No GPU's gpu_metrics layout is one the reader decodes (other firmware): said, not
            # left out -- a skipped check does not fail the validation.
            checks.append({"check": "xgmi_link_state", "ok": True, "skipped": True,
                           "why": "; ".join(sorted({h.get("error") or "unreadable" for h in health})) or "no GPU found"})
        pcie = rail_pcie_check(topo, sysfs_root)
        if pcie:
            checks.append(pcie)
        tf = Path(artifact_dir) / "rccl-topo.xml"
        if tf.exists():
            agree = topo_file_agrees(tf.read_text(), topo)
            checks.append(_check("rccl_topology_file", agree.pop("ok"), path=str(tf), **agree))
    except Exception as e:
        checks.append(_check("xgmi_topology", False, error=str(e)))

    # 2. xGMI probe (pull + push, byte exact)
    try:
        r = subprocess.run([str(native_bin("netop-xgmi-probe")), "--bytes=67108864", "--iters=5",
                            f"--max-gpus={gpus}"], capture_output=True, text=True, timeout=timeout)
        p = json.loads(r.stdout.strip().splitlines()[-1])
        n = p["gpus"]
        links = [p["link_GBps"][d][q] for d in range(n) for q in range(n) if d != q]
        ok = r.returncode == 0 and p["errors"] == 0 and p.get("push_errors", 0) == 0
        if links:
            ok = ok and min(links) >= min_link_GBps
        checks.append(_check("xgmi_probe", ok, gpus=n, min_link_GBps=min(links) if links else None,
                             pull_aggregate_GBps=p["aggregate_GBps"], push_aggregate_GBps=p.get("push_aggregate_GBps"),
                             errors=p["errors"] + p.get("push_errors", 0)))
    except Exception as e:
        checks.append(_check("xgmi_probe", False, error=str(e)[-500:]))

    # 3 + 4. RCCL sweep with counters around it
    before = None
    try:
        from .ops import smi

        before = smi.snapshot()
    except Exception as e:
        report["smi_error"] = str(e)
    #    RCCL runs the way jobs on this node run it: with the agent's rccl.env (its NCCL_TOPO_FILE
    #    included) and rccl-tuned.env sourced, and RCCL's own topology dump read back.
    from .parallel import fabric_artifacts as FA

    art_env = FA.load_env_dir(artifact_dir)
    scratch = tempfile.mkdtemp(prefix="netop-validate-")
    try:
        from .parallel import rccl_bench

        dump = os.path.join(scratch, FA.DUMP_FILE)
        rows = rccl_bench.run(op="all_reduce", gpus=gpus, min_bytes=1 << 20, max_bytes=max_bytes, factor=8,
                              iters=20, warmup=5, timeout=timeout, env=dict(art_env, NCCL_TOPO_DUMP_FILE=dump))
        wrong = sum(r.wrong for r in rows)
        peak = max((r.busbw_GBps for r in rows), default=0.0)
        ok = bool(rows) and wrong == 0 and (gpus == 1 or peak >= min_busbw)
        checks.append(_check("rccl_all_reduce", ok, peak_busbw_GBps=peak, wrong=wrong, min_busbw_GBps=min_busbw,
                             rccl_env=art_env, artifacts_applied=bool(art_env),
                             sizes=[{"bytes": r.bytes, "time_us": r.time_us, "busbw_GBps": r.busbw_GBps} for r in rows]))
        report["busbw_GBps"] = peak
        if art_env:
            checks.append(rccl_links_check(gpus, dump, art_env, scratch, timeout))
    except Exception as e:
        checks.append(_check("rccl_all_reduce", False, error=str(e)[-500:]))
    finally:
        shutil.rmtree(scratch, ignore_errors=True)
    if before is not None:
        try:
            t = smi.traffic(before, smi.snapshot())
            # Only GPUs taking part can be expected to move data; with n == 8 every up link must.
            ok = gpus < 8 or t["links_with_traffic"] >= t["links_up"]
            checks.append(_check("xgmi_counters", ok, links_up=t["links_up"],
                                 links_with_traffic=t["links_with_traffic"]))
        except Exception as e:
            checks.append(_check("xgmi_counters", False, error=str(e)))

    # 5. The direct xGMI all-reduce jobs can use (one process per GPU, HIP IPC buffers), exact.
    checks.append(direct_all_reduce_check(gpus, max_bytes, min(timeout, 300)))
    if tune_rccl and gpus > 1:
        try:
            from .parallel import rccl_bench

            # on top of the agent's rccl.env (its NCCL_TOPO_FILE): the environment jobs run with
            probes = rccl_bench.env_probe(gpus, max_bytes, budget_s=min(timeout, 300),
                                          base_env=FA.parse_env_text((Path(artifact_dir) / FA.ENV_FILE).read_text())
                                          if (Path(artifact_dir) / FA.ENV_FILE).is_file() else {})
            pick = rccl_bench.choose_env(probes)
            report["rccl_tuning"] = dict(pick, probes=probes)
            out = Path(artifact_dir) / "rccl-tuned.env"
            if pick["chosen"]:
                out.parent.mkdir(parents=True, exist_ok=True)
                tmp = out.with_suffix(".tmp")
                tmp.write_text("# Measured by the fabric validation Job (validate.py --tune-rccl): "
                               f"{pick['best_busbw_GBps']:.1f} vs {pick['baseline_busbw_GBps']:.1f} GB/s busbw "
                               "with RCCL's defaults\n" + "".join(f"{k}={v}\n" for k, v in sorted(pick["chosen"].items())))
                os.replace(tmp, out)
            elif out.exists():
                out.unlink()  # the defaults are best now: drop a stale override
        except Exception as e:
            report["rccl_tuning"] = {"error": str(e)[-500:]}
    report["checks"] = checks
    report["ok"] = all(c["ok"] for c in checks)
    report["seconds"] = time.time() - report.pop("started")
    if nfd_dir:
        path = Path(nfd_dir) / LABEL_FILE
        if report["ok"]:
            Path(nfd_dir).mkdir(parents=True, exist_ok=True)
            tmp = path.with_suffix(".tmp")
            tmp.write_text(f"{LABEL}=true\n{LABEL}.busbw-gbps={int(report.get('busbw_GBps', 0))}\n")
            os.replace(tmp, path)
        elif path.exists():
            path.unlink()
        report["label_file"] = str(path) if report["ok"] else None
    return report


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m network_operator_amd.validate", description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=8)
    ap.add_argument("--min-busbw", type=float, default=0.0,
                    help="required large-message all-reduce busbw in GB/s (n > 1); 0 = only correctness")
    ap.add_argument("--min-link", type=float, default=0.0, help="required per-link pull GB/s (n > 1)")
    ap.add_argument("--max-bytes", type=int, default=1 << 30)
    ap.add_argument("--sysfs-root", default=os.environ.get("SYSFS_ROOT", "/sys/"))
    ap.add_argument("--nfd-features-dir", default=None, help="write the validation label here when all checks pass")
    ap.add_argument("--artifact-dir", default="/etc/amd/scale-out", help="the agent's RCCL artifacts (rccl-topo.xml)")
    ap.add_argument("--tune-rccl", action="store_true",
                    help="measure RCCL knob variants and write the winner to <artifact-dir>/rccl-tuned.env")
    a = ap.parse_args(argv)
    rep = run(a.gpus, a.min_busbw, a.min_link, a.max_bytes, a.sysfs_root, a.nfd_features_dir,
              artifact_dir=a.artifact_dir, tune_rccl=a.tune_rccl)
    print(json.dumps(rep))
    return 0 if rep["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
