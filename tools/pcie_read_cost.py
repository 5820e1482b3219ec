import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import time, json
from network_operator_amd.agent import native
n = native()
d = n.discover("/sys/", "affine")
bdfs = [p["gpu"] for p in d["pairs"]] + [nn["bdf"] for nn in d["nics"] if any(nn["ifname"] == p["nic"] for p in d["pairs"])]
t = time.perf_counter(); [n.read_pcie_link("/sys/", b) for b in bdfs]; first = time.perf_counter() - t
t = time.perf_counter()
for _ in range(20): [n.read_pcie_link("/sys/", b) for b in bdfs]
again = (time.perf_counter() - t) / 20
t = time.perf_counter(); n.read_xgmi_health("/sys/", [p["gpu"] for p in d["pairs"]]); gm = time.perf_counter() - t
print(json.dumps({"functions": len(bdfs), "pcie_first_ms": first * 1e3, "pcie_ms": again * 1e3, "gpu_metrics_8_ms": gm * 1e3}))
