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
gpus = [g["bdf"] for g in d["gpus"]]
t = time.perf_counter(); n.read_xgmi_health("/sys/", gpus); gm = time.perf_counter() - t
# The agent's way since round 6: one thread per GPU, every read bounded (5 s), joined together.
serial, concurrent = [], []
for _ in range(10):
    t = time.perf_counter(); n.read_xgmi_health("/sys/", gpus); serial.append(time.perf_counter() - t)
    t = time.perf_counter(); h = n.read_xgmi_health("/sys/", gpus, 5000); concurrent.append(time.perf_counter() - t)
assert not any(x["late"] for x in h), h
med = lambda xs: sorted(xs)[len(xs) // 2] * 1e3  # noqa: E731
print(json.dumps({"functions": len(bdfs), "pcie_first_ms": first * 1e3, "pcie_ms": again * 1e3, "gpus": len(gpus),
                  "gpu_metrics_first_serial_ms": gm * 1e3, "gpu_metrics_serial_p50_ms": med(serial),
                  "gpu_metrics_concurrent_bounded_p50_ms": med(concurrent),
                  "links_up": sum(st == 1 for x in h for st in x["status"])}))
