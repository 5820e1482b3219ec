"""Node scale-out topology model: a typed view of the agent's native discovery
(native/src/topology.cpp), i.e. GPUs, GPU-affine NICs and their RDMA devices, the GPU<->NIC PCIe
pairing and the KFD xGMI mesh.

Consumers: ``validate.py`` (topology and GPU-NIC affinity checks, agreement of the agent's
NCCL_TOPO_FILE with the live PCIe tree), ``parallel/rail.py`` (a rank's own rail NIC when the
node has no ``rccl-net.json``, e.g. L2 mode)."""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple


@dataclass(frozen=True)
class GpuNicPair:
    gpu_bdf: str
    nic: str
    path: str          # NCCL path type: PIX / PXB / PHB / NODE / SYS
    common_depth: int


@dataclass
class XgmiMesh:
    gpus: List[str]
    pairs_expected: int
    pairs_connected: int
    per_gpu_bw_mbs: int
    missing: List[tuple] = field(default_factory=list)

    @property
    def full_mesh(self) -> bool:
        return self.pairs_connected == self.pairs_expected

    def busbw_ceiling_GBps(self) -> float:
        """All-reduce busbw ceiling implied by the advertised links (MB/s -> GB/s)."""
        return self.per_gpu_bw_mbs / 1000.0


@dataclass
class NodeTopology:
    gpus: List[str]
    nics: List[str]
    pairs: List[GpuNicPair]
    xgmi: XgmiMesh
    rdma: Dict[str, str] = field(default_factory=dict)  # scale-out ifname -> RDMA device ("" = none)

    @classmethod
    def discover(cls, sysfs_root: str = "/sys/", with_xgmi: bool = True) -> "NodeTopology":
        from ..agent import native

        n = native()
        d = n.discover(sysfs_root)
        x = n.read_xgmi(sysfs_root) if with_xgmi else {"gpus": [], "pairs_expected": 0, "pairs_connected": 0,
                                                       "per_gpu_bw_mbs": 0, "missing": []}
        return cls(gpus=[g["bdf"] for g in d["gpus"]], nics=list(d["ifnames"]),
                   pairs=[GpuNicPair(p["gpu"], p["nic"], p["path"], p["common_depth"]) for p in d["pairs"]],
                   xgmi=XgmiMesh(x["gpus"], x["pairs_expected"], x["pairs_connected"], x["per_gpu_bw_mbs"],
                                 [tuple(m) for m in x["missing"]]),
                   rdma={nic["ifname"]: nic["rdma_dev"] for nic in d["nics"] if nic["ifname"] in d["ifnames"]})

    def nic_for_gpu(self, bdf: str) -> Optional[str]:
        bdf = bdf.lower()
        for p in self.pairs:
            if p.gpu_bdf.lower() == bdf:
                return p.nic
        return None

    def rdma_for_gpu(self, bdf: str) -> Optional[Tuple[str, int]]:
        """(RDMA device, port) of the NIC paired with GPU ``bdf``; None without one."""
        nic = self.nic_for_gpu(bdf)
        dev = self.rdma.get(nic or "", "")
        return (dev, 1) if dev else None

    @property
    def unpaired_gpus(self) -> List[str]:
        paired = {p.gpu_bdf for p in self.pairs}
        return [g for g in self.gpus if g not in paired]
