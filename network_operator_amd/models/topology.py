"""Node scale-out topology model (typed view of the native discovery in native/src/topology.cpp)."""

from __future__ import annotations

from dataclasses import dataclass, field
from typing import List


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

    @classmethod
    def discover(cls, sysfs_root: str = "/sys/") -> "NodeTopology":
        from ..agent import native

        n = native()
        d = n.discover(sysfs_root)
        x = n.read_xgmi(sysfs_root)
        return cls(gpus=[g["bdf"] for g in d["gpus"]], nics=list(d["ifnames"]),
                   pairs=[GpuNicPair(p["gpu"], p["nic"], p["path"], p["common_depth"]) for p in d["pairs"]],
                   xgmi=XgmiMesh(x["gpus"], x["pairs_expected"], x["pairs_connected"], x["per_gpu_bw_mbs"],
                                 [tuple(m) for m in x["missing"]]))

    def nic_for_gpu(self, bdf: str) -> str | None:
        for p in self.pairs:
            if p.gpu_bdf == bdf:
                return p.nic
        return None
