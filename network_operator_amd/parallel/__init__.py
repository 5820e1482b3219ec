"""Distributed validation over RCCL (xGMI inside a node, RoCE across nodes)."""

from .collectives import (BUS_FACTORS, CollectiveResult, bandwidths, bus_factor, run_sweep, sweep_sizes,
                          time_collective, verify_all_reduce, xgmi_busbw_ceiling_GBps)

__all__ = ["BUS_FACTORS", "CollectiveResult", "bandwidths", "bus_factor", "run_sweep", "sweep_sizes", "time_collective",
           "verify_all_reduce", "xgmi_busbw_ceiling_GBps"]
