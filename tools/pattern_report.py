"""Summarises tools/gpu_pattern.sh's rocprofv3 output for the pattern kernels: per (buffer size,
ranks in the pattern, kernel) the median kernel time and HBM rate from the kernel trace, and
from the PMC passes the HBM bytes per call (FETCH_SIZE doubled: gfx950 reports half of a wide
streaming read, MI355X_MICROARCH.md) and the VALU instructions per 16-byte vector.

    python tools/pattern_report.py gpurun_out [TAG] > profiles/r4_pattern_kernels.json
"""
import csv
import json
import statistics
import sys
from pathlib import Path

# kernel_timing.py's order: for size in (64 MiB, 1 GiB): for ranks in (1, 8): fill, verify
SEQ = [(size, ranks, k) for size in (64 << 20, 1 << 30) for ranks in (1, 8) for k in ("fill", "verify")]


def _runs(rows):
    """Consecutive dispatches of the pattern kernels, grouped by kernel, in dispatch order."""
    out = []
    for r in sorted(rows, key=lambda r: int(r["Dispatch_Id"])):
        name = r["Kernel_Name"]
        k = "fill" if "fill_kernel" in name else "verify" if "verify_kernel" in name else None
        if k is None:
            continue
        if not out or out[-1][0] != k:
            out.append((k, []))
        out[-1][1].append(r)
    return out


def main(root: str, tag_prefix: str = "r4") -> dict:
    root = Path(root)
    trace = list(csv.DictReader(open(root / f"{tag_prefix}_prof_pattern" / "kern_kernel_trace.csv")))
    runs = _runs(trace)
    assert [k for k, _ in runs] == [k for _, _, k in SEQ], [k for k, _ in runs]
    table = []
    for (size, ranks, k), (_, rows) in zip(SEQ, runs):
        ns = statistics.median(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in rows)
        table.append({"kernel": k, "bytes": size, "ranks_in_pattern": ranks, "calls": len(rows),
                      "grid_threads": int(rows[0].get("Grid_Size_X") or rows[0].get("Grid_Size")), "median_us": round(ns / 1e3, 2),
                      "TBps": round(size / ns / 1e3, 2)})
    for tag, counters in (("FETCH_SIZE", ["FETCH_SIZE"]), ("WRITE_SIZE", ["WRITE_SIZE"]),
                          ("SQ_INSTS_VALU", ["SQ_INSTS_VALU", "SQ_WAVES", "SQ_INSTS_SALU", "GRBM_GUI_ACTIVE"])):
        f = root / f"{tag_prefix}_pmc_{tag}" / "pmc_counter_collection.csv"
        if not f.exists():
            continue
        rows = list(csv.DictReader(open(f)))
        by_dispatch: dict = {}
        for r in rows:
            by_dispatch.setdefault(r["Dispatch_Id"], dict(r)).setdefault("counters", {})[r["Counter_Name"]] = \
                float(r["Counter_Value"])
        runs = _runs(list(by_dispatch.values()))
        for row, (_, rs) in zip(table, runs):
            for c in counters:
                vals = [x["counters"].get(c) for x in rs if c in x["counters"]]
                if not vals:
                    continue
                v = statistics.median(vals)
                if c == "FETCH_SIZE":  # KB, half of a wide streaming read on gfx950
                    row["hbm_read_bytes_per_call"] = round(2 * v * 1024)
                    row["hbm_read_vs_buffer"] = round(2 * v * 1024 / row["bytes"], 3)
                elif c == "WRITE_SIZE":
                    row["hbm_write_bytes_per_call"] = round(v * 1024)
                    row["hbm_write_vs_buffer"] = round(v * 1024 / row["bytes"], 3)
                elif c == "SQ_INSTS_VALU":
                    row["valu_insts_per_vector"] = round(v * 64 / (row["bytes"] / 16), 1)  # wave instr x 64 lanes
                else:
                    row[c] = v
    return {"what": "HIP pattern kernels, SWAR pattern (round 4): rocprofv3 kernel trace + PMC, MI355X "
                    "(tools/gpu_pattern.sh, tools/pattern_report.py)",
            "round3": "profiles/r3_pattern_kernels.json: 1 GiB fill / verify 4.67 / 5.83 TB/s at 1 rank, 2.47 / ~2.0 "
                      "TB/s at 8 ranks",
            "rows": table}


if __name__ == "__main__":
    print(json.dumps(main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out", sys.argv[2] if len(sys.argv) > 2 else "r4"),
                     indent=1))
