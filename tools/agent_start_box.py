"""The node agent's unprivileged start phases on this node's real sysfs, repeated (per-phase
p50 / p95); see network_operator_amd/agent/start_timing.py.

    python tools/agent_start_box.py [--runs 30] [--sysfs /sys/]"""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

from network_operator_amd.agent.start_timing import main  # noqa: E402

if __name__ == "__main__":
    sys.exit(main())
