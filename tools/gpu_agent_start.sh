#!/bin/bash
# The agent's unprivileged start phases on this box's real sysfs, 30 runs; then the box tests of
# the agent (dry runs, readings against amd-smi and raw sysfs).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 tools/agent_start_box.py --runs 30 > gpurun_out/agent_start_box.json 2> gpurun_out/agent_start_box.err || { tail -20 gpurun_out/agent_start_box.err; cat gpurun_out/agent_start_box.json; exit 1; }
cat gpurun_out/agent_start_box.json
timeout -k 10 600 python3 -u -m pytest tests/test_agent_box.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_agent_box.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_agent_box.log
exit $rc
