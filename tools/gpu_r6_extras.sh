#!/bin/bash
# Round-6 box evidence: the GPU suite, then the sysfs read costs (serial vs the agent's bounded
# concurrent gpu_metrics read) and a require-rdma dry run of the agent on this node.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -4 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 tools/pcie_read_cost.py > gpurun_out/box_read_costs.json 2>&1 || { cat gpurun_out/box_read_costs.json; exit 1; }
cat gpurun_out/box_read_costs.json
timeout -k 10 60 network_operator_amd/_lib/bin/discover --dry-run --require-rdma --mode=L3 --xgmi-expect=0 \
  --status-file=gpurun_out/require_rdma_status.json -v=1 > gpurun_out/require_rdma_dry_run.log 2>&1 || { tail -20 gpurun_out/require_rdma_dry_run.log; exit 1; }
grep -E "would wait for RDMA|without an RDMA|xGMI links" gpurun_out/require_rdma_dry_run.log || true
timeout -k 10 120 python3 -m network_operator_amd.agent.report > gpurun_out/node_report_box.txt 2>&1; echo "report rc=$?"
head -3 gpurun_out/node_report_box.txt
