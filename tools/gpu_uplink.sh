#!/bin/bash
# The agent's default-route refusal on the box's real kernel: a dry run that names the box's
# uplink (the interface its default route leaves through) must report it refused, and a dry run
# with rdma discovery must not take it.  Unprivileged: reading routes needs no capability.
set -o pipefail
mkdir -p gpurun_out
cat /proc/net/route > gpurun_out/box_routes.txt
ls /sys/class/net > gpurun_out/box_netdevs.txt
UP=$(awk 'NR > 1 && $2 == "00000000" { print $1; exit }' /proc/net/route)
echo "uplink: ${UP:-none}" | tee gpurun_out/box_uplink.log
[ -n "$UP" ] || exit 0
timeout -k 5 60 network_operator_amd/_lib/bin/discover --dry-run --mode=L2 --nic-discovery=none --interfaces="$UP" \
  --status-file=gpurun_out/box_uplink_status.json >> gpurun_out/box_uplink.log 2>&1
echo "rc=$?" >> gpurun_out/box_uplink.log
timeout -k 5 60 network_operator_amd/_lib/bin/discover --dry-run --mode=L2 --nic-discovery=rdma --nic-drivers= \
  --status-file=gpurun_out/box_rdma_status.json > gpurun_out/box_rdma.log 2>&1
echo "rc=$?" >> gpurun_out/box_rdma.log
exit 0
