#!/bin/bash
# Raw amdgpu gpu_metrics blobs of every card on the box (unprivileged sysfs reads), with each
# card's PCI address and, right after, amd-smi's per-link xGMI view (netop-xgmi-counters), so the
# blob's xGMI fields can be located and checked against the library's reading.
set -o pipefail
mkdir -p gpurun_out/gpu_metrics
for c in /sys/class/drm/card*; do
  [ -e "$c/device/gpu_metrics" ] || continue
  n=$(basename "$c")
  cat "$c/device/gpu_metrics" > "gpurun_out/gpu_metrics/$n.bin" 2>/dev/null || echo "$n: unreadable"
  echo "$n $(basename "$(readlink -f "$c/device")")" >> gpurun_out/gpu_metrics/cards.txt
done
timeout -k 10 60 network_operator_amd/_lib/netop-xgmi-counters > gpurun_out/gpu_metrics/xgmi_counters.json 2>&1
for c in /sys/class/drm/card*; do
  [ -e "$c/device/gpu_metrics" ] || continue
  cat "$c/device/gpu_metrics" > "gpurun_out/gpu_metrics/$(basename "$c").after.bin" 2>/dev/null
done
ls -la gpurun_out/gpu_metrics | head -40
cat gpurun_out/gpu_metrics/cards.txt
