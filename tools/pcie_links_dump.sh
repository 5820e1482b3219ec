#!/bin/bash
# PCIe link state of every GPU and network PCI function on the box (unprivileged sysfs reads):
# negotiated vs maximum speed and width, for the function and the bridge above it.
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/pcie_links.txt
: > "$out"
for d in /sys/bus/pci/devices/*; do
  cls=$(cat "$d/class" 2>/dev/null)
  case "$cls" in 0x0200*|0x0207*|0x1200*|0x0380*) ;; *) continue ;; esac
  drv=$(basename "$(readlink -f "$d/driver" 2>/dev/null)" 2>/dev/null)
  up=$(basename "$(dirname "$(readlink -f "$d")")")
  printf '%s class=%s driver=%s cur=%s x%s max=%s x%s | up %s cur=%s x%s max=%s x%s\n' "$(basename "$d")" "$cls" "$drv" \
    "$(cat "$d/current_link_speed" 2>/dev/null)" "$(cat "$d/current_link_width" 2>/dev/null)" \
    "$(cat "$d/max_link_speed" 2>/dev/null)" "$(cat "$d/max_link_width" 2>/dev/null)" "$up" \
    "$(cat "/sys/bus/pci/devices/$up/current_link_speed" 2>/dev/null)" "$(cat "/sys/bus/pci/devices/$up/current_link_width" 2>/dev/null)" \
    "$(cat "/sys/bus/pci/devices/$up/max_link_speed" 2>/dev/null)" "$(cat "/sys/bus/pci/devices/$up/max_link_width" 2>/dev/null)" >> "$out"
done
cat "$out"
