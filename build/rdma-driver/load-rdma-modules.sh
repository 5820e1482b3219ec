#!/bin/sh
# The RDMA (verbs) driver of every RoCE NIC driver bound on this node, loaded from the host's
# /lib/modules (which the operator mounts there), then exit 0: the privileged init container of
# an agent Pod (amdScaleOut.driverImage / hostNic.driverImage).  With requireRdma the agent keeps
# the node unlabelled until every rail has its RDMA device; this is what makes them appear.
#
#   NIC driver  -> RDMA driver
#   ionic       -> ionic_rdma   (AMD Pensando Pollara)
#   mlx5_core   -> mlx5_ib      (NVIDIA ConnectX)
#   bnxt_en     -> bnxt_re      (Broadcom)
#   ice, i40e   -> irdma        (Intel E810 / X722)
#
# Arguments (or RDMA_MODULES) name the modules instead.  A module that is not built for the
# running kernel fails the container, naming it: the Pod's status then says why.
set -eu
sys=${SYSFS_ROOT:-/sys}
modules="$*"
[ -n "$modules" ] || modules="${RDMA_MODULES:-}"
if [ -z "$modules" ]; then
  for drv in "$sys"/class/net/*/device/driver; do
    [ -e "$drv" ] || continue
    case "$(basename "$(readlink -f "$drv")")" in
      ionic) m=ionic_rdma ;;
      mlx5_core) m=mlx5_ib ;;
      bnxt_en) m=bnxt_re ;;
      ice | i40e) m=irdma ;;
      *) continue ;;
    esac
    case " $modules " in
      *" $m "*) ;;
      *) modules="${modules:+$modules }$m" ;;
    esac
  done
fi
if [ -z "$modules" ]; then
  echo "no RoCE NIC driver is bound on this node: nothing to load"
  exit 0
fi
rc=0
for m in $modules; do
  if [ -d "$sys/module/$m" ]; then
    echo "$m: already loaded"
  elif modprobe "$m"; then
    echo "$m: loaded"
  else
    echo "$m: modprobe failed (is it built for kernel $(uname -r) under /lib/modules?)" >&2
    rc=1
  fi
done
exit $rc
