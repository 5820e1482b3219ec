#!/bin/bash
# HBM bytes of the round-6 kernels (nontemporal sum and copy), one counter per pass, kernel trace
# only: the 8-source sum (256 MiB per buffer) and the probe's loopback copy (256 MiB).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 5 120 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/pmc6_sum_$c -o sum --output-format csv -- python3 $R/tools/sum_rate_box.py --sources 8 --wg-per-cu 0 --iters 3 --mib 256 > $R/gpurun_out/pmc6_sum_$c.log 2>&1 || { echo "sum $c failed"; tail -5 $R/gpurun_out/pmc6_sum_$c.log; exit 1; }
  timeout -k 5 90 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/pmc6_copy_$c -o copy --output-format csv -- $R/network_operator_amd/_lib/netop-xgmi-probe --bytes=268435456 --iters=3 > $R/gpurun_out/pmc6_copy_$c.log 2>&1 || { echo "copy $c failed"; tail -5 $R/gpurun_out/pmc6_copy_$c.log; exit 1; }
done
echo PMC OK
find $R/gpurun_out -path '*pmc6_*' -name '*counter_collection*' | head
