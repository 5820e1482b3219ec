#!/bin/bash
# PMC counters (own runs, kernel-trace only, ONE derived counter per pass — two at once exceed
# the hardware's counter slots and rocprofv3 aborts): HBM bytes of the copy / reduce kernels.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
python3 -c 'import __graft_entry__ as g; g.build()' > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
cd /tmp
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -k 5 90 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/pmc_copy_$c -o copy --output-format csv -- $R/network_operator_amd/_lib/netop-xgmi-probe --bytes=268435456 --iters=3 > $R/gpurun_out/pmc_copy_$c.log 2>&1 || { echo "copy $c failed"; grep -v '^    @' $R/gpurun_out/pmc_copy_$c.log | tail -5; exit 1; }
  timeout -k 5 90 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/pmc_xa_$c -o xa --output-format csv -- $R/network_operator_amd/_lib/netop-xgmi-allreduce --ranks 1 -b 256M -e 256M -n 3 -w 1 --mode pull > $R/gpurun_out/pmc_xa_$c.log 2>&1 || { echo "xa $c failed"; exit 1; }
done
echo PMC OK
