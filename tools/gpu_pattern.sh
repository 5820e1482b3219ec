#!/bin/bash
# Pattern kernels after the SWAR rewrite (round 4): numerics vs the fp32 PyTorch reference, their
# time under rocprofv3 --kernel-trace --stats, then PMC passes of their own (HBM bytes, VALU work).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T=${TAG:-r4}  # output name prefix
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_ops.py -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/${T}_pytest_gpu_ops.log 2>&1 || { tail -30 gpurun_out/${T}_pytest_gpu_ops.log; exit 1; }
tail -3 gpurun_out/${T}_pytest_gpu_ops.log
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/${T}_prof_pattern -o kern --output-format csv -- python3 $R/tools/kernel_timing.py > $R/gpurun_out/${T}_prof_pattern.log 2>&1 || { tail -20 $R/gpurun_out/${T}_prof_pattern.log; exit 1; }
tail -3 $R/gpurun_out/${T}_prof_pattern.log
for c in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  tag=$(echo $c | cut -d' ' -f1)
  timeout -s KILL 90 rocprofv3 --pmc $c --kernel-trace -d $R/gpurun_out/${T}_pmc_$tag -o pmc --output-format csv -- python3 $R/tools/kernel_timing.py > $R/gpurun_out/${T}_pmc_$tag.log 2>&1 || { echo "pmc $c failed"; tail -5 $R/gpurun_out/${T}_pmc_$tag.log; exit 1; }
done
echo PATTERN OK
