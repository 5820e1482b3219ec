#!/bin/bash
# Build + GPU test suite only.
set -o pipefail
mkdir -p gpurun_out
python3 -c 'import __graft_entry__ as g; g.build()' > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 900 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -m network_operator_amd.validate --gpus 1 --max-bytes 268435456 > gpurun_out/validate.json 2>gpurun_out/validate.err
echo "validate rc=$?"; head -c 1500 gpurun_out/validate.json
