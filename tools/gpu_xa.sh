set -o pipefail
mkdir -p gpurun_out
python3 -c 'import __graft_entry__ as g; g.build()' > gpurun_out/build.log 2>&1 || { tail -30 gpurun_out/build.log; exit 1; }
timeout -k 10 600 python3 -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 network_operator_amd/_lib/netop-xgmi-allreduce --ranks 8 -b 1M -e 1G -f 32 -n 10 -w 2 > gpurun_out/xa8.jsonl 2> gpurun_out/xa8.txt; cat gpurun_out/xa8.txt
timeout -k 10 300 network_operator_amd/_lib/netop-xgmi-allreduce --ranks 1 -b 1M -e 1G -f 32 -n 10 -w 2 2>&1 | tail -8
