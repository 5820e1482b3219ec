#!/bin/bash
# The streaming copy's tuning sweep on one GPU (HBM loopback), with nontemporal-load variants.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 network_operator_amd/_lib/netop-copy-tune > gpurun_out/copy_tune.jsonl 2> gpurun_out/copy_tune.err || { tail -5 gpurun_out/copy_tune.err; exit 1; }
wc -l gpurun_out/copy_tune.jsonl
