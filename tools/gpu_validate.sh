#!/bin/bash
# The validation Job's program on the box, fed by the agent's own dry-run artifacts
# (rccl.env + NCCL_TOPO_FILE), as on a configured node.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
ART=$(mktemp -d)
timeout -k 10 60 network_operator_amd/_lib/bin/discover --dry-run --xgmi-expect=0 --rccl-topo=$ART/rccl-topo.xml \
  --rccl-env=$ART/rccl.env --status-file=$ART/status.json > gpurun_out/validate_agent.log 2>&1 || { tail -20 gpurun_out/validate_agent.log; exit 1; }
cat $ART/rccl.env
timeout -k 10 300 python3 -m network_operator_amd.validate --gpus 1 --max-bytes 268435456 --artifact-dir $ART \
  --nfd-features-dir $ART/features.d > gpurun_out/validate_n1.json 2> gpurun_out/validate_n1.err; rc=$?
python3 -c "import json; r=json.load(open('gpurun_out/validate_n1.json')); print(r['ok'], [(c['check'], c['ok']) for c in r['checks']])"
exit $rc
