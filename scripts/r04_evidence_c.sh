#!/bin/bash
# Round-4 evidence, part C: the group scaling model (scripts/shard_model.py) for bunny and vokselia.
set -o pipefail
TAG=${1:-r04a}
mkdir -p gpurun_out
timeout -k 10 500 python scripts/shard_model.py bunny > "gpurun_out/${TAG}_shard_model.jsonl" 2>&1 || exit 6
timeout -k 10 500 python scripts/shard_model.py vokselia >> "gpurun_out/${TAG}_shard_model.jsonl" 2>&1 || exit 7
echo "all done"
