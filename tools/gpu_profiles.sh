#!/bin/bash
# One gpurun call: the round's rocprofv3 kernel-trace + FETCH_SIZE passes of every bench configuration
# (tools/profile_config.sh) and the 8-rank shares of config 5 on the sharded path (tools/sim_shares.sh).
# usage (GPU box, repo root): tools/gpu_profiles.sh <round tag> [configs...]
set -eu
tag=$1; shift
configs=${*:-"dense_rbf_100k csr_rbf_1m fp22_rbf_2m csr_linear_1m"}
for c in $configs; do
  bash tools/profile_config.sh "${tag}_$c" "$c"
done
PLSSVM_MI_SHARD=1 bash tools/sim_shares.sh fp22_rbf_2m 8
