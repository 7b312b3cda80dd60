#!/bin/bash
# Round 6 profiles (one gpurun call): rocprofv3 kernel-trace + FETCH_SIZE passes of the bench configurations
# (tools/profile_config.sh) and the dense tile kernel's MFMA PMC pass (tools/pmc_dense.sh).
set -u
for c in ${*:-dense_rbf_100k csr_rbf_1m fp22_rbf_2m csr_linear_1m}; do
  bash tools/profile_config.sh "r06_$c" "$c" || exit $?
done
bash tools/pmc_dense.sh r06_dense_rbf_100k || exit $?
