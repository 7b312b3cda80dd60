set -u
mkdir -p gpurun_out/c3
timeout -k 10 120 tools/hbm_probe > gpurun_out/c3/hbm_probe.json 2> gpurun_out/c3/hbm_probe.err || exit $?
cat gpurun_out/c3/hbm_probe.json
bash tools/profile_config.sh r03_dense_rbf_100k dense_rbf_100k || exit $?
export PLSSVM_MI_SHARD=1
bash tools/prof_stats.sh fp22_share0of8 --config fp22_rbf_2m --sim-rank 0/8 --steps 10 --warmup 2 || exit $?
bash tools/prof_stats.sh fp22_share7of8 --config fp22_rbf_2m --sim-rank 7/8 --steps 10 --warmup 2 || exit $?
