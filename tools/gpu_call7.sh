set -u
mkdir -p gpurun_out/c7
timeout -k 10 300 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu tests/test_gpu_bench.py > gpurun_out/c7/pytest.log 2>&1 || exit $?
tail -2 gpurun_out/c7/pytest.log
bash tools/gpu_profiles.sh r03 csr_rbf_1m fp22_rbf_2m || exit $?
export PLSSVM_MI_SHARD=1
bash tools/prof_stats.sh fp22_share0of8 --config fp22_rbf_2m --sim-rank 0/8 --steps 10 --warmup 2 || exit $?
