set -e
export TMPDIR=/tmp
root=$(pwd)
mkdir -p gpurun_out/p1
cd /tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $root/gpurun_out/p1/trace -o run -- python3 $root/bench.py --config csr_rbf_1m --no-cpu --steps 10 --warmup 1 > $root/gpurun_out/p1/bench.json 2> $root/gpurun_out/p1/bench.err
cd $root
find gpurun_out/p1 -type f ! -name '*kernel_stats.csv' ! -name '*.json' ! -name '*.err' -delete
timeout -k 10 400 python3 bench.py --config fp22_rbf_2m --no-cpu --steps 10 --warmup 1 > gpurun_out/p1/fp22.json 2> gpurun_out/p1/fp22.err
