set -e
mkdir -p gpurun_out/pmc
hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/spmv_microbench.hip -o /tmp/mb 2>/dev/null
cd /tmp
export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc/a -o run -- /tmp/mb 256 > $GRAFT_REPO_ROOT/gpurun_out/pmc/a.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_SALU --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc/b -o run -- /tmp/mb 256 > $GRAFT_REPO_ROOT/gpurun_out/pmc/b.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE TCP_TCC_READ_REQ_sum --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/pmc/c -o run -- /tmp/mb 256 > $GRAFT_REPO_ROOT/gpurun_out/pmc/c.txt 2>&1
find $GRAFT_REPO_ROOT/gpurun_out/pmc -name "*.csv" | head
