# sparse correctness + the two sparse RBF configs (scratch session script)
tools/gpu_session.sh s6 \
 "timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py" \
 "timeout -k 10 300 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_overlap.py -k 'auto or expansion'" \
 "timeout -k 10 300 python -u bench.py --config csr_rbf_1m --no-cpu --steps 20" \
 "timeout -k 10 300 python -u bench.py --config fp22_rbf_2m --no-cpu --steps 20"
