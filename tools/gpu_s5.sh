# sparse correctness + the two sparse RBF configs (scratch session script)
tools/gpu_session.sh $1 \
 "timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_sparse.py" \
 "timeout -k 10 400 python -u -m pytest -q -s --timeout 300 --timeout-method thread tests/test_gpu_overlap.py tests/test_gpu_multirank.py -k 'auto or expansion or sparse'" \
 "timeout -k 10 300 python -u bench.py --config csr_rbf_1m --no-cpu --steps 20" \
 "timeout -k 10 300 python -u bench.py --config fp22_rbf_2m --no-cpu --steps 20"
