"""Time-to-solution of a sparse configuration twice in one process (the first run pays the lazy loading of the
library's code objects for its kernels; the second shows the setup without it). usage: learn_twice.py <config>"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import argparse  # noqa: E402

import bench  # noqa: E402

cfg = sys.argv[1]
args = argparse.Namespace(sparse_algo="auto", host_exchange=False)
for k in range(2):
    rec = bench.run_config(cfg, args, 0, 1, None, None, 2, 1, False, 0.0, 1, solve=True)
    print(cfg, "run", k, "learn_s", rec["learn"]["learn_s"], "setup_s", rec["learn"]["setup_s"], flush=True)
