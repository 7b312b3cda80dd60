"""One rank of a world-2 host-staged group running a long-trace case with the one-reduction CG (tests/test_gpu_cg1.py).

usage: python cg1_worker.py CASE RANK WORLD PORT OUTDIR VARIANT
"""
import datetime
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

import long_trace_cases as lc  # noqa: E402


def main():
    name, rank, world, port, out, variant = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), \
        sys.argv[5], sys.argv[6]
    import torch.distributed as dist

    import plssvm_sparse_fp22_amd as pm

    pm._abi.lib()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=90))  # a lost peer fails the case, not the suite
    kernel, dtype, _, _, _, _, algo, env, _ = lc.CASES[name]
    os.environ.update(env)
    s = lc.load(name)
    p = pm.Parameter(kernel, degree=3, gamma=float(s["gamma"]), coef0=float(s["coef0"]), cost=s["cost"],
                     epsilon=s["eps"], real_type=dtype)
    if "X" in s:
        p.data = s["X"]
    else:
        p.csr = s["csr"]
    p.labels = s["y"]
    svm = pm.CSVM(p, device=0, rank=rank, world_size=world, exchange=pm.torch_exchange(dist), sparse_algo=algo,
                  cg_variant=variant)
    svm.learn(imax=lc.IMAX)
    np.savez(os.path.join(out, f"rank{rank}.npz"), alpha=svm.alpha, trace=np.asarray(svm.trace), iters=svm.iters)
    svm.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
