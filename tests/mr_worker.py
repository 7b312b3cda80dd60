"""One rank of a world-2 host-staged group on one GPU (tests/test_gpu_multirank.py).

Started as a separate process per rank: gloo process group over 127.0.0.1, a context on the
box's GPU joined to the group with plssvm_mi_comm_init_host (the exchange = all-gather + rank-order
sum over gloo, the reference's device_reduction semantics), then the engine's real multi-rank path:
partition -> this rank's share of the implicit matrix -> exchange -> replicated device CG.
Writes q, one K·p (add = -1 and +1), the kernel part, and learn() (alpha, bias, delta trace) to
<out>/rank<r>.npz.

usage: python mr_worker.py CASE RANK WORLD PORT OUTDIR
"""
import datetime
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from mr_cases import ALGO, BUDGET, make_case  # noqa: E402


def main():
    case, rank, world, port, out = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    import torch.distributed as dist

    import plssvm_sparse_fp22_amd as pm

    pm._abi.lib()
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            timeout=datetime.timedelta(seconds=90))  # a lost peer fails the case, not the suite
    budget = BUDGET.get(case, {}).get(rank)
    if budget is not None:
        os.environ["PLSSVM_MI_MEM_BUDGET"] = budget
    prm, kp_mode, imax = make_case(case)
    svm = pm.CSVM(prm, device=0, rank=rank, world_size=world, kp_mode=kp_mode, exchange=pm.torch_exchange(dist),
                  sparse_algo=ALGO.get(case, "auto"))
    svm.setup_data_on_device()
    q = svm.generate_q()
    m = svm.m
    x = np.random.default_rng(21).uniform(1, 2, m).astype(svm.dtype)
    kp_minus = svm.run_device_kernel(None, np.zeros(m, svm.dtype), x, -1.0).copy()
    kp_plus = svm.run_device_kernel(None, np.zeros(m, svm.dtype), x, 1.0).copy()
    kpart = svm.kp_part(x, "kernel")
    svm.learn(imax=imax)
    info = svm.info()
    np.savez(os.path.join(out, f"rank{rank}.npz"), q=q, kp_minus=kp_minus, kp_plus=kp_plus, kpart=kpart,
             alpha=svm.alpha, bias=np.float64(svm.bias), trace=np.asarray(svm.trace), iters=svm.iters,
             QA=np.float64(svm.QA_cost), tiles_local=info["tiles_local"], tiles_total=info["tiles_total"],
             pairs=info["pairs"], world=info["world_size"], sparse_algo=info["sparse_algo"],
             exp_hbytes=info["exp_hbytes"])
    svm.close()
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
