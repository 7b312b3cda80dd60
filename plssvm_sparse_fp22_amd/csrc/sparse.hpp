// Sparse (CSR / CSC / packed-FP22) device data for the MI355X PLSSVM backend.
// Build-defined formats: the reference has no sparse device path.
#pragma once

#include "kernels.hpp"

namespace plssvm_mi {

template <typename T>
class dev_buf;

template <typename T>
struct csr_data {
    int64_t nnz = 0;
    int val_fmt = 0;  // PLSSVM_MI_VAL_REAL | PLSSVM_MI_VAL_FP22
};

template <typename T>
void launch_q_sparse(kfun<T> kf, const csr_data<T> &csr, int64_t m, const T *xlast, T *q, hipStream_t s);

}  // namespace plssvm_mi
