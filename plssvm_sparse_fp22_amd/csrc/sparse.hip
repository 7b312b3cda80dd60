// Sparse (CSR / CSC / packed FP22) K·p paths — see sparse.hpp.
#include "engine.hpp"

namespace plssvm_mi {

template <typename T>
void launch_q_sparse(kfun<T>, const csr_data<T> &, int64_t, const T *, T *, hipStream_t) {
    throw mi_error(-5, "sparse q not built yet");
}

template <typename T>
void engine<T>::sparse_kp_raw(const T *, const cg_scalars<T> *) {
    throw mi_error(-5, "sparse K·p not built yet");
}

template <typename T>
void engine<T>::sparse_dominant(const T *) {
    throw mi_error(-5, "sparse K·p not built yet");
}

template <typename T>
int64_t engine<T>::csr_bytes() const {
    return 0;
}

template void launch_q_sparse<float>(kfun<float>, const csr_data<float> &, int64_t, const float *, float *, hipStream_t);
template void launch_q_sparse<double>(kfun<double>, const csr_data<double> &, int64_t, const double *, double *,
                                      hipStream_t);
#define INST(T)                                                                 \
    template void engine<T>::sparse_kp_raw(const T *, const cg_scalars<T> *);   \
    template void engine<T>::sparse_dominant(const T *);                        \
    template int64_t engine<T>::csr_bytes() const;
INST(float)
INST(double)
#undef INST

}  // namespace plssvm_mi
