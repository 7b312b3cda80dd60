// RAII device buffer for the MI355X PLSSVM backend.
#pragma once

#include "common.hpp"

namespace plssvm_mi {

// RAII device buffer (the reference's move-only device_ptr, src/plssvm/backends/gpu_device_ptr.cpp:58-109,
// without its per-call hipSetDevice/synchronous copies: all traffic is async on the engine stream)
template <typename T>
class dev_buf {
  public:
    dev_buf() = default;
    dev_buf(const dev_buf &) = delete;
    dev_buf &operator=(const dev_buf &) = delete;
    dev_buf(dev_buf &&o) noexcept : p_(o.p_), n_(o.n_) { o.p_ = nullptr, o.n_ = 0; }
    dev_buf &operator=(dev_buf &&o) noexcept {
        if (this != &o) {
            reset();
            p_ = o.p_;
            n_ = o.n_;
            o.p_ = nullptr;
            o.n_ = 0;
        }
        return *this;
    }
    ~dev_buf() { reset(); }
    void alloc(int64_t n, hipStream_t s, bool zero = true) {
        reset();
        if (n <= 0) return;
        MI_HIP_CHECK(hipMalloc(&p_, sizeof(T) * (size_t) n));
        n_ = n;
        if (zero) MI_HIP_CHECK(hipMemsetAsync(p_, 0, sizeof(T) * (size_t) n, s));
    }
    void reset() {
        if (p_) (void) hipFree(p_);
        p_ = nullptr;
        n_ = 0;
    }
    T *get() const { return p_; }
    int64_t size() const { return n_; }
    int64_t bytes() const { return n_ * (int64_t) sizeof(T); }

  private:
    T *p_ = nullptr;
    int64_t n_ = 0;
};

}  // namespace plssvm_mi
