// ofdm_engine.hpp -- host-side helpers shared by the cpuLS.hpp / gpuLS.hpp
// mirrors: device buffers, host<->device staging and fail-loudly wrappers
// around the C ABI (include/ofdm_lsmrc.h).  Every computation goes to the GPU
// library; there is no CPU implementation of the receiver behind these
// headers.
#ifndef OFDM_ENGINE_HPP_
#define OFDM_ENGINE_HPP_

#include <hip/hip_runtime_api.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ofdm_lsmrc.h"

namespace ofdm {

[[noreturn]] inline void die(const char *what, const char *detail) {
    std::fprintf(stderr, "ofdm: %s failed: %s\n", what, detail);
    std::abort();
}
inline void check(int rc, const char *what) {
    if (rc < 0) die(what, ofdm_last_error());
}
inline void hcheck(hipError_t e, const char *what) {
    if (e != hipSuccess) die(what, hipGetErrorString(e));
}

// growable device buffer
struct DevBuf {
    void *p = nullptr;
    size_t n = 0;
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    // a buffer used as a frame workspace is dropped from the library's
    // estimate registry before its memory goes back (ofdm_workspace_release)
    ~DevBuf() {
        if (p) {
            (void)ofdm_workspace_release(p);
            (void)hipFree(p);
        }
    }
    template <typename T = void>
    T *get(size_t bytes) {
        if (bytes > n) {
            if (p) {
                (void)ofdm_workspace_release(p);
                hcheck(hipFree(p), "hipFree");
            }
            hcheck(hipMalloc(&p, bytes), "hipMalloc");
            n = bytes;
        }
        return static_cast<T *>(p);
    }
};

inline bool is_device_ptr(const void *p) {
    hipPointerAttribute_t a;
    if (hipPointerGetAttributes(&a, p) != hipSuccess) {
        (void)hipGetLastError();  // plain host memory: clear the sticky error
        return false;
    }
    return a.type == hipMemoryTypeDevice;
}

// copy between any two of {host, device} buffers
inline void copy_any(void *dst, const void *src, size_t bytes, hipStream_t s = nullptr) {
    hcheck(hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s), "hipMemcpyAsync");
    hcheck(hipStreamSynchronize(s), "hipStreamSynchronize");
}

// Staging engine for host-pointer APIs (cpuLS.hpp): one instance per process.
class HostEngine {
  public:
    static HostEngine &get() {
        static HostEngine e;
        return e;
    }
    hipStream_t stream() const { return s_; }

    // rows of C samples, in place, forward (inverse != 0: backward)
    void fft_rows(void *rows_host, int nrows, int C, int inverse = 0) {
        const size_t b = (size_t)nrows * C * sizeof(ofdm_cf32);
        auto *d = a_.get<ofdm_cf32>(b);
        up(d, rows_host, b);
        check(ofdm_fft_rows(d, d, nrows, C, inverse, s_), "ofdm_fft_rows");
        down(rows_host, d, b);
    }
    // LS from an R x C frequency-domain pilot symbol
    void ls(const void *Y, const void *X, int R, int C, void *Hconj, float *P) {
        const int K = C - 1;
        auto *dY = a_.get<ofdm_cf32>((size_t)R * C * 8);
        auto *dX = b_.get<ofdm_cf32>((size_t)K * 8);
        auto *dH = c_.get<ofdm_cf32>((size_t)R * K * 8);
        auto *dP = d_.get<float>((size_t)K * 4);
        up(dY, Y, (size_t)R * C * 8);
        up(dX, X, (size_t)K * 8);
        check(ofdm_ls_estimate(dY, dX, R, C, dH, dP, s_), "ofdm_ls_estimate");
        down(Hconj, dH, (size_t)R * K * 8);
        down(P, dP, (size_t)K * 4);
    }
    // MRC of one R x C frequency-domain symbol -> K rotated outputs
    void mrc(const void *Y, const void *Hconj, const float *P, int R, int C, void *out) {
        const int K = C - 1;
        auto *dY = a_.get<ofdm_cf32>((size_t)R * C * 8);
        auto *dH = c_.get<ofdm_cf32>((size_t)R * K * 8);
        auto *dP = d_.get<float>((size_t)K * 4);
        auto *dO = b_.get<ofdm_cf32>((size_t)K * 8);
        up(dY, Y, (size_t)R * C * 8);
        up(dH, Hconj, (size_t)R * K * 8);
        up(dP, P, (size_t)K * 4);
        check(ofdm_mrc_demod(dY, 1, dH, dP, R, C, dO, s_), "ofdm_mrc_demod");
        down(out, dO, (size_t)K * 8);
    }
    // sum_r Y[r][j] Hconj[r][j] for an R x K matrix Y (DC already dropped)
    void numerator(const void *Yk, const void *Hconj, int R, int K, void *out) {
        const int C = K + 1;
        auto *dY = a_.get<ofdm_cf32>((size_t)R * C * 8);
        auto *dH = c_.get<ofdm_cf32>((size_t)R * K * 8);
        auto *dO = b_.get<ofdm_cf32>((size_t)K * 8);
        put_with_dc(dY, Yk, R, K);
        up(dH, Hconj, (size_t)R * K * 8);
        check(ofdm_mrc_numerator(dY, 1, dH, R, C, dO, s_), "ofdm_mrc_numerator");
        down(out, dO, (size_t)K * 8);
    }
    void dist_sqrd(const void *H, int R, int K, float *P) {
        auto *dH = c_.get<ofdm_cf32>((size_t)R * K * 8);
        auto *dP = d_.get<float>((size_t)K * 4);
        up(dH, H, (size_t)R * K * 8);
        check(ofdm_dist_sqrd(dH, R, K, dP, s_), "ofdm_dist_sqrd");
        down(P, dP, (size_t)K * 4);
    }
    void shift(void *row, int K) {
        auto *dI = a_.get<ofdm_cf32>((size_t)K * 8);
        auto *dO = b_.get<ofdm_cf32>((size_t)K * 8);
        up(dI, row, (size_t)K * 8);
        check(ofdm_shift_rows(dI, 1, K, dO, s_), "ofdm_shift_rows");
        down(row, dO, (size_t)K * 8);
    }
    // A[j] = A[j] / B[j] (divideOneRow's naive formula) for K = C - 1 values:
    // conj(conj(A) / conj(B)) through the LS kernel, which computes conj(y/x).
    void divide(void *A, const void *B, int K) {
        std::vector<ofdm_cf32> a(K), b(K);
        std::memcpy(a.data(), A, (size_t)K * 8);
        std::memcpy(b.data(), B, (size_t)K * 8);
        for (int j = 0; j < K; ++j) { a[j].im = -a[j].im; b[j].im = -b[j].im; }
        const int C = K + 1;
        auto *dY = a_.get<ofdm_cf32>((size_t)C * 8);
        auto *dX = b_.get<ofdm_cf32>((size_t)K * 8);
        auto *dH = c_.get<ofdm_cf32>((size_t)K * 8);
        auto *dP = d_.get<float>((size_t)K * 4);
        put_with_dc(dY, a.data(), 1, K);
        up(dX, b.data(), (size_t)K * 8);
        check(ofdm_ls_estimate(dY, dX, 1, C, dH, dP, s_), "ofdm_ls_estimate");
        down(A, dH, (size_t)K * 8);
    }

    // zero-forcing matrix of a U x R x K channel cube -> W [K][U][R] (host)
    void zf_precoder(const void *Hin, int U, int R, int K, void *W) {
        const size_t b = (size_t)U * R * K * 8;
        auto *dH = a_.get<ofdm_cf32>(b);
        auto *dW = c_.get<ofdm_cf32>(b);
        up(dH, Hin, b);
        check(ofdm_zf_precoder(dH, U, R, K, dW, nullptr, s_), "ofdm_zf_precoder");
        down(W, dW, b);
    }
    // one symbol: Y[r][k] = sum_u W[k][u][r] X[u][k]  (W in the reference layout)
    void zf_apply(const void *W, const void *X, int U, int R, int K, void *Y) {
        const size_t bw = (size_t)U * R * K * 8;
        auto *dW = a_.get<ofdm_cf32>(bw);
        auto *dWt = c_.get<ofdm_cf32>(bw);
        auto *dX = b_.get<ofdm_cf32>((size_t)U * K * 8);
        auto *dY = d_.get<ofdm_cf32>((size_t)R * K * 8);
        up(dW, W, bw);
        up(dX, X, (size_t)U * K * 8);
        check(ofdm_zf_transpose(dW, U, R, K, dWt, s_), "ofdm_zf_transpose");
        check(ofdm_zf_apply(dWt, dX, U, R, K, 1, dY, s_), "ofdm_zf_apply");
        down(Y, dY, (size_t)R * K * 8);
    }

  private:
    HostEngine() { hcheck(hipStreamCreate(&s_), "hipStreamCreate"); }
    void up(void *d, const void *h, size_t b) {
        hcheck(hipMemcpyAsync(d, h, b, hipMemcpyHostToDevice, s_), "hipMemcpyAsync H2D");
    }
    void down(void *h, const void *d, size_t b) {
        hcheck(hipMemcpyAsync(h, d, b, hipMemcpyDeviceToHost, s_), "hipMemcpyAsync D2H");
        hcheck(hipStreamSynchronize(s_), "hipStreamSynchronize");
    }
    // R rows of K values -> R rows of C = K + 1 bins with an empty DC bin
    void put_with_dc(ofdm_cf32 *d, const void *h, int R, int K) {
        hcheck(hipMemsetAsync(d, 0, (size_t)R * (K + 1) * 8, s_), "hipMemsetAsync");
        hcheck(hipMemcpy2DAsync(d + 1, (size_t)(K + 1) * 8, h, (size_t)K * 8, (size_t)K * 8, R,
                                hipMemcpyHostToDevice, s_),
               "hipMemcpy2DAsync");
    }
    hipStream_t s_ = nullptr;
    DevBuf a_, b_, c_, d_;
};

}  // namespace ofdm

#endif  // OFDM_ENGINE_HPP_
