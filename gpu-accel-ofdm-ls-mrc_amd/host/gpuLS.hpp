// gpuLS.hpp -- the reference's GPU receiver class on MI355X.
//
// Drop-in for class gpuLS (gpuLS.cuh:72-113, gpuLS.cu:44-858): same class
// name, members (buffPtr, devProp), method names, argument order and pointer
// ownership (the caller allocates every device buffer, as gpuLS_main.cu:73-91
// does), with the CUDA types replaced by their HIP equivalents
// (cuFloatComplex -> hipFloatComplex, cudaStream_t -> hipStream_t,
// cudaDeviceProp -> hipDeviceProp_t).  Header-only because, as in the
// reference, the ring geometry (numOfRows, dimension, prefix, lenOfBuffer) is
// fixed per driver at compile time.
//
// Every method runs on the HIP library (include/ofdm_lsmrc.h); kernels pick
// their own launch geometry, so the dim3 arguments of the per-stage methods
// only carry the symbol count where the reference derives it from the grid
// (ShiftOneRow / CombineForMRC: gridDim.y rows).  Intended semantics replace
// the reference's defects: FFT plans are not rebuilt per
// symbol, scratch is not allocated per call, findHs never reads the next
// row, combineForMRC is race-free and in order, the cuBLAS variant computes
// |H|^2 (not |H|) and sum Y conj(H) (not sum Y H), and errors abort with a
// message instead of passing silently.
#ifndef OFDM_GPULS_HPP_
#define OFDM_GPULS_HPP_

// system and HIP headers first: the reference's configuration macros
// (prefix, dimension, ...) are plain identifiers
#include <hip/hip_complex.h>
#include <hip/hip_runtime_api.h>

#include <cstring>
#include <string>
#include <vector>

#include "ofdm_engine.hpp"
#include "ShMemSymBuff_gpu.hpp"  // as gpuLS.cuh:35

#define FFT_size dimension
#define cp_size prefix
#define numSymbols lenOfBuffer
#define threadsPerBlock FFT_size
#define numOfBlocks numOfRows
#ifndef fileNameForX
#define fileNameForX "Pilots.dat"
#endif

class gpuLS {
  public:
    ShMemSymBuff *buffPtr;
    hipDeviceProp_t devProp;

    // opens the ring as a slave (gpuLS.cu:44-48)
    gpuLS() {
        buffPtr = new ShMemSymBuff(shmemID, 0);
        int dev = 0;
        ofdm::hcheck(hipGetDevice(&dev), "hipGetDevice");
        ofdm::hcheck(hipGetDeviceProperties(&devProp, dev), "hipGetDeviceProperties");
    }
    ~gpuLS() {
        if (pipe_) (void)ofdm_pipeline_destroy(pipe_);
        delete buffPtr;
    }

    // K pilots from Pilots.dat, rotated; 1 + 1i if missing (gpuLS.cu:53-86)
    void matrix_readX(hipFloatComplex *X, int cols) {
        if (ofdm_read_pilots(fileNameForX, cols, 1.0f, reinterpret_cast<ofdm_cf32 *>(X)) == 1)
            std::cerr << "Unable to open file " << fileNameForX << ", filling in 1+i for x\n";
    }

    // dX (device, rows x (cols-1)) = the pilots replicated per antenna (gpuLS.cu:88-106)
    void copyPilotToGPU(hipFloatComplex *dX, int rows, int cols) {
        const int K = cols - 1;
        std::vector<hipFloatComplex> X((size_t)rows * K);
        for (int i = 0; i < rows; i++) matrix_readX(&X[(size_t)i * K], K);
        ofdm::copy_any(dX, X.data(), X.size() * sizeof(hipFloatComplex));
    }

    // output rotation of host row `row` (gpuLS.cu:127-141)
    void shiftOneRowCPU(hipFloatComplex *Y, int cols, int row) {
        hipFloatComplex *y = &Y[(size_t)row * cols];
        std::vector<hipFloatComplex> t(y, y + cols);
        const int h = (cols - 1) / 2, h1 = (cols + 1) / 2;
        for (int k = 0; k < h1; ++k) y[k] = t[k + h];
        for (int k = h1; k < cols; ++k) y[k] = t[k - h1];
    }

    // ---- per-stage methods (gpuLS.cu:261-293) ----------------------------
    // rotate gridDim.y device rows of cols1 values in place
    void ShiftOneRow(hipFloatComplex *Y, int cols1, int rows1, dim3 blockDim, dim3 gridDim,
                     hipStream_t *stream) {
        (void)rows1; (void)blockDim;
        const long long n = gridDim.y;
        auto *tmp = scratch_.get<ofdm_cf32>((size_t)n * cols1 * sizeof(ofdm_cf32));
        ofdm::check(ofdm_shift_rows(C(Y), n, cols1, tmp, S(stream)), "ofdm_shift_rows");
        ofdm::hcheck(hipMemcpyAsync(Y, tmp, (size_t)n * cols1 * 8, hipMemcpyDeviceToDevice, HS(stream)),
                     "hipMemcpyAsync");
    }
    // Y (rows x cols) = dY (rows x (cols+prefix)) without the cyclic prefix
    void DropPrefix(hipFloatComplex *Y, hipFloatComplex *dY, int rows1, int cols1, dim3 blockDim,
                    dim3 gridDim, hipStream_t *stream) {
        (void)blockDim; (void)gridDim;
        ofdm::hcheck(hipMemcpy2DAsync(Y, (size_t)cols1 * 8, dY + prefix, (size_t)(cols1 + prefix) * 8,
                                      (size_t)cols1 * 8, rows1, hipMemcpyDeviceToDevice, HS(stream)),
                     "hipMemcpy2DAsync");
    }
    // dH (rows x (cols-1)) = conj(dY[r][j+1] / dX[r][j])  (findHs, gpuLS.cu:158-182)
    void FindLeastSquaresGPU(hipFloatComplex *dY, hipFloatComplex *dH, hipFloatComplex *dX, int rows1,
                             int cols1, dim3 blockDim, dim3 gridDim, hipStream_t *stream) {
        (void)blockDim; (void)gridDim;
        auto *p = scratchP_.get<float>((size_t)cols1 * 4);
        ofdm::check(ofdm_ls_estimate(C(dY), C(dX), rows1, cols1, C(dH), p, S(stream)), "ofdm_ls_estimate");
    }
    // Hsqrd (cols1 floats) = sum_r |H[r][j]|^2  (findDistSqrd, gpuLS.cu:185-209)
    void FindHsqrdforMRC(hipFloatComplex *H, float *Hsqrd, int rows1, int cols1, dim3 blockDim,
                         dim3 gridDim, hipStream_t *stream) {
        (void)blockDim; (void)gridDim;
        ofdm::check(ofdm_dist_sqrd(C(H), rows1, cols1, Hsqrd, S(stream)), "ofdm_dist_sqrd");
    }
    // Yf[s][r][j] = Y[s][r][j+1] * Hconj[r][j]  (multiplyWithChannelConj, gpuLS.cu:212-233)
    void MultiplyWithChannelConj(hipFloatComplex *Y, hipFloatComplex *Hconj, hipFloatComplex *Yf,
                                 int rows1, int cols1, int syms1, dim3 blockDim, dim3 gridDim,
                                 hipStream_t *stream) {
        (void)blockDim; (void)gridDim;
        ofdm::check(ofdm_channel_conj_product(C(Y), syms1, C(Hconj), rows1, cols1, C(Yf), S(stream)),
                    "ofdm_channel_conj_product");
    }
    // Y[s][j] = sum_r Y[s][r][j] / Hsqrd[j] for gridDim.y symbols, written over
    // the head of Y (combineForMRC, gpuLS.cu:236-259; not rotated)
    void CombineForMRC(hipFloatComplex *Y, float *Hsqrd, int rows1, int cols1, dim3 blockDim,
                       dim3 gridDim, hipStream_t *stream) {
        (void)blockDim;
        const long long n = gridDim.y;
        auto *tmp = scratch_.get<ofdm_cf32>((size_t)n * cols1 * 8);
        ofdm::check(ofdm_combine_products(C(Y), n, Hsqrd, rows1, cols1, 0, tmp, S(stream)),
                    "ofdm_combine_products");
        ofdm::hcheck(hipMemcpyAsync(Y, tmp, (size_t)n * cols1 * 8, hipMemcpyDeviceToDevice, HS(stream)),
                     "hipMemcpyAsync");
    }
    // forward C2C FFT of `rows` device rows of `cols`, in place (gpuLS.cu:343-349)
    void batchedFFT(hipFloatComplex *Y, int rows, int cols, hipStream_t *stream) {
        ofdm::check(ofdm_fft_rows(C(Y), C(Y), rows, cols, 0, S(stream)), "ofdm_fft_rows");
    }

    // ---- per-symbol flow (gpuLS.cu:351-473) ------------------------------
    // Pilot symbol from the ring into dY (host or device staging buffer);
    // dH = conj(Y/X) (rows x (cols-1), device), Hsqrd = |H|^2 (cols-1).
    // C in {1024, 2048, 4096}: ONE fused FFT + LS launch straight from the
    // staging buffer (prefix skipped in the kernel) into this object's
    // workspace, then its export into dH / Hsqrd, one sync; the workspace
    // estimate is kept for demodOneSymbol.  Other C: FFT rows in Y, then LS.
    void firstVector(hipFloatComplex *dY, hipFloatComplex *Y, hipFloatComplex *dH,
                     hipFloatComplex *dX, float *Hsqrd, int rows, int cols, int it) {
        int pfx = 0;
        const hipFloatComplex *src = read_symbol(dY, Y, rows, cols, it, false, fused(cols) ? &pfx : nullptr);
        clock_t t0 = clock();
        est_H_ = nullptr;
        est_P_ = nullptr;
        if (fused(cols)) {
            const size_t wsb = ofdm_frame_workspace_bytes(1, 2, rows, cols);
            void *ws = ws1_.get(wsb);
            ofdm::check(ofdm_frame_estimate(C(src), 1, 2, rows, cols, pfx, C(dX), ws, wsb, nullptr),
                        "ofdm_frame_estimate");
            ofdm::check(ofdm_frame_export_estimate(ws, wsb, 1, 2, rows, cols, 0, C(dH), Hsqrd, nullptr),
                        "ofdm_frame_export_estimate");
            sync();
            buffPtr->setFft(0.f, it);  // fused into the LS kernel
            buffPtr->setDecode(secs(t0), it);
            est_H_ = dH;
            est_P_ = Hsqrd;
            est_rows_ = rows;
            est_cols_ = cols;
            est_wsb_ = wsb;
            est_hash_ = estimate_hash(dH, Hsqrd, rows, cols);
            return;
        }
        batchedFFT(Y, rows, cols, nullptr);
        sync();
        buffPtr->setFft(secs(t0), it);
        t0 = clock();
        ofdm::check(ofdm_ls_estimate(C(Y), C(dX), rows, cols, C(dH), Hsqrd, nullptr), "ofdm_ls_estimate");
        sync();
        buffPtr->setDecode(secs(t0), it);
    }
    // Data symbol `it` from the ring; K rotated outputs land in dY[0..K)
    // (host or device), as gpuLS_main.cu:112-117 expects.  When Hconj /
    // Hsqrd are the buffers the last firstVector filled (the reference's
    // call sequence, gpuLS_main.cu:107-112) and C is fused: ONE fused FFT +
    // MRC + normalise + rotate launch (ofdm_symbols_demod) on the staging
    // buffer against the kept estimate, one synchronising copy of the K
    // outputs.  Otherwise FFT rows in Y, then MRC from Hconj / Hsqrd.
    // The fused path demodulates against the workspace copy of the estimate
    // firstVector exported, so it is taken only while Hconj / Hsqrd still
    // hold exactly those bytes: their device hash (ofdm_buffer_hash, one
    // small kernel + an 16-B read-back per symbol) must equal the one taken
    // at export.  A caller that edits them in place after firstVector
    // (smoothing, interpolation, another estimate copied in) -- as reference
    // callers may, without telling anyone -- therefore gets the reference's
    // behaviour, Hconj / Hsqrd read afresh (gpuLS.cu:410-473).
    // estimateChanged() drops the kept estimate outright.
    void estimateChanged() {
        est_H_ = nullptr;
        est_P_ = nullptr;
    }
    void demodOneSymbol(hipFloatComplex *dY, hipFloatComplex *Y, hipFloatComplex *Hconj,
                        float *Hsqrd, int rows1, int cols1, int it) {
        const int K = cols1 - 1;
        const bool use_est = fused(cols1) && Hconj == est_H_ && Hsqrd == est_P_ && rows1 == est_rows_ &&
                             cols1 == est_cols_ && estimate_hash(Hconj, Hsqrd, rows1, cols1) == est_hash_;
        int pfx = 0;
        const hipFloatComplex *src = read_symbol(dY, Y, rows1, cols1, it, it == numberOfSymbolsToTest - 1,
                                                 use_est ? &pfx : nullptr);
        clock_t t0 = clock();
        auto *out = scratch_.get<ofdm_cf32>((size_t)K * 8);
        if (use_est) {
            ofdm::check(ofdm_symbols_demod(C(src), 1, rows1, cols1, pfx, ws1_.p, est_wsb_, 0, out, nullptr),
                        "ofdm_symbols_demod");
            ofdm::copy_any(dY, out, (size_t)K * 8);
            buffPtr->setFft(0.f, it);  // fused into the MRC kernel
            buffPtr->setDecode(secs(t0), it);
            return;
        }
        batchedFFT(Y, rows1, cols1, nullptr);
        sync();
        buffPtr->setFft(secs(t0), it);
        t0 = clock();
        ofdm::check(ofdm_mrc_demod(C(Y), 1, C(Hconj), Hsqrd, rows1, cols1, out, nullptr), "ofdm_mrc_demod");
        ofdm::copy_any(dY, out, (size_t)K * 8);
        buffPtr->setDecode(secs(t0), it);
    }

    // ---- frame flow (gpuLS.cu:475-858) -----------------------------------
    // lenOfBuffer symbols from the ring into dY (host), then as demodOneFrameCUDA
    void demodOneFrame(hipFloatComplex *dY, hipFloatComplex *Y, hipFloatComplex *dX,
                       hipFloatComplex *Hconj, float *Hsqrd, int rows1, int cols1) {
        const size_t sym = (size_t)rows1 * cols1;
        for (int it = 0; it < numberOfSymbolsToTest; it++) {
            if (it == numberOfSymbolsToTest - 1)
                buffPtr->readLastSymbol(&dY[sym * it]);
            else
                buffPtr->readNextSymbol(&dY[sym * it], it);
        }
        clock_t t0 = clock();
        ofdm::copy_any(Y, dY, sym * lenOfBuffer * sizeof(hipFloatComplex));
        buffPtr->setReadT(secs(t0), 1);
        demodOneFrameCUDA(dY, Y, dX, Hconj, Hsqrd, rows1, cols1);
    }
    // Y (device): one frame of lenOfBuffer time-domain symbols, pilot first.
    // One pass of the fused receiver (ofdm_frame_estimate + ofdm_frame_combine:
    // FFT + LS, then FFT + MRC + normalise + rotate, each row read once) in
    // place of the reference's cuFFT + findHs + findDistSqrd +
    // multiplyWithChannelConj + combineForMRC + shiftOneRow chain
    // (gpuLS.cu:599-662).  Outputs as the reference leaves them: the
    // (lenOfBuffer-1) x (cols1-1) rotated symbols in dY (host or device),
    // the LS estimate in Hconj (rows1 x (cols1-1), device) and |H|^2 in
    // Hsqrd (cols1-1, device).  Unlike the reference, Y is left in the time
    // domain (the transform never goes back to memory).
    void demodOneFrameCUDA(hipFloatComplex *dY, hipFloatComplex *Y, hipFloatComplex *dX,
                           hipFloatComplex *Hconj, float *Hsqrd, int rows1, int cols1) {
        const int K = cols1 - 1;
        const size_t wsb = ofdm_frame_workspace_bytes(1, lenOfBuffer, rows1, cols1);
        void *ws = ws_.get(wsb);
        auto *out = scratch_.get<ofdm_cf32>((size_t)K * (lenOfBuffer - 1) * 8);
        clock_t t0 = clock();
        ofdm::check(ofdm_frame_estimate(C(Y), 1, lenOfBuffer, rows1, cols1, 0, C(dX), ws, wsb, nullptr),
                    "ofdm_frame_estimate");
        ofdm::check(ofdm_frame_export_estimate(ws, wsb, 1, lenOfBuffer, rows1, cols1, 0, C(Hconj), Hsqrd,
                                               nullptr),
                    "ofdm_frame_export_estimate");
        sync();
        buffPtr->setFft(0.f, 1);  // fused into the LS / MRC kernels
        buffPtr->setDecode(secs(t0), 0);
        t0 = clock();
        ofdm::check(ofdm_frame_combine(C(Y), 1, lenOfBuffer, rows1, cols1, 0, ws, wsb, out, nullptr),
                    "ofdm_frame_combine");
        ofdm::copy_any(dY, out, (size_t)K * (lenOfBuffer - 1) * 8);
        buffPtr->setDecode(secs(t0), 1);
    }
    // demodOptimized / demodCuBlas compute the same frame result
    // (gpuLS.cu:677-858; their launch-shape and cuBLAS variations are moot here)
    void demodOptimized(hipFloatComplex *dY, hipFloatComplex *Y, hipFloatComplex *dX,
                        hipFloatComplex *Hconj, float *Hsqrd, int rows1, int cols1) {
        demodOneFrameCUDA(dY, Y, dX, Hconj, Hsqrd, rows1, cols1);
    }
    void demodCuBlas(hipFloatComplex *dY, hipFloatComplex *Y, hipFloatComplex *dX,
                     hipFloatComplex *Hconj, float *Hsqrd, int rows1, int cols1) {
        demodOneFrameCUDA(dY, Y, dX, Hconj, Hsqrd, rows1, cols1);
    }

    // ---- streaming frames (the batched demod entry next to
    // demodOneFrameCUDA; 8(f) rank 2: line-rate ingest) --------------------
    // Reads nframes frames of lenOfBuffer symbols from the ring with the
    // pipelined bulk reader (ShMemSymBuff::readSymbolsCUDA) straight into the
    // device slots of an ofdm_pipeline: while chunk i streams in over PCIe,
    // chunk i-1 is demodulated and chunk i-2's outputs stream out.  out (host
    // or device; page-locked host memory for full overlap) receives
    // nframes x (lenOfBuffer-1) x (cols1-1) rotated outputs, frames in order.
    // dX: the pilots as copyPilotToGPU fills them (the first cols1-1 values).
    // last: the run ends with these frames (readLastSymbol semantics for the
    // final symbol).
    void demodFrames(hipFloatComplex *out, int nframes, hipFloatComplex *dX, int rows1, int cols1,
                     bool last = true, int framesPerChunk = 4, int depth = 3) {
        const int K = cols1 - 1;
        if (!pipe_ || pipeChunk_ != framesPerChunk || pipeDepth_ != depth || pipeX_ != dX) {
            if (pipe_) ofdm::check(ofdm_pipeline_destroy(pipe_), "ofdm_pipeline_destroy");
            pipe_ = nullptr;
            ofdm::check(ofdm_pipeline_create(lenOfBuffer, rows1, cols1, prefix, C(dX), framesPerChunk,
                                             depth, &pipe_),
                        "ofdm_pipeline_create");
            pipeChunk_ = framesPerChunk;
            pipeDepth_ = depth;
            pipeX_ = dX;
        }
        for (int f0 = 0; f0 < nframes; f0 += framesPerChunk) {
            const int n = nframes - f0 < framesPerChunk ? nframes - f0 : framesPerChunk;
            ofdm_cf32 *d = nullptr;
            ofdm_stream_t cs = nullptr;
            ofdm::check(ofdm_pipeline_acquire(pipe_, &d, &cs), "ofdm_pipeline_acquire");
            buffPtr->readSymbolsCUDA(d, n * lenOfBuffer, reinterpret_cast<hipStream_t>(cs),
                                     last && f0 + n == nframes);
            ofdm::check(ofdm_pipeline_submit(pipe_, n, C(out + (size_t)f0 * (lenOfBuffer - 1) * K)),
                        "ofdm_pipeline_submit");
        }
        ofdm::check(ofdm_pipeline_sync(pipe_), "ofdm_pipeline_sync");
    }

  private:
    ofdm_pipeline *pipe_ = nullptr;
    int pipeChunk_ = 0, pipeDepth_ = 0;
    const hipFloatComplex *pipeX_ = nullptr;

    static ofdm_cf32 *C(hipFloatComplex *p) { return reinterpret_cast<ofdm_cf32 *>(p); }
    static const ofdm_cf32 *C(const hipFloatComplex *p) {
        return reinterpret_cast<const ofdm_cf32 *>(p);
    }
    static ofdm_stream_t S(hipStream_t *s) { return s ? *s : nullptr; }
    static hipStream_t HS(hipStream_t *s) { return s ? *s : nullptr; }
    static float secs(clock_t t0) { return (float)(clock() - t0) / (float)CLOCKS_PER_SEC; }
    static void sync() { ofdm::hcheck(hipDeviceSynchronize(), "hipDeviceSynchronize"); }

    static bool fused(int cols) { return cols == 1024 || cols == 2048 || cols == 4096; }

    // ring -> staging buffer dY (host: plain read; device: *CUDA read) -> Y;
    // the cyclic prefix is dropped on the way.  Returns the device symbol to
    // compute on: with pfx non-null and a device dY, dY itself (no copy to Y;
    // *pfx = prefix, skipped by the fused kernel), else Y (*pfx = 0).
    const hipFloatComplex *read_symbol(hipFloatComplex *dY, hipFloatComplex *Y, int rows, int cols, int it,
                                       bool last, int *pfx = nullptr) {
        const size_t bytes = (size_t)rows * cols * sizeof(hipFloatComplex);
        clock_t t0 = clock();
        if (pfx) *pfx = 0;
        if (ofdm::is_device_ptr(dY)) {
            if (last)
                buffPtr->readLastSymbolCUDA(dY);
            else
                buffPtr->readNextSymbolCUDA(dY, it);
            if (pfx) {
                *pfx = prefix;
                buffPtr->setReadT(secs(t0), it);
                return dY;
            }
            if (prefix > 0)
                ofdm::hcheck(hipMemcpy2D(Y, (size_t)cols * 8, dY + prefix, (size_t)(cols + prefix) * 8,
                                         (size_t)cols * 8, rows, hipMemcpyDeviceToDevice),
                             "hipMemcpy2D");
            else
                ofdm::copy_any(Y, dY, bytes);
        } else {
            if (last)
                buffPtr->readLastSymbol(dY);
            else
                buffPtr->readNextSymbol(dY, it);
            ofdm::copy_any(Y, dY, bytes);
        }
        buffPtr->setReadT(secs(t0), it);
        return Y;
    }

    // hash of the caller's Hconj [rows][cols-1] and Hsqrd [cols-1] (device)
    struct EstHash {
        unsigned long long h, p;
        bool operator==(const EstHash &o) const { return h == o.h && p == o.p; }
    };
    EstHash estimate_hash(const hipFloatComplex *H, const float *P, int rows, int cols) {
        auto *d = hash_.get<unsigned long long>(2 * sizeof(unsigned long long));
        const size_t K = (size_t)cols - 1;
        ofdm::check(ofdm_buffer_hash(H, (size_t)rows * K * sizeof(hipFloatComplex), d, nullptr), "ofdm_buffer_hash");
        ofdm::check(ofdm_buffer_hash(P, K * sizeof(float), d + 1, nullptr), "ofdm_buffer_hash");
        EstHash e;
        ofdm::copy_any(&e, d, sizeof(e));
        return e;
    }
    ofdm::DevBuf scratch_, scratchP_, ws_, ws1_, hash_;
    EstHash est_hash_{0, 0};
    // the estimate firstVector keeps in ws1_ and the buffers it exported to
    const hipFloatComplex *est_H_ = nullptr;
    const float *est_P_ = nullptr;
    int est_rows_ = 0, est_cols_ = 0;
    size_t est_wsb_ = 0;
};

#endif  // OFDM_GPULS_HPP_
