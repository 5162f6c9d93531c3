// e2e_reader.cpp -- slave/reader side of the end-to-end test: one of the
// reference's receiver flows, written like its drivers (cpuLS_main.cpp:57-106,
// gpuLS_main.cu:66-145), against this package's headers.
//   cpuls   firstVector + doOneSymbol x (S-1)          -> Output_cpu.dat
//   symbol  gpuLS firstVector + demodOneSymbol x (S-1)  -> Output_gpu.dat
//   frame   gpuLS demodOneFrame                          -> Output_gpu.dat
//   symbolcuda  as symbol, with a device staging buffer (readNextSymbolCUDA)
//   symboledit  as symbol, the caller doubling Hsqrd in place after firstVector
//           (no estimateChanged(): the outputs must follow the edit, x 1/2)
//   frames N [chunk depth]  gpuLS demodFrames: N frames through the pipelined
//           ring reader and ofdm_pipeline (page-locked output) -> Output_gpu.dat,
//           and the ingest rate on stdout
// Run in a directory holding Pilots.dat.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#include "cpuLS.hpp"
#include "gpuLS.hpp"

static int run_cpuls() {
    const int rows = numOfRows, cols = dimension;
    std::vector<complexF> Y((size_t)rows * cols), Hconj((size_t)rows * (cols - 1)), X(cols - 1);
    buffPtr = new ShMemSymBuff(shmemID, 0);
    firstVector(Y.data(), Hconj.data(), X.data(), rows, cols);
    for (int i = 1; i < numberOfSymbolsToTest; i++) {
        doOneSymbol(Y.data(), Hconj.data(), X.data(), rows, cols, i);
        buffIter = i;
    }
    delete buffPtr;
    buffPtr = nullptr;
    return 0;
}

static int run_gpuls(bool frame, bool dev_staging, bool edit = false) {
    const int rows = numOfRows, cols = dimension, K = cols - 1;
    gpuLS g;
    hipFloatComplex *Y, *dH, *dX;
    float *Hsqrd;
    ofdm::hcheck(hipMalloc(&Y, sizeof(hipFloatComplex) * rows * cols * lenOfBuffer), "hipMalloc");
    ofdm::hcheck(hipMalloc(&dH, sizeof(hipFloatComplex) * rows * K), "hipMalloc");
    ofdm::hcheck(hipMalloc(&dX, sizeof(hipFloatComplex) * rows * K), "hipMalloc");
    ofdm::hcheck(hipMalloc(&Hsqrd, sizeof(float) * K), "hipMalloc");
    g.copyPilotToGPU(dX, rows, cols);
    std::ofstream out("Output_gpu.dat", std::ofstream::binary | std::ofstream::trunc);
    const auto t0 = std::chrono::steady_clock::now();
    if (frame) {
        // host staging for lenOfBuffer symbols (gpuLS.cu:484-491)
        std::vector<hipFloatComplex> dY((size_t)rows * cols * lenOfBuffer);
        g.demodOneFrame(dY.data(), Y, dX, dH, Hsqrd, rows, cols);
        out.write(reinterpret_cast<const char *>(dY.data()),
                  (std::streamsize)sizeof(hipFloatComplex) * K * (lenOfBuffer - 1));
    } else {
        // host staging buffer as gpuLS_main.cu:73-74 allocates it, or a
        // device one (the readNextSymbolCUDA path, gpuLS.cu:359)
        std::vector<hipFloatComplex> hY((size_t)rows * (cols + prefix)), o(K);
        hipFloatComplex *dY = hY.data();
        if (dev_staging) ofdm::hcheck(hipMalloc(&dY, hY.size() * sizeof(hipFloatComplex)), "hipMalloc");
        g.firstVector(dY, Y, dH, dX, Hsqrd, rows, cols, 0);
        if (edit) {  // a caller's in-place edit of the estimate, without estimateChanged(): Hsqrd x 2
            std::vector<float> p(K);
            ofdm::copy_any(p.data(), Hsqrd, p.size() * sizeof(float));
            for (float &v : p) v *= 2.f;
            ofdm::copy_any(Hsqrd, p.data(), p.size() * sizeof(float));
        }
        for (int i = 1; i < numberOfSymbolsToTest; i++) {
            g.demodOneSymbol(dY, Y, dH, Hsqrd, rows, cols, i);
            ofdm::copy_any(o.data(), dY, (size_t)K * sizeof(hipFloatComplex));
            out.write(reinterpret_cast<const char *>(o.data()), (std::streamsize)sizeof(hipFloatComplex) * K);
        }
        if (dev_staging) (void)hipFree(dY);
    }
    const double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    // the estimate the flow leaves in Hconj / Hsqrd (firstVector, demodOneFrameCUDA)
    std::vector<hipFloatComplex> h((size_t)rows * K);
    std::vector<float> p(K);
    ofdm::copy_any(h.data(), dH, h.size() * sizeof(hipFloatComplex));
    ofdm::copy_any(p.data(), Hsqrd, p.size() * sizeof(float));
    std::ofstream("Hconj_gpu.dat", std::ofstream::binary)
        .write(reinterpret_cast<const char *>(h.data()), (std::streamsize)(h.size() * sizeof(hipFloatComplex)));
    std::ofstream("Hsqrd_gpu.dat", std::ofstream::binary)
        .write(reinterpret_cast<const char *>(p.data()), (std::streamsize)(p.size() * sizeof(float)));
    std::printf("{\"frames\": 1, \"seconds\": %.6f, \"data_symbols_per_s\": %.1f}\n", sec,
                (lenOfBuffer - 1) / sec);
    (void)hipFree(Y); (void)hipFree(dH); (void)hipFree(dX); (void)hipFree(Hsqrd);
    return 0;
}

static int run_frames(int nframes, int chunk, int depth) {
    const int rows = numOfRows, cols = dimension, K = cols - 1;
    gpuLS g;
    hipFloatComplex *dX;
    ofdm::hcheck(hipMalloc(&dX, sizeof(hipFloatComplex) * rows * K), "hipMalloc");
    g.copyPilotToGPU(dX, rows, cols);
    const size_t n_out = (size_t)nframes * (lenOfBuffer - 1) * K;
    hipFloatComplex *out;
    ofdm::hcheck(hipHostMalloc(&out, n_out * sizeof(hipFloatComplex), hipHostMallocDefault), "hipHostMalloc");
    const auto t0 = std::chrono::steady_clock::now();
    g.demodFrames(out, nframes, dX, rows, cols, true, chunk, depth);
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    const double in_bytes = (double)nframes * lenOfBuffer * rows * (cols + prefix) * 8.0;
    std::printf("{\"frames\": %d, \"seconds\": %.6f, \"data_symbols_per_s\": %.1f, "
                "\"ingest_GBps\": %.3f}\n",
                nframes, s, nframes * (lenOfBuffer - 1) / s, in_bytes / s / 1e9);
    std::ofstream f("Output_gpu.dat", std::ofstream::binary | std::ofstream::trunc);
    f.write(reinterpret_cast<const char *>(out), (std::streamsize)(n_out * sizeof(hipFloatComplex)));
    (void)hipHostFree(out);
    (void)hipFree(dX);
    return 0;
}

int main(int argc, char **argv) {
    const std::string m = argc > 1 ? argv[1] : "cpuls";
    if (m == "cpuls") return run_cpuls();
    if (m == "symbol") return run_gpuls(false, false);
    if (m == "symbolcuda") return run_gpuls(false, true);
    if (m == "symboledit") return run_gpuls(false, false, true);
    if (m == "frame") return run_gpuls(true, false);
    if (m == "frames" && argc > 2)
        return run_frames(std::atoi(argv[2]), argc > 3 ? std::atoi(argv[3]) : 4,
                          argc > 4 ? std::atoi(argv[4]) : 3);
    return 2;
}
