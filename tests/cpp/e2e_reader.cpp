// e2e_reader.cpp -- slave/reader side of the end-to-end test: one of the
// reference's receiver flows, written like its drivers (cpuLS_main.cpp:57-106,
// gpuLS_main.cu:66-145), against this package's headers.
//   cpuls   firstVector + doOneSymbol x (S-1)          -> Output_cpu.dat
//   symbol  gpuLS firstVector + demodOneSymbol x (S-1)  -> Output_gpu.dat
//   frame   gpuLS demodOneFrame                          -> Output_gpu.dat
// Run in a directory holding Pilots.dat.
#include <cstdio>
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

static int run_gpuls(bool frame) {
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
    if (frame) {
        // host staging for lenOfBuffer symbols (gpuLS.cu:484-491)
        std::vector<hipFloatComplex> dY((size_t)rows * cols * lenOfBuffer);
        g.demodOneFrame(dY.data(), Y, dX, dH, Hsqrd, rows, cols);
        out.write(reinterpret_cast<const char *>(dY.data()),
                  (std::streamsize)sizeof(hipFloatComplex) * K * (lenOfBuffer - 1));
    } else {
        // host staging buffer as gpuLS_main.cu:73-74 allocates it
        std::vector<hipFloatComplex> dY((size_t)rows * (cols + prefix));
        g.firstVector(dY.data(), Y, dH, dX, Hsqrd, rows, cols, 0);
        for (int i = 1; i < numberOfSymbolsToTest; i++) {
            g.demodOneSymbol(dY.data(), Y, dH, Hsqrd, rows, cols, i);
            out.write(reinterpret_cast<const char *>(dY.data()), (std::streamsize)sizeof(hipFloatComplex) * K);
        }
    }
    (void)hipFree(Y); (void)hipFree(dH); (void)hipFree(dX); (void)hipFree(Hsqrd);
    return 0;
}

int main(int argc, char **argv) {
    const std::string m = argc > 1 ? argv[1] : "cpuls";
    if (m == "cpuls") return run_cpuls();
    if (m == "symbol") return run_gpuls(false);
    if (m == "frame") return run_gpuls(true);
    return 2;
}
