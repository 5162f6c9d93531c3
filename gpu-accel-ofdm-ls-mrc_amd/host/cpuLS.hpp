// cpuLS.hpp -- the reference's host-pointer receiver API, run on MI355X.
//
// Drop-in for the RX part of the reference's cpuLS.hpp (cpuLS.hpp:55-389):
// same global names (buffPtr, file, outfile, numTimes, the per-phase timing
// arrays, buffIter), same free functions and signatures, same buffer
// ownership (the caller allocates Y [rows x cols], Hconj [rows x (cols-1)],
// X [cols-1], which firstVector turns into |H|^2 in X[j].real), same output
// file (Output_cpu.dat: K rotated complex floats appended per data symbol,
// truncated on the first one).  Behind each call the data is staged to the
// GPU and computed by the HIP library -- there is no host implementation of
// the FFT, LS or MRC arithmetic here.
//
// Intended semantics are implemented where the reference's code defeats
// them:
//   * firstVector reads the pilot (symbol 0) from the ring, as
//     gpuLS::firstVector does; the reference zeroes Y instead and every output
//     becomes NaN (cpuLS.hpp:251-272);
//   * a missing Pilots.dat fills 0.707 + 0.707i, as cpuLS.hpp:84-90 does;
//   * the FFT plan is not rebuilt per row and doOneSymbol does not leak.
// The multi-user zero-forcing helpers (rotCube, createZeroForcingMatrix,
// multiplyWithChannelInv; cpuLS.hpp:400-463) are provided, computed by the
// library's ZF kernels.  The remaining TX-side
// helpers (ifftShiftOneRow, addPrefix, modRefSymbol, modOneSymbol;
// cpuLS.hpp:119-132, 391-398, 466-529) are not part of the receiver path and
// are not provided.
#ifndef _CPULS_HPP_
#define _CPULS_HPP_

#include <algorithm>
#include <csignal>
#include <cmath>
#include <cstdlib>
#include <ctime>
#include <fstream>
#include <string>

#include <vector>

#include "ofdm_engine.hpp"  // before the ring: its config macros are plain identifiers
#include "CSharedMemSimple.hpp"
#include "ShMemSymBuff_cucomplex.hpp"  // as cpuLS.hpp:34; a ring header included first wins

#define fileNameForX "Pilots.dat"
#ifndef mode
#define mode 1
#endif

using namespace std;

// ---- globals of the reference (cpuLS.hpp:61-66); outfile, numTimes, the
// timing arrays, buffIter and printTimes/storeTimes come with the ring header
// (ShMemSymBuff.hpp:62-191) --------------------------------------------------
inline ShMemSymBuff *buffPtr = nullptr;
inline string file = "Output_cpu.dat";
inline string in_file = "Input_cpu.dat";
inline int num_syms = 0;

namespace ofdm_cpuls {
inline clock_t tic() { return timerEn ? clock() : 0; }
inline void toc(float *arr, int it, clock_t t0) {
    if (timerEn && it >= 0 && it < numberOfSymbolsToTest)
        arr[it] += (float)(clock() - t0) / (float)CLOCKS_PER_SEC;
}
}  // namespace ofdm_cpuls

// matrix_readX (cpuLS.hpp:80-117): K pilots from Pilots.dat, rotated
inline void matrix_readX(complexF *X, int cols) {
    if (ofdm_read_pilots(fileNameForX, cols, 0.707f, reinterpret_cast<ofdm_cf32 *>(X)) == 1)
        std::cerr << "Unable to open file data file, filling in 1+i for x\n";
}

// shiftOneRow (cpuLS.hpp:135-149): output rotation of row `row`
inline void shiftOneRow(complexF *Y, int cols, int row) {
    ofdm::HostEngine::get().shift(&Y[(size_t)row * cols], cols);
}

// fftOneRow / ifftOneRow (cpuLS.hpp:152-174): unnormalised C2C of row `row`
inline void fftOneRow(complexF *Y, int cols, int row) {
    ofdm::HostEngine::get().fft_rows(&Y[(size_t)row * cols], 1, cols, 0);
}
inline void ifftOneRow(complexF *Y, int cols, int row) {
    ofdm::HostEngine::get().fft_rows(&Y[(size_t)row * cols], 1, cols, 1);
}

// numSyms (cpuLS.hpp:176-184): symbols of cols-1 samples in a file
inline void numSyms(std::string in_file1, int cols) {
    std::ifstream f(in_file1.c_str(), std::ifstream::binary | std::ifstream::ate);
    const size_t n = f ? (size_t)f.tellg() / sizeof(complexF) : 0;
    num_syms = (int)std::ceil((float)n / (float)(cols - 1));
}

// matrixMultThenSum (cpuLS.hpp:187-208): Yf[j] = sum_r Y[r][j] * Hconj[r][j],
// Y and Hconj rows x (cols-1)
inline void matrixMultThenSum(complexF *Y, complexF *Hconj, complexF *Yf, int rows, int cols) {
    ofdm::HostEngine::get().numerator(Y, Hconj, rows, cols - 1, Yf);
}

// findDistSqrd (cpuLS.hpp:211-228): Hsqrd[j] = {sum_r |H[r][j]|^2, 0}
inline void findDistSqrd(complexF *H, complexF *Hsqrd, int rows, int cols) {
    std::vector<float> p((size_t)cols);
    ofdm::HostEngine::get().dist_sqrd(H, rows, cols, p.data());
    for (int j = 0; j < cols; j++) Hsqrd[j] = complexF{p[j], 0.f};
}

// divideOneRow (cpuLS.hpp:233-244): A[row][j] /= B[j]
inline void divideOneRow(complexF *A, complexF *B, int cols, int row) {
    ofdm::HostEngine::get().divide(&A[(size_t)row * cols], B, cols);
}

// firstVector (cpuLS.hpp:247-317): pilots, then the pilot symbol from the
// ring -> Hconj (rows x (cols-1)) and |H|^2 in X[j].real (X[j].imag = 0).
inline void firstVector(complexF *Y, complexF *Hconj, complexF *X, int rows, int cols,
                        int iter = 0) {
    const int K = cols - 1;
    matrix_readX(X, K);
    if (iter < numberOfSymbolsToTest - 1)
        buffPtr->readNextSymbol(Y, iter);
    else
        buffPtr->readLastSymbol(Y);
    auto &e = ofdm::HostEngine::get();
    clock_t t0 = ofdm_cpuls::tic();
    e.fft_rows(Y, rows, cols, 0);
    ofdm_cpuls::toc(fft, iter, t0);
    t0 = ofdm_cpuls::tic();
    std::vector<float> p((size_t)K);
    e.ls(Y, X, rows, cols, Hconj, p.data());
    for (int j = 0; j < K; j++) X[j] = complexF{p[j], 0.f};
    ofdm_cpuls::toc(decode, iter, t0);
}

// doOneSymbol (cpuLS.hpp:319-389): data symbol `it` from the ring -> K
// rotated MRC outputs appended to Output_cpu.dat (truncated when it <= 1).
inline void doOneSymbol(complexF *Y, complexF *Hconj, complexF *Hsqrd, int rows, int cols, int it) {
    const int K = cols - 1;
    if (it == numberOfSymbolsToTest - 1)
        buffPtr->readLastSymbol(Y);
    else
        buffPtr->readNextSymbol(Y, it);
    auto &e = ofdm::HostEngine::get();
    clock_t t0 = ofdm_cpuls::tic();
    e.fft_rows(Y, rows, cols, 0);
    ofdm_cpuls::toc(fft, it, t0);
    t0 = ofdm_cpuls::tic();
    std::vector<float> p((size_t)K);
    for (int j = 0; j < K; j++) p[j] = Hsqrd[j].real;
    std::vector<complexF> Yf((size_t)K);
    e.mrc(Y, Hconj, p.data(), rows, cols, Yf.data());
    ofdm_cpuls::toc(decode, it, t0);
    outfile.open(file.c_str(), it <= 1 ? (std::ofstream::binary | std::ofstream::trunc)
                                       : (std::ofstream::binary | std::ofstream::app));
    outfile.write(reinterpret_cast<const char *>(Yf.data()), (std::streamsize)K * sizeof(complexF));
    outfile.close();
}

// rotCube (cpuLS.hpp:400-413): X[user][row][col] -> X[col][row][user], in
// place (a layout permutation, no arithmetic).
inline void rotCube(complexF *X, int rows, int cols, int users) {
    std::vector<complexF> t((size_t)rows * cols * users);
    for (int col = 0; col < cols; col++)
        for (int row = 0; row < rows; row++)
            for (int user = 0; user < users; user++)
                t[((size_t)col * rows + row) * users + user] = X[((size_t)user * rows + row) * cols + col];
    std::memcpy(X, t.data(), t.size() * sizeof(complexF));
}

// createZeroForcingMatrix (cpuLS.hpp:415-447): X is the users x rows x K
// channel cube (K = max(1, cols-1)); H receives, per subcarrier, the rows x
// users matrix A^H (A A^H)^-1, column-major (H[k*rows*users + u*rows + r]).
// As in the reference, X is left rotated (rotCube) on return.  The
// reference's debug print of the first six rotated values (431-434) is
// omitted.
inline void createZeroForcingMatrix(complexF *H, complexF *X, int rows, int cols, int users) {
    const int K = std::max(1, cols - 1);
    ofdm::HostEngine::get().zf_precoder(X, users, rows, K, H);
    rotCube(X, rows, K, users);
}

// multiplyWithChannelInv (cpuLS.hpp:449-463): for each subcarrier i < cols-1,
// HX[r*(cols-1) + i] = sum_u H[i*rows*users + u*rows + r] X[u*(cols-1) + i].
inline void multiplyWithChannelInv(complexF *HX, complexF *X, complexF *H, int rows, int cols,
                                   int users) {
    ofdm::HostEngine::get().zf_apply(H, X, users, rows, cols - 1, HX);
}

#endif  // _CPULS_HPP_
