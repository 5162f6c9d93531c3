// ShMemSymBuff_impl.hpp -- shared-memory ring of OFDM symbols between the
// radio front-end process (writer, master) and the receiver (reader, slave).
// Included through one of the three public headers, which mirror the
// reference's three ring headers and their default configuration:
//   ShMemSymBuff.hpp           numOfRows 16, lenOfBuffer 10   (ShMemSymBuff.hpp:42-72)
//   ShMemSymBuff_cucomplex.hpp numOfRows 1,  lenOfBuffer 117  (ShMemSymBuff_cucomplex.hpp:48-83)
//   ShMemSymBuff_gpu.hpp       numOfRows 16, lenOfBuffer 101  (ShMemSymBuff_gpu.hpp:48-80)
// As in the reference the three share the include guard _SHMEMSYMBUFF_HPP_:
// the first one a translation unit includes fixes the ring geometry.
//
// Same shared-memory wire format (struct symbolBuffer, ShMemSymBuff_gpu.hpp:89-103
// -- writer and reader built from either header interoperate), same globals
// (outfile, numTimes, readT/decode/drop/fft, buffIter, printTimes/storeTimes:
// ShMemSymBuff.hpp:62-191), same class and method names and the same
// reader/writer protocol (ShMemSymBuff_gpu.hpp:265-503):
//   * the master initialises {size = lenOfBuffer, readPtr = 0, writePtr = -1};
//     a slave spins until size > 0; a slave's destructor sets size = -1;
//   * readNextSymbol waits for data, copies the slot (dropping the cyclic
//     prefix), then advances readPtr only once the writer has moved past the
//     next slot -- the reader stays one slot behind; readLastSymbol advances
//     without that wait and ends a run;
//   * writeNextSymbolNoWait overwrites without looking at the reader;
//     writeNextSymbolWithWait waits for the reader.
// Differences, all correctness fixes that leave call sites unchanged:
//   * ring indices are accessed with acquire/release atomics (the reference's
//     plain int busy-waits are compiled away at -O2);
//   * the master publishes readPtr/writePtr before size;
//   * writeNextSymbolWithWait's wrap-around waits for readPtr != 0 (the
//     plain variant, ShMemSymBuff.hpp:451) instead of readPtr >= 0 (never
//     true again, ShMemSymBuff_gpu.hpp:471);
//   * the *CUDA readers (kept under their reference names for drop-in use)
//     copy with hipMemcpyAsync and wait for the copy before releasing the
//     slot, so the writer can no longer overwrite a slot in flight; the shm
//     segment is page-locked (hipHostRegister) on first device read;
//   * the master's destructor always unmaps/unlinks once (the reference
//     loops on delete while size == -1); the slave frees its handle too.
// Device-side methods are compiled when HIP is available (hipcc, or
// -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include with a host compiler).
#ifndef OFDM_SHMEMSYMBUFF_IMPL_HPP_
#define OFDM_SHMEMSYMBUFF_IMPL_HPP_

#include <cstddef>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <fstream>
#include <iostream>
#include <string>
#include <vector>

#include "CSharedMemSimple.hpp"

#if defined(__HIPCC__) || defined(__HIP_PLATFORM_AMD__)
#define OFDM_RING_HIP 1
#include <hip/hip_runtime_api.h>
#endif

// ---- configuration (names as the reference; defaults set by the public
// header that included this one, each overridable with -D) ----------------
#if !defined(numOfRows) || !defined(lenOfBuffer)
#error "include ShMemSymBuff.hpp, ShMemSymBuff_cucomplex.hpp or ShMemSymBuff_gpu.hpp"
#endif
#ifndef numUsers
#define numUsers 4
#endif
#ifndef dimension
#define dimension 1024
#endif
#ifndef prefix
#define prefix 0
#endif
#ifndef timerEnabled
#define timerEnabled true
#endif
#ifndef testEnabled
#define testEnabled true
#endif
#define numberOfSymbolsToTest lenOfBuffer
#ifndef shmemID
#define shmemID "/blah"
#endif
#define PL printf("Line #: %d \n", __LINE__);
#define timerEn timerEnabled
#define testEn testEnabled

// ---- wire format --------------------------------------------------------
struct complexF {
    float real;
    float imag;
};

struct symbol {  // one time slot: numOfRows antenna rows of dimension+prefix samples
    complexF data[numOfRows * (dimension + prefix)];
};

struct symbolBuffer {
    int size;      // symbols in the ring (master), -1 once the slave detached
    int readPtr;   // slot the reader is on
    int writePtr;  // next slot the writer fills, -1 before the first write
    symbol symbols[lenOfBuffer];
};
static_assert(offsetof(symbolBuffer, symbols) == 12, "symbolBuffer wire layout");

// ---- globals and timing helpers (ShMemSymBuff.hpp:62-191) ---------------
inline std::ofstream outfile;
inline int numTimes = 1;  // runs of the receiver loop (cpuLS_main.cpp:80)
inline float readT[numberOfSymbolsToTest];
inline float decode[numberOfSymbolsToTest];  // [0]: channel estimate
inline float drop[numberOfSymbolsToTest];
inline float fft[numberOfSymbolsToTest];
inline int buffIter = 0;

inline void printOutArr(complexF *a, int rows, int cols) {
    for (int i = 0; i < rows; i++) {
        for (int j = 0; j < cols; j++)
            std::cout << "(" << a[i * cols + j].real << ", " << a[i * cols + j].imag << "), ";
        std::printf("\n");
    }
}
inline void printInfo() {
    std::printf("\tSymbol Dimension(w/o prefix) = %d x %d \n", numOfRows, dimension);
    std::printf("\tPrefix = %d\n", prefix);
    std::printf("\t# Of Symbols To Test = %d\n", numberOfSymbolsToTest);
}
// {real = mean, imag = population variance} of times[0..amt)
inline complexF findAvgAndVar(float *times, int amt) {
    float mean = 0.f, var = 0.f;
    for (int i = 0; i < amt; i++) mean += times[i];
    mean /= amt;
    for (int i = 0; i < amt; i++) var += (times[i] - mean) * (times[i] - mean);
    return complexF{mean, var / amt};
}
// per-phase averages over the run (ShMemSymBuff.hpp:149-164)
inline void printTimes(bool cpu) {
    complexF rd = findAvgAndVar(readT, numberOfSymbolsToTest);
    complexF dec = findAvgAndVar(&decode[1], numberOfSymbolsToTest - 1);
    complexF ff = findAvgAndVar(fft, numberOfSymbolsToTest);
    std::printf("\t \t Avg Time(s) \t Variance (s^2) \n");
    std::printf("Read: \t \t %e \t %e \n", rd.real / numTimes, rd.imag / numTimes);
    std::printf("ChanEst: \t %e \n", decode[0] / numTimes);
    std::printf("Decode: \t %e \t %e \n", dec.real / numTimes, dec.imag / numTimes);
    std::printf("FFT: \t \t %e \t %e \n", ff.real / numTimes, ff.imag / numTimes);
    if (cpu) {
        complexF dr = findAvgAndVar(drop, numberOfSymbolsToTest);
        std::printf("Drop: \t \t %e \t %e \n", dr.real / numTimes, dr.imag / numTimes);
    }
}
// time_{cpu,gpu}.dat: mean read, channel estimate, decode, fft, drop (5
// floats; ShMemSymBuff.hpp:166-189)
inline void storeTimes(bool cpu) {
    complexF rd = findAvgAndVar(readT, numberOfSymbolsToTest);
    complexF dec = findAvgAndVar(&decode[1], numberOfSymbolsToTest - 1);
    complexF ff = findAvgAndVar(fft, numberOfSymbolsToTest);
    complexF dr = findAvgAndVar(drop, numberOfSymbolsToTest);
    const float v[5] = {rd.real / numTimes, decode[0] / numTimes, dec.real / numTimes,
                        ff.real / numTimes, dr.real / numTimes};
    std::ofstream out(cpu ? "time_cpu.dat" : "time_gpu.dat", std::ofstream::binary);
    out.write(reinterpret_cast<const char *>(v), sizeof v);
}

namespace ofdm_ring {
inline int load(const int *p) { return __atomic_load_n(p, __ATOMIC_ACQUIRE); }
inline void store(int *p, int v) { __atomic_store_n(p, v, __ATOMIC_RELEASE); }
inline void relax() {
#if defined(__x86_64__) || defined(__i386__)
    __builtin_ia32_pause();
#endif
}
}  // namespace ofdm_ring

class ShMemSymBuff {
  public:
    // isMaster == 1: create and initialise the ring; otherwise wait for it.
    ShMemSymBuff(std::string shm_uid, int isMaster) {
        shm_ = new CSharedMemSimple(shm_uid, sizeof(struct symbolBuffer));
        buff_ = static_cast<symbolBuffer *>(shm_->ptr());
        master_ = (isMaster == 1);
        if (master_) {
            shm_->set_master_mode();
            ofdm_ring::store(&buff_->readPtr, 0);
            ofdm_ring::store(&buff_->writePtr, -1);
            ofdm_ring::store(&buff_->size, lenOfBuffer);
        } else {
            while (ofdm_ring::load(&buff_->size) <= 0) ofdm_ring::relax();
        }
    }

    ~ShMemSymBuff() {
#ifdef OFDM_RING_HIP
        for (int i = 0; i < lenOfBuffer; ++i) {
            if (streams_[i]) (void)hipStreamDestroy(streams_[i]);
            if (events_[i]) (void)hipEventDestroy(events_[i]);
        }
        if (io_stream_) (void)hipStreamDestroy(io_stream_);
        if (registered_) (void)hipHostUnregister(buff_);
#endif
        if (!master_) ofdm_ring::store(&buff_->size, -1);  // tell the writer we left
        delete shm_;  // a slave's segment object only unmaps nothing (reference semantics)
    }

    ShMemSymBuff(const ShMemSymBuff &) = delete;
    ShMemSymBuff &operator=(const ShMemSymBuff &) = delete;

    void info() { shm_->info(); }
    void setBuffLen(int size_) { ofdm_ring::store(&buff_->size, size_); }

    // ---- timing (ShMemSymBuff_gpu.hpp:157-257) ---------------------------
    void setReadT(float value, int iter) { readT[iter] = value; }
    void setFft(float value, int iter) { fft[iter] = value; }
    void setDecode(float value, int iter) { decode[iter] = value; }
    void setDrop(float value, int iter) { drop[iter] = value; }

    void printOutArr(complexF *a, int rows, int cols) { ::printOutArr(a, rows, cols); }
    void printInfo() { ::printInfo(); }
    complexF findAvgAndVar(float *times, int amt) { return ::findAvgAndVar(times, amt); }
    // the _gpu variant's member forms (ShMemSymBuff_gpu.hpp:190-257)
    void printTimes(bool cpu) {
        complexF rd = findAvgAndVar(readT, numberOfSymbolsToTest);
        complexF dec = findAvgAndVar(&decode[1], numberOfSymbolsToTest - 1);
        complexF ff = findAvgAndVar(&fft[1], numberOfSymbolsToTest - 1);
        std::printf("\t \t Avg Time(s) \t Variance (s^2) \n");
        std::printf("R/W: \t \t %e \t %e \n", rd.real, rd.imag);
        std::printf("ChanEst: \t %e \n", decode[0] + ff.real + rd.real);
        std::printf("Mod/Demod: \t %e \t %e \n", dec.real, dec.imag);
        std::printf("FFT: \t \t %e \t %e \n", ff.real, ff.imag);
        std::printf("Frame: \t \t %e \n", (ff.real + rd.real + dec.real) * (lenOfBuffer - 1));
        if (cpu) {
            complexF dr = findAvgAndVar(drop, numberOfSymbolsToTest);
            std::printf("Drop: \t \t %e \t %e \n", dr.real, dr.imag);
        }
    }
    // time_{cpu,gpu}.dat: mean read, channel-estimate, decode, fft, drop (5 floats)
    void storeTimes(bool cpu) {
        complexF rd = findAvgAndVar(readT, numberOfSymbolsToTest);
        complexF dec = findAvgAndVar(&decode[1], numberOfSymbolsToTest - 1);
        complexF ff = findAvgAndVar(fft, numberOfSymbolsToTest - 1);
        complexF dr = findAvgAndVar(drop, numberOfSymbolsToTest);
        std::ofstream out(cpu ? "time_cpu.dat" : "time_gpu.dat", std::ofstream::binary);
        const float v[5] = {rd.real, decode[0], dec.real, ff.real, dr.real};
        out.write(reinterpret_cast<const char *>(v), sizeof v);
    }

    // ---- reader (ShMemSymBuff_gpu.hpp:263-360) ---------------------------
    template <typename T>
    void readNextSymbol(T *Y, int it) {
        const int r = wait_readable();
        tic();
        copy_drop_prefix(Y, r);
        toc(readT, it);
        advance_reader(r, /*last=*/false);
    }

    template <typename T>
    void readLastSymbol(T *Y) {
        const int r = wait_readable();
        copy_drop_prefix(Y, r);
        advance_reader(r, /*last=*/true);
    }

#ifdef OFDM_RING_HIP
    // ---- reader into device memory (ShMemSymBuff_gpu.hpp:364-447) --------
    // Copies the whole slot (cyclic prefix included, as the reference does:
    // the receiver drops it on the device) on streams[it].
    hipStream_t *createStream(int it) {
        if (!streams_[it]) (void)hipStreamCreate(&streams_[it]);
        return &streams_[it];
    }
    void destroyStream(int it) {
        if (streams_[it]) (void)hipStreamDestroy(streams_[it]);
        streams_[it] = nullptr;
    }

    template <typename T>
    void readNextSymbolCUDA(T *dY, int it) {
        const int r = wait_readable();
        tic();
        copy_to_device(dY, r, io_stream());
        toc(readT, it);
        advance_reader(r, /*last=*/false);
    }

    template <typename T>
    void readLastSymbolCUDA(T *dY) {
        const int r = wait_readable();
        tic();
        copy_to_device(dY, r, io_stream());
        toc(readT, numberOfSymbolsToTest - 1);
        advance_reader(r, /*last=*/true);
    }

    // Bulk, pipelined form of readNextSymbolCUDA (no reference counterpart;
    // SURVEY.md 8(f) rank 2): the next n symbols (whole slots, cyclic prefix
    // included) are copied to dY + i * numOfRows * (dimension + prefix) on
    // stream s as soon as the writer has filled them, without waiting for
    // earlier copies.  The ring protocol is unchanged: readPtr only moves
    // past a slot once that slot's copy has completed (so a WithWait writer
    // never overwrites a slot in flight) and, as in readNextSymbol, only
    // onto a slot the writer has already filled; the run's final symbol is
    // released like readLastSymbol when `last` is set.  Returns once every
    // slot of the run has been copied and released.
    template <typename T>
    void readSymbolsCUDA(T *dY, int n, hipStream_t s, bool last = false) {
        static_assert(sizeof(T) == sizeof(complexF), "8-byte complex samples");
        if (n <= 0) return;
        register_ring();
        if (!events_[0])
            for (auto &e : events_)
                if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) fail_copy();
        const size_t bytes = kSymbolElems * sizeof(T);
        while (ofdm_ring::load(&buff_->writePtr) == -1) ofdm_ring::relax();
        int rp = ofdm_ring::load(&buff_->readPtr);  // slot of run index `released`
        int issued = 0, released = 0;
        while (released < n) {
            bool progress = false;
            // issue every filled slot ahead of the reader (at most lenOfBuffer - 1 in flight)
            const int w = ofdm_ring::load(&buff_->writePtr);
            const int filled = (w - rp + lenOfBuffer) % lenOfBuffer;  // slots [rp, w)
            while (issued < n && issued - released < filled) {
                const int slot = (rp + issued - released) % lenOfBuffer;
                if (hipMemcpyAsync(reinterpret_cast<char *>(dY) + (size_t)issued * bytes,
                                   buff_->symbols[slot].data, bytes, hipMemcpyHostToDevice,
                                   s) != hipSuccess ||
                    hipEventRecord(events_[issued % lenOfBuffer], s) != hipSuccess)
                    fail_copy();
                ++issued;
                progress = true;
            }
            // release completed copies in order
            while (released < issued) {
                const hipError_t q = hipEventQuery(events_[released % lenOfBuffer]);
                if (q == hipErrorNotReady) break;
                if (q != hipSuccess) fail_copy();
                const int p = (rp + 1) % lenOfBuffer;
                const bool final_ = last && released == n - 1;
                if (!final_ && ofdm_ring::load(&buff_->writePtr) == p) break;  // stay one behind
                ofdm_ring::store(&buff_->readPtr, p);
                rp = p;
                ++released;
                progress = true;
            }
            if (!progress) ofdm_ring::relax();
        }
    }
#endif

    // ---- writer (ShMemSymBuff_gpu.hpp:447-503) ---------------------------
    template <typename T>
    void writeNextSymbolWithWait(T *Yf) {
        int w = ofdm_ring::load(&buff_->writePtr);
        if (w == -1) {
            put(0, Yf);
            ofdm_ring::store(&buff_->writePtr, 1);
            return;
        }
        // do not write the slot the reader is on
        while (w == ofdm_ring::load(&buff_->readPtr)) ofdm_ring::relax();
        put(w, Yf);
        const int p = w + 1;
        while (ofdm_ring::load(&buff_->readPtr) == p) ofdm_ring::relax();
        if (p >= lenOfBuffer) {
            while (ofdm_ring::load(&buff_->readPtr) == 0) ofdm_ring::relax();
            ofdm_ring::store(&buff_->writePtr, 0);
        } else {
            ofdm_ring::store(&buff_->writePtr, p);
        }
    }

    template <typename T>
    void writeNextSymbolNoWait(T *Yf) {
        const int w = ofdm_ring::load(&buff_->writePtr);
        if (w == -1) {
            put(0, Yf);
            ofdm_ring::store(&buff_->writePtr, 1);
            return;
        }
        put(w, Yf);
        const int p = w + 1;
        ofdm_ring::store(&buff_->writePtr, p >= lenOfBuffer ? 0 : p);
    }

  private:
    static constexpr size_t kRowIn = dimension + prefix;
    static constexpr size_t kSymbolElems = (size_t)numOfRows * kRowIn;

    int wait_readable() {
        while (ofdm_ring::load(&buff_->writePtr) == -1) ofdm_ring::relax();
        int r;
        while ((r = ofdm_ring::load(&buff_->readPtr)) == ofdm_ring::load(&buff_->writePtr))
            ofdm_ring::relax();
        return r;
    }

    // the reader stays one slot behind the writer unless this is the last read
    void advance_reader(int r, bool last) {
        const int p = r + 1;
        if (!last)
            while (ofdm_ring::load(&buff_->writePtr) == p) ofdm_ring::relax();
        if (p >= lenOfBuffer) {
            if (!last)
                while (ofdm_ring::load(&buff_->writePtr) == 0) ofdm_ring::relax();
            ofdm_ring::store(&buff_->readPtr, 0);
        } else {
            ofdm_ring::store(&buff_->readPtr, p);
        }
    }

    template <typename T>
    void copy_drop_prefix(T *Y, int slot) {
        static_assert(sizeof(T) == sizeof(complexF), "8-byte complex samples");
        const complexF *s = buff_->symbols[slot].data;
        if (prefix > 0) {
            tic();
            for (int i = 0; i < numOfRows; ++i)
                std::memcpy(reinterpret_cast<char *>(Y) + (size_t)i * dimension * sizeof(T),
                            s + (size_t)i * kRowIn + prefix, (size_t)dimension * sizeof(T));
            toc(drop, current_it_);
        } else {
            std::memcpy(Y, s, kSymbolElems * sizeof(T));
        }
    }

    template <typename T>
    void put(int slot, const T *Yf) {
        static_assert(sizeof(T) == sizeof(complexF), "8-byte complex samples");
        std::memcpy(buff_->symbols[slot].data, Yf, kSymbolElems * sizeof(T));
    }

#ifdef OFDM_RING_HIP
    template <typename T>
    void copy_to_device(T *dY, int slot, hipStream_t s) {
        static_assert(sizeof(T) == sizeof(complexF), "8-byte complex samples");
        register_ring();
        const size_t bytes = kSymbolElems * sizeof(T);
        if (hipMemcpyAsync(dY, buff_->symbols[slot].data, bytes, hipMemcpyHostToDevice, s) !=
                hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            fail_copy();
    }
    // The per-symbol readers copy on ONE stream of this object, created once
    // (the reference creates a stream per symbol index and never destroys it,
    // ShMemSymBuff_gpu.hpp:375-447; each creation costs far more than the
    // 512 KiB copy).  createStream / destroyStream stay for callers.
    hipStream_t io_stream() {
        if (!io_stream_ && hipStreamCreateWithFlags(&io_stream_, hipStreamNonBlocking) != hipSuccess) fail_copy();
        return io_stream_;
    }
    // page-lock the ring once: true async DMA from shm
    void register_ring() {
        if (!registered_)
            registered_ = hipHostRegister(buff_, sizeof(symbolBuffer), hipHostRegisterDefault) ==
                          hipSuccess;
    }
    [[noreturn]] static void fail_copy() {
        std::fprintf(stderr, "ShMemSymBuff: device copy failed\n");
        std::exit(EXIT_FAILURE);
    }
    hipStream_t streams_[lenOfBuffer] = {};
    hipEvent_t events_[lenOfBuffer] = {};
    hipStream_t io_stream_ = nullptr;
    bool registered_ = false;
#endif

    void tic() {
        if (timerEn) start_ = clock();
    }
    void toc(float *arr, int it) {
        if (timerEn && it >= 0 && it < numberOfSymbolsToTest)
            arr[it] = (float)(clock() - start_) / (float)CLOCKS_PER_SEC;
        current_it_ = it;
    }

    CSharedMemSimple *shm_ = nullptr;
    symbolBuffer *buff_ = nullptr;
    bool master_ = false;
    clock_t start_ = 0;
    int current_it_ = 0;

  public:
    // per-symbol phase timings (seconds): the _gpu variant's members
    // (ShMemSymBuff_gpu.hpp:113-118), here views of the globals the plain
    // variant records into, so both printTimes forms see the same numbers
    float *const readT = ::readT;
    float *const decode = ::decode;
    float *const drop = ::drop;
    float *const fft = ::fft;
};

#endif  // OFDM_SHMEMSYMBUFF_IMPL_HPP_
