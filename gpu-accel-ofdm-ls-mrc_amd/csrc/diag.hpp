// diag.hpp -- per-workgroup clock stamps of the diagnostic build.
//
// The product library (make) compiles every macro below to nothing.  The
// diagnostic build (make diag -> lib/libofdm_lsmrc_diag.so, OFDM_DIAG_STAMPS=1)
// compiles the SAME kernels with three stamps per workgroup: thread 0 reads
// s_memrealtime (100 MHz wall clock) and s_memtime (shader clock) at the
// workgroup's start, at one mark (the receivers: the estimate hand-off done)
// and at its end (after a workgroup barrier), and stores them with vector
// stores into a buffer of their own (g_diag_<tag>) that no kernel reads and
// no output is computed from (MI355X_MICROARCH.md "DVFS give-back" (6)).
// bench.py reads them after the timed loop: the effective clock of the timed
// kernel = delta s_memtime / delta s_memrealtime x 100 MHz, median over
// workgroups, and the workgroup timeline (start, hand-off, end, XCC, CU).
#pragma once
#include <hip/hip_runtime.h>

#if defined(OFDM_DIAG_STAMPS) && OFDM_DIAG_STAMPS
namespace ofdm {
namespace diag {
constexpr long long MAX_WG = 1 << 20;  // records in the buffer (96 MiB); later workgroups are not stamped
// kernels that know a per-launch counter (k_demod_td1024: the low bits of its
// flag epoch) stamp into slot (counter % SLOTS) of SLOT_WG records, so the
// last SLOTS launches of a back-to-back run can be read at once
constexpr int SLOTS = 32;
constexpr long long SLOT_WG = MAX_WG / SLOTS;
constexpr int WORDS = 12;              // u64 per workgroup record
// record: rt_start, rt_mark, rt_end, mt_start, mt_end, hw_id, xcc_id, blockIdx,
// then up to 4 extra marks (OFDM_DIAG_MARKN(i), 0 = not reached)
__device__ __forceinline__ unsigned long long rt() { return __builtin_amdgcn_s_memrealtime(); }
__device__ __forceinline__ unsigned long long mt() { return __builtin_amdgcn_s_memtime(); }
constexpr int HWREG_HW_ID = (31 << 11) | 4;   // s_getreg_b32 HW_REG_HW_ID, 32 bits
constexpr int HWREG_XCC_ID = (31 << 11) | 20; // s_getreg_b32 HW_REG_XCC_ID, 32 bits
}  // namespace diag
}  // namespace ofdm

// one per translation unit: the stamp buffer and its host reader/clearer
#define OFDM_DIAG_TU(tag)                                                                                   \
    namespace ofdm { namespace diag {                                                                       \
    __device__ unsigned long long g_diag_##tag[MAX_WG * WORDS];                                             \
    } }                                                                                                     \
    extern "C" int ofdm_diag_read_##tag(void *host, long long nwg) {                                        \
        if (nwg > ofdm::diag::MAX_WG) nwg = ofdm::diag::MAX_WG;                                             \
        return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(ofdm::diag::g_diag_##tag),                         \
                                        (size_t)nwg * ofdm::diag::WORDS * 8, 0, hipMemcpyDeviceToHost);     \
    }                                                                                                       \
    extern "C" int ofdm_diag_clear_##tag() {                                                                \
        void *p = nullptr;                                                                                  \
        if (hipGetSymbolAddress(&p, HIP_SYMBOL(ofdm::diag::g_diag_##tag)) != hipSuccess) return -1;         \
        return (int)hipMemset(p, 0, sizeof(ofdm::diag::g_diag_##tag));                                      \
    }
#define OFDM_DIAG_BEGIN()                                                                                   \
    const unsigned long long dg_rt0 = ofdm::diag::rt(), dg_mt0 = ofdm::diag::mt();                         \
    unsigned long long dg_rt1 = 0, dg_mx[4] = {0, 0, 0, 0};
#define OFDM_DIAG_MARK() dg_rt1 = ofdm::diag::rt();
#define OFDM_DIAG_MARKN(i) dg_mx[i] = ofdm::diag::rt();
// marks inside a device function: the caller passes OFDM_DIAG_ARG
#define OFDM_DIAG_ARG dg_mx
#define OFDM_DIAG_MARKP(p, i) if (p) (p)[i] = ofdm::diag::rt();
// every thread of the workgroup reaches this point (it holds a barrier)
#define OFDM_DIAG_END(tag) OFDM_DIAG_END_AT(tag, 0, ofdm::diag::MAX_WG, 0)
#define OFDM_DIAG_END_SLOT(tag, counter)                                                                    \
    OFDM_DIAG_END_AT(tag, (long long)((counter) % ofdm::diag::SLOTS) * ofdm::diag::SLOT_WG, ofdm::diag::SLOT_WG, \
                     (unsigned)(counter))
// word 7 = blockIdx | (launch counter low 32 bits << 32): a slot's records of
// one launch are told from stale ones of an earlier launch in the same slot
#define OFDM_DIAG_END_AT(tag, base, cap, ctag)                                                              \
    do {                                                                                                    \
        __syncthreads();                                                                                    \
        if (threadIdx.x == 0 && (long long)blockIdx.x < (cap)) {                                            \
            const unsigned long long rt2 = ofdm::diag::rt(), mt2 = ofdm::diag::mt();                        \
            unsigned long long *d = ofdm::diag::g_diag_##tag + ((base) + (long long)blockIdx.x) * ofdm::diag::WORDS; \
            d[0] = dg_rt0; d[1] = dg_rt1 ? dg_rt1 : dg_rt0; d[2] = rt2; d[3] = dg_mt0; d[4] = mt2;          \
            d[5] = (unsigned)__builtin_amdgcn_s_getreg(ofdm::diag::HWREG_HW_ID);                            \
            d[6] = (unsigned)__builtin_amdgcn_s_getreg(ofdm::diag::HWREG_XCC_ID);                           \
            d[7] = (unsigned long long)blockIdx.x | ((unsigned long long)(ctag) << 32);                     \
            d[8] = dg_mx[0]; d[9] = dg_mx[1]; d[10] = dg_mx[2]; d[11] = dg_mx[3];                           \
        }                                                                                                   \
    } while (0)
#else
#define OFDM_DIAG_TU(tag)
#define OFDM_DIAG_BEGIN()
#define OFDM_DIAG_MARK()
#define OFDM_DIAG_MARKN(i)
#define OFDM_DIAG_ARG nullptr
#define OFDM_DIAG_MARKP(p, i)
#define OFDM_DIAG_END(tag) do { } while (0)
#define OFDM_DIAG_END_SLOT(tag, counter) do { } while (0)
#endif
