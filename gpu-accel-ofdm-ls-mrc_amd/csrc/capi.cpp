// capi.cpp -- the C ABI (include/ofdm_lsmrc.h): argument validation, error
// reporting, workspace carving and kernel dispatch.  Compiled by hipcc as HIP.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <random>
#include <string>

#include "../../include/ofdm_lsmrc.h"
#include "launch.hpp"

namespace {

thread_local std::string g_err;

int fail(int code, const char *fmt, ...) __attribute__((format(printf, 2, 3)));
int fail(int code, const char *fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

int hip_check(hipError_t e, const char *what) {
    if (e == hipSuccess) return OFDM_OK;
    return fail(OFDM_E_HIP, "%s: %s", what, hipGetErrorString(e));
}

// Every FFT length in [2, 8192]: the fused receivers at 1024 / 2048 / 4096,
// the radix-4 row FFT for the other powers of two up to 4096 and the
// mixed-radix one (fft_any.hip) for the rest; the reference takes whatever
// `dimension` it is built with (ShMemSymBuff.hpp:47, FFTW / cuFFT).
bool valid_c(int C) { return C >= 2 && C <= ofdm::FFT_ANY_MAX; }

inline hipStream_t hs(ofdm_stream_t s) { return reinterpret_cast<hipStream_t>(s); }
inline const float2 *F2(const ofdm_cf32 *p) { return reinterpret_cast<const float2 *>(p); }
inline float2 *F2(ofdm_cf32 *p) { return reinterpret_cast<float2 *>(p); }
inline bool aligned(const void *p, size_t a) { return (reinterpret_cast<uintptr_t>(p) % a) == 0; }

size_t up256(size_t x) { return (x + 255) & ~size_t(255); }

// fused one-pass kernels exist for these FFT sizes
bool fused_c(int C) { return C == 1024 || C == 2048 || C == 4096; }
// sizes whose workspace estimate is in a receiver's lane order: the fused
// ones and C = 128 / 256 / 512 / 1536 / 3072 / 6144 (staged pilot FFT, then
// k_ls_* / k_mrc_td* of frame_td_fft512.hip)
bool small_c(int C) { return C == 128 || C == 256 || C == 512; }
bool lane_c(int C) { return fused_c(C) || small_c(C) || C == 1536 || C == 3072 || C == 6144; }

// fused time-domain kernels by C (fused_c(C) must hold)
hipError_t ls_fused(const float2 *iq, long long F, int S, int R, int C, int prefix, const float2 *X,
                    float2 *Hc, float *P, int partial, hipStream_t s) {
    if (C == 1024) return ofdm::launch_ls_td1024(iq, F, S, R, prefix, X, Hc, P, partial, s);
    if (C == 2048) return ofdm::launch_ls_td2048(iq, F, S, R, prefix, X, Hc, P, partial, s);
    return ofdm::launch_ls_td4096(iq, F, S, R, prefix, X, Hc, P, partial, s);
}
hipError_t tickets_for(unsigned long long *area, hipStream_t s, ofdm::Tickets *tk);
// tickets: the frame workspace's ticket area (work-ticketed kernels: C = 2048 and 4096)
hipError_t mrc_fused(const float2 *iq, long long F, int S, int R, int C, int prefix, const float2 *Hc,
                     const float *P, float2 *out, int mode, hipStream_t s, unsigned long long *tickets) {
    if (C == 1024) return ofdm::launch_mrc_td1024(iq, F, S, R, prefix, Hc, P, out, mode, s);
    ofdm::Tickets tk;
    if (hipError_t e = tickets_for(tickets, s, &tk); e != hipSuccess) return e;
    return C == 2048 ? ofdm::launch_mrc_td2048(iq, F, S, R, prefix, Hc, P, out, mode, tk, s)
                     : ofdm::launch_mrc_td4096(iq, F, S, R, prefix, Hc, P, out, mode, tk, s);
}

// ofdm_frame_demod at C = 1024 runs LS and MRC as ONE launch (k_demod_td1024)
// unless the stream is being captured into a graph: its per-launch flag
// epoch would be frozen in the graph, and a replay would find every flag
// already set.  The same design at C = 2048 / 4096 measured no faster than
// the two launches (kept as scripts/experiments/ab_knobs_r3.patch).
bool one_launch_demod(int C, hipStream_t s) {
    if (C != 1024) return false;
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess) return false;
    return st == hipStreamCaptureStatusNone;
}

// Per-launch flag values of the one-launch demod: 64 bits, never 0, and not
// repeated in this process before 2^64 launches (a 64-bit counter added to a
// 64-bit offset drawn once per process, so that flags left in recycled
// memory by another process do not match either).
unsigned long long next_epoch() {
    static std::atomic<unsigned long long> ctr{0};
    static const unsigned long long salt = [] {
        std::random_device rd;
        return ((unsigned long long)rd() << 32) ^ (unsigned long long)rd();
    }();
    for (;;) {
        const unsigned long long e = salt + ctr.fetch_add(1);
        if (e != 0) return e;
    }
}

long long staging_frames(long long nframes, int S, int R, int C) {
    const long long per = (long long)S * R * C * (long long)sizeof(float2);
    long long n = (256ll << 20) / (per > 0 ? per : 1);
    if (n < 1) n = 1;
    return n < nframes ? n : nframes;
}

struct Workspace {
    float2 *Hc;                 // [F][R][C] bin layout
    float *P;                   // [F][C]   bin layout
    unsigned long long *flags;  // [F] per-frame estimate flags of the one-launch demod
    unsigned long long *tickets;  // 8 work-ticket counters, 128 B apart (wave_fft1024.hpp take_ticket)
    float2 *staging;            // [chunk][S][R][C] (non-fused C only)
    long long chunk;
};

constexpr size_t TICKET_BYTES = 4096;  // the ticket area: 8 counters, one 128-B line each (+ room)
constexpr int TICKET_WORDS = 8 * 16;

// Work-ticket tags (wave_fft1024.hpp, take_ticket): one per ticketed launch,
// never 0, not repeated in this process before 2^32 launches, from an offset
// drawn once per process (so counters another process left in recycled
// memory do not carry it either, but for a 2^-32 chance per word).
unsigned next_tag() {
    static std::atomic<unsigned> ctr{0};
    static const unsigned salt = [] {
        std::random_device rd;
        return (unsigned)rd();
    }();
    for (;;) {
        const unsigned t = salt + ctr.fetch_add(1);
        if (t != 0) return t;
    }
}

// The sticky device status word: host-mapped, library-owned (one per
// process, every device writes it), allocated at the first ticketed launch.
// A ticketed launch that meets a counter it cannot trust stores a TK_* bit
// there (wave_fft1024.hpp, ticket_fault); every entry that launches ticketed
// kernels reads it first (a host-side atomic exchange, no device
// synchronisation) and, if set,
// clears it and returns OFDM_E_DEVICE, as ofdm_device_status() does.
// g_status_host stands in before the mapped word exists (and for
// ofdm_device_status_inject on a machine without a GPU).
std::once_flag g_status_once;
std::atomic<unsigned *> g_status_mapped{nullptr};
std::atomic<unsigned> g_status_host{0};
unsigned *status_word_for_device() {
    std::call_once(g_status_once, [] {
        void *p = nullptr;
        if (hipHostMalloc(&p, 64, hipHostMallocMapped | hipHostMallocPortable | hipHostMallocCoherent) ==
            hipSuccess) {
            std::memset(p, 0, 64);
            g_status_mapped.store(static_cast<unsigned *>(p), std::memory_order_release);
        } else {
            (void)hipGetLastError();  // no mapped word: launches run without fault reporting
        }
    });
    return g_status_mapped.load(std::memory_order_acquire);
}
// read-and-clear, each word by one atomic exchange (a device store landing
// between a read and a clear is never lost)
int take_status(const char *fn) {
    unsigned v = g_status_host.exchange(0u, std::memory_order_acq_rel);
    if (unsigned *m = g_status_mapped.load(std::memory_order_acquire)) v |= __atomic_exchange_n(m, 0u, __ATOMIC_ACQ_REL);
    if (!v) return OFDM_OK;
    return fail(OFDM_E_DEVICE,
                "%s: an earlier work-ticketed launch (C = 1024 one-launch demod, C = 2048 / 4096 MRC) found its "
                "work-ticket counters taken by another launch (status 0x%x: %s%s%s); its output may be incomplete "
                "-- one workspace was used by two launches at once", fn, v,
                (v & ofdm::TK_FOREIGN) ? "foreign count " : "", (v & ofdm::TK_RANGE) ? "count out of range " : "",
                (v & ofdm::TK_CONTENDED) ? "contended claim" : "");
}

// The tickets of one launch.  Under stream capture the tag is frozen in the
// graph and every replay would meet the counts of the previous one: a
// captured launch is preceded by a zeroing kernel node over the counters (a
// captured hipMemsetAsync node replayed with a wrong value here), so every
// replay claims zero words.
hipError_t tickets_for(unsigned long long *area, hipStream_t s, ofdm::Tickets *tk) {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(s, &st) != hipSuccess) st = hipStreamCaptureStatusNone;
    tk->set = area;
    tk->tag = next_tag();
    tk->status = st == hipStreamCaptureStatusNone ? status_word_for_device()
                                                  : g_status_mapped.load(std::memory_order_acquire);
    if (st != hipStreamCaptureStatusNone) return ofdm::launch_zero_words(area, TICKET_WORDS, s);
    return hipSuccess;
}

size_t ws_bytes(long long F, int S, int R, int C, bool need_staging) {
    size_t b = up256((size_t)F * R * C * sizeof(float2)) + up256((size_t)F * C * sizeof(float)) +
               up256((size_t)F * sizeof(unsigned long long)) + TICKET_BYTES;
    if (need_staging) b += up256((size_t)staging_frames(F, S, R, C) * S * R * C * sizeof(float2));
    return b;
}

int carve(void *d_ws, size_t bytes, long long F, int S, int R, int C, bool need_staging,
          Workspace &w) {
    const size_t need = ws_bytes(F, S, R, C, need_staging);
    if (!d_ws || bytes < need)
        return fail(OFDM_E_ARG, "workspace too small: %zu bytes given, %zu needed", bytes, need);
    if (!aligned(d_ws, 256)) return fail(OFDM_E_ARG, "workspace must be 256-byte aligned");
    char *p = static_cast<char *>(d_ws);
    w.Hc = reinterpret_cast<float2 *>(p);
    p += up256((size_t)F * R * C * sizeof(float2));
    w.P = reinterpret_cast<float *>(p);
    p += up256((size_t)F * C * sizeof(float));
    w.flags = reinterpret_cast<unsigned long long *>(p);
    p += up256((size_t)F * sizeof(unsigned long long));
    w.tickets = reinterpret_cast<unsigned long long *>(p);
    p += TICKET_BYTES;
    w.staging = need_staging ? reinterpret_cast<float2 *>(p) : nullptr;
    w.chunk = need_staging ? staging_frames(F, S, R, C) : F;
    return OFDM_OK;
}

// What each frame workspace holds (host-side registry, per process): the
// geometry of the estimate last stored in it, the workspace size it was
// carved for, whether its Hc rows are in a fused kernel's lane order and
// whether P is an antenna-split partial.  The consumers (combine,
// mrc_partial, export) refuse a workspace whose estimate was made for another
// geometry or layout instead of dividing by the wrong |H|^2.  An estimate
// call drops the workspace's entry before it launches anything and records
// the new one only once every launch has been enqueued, so a failed estimate
// leaves no tag behind; ofdm_workspace_release() drops the entry when the
// caller frees the memory (the Python binding does it from the workspace
// tensor's finaliser), so a new workspace at a recycled address holds no
// estimate until one is made in it.
struct WsTag {
    long long F;
    int S, R, C;
    size_t bytes;
    bool lane_order, partial;
};
std::mutex g_ws_mu;
std::map<const void *, WsTag> g_ws;

void ws_record(const void *ws, size_t bytes, long long F, int S, int R, int C, bool lane_order, bool partial) {
    std::lock_guard<std::mutex> lock(g_ws_mu);
    g_ws[ws] = WsTag{F, S, R, C, bytes, lane_order, partial};
}

void ws_forget(const void *ws) {
    std::lock_guard<std::mutex> lock(g_ws_mu);
    g_ws.erase(ws);
}

// need_full: the consumer divides by P, so a partial (antenna-split) P is refused
int ws_check(const void *ws, size_t bytes, long long F, int S, int R, int C, bool need_full, const char *fn,
             WsTag *out = nullptr) {
    std::lock_guard<std::mutex> lock(g_ws_mu);
    auto it = g_ws.find(ws);
    if (it == g_ws.end())
        return fail(OFDM_E_ARG, "%s: the workspace holds no estimate (run ofdm_frame_estimate, "
                                "ofdm_frame_demod or ofdm_frame_ls_partial on it first)", fn);
    const WsTag &t = it->second;
    if (t.F != F || t.S != S || t.R != R || t.C != C)
        return fail(OFDM_E_ARG, "%s: the workspace estimate is for nframes=%lld S=%d R=%d C=%d, "
                                "called with nframes=%lld S=%d R=%d C=%d", fn, t.F, t.S, t.R, t.C, F, S, R, C);
    if (t.bytes != bytes)
        return fail(OFDM_E_ARG, "%s: the workspace was filled as %zu bytes, called with %zu", fn, t.bytes, bytes);
    if (need_full && t.partial)
        return fail(OFDM_E_ARG, "%s: the workspace holds a partial (antenna-split) |H|^2; "
                                "finalise with ofdm_mrc_finalize instead", fn);
    if (out) *out = t;
    return OFDM_OK;
}

int check_frame_args(const void *in, long long F, int S, int R, int C, int prefix,
                     const void *out, const char *fn) {
    if (F < 0) return fail(OFDM_E_ARG, "%s: nframes < 0", fn);
    if (F > 0 && (!in || !out)) return fail(OFDM_E_ARG, "%s: null pointer", fn);
    if (S < 2) return fail(OFDM_E_ARG, "%s: S=%d, a frame needs a pilot and >= 1 data symbol", fn, S);
    if (R < 1) return fail(OFDM_E_ARG, "%s: R=%d < 1", fn, R);
    if (!valid_c(C)) return fail(OFDM_E_UNSUPPORTED, "%s: C=%d out of [2, 8192]", fn, C);
    if (prefix < 0 || prefix > C) return fail(OFDM_E_ARG, "%s: prefix=%d out of [0, C]", fn, prefix);
    if (!aligned(in, 16)) return fail(OFDM_E_ARG, "%s: input must be 16-byte aligned", fn);
    return OFDM_OK;
}

// Generic (non-fused) time-domain frames.  LS: the pilot rows of each chunk
// of frames FFT'd into the staging buffer (fft_any / k_fft_rows), then the
// frequency-domain LS kernel (bin-layout Hc, P).  MRC: one fused pass over the
// IQ (k_mrc_any: FFT + combine + normalise + rotate per symbol in LDS).
// mode: 0 = full demod, 1 = MRC numerator only, 2 = LS only,
//       3 = full demod against an estimate already in the workspace
int td_staged(const float2 *iq, long long F, int S, int R, int C, int prefix, const float2 *X,
              const Workspace &w, float2 *out, int mode, hipStream_t s) {
    const long long frame_in = (long long)S * R * (C + prefix);
    hipError_t e;
    if (mode == 0 || mode == 2) {
        // the staging buffer holds w.chunk whole frames = w.chunk * S frames' pilot rows
        const long long per = w.chunk * S, pilot = (long long)R * C;
        for (long long f0 = 0; f0 < F; f0 += per) {
            const long long n = F - f0 < per ? F - f0 : per;
            e = ofdm::launch_fft_any_b(iq + f0 * frame_in, C + prefix, R, frame_in, prefix, w.staging, C, 0, n * R,
                                       C, false, 1.f, s);
            if (e != hipSuccess) return hip_check(e, "fft (pilot rows)");
            e = C == 1536   ? ofdm::launch_ls_1536(w.staging, n, R, X, w.Hc + f0 * pilot, w.P + f0 * C, s)
                : C == 3072 ? ofdm::launch_ls_3072(w.staging, n, R, X, w.Hc + f0 * pilot, w.P + f0 * C, s)
                : C == 6144 ? ofdm::launch_ls_6144(w.staging, n, R, X, w.Hc + f0 * pilot, w.P + f0 * C, s)
                : small_c(C) ? ofdm::launch_ls_small(C, w.staging, n, R, X, w.Hc + f0 * pilot, w.P + f0 * C, s)
                            : ofdm::launch_ls_freq(w.staging, pilot, n, R, C, X, w.Hc + f0 * pilot, pilot, C, 1,
                                                   w.P + f0 * C, C, 1, s);
            if (e != hipSuccess) return hip_check(e, "ls_freq");
        }
    }
    if (mode == 2) return OFDM_OK;
    if (C == 1536)
        return hip_check(ofdm::launch_mrc_td1536(iq, F, S, R, prefix, w.Hc, w.P, out, mode == 1 ? 1 : 0, s),
                         "mrc_td1536");
    if (C == 3072)
        return hip_check(ofdm::launch_mrc_td3072(iq, F, S, R, prefix, w.Hc, w.P, out, mode == 1 ? 1 : 0, s),
                         "mrc_td3072");
    if (C == 6144)
        return hip_check(ofdm::launch_mrc_td6144(iq, F, S, R, prefix, w.Hc, w.P, out, mode == 1 ? 1 : 0, s),
                         "mrc_td6144");
    if (small_c(C))
        return hip_check(ofdm::launch_mrc_small(C, iq, F, S, R, prefix, w.Hc, w.P, out, mode == 1 ? 1 : 0, s),
                         "mrc_small");
    return hip_check(ofdm::launch_mrc_any(iq, F, S, R, C, prefix, w.Hc, w.P, out, mode == 1 ? 1 : 0, s),
                     "mrc_any");
}

}  // namespace

namespace ofdm {
// error reporting for the other host-side translation units (pipeline.cpp)
int set_error(int code, const char *msg) {
    g_err = msg;
    return code;
}
}  // namespace ofdm

extern "C" {

int ofdm_version(void) { return OFDM_LSMRC_VERSION; }

const char *ofdm_last_error(void) { return g_err.c_str(); }

int ofdm_pilot_rotate(const ofdm_cf32 *raw, int K, ofdm_cf32 *X) {
    if (!raw || !X || K < 1) return fail(OFDM_E_ARG, "ofdm_pilot_rotate: bad arguments");
    // X[j] = raw[(j + (K+1)/2) mod K] for odd K; literal memmove semantics of
    // matrix_readX (cpuLS.hpp:105-112) for any K.
    const int nt = (K - 1) / 2;
    ofdm_cf32 *tmp = new ofdm_cf32[nt > 0 ? nt : 1];
    if (X != raw) std::memmove(X, raw, sizeof(ofdm_cf32) * K);
    std::memmove(tmp, &X[(K + 1) / 2], sizeof(ofdm_cf32) * nt);
    std::memmove(&X[(K - 1) / 2], X, sizeof(ofdm_cf32) * ((K + 1) / 2));
    std::memmove(X, tmp, sizeof(ofdm_cf32) * nt);
    delete[] tmp;
    return OFDM_OK;
}

int ofdm_read_pilots(const char *path, int K, float fill, ofdm_cf32 *X) {
    if (!X || K < 1) return fail(OFDM_E_ARG, "ofdm_read_pilots: bad arguments");
    FILE *fp = path ? std::fopen(path, "rb") : nullptr;
    if (!fp) {
        for (int j = 0; j < K; ++j) X[j] = ofdm_cf32{fill, fill};
        fail(1, "ofdm_read_pilots: cannot open %s, filled %g+%gi", path ? path : "(null)", fill, fill);
        return 1;
    }
    // the reference reads K values without checking the count (cpuLS.hpp:93);
    // a short file leaves the tail as it was -- here it is zero-filled.
    std::memset(X, 0, sizeof(ofdm_cf32) * K);
    size_t got = std::fread(X, sizeof(ofdm_cf32), (size_t)K, fp);
    std::fclose(fp);
    (void)got;
    return ofdm_pilot_rotate(X, K, X);
}

int ofdm_fft_rows(const ofdm_cf32 *d_in, ofdm_cf32 *d_out, long long nrows, int C, int inverse,
                  ofdm_stream_t stream) {
    if (!d_in || !d_out || nrows < 0) return fail(OFDM_E_ARG, "ofdm_fft_rows: bad arguments");
    if (!valid_c(C)) return fail(OFDM_E_UNSUPPORTED, "ofdm_fft_rows: C=%d out of [2, 8192]", C);
    return hip_check(ofdm::launch_fft_rows(F2(d_in), C, 0, F2(d_out), C, 0, nrows, C, inverse != 0,
                                           1.f, hs(stream)),
                     "ofdm_fft_rows");
}

int ofdm_ls_estimate(const ofdm_cf32 *d_Y, const ofdm_cf32 *d_X, int R, int C, ofdm_cf32 *d_Hconj,
                     float *d_Hsqrd, ofdm_stream_t stream) {
    if (!d_Y || !d_X || !d_Hconj || !d_Hsqrd || R < 1)
        return fail(OFDM_E_ARG, "ofdm_ls_estimate: bad arguments");
    if (!valid_c(C)) return fail(OFDM_E_UNSUPPORTED, "ofdm_ls_estimate: C=%d out of [2, 8192]", C);
    const int K = C - 1;
    return hip_check(ofdm::launch_ls_freq(F2(d_Y), 0, 1, R, C, F2(d_X), F2(d_Hconj), 0, K, 0, d_Hsqrd,
                                          0, 0, hs(stream)),
                     "ofdm_ls_estimate");
}

static int mrc_common(const ofdm_cf32 *d_Y, long long nsyms, const ofdm_cf32 *d_Hconj,
                      const float *d_Hsqrd, int R, int C, ofdm_cf32 *d_out, int mode,
                      ofdm_stream_t stream, const char *fn) {
    if (!d_Y || !d_Hconj || !d_out || (mode == 0 && !d_Hsqrd) || R < 1 || nsyms < 0)
        return fail(OFDM_E_ARG, "%s: bad arguments", fn);
    if (!valid_c(C)) return fail(OFDM_E_UNSUPPORTED, "%s: C=%d out of [2, 8192]", fn, C);
    if (!aligned(d_Y, 16)) return fail(OFDM_E_ARG, "%s: d_Y must be 16-byte aligned", fn);
    const int K = C - 1;
    // all symbols share one estimate: one "frame" holding nsyms data symbols
    return hip_check(ofdm::launch_mrc_freq(F2(d_Y), 0, (long long)R * C, 1, (int)nsyms, R, C,
                                           F2(d_Hconj), 0, K, 0, d_Hsqrd, 0, 0, F2(d_out), mode,
                                           hs(stream)),
                     fn);
}

int ofdm_mrc_demod(const ofdm_cf32 *d_Y, long long nsyms, const ofdm_cf32 *d_Hconj,
                   const float *d_Hsqrd, int R, int C, ofdm_cf32 *d_out, ofdm_stream_t stream) {
    if (nsyms > 0x7fffffffll) return fail(OFDM_E_ARG, "ofdm_mrc_demod: nsyms too large");
    return mrc_common(d_Y, nsyms, d_Hconj, d_Hsqrd, R, C, d_out, 0, stream, "ofdm_mrc_demod");
}

int ofdm_mrc_numerator(const ofdm_cf32 *d_Y, long long nsyms, const ofdm_cf32 *d_Hconj, int R,
                       int C, ofdm_cf32 *d_num, ofdm_stream_t stream) {
    if (nsyms > 0x7fffffffll) return fail(OFDM_E_ARG, "ofdm_mrc_numerator: nsyms too large");
    return mrc_common(d_Y, nsyms, d_Hconj, nullptr, R, C, d_num, 1, stream, "ofdm_mrc_numerator");
}

int ofdm_mrc_finalize(const ofdm_cf32 *d_num, long long e0, long long count, int nsym, int K,
                      const float *d_Hsqrd, ofdm_cf32 *d_out, ofdm_stream_t stream) {
    if (!d_num || !d_Hsqrd || !d_out || e0 < 0 || count < 0 || nsym < 1 || K < 1)
        return fail(OFDM_E_ARG, "ofdm_mrc_finalize: bad arguments");
    return hip_check(ofdm::launch_mrc_finalize(F2(d_num), e0, count, nsym, K, d_Hsqrd, F2(d_out),
                                               hs(stream)),
                     "ofdm_mrc_finalize");
}

int ofdm_channel_conj_product(const ofdm_cf32 *d_Y, long long nsyms, const ofdm_cf32 *d_Hconj,
                              int R, int C, ofdm_cf32 *d_prod, ofdm_stream_t stream) {
    if (!d_Y || !d_Hconj || !d_prod || nsyms < 0 || R < 1)
        return fail(OFDM_E_ARG, "ofdm_channel_conj_product: bad arguments");
    if (!valid_c(C)) return fail(OFDM_E_UNSUPPORTED, "ofdm_channel_conj_product: C=%d out of [2, 8192]", C);
    if (nsyms == 0) return OFDM_OK;
    return hip_check(ofdm::launch_conj_product(F2(d_Y), nsyms, R, C, F2(d_Hconj), F2(d_prod), hs(stream)),
                     "ofdm_channel_conj_product");
}

int ofdm_combine_products(const ofdm_cf32 *d_prod, long long nsyms, const float *d_Hsqrd, int R,
                          int K, int rotate, ofdm_cf32 *d_out, ofdm_stream_t stream) {
    if (!d_prod || !d_Hsqrd || !d_out || nsyms < 0 || R < 1 || K < 1)
        return fail(OFDM_E_ARG, "ofdm_combine_products: bad arguments");
    if (nsyms == 0) return OFDM_OK;
    return hip_check(ofdm::launch_combine(F2(d_prod), nsyms, R, K, d_Hsqrd, rotate, F2(d_out), hs(stream)),
                     "ofdm_combine_products");
}

int ofdm_shift_rows(const ofdm_cf32 *d_in, long long nrows, int K, ofdm_cf32 *d_out,
                    ofdm_stream_t stream) {
    if (!d_in || !d_out || nrows < 0 || K < 1 || d_in == d_out)
        return fail(OFDM_E_ARG, "ofdm_shift_rows: bad arguments (out of place only)");
    if (nrows == 0) return OFDM_OK;
    return hip_check(ofdm::launch_shift_rows(F2(d_in), nrows, K, F2(d_out), hs(stream)), "ofdm_shift_rows");
}

int ofdm_dist_sqrd(const ofdm_cf32 *d_H, int R, int K, float *d_Hsqrd, ofdm_stream_t stream) {
    if (!d_H || !d_Hsqrd || R < 1 || K < 1) return fail(OFDM_E_ARG, "ofdm_dist_sqrd: bad arguments");
    return hip_check(ofdm::launch_dist_sqrd(F2(d_H), R, K, d_Hsqrd, hs(stream)), "ofdm_dist_sqrd");
}

size_t ofdm_frame_workspace_bytes(long long nframes, int S, int R, int C) {
    if (nframes < 0 || S < 2 || R < 1 || !valid_c(C)) return 0;
    return ws_bytes(nframes, S, R, C, !fused_c(C));
}

int ofdm_workspace_release(const void *d_ws) {
    ws_forget(d_ws);
    return OFDM_OK;
}

int ofdm_device_status(void) { return take_status("ofdm_device_status"); }

int ofdm_device_status_inject(unsigned bits) {
    g_status_host.fetch_or(bits, std::memory_order_acq_rel);
    return OFDM_OK;
}

int ofdm_frame_estimate(const ofdm_cf32 *d_iq, long long nframes, int S, int R, int C, int prefix,
                        const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes_, ofdm_stream_t stream) {
    int rc = check_frame_args(d_iq, nframes, S, R, C, prefix, d_ws, "ofdm_frame_estimate");
    if (rc) return rc;
    if (!d_X) return fail(OFDM_E_ARG, "ofdm_frame_estimate: null pilots");
    if (nframes == 0) return OFDM_OK;
    Workspace w;
    if ((rc = carve(d_ws, ws_bytes_, nframes, S, R, C, !fused_c(C), w))) return rc;
    ws_forget(d_ws);
    hipStream_t s = hs(stream);
    if (fused_c(C))
        rc = hip_check(ls_fused(F2(d_iq), nframes, S, R, C, prefix, F2(d_X), w.Hc, w.P, 0, s), "ls_fused");
    else
        rc = td_staged(F2(d_iq), nframes, S, R, C, prefix, F2(d_X), w, nullptr, 2, s);
    if (rc == OFDM_OK) ws_record(d_ws, ws_bytes_, nframes, S, R, C, lane_c(C), false);
    return rc;
}

int ofdm_frame_combine(const ofdm_cf32 *d_iq, long long nframes, int S, int R, int C, int prefix,
                       void *d_ws, size_t ws_bytes_, ofdm_cf32 *d_out, ofdm_stream_t stream) {
    if (int st = take_status("ofdm_frame_combine")) return st;
    int rc = check_frame_args(d_iq, nframes, S, R, C, prefix, d_out, "ofdm_frame_combine");
    if (rc) return rc;
    if (nframes == 0) return OFDM_OK;
    WsTag tag;
    if ((rc = ws_check(d_ws, ws_bytes_, nframes, S, R, C, true, "ofdm_frame_combine", &tag))) return rc;
    if (tag.lane_order != lane_c(C))
        return fail(OFDM_E_ARG, "ofdm_frame_combine: the workspace holds a frequency-domain estimate "
                                "(use ofdm_frame_combine_freq)");
    Workspace w;
    if ((rc = carve(d_ws, ws_bytes_, nframes, S, R, C, !fused_c(C), w))) return rc;
    hipStream_t s = hs(stream);
    if (fused_c(C))
        return hip_check(mrc_fused(F2(d_iq), nframes, S, R, C, prefix, w.Hc, w.P,
                                                 F2(d_out), 0, s, w.tickets),
                         "mrc_fused");
    // staged path: the FFT of every chunk is redone here (estimate kept only Hc/P)
    return td_staged(F2(d_iq), nframes, S, R, C, prefix, nullptr, w, F2(d_out), 3, s);
}

int ofdm_frame_demod(const ofdm_cf32 *d_iq, long long nframes, int S, int R, int C, int prefix,
                     const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes_, ofdm_cf32 *d_out,
                     ofdm_stream_t stream) {
    return ofdm_frame_demod_ex(d_iq, nframes, S, R, C, prefix, d_X, d_ws, ws_bytes_, d_out, OFDM_FLOW_AUTO, -1,
                               stream);
}

int ofdm_frame_demod_ex(const ofdm_cf32 *d_iq, long long nframes, int S, int R, int C, int prefix,
                        const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes_, ofdm_cf32 *d_out, int flow,
                        long long spin_ticks, ofdm_stream_t stream) {
    if (int st = take_status("ofdm_frame_demod")) return st;
    int rc = check_frame_args(d_iq, nframes, S, R, C, prefix, d_out, "ofdm_frame_demod");
    if (rc) return rc;
    if (!d_X) return fail(OFDM_E_ARG, "ofdm_frame_demod: null pilots");
    if (flow != OFDM_FLOW_AUTO && flow != OFDM_FLOW_TWO_LAUNCH)
        return fail(OFDM_E_ARG, "ofdm_frame_demod_ex: flow=%d (OFDM_FLOW_AUTO or OFDM_FLOW_TWO_LAUNCH)", flow);
    if (nframes == 0) return OFDM_OK;
    Workspace w;
    if ((rc = carve(d_ws, ws_bytes_, nframes, S, R, C, !fused_c(C), w))) return rc;
    hipStream_t s = hs(stream);
    ws_forget(d_ws);
    if (flow == OFDM_FLOW_AUTO && one_launch_demod(C, s)) {
        ofdm::Tickets tk;
        if ((rc = hip_check(tickets_for(w.tickets, s, &tk), "work tickets"))) return rc;
        rc = hip_check(ofdm::launch_demod_td1024(F2(d_iq), nframes, S, R, prefix, F2(d_X), w.Hc, w.P, F2(d_out), tk,
                                                 w.flags, next_epoch(), spin_ticks, s),
                       "launch_demod_td");
        if (rc == OFDM_OK) ws_record(d_ws, ws_bytes_, nframes, S, R, C, true, false);
        return rc;
    }
    if (fused_c(C)) {
        rc = hip_check(ls_fused(F2(d_iq), nframes, S, R, C, prefix, F2(d_X), w.Hc, w.P, 0, s),
                       "ls_fused");
        if (rc) return rc;
        // the estimate is in the workspace once the LS launch is enqueued
        ws_record(d_ws, ws_bytes_, nframes, S, R, C, true, false);
        return hip_check(mrc_fused(F2(d_iq), nframes, S, R, C, prefix, w.Hc, w.P, F2(d_out), 0, s, w.tickets),
                         "mrc_fused");
    }
    rc = td_staged(F2(d_iq), nframes, S, R, C, prefix, F2(d_X), w, F2(d_out), 0, s);
    if (rc == OFDM_OK) ws_record(d_ws, ws_bytes_, nframes, S, R, C, lane_c(C), false);
    return rc;
}

int ofdm_frame_estimate_freq(const ofdm_cf32 *d_Y, long long nframes, int S, int R, int C,
                             const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes_, ofdm_stream_t stream) {
    int rc = check_frame_args(d_Y, nframes, S, R, C, 0, d_ws, "ofdm_frame_estimate_freq");
    if (rc) return rc;
    if (!d_X) return fail(OFDM_E_ARG, "ofdm_frame_estimate_freq: null pilots");
    if (nframes == 0) return OFDM_OK;
    Workspace w;
    if ((rc = carve(d_ws, ws_bytes_, nframes, S, R, C, !fused_c(C), w))) return rc;
    ws_forget(d_ws);
    rc = hip_check(ofdm::launch_ls_freq(F2(d_Y), (long long)S * R * C, nframes, R, C, F2(d_X), w.Hc,
                                        (long long)R * C, C, 1, w.P, C, 1, hs(stream)),
                   "ls_freq");
    if (rc == OFDM_OK) ws_record(d_ws, ws_bytes_, nframes, S, R, C, false, false);
    return rc;
}

int ofdm_frame_combine_freq(const ofdm_cf32 *d_Y, long long nframes, int S, int R, int C, void *d_ws,
                            size_t ws_bytes_, ofdm_cf32 *d_out, ofdm_stream_t stream) {
    int rc = check_frame_args(d_Y, nframes, S, R, C, 0, d_out, "ofdm_frame_combine_freq");
    if (rc) return rc;
    if (nframes == 0) return OFDM_OK;
    WsTag tag;
    if ((rc = ws_check(d_ws, ws_bytes_, nframes, S, R, C, true, "ofdm_frame_combine_freq", &tag))) return rc;
    if (tag.lane_order)
        return fail(OFDM_E_ARG, "ofdm_frame_combine_freq: the workspace holds a time-domain estimate in the "
                                "fused kernels' lane order (use ofdm_frame_combine)");
    Workspace w;
    if ((rc = carve(d_ws, ws_bytes_, nframes, S, R, C, !fused_c(C), w))) return rc;
    const long long fst = (long long)S * R * C;
    return hip_check(ofdm::launch_mrc_freq(F2(d_Y) + (long long)R * C, fst, (long long)R * C, nframes,
                                           S - 1, R, C, w.Hc, (long long)R * C, C, 0, w.P, C, 1,
                                           F2(d_out), 0, hs(stream)),
                     "mrc_freq");
}

int ofdm_frame_demod_freq(const ofdm_cf32 *d_Y, long long nframes, int S, int R, int C,
                          const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes_, ofdm_cf32 *d_out,
                          ofdm_stream_t stream) {
    int rc = check_frame_args(d_Y, nframes, S, R, C, 0, d_out, "ofdm_frame_demod_freq");
    if (rc) return rc;
    if ((rc = ofdm_frame_estimate_freq(d_Y, nframes, S, R, C, d_X, d_ws, ws_bytes_, stream))) return rc;
    return ofdm_frame_combine_freq(d_Y, nframes, S, R, C, d_ws, ws_bytes_, d_out, stream);
}

int ofdm_frame_demod_freq_mfma(const ofdm_cf32 *d_Y, long long nframes, int S, int R, int C,
                               const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes_, ofdm_cf32 *d_out,
                               ofdm_stream_t stream) {
    int rc = check_frame_args(d_Y, nframes, S, R, C, 0, d_out, "ofdm_frame_demod_freq_mfma");
    if (rc) return rc;
    if (C % 64) return fail(OFDM_E_UNSUPPORTED, "ofdm_frame_demod_freq_mfma: C=%d not a multiple of 64", C);
    if (!d_X) return fail(OFDM_E_ARG, "ofdm_frame_demod_freq_mfma: null pilots");
    if (nframes == 0) return OFDM_OK;
    Workspace w;
    if ((rc = carve(d_ws, ws_bytes_, nframes, S, R, C, !fused_c(C), w))) return rc;
    hipStream_t s = hs(stream);
    const long long fst = (long long)S * R * C;
    ws_forget(d_ws);
    rc = hip_check(ofdm::launch_ls_freq(F2(d_Y), fst, nframes, R, C, F2(d_X), w.Hc, (long long)R * C, C,
                                        1, w.P, C, 1, s),
                   "ls_freq");
    if (rc) return rc;
    ws_record(d_ws, ws_bytes_, nframes, S, R, C, false, false);
    return hip_check(ofdm::launch_mrc_freq_mfma(F2(d_Y) + (long long)R * C, fst, (long long)R * C, nframes,
                                                S - 1, R, C, w.Hc, (long long)R * C, w.P, C, F2(d_out), 0, s),
                     "mrc_freq_mfma");
}

int ofdm_frame_ls_partial(const ofdm_cf32 *d_iq, long long nframes, int S, int R, int C, int prefix,
                          const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes_, float *d_P,
                          ofdm_stream_t stream) {
    int rc = check_frame_args(d_iq, nframes, S, R, C, prefix, d_P, "ofdm_frame_ls_partial");
    if (rc) return rc;
    if (!d_X) return fail(OFDM_E_ARG, "ofdm_frame_ls_partial: null pilots");
    if (nframes == 0) return OFDM_OK;
    Workspace w;
    if ((rc = carve(d_ws, ws_bytes_, nframes, S, R, C, !fused_c(C), w))) return rc;
    hipStream_t s = hs(stream);
    ws_forget(d_ws);
    if (fused_c(C))
        rc = hip_check(ls_fused(F2(d_iq), nframes, S, R, C, prefix, F2(d_X), w.Hc, w.P, 1, s),
                       "ls_fused");
    else
        rc = td_staged(F2(d_iq), nframes, S, R, C, prefix, F2(d_X), w, nullptr, 2, s);
    if (rc) return rc;
    ws_record(d_ws, ws_bytes_, nframes, S, R, C, lane_c(C), true);
    // bins 1..C-1 of the bin-layout P -> [F][K]
    const int K = C - 1;
    return hip_check(hipMemcpy2DAsync(d_P, K * sizeof(float), w.P + 1, C * sizeof(float),
                                      K * sizeof(float), (size_t)nframes, hipMemcpyDeviceToDevice, s),
                     "copy partial P");
}

int ofdm_frame_mrc_partial(const ofdm_cf32 *d_iq, long long nframes, int S, int R, int C,
                           int prefix, void *d_ws, size_t ws_bytes_, ofdm_cf32 *d_num,
                           ofdm_stream_t stream) {
    if (int st = take_status("ofdm_frame_mrc_partial")) return st;
    int rc = check_frame_args(d_iq, nframes, S, R, C, prefix, d_num, "ofdm_frame_mrc_partial");
    if (rc) return rc;
    if (nframes == 0) return OFDM_OK;
    WsTag tag;
    if ((rc = ws_check(d_ws, ws_bytes_, nframes, S, R, C, false, "ofdm_frame_mrc_partial", &tag))) return rc;
    if (tag.lane_order != lane_c(C))
        return fail(OFDM_E_ARG, "ofdm_frame_mrc_partial: the workspace holds a frequency-domain estimate, "
                                "not the time-domain one of ofdm_frame_ls_partial / ofdm_frame_estimate");
    Workspace w;
    if ((rc = carve(d_ws, ws_bytes_, nframes, S, R, C, !fused_c(C), w))) return rc;
    hipStream_t s = hs(stream);
    if (fused_c(C))
        return hip_check(mrc_fused(F2(d_iq), nframes, S, R, C, prefix, w.Hc, w.P,
                                                 F2(d_num), 1, s, w.tickets),
                         "mrc_fused");
    return td_staged(F2(d_iq), nframes, S, R, C, prefix, nullptr, w, F2(d_num), 1, s);
}

int ofdm_frame_mrc_partial_range(const ofdm_cf32 *d_iq, long long nframes, long long f0, long long count, int S,
                                 int R, int C, int prefix, void *d_ws, size_t ws_bytes_, ofdm_cf32 *d_num,
                                 ofdm_stream_t stream) {
    static const char *fn = "ofdm_frame_mrc_partial_range";
    if (int st = take_status(fn)) return st;
    if (nframes < 0 || f0 < 0 || count < 0 || f0 > nframes || count > nframes - f0)
        return fail(OFDM_E_ARG, "%s: frames [%lld, %lld) outside [0, %lld)", fn, f0, f0 + count, nframes);
    if (count == 0) return OFDM_OK;
    int rc = check_frame_args(d_iq, nframes, S, R, C, prefix, d_num, fn);
    if (rc) return rc;
    WsTag tag;
    if ((rc = ws_check(d_ws, ws_bytes_, nframes, S, R, C, false, fn, &tag))) return rc;
    if (tag.lane_order != lane_c(C))
        return fail(OFDM_E_ARG, "%s: the workspace holds a frequency-domain estimate, not the time-domain one of "
                                "ofdm_frame_ls_partial / ofdm_frame_estimate", fn);
    Workspace w;
    if ((rc = carve(d_ws, ws_bytes_, nframes, S, R, C, !fused_c(C), w))) return rc;
    hipStream_t s = hs(stream);
    const float2 *iq = F2(d_iq) + f0 * (long long)S * R * (C + prefix);
    Workspace v = w;  // the range's estimate: frames f0 .. in the same [F][R][C] / [F][C] layout
    v.Hc += f0 * (long long)R * C;
    v.P += f0 * C;
    if (fused_c(C))
        return hip_check(mrc_fused(iq, count, S, R, C, prefix, v.Hc, v.P, F2(d_num), 1, s, w.tickets), fn);
    return td_staged(iq, count, S, R, C, prefix, nullptr, v, F2(d_num), 1, s);
}

int ofdm_symbols_demod(const ofdm_cf32 *d_sym, long long nsym, int R, int C, int prefix, const void *d_ws,
                       size_t ws_bytes_, long long frame, ofdm_cf32 *d_out, ofdm_stream_t stream) {
    static const char *fn = "ofdm_symbols_demod";
    if (int st = take_status(fn)) return st;
    if (nsym < 0 || nsym > 0x7ffffffell) return fail(OFDM_E_ARG, "%s: nsym=%lld out of range", fn, nsym);
    if (nsym > 0 && (!d_sym || !d_out)) return fail(OFDM_E_ARG, "%s: null pointer", fn);
    if (R < 1) return fail(OFDM_E_ARG, "%s: R=%d < 1", fn, R);
    if (!fused_c(C))
        return fail(OFDM_E_UNSUPPORTED, "%s: C=%d (the fused receivers cover C = 1024, 2048, 4096)", fn, C);
    if (prefix < 0 || prefix > C) return fail(OFDM_E_ARG, "%s: prefix=%d out of [0, C]", fn, prefix);
    if (!aligned(d_sym, 16)) return fail(OFDM_E_ARG, "%s: input must be 16-byte aligned", fn);
    WsTag tag;
    {
        std::lock_guard<std::mutex> lock(g_ws_mu);
        auto it = g_ws.find(d_ws);
        if (it == g_ws.end())
            return fail(OFDM_E_ARG, "%s: the workspace holds no estimate (run ofdm_frame_estimate on it first)", fn);
        tag = it->second;
    }
    if (tag.R != R || tag.C != C || tag.bytes != ws_bytes_)
        return fail(OFDM_E_ARG, "%s: the workspace estimate is for R=%d C=%d (%zu bytes), called with R=%d C=%d "
                                "(%zu bytes)", fn, tag.R, tag.C, tag.bytes, R, C, ws_bytes_);
    if (!tag.lane_order || tag.partial)
        return fail(OFDM_E_ARG, "%s: the workspace holds a %s estimate, not ofdm_frame_estimate's", fn,
                    tag.partial ? "partial (antenna-split)" : "frequency-domain");
    if (frame < 0 || frame >= tag.F)
        return fail(OFDM_E_ARG, "%s: frame %lld outside the workspace's [0, %lld)", fn, frame, tag.F);
    if (nsym == 0) return OFDM_OK;
    Workspace w;
    int rc = carve(const_cast<void *>(d_ws), ws_bytes_, tag.F, tag.S, R, C, false, w);
    if (rc) return rc;
    // The fused MRC kernels read data symbols 1..S-1 of frame 0 at
    // iq + s * R * (C + prefix) and never touch symbol 0 (the pilot, read by
    // the LS kernels only): a "frame" whose symbol 1 is d_sym[0] is the run.
    const long long row = (long long)R * (C + prefix);
    const float2 *iq = reinterpret_cast<const float2 *>(reinterpret_cast<uintptr_t>(d_sym) - (uintptr_t)(row * 8));
    return hip_check(mrc_fused(iq, 1, (int)(nsym + 1), R, C, prefix, w.Hc + frame * (long long)R * C,
                               w.P + frame * C, F2(d_out), 0, hs(stream), w.tickets),
                     fn);
}

int ofdm_frame_export_estimate(const void *d_ws, size_t ws_bytes_, long long nframes, int S, int R, int C,
                               long long frame, ofdm_cf32 *d_Hconj, float *d_Hsqrd, ofdm_stream_t stream) {
    if (!d_Hconj) return fail(OFDM_E_ARG, "ofdm_frame_export_estimate: null d_Hconj");
    if (nframes < 1 || frame < 0 || frame >= nframes)
        return fail(OFDM_E_ARG, "ofdm_frame_export_estimate: frame %lld outside [0, %lld)", frame, nframes);
    if (S < 2 || R < 1 || !valid_c(C)) return fail(OFDM_E_ARG, "ofdm_frame_export_estimate: bad geometry");
    WsTag tag;
    int rc = ws_check(d_ws, ws_bytes_, nframes, S, R, C, false, "ofdm_frame_export_estimate", &tag);
    if (rc) return rc;
    Workspace w;
    if ((rc = carve(const_cast<void *>(d_ws), ws_bytes_, nframes, S, R, C, !fused_c(C), w))) return rc;
    return hip_check(ofdm::launch_export_estimate(w.Hc + frame * R * C, w.P + frame * C, R, C, tag.lane_order,
                                                  F2(d_Hconj), d_Hsqrd, hs(stream)),
                     "ofdm_frame_export_estimate");
}

int ofdm_synth_frames(ofdm_cf32 *d_iq, long long nframes, int S, int R, int C, int prefix,
                      const ofdm_cf32 *d_X, unsigned long long seed, long long frame0,
                      float noise_std, int freq_domain, int r0, ofdm_stream_t stream) {
    if (!d_iq || !d_X || nframes < 0 || S < 1 || R < 1 || prefix < 0 || prefix > C || r0 < 0)
        return fail(OFDM_E_ARG, "ofdm_synth_frames: bad arguments");
    if (!valid_c(C)) return fail(OFDM_E_UNSUPPORTED, "ofdm_synth_frames: C=%d out of [2, 8192]", C);
    return hip_check(ofdm::launch_synth(F2(d_iq), nframes, S, R, C, freq_domain ? 0 : prefix, F2(d_X),
                                        seed, frame0, noise_std, freq_domain, r0, hs(stream)),
                     "ofdm_synth_frames");
}

int ofdm_count_symbol_errors(const ofdm_cf32 *d_out, long long nframes, int S, int C,
                             unsigned long long seed, long long frame0,
                             unsigned long long *d_errors, ofdm_stream_t stream) {
    if (!d_out || !d_errors || nframes < 0 || S < 2 || !valid_c(C))
        return fail(OFDM_E_ARG, "ofdm_count_symbol_errors: bad arguments");
    return hip_check(ofdm::launch_count_errors(F2(d_out), nframes, S, C, seed, frame0, d_errors,
                                               hs(stream)),
                     "ofdm_count_symbol_errors");
}

int ofdm_buffer_hash(const void *d_buf, size_t bytes, unsigned long long *d_hash, ofdm_stream_t stream) {
    if (!d_hash || (bytes && !d_buf) || bytes % 4 || !aligned(d_buf, 4))
        return fail(OFDM_E_ARG, "ofdm_buffer_hash: a 4-B aligned buffer of whole 32-bit words and a hash slot");
    return hip_check(ofdm::launch_hash_words(d_buf, (long long)(bytes / 4), d_hash, hs(stream)),
                     "ofdm_buffer_hash");
}

int ofdm_hbm_probe(int mode, const void *d_src, void *d_dst, size_t bytes, size_t dst_bytes, ofdm_stream_t stream) {
    if ((mode != 0 && mode != 1) || !d_src || !d_dst)
        return fail(OFDM_E_ARG, "ofdm_hbm_probe: mode 0 (copy) or 1 (read) and non-null buffers");
    const size_t need = mode == 0 ? bytes : (size_t)OFDM_HBM_PROBE_SINK_BYTES;
    if (dst_bytes < need)
        return fail(OFDM_E_ARG, "ofdm_hbm_probe: d_dst holds %zu bytes, mode %d writes %zu", dst_bytes, mode, need);
    if ((reinterpret_cast<size_t>(d_src) | reinterpret_cast<size_t>(d_dst) | bytes) % 16)
        return fail(OFDM_E_ARG, "ofdm_hbm_probe: 16-B aligned buffers and a multiple of 16 bytes");
    return hip_check(ofdm::launch_hbm_probe(mode, d_src, d_dst, (long long)(bytes / 16), hs(stream)),
                     "ofdm_hbm_probe");
}

int ofdm_pn_correlate(const ofdm_cf32 *d_buf, int R, long long N, const ofdm_cf32 *d_pn, int L,
                      float thres, long long *d_pos, float *d_mag, ofdm_stream_t stream) {
    if (!d_pos) return fail(OFDM_E_ARG, "ofdm_pn_correlate: null d_pos");
    if (R < 0 || N < 0 || L < 1) return fail(OFDM_E_ARG, "ofdm_pn_correlate: R >= 0, N >= 0, L >= 1 required");
    if (R > 0 && N >= L && (!d_buf || !d_pn))
        return fail(OFDM_E_ARG, "ofdm_pn_correlate: null buffer");
    return hip_check(ofdm::launch_pn_correlate(F2(d_buf), R, N, F2(d_pn), L, thres, d_pos, d_mag,
                                               hs(stream)),
                     "ofdm_pn_correlate");
}

int ofdm_pn_extract(const ofdm_cf32 *d_buf1, const ofdm_cf32 *d_buf2, int R, long long N, int L,
                    const long long *d_pos, int C, int cp, int nsym, ofdm_cf32 *d_sym,
                    ofdm_stream_t stream) {
    if (R < 1 || L < 1 || C < 1 || cp < 0 || nsym < 0 || N < L)
        return fail(OFDM_E_ARG, "ofdm_pn_extract: bad geometry");
    if ((long long)nsym * (C + cp) > N - L)
        return fail(OFDM_E_ARG, "ofdm_pn_extract: nsym*(C+cp)=%lld exceeds the N-L=%lld samples after the PN",
                    (long long)nsym * (C + cp), N - L);
    if (!d_buf1 || !d_buf2 || !d_pos || (nsym > 0 && !d_sym))
        return fail(OFDM_E_ARG, "ofdm_pn_extract: null pointer");
    return hip_check(ofdm::launch_pn_extract(F2(d_buf1), F2(d_buf2), R, N, L, d_pos, C, cp, nsym,
                                             F2(d_sym), hs(stream)),
                     "ofdm_pn_extract");
}

static int zf_geometry(int users, int rows, int K, const char *fn) {
    if (users < 1 || users > OFDM_ZF_MAX_USERS)
        return fail(OFDM_E_UNSUPPORTED, "%s: users=%d outside [1, %d]", fn, users, OFDM_ZF_MAX_USERS);
    if (rows < 1 || K < 0) return fail(OFDM_E_ARG, "%s: rows=%d, K=%d", fn, rows, K);
    if ((long long)users * rows > OFDM_ZF_MAX_USERS_X_ROWS)
        return fail(OFDM_E_UNSUPPORTED, "%s: users*rows=%lld > %d", fn, (long long)users * rows,
                    OFDM_ZF_MAX_USERS_X_ROWS);
    return OFDM_OK;
}

int ofdm_zf_precoder(const ofdm_cf32 *d_H, int users, int rows, int K, ofdm_cf32 *d_W, ofdm_cf32 *d_Wt,
                     ofdm_stream_t stream) {
    int rc = zf_geometry(users, rows, K, "ofdm_zf_precoder");
    if (rc) return rc;
    if (K > 0 && (!d_H || (!d_W && !d_Wt))) return fail(OFDM_E_ARG, "ofdm_zf_precoder: null pointer");
    return hip_check(ofdm::launch_zf_precoder(F2(d_H), users, rows, K, F2(d_W), F2(d_Wt), hs(stream)),
                     "ofdm_zf_precoder");
}

int ofdm_zf_transpose(const ofdm_cf32 *d_W, int users, int rows, int K, ofdm_cf32 *d_Wt,
                      ofdm_stream_t stream) {
    int rc = zf_geometry(users, rows, K, "ofdm_zf_transpose");
    if (rc) return rc;
    if (K > 0 && (!d_W || !d_Wt || d_W == d_Wt))
        return fail(OFDM_E_ARG, "ofdm_zf_transpose: null or aliased pointers");
    return hip_check(ofdm::launch_zf_transpose(F2(d_W), users, rows, K, F2(d_Wt), hs(stream)),
                     "ofdm_zf_transpose");
}

int ofdm_zf_apply(const ofdm_cf32 *d_Wt, const ofdm_cf32 *d_X, int users, int rows, int K, long long nsym,
                  ofdm_cf32 *d_Y, ofdm_stream_t stream) {
    int rc = zf_geometry(users, rows, K, "ofdm_zf_apply");
    if (rc) return rc;
    if (nsym < 0) return fail(OFDM_E_ARG, "ofdm_zf_apply: nsym < 0");
    if (K > 0 && nsym > 0 && (!d_Wt || !d_X || !d_Y)) return fail(OFDM_E_ARG, "ofdm_zf_apply: null pointer");
    return hip_check(ofdm::launch_zf_apply(F2(d_Wt), F2(d_X), users, rows, K, nsym, F2(d_Y), hs(stream)),
                     "ofdm_zf_apply");
}

int ofdm_zf_detect(const ofdm_cf32 *d_Wt, const ofdm_cf32 *d_Y, int users, int rows, int K, long long nsym,
                   ofdm_cf32 *d_X, ofdm_stream_t stream) {
    int rc = zf_geometry(users, rows, K, "ofdm_zf_detect");
    if (rc) return rc;
    if (nsym < 0) return fail(OFDM_E_ARG, "ofdm_zf_detect: nsym < 0");
    if (K > 0 && nsym > 0 && (!d_Wt || !d_X || !d_Y)) return fail(OFDM_E_ARG, "ofdm_zf_detect: null pointer");
    return hip_check(ofdm::launch_zf_detect(F2(d_Wt), F2(d_Y), users, rows, K, nsym, F2(d_X), hs(stream)),
                     "ofdm_zf_detect");
}

int ofdm_zf_apply_ex(const ofdm_cf32 *d_Wt, const ofdm_cf32 *d_X, long long ldx, int users, int rows, int K,
                     long long nsym, ofdm_cf32 *d_Y, long long ldy, ofdm_stream_t stream) {
    static const char *fn = "ofdm_zf_apply_ex";
    int rc = zf_geometry(users, rows, K, fn);
    if (rc) return rc;
    if (nsym < 0) return fail(OFDM_E_ARG, "%s: nsym < 0", fn);
    if (ldx < K || ldy < K) return fail(OFDM_E_ARG, "%s: ldx=%lld, ldy=%lld below K=%d", fn, ldx, ldy, K);
    if ((ldx != K || ldy != K) && !ofdm::zf_apply_pitched_supported(users, rows, K))
        return fail(OFDM_E_UNSUPPORTED, "%s: row pitches other than K need K >= 2, rows >= 8 and users <= 40", fn);
    if (K > 0 && nsym > 0 && (!d_Wt || !d_X || !d_Y)) return fail(OFDM_E_ARG, "%s: null pointer", fn);
    return hip_check(ofdm::launch_zf_apply_ld(F2(d_Wt), F2(d_X), ldx, users, rows, K, nsym, F2(d_Y), ldy,
                                              hs(stream)),
                     fn);
}

int ofdm_zf_detect_ex(const ofdm_cf32 *d_Wt, const ofdm_cf32 *d_Y, long long ldy, int users, int rows, int K,
                      long long nsym, ofdm_cf32 *d_X, long long ldx, ofdm_stream_t stream) {
    static const char *fn = "ofdm_zf_detect_ex";
    int rc = zf_geometry(users, rows, K, fn);
    if (rc) return rc;
    if (nsym < 0) return fail(OFDM_E_ARG, "%s: nsym < 0", fn);
    if (ldy < K || ldx < K) return fail(OFDM_E_ARG, "%s: ldy=%lld, ldx=%lld below K=%d", fn, ldy, ldx, K);
    if ((ldy != K || ldx != K) && !ofdm::zf_detect_pitched_supported(users, rows))
        return fail(OFDM_E_UNSUPPORTED, "%s: row pitches other than K need rows <= 72 (rows=%d)", fn, rows);
    if (K > 0 && nsym > 0 && (!d_Wt || !d_X || !d_Y)) return fail(OFDM_E_ARG, "%s: null pointer", fn);
    return hip_check(ofdm::launch_zf_detect_ld(F2(d_Wt), F2(d_Y), ldy, users, rows, K, nsym, F2(d_X), ldx,
                                               hs(stream)),
                     fn);
}

}  // extern "C"
