// launch.hpp -- internal host-side launchers for the LS/MRC kernels.
// Arguments are validated by the C-ABI layer (capi.cpp) before these run;
// every launcher returns hipGetLastError() of its launch(es).
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <mutex>
#include <set>
#include <tuple>

namespace ofdm {

// Opts `kernel` into `bytes` of dynamic LDS (launches above 64 KiB need it)
// once per (kernel, device, size) in this process; thread-safe, so a process
// driving several GPUs or launching from several host threads is covered.
inline hipError_t opt_in_lds(const void *kernel, int bytes) {
    static std::mutex mu;
    static std::set<std::tuple<const void *, int, int>> done;
    int dev = 0;
    hipError_t e = hipGetDevice(&dev);
    if (e != hipSuccess) return e;
    std::lock_guard<std::mutex> lock(mu);
    const auto key = std::make_tuple(kernel, dev, bytes);
    if (done.count(key)) return hipSuccess;
    e = hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
    if (e == hipSuccess) done.insert(key);
    return e;
}

// Sets ofdm_last_error() for the calling thread and returns `code`.
int set_error(int code, const char *msg);

// The work tickets of ONE launch of a ticketed receiver (wave_fft1024.hpp,
// take_unit): set = 8 counter words 128 B apart (the workspace's ticket
// area); tag = this launch's value, never 0, in the high half of every word
// the launch counts in (a word holding anything else is claimed afresh, so
// no stale or foreign value is ever consumed as a count); status = the
// library's host-mapped sticky status word (capi.cpp, OFDM_E_DEVICE), or null.
struct Tickets {
    unsigned long long *set;
    unsigned *status;
    unsigned tag;
};
// status bits a ticketed launch raises
constexpr unsigned TK_FOREIGN = 1u;     // a count of another launch in a fetch_add result
constexpr unsigned TK_RANGE = 2u;       // a count beyond units + grid
constexpr unsigned TK_CONTENDED = 4u;   // a claim that did not settle in 64 compare-and-swaps

// Generic batched row FFT (Stockham in LDS), in place or out of place.
// Row i is read from in + i*in_stride + in_off and written to
// out + i*out_stride + out_off.  Any 2 <= C <= FFT_ANY_MAX: powers of two up
// to 4096 run the radix-4 kernel (fft_synth.hip), every other length the
// mixed-radix one (fft_any.hip).
constexpr int FFT_ANY_MAX = 8192;
hipError_t launch_fft_rows(const float2 *in, long long in_stride, int in_off, float2 *out,
                           long long out_stride, int out_off, long long nrows, int C,
                           bool inverse, float scale, hipStream_t s);
// The mixed-radix kernel alone (any C in [2, FFT_ANY_MAX]).
hipError_t launch_fft_any(const float2 *in, long long in_stride, int in_off, float2 *out,
                          long long out_stride, int out_off, long long nrows, int C, bool inverse,
                          float scale, hipStream_t s);
// ... with input row i at in + (i / in_rb) * in_bstride + (i % in_rb) * in_stride
// + in_off (e.g. the R pilot rows of every frame of a batch in one launch).
hipError_t launch_fft_any_b(const float2 *in, long long in_stride, long long in_rb, long long in_bstride,
                            int in_off, float2 *out, long long out_stride, int out_off, long long nrows, int C,
                            bool inverse, float scale, hipStream_t s);
bool fft_any_supported(int C);
// C = 1536 (frame_td_fft512.hip): LS from FFT'd pilot rows (staging, frame
// stride R*C) into the lane-order Hc + bin-layout P, and the fused MRC.
hipError_t launch_ls_1536(const float2 *Y, long long nframes, int R, const float2 *X, float2 *Hl, float *P,
                          hipStream_t s);
hipError_t launch_mrc_td1536(const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *Hl,
                             const float *P, float2 *out, int mode, hipStream_t s);
// ... and C = 3072 on a wave pair per symbol (same file)
hipError_t launch_ls_3072(const float2 *Y, long long nframes, int R, const float2 *X, float2 *Hl, float *P,
                          hipStream_t s);
hipError_t launch_mrc_td3072(const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *Hl,
                             const float *P, float2 *out, int mode, hipStream_t s);
// ... C = 512 / 256 / 128 on one wave per symbol (same file; other C:
// hipErrorInvalidValue)
hipError_t launch_ls_small(int C, const float2 *Y, long long nframes, int R, const float2 *X, float2 *Hl, float *P,
                           hipStream_t s);
hipError_t launch_mrc_small(int C, const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *Hl,
                            const float *P, float2 *out, int mode, hipStream_t s);
// ... and C = 6144 on a wave quad per symbol (same file)
hipError_t launch_ls_6144(const float2 *Y, long long nframes, int R, const float2 *X, float2 *Hl, float *P,
                          hipStream_t s);
hipError_t launch_mrc_td6144(const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *Hl,
                             const float *P, float2 *out, int mode, hipStream_t s);
// Fused any-C MRC (fft_any.hip k_mrc_any): data symbols of frames
// iq + f*S*R*(C+prefix) (symbols 1..S-1) against the staged estimate in the
// bin layout (Hc [F][R][C], P [F][C]); mode 0: out[q][out_pos_any(j)] =
// sum_r Y*Hc / P, mode 1: out[q][j] = sum_r Y*Hc.
hipError_t launch_mrc_any(const float2 *iq, long long nframes, int S, int R, int C, int prefix, const float2 *Hc,
                          const float *P, float2 *out, int mode, hipStream_t s);

// LS channel estimate on frequency-domain pilot symbols.
// Pilot of frame f: Y + f*frame_stride, R rows of C bins.
// Hconj(f, r, j) at Hc + f*hc_fstride + r*hc_ld + j + hc_jofs  (j = 0..K-1)
// P(f, j)        at P  + f*p_fstride + j + p_jofs
// (reference layout: hc_ld = K, jofs = 0; bin layout: hc_ld = C, jofs = 1).
hipError_t launch_ls_freq(const float2 *Y, long long frame_stride, long long nframes, int R,
                          int C, const float2 *X, float2 *Hc, long long hc_fstride, int hc_ld,
                          int hc_jofs, float *P, long long p_fstride, int p_jofs, hipStream_t s);

// MRC on frequency-domain data symbols.  Data symbol q (q < nframes*nsym)
// belongs to frame q / nsym and lives at
// Y + (q / nsym)*frame_stride + (q % nsym)*sym_stride (R rows of C bins).
// mode 0: full demod  out[q][out_pos(j)] = (sum_r Y*Hc) / P
// mode 1: numerator   out[q][j] = sum_r Y*Hc  (antenna-split partial)
hipError_t launch_mrc_freq(const float2 *Y, long long frame_stride, long long sym_stride,
                           long long nframes, int nsym, int R, int C, const float2 *Hc,
                           long long hc_fstride, int hc_ld, int hc_jofs, const float *P,
                           long long p_fstride, int p_jofs, float2 *out, int mode,
                           hipStream_t s);

// The same combine on the matrix cores (mrc_mfma.hip): bin-layout Hc
// (hc_ld = C, DC slot zero), bin-indexed P (P[f*p_fstride + b]); C >= 64.
hipError_t launch_mrc_freq_mfma(const float2 *Y, long long frame_stride, long long sym_stride,
                                long long nframes, int nsym, int R, int C, const float2 *Hc,
                                long long hc_fstride, const float *P, long long p_fstride,
                                float2 *out, int mode, hipStream_t s);

// Finalise antenna-split numerators: elements [e0, e0+count) of the flat
// [nframes][nsym][K] numerator array (num points at element e0) are divided
// by P[f][j] and stored rotated into out ([nframes][nsym][K], full array).
hipError_t launch_mrc_finalize(const float2 *num, long long e0, long long count, int nsym,
                               int K, const float *P, float2 *out, hipStream_t s);

// Fused time-domain receiver, C = 1024 (32 x 32 wave FFT).
// Frames: iq + f*S*R*(C+prefix); pilot = symbol 0, data = symbols 1..S-1.
// Workspace: Hc [F][R][C] (bin layout), P [F][C].
hipError_t launch_ls_td1024(const float2 *iq, long long nframes, int S, int R, int prefix,
                            const float2 *X, float2 *Hc, float *P, int partial,
                            hipStream_t s);
hipError_t launch_mrc_td1024(const float2 *iq, long long nframes, int S, int R, int prefix,
                             const float2 *Hc, const float *P, float2 *out, int mode,
                             hipStream_t s);
// Both in one grid (frame_td.hip k_demod_td1024): estimator workgroups
// publish each frame's estimate through flags[f] = epoch (agent scope), the
// MRC workgroups wait for it.  flags: nframes words in the workspace; epoch:
// a per-launch value no flag holds.  mode 0 (full demod) only.
hipError_t launch_demod_td1024(const float2 *iq, long long nframes, int S, int R, int prefix, const float2 *X,
                               float2 *Hc, float *P, float2 *out, Tickets tk,
                               unsigned long long *flags, unsigned long long epoch, long long spin_ticks,
                               hipStream_t s);

// Stage-wise operations of the reference's per-stage gpuLS methods (stages.hip).
// fused time-domain receiver, C = 2048 (frame_td2048.hip); same contracts
hipError_t launch_ls_td2048(const float2 *iq, long long nframes, int S, int R, int prefix,
                            const float2 *X, float2 *Hc, float *P, int partial, hipStream_t s);
hipError_t launch_mrc_td2048(const float2 *iq, long long nframes, int S, int R, int prefix,
                             const float2 *Hc, const float *P, float2 *out, int mode, Tickets tk,
                             hipStream_t s);
// fused time-domain receiver, C = 4096 (frame_td4096.hip); same contracts
hipError_t launch_ls_td4096(const float2 *iq, long long nframes, int S, int R, int prefix,
                            const float2 *X, float2 *Hc, float *P, int partial, hipStream_t s);
hipError_t launch_mrc_td4096(const float2 *iq, long long nframes, int S, int R, int prefix,
                             const float2 *Hc, const float *P, float2 *out, int mode, Tickets tk,
                             hipStream_t s);
hipError_t launch_conj_product(const float2 *Y, long long nsyms, int R, int C, const float2 *Hc,
                               float2 *prod, hipStream_t s);
hipError_t launch_combine(const float2 *prod, long long nsyms, int R, int K, const float *P,
                          int rotate, float2 *out, hipStream_t s);
hipError_t launch_shift_rows(const float2 *in, long long nrows, int K, float2 *out, hipStream_t s);
hipError_t launch_hash_words(const void *d, long long nwords, unsigned long long *h, hipStream_t s);
hipError_t launch_zero_words(unsigned long long *p, int n, hipStream_t s);
hipError_t launch_dist_sqrd(const float2 *H, int R, int K, float *P, hipStream_t s);
// One frame's workspace estimate (Hc rows of C float2: lane_order = the
// fused LS kernel for C wrote them, else bin layout; P bin-indexed) ->
// Hconj [R][K], Hsqrd [K] (may be null).
hipError_t launch_export_estimate(const float2 *Hc, const float *P, int R, int C, bool lane_order,
                                  float2 *Hconj, float *Hsqrd, hipStream_t s);

// Synthetic frames: time-domain (freq_domain=0, rows of C+prefix with a
// cyclic prefix) or frequency-domain (freq_domain=1, rows of C) IQ.
hipError_t launch_synth(float2 *iq, long long nframes, int S, int R, int C, int prefix,
                        const float2 *X, uint64_t seed, long long frame0, float noise_std,
                        int freq_domain, int r0, hipStream_t s);
// Hard-decision QPSK errors of demodulated output against the synthetic data.
// HBM probes (bench.py): mode 0 float4 copy src -> dst, mode 1 float4 read
// of src (dst: 1024 x 256 floats of sums); n4 float4s
hipError_t launch_hbm_probe(int mode, const void *src, void *dst, long long n4, hipStream_t s);
hipError_t launch_count_errors(const float2 *out, long long nframes, int S, int C,
                               uint64_t seed, long long frame0, unsigned long long *errors,
                               hipStream_t s);

// PN frame sync (pn_sync.hip): first (channel, lag) whose |correlation| / L
// reaches thres, as ch * (N-L+1) + lag in *pos (-1: none); mag optional.
hipError_t launch_pn_correlate(const float2 *buf, int R, long long N, const float2 *pn, int L,
                               float thres, long long *pos, float *mag, hipStream_t s);
hipError_t launch_pn_extract(const float2 *buf1, const float2 *buf2, int R, long long N, int L,
                             const long long *pos, int C, int cp, int nsym, float2 *sym,
                             hipStream_t s);

// Zero forcing (zf.hip).  Hin [U][R][K]; W [K][U][R] (reference layout, may be
// null); Wt [U][R][K] (subcarrier-fastest, may be null).  1 <= U <= 32,
// U*R <= 8192 (checked by capi.cpp).
size_t zf_precoder_lds_bytes(int U, int R);
hipError_t launch_zf_precoder(const float2 *Hin, int U, int R, int K, float2 *W, float2 *Wt,
                              hipStream_t s);
hipError_t launch_zf_transpose(const float2 *W, int U, int R, int K, float2 *Wt, hipStream_t s);
// apply: Y[s][r][k] = sum_u W(r,u) X[s][u][k]; detect: X[s][u][k] = sum_r conj(W(r,u)) Y[s][r][k]
hipError_t launch_zf_apply(const float2 *Wt, const float2 *X, int U, int R, int K, long long nsym,
                           float2 *Y, hipStream_t s);
hipError_t launch_zf_detect(const float2 *Wt, const float2 *Y, int U, int R, int K, long long nsym,
                            float2 *X, hipStream_t s);
// ... with row pitches (elements, >= K); pitched apply: K >= 2, R >= 8, U <= 40
bool zf_apply_pitched_supported(int U, int R, int K);
hipError_t launch_zf_apply_ld(const float2 *Wt, const float2 *X, long long ldx, int U, int R, int K, long long nsym,
                              float2 *Y, long long ldy, hipStream_t s);
// ... with row pitches ldy / ldx (elements, >= K); pitched calls need R <= 72
bool zf_detect_pitched_supported(int U, int R);
hipError_t launch_zf_detect_ld(const float2 *Wt, const float2 *Y, long long ldy, int U, int R, int K,
                               long long nsym, float2 *X, long long ldx, hipStream_t s);

}  // namespace ofdm
