/*
 * ofdm_oracle.h -- CPU restatement of the reference's LS + MRC receiver path.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (the HIP library under
 * gpu-accel-ofdm-ls-mrc_amd/) links, calls or executes this code.  Only tests/,
 * __graft_entry__.smoke() and bench.py's `cpu_baseline` leg may load it, and
 * only as the checker / the timed CPU baseline.
 *
 * Every function cites the reference file:line it restates (paths are into the
 * read-only reference checkout, bhargav0410/gpu-accel-ofdm-ls-mrc).
 *
 * Parity pinning (see DESIGN.md "Oracle"):
 *   - the post-FFT arithmetic (pilot rotation, LS divide, conj, |H|^2, MRC sum,
 *     normalise, output rotation) is checked bit-for-bit against the reference's
 *     own functions compiled from /root/reference/cpuLS.hpp by
 *     oracle/build_ref.sh (oracle/_ref/), and through them against the golden
 *     fixtures in tests/golden/;
 *   - the FFT stage belongs to FFTW3 (single precision, version unpinned by the
 *     reference, absent from this image): it is restated as the exact DFT
 *     (double-precision radix-2, rounded to float) and pinned against numpy's
 *     pocketfft in float64.
 *
 * Complex layout: interleaved {float re, float im} -- identical to the
 * reference's complexF (ShMemSymBuff.hpp:86-89), cuFloatComplex and
 * hipFloatComplex.
 */
#ifndef OFDM_ORACLE_H_
#define OFDM_ORACLE_H_

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { float re, im; } oracle_cf32;

/* matrix_readX rotation (cpuLS.hpp:105-112): X[j] = raw[(j + (K+1)/2) mod K]
 * for odd K (literal memmove semantics for any K). */
void oracle_pilot_rotate(const oracle_cf32 *raw, int K, oracle_cf32 *X);

/* shiftOneRow (cpuLS.hpp:135-149) on one row of K values, in place. */
void oracle_shift_one_row(oracle_cf32 *row, int K);

/* fftOneRow (cpuLS.hpp:165-174): unnormalised forward DFT (sign -1), in place,
 * on one row of C values.  inverse!=0 gives the unnormalised backward DFT
 * (ifftOneRow, cpuLS.hpp:152-162).  C must be a power of two. */
void oracle_fft_row(oracle_cf32 *row, int C, int inverse);

/* firstVector post-FFT part (cpuLS.hpp:290-311): drop DC, divideOneRow,
 * conjugate, findDistSqrd.  Yfft: R x C (already FFT'd), X: K rotated pilots.
 * Outputs Hconj: R x K, Hsqrd: K floats (the reference keeps it in X[j].real). */
void oracle_ls(const oracle_cf32 *Yfft, const oracle_cf32 *X, int R, int C,
               oracle_cf32 *Hconj, float *Hsqrd);

/* doOneSymbol post-FFT part (cpuLS.hpp:354-368): drop DC, matrixMultThenSum,
 * divide by Hsqrd, shiftOneRow.  out: K values. */
void oracle_mrc(const oracle_cf32 *Yfft, const oracle_cf32 *Hconj,
                const float *Hsqrd, int R, int C, oracle_cf32 *out);

/* MRC numerator only (matrixMultThenSum, cpuLS.hpp:187-208), bins j=0..K-1,
 * for antennas [0, R): used to check the antenna-split partial path. */
void oracle_mrc_numerator(const oracle_cf32 *Yfft, const oracle_cf32 *Hconj,
                          int R, int C, oracle_cf32 *num);

/* One frame, time-domain input (firstVector + doOneSymbol loop,
 * cpuLS_main.cpp:80-92, with symbol 0 read as the pilot as gpuLS::firstVector
 * does, gpuLS.cu:359): iq is S symbols x R rows x (C+prefix) samples; the
 * cyclic prefix is dropped as ShMemSymBuff::readNextSymbol does
 * (ShMemSymBuff.hpp:281-322).  out: (S-1) x K.  Hconj/Hsqrd may be NULL. */
void oracle_frame_demod(const oracle_cf32 *iq, int S, int R, int C, int prefix,
                        const oracle_cf32 *X, oracle_cf32 *out,
                        oracle_cf32 *Hconj, float *Hsqrd);

/* nframes consecutive frames, OpenMP over frames with nthreads threads
 * (nthreads<=0: OpenMP default).  Used as the timed CPU baseline. */
void oracle_frames_demod(const oracle_cf32 *iq, long long nframes, int S, int R,
                         int C, int prefix, const oracle_cf32 *X,
                         oracle_cf32 *out, int nthreads);

/* The same receiver with a single-precision radix-2 FFT (oracle_fft_row_f32,
 * the precision of the reference's fftwf): the timed CPU baseline of
 * bench.py.  Not a parity path (oracle_frames_demod is). */
void oracle_fft_row_f32(oracle_cf32 *row, int C);
/* bench.py's CPU baseline only (fft_fast.c): the same transform, vectorised
 * (split arrays, unit-stride per-stage twiddles, -O3 -march=x86-64-v3) */
void oracle_fft_row_fast(oracle_cf32 *row, int C);
void oracle_frames_demod_fftfast(const oracle_cf32 *iq, long long nframes, int S, int R, int C, int prefix,
                                 const oracle_cf32 *X, oracle_cf32 *out, int nthreads);
void oracle_frames_demod_fft32(const oracle_cf32 *iq, long long nframes, int S, int R,
                               int C, int prefix, const oracle_cf32 *X,
                               oracle_cf32 *out, int nthreads);

/* Frequency-domain frames (FFT already applied, no prefix): pilot + (S-1)
 * data symbols of R x C each.  OpenMP over frames. */
void oracle_frames_demod_freq(const oracle_cf32 *yf, long long nframes, int S,
                              int R, int C, const oracle_cf32 *X,
                              oracle_cf32 *out, int nthreads);

int oracle_max_threads(void);

/* ---- PN frame-sync correlator (pn_oracle.c; rx_and_corr.cpp) ----------- */

/* rx_and_corr.cpp:332-360: for channel ch = 0.. and lag i = 0..N-L, in that
 * order, temp = sum_j pn[j] * buf[ch][i+j] (std::complex<float>, sequential
 * j), v = std::abs(temp) / (float)L; the first (ch, i) with v >= thres stops
 * the search.  *pos = ch * (N-L+1) + i, or -1 if no lag reaches thres.  If
 * mag != NULL every lag of every channel is evaluated (no early exit) and
 * mag[ch * (N-L+1) + i] = v; *pos is the same. */
void oracle_pn_correlate(const oracle_cf32 *buf, int R, long long N,
                         const oracle_cf32 *pn, int L, float thres,
                         long long *pos, float *mag);

/* Frame extraction after a hit at lag `lag` (rx_and_corr.cpp:370-392, then
 * copy_to_shared_mem 64-87): per channel the sequence seq = buf1[ch][lag+L ..
 * N) followed by buf2[ch][0 .. lag) (N-L samples) is cut into nsym symbols of
 * C+cp samples with the cyclic prefix dropped:
 *   sym[s][ch][k] = seq[s*(C+cp) + cp + k],  s < nsym, k < C.
 * Requires nsym*(C+cp) <= N-L. */
void oracle_pn_extract(const oracle_cf32 *buf1, const oracle_cf32 *buf2, int R,
                       long long N, int L, long long lag, int C, int cp,
                       int nsym, oracle_cf32 *sym);

/* ---- zero-forcing precoder (zf_oracle.c; cpuLS.hpp:401-466) ------------ */

/* createZeroForcingMatrix (cpuLS.hpp:415-449) for K = cols-1 subcarriers:
 * Hin: users x rows x K channel cube (the layout before rotCube, 401-413; not
 * modified here).  Per subcarrier A[u][r] = Hin[u][r][k], G = A A^H
 * (cblas_cgemm NoTrans/ConjTrans), G^-1 by LU with partial pivoting (cgetrf:
 * unblocked, pivot = max |re|+|im|) and the LU inverse (cgetri), then
 * W = A^H G^-1 (cgemm ConjTrans/NoTrans) stored as the reference's H:
 * W[k*rows*users + u*rows + r]. */
void oracle_zf_precoder(const oracle_cf32 *Hin, int users, int rows, int K, oracle_cf32 *W);

/* multiplyWithChannelInv (cpuLS.hpp:451-466, cblas_cgemv per subcarrier) with
 * the intended operands (modOneSymbol passes them swapped, 494): for nsym
 * symbols, Y[s][r][k] = sum_u W[k][u][r] X[s][u][k]. */
void oracle_zf_apply(const oracle_cf32 *W, const oracle_cf32 *X, int users, int rows, int K,
                     int nsym, oracle_cf32 *Y);

/* The uplink counterpart (no reference function): ZF detection with the same
 * W, x[s][u][k] = sum_r conj(W[k][u][r]) Y[s][r][k] (W^H = G^-1 A, the
 * pseudo-inverse of the R x U uplink channel A^H). */
void oracle_zf_detect(const oracle_cf32 *W, const oracle_cf32 *Y, int users, int rows, int K,
                      int nsym, oracle_cf32 *X);

#ifdef __cplusplus
}
#endif
#endif
