/*
 * ofdm_lsmrc.h -- C ABI of the MI355X (gfx950) OFDM uplink receiver hot path:
 * per-subcarrier Least-Squares channel estimation from a pilot symbol and
 * Maximal-Ratio-Combining demodulation of data symbols across RX antennas.
 *
 * Library: gpu-accel-ofdm-ls-mrc_amd/lib/libofdm_lsmrc.so (hand-written HIP
 * kernels for CDNA4; no CPU fallback -- every compute entry point runs on the
 * GPU and returns an error if it cannot).
 *
 * Conventions (all cite the reference bhargav0410/gpu-accel-ofdm-ls-mrc):
 *   R  = RX antennas (numOfRows), C = FFT size / subcarriers (dimension:
 *        any 2 <= C <= 8192, like the reference's FFTW / cuFFT plans; else
 *        OFDM_E_UNSUPPORTED), K = C - 1 used subcarriers (the DC bin is dropped,
 *        cpuLS.hpp:290-292), S = symbols per frame (lenOfBuffer), symbol 0 of
 *        a frame is the pilot, symbols 1..S-1 carry data.
 *   ofdm_cf32 = {float re, im}, layout-identical to complexF
 *        (ShMemSymBuff.hpp:86-89), cuFloatComplex and hipFloatComplex.
 *   A symbol is R rows of C (+prefix) samples, row-major by antenna
 *        (struct symbol, ShMemSymBuff.hpp:92-94); frames are consecutive
 *        symbols, batches are consecutive frames.
 *   Output of a data symbol: K values, shiftOneRow-rotated (cpuLS.hpp:135-149):
 *        out[k] = Z[(k + (K-1)/2) mod K], Z[j] = sum_r Y[r][j+1] conj(H[r][j])
 *        / sum_r |H[r][j]|^2, for odd K (even C); for even K (odd C) the
 *        three memmoves of shiftOneRow literally: out[k] = Z[k + K/2 - 1] for
 *        k < K/2, Z[k - K/2] for K/2 <= k < K-1, and out[K-1] = Z[K-1].
 *   Pointers named d_* are device pointers; `stream` is a hipStream_t (NULL =
 *   the default stream).  Calls are asynchronous on that stream.
 *   Return value: 0 (OFDM_OK) or a negative OFDM_E_* code; ofdm_last_error()
 *   describes the last failure on the calling thread.
 */
#ifndef OFDM_LSMRC_H_
#define OFDM_LSMRC_H_

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: ofdm_hbm_probe takes dst_bytes; OFDM_E_DEVICE, ofdm_device_status(_inject),
 *    ofdm_zf_detect_ex / ofdm_zf_apply_ex added (round 6) */
#define OFDM_LSMRC_VERSION 2

typedef struct ofdm_cf32 { float re, im; } ofdm_cf32;
typedef void *ofdm_stream_t; /* hipStream_t */

enum {
    OFDM_OK = 0,
    OFDM_E_ARG = -1,         /* invalid argument (shape, null, alignment) */
    OFDM_E_HIP = -2,         /* HIP runtime / launch failure */
    OFDM_E_UNSUPPORTED = -3, /* shape not supported by this build */
    OFDM_E_IO = -4,          /* file I/O */
    OFDM_E_DEVICE = -5       /* an EARLIER launch reported a fault from the device (see
                                ofdm_device_status); its output may be incomplete */
};

int ofdm_version(void);
const char *ofdm_last_error(void);

/* ---------------------------------------------------------------- host --- */

/* Pilot rotation of matrix_readX (cpuLS.hpp:105-112, gpuLS.cu:75-82):
 * X[j] = raw[(j + (K+1)/2) mod K].  raw may equal X. */
int ofdm_pilot_rotate(const ofdm_cf32 *raw, int K, ofdm_cf32 *X);

/* matrix_readX (cpuLS.hpp:80-117 / gpuLS::matrix_readX, gpuLS.cu:53-86):
 * read K raw complex floats from `path` and rotate.  If the file cannot be
 * opened every X[j] = fill + i*fill (the reference uses 0.707 on the CPU path,
 * cpuLS.hpp:84-90, and 1.0 on the GPU path, gpuLS.cu:57-63) and 1 is
 * returned. */
int ofdm_read_pilots(const char *path, int K, float fill, ofdm_cf32 *X);

/* ------------------------------------------------------ device: stages --- */

/* Batched forward (inverse != 0: backward) unnormalised C2C FFT of nrows
 * contiguous rows of C samples, in place or out of place.
 * Replaces gpuLS::batchedFFT (gpuLS.cu:343-349) / cufftPlan1d + cufftExecC2C
 * (gpuLS.cu:377-381, 441-445) and fftOneRow (cpuLS.hpp:165-174).
 * Any 2 <= C <= 8192: powers of two up to 4096 by radix-4 Stockham stages,
 * every other length by mixed-radix stages (radices 8, 4, 2, 3, 5, 7 and a
 * direct stage with double accumulation for larger prime factors). */
int ofdm_fft_rows(const ofdm_cf32 *d_in, ofdm_cf32 *d_out, long long nrows, int C, int inverse,
                  ofdm_stream_t stream);

/* LS channel estimate from one frequency-domain pilot symbol d_Y (R x C,
 * bin 0 = DC) and the rotated pilots d_X (K values):
 *   d_Hconj[r][j] = conj(Y[r][j+1] / X[j])  (R x K)
 *   d_Hsqrd[j]    = sum_r |Hconj[r][j]|^2   (K floats)
 * Replaces findHs (gpuLS.cu:158-182) + findDistSqrd (gpuLS.cu:185-209) and
 * the post-FFT part of firstVector (cpuLS.hpp:290-311). */
int ofdm_ls_estimate(const ofdm_cf32 *d_Y, const ofdm_cf32 *d_X, int R, int C, ofdm_cf32 *d_Hconj,
                     float *d_Hsqrd, ofdm_stream_t stream);

/* MRC demodulation of nsyms frequency-domain symbols d_Y (nsyms x R x C)
 * against one estimate: d_out (nsyms x K) = rotated sum_r Y Hconj / Hsqrd.
 * Replaces multiplyWithChannelConj + combineForMRC + shiftOneRow
 * (gpuLS.cu:109-125, 212-259) and the post-FFT part of doOneSymbol
 * (cpuLS.hpp:354-368). */
int ofdm_mrc_demod(const ofdm_cf32 *d_Y, long long nsyms, const ofdm_cf32 *d_Hconj,
                   const float *d_Hsqrd, int R, int C, ofdm_cf32 *d_out, ofdm_stream_t stream);

/* MRC numerator only (matrixMultThenSum, cpuLS.hpp:187-208):
 * d_num (nsyms x K, subcarrier order, not rotated) = sum_r Y[r][j+1] Hconj[r][j].
 * With a subset of antennas this is the partial numerator of the antenna-split
 * multi-GPU path. */
int ofdm_mrc_numerator(const ofdm_cf32 *d_Y, long long nsyms, const ofdm_cf32 *d_Hconj, int R,
                       int C, ofdm_cf32 *d_num, ofdm_stream_t stream);

/* Finalise (summed) numerators: elements [e0, e0+count) of a flat
 * [nframes][nsym][K] numerator array (d_num points at element e0) are divided
 * by d_Hsqrd[f][j] ([nframes][K]) and stored rotated into d_out, the full
 * [nframes][nsym][K] output array.  (combineForMRC's divide + shiftOneRow,
 * gpuLS.cu:254-256, 109-125.) */
int ofdm_mrc_finalize(const ofdm_cf32 *d_num, long long e0, long long count, int nsym, int K,
                      const float *d_Hsqrd, ofdm_cf32 *d_out, ofdm_stream_t stream);

/* Stage-wise operations behind the reference's per-stage GPU methods, which
 * materialise their intermediates (the fused entry points above do not):
 *   ofdm_channel_conj_product: d_prod[s][r][j] = Y[s][r][j+1] * Hconj[r][j]
 *       (nsyms x R x K; multiplyWithChannelConj, gpuLS.cu:212-233)
 *   ofdm_combine_products: d_out[s][k] = sum_r prod[s][r][j] / Hsqrd[j], at
 *       k = rotated position of j if rotate != 0, else k = j
 *       (combineForMRC [+ shiftOneRow], gpuLS.cu:236-259, 109-125)
 *   ofdm_shift_rows: shiftOneRow on nrows device rows of K, out of place
 *       (gpuLS.cu:109-125, cpuLS.hpp:135-149)
 *   ofdm_dist_sqrd: d_Hsqrd[j] = sum_r |H[r][j]|^2 of an R x K matrix
 *       (findDistSqrd, gpuLS.cu:185-209, cpuLS.hpp:211-228) */
int ofdm_channel_conj_product(const ofdm_cf32 *d_Y, long long nsyms, const ofdm_cf32 *d_Hconj,
                              int R, int C, ofdm_cf32 *d_prod, ofdm_stream_t stream);
int ofdm_combine_products(const ofdm_cf32 *d_prod, long long nsyms, const float *d_Hsqrd, int R,
                          int K, int rotate, ofdm_cf32 *d_out, ofdm_stream_t stream);
int ofdm_shift_rows(const ofdm_cf32 *d_in, long long nrows, int K, ofdm_cf32 *d_out,
                    ofdm_stream_t stream);
int ofdm_dist_sqrd(const ofdm_cf32 *d_H, int R, int K, float *d_Hsqrd, ofdm_stream_t stream);

/* ------------------------------------------------------ device: frames --- */

/* Workspace for ofdm_frame_demod / ofdm_frame_demod_freq and the two-stage
 * and antenna-split calls (bytes, 256-aligned pieces): per-frame channel
 * estimates [F][R][C], |H|^2 [F][C], one 64-bit word per frame (the
 * estimate flags of the one-launch C = 1024 demod below) and, for C outside
 * {1024, 2048, 4096}
 * (no fused kernel), a frequency-domain staging buffer of at most 256 MiB.
 * A workspace carries the estimate of ONE geometry: the calls that consume it
 * (ofdm_frame_combine, ofdm_frame_mrc_partial, ofdm_frame_export_estimate)
 * must pass the nframes, S, R, C and ws_bytes of the call that filled it, and
 * return OFDM_E_ARG otherwise (checked per process, on the host, by a registry
 * keyed on d_ws).  An estimate call clears the workspace's entry before it
 * launches and records it only after every launch was enqueued, so a failed
 * estimate leaves a workspace that the consumers refuse. */
size_t ofdm_frame_workspace_bytes(long long nframes, int S, int R, int C);

/* Work tickets.  The C = 1024 one-launch demod and the C = 2048 / 4096 MRC
 * kernels (ofdm_frame_demod, _combine, _mrc_partial(_range),
 * ofdm_symbols_demod) deal their blocks to workgroups at run time through 8
 * counter words in the workspace (after the flag words).  These entry points
 * therefore WRITE the workspace, ofdm_symbols_demod's const d_ws included.
 * A counter holds tag << 32 | count with a per-launch tag, so whatever the
 * words hold when a launch starts (zeros, an earlier launch's counts, an
 * estimate of another geometry, recycled memory) is claimed afresh and never
 * consumed as a count: no zeroing, release or registry state is needed for
 * them.  One workspace serves one launch at a time (one stream, as for its
 * estimate).  Two ticketed launches that overlap on one workspace either
 * both complete (a block may be processed twice: same bytes) or one of them
 * sees the other's tag and raises the sticky device status below.
 *
 * Sticky device status: a library-owned, host-mapped word that ticketed
 * launches set when they meet a counter they cannot trust.  Every ticketed
 * entry point reads it first (no synchronisation) and, if set, clears it and
 * returns OFDM_E_DEVICE without launching anything; ofdm_device_status()
 * does the same on demand (synchronise the stream first to see the status of
 * launches still in flight).  ofdm_device_status_inject() ORs `bits` into
 * the status (tests of the reporting path; no device needed). */
int ofdm_device_status(void);
int ofdm_device_status_inject(unsigned bits);

/* Drops what the registry above knows about d_ws.  Call it before the memory
 * is freed (or handed to another user): a workspace later allocated at the
 * same address then holds no estimate until an estimate call fills it, and
 * the consumers return OFDM_E_ARG instead of dividing by a stale |H|^2.  The
 * Python binding calls it from the workspace tensor's finaliser.  NULL or an
 * unknown pointer is a no-op; always returns OFDM_OK. */
int ofdm_workspace_release(const void *d_ws);

/* Frame-batched receiver on time-domain IQ (what ShMemSymBuff delivers):
 * d_iq = nframes x S x R x (C + cp_len) samples; the cyclic prefix of every
 * row is skipped (ShMemSymBuff.hpp:309-322), each row is FFT'd, symbol 0 of
 * each frame gives the LS estimate, symbols 1..S-1 are MRC-demodulated into
 * d_out = nframes x (S-1) x K.  Replaces demodOneFrameCUDA / demodOptimized
 * (gpuLS.cu:575-769) and the cpuLS_main loop (cpuLS_main.cpp:80-92), for a
 * whole batch of frames in one call.  C in {1024, 2048, 4096} runs the fused
 * one-pass kernels (FFT + LS, FFT + MRC + normalise + rotate); at C = 1024
 * both run in ONE launch (estimator workgroups publish each frame's estimate
 * to the MRC workgroups through the workspace's flag words, agent-scope
 * release/acquire), except on a stream being captured into a graph, where
 * the two launches are used.  Every other C in [2, 8192] runs FFT, LS
 * and MRC as stages through the workspace's staging buffer. */
int ofdm_frame_demod(const ofdm_cf32 *d_iq, long long nframes, int S, int R, int C, int cp_len,
                     const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes, ofdm_cf32 *d_out,
                     ofdm_stream_t stream);

/* ofdm_frame_demod with its two scheduling choices exposed (same results,
 * same workspace contract):
 *   flow        OFDM_FLOW_AUTO (what ofdm_frame_demod does) or
 *               OFDM_FLOW_TWO_LAUNCH (estimate, then combine, as two launches
 *               on the stream, at every C);
 *   spin_ticks  one-launch path (C = 1024): how long, in ticks of the 100 MHz
 *               device clock, an MRC workgroup waits for the estimate of a
 *               frame it reads before it estimates that frame itself (the
 *               same code and bytes as the estimator workgroup); < 0 = the
 *               default (200 000 = 2 ms), 0 = never wait.  The result does
 *               not depend on it; a shared GPU that delays the estimator
 *               workgroups only trades the wait for a re-estimate. */
#define OFDM_FLOW_AUTO 0
#define OFDM_FLOW_TWO_LAUNCH 1
int ofdm_frame_demod_ex(const ofdm_cf32 *d_iq, long long nframes, int S, int R, int C, int cp_len,
                        const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes, ofdm_cf32 *d_out, int flow,
                        long long spin_ticks, ofdm_stream_t stream);

/* The two stages of ofdm_frame_demod, for callers that pipeline or time them
 * separately: ofdm_frame_estimate FFTs the pilot symbol of every frame and
 * stores the LS estimate (Hconj, |H|^2) in d_ws (gpuLS::firstVector,
 * gpuLS.cu:351-408, per frame); ofdm_frame_combine MRC-demodulates the data
 * symbols against it (gpuLS::demodOneSymbol, gpuLS.cu:410-473, per symbol).
 * ofdm_frame_demod == estimate then combine on the same stream. */
int ofdm_frame_estimate(const ofdm_cf32 *d_iq, long long nframes, int S, int R, int C, int cp_len,
                        const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes, ofdm_stream_t stream);
int ofdm_frame_combine(const ofdm_cf32 *d_iq, long long nframes, int S, int R, int C, int cp_len,
                       void *d_ws, size_t ws_bytes, ofdm_cf32 *d_out, ofdm_stream_t stream);

/* One frame's LS estimate out of a workspace filled by ofdm_frame_estimate /
 * ofdm_frame_demod / ofdm_frame_demod_freq / ofdm_frame_ls_partial (same
 * nframes, S, R, C), in the reference's layout: d_Hconj[r][j] = conj(Y0/X)
 * (R x K), d_Hsqrd[j] = sum_r |Hconj[r][j]|^2 (K floats; NULL = not wanted;
 * for an ls_partial workspace the local antennas' partial sum).  These are
 * the Hconj / Hsqrd outputs of demodOneFrameCUDA (gpuLS.cu:617-629) and
 * firstVector (gpuLS.cu:392-395), which the fused kernels keep in their own
 * lane order. */
int ofdm_frame_export_estimate(const void *d_ws, size_t ws_bytes, long long nframes, int S, int R, int C,
                               long long frame, ofdm_cf32 *d_Hconj, float *d_Hsqrd, ofdm_stream_t stream);

/* Per-symbol receiver (gpuLS::demodOneSymbol, gpuLS.cu:410-473, which runs
 * cuFFT + multiplyWithChannelConj + combineForMRC + a CPU shift per symbol):
 * nsym consecutive time-domain data symbols d_sym (nsym x R x (C + cp_len),
 * each row's cyclic prefix skipped) demodulated against the LS estimate of
 * frame `frame` of a workspace filled by ofdm_frame_estimate (any nframes and
 * S; R, C and ws_bytes must match), in ONE fused launch (FFT + MRC +
 * normalise + rotate, each row read once) -> d_out (nsym x K).  C in {1024,
 * 2048, 4096} (else OFDM_E_UNSUPPORTED); a frequency-domain or partial
 * estimate is refused with OFDM_E_ARG. */
int ofdm_symbols_demod(const ofdm_cf32 *d_sym, long long nsym, int R, int C, int cp_len, const void *d_ws,
                       size_t ws_bytes, long long frame, ofdm_cf32 *d_out, ofdm_stream_t stream);

/* ofdm_frame_demod on frequency-domain symbols (FFT done upstream, no prefix):
 * d_Y = nframes x S x R x C.  The LS + MRC of the reference's GPU path on
 * its own (findHs + findDistSqrd, gpuLS.cu:158-209; multiplyWithChannelConj +
 * combineForMRC + shiftOneRow, gpuLS.cu:109-125, 212-259, per frame as in
 * demodOneFrameCUDA, gpuLS.cu:575-675, after its cuFFT). */
int ofdm_frame_demod_freq(const ofdm_cf32 *d_Y, long long nframes, int S, int R, int C,
                          const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes, ofdm_cf32 *d_out,
                          ofdm_stream_t stream);

/* Its two stages (as ofdm_frame_estimate / ofdm_frame_combine): the LS
 * estimate of every frame's pilot symbol into d_ws, then the MRC of the data
 * symbols against it.  At every C that has a fused time-domain receiver --
 * 128, 256, 512, 1024, 1536, 2048, 3072, 4096, 6144 -- the time-domain
 * ofdm_frame_estimate leaves its estimate in that receiver's lane order:
 * ofdm_frame_combine_freq refuses such a workspace and ofdm_frame_combine
 * refuses one filled here, with OFDM_E_ARG.  (Until round 4, C = 128 / 256 /
 * 512 had no fused receiver and their time-domain estimates were in the bin
 * layout, which ofdm_frame_combine_freq accepted.)  At every other C both
 * estimators write the bin layout, and each combine accepts either one. */
int ofdm_frame_estimate_freq(const ofdm_cf32 *d_Y, long long nframes, int S, int R, int C,
                             const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes, ofdm_stream_t stream);
int ofdm_frame_combine_freq(const ofdm_cf32 *d_Y, long long nframes, int S, int R, int C, void *d_ws,
                            size_t ws_bytes, ofdm_cf32 *d_out, ofdm_stream_t stream);

/* ofdm_frame_demod_freq with the antenna combine on the matrix cores: per
 * subcarrier the (S-1) x R x R-by-1 product sum_r Y[s][r] Hconj[r] as
 * v_mfma_f32 tiles (mrc_mfma.hip) -- the MFMA-cgemm formulation BASELINE
 * configs[4] asks to compare with the elementwise combine.  Same results
 * within f32 rounding (antenna order per MFMA block); C >= 64. */
int ofdm_frame_demod_freq_mfma(const ofdm_cf32 *d_Y, long long nframes, int S, int R, int C,
                               const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes, ofdm_cf32 *d_out,
                               ofdm_stream_t stream);

/* Antenna-split pieces (time-domain frames holding this GPU's R antennas):
 * partial |H|^2 per frame into d_P ([nframes][K], sum over the local
 * antennas; sum the partials across GPUs), and partial MRC numerators
 * d_num ([nframes][S-1][K], subcarrier order; sum across GPUs, then
 * ofdm_mrc_finalize).  d_ws as for ofdm_frame_demod. */
int ofdm_frame_ls_partial(const ofdm_cf32 *d_iq, long long nframes, int S, int R, int C, int cp_len,
                          const ofdm_cf32 *d_X, void *d_ws, size_t ws_bytes, float *d_P,
                          ofdm_stream_t stream);
int ofdm_frame_mrc_partial(const ofdm_cf32 *d_iq, long long nframes, int S, int R, int C,
                           int cp_len, void *d_ws, size_t ws_bytes, ofdm_cf32 *d_num,
                           ofdm_stream_t stream);
/* ofdm_frame_mrc_partial for frames [f0, f0 + count) of a batch of nframes
 * whose estimate ONE ofdm_frame_ls_partial call put in d_ws (no reference
 * counterpart: the pipelined antenna split estimates the whole batch in one
 * launch and streams the MRC in chunks).  d_iq is the whole batch, d_num
 * [count][S-1][K].  OFDM_E_ARG for a range outside [0, nframes). */
int ofdm_frame_mrc_partial_range(const ofdm_cf32 *d_iq, long long nframes, long long f0, long long count, int S,
                                 int R, int C, int cp_len, void *d_ws, size_t ws_bytes, ofdm_cf32 *d_num,
                                 ofdm_stream_t stream);

/* ---------------------------------------------------- streaming ingest --- */

/* Pipelined receiver for IQ that lives in HOST memory (the ShMemSymBuff ring,
 * a capture file): SURVEY.md 8(f) rank 2.  `depth` device slots of
 * `chunk_frames` frames each cycle through three HIP streams -- host->device
 * copy, compute (ofdm_frame_demod), device->host copy of the outputs -- so
 * PCIe traffic in both directions overlaps the kernels.  Replaces the
 * reference's per-symbol copy + sync on a fresh stream
 * (readNextSymbolCUDA, ShMemSymBuff_gpu.hpp:375-447; createStream 364-368)
 * and the host staging of demodOneFrame (gpuLS.cu:475-573).
 *   ofdm_pipeline_create: geometry as ofdm_frame_demod; X = the K rotated
 *       pilots (host or device pointer, copied).  Device = the current one.
 *   ofdm_pipeline_acquire: the next slot's device IQ buffer (chunk_frames x S
 *       x R x (C+cp_len)) and the copy stream; the caller enqueues its own
 *       host->device copies on that stream (the ring reader does), then
 *   ofdm_pipeline_submit: demodulates the first nframes frames of that slot
 *       and copies the nframes x (S-1) x K outputs to `out` (host or device;
 *       NULL = leave them in the slot) on the output stream.
 *   ofdm_pipeline_demod: acquire + copy + submit over nframes host frames.
 *   ofdm_pipeline_sync: waits for everything submitted.
 * Each call makes the pipeline's device current and restores the caller's
 * current device before returning.  A failed submit releases its slot (those
 * frames are not demodulated); the pipeline stays usable.
 * Calls return before the copies finish: `iq` and `out` must stay valid until
 * ofdm_pipeline_sync.  For copies that overlap, host buffers must be
 * page-locked (ofdm_host_register); pageable buffers work but serialise. */
typedef struct ofdm_pipeline ofdm_pipeline;
int ofdm_pipeline_create(int S, int R, int C, int cp_len, const ofdm_cf32 *X, int chunk_frames,
                         int depth, ofdm_pipeline **out);
int ofdm_pipeline_destroy(ofdm_pipeline *p);
int ofdm_pipeline_acquire(ofdm_pipeline *p, ofdm_cf32 **d_iq, ofdm_stream_t *copy_stream);
int ofdm_pipeline_submit(ofdm_pipeline *p, long long nframes, ofdm_cf32 *out);
int ofdm_pipeline_demod(ofdm_pipeline *p, const ofdm_cf32 *iq, long long nframes,
                        ofdm_cf32 *out);
int ofdm_pipeline_sync(ofdm_pipeline *p);

/* Page-lock / release a host range for asynchronous DMA (hipHostRegister). */
int ofdm_host_register(void *p, size_t bytes);
int ofdm_host_unregister(void *p);

/* ------------------------------------------------------ PN frame sync --- */

/* Frame synchronisation of the receive driver, on
 * the device.  ofdm_pn_correlate replaces the sliding correlator of
 * rx_and_corr.cpp:332-360: for channel ch = 0..R-1 and lag i = 0..N-L in that
 * order, v = |sum_j pn[j] * buf[ch][i+j]| / L (no conjugate, as the
 * reference); the first (ch, i) with v >= thres is the hit.  d_buf: R rows of
 * N samples; d_pn: L samples.  *d_pos (device) = ch * (N-L+1) + i, or -1 if
 * no lag reaches thres.  d_mag (optional, R x (N-L+1) floats, NULL = not
 * stored) receives v for every lag (then no lag is skipped).  The index is
 * bit-exact with the reference: each lag is summed in its f32 order.
 *
 * ofdm_pn_extract replaces the copy_buff assembly (rx_and_corr.cpp:370-392)
 * and copy_to_shared_mem (64-87): with lag = *d_pos mod (N-L+1), each
 * channel's N-L samples after the PN -- d_buf1[ch][lag+L..N) then
 * d_buf2[ch][0..lag) -- are cut into nsym symbols of C+cp samples with the
 * cyclic prefix dropped, d_sym[s][ch][k] = seq[s*(C+cp)+cp+k]: the ring's
 * symbol layout, ready for ofdm_frame_demod (cp_len 0).  Nothing is written
 * when *d_pos < 0.  nsym*(C+cp) <= N-L. */
int ofdm_pn_correlate(const ofdm_cf32 *d_buf, int R, long long N, const ofdm_cf32 *d_pn, int L,
                      float thres, long long *d_pos, float *d_mag, ofdm_stream_t stream);
int ofdm_pn_extract(const ofdm_cf32 *d_buf1, const ofdm_cf32 *d_buf2, int R, long long N, int L,
                    const long long *d_pos, int C, int cp, int nsym, ofdm_cf32 *d_sym,
                    ofdm_stream_t stream);

/* ------------------------------------------------------ zero forcing --- */

/* Multi-user zero forcing, U users x R antennas per
 * subcarrier, K subcarriers (the reference passes cols and uses K = cols-1).
 *
 * ofdm_zf_precoder replaces createZeroForcingMatrix (cpuLS.hpp:415-447):
 *   d_H: users x rows x K channel cube, the layout the reference hands to
 *   rotCube (cpuLS.hpp:400-413, X[user*rows*cols + row*cols + col]); it is
 *   not modified (the reference rotates it in place).  Per subcarrier k,
 *   A(u, r) = H[u][r][k], G = A A^H, W = A^H G^-1 (R x U), inverted by
 *   Gauss-Jordan with partial pivoting in f32 (the reference: cgetrf +
 *   cgetri; results agree to f32 rounding of a well-conditioned G, not
 *   bit-for-bit).  Outputs (either may be NULL, not both):
 *     d_W  [K][U][R]: W(r, u) at d_W[k*R*U + u*R + r] -- the reference's H
 *          output (cgemm ldc = rows, cpuLS.hpp:440);
 *     d_Wt [U][R][K]: W(r, u) at d_Wt[(u*R + r)*K + k] -- the layout
 *          ofdm_zf_apply / ofdm_zf_detect read (subcarrier-fastest).
 * ofdm_zf_transpose: d_W (reference layout) -> d_Wt.
 * ofdm_zf_apply replaces multiplyWithChannelInv (cpuLS.hpp:449-463, cgemv
 *   per subcarrier) for nsym symbols at once: d_Y[s][r][k] = sum_u W(r, u)
 *   d_X[s][u][k]  (X: nsym x U x K, Y: nsym x R x K).
 * ofdm_zf_detect (uplink counterpart, no reference function):
 *   d_X[s][u][k] = sum_r conj(W(r, u)) d_Y[s][r][k] -- W^H = G^-1 A is the
 *   pseudo-inverse of the R x U uplink channel A^H.
 * Limits: 1 <= users <= OFDM_ZF_MAX_USERS, users*rows <= OFDM_ZF_MAX_USERS_X_ROWS. */
#define OFDM_ZF_MAX_USERS 32
#define OFDM_ZF_MAX_USERS_X_ROWS 8192
int ofdm_zf_precoder(const ofdm_cf32 *d_H, int users, int rows, int K, ofdm_cf32 *d_W, ofdm_cf32 *d_Wt,
                     ofdm_stream_t stream);
int ofdm_zf_transpose(const ofdm_cf32 *d_W, int users, int rows, int K, ofdm_cf32 *d_Wt,
                      ofdm_stream_t stream);
int ofdm_zf_apply(const ofdm_cf32 *d_Wt, const ofdm_cf32 *d_X, int users, int rows, int K, long long nsym,
                  ofdm_cf32 *d_Y, ofdm_stream_t stream);
int ofdm_zf_detect(const ofdm_cf32 *d_Wt, const ofdm_cf32 *d_Y, int users, int rows, int K, long long nsym,
                   ofdm_cf32 *d_X, ofdm_stream_t stream);
/* ofdm_zf_apply on row-padded layouts (no reference counterpart):
 * d_X[(s*users + u)*ldx + k] and d_Y[(s*rows + r)*ldy + k], ldx, ldy >= K
 * (ldx = ldy = K is ofdm_zf_apply); pitches other than K need K >= 2,
 * rows >= 8 and users <= 40 (else OFDM_E_UNSUPPORTED). */
int ofdm_zf_apply_ex(const ofdm_cf32 *d_Wt, const ofdm_cf32 *d_X, long long ldx, int users, int rows, int K,
                     long long nsym, ofdm_cf32 *d_Y, long long ldy, ofdm_stream_t stream);
/* ofdm_zf_detect on row-padded layouts (no reference counterpart):
 * d_Y[(s*rows + r)*ldy + k] and d_X[(s*users + u)*ldx + k], ldy, ldx >= K
 * (the pad is neither read nor written; ldy = ldx = K is ofdm_zf_detect).
 * Rows padded to a multiple of 16 elements (K = 1023 -> 1024) start on
 * 128-B lines, so no part of a line is left for another workgroup to
 * complete.  Pitches other than K need rows <= 72 (else OFDM_E_UNSUPPORTED). */
int ofdm_zf_detect_ex(const ofdm_cf32 *d_Wt, const ofdm_cf32 *d_Y, long long ldy, int users, int rows, int K,
                      long long nsym, ofdm_cf32 *d_X, long long ldx, ofdm_stream_t stream);

/* --------------------------------------------------- synthetic frames --- */

/* Deterministic synthetic frames for tests and benchmarks:
 * H ~ CN(0,1) per (frame, antenna, subcarrier), pilot = d_X, data = QPSK,
 * bins j+1 carry H x (bin 0 empty), y = IFFT(Y)/sqrt(C) + CN(0, noise_std^2)
 * with a cyclic prefix (freq_domain = 0), or y = Y + noise (freq_domain = 1,
 * cp_len ignored).  Frame f of the buffer is global frame frame0 + f; antenna
 * r is global antenna r0 + r (antenna-split shards). */
int ofdm_synth_frames(ofdm_cf32 *d_iq, long long nframes, int S, int R, int C, int cp_len,
                      const ofdm_cf32 *d_X, unsigned long long seed, long long frame0,
                      float noise_std, int freq_domain, int r0, ofdm_stream_t stream);

/* Adds to *d_errors the number of demodulated symbols in d_out
 * (nframes x (S-1) x K) whose QPSK hard decision differs from the synthetic
 * data of ofdm_synth_frames(seed, frame0). */
int ofdm_count_symbol_errors(const ofdm_cf32 *d_out, long long nframes, int S, int C,
                             unsigned long long seed, long long frame0,
                             unsigned long long *d_errors, ofdm_stream_t stream);

/* Host-mirror helper (no reference counterpart): an order-sensitive 64-bit
 * hash of `bytes` (a multiple of 4) of device memory into *d_hash (device).
 * gpuLS::demodOneSymbol hashes the caller's Hconj / Hsqrd to tell whether
 * they still hold the estimate firstVector exported (gpuLS.cu:410-473 reads
 * them afresh for every symbol). */
int ofdm_buffer_hash(const void *d_buf, size_t bytes, unsigned long long *d_hash, ofdm_stream_t stream);

/* Box probe for bench.py (no reference counterpart): mode 0 copies `bytes`
 * from d_src to d_dst, mode 1 reads them (d_dst receives 1024 x 256 float
 * partial sums, OFDM_HBM_PROBE_SINK_BYTES): every wave streams 16 KiB chunks
 * with 16 non-temporal 16-B loads per lane in flight -- the receivers' access
 * pattern.  `bytes` and both pointers 16-B aligned; dst_bytes = the size of
 * d_dst, at least `bytes` (mode 0) or OFDM_HBM_PROBE_SINK_BYTES (mode 1),
 * else OFDM_E_ARG. */
#define OFDM_HBM_PROBE_SINK_BYTES (1024 * 256 * 4)
int ofdm_hbm_probe(int mode, const void *d_src, void *d_dst, size_t bytes, size_t dst_bytes,
                   ofdm_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* OFDM_LSMRC_H_ */
