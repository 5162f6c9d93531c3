// pipeline.cpp -- streaming ingest (include/ofdm_lsmrc.h, "streaming ingest";
// SURVEY.md 8(f) rank 2): host-resident IQ -> device -> fused receiver ->
// host outputs, with the two PCIe directions and the kernels overlapped.
//
// The reference moves one symbol at a time: readNextSymbolCUDA issues a
// cudaMemcpyAsync on a freshly created stream per symbol and the caller
// synchronises before the FFT (ShMemSymBuff_gpu.hpp:364-447, gpuLS.cu:351-473),
// so copy and compute never overlap and every 512 KiB symbol pays a launch +
// sync round trip.  Here a slot holds `chunk` whole frames; slot i's copy-in,
// compute and copy-out run on three streams ordered by events:
//
//   copy-in(i)  waits compute(i - depth)   (the slot's IQ buffer is free)
//   compute(i)  waits copy-in(i), copy-out(i - depth) (its output buffer is free)
//   copy-out(i) waits compute(i)
//
// so with depth >= 3 the H2D of chunk i+1, the kernels of chunk i and the D2H
// of chunk i-1 are in flight together.  No host thread blocks except in
// ofdm_pipeline_sync (and inside HIP when a host buffer is pageable).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <new>
#include <vector>

#include "../../include/ofdm_lsmrc.h"
#include "launch.hpp"

struct ofdm_pipeline {
    struct Slot {
        ofdm_cf32 *iq = nullptr;
        ofdm_cf32 *out = nullptr;
        void *ws = nullptr;
        hipEvent_t in_done = nullptr, comp_done = nullptr, out_done = nullptr;
        bool used = false;       // has been submitted at least once
        bool acquired = false;   // acquire() called, submit() pending
    };
    int S = 0, R = 0, C = 0, cp = 0, K = 0, device = 0;
    long long chunk = 0;
    size_t ws_bytes = 0, frame_in = 0, frame_out = 0;  // elements
    ofdm_cf32 *X = nullptr;
    hipStream_t s_in = nullptr, s_comp = nullptr, s_out = nullptr;
    std::vector<Slot> slots;
    int next = 0;
};

namespace {

int err(int code, const char *fn, const char *what) {
    char buf[384];
    std::snprintf(buf, sizeof buf, "%s: %s", fn, what);
    return ofdm::set_error(code, buf);
}

int herr(hipError_t e, const char *fn, const char *what) {
    if (e == hipSuccess) return OFDM_OK;
    char buf[384];
    std::snprintf(buf, sizeof buf, "%s: %s: %s", fn, what, hipGetErrorString(e));
    return ofdm::set_error(OFDM_E_HIP, buf);
}

#define PL_TRY(expr, fn, what)                           \
    do {                                                 \
        int rc_ = herr((expr), fn, what);                \
        if (rc_) return rc_;                             \
    } while (0)

// Makes the pipeline's device current for the scope of a call and restores
// the caller's current device on every return path (a host thread driving
// pipelines on several GPUs keeps its own device selection).
struct DeviceGuard {
    int prev = -1;
    hipError_t e = hipSuccess;
    explicit DeviceGuard(int dev) {
        e = hipGetDevice(&prev);
        if (e == hipSuccess && prev != dev) e = hipSetDevice(dev);
    }
    ~DeviceGuard() {
        if (prev >= 0) (void)hipSetDevice(prev);
    }
};

void release(ofdm_pipeline *p) {
    if (!p) return;
    DeviceGuard dg(p->device);
    for (auto &s : p->slots) {
        if (s.iq) (void)hipFree(s.iq);
        if (s.out) (void)hipFree(s.out);
        if (s.ws) {
            (void)ofdm_workspace_release(s.ws);  // its registry entry must not outlive the memory
            (void)hipFree(s.ws);
        }
        if (s.in_done) (void)hipEventDestroy(s.in_done);
        if (s.comp_done) (void)hipEventDestroy(s.comp_done);
        if (s.out_done) (void)hipEventDestroy(s.out_done);
    }
    if (p->X) (void)hipFree(p->X);
    if (p->s_in) (void)hipStreamDestroy(p->s_in);
    if (p->s_comp) (void)hipStreamDestroy(p->s_comp);
    if (p->s_out) (void)hipStreamDestroy(p->s_out);
    delete p;
}

}  // namespace

extern "C" {

int ofdm_pipeline_create(int S, int R, int C, int cp_len, const ofdm_cf32 *X, int chunk_frames,
                         int depth, ofdm_pipeline **out) {
    static const char *fn = "ofdm_pipeline_create";
    if (!out || !X) return err(OFDM_E_ARG, fn, "null pointer");
    *out = nullptr;
    if (chunk_frames < 1 || depth < 1 || depth > 64)
        return err(OFDM_E_ARG, fn, "chunk_frames >= 1 and 1 <= depth <= 64 required");
    const size_t ws = ofdm_frame_workspace_bytes(chunk_frames, S, R, C);
    if (ws == 0) return err(OFDM_E_UNSUPPORTED, fn, "bad frame geometry (S >= 2, R >= 1, 2 <= C <= 8192)");
    if (cp_len < 0 || cp_len > C) return err(OFDM_E_ARG, fn, "cp_len out of [0, C]");
    auto *p = new (std::nothrow) ofdm_pipeline;
    if (!p) return err(OFDM_E_ARG, fn, "out of host memory");
    p->S = S; p->R = R; p->C = C; p->cp = cp_len; p->K = C - 1;
    p->chunk = chunk_frames;
    p->ws_bytes = ws;
    p->frame_in = (size_t)S * R * (C + cp_len);
    p->frame_out = (size_t)(S - 1) * (C - 1);
    int rc;
#define CR(expr, what)                       \
    if ((rc = herr((expr), fn, what))) {     \
        release(p);                          \
        return rc;                           \
    }
    CR(hipGetDevice(&p->device), "hipGetDevice");
    CR(hipStreamCreateWithFlags(&p->s_in, hipStreamNonBlocking), "hipStreamCreate");
    CR(hipStreamCreateWithFlags(&p->s_comp, hipStreamNonBlocking), "hipStreamCreate");
    CR(hipStreamCreateWithFlags(&p->s_out, hipStreamNonBlocking), "hipStreamCreate");
    CR(hipMalloc(&p->X, (size_t)(C - 1) * sizeof(ofdm_cf32)), "hipMalloc(X)");
    CR(hipMemcpy(p->X, X, (size_t)(C - 1) * sizeof(ofdm_cf32), hipMemcpyDefault), "copy X");
    p->slots.resize(depth);
    for (auto &s : p->slots) {
        CR(hipMalloc(&s.iq, p->frame_in * chunk_frames * sizeof(ofdm_cf32)), "hipMalloc(iq slot)");
        CR(hipMalloc(&s.out, p->frame_out * chunk_frames * sizeof(ofdm_cf32)), "hipMalloc(out slot)");
        CR(hipMalloc(&s.ws, ws), "hipMalloc(workspace)");
        CR(hipEventCreateWithFlags(&s.in_done, hipEventDisableTiming), "hipEventCreate");
        CR(hipEventCreateWithFlags(&s.comp_done, hipEventDisableTiming), "hipEventCreate");
        CR(hipEventCreateWithFlags(&s.out_done, hipEventDisableTiming), "hipEventCreate");
    }
#undef CR
    *out = p;
    return OFDM_OK;
}

int ofdm_pipeline_destroy(ofdm_pipeline *p) {
    if (!p) return OFDM_OK;
    const int rc = ofdm_pipeline_sync(p);
    release(p);
    return rc;
}

int ofdm_pipeline_acquire(ofdm_pipeline *p, ofdm_cf32 **d_iq, ofdm_stream_t *copy_stream) {
    static const char *fn = "ofdm_pipeline_acquire";
    if (!p || !d_iq) return err(OFDM_E_ARG, fn, "null pointer");
    auto &s = p->slots[p->next];
    if (s.acquired) return err(OFDM_E_ARG, fn, "slot already acquired: submit it first");
    DeviceGuard dg(p->device);
    PL_TRY(dg.e, fn, "hipSetDevice");
    // the copy into this slot must not overwrite IQ its previous compute still reads
    if (s.used) PL_TRY(hipStreamWaitEvent(p->s_in, s.comp_done, 0), fn, "hipStreamWaitEvent");
    s.acquired = true;
    *d_iq = s.iq;
    if (copy_stream) *copy_stream = reinterpret_cast<ofdm_stream_t>(p->s_in);
    return OFDM_OK;
}

int ofdm_pipeline_submit(ofdm_pipeline *p, long long nframes, ofdm_cf32 *out) {
    static const char *fn = "ofdm_pipeline_submit";
    if (!p) return err(OFDM_E_ARG, fn, "null pipeline");
    auto &s = p->slots[p->next];
    if (!s.acquired) return err(OFDM_E_ARG, fn, "no acquired slot");
    if (nframes < 0 || nframes > p->chunk) return err(OFDM_E_ARG, fn, "nframes out of [0, chunk_frames]");
    DeviceGuard dg(p->device);
    // any failure below releases the slot (its frames are not demodulated) so
    // the pipeline stays usable: the next acquire hands out the same slot.
    // Once anything may have been enqueued on the compute stream for this slot
    // (from the wait on in_done on), the failure path still records
    // comp_done / out_done and marks the slot used (best effort), so that the
    // next acquire makes the copy-in wait for whatever kernel of this submit
    // is still reading the slot's IQ.
    struct Release {
        ofdm_pipeline *p;
        ofdm_pipeline::Slot &s;
        bool ok = false, enqueued = false;
        ~Release() {
            if (ok) return;
            if (enqueued) {
                (void)hipEventRecord(s.comp_done, p->s_comp);
                (void)hipStreamWaitEvent(p->s_out, s.comp_done, 0);
                (void)hipEventRecord(s.out_done, p->s_out);
                s.used = true;
            }
            s.acquired = false;
        }
    } rel{p, s};
    PL_TRY(dg.e, fn, "hipSetDevice");
    PL_TRY(hipEventRecord(s.in_done, p->s_in), fn, "hipEventRecord");
    rel.enqueued = true;
    PL_TRY(hipStreamWaitEvent(p->s_comp, s.in_done, 0), fn, "hipStreamWaitEvent");
    if (s.used) PL_TRY(hipStreamWaitEvent(p->s_comp, s.out_done, 0), fn, "hipStreamWaitEvent");
    if (nframes > 0) {
        const int rc = ofdm_frame_demod(s.iq, nframes, p->S, p->R, p->C, p->cp, p->X, s.ws,
                                        p->ws_bytes, s.out, p->s_comp);
        if (rc) return rc;
    }
    PL_TRY(hipEventRecord(s.comp_done, p->s_comp), fn, "hipEventRecord");
    PL_TRY(hipStreamWaitEvent(p->s_out, s.comp_done, 0), fn, "hipStreamWaitEvent");
    if (out && nframes > 0)
        PL_TRY(hipMemcpyAsync(out, s.out, p->frame_out * nframes * sizeof(ofdm_cf32),
                              hipMemcpyDefault, p->s_out),
               fn, "copy-out");
    PL_TRY(hipEventRecord(s.out_done, p->s_out), fn, "hipEventRecord");
    rel.ok = true;
    s.used = true;
    s.acquired = false;
    p->next = (p->next + 1) % (int)p->slots.size();
    return OFDM_OK;
}

int ofdm_pipeline_demod(ofdm_pipeline *p, const ofdm_cf32 *iq, long long nframes,
                        ofdm_cf32 *out) {
    static const char *fn = "ofdm_pipeline_demod";
    if (!p) return err(OFDM_E_ARG, fn, "null pipeline");
    if (nframes < 0 || (nframes > 0 && (!iq || !out))) return err(OFDM_E_ARG, fn, "bad arguments");
    for (long long f0 = 0; f0 < nframes; f0 += p->chunk) {
        const long long n = nframes - f0 < p->chunk ? nframes - f0 : p->chunk;
        ofdm_cf32 *d = nullptr;
        ofdm_stream_t cs = nullptr;
        int rc = ofdm_pipeline_acquire(p, &d, &cs);
        if (rc) return rc;
        PL_TRY(hipMemcpyAsync(d, iq + (size_t)f0 * p->frame_in, (size_t)n * p->frame_in * sizeof(ofdm_cf32),
                              hipMemcpyDefault, reinterpret_cast<hipStream_t>(cs)),
               fn, "copy-in");
        if ((rc = ofdm_pipeline_submit(p, n, out + (size_t)f0 * p->frame_out))) return rc;
    }
    return OFDM_OK;
}

int ofdm_pipeline_sync(ofdm_pipeline *p) {
    static const char *fn = "ofdm_pipeline_sync";
    if (!p) return err(OFDM_E_ARG, fn, "null pipeline");
    DeviceGuard dg(p->device);
    PL_TRY(dg.e, fn, "hipSetDevice");
    PL_TRY(hipStreamSynchronize(p->s_in), fn, "sync copy-in");
    PL_TRY(hipStreamSynchronize(p->s_comp), fn, "sync compute");
    PL_TRY(hipStreamSynchronize(p->s_out), fn, "sync copy-out");
    return OFDM_OK;
}

int ofdm_host_register(void *ptr, size_t bytes) {
    if (!ptr || bytes == 0) return err(OFDM_E_ARG, "ofdm_host_register", "bad arguments");
    return herr(hipHostRegister(ptr, bytes, hipHostRegisterDefault), "ofdm_host_register",
                "hipHostRegister");
}

int ofdm_host_unregister(void *ptr) {
    if (!ptr) return err(OFDM_E_ARG, "ofdm_host_unregister", "null pointer");
    return herr(hipHostUnregister(ptr), "ofdm_host_unregister", "hipHostUnregister");
}

}  // extern "C"
