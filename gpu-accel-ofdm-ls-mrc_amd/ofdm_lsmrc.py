"""Python binding of the C ABI in include/ofdm_lsmrc.h (libofdm_lsmrc.so).

Plumbing for tests and bench.py: device memory and streams come from PyTorch
(ROCm build), the compute is the HIP library.  There is no CPU fallback:
every compute call goes through libofdm_lsmrc.so and raises if it fails.

Mirrors the reference's operator surface:
  gpuLS::batchedFFT / cufft        -> fft_rows
  findHs + findDistSqrd            -> ls_estimate
  multiplyWithChannelConj + combineForMRC + shiftOneRow -> mrc_demod
  demodOneFrameCUDA (batched)      -> frame_demod / frame_demod_freq
  matrix_readX                     -> read_pilots / pilot_rotate
"""
import ctypes
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# OFDM_LSMRC_LIB=<v> loads lib/libofdm_lsmrc_<v>.so instead, a build of
# experiment sources for scripts/ comparisons (scripts/libab.py); the product
# library has no switches.
_LIBSEL = os.environ.get("OFDM_LSMRC_LIB", "")
LIB_PATH = os.path.join(HERE, "lib", f"libofdm_lsmrc_{_LIBSEL}.so" if _LIBSEL else "libofdm_lsmrc.so")
HEADER_PATH = os.path.join(os.path.dirname(HERE), "include", "ofdm_lsmrc.h")

_c = ctypes
_P = _c.c_void_p
_LL = _c.c_longlong
_I = _c.c_int

# name -> (restype, argtypes)
_SIGS = {
    "ofdm_version": (_I, []),
    "ofdm_last_error": (_c.c_char_p, []),
    "ofdm_pilot_rotate": (_I, [_P, _I, _P]),
    "ofdm_read_pilots": (_I, [_c.c_char_p, _I, _c.c_float, _P]),
    "ofdm_fft_rows": (_I, [_P, _P, _LL, _I, _I, _P]),
    "ofdm_ls_estimate": (_I, [_P, _P, _I, _I, _P, _P, _P]),
    "ofdm_mrc_demod": (_I, [_P, _LL, _P, _P, _I, _I, _P, _P]),
    "ofdm_mrc_numerator": (_I, [_P, _LL, _P, _I, _I, _P, _P]),
    "ofdm_mrc_finalize": (_I, [_P, _LL, _LL, _I, _I, _P, _P, _P]),
    "ofdm_channel_conj_product": (_I, [_P, _LL, _P, _I, _I, _P, _P]),
    "ofdm_combine_products": (_I, [_P, _LL, _P, _I, _I, _I, _P, _P]),
    "ofdm_shift_rows": (_I, [_P, _LL, _I, _P, _P]),
    "ofdm_dist_sqrd": (_I, [_P, _I, _I, _P, _P]),
    "ofdm_frame_workspace_bytes": (_c.c_size_t, [_LL, _I, _I, _I]),
    "ofdm_workspace_release": (_I, [_P]),
    "ofdm_frame_demod": (_I, [_P, _LL, _I, _I, _I, _I, _P, _P, _c.c_size_t, _P, _P]),
    "ofdm_frame_demod_ex": (_I, [_P, _LL, _I, _I, _I, _I, _P, _P, _c.c_size_t, _P, _I, _LL, _P]),
    "ofdm_frame_estimate": (_I, [_P, _LL, _I, _I, _I, _I, _P, _P, _c.c_size_t, _P]),
    "ofdm_frame_combine": (_I, [_P, _LL, _I, _I, _I, _I, _P, _c.c_size_t, _P, _P]),
    "ofdm_frame_demod_freq": (_I, [_P, _LL, _I, _I, _I, _P, _P, _c.c_size_t, _P, _P]),
    "ofdm_frame_estimate_freq": (_I, [_P, _LL, _I, _I, _I, _P, _P, _c.c_size_t, _P]),
    "ofdm_frame_combine_freq": (_I, [_P, _LL, _I, _I, _I, _P, _c.c_size_t, _P, _P]),
    "ofdm_frame_demod_freq_mfma": (_I, [_P, _LL, _I, _I, _I, _P, _P, _c.c_size_t, _P, _P]),
    "ofdm_frame_ls_partial": (_I, [_P, _LL, _I, _I, _I, _I, _P, _P, _c.c_size_t, _P, _P]),
    "ofdm_frame_mrc_partial": (_I, [_P, _LL, _I, _I, _I, _I, _P, _c.c_size_t, _P, _P]),
    "ofdm_frame_mrc_partial_range": (_I, [_P, _LL, _LL, _LL, _I, _I, _I, _I, _P, _c.c_size_t, _P, _P]),
    "ofdm_frame_export_estimate": (_I, [_P, _c.c_size_t, _LL, _I, _I, _I, _LL, _P, _P, _P]),
    "ofdm_symbols_demod": (_I, [_P, _LL, _I, _I, _I, _P, _c.c_size_t, _LL, _P, _P]),
    "ofdm_synth_frames": (_I, [_P, _LL, _I, _I, _I, _I, _P, _c.c_ulonglong, _LL, _c.c_float,
                               _I, _I, _P]),
    "ofdm_count_symbol_errors": (_I, [_P, _LL, _I, _I, _c.c_ulonglong, _LL, _P, _P]),
    "ofdm_pipeline_create": (_I, [_I, _I, _I, _I, _P, _I, _I, _c.POINTER(_P)]),
    "ofdm_pipeline_destroy": (_I, [_P]),
    "ofdm_pipeline_acquire": (_I, [_P, _c.POINTER(_P), _c.POINTER(_P)]),
    "ofdm_pipeline_submit": (_I, [_P, _LL, _P]),
    "ofdm_pipeline_demod": (_I, [_P, _P, _LL, _P]),
    "ofdm_pipeline_sync": (_I, [_P]),
    "ofdm_host_register": (_I, [_P, _c.c_size_t]),
    "ofdm_host_unregister": (_I, [_P]),
    "ofdm_pn_correlate": (_I, [_P, _I, _LL, _P, _I, _c.c_float, _P, _P, _P]),
    "ofdm_pn_extract": (_I, [_P, _P, _I, _LL, _I, _P, _I, _I, _I, _P, _P]),
    "ofdm_zf_precoder": (_I, [_P, _I, _I, _I, _P, _P, _P]),
    "ofdm_zf_transpose": (_I, [_P, _I, _I, _I, _P, _P]),
    "ofdm_zf_apply": (_I, [_P, _P, _I, _I, _I, _LL, _P, _P]),
    "ofdm_zf_detect": (_I, [_P, _P, _I, _I, _I, _LL, _P, _P]),
    "ofdm_zf_detect_ex": (_I, [_P, _P, _LL, _I, _I, _I, _LL, _P, _LL, _P]),
    "ofdm_zf_apply_ex": (_I, [_P, _P, _LL, _I, _I, _I, _LL, _P, _LL, _P]),
    "ofdm_hbm_probe": (_I, [_I, _P, _P, _c.c_size_t, _c.c_size_t, _P]),
    "ofdm_device_status": (_I, []),
    "ofdm_device_status_inject": (_I, [_c.c_uint]),
    "ofdm_buffer_hash": (_I, [_P, _c.c_size_t, _P, _P]),
}

_lib = None


def build_id():
    """Identity of the product library's build: the first 16 hex digits of
    a SHA-256 over its sources (csrc/, the Makefile, include/ofdm_lsmrc.h),
    in sorted order.  PMC profiles record it (scripts/pmc_summary.py) and
    bench.py attaches a profile's traffic only to the build it measured."""
    import hashlib
    h = hashlib.sha256()
    csrc = os.path.join(HERE, "csrc")
    files = [os.path.join(csrc, f) for f in sorted(os.listdir(csrc))] + [os.path.join(HERE, "Makefile"), HEADER_PATH]
    for f in files:
        if os.path.isfile(f):
            h.update(os.path.basename(f).encode() + b"\0")
            with open(f, "rb") as fp:
                h.update(fp.read())
    return h.hexdigest()[:16]


class OfdmError(RuntimeError):
    pass


def lib():
    """Load libofdm_lsmrc.so (raises if it has not been built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise OfdmError(f"{LIB_PATH} not built: run `make -C gpu-accel-ofdm-ls-mrc_amd` "
                            "(or __graft_entry__.build())")
        # One HIP runtime per process: torch's wheel bundles libamdhip64
        # (SONAME libamdhip64.so.7).  Loading torch first lets our NEEDED
        # libamdhip64.so.7 bind to that copy; loading ours first would pull
        # in /opt/rocm's and torch would then load a second runtime.
        import torch  # noqa: F401
        L = _c.CDLL(LIB_PATH)
        for name, (res, args) in _SIGS.items():
            if _LIBSEL and not hasattr(L, name):
                continue  # an older variant build (OFDM_LSMRC_LIB): its missing entries fail when called
            fn = getattr(L, name)  # the product library: every entry, or AttributeError here
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def load_library(path):
    """Another build of this library (the diagnostic build, lib/
    libofdm_lsmrc_diag.so, or an A/B variant) loaded beside the product one,
    with the same signatures; call it through `using(L)`.  Its device state
    (workspace registry, flag epochs, twiddle tables) is its own."""
    import torch  # noqa: F401  (same HIP runtime as torch, see lib())
    L = _c.CDLL(path)
    for name, (res, args) in _SIGS.items():
        if hasattr(L, name):
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
    return L


class using:
    """with using(L): ... -- the binding's calls go to library L."""

    def __init__(self, L):
        self.L = L

    def __enter__(self):
        global _lib
        lib()
        self.prev, _lib = _lib, self.L
        return self.L

    def __exit__(self, *exc):
        global _lib
        _lib = self.prev
        return False


def hbm_probe(mode, src, dst, stream=None):
    """Box probe: mode 0 copies src -> dst (float4), mode 1 reads src (dst:
    >= 1 MiB of partial sums).  Byte tensors on the device, 16-B multiples."""
    nbytes = src.numel() * src.element_size()
    _check(lib().ofdm_hbm_probe(mode, _dptr(src, "src"), _dptr(dst, "dst"), nbytes, dst.numel() * dst.element_size(),
                                _stream(stream)),
           "ofdm_hbm_probe")


def device_status():
    """Raises OfdmError (OFDM_E_DEVICE) if a ticketed launch reported a fault
    since the last check, and clears it (include/ofdm_lsmrc.h)."""
    _check(lib().ofdm_device_status(), "ofdm_device_status")


def _check(rc, fn):
    if rc < 0:
        msg = lib().ofdm_last_error().decode(errors="replace")
        raise OfdmError(f"{fn} failed ({rc}): {msg}")
    return rc


def _dptr(t, name="tensor"):
    import torch
    if not isinstance(t, torch.Tensor) or not t.is_cuda:
        raise OfdmError(f"{name} must be a device tensor")
    if not t.is_contiguous():
        raise OfdmError(f"{name} must be contiguous")
    return _P(t.data_ptr())


def _stream(stream):
    import torch
    if stream is None:
        stream = torch.cuda.current_stream()
    return _P(stream.cuda_stream)


def c64(shape, device="cuda"):
    import torch
    return torch.empty(shape, dtype=torch.complex64, device=device)


# ---------------------------------------------------------------- host side

def pilot_rotate(raw):
    raw = np.ascontiguousarray(raw, np.complex64)
    X = np.empty_like(raw)
    _check(lib().ofdm_pilot_rotate(raw.ctypes.data_as(_P), raw.size, X.ctypes.data_as(_P)),
           "ofdm_pilot_rotate")
    return X


def read_pilots(path, K, fill=0.707):
    """matrix_readX: returns (X, used_fill)."""
    X = np.empty(K, np.complex64)
    rc = _check(lib().ofdm_read_pilots(None if path is None else path.encode(), K, fill,
                                       X.ctypes.data_as(_P)), "ofdm_read_pilots")
    return X, rc == 1


# -------------------------------------------------------------- device side

def fft_rows(x, out=None, inverse=False, stream=None):
    C = x.shape[-1]
    nrows = x.numel() // C
    if out is None:
        out = x
    _check(lib().ofdm_fft_rows(_dptr(x, "x"), _dptr(out, "out"), nrows, C, int(inverse),
                               _stream(stream)), "ofdm_fft_rows")
    return out


def ls_estimate(Y, X, stream=None):
    """Y: (R, C) freq-domain pilot symbol, X: (K,) rotated pilots -> (Hconj (R,K), Hsqrd (K,))."""
    import torch
    R, C = Y.shape
    H = c64((R, C - 1), Y.device)
    P = torch.empty(C - 1, dtype=torch.float32, device=Y.device)
    _check(lib().ofdm_ls_estimate(_dptr(Y), _dptr(X), R, C, _dptr(H), _dptr(P), _stream(stream)),
           "ofdm_ls_estimate")
    return H, P


def mrc_demod(Y, H, P, stream=None):
    """Y: (nsyms, R, C) freq-domain data symbols -> (nsyms, K)."""
    n, R, C = Y.shape
    out = c64((n, C - 1), Y.device)
    _check(lib().ofdm_mrc_demod(_dptr(Y), n, _dptr(H), _dptr(P), R, C, _dptr(out),
                                _stream(stream)), "ofdm_mrc_demod")
    return out


def mrc_numerator(Y, H, stream=None):
    n, R, C = Y.shape
    out = c64((n, C - 1), Y.device)
    _check(lib().ofdm_mrc_numerator(_dptr(Y), n, _dptr(H), R, C, _dptr(out), _stream(stream)),
           "ofdm_mrc_numerator")
    return out


def mrc_finalize(num_chunk, e0, nsym, K, P, out, stream=None):
    _check(lib().ofdm_mrc_finalize(_dptr(num_chunk), e0, num_chunk.numel(), nsym, K, _dptr(P),
                                   _dptr(out), _stream(stream)), "ofdm_mrc_finalize")
    return out


def channel_conj_product(Y, H, stream=None):
    """multiplyWithChannelConj: Y (nsyms, R, C), H (R, K) -> (nsyms, R, K)."""
    n, R, C = Y.shape
    out = c64((n, R, C - 1), Y.device)
    _check(lib().ofdm_channel_conj_product(_dptr(Y), n, _dptr(H), R, C, _dptr(out),
                                           _stream(stream)), "ofdm_channel_conj_product")
    return out


def combine_products(prod, P, rotate=True, stream=None):
    """combineForMRC [+ shiftOneRow]: prod (nsyms, R, K) -> (nsyms, K)."""
    n, R, K = prod.shape
    out = c64((n, K), prod.device)
    _check(lib().ofdm_combine_products(_dptr(prod), n, _dptr(P), R, K, int(rotate), _dptr(out),
                                       _stream(stream)), "ofdm_combine_products")
    return out


def shift_rows(x, stream=None):
    K = x.shape[-1]
    out = c64(x.shape, x.device)
    _check(lib().ofdm_shift_rows(_dptr(x), x.numel() // K, K, _dptr(out), _stream(stream)),
           "ofdm_shift_rows")
    return out


def dist_sqrd(H, stream=None):
    import torch
    R, K = H.shape
    P = torch.empty(K, dtype=torch.float32, device=H.device)
    _check(lib().ofdm_dist_sqrd(_dptr(H), R, K, _dptr(P), _stream(stream)), "ofdm_dist_sqrd")
    return P


def workspace_bytes(nframes, S, R, C):
    return int(lib().ofdm_frame_workspace_bytes(nframes, S, R, C))


def workspace(nframes, S, R, C, device="cuda"):
    """A frame workspace.  When the tensor is collected its estimate tag is
    dropped from the library's registry (ofdm_workspace_release), so that a
    workspace the caching allocator later hands out at the same address is
    refused by combine / mrc_partial / export until an estimate fills it."""
    import torch
    import weakref
    ws = torch.empty(max(workspace_bytes(nframes, S, R, C), 256), dtype=torch.uint8, device=device)
    weakref.finalize(ws, lib().ofdm_workspace_release, _c.c_void_p(ws.data_ptr()))
    return ws


def workspace_release(ws):
    """Forget the estimate held in `ws` (a tensor or a raw device address)."""
    ptr = ws if isinstance(ws, int) else ws.data_ptr()
    lib().ofdm_workspace_release(_c.c_void_p(ptr))


FLOW_AUTO, FLOW_TWO_LAUNCH = 0, 1  # OFDM_FLOW_* of ofdm_frame_demod_ex


def frame_demod(iq, X, prefix=0, ws=None, out=None, stream=None, flow=None, spin_ticks=None):
    """iq: (F, S, R, C+prefix) time domain -> (F, S-1, K).  flow / spin_ticks:
    ofdm_frame_demod_ex's scheduling choices (default: ofdm_frame_demod's)."""
    F, S, R, Cp = iq.shape
    C = Cp - prefix
    if ws is None:
        ws = workspace(F, S, R, C, iq.device)
    if out is None:
        out = c64((F, S - 1, C - 1), iq.device)
    if flow is None and spin_ticks is None:
        _check(lib().ofdm_frame_demod(_dptr(iq), F, S, R, C, prefix, _dptr(X), _dptr(ws), ws.numel(),
                                      _dptr(out), _stream(stream)), "ofdm_frame_demod")
    else:
        _check(lib().ofdm_frame_demod_ex(_dptr(iq), F, S, R, C, prefix, _dptr(X), _dptr(ws), ws.numel(),
                                         _dptr(out), FLOW_AUTO if flow is None else flow,
                                         -1 if spin_ticks is None else spin_ticks, _stream(stream)),
               "ofdm_frame_demod_ex")
    return out


def frame_estimate(iq, X, prefix, ws, stream=None):
    """LS stage of frame_demod: estimates of every frame into the workspace."""
    F, S, R, Cp = iq.shape
    _check(lib().ofdm_frame_estimate(_dptr(iq), F, S, R, Cp - prefix, prefix, _dptr(X), _dptr(ws),
                                     ws.numel(), _stream(stream)), "ofdm_frame_estimate")
    return ws


def frame_combine(iq, prefix, ws, out, stream=None):
    """MRC stage of frame_demod against the estimates in the workspace."""
    F, S, R, Cp = iq.shape
    _check(lib().ofdm_frame_combine(_dptr(iq), F, S, R, Cp - prefix, prefix, _dptr(ws),
                                    ws.numel(), _dptr(out), _stream(stream)),
           "ofdm_frame_combine")
    return out


def symbols_demod(sym, ws, prefix=0, frame=0, out=None, stream=None):
    """sym: (nsym, R, C+prefix) time-domain data symbols -> (nsym, K), against
    frame `frame`'s estimate in ws (filled by frame_estimate)."""
    n, R, Cp = sym.shape
    C = Cp - prefix
    if out is None:
        out = c64((n, C - 1), sym.device)
    _check(lib().ofdm_symbols_demod(_dptr(sym), n, R, C, prefix, _dptr(ws), ws.numel(), frame, _dptr(out),
                                    _stream(stream)), "ofdm_symbols_demod")
    return out


def frame_demod_freq(Y, X, ws=None, out=None, stream=None):
    """Y: (F, S, R, C) frequency domain -> (F, S-1, K)."""
    F, S, R, C = Y.shape
    if ws is None:
        ws = workspace(F, S, R, C, Y.device)
    if out is None:
        out = c64((F, S - 1, C - 1), Y.device)
    _check(lib().ofdm_frame_demod_freq(_dptr(Y), F, S, R, C, _dptr(X), _dptr(ws), ws.numel(),
                                       _dptr(out), _stream(stream)), "ofdm_frame_demod_freq")
    return out


def frame_estimate_freq(Y, X, ws, stream=None):
    """LS stage of frame_demod_freq: estimates of every frame into the workspace."""
    F, S, R, C = Y.shape
    _check(lib().ofdm_frame_estimate_freq(_dptr(Y), F, S, R, C, _dptr(X), _dptr(ws), ws.numel(),
                                          _stream(stream)), "ofdm_frame_estimate_freq")
    return ws


def frame_combine_freq(Y, ws, out, stream=None):
    """MRC stage of frame_demod_freq against the estimates in the workspace."""
    F, S, R, C = Y.shape
    _check(lib().ofdm_frame_combine_freq(_dptr(Y), F, S, R, C, _dptr(ws), ws.numel(), _dptr(out),
                                         _stream(stream)), "ofdm_frame_combine_freq")
    return out


def frame_demod_freq_mfma(Y, X, ws=None, out=None, stream=None):
    """frame_demod_freq with the antenna combine on the matrix cores."""
    F, S, R, C = Y.shape
    if ws is None:
        ws = workspace(F, S, R, C, Y.device)
    if out is None:
        out = c64((F, S - 1, C - 1), Y.device)
    _check(lib().ofdm_frame_demod_freq_mfma(_dptr(Y), F, S, R, C, _dptr(X), _dptr(ws), ws.numel(),
                                            _dptr(out), _stream(stream)), "ofdm_frame_demod_freq_mfma")
    return out


def frame_ls_partial(iq, X, prefix=0, ws=None, P=None, stream=None):
    import torch
    F, S, R, Cp = iq.shape
    C = Cp - prefix
    if ws is None:
        ws = workspace(F, S, R, C, iq.device)
    if P is None:
        P = torch.empty((F, C - 1), dtype=torch.float32, device=iq.device)
    _check(lib().ofdm_frame_ls_partial(_dptr(iq), F, S, R, C, prefix, _dptr(X), _dptr(ws),
                                       ws.numel(), _dptr(P), _stream(stream)),
           "ofdm_frame_ls_partial")
    return P, ws


def frame_mrc_partial(iq, ws, prefix=0, num=None, stream=None):
    F, S, R, Cp = iq.shape
    C = Cp - prefix
    if num is None:
        num = c64((F, S - 1, C - 1), iq.device)
    _check(lib().ofdm_frame_mrc_partial(_dptr(iq), F, S, R, C, prefix, _dptr(ws), ws.numel(),
                                        _dptr(num), _stream(stream)), "ofdm_frame_mrc_partial")
    return num


def frame_mrc_partial_range(iq, ws, prefix, f0, count, num=None, stream=None):
    """Partial MRC numerators of frames [f0, f0 + count) of the batch `iq`
    whose estimate one frame_ls_partial call left in `ws`."""
    F, S, R, Cp = iq.shape
    C = Cp - prefix
    if num is None:
        num = c64((count, S - 1, C - 1), iq.device)
    _check(lib().ofdm_frame_mrc_partial_range(_dptr(iq), F, f0, count, S, R, C, prefix, _dptr(ws), ws.numel(),
                                              _dptr(num), _stream(stream)), "ofdm_frame_mrc_partial_range")
    return num


def frame_export_estimate(ws, F, S, R, C, frame=0, stream=None):
    """Frame `frame`'s estimate in the reference layout: (Hconj (R, K), Hsqrd (K,))."""
    import torch
    H = c64((R, C - 1), ws.device)
    P = torch.empty(C - 1, dtype=torch.float32, device=ws.device)
    _check(lib().ofdm_frame_export_estimate(_dptr(ws), ws.numel(), F, S, R, C, frame, _dptr(H), _dptr(P),
                                            _stream(stream)), "ofdm_frame_export_estimate")
    return H, P


def synth_frames(F, S, R, C, X, prefix=0, seed=1234, frame0=0, noise_std=0.01,
                 freq_domain=False, r0=0, out=None, stream=None):
    Cp = C if freq_domain else C + prefix
    if out is None:
        out = c64((F, S, R, Cp), X.device)
    _check(lib().ofdm_synth_frames(_dptr(out), F, S, R, C, prefix, _dptr(X), seed, frame0,
                                   noise_std, int(freq_domain), r0, _stream(stream)),
           "ofdm_synth_frames")
    return out


def count_symbol_errors(out, S, seed=1234, frame0=0, stream=None):
    import torch
    F = out.shape[0]
    K = out.shape[-1]
    err = torch.zeros(1, dtype=torch.int64, device=out.device)
    _check(lib().ofdm_count_symbol_errors(_dptr(out), F, S, K + 1, seed, frame0, _dptr(err),
                                          _stream(stream)), "ofdm_count_symbol_errors")
    return err


def pn_correlate(buf, pn, thres, mag=False, stream=None):
    """PN frame sync (rx_and_corr.cpp:332-360): buf (R, N), pn (L,) device
    complex64 -> (pos, mag): pos = device int64 tensor [ch*(N-L+1) + lag] or
    [-1]; mag = (R, N-L+1) float32 |corr|/L for every lag if requested."""
    import torch
    R, N = buf.shape
    L = pn.shape[0]
    pos = torch.empty(1, dtype=torch.int64, device=buf.device)
    m = torch.empty((R, max(N - L + 1, 0)), dtype=torch.float32, device=buf.device) if mag else None
    _check(lib().ofdm_pn_correlate(_dptr(buf), R, N, _dptr(pn), L, thres, _dptr(pos),
                                   _dptr(m) if mag else None, _stream(stream)),
           "ofdm_pn_correlate")
    return pos, m


def pn_extract(buf1, buf2, L, pos, C, cp, nsym, out=None, stream=None):
    """Frame after the PN (rx_and_corr.cpp:370-392 + copy_to_shared_mem):
    -> (nsym, R, C) symbols, cyclic prefix dropped."""
    R, N = buf1.shape
    if out is None:
        out = c64((nsym, R, C), buf1.device)
    _check(lib().ofdm_pn_extract(_dptr(buf1), _dptr(buf2), R, N, L, _dptr(pos), C, cp, nsym,
                                 _dptr(out), _stream(stream)), "ofdm_pn_extract")
    return out


def _opt_ptr(t, name):
    return None if t is None else _dptr(t, name)


def zf_precoder(H, W=True, Wt=True, stream=None):
    """createZeroForcingMatrix (cpuLS.hpp:415-447): H (U, R, K) device
    complex64 -> (W (K, U, R) reference layout or None, Wt (U, R, K) or None)."""
    U, R, K = H.shape
    W = c64((K, U, R), H.device) if W is True else (None if W is False else W)
    Wt = c64((U, R, K), H.device) if Wt is True else (None if Wt is False else Wt)
    _check(lib().ofdm_zf_precoder(_dptr(H, "H"), U, R, K, _opt_ptr(W, "W"), _opt_ptr(Wt, "Wt"),
                                  _stream(stream)), "ofdm_zf_precoder")
    return W, Wt


def zf_transpose(W, stream=None):
    """(K, U, R) reference layout -> (U, R, K)."""
    K, U, R = W.shape
    Wt = c64((U, R, K), W.device)
    _check(lib().ofdm_zf_transpose(_dptr(W, "W"), U, R, K, _dptr(Wt, "Wt"), _stream(stream)),
           "ofdm_zf_transpose")
    return Wt


def zf_apply(Wt, X, out=None, stream=None):
    """multiplyWithChannelInv (cpuLS.hpp:449-463) over symbols: X (nsym, U, K) -> (nsym, R, K)."""
    U, R, K = Wt.shape
    n = X.shape[0]
    assert tuple(X.shape) == (n, U, K), X.shape
    if out is None:
        out = c64((n, R, K), X.device)
    _check(lib().ofdm_zf_apply(_dptr(Wt, "Wt"), _dptr(X, "X"), U, R, K, n, _dptr(out, "out"),
                               _stream(stream)), "ofdm_zf_apply")
    return out


def zf_detect(Wt, Y, out=None, stream=None):
    """ZF detection with the same matrix: Y (nsym, R, K) -> (nsym, U, K)."""
    U, R, K = Wt.shape
    n = Y.shape[0]
    assert tuple(Y.shape) == (n, R, K), Y.shape
    if out is None:
        out = c64((n, U, K), Y.device)
    _check(lib().ofdm_zf_detect(_dptr(Wt, "Wt"), _dptr(Y, "Y"), U, R, K, n, _dptr(out, "out"),
                                _stream(stream)), "ofdm_zf_detect")
    return out


def zf_apply_pitched(Wt, X, out=None, ldy=None, stream=None):
    """ofdm_zf_apply_ex: X (nsym, U, ldx) with rows padded to ldx >= K -> out
    (nsym, R, ldy), first K columns written (ldy default: ldx)."""
    U, R, K = Wt.shape
    n, u, ldx = X.shape
    assert u == U and ldx >= K, X.shape
    if out is None:
        out = c64((n, R, ldy or ldx), X.device)
    assert out.shape[0] == n and out.shape[1] == R and out.shape[2] >= K, out.shape
    _check(lib().ofdm_zf_apply_ex(_dptr(Wt, "Wt"), _dptr(X, "X"), ldx, U, R, K, n, _dptr(out, "out"),
                                  out.shape[2], _stream(stream)), "ofdm_zf_apply_ex")
    return out


def zf_detect_pitched(Wt, Y, out=None, ldx=None, stream=None):
    """ofdm_zf_detect_ex: Y (nsym, R, ldy) with rows padded to ldy >= K (only
    the first K columns read) -> out (nsym, U, ldx), first K columns written
    (ldx default: ldy)."""
    U, R, K = Wt.shape
    n, r, ldy = Y.shape
    assert r == R and ldy >= K, Y.shape
    if out is None:
        out = c64((n, U, ldx or ldy), Y.device)
    assert out.shape[0] == n and out.shape[1] == U and out.shape[2] >= K, out.shape
    _check(lib().ofdm_zf_detect_ex(_dptr(Wt, "Wt"), _dptr(Y, "Y"), ldy, U, R, K, n, _dptr(out, "out"),
                                   out.shape[2], _stream(stream)), "ofdm_zf_detect_ex")
    return out


class Pipeline:
    """Streaming receiver over host-resident frames (ofdm_pipeline_*):
    `depth` device slots of `chunk_frames` frames, copy-in / compute /
    copy-out on three HIP streams.  demod() is asynchronous: keep `iq` and
    `out` alive until sync()."""

    def __init__(self, S, R, C, X, prefix=0, chunk_frames=4, depth=3):
        self.S, self.R, self.C, self.prefix = S, R, C, prefix
        Xp = X.data_ptr() if hasattr(X, "data_ptr") else np.ascontiguousarray(
            X, np.complex64).ctypes.data
        h = _P()
        _check(lib().ofdm_pipeline_create(S, R, C, prefix, _P(Xp), chunk_frames, depth,
                                          _c.byref(h)), "ofdm_pipeline_create")
        self._h = h

    @staticmethod
    def _ptr(a):
        return _P(a.data_ptr() if hasattr(a, "data_ptr") else a.ctypes.data)

    def demod(self, iq, out):
        """iq: (F, S, R, C+prefix) complex64, out: (F, S-1, K) complex64 --
        numpy arrays or tensors (host or device), contiguous."""
        F = iq.shape[0]
        assert tuple(iq.shape[1:]) == (self.S, self.R, self.C + self.prefix), iq.shape
        assert tuple(out.shape) == (F, self.S - 1, self.C - 1), out.shape
        _check(lib().ofdm_pipeline_demod(self._h, self._ptr(iq), F, self._ptr(out)),
               "ofdm_pipeline_demod")
        return out

    def acquire(self):
        d, s = _P(), _P()
        _check(lib().ofdm_pipeline_acquire(self._h, _c.byref(d), _c.byref(s)),
               "ofdm_pipeline_acquire")
        return d.value, s.value

    def submit(self, nframes, out=None):
        _check(lib().ofdm_pipeline_submit(self._h, nframes,
                                          None if out is None else self._ptr(out)),
               "ofdm_pipeline_submit")

    def sync(self):
        _check(lib().ofdm_pipeline_sync(self._h), "ofdm_pipeline_sync")

    def close(self):
        if getattr(self, "_h", None):
            h, self._h = self._h, None
            _check(lib().ofdm_pipeline_destroy(h), "ofdm_pipeline_destroy")

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def host_register(a):
    """Page-lock a host numpy array / CPU tensor for asynchronous DMA."""
    p = a.data_ptr() if hasattr(a, "data_ptr") else a.ctypes.data
    n = a.numel() * a.element_size() if hasattr(a, "numel") else a.nbytes
    _check(lib().ofdm_host_register(_P(p), n), "ofdm_host_register")


def host_unregister(a):
    p = a.data_ptr() if hasattr(a, "data_ptr") else a.ctypes.data
    _check(lib().ofdm_host_unregister(_P(p)), "ofdm_host_unregister")


def header_symbols(path=HEADER_PATH):
    """Function names declared in include/ofdm_lsmrc.h."""
    import re
    txt = open(path).read()
    return sorted(set(re.findall(r"^\s*(?:int|size_t|const char \*)\s*(ofdm_\w+)\s*\(", txt,
                                 re.M)))
