"""ctypes bindings for the CPU oracle (oracle/) and the reference build
(oracle/_ref/).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by the product package.
"""
import ctypes
import os
import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "libofdm_oracle.so")
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_cpuls.so")

_c = ctypes
_P = _c.c_void_p


def _ptr(a):
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_P)


def c64(a):
    return np.ascontiguousarray(a, dtype=np.complex64)


class Oracle:
    """CPU restatement of cpuLS.hpp (see oracle/ofdm_oracle.h)."""

    def __init__(self, path=ORACLE_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} missing: run `make -C oracle`")
        L = self.lib = _c.CDLL(path)
        L.oracle_pilot_rotate.argtypes = [_P, _c.c_int, _P]
        L.oracle_shift_one_row.argtypes = [_P, _c.c_int]
        L.oracle_fft_row.argtypes = [_P, _c.c_int, _c.c_int]
        L.oracle_ls.argtypes = [_P, _P, _c.c_int, _c.c_int, _P, _P]
        L.oracle_mrc.argtypes = [_P, _P, _P, _c.c_int, _c.c_int, _P]
        L.oracle_mrc_numerator.argtypes = [_P, _P, _c.c_int, _c.c_int, _P]
        L.oracle_frame_demod.argtypes = [_P, _c.c_int, _c.c_int, _c.c_int, _c.c_int,
                                         _P, _P, _P, _P]
        L.oracle_frames_demod.argtypes = [_P, _c.c_longlong, _c.c_int, _c.c_int,
                                          _c.c_int, _c.c_int, _P, _P, _c.c_int]
        L.oracle_frames_demod_fft32.argtypes = [_P, _c.c_longlong, _c.c_int, _c.c_int,
                                                _c.c_int, _c.c_int, _P, _P, _c.c_int]
        L.oracle_fft_row_f32.argtypes = [_P, _c.c_int]
        L.oracle_fft_row_fast.argtypes = [_P, _c.c_int]
        L.oracle_frames_demod_fftfast.argtypes = [_P, _c.c_longlong, _c.c_int, _c.c_int,
                                                  _c.c_int, _c.c_int, _P, _P, _c.c_int]
        L.oracle_frames_demod_freq.argtypes = [_P, _c.c_longlong, _c.c_int, _c.c_int,
                                               _c.c_int, _P, _P, _c.c_int]
        L.oracle_max_threads.restype = _c.c_int
        L.oracle_pn_correlate.argtypes = [_P, _c.c_int, _c.c_longlong, _P, _c.c_int, _c.c_float,
                                          _P, _P]
        L.oracle_pn_extract.argtypes = [_P, _P, _c.c_int, _c.c_longlong, _c.c_int, _c.c_longlong,
                                        _c.c_int, _c.c_int, _c.c_int, _P]
        L.oracle_zf_precoder.argtypes = [_P, _c.c_int, _c.c_int, _c.c_int, _P]
        L.oracle_zf_apply.argtypes = [_P, _P, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P]
        L.oracle_zf_detect.argtypes = [_P, _P, _c.c_int, _c.c_int, _c.c_int, _c.c_int, _P]

    def zf_precoder(self, H):
        """createZeroForcingMatrix (cpuLS.hpp:415-447): H (U, R, K) -> W (K, U, R)."""
        H = c64(H)
        U, R, K = H.shape
        W = np.empty((K, U, R), np.complex64)
        self.lib.oracle_zf_precoder(_ptr(H), U, R, K, _ptr(W))
        return W

    def zf_apply(self, W, X):
        """multiplyWithChannelInv per symbol: W (K, U, R), X (n, U, K) -> (n, R, K)."""
        W, X = c64(W), c64(X)
        K, U, R = W.shape
        n = X.shape[0]
        Y = np.empty((n, R, K), np.complex64)
        self.lib.oracle_zf_apply(_ptr(W), _ptr(X), U, R, K, n, _ptr(Y))
        return Y

    def zf_detect(self, W, Y):
        """W^H y per subcarrier: Y (n, R, K) -> (n, U, K)."""
        W, Y = c64(W), c64(Y)
        K, U, R = W.shape
        n = Y.shape[0]
        X = np.empty((n, U, K), np.complex64)
        self.lib.oracle_zf_detect(_ptr(W), _ptr(Y), U, R, K, n, _ptr(X))
        return X

    def pn_correlate(self, buf, pn, thres, mag=False):
        """rx_and_corr.cpp:332-360 -> (pos, mag or None)."""
        buf, pn = c64(buf), c64(pn)
        R, N = buf.shape
        pos = _c.c_longlong(0)
        m = np.empty((R, max(N - pn.size + 1, 0)), np.float32) if mag else None
        self.lib.oracle_pn_correlate(_ptr(buf), R, N, _ptr(pn), pn.size, float(thres),
                                     _c.byref(pos), _ptr(m) if mag else None)
        return pos.value, m

    def pn_extract(self, buf1, buf2, L, lag, C, cp, nsym):
        buf1, buf2 = c64(buf1), c64(buf2)
        R, N = buf1.shape
        out = np.empty((nsym, R, C), np.complex64)
        self.lib.oracle_pn_extract(_ptr(buf1), _ptr(buf2), R, N, L, lag, C, cp, nsym, _ptr(out))
        return out

    def pilot_rotate(self, raw):
        raw = c64(raw)
        X = np.empty_like(raw)
        self.lib.oracle_pilot_rotate(_ptr(raw), raw.size, _ptr(X))
        return X

    def shift_one_row(self, row):
        row = c64(row).copy()
        self.lib.oracle_shift_one_row(_ptr(row), row.size)
        return row

    def fft_rows(self, rows, inverse=False):
        rows = c64(rows).copy()
        C = rows.shape[-1]
        flat = rows.reshape(-1, C)
        for i in range(flat.shape[0]):
            self.lib.oracle_fft_row(flat[i:].ctypes.data_as(_P), C, int(inverse))
        return rows

    def ls(self, Yfft, X):
        Yfft, X = c64(Yfft), c64(X)
        R, C = Yfft.shape
        H = np.empty((R, C - 1), np.complex64)
        P = np.empty(C - 1, np.float32)
        self.lib.oracle_ls(_ptr(Yfft), _ptr(X), R, C, _ptr(H), _ptr(P))
        return H, P

    def mrc(self, Yfft, H, P):
        Yfft, H = c64(Yfft), c64(H)
        P = np.ascontiguousarray(P, np.float32)
        R, C = Yfft.shape
        out = np.empty(C - 1, np.complex64)
        self.lib.oracle_mrc(_ptr(Yfft), _ptr(H), _ptr(P), R, C, _ptr(out))
        return out

    def mrc_numerator(self, Yfft, H):
        Yfft, H = c64(Yfft), c64(H)
        R, C = Yfft.shape
        out = np.empty(C - 1, np.complex64)
        self.lib.oracle_mrc_numerator(_ptr(Yfft), _ptr(H), R, C, _ptr(out))
        return out

    def frame_demod(self, iq, X, prefix=0):
        """iq: (S, R, C+prefix) time domain -> (out (S-1,K), H (R,K), P (K,))."""
        iq, X = c64(iq), c64(X)
        S, R, Cp = iq.shape
        C = Cp - prefix
        out = np.empty((S - 1, C - 1), np.complex64)
        H = np.empty((R, C - 1), np.complex64)
        P = np.empty(C - 1, np.float32)
        self.lib.oracle_frame_demod(_ptr(iq), S, R, C, prefix, _ptr(X), _ptr(out),
                                    _ptr(H), _ptr(P))
        return out, H, P

    def frames_demod(self, iq, X, prefix=0, nthreads=0):
        """iq: (F, S, R, C+prefix) -> (F, S-1, K)."""
        iq, X = c64(iq), c64(X)
        F, S, R, Cp = iq.shape
        C = Cp - prefix
        out = np.empty((F, S - 1, C - 1), np.complex64)
        self.lib.oracle_frames_demod(_ptr(iq), F, S, R, C, prefix, _ptr(X), _ptr(out),
                                     nthreads)
        return out

    def frames_demod_fft32(self, iq, X, prefix=0, nthreads=0):
        """frames_demod with the single-precision FFT (timed CPU baseline only)."""
        iq, X = c64(iq), c64(X)
        F, S, R, Cp = iq.shape
        C = Cp - prefix
        out = np.empty((F, S - 1, C - 1), np.complex64)
        self.lib.oracle_frames_demod_fft32(_ptr(iq), F, S, R, C, prefix, _ptr(X), _ptr(out),
                                           nthreads)
        return out

    def frames_demod_fast(self, iq, X, prefix=0, nthreads=0):
        """frames_demod with the vectorised single-precision FFT of fft_fast.c
        (bench.py's timed CPU baseline only; not the parity oracle)."""
        iq, X = c64(iq), c64(X)
        F, S, R, Cp = iq.shape
        C = Cp - prefix
        out = np.empty((F, S - 1, C - 1), np.complex64)
        self.lib.oracle_frames_demod_fftfast(_ptr(iq), F, S, R, C, prefix, _ptr(X), _ptr(out),
                                             nthreads)
        return out

    def fft_rows_fast(self, rows):
        rows = c64(rows).copy()
        for r in rows.reshape(-1, rows.shape[-1]):
            self.lib.oracle_fft_row_fast(_ptr(r), r.shape[-1])
        return rows

    def fft_rows_f32(self, rows):
        rows = c64(rows).copy()
        for r in rows.reshape(-1, rows.shape[-1]):
            self.lib.oracle_fft_row_f32(_ptr(r), r.shape[-1])
        return rows

    def frames_demod_freq(self, yf, X, nthreads=0):
        yf, X = c64(yf), c64(X)
        F, S, R, C = yf.shape
        out = np.empty((F, S - 1, C - 1), np.complex64)
        self.lib.oracle_frames_demod_freq(_ptr(yf), F, S, R, C, _ptr(X), _ptr(out),
                                          nthreads)
        return out

    def max_threads(self):
        return self.lib.oracle_max_threads()


class Reference:
    """The reference's own RX arithmetic compiled from /root/reference
    (oracle/build_ref.sh).  Absent on the GPU box."""

    def __init__(self, path=REF_SO):
        if not os.path.exists(path):
            raise FileNotFoundError(path)
        L = self.lib = _c.CDLL(path)
        L.ref_matrix_readX.argtypes = [_P, _c.c_int, _c.c_char_p]
        L.ref_shift_one_row.argtypes = [_P, _c.c_int]
        L.ref_ls_post_fft.argtypes = [_P, _P, _c.c_int, _c.c_int, _P, _P]
        L.ref_mrc_post_fft.argtypes = [_P, _P, _P, _c.c_int, _c.c_int, _P]
        L.ref_rot_cube.argtypes = [_P, _c.c_int, _c.c_int, _c.c_int]

    def rot_cube(self, X):
        """rotCube (cpuLS.hpp:400-413) in place on a copy: X (users, rows, cols)
        -> the rotated buffer, returned flat."""
        X = c64(X).copy()
        users, rows, cols = X.shape
        self.lib.ref_rot_cube(_ptr(X), rows, cols, users)
        return X.ravel()

    def matrix_readX(self, path, K):
        X = np.zeros(K, np.complex64)
        self.lib.ref_matrix_readX(_ptr(X), K, path.encode())
        return X

    def shift_one_row(self, row):
        row = c64(row).copy()
        self.lib.ref_shift_one_row(_ptr(row), row.size)
        return row

    def ls(self, Yfft, X):
        Yfft, X = c64(Yfft), c64(X).copy()
        R, C = Yfft.shape
        H = np.empty((R, C - 1), np.complex64)
        P = np.empty(C - 1, np.float32)
        self.lib.ref_ls_post_fft(_ptr(Yfft), _ptr(X), R, C, _ptr(H), _ptr(P))
        return H, P

    def mrc(self, Yfft, H, P):
        Yfft, H = c64(Yfft), c64(H).copy()
        P = np.ascontiguousarray(P, np.float32)
        R, C = Yfft.shape
        out = np.empty(C - 1, np.complex64)
        self.lib.ref_mrc_post_fft(_ptr(Yfft), _ptr(H), _ptr(P), R, C, _ptr(out))
        return out


def reference_available():
    return os.path.exists(REF_SO)
