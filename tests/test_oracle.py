"""CPU tests of the oracle (test infrastructure): pinned against the golden
fixtures (generated from the reference's own arithmetic) and, in the build
container, against oracle/_ref built from /root/reference/cpuLS.hpp."""
import os

import numpy as np
import pytest

from helpers import GOLDEN, golden_cases
from oracle_bindings import Reference, reference_available

needs_ref = pytest.mark.skipif(not reference_available(), reason="oracle/_ref not built "
                               "(/root/reference absent)")


def bits(a):
    return np.ascontiguousarray(a).view(np.uint32)


@pytest.mark.parametrize("name,z", golden_cases("time"), ids=lambda v: v if isinstance(v, str) else "")
def test_oracle_bitexact_on_golden_time(oracle, name, z):
    prefix = int(z["prefix"])
    for f in range(z["iq"].shape[0]):
        out, H, P = oracle.frame_demod(z["iq"][f], z["X"], prefix)
        assert np.array_equal(bits(out), bits(z["out"][f])), name
        assert np.array_equal(bits(H), bits(z["H"][f]))
        assert np.array_equal(bits(P), bits(z["P"][f]))
    # the OpenMP batch entry point gives the same bits
    outs = oracle.frames_demod(z["iq"], z["X"], prefix, nthreads=4)
    assert np.array_equal(bits(outs), bits(z["out"]))


@pytest.mark.parametrize("name,z", golden_cases("freq"), ids=lambda v: v if isinstance(v, str) else "")
def test_oracle_bitexact_on_golden_freq(oracle, name, z):
    outs = oracle.frames_demod_freq(z["yf"], z["X"], nthreads=2)
    assert np.array_equal(bits(outs), bits(z["out"]))


def test_pilot_rotation_and_file(oracle):
    K = 1023
    raw = np.fromfile(os.path.join(GOLDEN, "Pilots.dat"), np.complex64)
    assert raw.size == K
    X = oracle.pilot_rotate(raw)
    assert np.array_equal(bits(X), bits(np.load(os.path.join(GOLDEN, "pilots_rotated_k1023.npy"))))
    # closed form for odd K: X[j] = raw[(j + (K+1)/2) mod K]  (cpuLS.hpp:105-112)
    for K in (3, 7, 255, 1023, 4095):
        r = np.arange(K).astype(np.complex64)
        assert np.array_equal(oracle.pilot_rotate(r).real, ((np.arange(K) + (K + 1) // 2) % K))


def test_shift_closed_form(oracle):
    # shiftOneRow (cpuLS.hpp:135-149): out[k] = Z[(k + (K-1)/2) mod K]
    for K in (3, 63, 1023, 2047):
        z = np.arange(K).astype(np.complex64)
        assert np.array_equal(oracle.shift_one_row(z).real, (np.arange(K) + (K - 1) // 2) % K)
    # shift undoes the pilot rotation
    z = np.arange(1023).astype(np.complex64)
    assert np.array_equal(oracle.shift_one_row(oracle.pilot_rotate(z)), z)
    # even K (odd C): the three memmoves rotate the first K-1 values by K/2-1
    # and leave the last in place (what the library's out_pos_any reproduces)
    for K in (2, 6, 1022, 1534):
        z = np.arange(K).astype(np.complex64)
        exp = np.concatenate([(np.arange(K - 1) + K // 2 - 1) % (K - 1), [K - 1]])
        assert np.array_equal(oracle.shift_one_row(z).real, exp)


@pytest.mark.parametrize("C", [4, 8, 64, 256, 1024, 2048, 4096, 2, 3, 6, 12, 600, 1021, 1200, 1536, 6144, 8192])
def test_oracle_fft_matches_numpy(oracle, C):
    rng = np.random.default_rng(C)
    x = (rng.standard_normal((3, C)) + 1j * rng.standard_normal((3, C))).astype(np.complex64)
    ref = np.fft.fft(x.astype(np.complex128), axis=-1)
    got = oracle.fft_rows(x)
    # exact DFT rounded once to float32
    assert np.max(np.abs(got - ref)) <= 1e-6 * np.max(np.abs(ref))
    inv = oracle.fft_rows(x, inverse=True)
    refi = np.fft.ifft(x.astype(np.complex128), axis=-1) * C
    assert np.max(np.abs(inv - refi)) <= 1e-6 * np.max(np.abs(refi))


@pytest.mark.parametrize("C", [4, 64, 1024, 4096])
def test_oracle_f32_fft_for_cpu_baseline(oracle, C):
    """The single-precision FFT that bench.py's cpu_baseline times (the
    precision class of the reference's fftwf) computes the same transform:
    within f32 radix-2 rounding of the exact DFT, and the receiver built on it
    within the north-star tolerance of the float64-FFT oracle."""
    rng = np.random.default_rng(C + 1)
    x = (rng.standard_normal((3, C)) + 1j * rng.standard_normal((3, C))).astype(np.complex64)
    ref = np.fft.fft(x.astype(np.complex128), axis=-1)
    got = oracle.fft_rows_f32(x)
    assert np.max(np.abs(got - ref)) <= 2e-6 * np.log2(C) * np.max(np.abs(ref))
    if C == 1024:
        z = np.load(os.path.join(GOLDEN, "cfg1_r4_c1024_s10.npz"))
        a = oracle.frames_demod(z["iq"], z["X"], int(z["prefix"]))
        b = oracle.frames_demod_fft32(z["iq"], z["X"], int(z["prefix"]))
        assert np.linalg.norm(b - a) <= 1e-5 * np.linalg.norm(a)


@needs_ref
@pytest.mark.parametrize("R,C", [(1, 4), (3, 64), (16, 1024), (64, 1024), (7, 2048), (2, 7), (3, 12), (4, 1536),
                                 (2, 1023)])
def test_oracle_bitexact_vs_reference_build(oracle, R, C):
    ref = Reference()
    rng = np.random.default_rng(R * C)
    Y = (rng.standard_normal((R, C)) + 1j * rng.standard_normal((R, C))).astype(np.complex64)
    X = (rng.standard_normal(C - 1) + 1j * rng.standard_normal(C - 1)).astype(np.complex64)
    H1, P1 = oracle.ls(Y, X)
    H2, P2 = ref.ls(Y, X)
    assert np.array_equal(bits(H1), bits(H2)) and np.array_equal(bits(P1), bits(P2))
    Y2 = (rng.standard_normal((R, C)) + 1j * rng.standard_normal((R, C))).astype(np.complex64)
    assert np.array_equal(bits(oracle.mrc(Y2, H1, P1)), bits(ref.mrc(Y2, H2, P2)))
    row = (rng.standard_normal(C - 1) + 0j).astype(np.complex64)
    assert np.array_equal(bits(oracle.shift_one_row(row)), bits(ref.shift_one_row(row)))


@needs_ref
def test_reference_matrix_readX_vs_oracle(oracle, tmp_path):
    ref = Reference()
    for K in (1023, 2047, 255):
        raw = (np.arange(K) + 1j * np.arange(K)).astype(np.complex64)
        p = tmp_path / f"p{K}.dat"
        raw.tofile(p)
        assert np.array_equal(bits(ref.matrix_readX(str(p), K)), bits(oracle.pilot_rotate(raw)))
    # missing file: the CPU path fills 0.707 + 0.707i (cpuLS.hpp:84-90)
    X = ref.matrix_readX(str(tmp_path / "missing.dat"), 15)
    assert np.all(X == np.complex64(0.707 + 0.707j))


def test_fast_fft_matches_scalar_oracle_fft(oracle):
    """oracle/fft_fast.c (the timed CPU baseline's vectorised FFT) computes
    the same transform as oracle_fft_row_f32, bit for bit, at every power of
    two the scalar one handles; and a frame demod through it equals the
    scalar-FFT demod."""
    rng = np.random.default_rng(17)
    for C in (4, 16, 128, 1024, 2048, 4096):
        x = (rng.standard_normal((3, C)) + 1j * rng.standard_normal((3, C))).astype(np.complex64)
        assert np.array_equal(oracle.fft_rows_fast(x), oracle.fft_rows_f32(x)), C
    F, S, R, C = 2, 5, 4, 1024
    iq = (rng.standard_normal((F, S, R, C + 8)) + 1j * rng.standard_normal((F, S, R, C + 8))).astype(np.complex64)
    X = ((rng.choice([-1, 1], C - 1) + 1j * rng.choice([-1, 1], C - 1)) * 0.7071).astype(np.complex64)
    assert np.array_equal(oracle.frames_demod_fast(iq, X, 8, nthreads=2), oracle.frames_demod_fft32(iq, X, 8, nthreads=2))
