#!/usr/bin/env python3
"""Generate the golden fixtures in tests/golden/ (run in the build container,
where /root/reference exists).

Inputs: seeded numpy frames in the receiver's convention (SURVEY.md 8(a)
item 7): bins j+1 carry H[r][j] * x[j], bin 0 empty, y = ifft(Y) * sqrt(C)
plus complex Gaussian noise, optional cyclic prefix.
Expected outputs: the reference's own RX arithmetic (oracle/_ref, compiled
from /root/reference/cpuLS.hpp by oracle/build_ref.sh: divideOneRow,
findDistSqrd, matrixMultThenSum, shiftOneRow, matrix_readX) applied to the
FFT of each row.  FFTW3 is absent from the image, so the FFT stage is the
exact DFT (float64, rounded to float32), which matches numpy/pocketfft.

Each fixture .npz holds: iq (F,S,R,C+prefix) or yf (F,S,R,C) complex64,
X (K,) complex64 rotated pilots, out (F,S-1,K) complex64, H (F,R,K), P (F,K),
plus scalars R, C, S, prefix, seed, domain ('time'|'freq').
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from oracle_bindings import Oracle, Reference  # noqa: E402

CASES = [
    # name, F, S, R, C, prefix, domain, noise
    ("cfg1_r4_c1024_s10", 1, 10, 4, 1024, 0, "time", 0.01),
    ("r16_c1024_s4_2frames", 2, 4, 16, 1024, 0, "time", 0.01),
    ("r64_c1024_s2", 1, 2, 64, 1024, 0, "time", 0.01),
    ("r8_c2048_s3_cp16", 1, 3, 8, 2048, 16, "time", 0.01),
    ("r4_c256_s5_cp32", 2, 5, 4, 256, 32, "time", 0.05),
    ("r3_c64_s4_odd_antennas", 2, 4, 3, 64, 0, "time", 0.01),
    ("freq_r16_c1024_s3", 1, 3, 16, 1024, 0, "freq", 0.01),
    # round 4: configs[4]'s C (the wave-pair kernels k_ls_td4096 / k_mrc_td4096h)
    ("r8_c4096_s3_cp32", 1, 3, 8, 4096, 32, "time", 0.01),
    ("r32_c4096_s2", 1, 2, 32, 4096, 0, "time", 0.01),
]


def qpsk(rng, shape):
    a = np.float32(0.70710678)
    return (rng.choice([-a, a], shape) + 1j * rng.choice([-a, a], shape)).astype(np.complex64)


def make_case(o, ref, name, F, S, R, C, prefix, domain, noise, seed, raw_pilots_path):
    rng = np.random.default_rng(seed)
    K = C - 1
    X = ref.matrix_readX(raw_pilots_path, K) if C == 1024 else o.pilot_rotate(qpsk(rng, K))
    iq = []
    outs, Hs, Ps = [], [], []
    for f in range(F):
        H = ((rng.standard_normal((R, K)) + 1j * rng.standard_normal((R, K))) / np.sqrt(2))
        syms = [X] + [qpsk(rng, K) for _ in range(S - 1)]
        frame = np.zeros((S, R, C + (prefix if domain == "time" else 0)), np.complex64)
        for s in range(S):
            Yb = np.zeros((R, C), np.complex128)
            Yb[:, 1:] = H * syms[s][None, :]
            nz = noise / np.sqrt(2) * (rng.standard_normal((R, C)) + 1j * rng.standard_normal((R, C)))
            if domain == "time":
                y = (np.fft.ifft(Yb, axis=-1) * np.sqrt(C) + nz).astype(np.complex64)
                frame[s, :, prefix:] = y
                if prefix:
                    frame[s, :, :prefix] = y[:, C - prefix:]
            else:
                frame[s] = (Yb + nz).astype(np.complex64)
        iq.append(frame)
        # expected: reference arithmetic on the FFT'd symbols
        if domain == "time":
            Yf = o.fft_rows(frame[:, :, prefix:])
        else:
            Yf = frame
        Hc, P = ref.ls(Yf[0], X)
        out = np.stack([ref.mrc(Yf[s], Hc, P) for s in range(1, S)])
        outs.append(out)
        Hs.append(Hc)
        Ps.append(P)
    key = "iq" if domain == "time" else "yf"
    np.savez_compressed(os.path.join(HERE, name + ".npz"), **{key: np.stack(iq)}, X=X,
                        out=np.stack(outs), H=np.stack(Hs), P=np.stack(Ps), R=R, C=C, S=S,
                        prefix=prefix, seed=seed, domain=domain)


def main():
    o, ref = Oracle(), Reference()
    rng = np.random.default_rng(20181)
    # a raw Pilots.dat (K = 1023 complex floats, the file matrix_readX reads)
    raw = qpsk(rng, 1023)
    pil = os.path.join(HERE, "Pilots.dat")
    raw.tofile(pil)
    X = ref.matrix_readX(pil, 1023)
    np.save(os.path.join(HERE, "pilots_rotated_k1023.npy"), X)
    only = sys.argv[1:]  # optional: regenerate only the named cases (seeds stay by position)
    for i, c in enumerate(CASES):
        if only and c[0] not in only:
            continue
        make_case(o, ref, *c, seed=1234 + i, raw_pilots_path=pil)
        print("wrote", c[0])


if __name__ == "__main__":
    main()
