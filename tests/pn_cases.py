"""Synthetic receive buffers for the PN frame-sync tests (rx_and_corr.cpp:
a BPSK PN sequence of length L embedded at a lag of one channel, scaled by a
complex gain, in complex Gaussian noise).  The reference correlates without a
conjugate (temp += pn[j] * buff[i+j], rx_and_corr.cpp:347), so a real +-1 PN
peaks at |gain| there."""
import numpy as np


def pn_seq(L, seed=5):
    rng = np.random.default_rng(seed)
    return rng.choice([-1.0, 1.0], L).astype(np.complex64)


def rx_buffer(R, N, L, hits, noise=0.05, seed=1):
    """hits: {channel: (lag, gain)}; returns (buf (R, N) complex64, pn (L,))."""
    rng = np.random.default_rng(seed)
    pn = pn_seq(L, seed + 100)
    buf = noise * (rng.standard_normal((R, N)) + 1j * rng.standard_normal((R, N))) / np.sqrt(2)
    for ch, (lag, gain) in hits.items():
        buf[ch, lag:lag + L] += gain * pn
    return buf.astype(np.complex64), pn
