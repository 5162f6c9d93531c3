"""PN frame sync on the GPU (ofdm_pn_correlate / ofdm_pn_extract, SURVEY.md
8(f) rank 3) against the oracle restatement of rx_and_corr.cpp:332-392.
The hit (channel, lag) is an index: it must equal the oracle's exactly, also
when the threshold equals a lag's value to the last bit; the per-lag
magnitudes are computed in the reference's f32 order and must be bit-equal.
Extraction is a copy: bit-equal.  End to end: buffer -> correlate -> extract
-> ofdm_frame_demod equals the receiver on the original frames."""
import numpy as np
import pytest

from helpers import parity
from pn_cases import pn_seq, rx_buffer

pytestmark = pytest.mark.gpu


def dev_t(a, dev):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).to(dev)


@pytest.mark.parametrize("R,N,L", [(2, 5000, 127), (3, 3000, 1500), (1, 2100, 2047),
                                   (4, 1030, 1024), (2, 9000, 1023), (5, 1100, 1)])
def test_pn_mags_and_hit_bitexact(ofdm, oracle, dev, R, N, L):
    lag = (N - L) // 2
    buf, pn = rx_buffer(R, N, L, {R - 1: (lag, 0.7 + 0.4j)}, seed=R * N + L)
    ref_pos, ref_mag = oracle.pn_correlate(buf, pn, 0.5, mag=True)
    pos, mag = ofdm.pn_correlate(dev_t(buf, dev), dev_t(pn, dev), 0.5, mag=True)
    mag = mag.cpu().numpy()
    bad = np.flatnonzero(mag.ravel() != ref_mag.ravel())
    assert bad.size == 0, (bad.size, mag.ravel()[bad[:4]], ref_mag.ravel()[bad[:4]])
    assert int(pos.item()) == ref_pos
    pos2, _ = ofdm.pn_correlate(dev_t(buf, dev), dev_t(pn, dev), 0.5)  # early-exit form
    assert int(pos2.item()) == ref_pos


def test_pn_search_order_and_threshold_edges(ofdm, oracle, dev):
    R, N, L = 4, 20000, 255
    buf, pn = rx_buffer(R, N, L, {1: (15000, 1.0), 3: (100, 1.2)}, seed=9)
    nl = N - L + 1
    _, mag = oracle.pn_correlate(buf, pn, 0.0, mag=True)
    db, dp = dev_t(buf, dev), dev_t(pn, dev)
    t1 = np.float32(mag[1].max())
    t_up = np.nextafter(t1, np.float32(np.inf))
    cases = [0.5,                    # channel 1 first although channel 3's peak is earlier in time
             float(mag[3].max()),    # only channel 3's peak reaches it
             float(t1),              # == channel 1's peak value: >= holds there
             float(t_up),            # one ulp above: channel 1 drops out
             float(mag.max()) * 2,   # no hit
             0.0]                    # every lag reaches it: (0, 0)
    for th in cases:
        ref_pos, _ = oracle.pn_correlate(buf, pn, th)
        for want_mag in (False, True):
            pos, _ = ofdm.pn_correlate(db, dp, th, mag=want_mag)
            assert int(pos.item()) == ref_pos, (th, want_mag, int(pos.item()), ref_pos)
    assert oracle.pn_correlate(buf, pn, 0.5)[0] == 1 * nl + 15000


def test_pn_short_and_empty(ofdm, dev):
    buf, pn = rx_buffer(2, 50, 63, {})
    pos, mag = ofdm.pn_correlate(dev_t(buf, dev), dev_t(pn, dev), 0.0, mag=True)
    assert int(pos.item()) == -1 and mag.numel() == 0


@pytest.mark.parametrize("lag,cp", [(0, 0), (1, 16), (4000, 72)])
def test_pn_extract_bitexact(ofdm, oracle, dev, lag, cp):
    import torch
    R, N, L, C = 3, 12000, 511, 1024
    rng = np.random.default_rng(lag + cp)
    b1 = (rng.standard_normal((R, N)) + 1j * rng.standard_normal((R, N))).astype(np.complex64)
    b2 = (rng.standard_normal((R, N)) + 1j * rng.standard_normal((R, N))).astype(np.complex64)
    nsym = (N - L) // (C + cp)
    pos = torch.tensor([2 * (N - L + 1) + lag], dtype=torch.int64, device=dev)  # hit on channel 2
    got = ofdm.pn_extract(dev_t(b1, dev), dev_t(b2, dev), L, pos, C, cp, nsym).cpu().numpy()
    assert np.array_equal(got, oracle.pn_extract(b1, b2, L, lag, C, cp, nsym))
    # no hit: the output is left untouched
    out = torch.full((nsym, R, C), 7.0, dtype=torch.complex64, device=dev)
    ofdm.pn_extract(dev_t(b1, dev), dev_t(b2, dev), L, torch.tensor([-1], device=dev), C, cp,
                    nsym, out=out)
    assert bool((out == 7.0).all())


def test_pn_sync_to_demod_end_to_end(ofdm, oracle, dev):
    """rx_and_corr's two receive buffers, PN at `lag` on every channel,
    followed by one frame (S symbols of C + cp samples per channel) ->
    correlate -> extract -> ofdm_frame_demod == the receiver on the frame."""
    import torch
    S, R, C, cp, L, lag = 11, 8, 1024, 72, 1023, 3333
    a = np.float32(0.70710678)
    rng = np.random.default_rng(21)
    Xh = (rng.choice([-a, a], C - 1) + 1j * rng.choice([-a, a], C - 1)).astype(np.complex64)
    X = dev_t(Xh, dev)
    iq = ofdm.synth_frames(1, S, R, C, X, prefix=cp, seed=77, noise_std=0.01)  # (1, S, R, C+cp)
    stream = iq[0].permute(1, 0, 2).reshape(R, S * (C + cp)).cpu().numpy()  # per-channel time series
    pn = pn_seq(L, 3)
    N = lag + L + S * (C + cp) - 500  # the frame spills 500 samples into the second buffer
    tot = np.zeros((R, 2 * N), np.complex64)
    tot += (0.01 * (rng.standard_normal((R, 2 * N)) + 1j * rng.standard_normal((R, 2 * N)))
            ).astype(np.complex64)
    tot[:, lag:lag + L] += 0.5 * pn
    tot[:, lag + L:lag + L + S * (C + cp)] = stream
    b1, b2 = tot[:, :N].copy(), tot[:, N:].copy()
    pos, _ = ofdm.pn_correlate(dev_t(b1, dev), dev_t(pn, dev), 0.1)
    ref_pos, _ = oracle.pn_correlate(b1, pn, 0.1)
    assert int(pos.item()) == ref_pos == lag  # channel 0
    sym = ofdm.pn_extract(dev_t(b1, dev), dev_t(b2, dev), L, pos, C, cp, S)
    assert torch.equal(sym.cpu(), iq[0, :, :, cp:].cpu())
    out = ofdm.frame_demod(sym.view(1, S, R, C), X, 0)
    ref = ofdm.frame_demod(iq, X, cp)
    parity(out.cpu().numpy(), ref.cpu().numpy())
    assert int(ofdm.count_symbol_errors(out, S, seed=77).item()) == 0
