"""olsdif_model.py -- numpy model of fir_dif2_kernel (csrc/fir_fft.hip):
overlap-save with an 8192-point channel-pair frame split over two waves,
decimated in FREQUENCY (one exchange, of the outputs).

Frame f covers input [f P - 1024, f P + 7168), P = 7168, u = x0 + i x1,
and owns outputs [f P, (f + 1) P):

  wave 0   a[m] = u[m] + u[m + 4096]                       m < 4096
           ye = IDFT4096(DFT4096(a) * H[0::2])             (unnormalised)
  wave 1   b[m] = (u[m] - u[m + 4096]) W8192^m
           t[n] = W8192^-n IDFT4096(DFT4096(b) * H[1::2])[n]
  y[n] = ye[n] + t[n] (wave 0 stores n in [1024, 4096)),
  y[n + 4096] = ye[n] - t[n] (wave 1 stores n in [0, 4096));
  H = FFT_8192(taps) / 8192 (the unnormalised inverses' scale: exact).

The lane / register layout is the 4096-point transforms' own (m = l + 64 r,
k = l + 64 q with the (q, q + 32) pairing of the packed combine); `table`
is capi.cpp dif2_table's layout of H, read back here in that pairing.

    python tools/olsdif_model.py     (against np.convolve in float64)
"""
import numpy as np

N, M, P, HIST = 8192, 4096, 7168, 1024


def W(n, e):
    return np.exp(-2j * np.pi * np.asarray(e, dtype=float) / n)


def table(taps):
    """dif2_table: [odd][q][lane] -> (H[2k + odd], H[2k' + odd]), k = l + 64 q,
    k' = k + 2048, as complex pairs (the float4 re, re, im, im)."""
    h = np.zeros(N)
    h[:len(taps)] = taps
    H = np.fft.fft(h) / N
    t = np.zeros((2, 32, 64, 2), complex)
    for odd in range(2):
        for q in range(32):
            for l in range(64):
                k = l + 64 * q
                t[odd, q, l] = (H[2 * k + odd], H[2 * (k + 2048) + odd])
    return t


def spectrum_of(t, odd):
    """The wave's 4096 bins back out of the table's pairing."""
    Hw = np.zeros(M, complex)
    for q in range(32):
        for l in range(64):
            k = l + 64 * q
            Hw[k], Hw[k + 2048] = t[odd, q, l]
    return Hw


def frame(u, t):
    m = np.arange(M)
    a = u[:M] + u[M:]
    b = (u[:M] - u[M:]) * W(N, m)
    ye = np.fft.ifft(np.fft.fft(a) * spectrum_of(t, 0)) * M            # wave 0
    tt = np.conj(W(N, m)) * np.fft.ifft(np.fft.fft(b) * spectrum_of(t, 1)) * M  # wave 1
    y = np.empty(N, complex)
    y[:M], y[M:] = ye + tt, ye - tt
    return y[HIST:]


def render(x0, x1, taps):
    L = len(x0)
    t = table(taps)
    F = -(-L // P)
    out = np.zeros(F * P, complex)
    for f in range(F):
        s0 = f * P - HIST
        u = np.zeros(N, complex)
        lo, hi = max(0, s0), min(L, s0 + N)
        if lo < hi:
            u[lo - s0:hi - s0] = x0[lo:hi] + 1j * x1[lo:hi]
        out[f * P:(f + 1) * P] = frame(u, t)
    return out[:L]


def main():
    rng = np.random.default_rng(9)
    for L, T in [(7168 * 3 + 555, 1024), (100, 1024), (7168 * 2, 1025), (50_000, 17)]:
        taps = rng.standard_normal(T) / np.sqrt(T)
        x0, x1 = rng.uniform(-1, 1, L), rng.uniform(-1, 1, L)
        y = render(x0, x1, taps)
        err = max(np.abs(y.real - np.convolve(x0, taps)[:L]).max(), np.abs(y.imag - np.convolve(x1, taps)[:L]).max())
        print(f"L = {L:6d}, taps = {T:5d}: max |err| vs np.convolve = {err:.2e}")
        assert err < 1e-9, err
    print("ok")


if __name__ == "__main__":
    main()
