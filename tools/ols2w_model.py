"""ols2w_model.py -- numpy model of the next FIR kernel:
overlap-save with an 8192-point channel-pair frame split over two waves.

Frame f covers input [f P - 1024, f P + 7168), P = 7168, and owns outputs
[f P, (f + 1) P).  u[n] = x0[s] + i x1[s] (s = f P - 1024 + n; zero outside
[0, L) and for a channel the file lacks).  Decimation in time over the two
waves of the frame -- no exchange of the input:

  wave A   loads the even samples u[2m] (lane l, register r: m = l + 64 r;
           dword loads at a stride of 2 floats), E = DFT4096(u[2m])
  wave B   loads the odd samples u[2m + 1], O = DFT4096(u[2m + 1]),
           then T[k] = W8192^k O[k]
  exch 1   A sends E[k], B sends T[k] (same lane / register for the same k)
  A        Y[k]        = (E[k] + T[k]) H[k]            k < 4096
  B        Y[k + 4096] = (E[k] - T[k]) H[k + 4096]
  exch 2   A sends Y[k], B sends Y[k + 4096]
  A        y[2m]     = IDFT4096(Y[k] + Y[k + 4096])[m]
  B        y[2m + 1] = IDFT4096((Y[k] - Y[k + 4096]) W8192^-k)[m]
  store    m >= 512 (n = 2m + e >= 1024): out0 = Re, out1 = Im, at
           f P + n - 1024, stride-2 dword stores per wave

H = FFT_8192(taps) / 8192 (the two unnormalised inverse halves' scale, a
power of two: exact); A reads H[0, 4096), B H[4096, 8192).  Per wave the
work is one forward and one inverse 4096-point transform (the pair kernel's)
plus, on B, a twiddle multiply each way, for 7,168 outputs per channel
instead of 3,072 per 4096-point frame.

This checks the index math, the twiddle signs, the scaling and the edges
against np.convolve in float64:  python tools/ols2w_model.py
"""
import numpy as np

N, M, P, HIST = 8192, 4096, 7168, 1024


def W(n, e):
    return np.exp(-2j * np.pi * np.asarray(e, dtype=float) / n)


def tables(taps):
    """H8192 = FFT_8192(taps zero-padded) / 8192, split per wave."""
    h = np.zeros(N)
    h[:len(taps)] = taps
    H = np.fft.fft(h) / N
    return H[:M], H[M:]


def frame(u, HA, HB):
    """One frame's 7,168 outputs per channel (complex: out0 + i out1)."""
    k = np.arange(M)
    # the waves' loads: lane l, register r -> m = l + 64 r (the model keeps m order)
    ue, uo = u[0::2], u[1::2]
    E = np.fft.fft(ue)                      # wave A
    T = W(N, k) * np.fft.fft(uo)            # wave B
    # exchange 1 (the same k on the same lane / register in both waves)
    YA = (E + T) * HA                       # wave A: Y[k]
    YB = (E - T) * HB                       # wave B: Y[k + 4096]
    # exchange 2
    ye = np.fft.ifft(YA + YB) * M           # wave A: y[2m] (unnormalised IDFT4096)
    yo = np.fft.ifft((YA - YB) * np.conj(W(N, k))) * M   # wave B: y[2m + 1]
    y = np.empty(N, complex)
    y[0::2], y[1::2] = ye, yo
    return y[HIST:]                         # n >= 1024: m >= 512 on both waves


def render(x0, x1, taps):
    L = len(x0)
    HA, HB = tables(taps)
    F = -(-L // P)
    out = np.zeros(F * P, complex)
    for f in range(F):
        s0 = f * P - HIST
        u = np.zeros(N, complex)
        lo, hi = max(0, s0), min(L, s0 + N)
        if lo < hi:
            u[lo - s0:hi - s0] = x0[lo:hi] + 1j * x1[lo:hi]
        out[f * P:(f + 1) * P] = frame(u, HA, HB)
    return out[:L]


def main():
    rng = np.random.default_rng(7)
    for L, T in [(7168 * 3 + 555, 1024), (100, 1024), (7168 * 2, 1025), (50_000, 17)]:
        taps = rng.standard_normal(T) / np.sqrt(T)
        x0, x1 = rng.uniform(-1, 1, L), rng.uniform(-1, 1, L)
        y = render(x0, x1, taps)
        r0, r1 = np.convolve(x0, taps)[:L], np.convolve(x1, taps)[:L]
        err = max(np.abs(y.real - r0).max(), np.abs(y.imag - r1).max())
        print(f"L = {L:6d}, taps = {T:5d}: max |err| vs np.convolve = {err:.2e}")
        assert err < 1e-9, err
    # the work per output against the pair kernel's 4096-point frame
    print("outputs per channel per two-wave frame: 7168 (pair kernel: 3072 per one-wave frame, 6144 per two waves)")
    print("ok")


if __name__ == "__main__":
    main()
