"""olsave_model.py -- numpy model of the overlap-save FIR kernel (fir_fft.hip):
one 8192-point frame per wavefront, lane l / register b layout m = l + 64 b,
forward 64x64 four-step + paired real split, H multiply, inverse split with
the partner exchange, inverse four-step.  Checks index math and scaling."""
import numpy as np

M, N = 4096, 8192


def W(n, e):
    return np.exp(-2j * np.pi * e / n)


def fwd4096(z):  # z[l + 64 b] -> Z[kb + 64 ka] as array [lane kb][ka]
    v = z.reshape(64, 64).T.copy()               # v[l][b] = z[l + 64 b]
    Y = np.fft.fft(v, axis=1)                    # DFT over b -> kb, per lane l
    Y *= W(4096, np.outer(np.arange(64), np.arange(64)))   # W^(l kb)
    T = Y.T.copy()                               # lane kb, reg a = l
    return np.fft.fft(T, axis=1)                 # DFT over a -> ka: Z[kb + 64 ka]


def inv4096(Zl):  # Zl[lane kb][ka] -> z'[l + 64 b] (unnormalised inverse)
    S = np.fft.ifft(Zl, axis=1) * 64             # IDFT over ka -> a (unnormalised)
    S *= np.conj(W(4096, np.outer(np.arange(64), np.arange(64))))  # W^-(a kb), [kb][a]
    T = S.T.copy()                               # lane a, reg kb
    z = np.fft.ifft(T, axis=1) * 64              # IDFT over kb -> b: [a][b]
    return z.T.reshape(-1)                       # m = a + 64 b -> index via [b][a]


def frame(x8192, Hs):
    z = x8192[0::2] + 1j * x8192[1::2]
    Z = fwd4096(z)                               # [lane][ka] = Z[lane + 64 ka]
    Zf = np.empty(M, complex)
    for l in range(64):
        for ka in range(64):
            Zf[l + 64 * ka] = Z[l, ka]
    assert np.allclose(Zf, np.fft.fft(z))
    Zp = np.empty((64, 64), complex)             # Z' in the same layout
    for l in range(64):
        for ka in range(32):
            k = l + 64 * ka
            P = Zf[(M - k) % M]                  # partner (lane 0: own Z[64 - ka])
            E = Zf[k] + np.conj(P)
            D = Zf[k] - np.conj(P)
            T = -1j * D * W(N, k)
            X1, X2 = E + T, E - T                # 2 X[k], conj(2 X[M - k])
            Yk = X1 * Hs[k]
            YMk = np.conj(X2) * Hs[M - k]
            E2 = Yk + np.conj(YMk)
            O2 = (Yk - np.conj(YMk)) * np.conj(W(N, k))
            Zk = E2 + 1j * O2
            ZMk = np.conj(E2) + 1j * np.conj(O2)
            Zp[l, ka] = Zk
            if k == 0:
                continue                         # pair (0, M): one output
            kk = M - k                           # lands at lane kk % 64, reg kk // 64
            Zp[kk % 64, kk // 64] = ZMk
    # self-paired k = 2048 (lane 0, ka = 32)
    k = 2048
    Y2 = (Zf[k] + np.conj(Zf[k]) + (-1j) * (Zf[k] - np.conj(Zf[k])) * W(N, k)) * Hs[k]
    E2 = Y2 + np.conj(Y2)
    O2 = (Y2 - np.conj(Y2)) * np.conj(W(N, k))
    Zp[0, 32] = E2 + 1j * O2
    zp = inv4096(Zp)
    y = np.empty(N)
    y[0::2] = zp.real
    y[1::2] = zp.imag
    return y


rng = np.random.default_rng(0)
T_ = 1024
h = rng.standard_normal(T_)
Hf = np.fft.fft(np.concatenate([h, np.zeros(N - T_)]))
Hs = Hf / 16384.0
x = rng.standard_normal(N)
y = frame(x, Hs)
ref = np.real(np.fft.ifft(np.fft.fft(x) * Hf))  # circular convolution
print("max err vs circular conv:", np.max(np.abs(y - ref)))
lin = np.convolve(x, h)[:N]
print("valid part n>=1023 err:", np.max(np.abs(y[1023:] - lin[1023:])))
