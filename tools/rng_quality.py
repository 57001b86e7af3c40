"""Statistical screen of dropout-mask generators (round 5 RNG redesign): keep rate, neighbour correlations along
rows / columns / the pair halves / strides, and 2x2-block pattern chi-square, on [rows, W] element grids.

    python tools/rng_quality.py [rows] [W]

Each generator maps (key, row, column-pair) -> 32 random bits (lo16 -> even column, hi16 -> odd column)."""
import sys

import numpy as np

M32 = np.uint64(0xFFFFFFFF)


def mix32(x):
    x = x.astype(np.uint64) & M32
    x ^= x >> np.uint64(16)
    x = (x * np.uint64(0x7FEB352D)) & M32
    x ^= x >> np.uint64(15)
    x = (x * np.uint64(0x846CA68B)) & M32
    x ^= x >> np.uint64(16)
    return x


def fmix1(x, m=0x2C1B3C6D):
    y = (x * np.uint64(m)) & M32
    return y ^ (y >> np.uint64(16))


G = np.uint64(0x9E3779B9)


def gen_current(key, r, cp, W):
    pair = (r * np.uint64(W // 2) + cp) & M32
    return mix32(pair ^ np.uint64(key))


def gen_weyl_xor(key, r, cp, W):
    R = mix32(r ^ np.uint64(key))
    return fmix1(R ^ ((cp * G) & M32))


def gen_weyl_add(key, r, cp, W):  # negative control: x*M distributes over +
    R = mix32(r ^ np.uint64(key))
    return fmix1((R + cp * G) & M32)


def gen_weyl_xs(key, r, cp, W):
    R = mix32(r ^ np.uint64(key))
    x = R ^ ((cp * G) & M32)
    x ^= x >> np.uint64(16)
    return fmix1(x)


def gen_colhash(key, r, cp, W):
    R = mix32(r ^ np.uint64(key))
    Cc = mix32(cp ^ np.uint64(key ^ 0x5BD1E995))
    return fmix1(R ^ Cc)


def clmul32(v, k):
    v = v.astype(np.uint64) & M32
    out = np.zeros(np.broadcast(v, v).shape, dtype=np.uint64)
    for i in range(32):
        if (k >> i) & 1:
            out ^= (v << np.uint64(i)) & M32
    return out


def gen_rowmix_clmul(key, r, cp, W, kc=0x6D2B79F5, m=0x9E3779B1):
    R = mix32(r ^ np.uint64(key))
    return fmix1(R ^ clmul32(cp, kc), m)


def gen_rowmix_lin(key, r, cp, W):  # negative-ish control: sparse linear column word
    R = mix32(r ^ np.uint64(key))
    return fmix1(R ^ (cp ^ (cp << np.uint64(7)) & M32), 0x9E3779B1)


GENS = {"rowmix_clmul": gen_rowmix_clmul, "rowmix_lin": gen_rowmix_lin, "current": gen_current, "weyl_xor": gen_weyl_xor, "weyl_add": gen_weyl_add, "weyl_xs": gen_weyl_xs,
        "colhash": gen_colhash}


def keep_grid(gen, key, rows, W, thr, row0=0):
    r = (np.arange(rows, dtype=np.uint64) + np.uint64(row0))[:, None]
    cp = np.arange(W // 2, dtype=np.uint64)[None, :]
    h = gen(key, r, cp, W)
    lo = (h & np.uint64(0xFFFF)) >= thr
    hi = (h >> np.uint64(16)) >= thr
    k = np.empty((rows, W), dtype=bool)
    k[:, 0::2] = lo
    k[:, 1::2] = hi
    return k


def corr(a, b):
    a = a.astype(np.float64).ravel()
    b = b.astype(np.float64).ravel()
    a -= a.mean()
    b -= b.mean()
    return float((a * b).mean() / np.sqrt((a * a).mean() * (b * b).mean()))


def screen(name, rows, W, p=0.1, keys=(1, 0xDEADBEEF, 12345)):
    thr = np.uint64(int(round(p * 65536)))
    q = 1.0 - int(thr) / 65536.0
    n = 0
    kept = 0
    worst = {}
    chis = []
    for key in keys:
        k = keep_grid(GENS[name], key, rows, W, thr)
        n += k.size
        kept += int(k.sum())
        N = k.size
        sig = 1.0 / np.sqrt(N)  # correlation noise floor
        tests = {"pair_halves": (k[:, 0::2], k[:, 1::2]), "col+2": (k[:, :-2], k[:, 2:]),
                 "col+1": (k[:, :-1], k[:, 1:]), "row+1": (k[:-1], k[1:]), "diag": (k[:-1, :-2], k[1:, 2:])}
        for s in (4, 8, 16, 32, 64, 128):
            if s < W:
                tests[f"col+{s}"] = (k[:, :-s], k[:, s:])
            tests[f"row+{s}"] = (k[:-s], k[s:])
        for t, (a, b) in tests.items():
            z = corr(a, b) / sig
            worst[t] = max(worst.get(t, 0.0), abs(z))
        # 2x2 block patterns (rows r, r+1; columns 2j, 2j+2 -> two different pairs, two rows): 16 categories
        a = k[0::2, 0::2][:, 0::2].astype(np.int64)
        b = k[0::2, 0::2][:, 1::2].astype(np.int64)
        c = k[1::2, 0::2][:, 0::2].astype(np.int64)
        d = k[1::2, 0::2][:, 1::2].astype(np.int64)
        m = min(a.shape[1], b.shape[1])
        pat = (a[:, :m] + 2 * b[:, :m] + 4 * c[:, :m] + 8 * d[:, :m]).ravel()
        obs = np.bincount(pat, minlength=16).astype(np.float64)
        ones = np.array([bin(i).count("1") for i in range(16)])
        exp = pat.size * (q ** ones) * ((1 - q) ** (4 - ones))
        chis.append(float(((obs - exp) ** 2 / exp).sum()))
    rate = kept / n
    z_rate = (rate - q) / np.sqrt(q * (1 - q) / n)
    bad = {t: round(z, 1) for t, z in worst.items() if z > 4.5}
    print(f"{name:10s} W={W} n={n:.2e} keep={rate:.6f} (z={z_rate:+.2f} vs {q:.6f})  chi2_2x2(15 dof)="
          f"{[round(c, 1) for c in chis]}  max|z|={max(worst.values()):.1f}  fails={bad}", flush=True)


if __name__ == "__main__":
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 8192
    W = int(sys.argv[2]) if len(sys.argv) > 2 else 512
    names = sys.argv[3].split(",") if len(sys.argv) > 3 else list(GENS)
    for nm in names:
        screen(nm, rows, W)
