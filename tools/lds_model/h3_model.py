"""LDS bank model of conv_kernel_h2<512>'s h3-entry / h2-residual accesses (csrc/fdr_impala_h.hip): array cycles and
conflict cycles per env step, per access site.  python tools/lds_model/h3_model.py"""
import collections
from check import R128, R64, W64, W128

R32 = [list(range(32)), list(range(32, 64))]


def cycles(addrs, groups, nd, mod):
    """LDS-array cycles of one wave-instruction: per lane group, the max number of distinct dwords on one bank
    (addrs: lane -> first dword or None)."""
    tot = 0
    for g in groups:
        banks = collections.defaultdict(set)
        for l in g:
            a = addrs[l]
            if a is None:
                continue
            for k in range(nd):
                banks[(a + k) % mod].add(a + k)
        tot += max((len(v) for v in banks.values()), default=0)
    return tot


KIND = {  # (groups, dwords per lane, bank modulus)
    "r128": (R128, 4, 64), "r64": (R64, 2, 64), "r32": (R32, 1, 32),
    "w64": (W64, 2, 32), "w128": (W128, 4, 32), "w32": (R32, 1, 32),
}
t16 = lambda q: (q >> 2) & 1
t32 = lambda q: (q >> 1) & 3
x16 = lambda m: (m >> 3) & 1
x32 = lambda m: (m >> 2) & 3


def tidx(C, q, ch):
    return q * C + (((ch >> 3) ^ (t16(q) if C == 16 else t32(q))) << 3) + (ch & 7)


def xidx(C, m, ch):
    return m * C + (((ch >> 3) ^ (x16(m) if C == 16 else x32(m))) << 3) + (ch & 7)


site = collections.defaultdict(lambda: [0, 0, 0])  # name -> [instructions, array cycles, ideal cycles]


def acc(name, kind, halves, count=1):
    """halves: lane -> halves offset (or None); count: how many times per env step"""
    groups, nd, mod = KIND[kind]
    a = [None if h is None else h // 2 for h in halves]
    c = cycles(a, groups, nd, mod)
    ideal = sum(1 for g in groups if any(a[l] is not None for l in g))
    s = site[name]
    s[0] += count
    s[1] += c * count
    s[2] += ideal * count


# ---- frame bands (18 padded rows x 66 x 4 halves; r0 = 2 for bands 1..3): 8 b16 / b32 stores per item
for band in range(4):
    r0 = 0 if band == 0 else 2
    for wave in range(8):
        for j in range(8):
            hv = [None] * 64
            for l in range(64):
                i = wave * 64 + l
                if i >= (18 - r0) * 24:
                    continue
                c = i % 3; w = (i // 3) & 7; r = r0 + i // 24
                hv[l] = (r * 66 + 1 + w * 8) * 4 + c + 4 * j
            if any(h is not None for h in hv):
                acc("frame stores", "w32", hv)
# ---- stage-1 band conv reads (conv_band_s1): 8 tiles x (lo, hi b64 + tap-8 b64) per wave per band
def koff3(tap):
    return ((tap // 3) * 66 + tap % 3) * 4
for wave in range(8):
    for i in range(8):
        for part in range(3):
            hv = [None] * 64
            for l in range(64):
                g = l >> 4; ll = l & 15
                off = ((i >> 2) * 66 + 32 * ((i >> 1) & 1) + (i & 1)) * 4
                p = (2 * wave * 66 + 2 * ll) * 4
                tap = (2 * g + part) if part < 2 else 8
                hv[l] = p + off + koff3(tap if tap < 9 else 0)
            acc("s1 band conv B reads", "r64", hv, 4)
# ---- band_out_h3 (stage 1: COUT 16, H 64, EO; stage 2: 32, 32; stage 3: 32, 16)
def band_out(stage, COUT, H, EO, nbands, T):
    NT = COUT // 16; NV = (2 if EO else 2 * (H // 16)) if COUT == 16 else 2 * (H // 16)
    if stage == 1:
        NV = 2
    SLOT = (H // 2) * COUT
    for band in range(nbands):
        for wave in range(8):
            for v in range(NV):
                ex = [None] * 64; rd = [None] * 64; xs = [None] * 64; ts = [None] * 64
                for l in range(64):
                    g = l >> 4; ll = l & 15
                    st = EO or (ll & 1) == 0
                    p = 16 * (v // NT) + ll if EO else 8 * (v // NT) + (ll >> 1)
                    ch = (v % NT) * 16 + 4 * g
                    if st:
                        ex[l] = ((band & 1) * 8 + wave) * SLOT + p * COUT + ch
                        xs[l] = xidx(COUT, (8 * band + wave) * (H // 2) + p, ch)
                        if T:
                            HO = H // 2
                            ts[l] = tidx(COUT, (8 * band + wave + 1) * (HO + 2) + p + 1, ch)
                    rd[l] = ((band & 1) * 8 + max(wave - 1, 0)) * SLOT + p * COUT + ch
                acc("s%d exchange stores" % stage, "w64", ex)
                acc("s%d exchange reads" % stage, "r64", rd)
                acc("s%d X stores" % stage, "w64", xs)
                if T and (stage == 3 or band == 1):
                    acc("s%d T stores (BN->padded)" % stage, "w64", ts)
band_out(1, 16, 64, True, 4, False)
band_out(2, 32, 32, False, 2, True)
band_out(3, 32, 16, False, 1, True)
# ---- stage-2/3 band conv B reads (conv_band_nat<CIN, H>), A reads contiguous
def band_nat(stage, CIN, H, nbands):
    TR = H // 16; NF = (9 * CIN) // 32; cpg = CIN // 8; tpk = 32 // CIN
    WP = H + 2
    for band in range(nbands):
        r0 = 16 * band
        for wave in range(8):
            for s in range(NF):
                for rho in range(2):
                    for k in range(TR):
                        hv = [None] * 64
                        for l in range(64):
                            g = l >> 4; ll = l & 15
                            tap = s * tpk + g // cpg
                            q = (r0 + 2 * wave) * WP + ll + rho * WP + (tap // 3) * WP + tap % 3 + 16 * k
                            hv[l] = tidx(CIN, q, 8 * (g % cpg))
                        acc("s%d band conv B reads" % stage, "r128", hv)
                acc("s%d band conv A reads" % stage, "r128", [l * 8 for l in range(64)], 2)
            if CIN == 16:  # tap 8 on K = 16
                for rho in range(2):
                    for k in range(TR):
                        hv = [None] * 64
                        for l in range(64):
                            g = l >> 4; ll = l & 15
                            q = (r0 + 2 * wave) * WP + ll + rho * WP + 2 * WP + 2 + 16 * k
                            hv[l] = q * CIN + (((g >> 1) ^ t16(q)) << 3) + 4 * (g & 1)
                        acc("s%d band conv B reads" % stage, "r64", hv)
band_nat(2, 16, 32, 2)
band_nat(3, 32, 16, 1)
# ---- residual convs (conv_h2): B reads; epilogue T stores, X reads / stores
def res(stage, C, H, split):
    W = H; WP = H + 2; MT = H * W // 16; NTA = C // 16
    NW = 8 // (2 if split else 1); NT = NTA // (2 if split else 1)
    TPW = (MT + NW - 1) // NW
    NF = (9 * C) // 32; cpg = C // 8; tpk = 32 // C
    for wv in range(8):
        wave = wv % NW; nt0 = (wv // NW) * NT if split else 0
        for i in range(TPW):
            mt = wave + NW * i
            if mt >= MT:
                continue
            for s in range(NF):
                hv = [None] * 64
                for l in range(64):
                    g = l >> 4; m = mt * 16 + (l & 15); q0 = (m // W) * WP + m % W
                    tap = s * tpk + g // cpg
                    q = q0 + (tap // 3) * WP + tap % 3
                    hv[l] = tidx(C, q, 8 * (g % cpg))
                acc("s%d res conv B reads" % stage, "r128", hv, 4)
            if C == 16:
                hv = [None] * 64
                for l in range(64):
                    g = l >> 4; m = mt * 16 + (l & 15); q = (m // W) * WP + m % W + 2 * WP + 2
                    hv[l] = q * C + (((g >> 1) ^ t16(q)) << 3) + 4 * (g & 1)
                acc("s%d res conv B reads" % stage, "r64", hv, 4)
            for nt in range(NT):
                ts = [None] * 64; xs = [None] * 64
                for l in range(64):
                    g = l >> 4; m = mt * 16 + (l & 15); q = (m // H + 1) * WP + m % H + 1
                    ch = (nt0 + nt) * 16 + 4 * g
                    ts[l] = tidx(C, q, ch); xs[l] = xidx(C, m, ch)
                acc("s%d res epilogue T stores" % stage, "w64", ts, 4)
                acc("s%d res epilogue X reads" % stage, "r64", xs, 2)
                acc("s%d res epilogue X stores" % stage, "w64", xs, 1)
        if C == 32:
            for s in range(NF):
                acc("s%d res conv A reads" % stage, "r128", [l * 8 for l in range(64)], 4 * NT)
res(1, 16, 32, False)
res(2, 32, 16, False)
res(3, 32, 8, True)

tot = [0, 0, 0]
print("%-32s %8s %10s %10s %10s" % ("site", "insts", "cycles", "ideal", "conflict"))
for k, (n, c, i) in sorted(site.items(), key=lambda kv: -(kv[1][1] - kv[1][2])):
    print("%-32s %8d %10d %10d %10d" % (k, n, c, i, c - i))
    tot = [tot[0] + n, tot[1] + c, tot[2] + i]
print("%-32s %8d %10d %10d %10d" % ("total (modelled)", *tot, tot[1] - tot[2]))
