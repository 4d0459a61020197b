// fdr_impala_h.hip -- fp16 mode of the ImpalaPolicy path (BASELINE config 5: "impala policy fp16
// rollouts").  Same network and step structure as fdr_impala.hip; what changes:
//   * weights: theta' (computed in f32, bit-exact) rounded once to f16 into the half pack;
//   * conv stack: activations f16 in LDS, HWC layout, v_mfma_f32_16x16x32_f16 with f32 accumulation;
//     BN / bias / ReLU / residual adds in f32, rounded to f16 when stored;
//   * fc + LSTM: f16 weights streamed (half the HBM bytes), f32 activations and accumulation.
// Orientation: the WEIGHTS are the MFMA A operand (16 output channels x 32 K), the pixels the B
// operand (32 K x 16 pixels), so a lane's 4 results are 4 consecutive channels of one pixel -> one
// 8-byte LDS store, and one 16-byte pixel fragment feeds both output-channel tiles.
#include <hip/hip_runtime.h>

#include <cfloat>
#include <cmath>

#include "fdr_impala.h"

namespace fdr {
namespace impala {

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef _Float16 h2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

// pixel stride (halves) of an MFMA input image: unpadded (the chunk swizzle below spreads the banks); the
// frame image keeps its 4 channel slots.
template <int C>
struct Pix {
  static constexpr int CS = C == 3 ? 4 : C;
};

// Chunk swizzles (a chunk = 8 channels = one 16-B fragment read; the chunk index is XORed with a few bits of
// the pixel index, so every access below stays a whole aligned chunk or half chunk).  Chosen with a bank
// model of every access of the stack over the lane groups of MI355X_MICROARCH.md's LDS table
// (ds_read_b128 4 x 16 / b64 2 x 32 lanes, 64 banks; ds_write_b64 4 x 16 / b128 8 x 8 lanes, 32 banks):
//   padded images T: conv B-fragment reads (b128) conflict-free at 16 x 16 / 32 x 32 (2-way: the K = 16 tap-8
//   read, the 8 x 8 stage's 2-row tiles), epilogue stores (b64) 2-way, to_padded stores (b128) free;
//   X / S (unpadded [pixel][C]): residual reads free, residual / band-scratch stores 2-way, pool reads 2-way,
//   to_padded reads and pool stores free.
// Without them (r05g PMC, conv_kernel_h): SQ_LDS_BANK_CONFLICT = 44 % of SQ_LDS_IDX_ACTIVE -- the residual
// and band-scratch stores were 8-way at 32 channels (pixel pitch 64 B = 16 banks), the epilogue stores 4-way.
template <int C>
__device__ __forceinline__ int tsw(int q) { return C == 16 ? (q >> 2) & 1 : (q >> 1) & 3; }
template <int C>
__device__ __forceinline__ int xsw(int m) { return C == 16 ? (m >> 3) & 1 : (m >> 2) & 3; }
// halves offset of channel ch of padded pixel q (T) / of pixel m (X, S)
template <int C>
__device__ __forceinline__ int tidx(int q, int ch) { return q * Pix<C>::CS + (((ch >> 3) ^ tsw<C>(q)) << 3) + (ch & 7); }
template <int C>
__device__ __forceinline__ int xidx(int m, int ch) { return m * C + (((ch >> 3) ^ xsw<C>(m)) << 3) + (ch & 7); }

// conv weight staging buffer WB (halves): the A fragments of the widest conv (32 -> 32, 9 k-steps x 2
// channel tiles).  Every wave of the workgroup needs the same fragments; fetched from the pack by
// all 8 waves they cost 8 x 18 KB of vector-memory traffic per conv (~2,000 clocks of TA issue the
// waves stall on).  Instead the workgroup copies each conv's block ONCE into WB (16 B per thread per
// chunk) and the waves read their fragments from LDS.
constexpr int kWB = 9 * 2 * 64 * 8;

// ---- conv on f16 MFMA ---------------------------------------------------------------------------
template <int CIN>
struct KSteps {
  static constexpr int N = CIN == 3 ? 2 : (9 * CIN + 31) / 32;
  // The last K-step of the Cin = 3 and Cin = 16 convs is mostly padding (taps 8 + zeros: 27 -> 64,
  // 144 -> 160): it runs as v_mfma_f32_16x16x16_f16, K = 16 (lane group g supplies k = 4g .. 4g+3 of
  // tap 8), so the executed K is 48 and 144.
  static constexpr bool kRem = CIN == 3 || CIN == 16;
  static constexpr int NF = kRem ? N - 1 : N;  // full K = 32 steps
};

typedef unsigned u32x4 __attribute__((ext_vector_type(4)));

// Cin = 16: the last fragment in the K = 16 layout (lane (o, g) holds tap 8 channels 4g .. 4g+3), read
// straight from the K = 32 layout of the pack / WB (lane (o, g') holds k = 128 + 8g' .. +7, i.e. tap 8
// channels 8g' .. 8g'+7 for g' < 2, zeros above): halves 4(g & 1) .. +3 of lane (o, g >> 1)'s chunk.
// Cin = 3 needs no move: lane (o, 0) holds tap 8's four channel slots in halves 0..3 and every other lane
// zeros there.
template <int CIN, int NT>
__device__ __forceinline__ void rem_fragment(const _Float16* w, h8 (&af)[KSteps<CIN>::N][NT], int lane) {
  if constexpr (CIN == 16) {
    constexpr int s = KSteps<CIN>::N - 1;
    const int g = lane >> 4, src = (lane & 15) + 16 * (g >> 1);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) {
      const h4 v = *reinterpret_cast<const h4*>(w + (((s * NT + nt) * 64) + src) * 8 + 4 * (g & 1));
      af[s][nt] = h8{v[0], v[1], v[2], v[3], 0, 0, 0, 0};
    }
  }
}

// A fragments of one conv for ALL output-channel tiles, af[s][nt] (4 VGPRs each), from the workgroup's LDS copy of
// the block (layout identical to the pack's).  R32: the last
// fragment stays in the pack's K = 32 layout (tap 8 + zeros; conv_h2 R32).
template <int CIN, int NT, bool R32 = false>
__device__ __forceinline__ void load_af_lds(const _Float16* wb, h8 (&af)[KSteps<CIN>::N][NT], int lane) {
#pragma unroll
  for (int s = 0; s < KSteps<CIN>::N; ++s)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) af[s][nt] = *reinterpret_cast<const h8*>(wb + (((s * NT + nt) * 64) + lane) * 8);
  if constexpr (!R32) rem_fragment<CIN, NT>(wb, af, lane);
}
template <int CIN, int NT>
constexpr int kBlockHalves = KSteps<CIN>::N * NT * 64 * 8;

// Workgroup copy of one conv's weight block into WB, split so the HBM/L2 latency hides behind other
// work: issue() starts the loads (16-B chunks, chunk c by thread c mod 512), commit() stores them to
// WB.  WB protocol (every phase ends in a barrier): read WB -> af in phase k, commit the next block
// in phase k+1 or later, read it in a phase after the commit.
template <int NTH>
struct WStageT {
  // a block = NC 16-B chunks: NC / NTH full rounds of one chunk per thread in r[], and the remainder REM = NC % NTH
  // either as one more chunk for threads < REM (rq) or, when it fits, as one dword per thread (rd): the 32 -> 32
  // blocks' 1,152 chunks over 512 threads then take 2 chunks + 1 dword = 9 VGPRs, not 12 (the 12th..9th were
  // spilled right behind their global load, which stalled the issuing wave on the load)
  static constexpr int kMaxFull = (kWB / 8) / NTH;
  u32x4 r[kMaxFull > 0 ? kMaxFull : 1];
  u32x4 rq;
  uint32_t rd;
  template <int NH>
  __device__ __forceinline__ void issue(const _Float16* __restrict__ src) {
    constexpr int NC = NH / 8, PERF = NC / NTH, REM = NC % NTH;
    static_assert(NH % 8 == 0 && NH <= kWB && PERF <= kMaxFull, "weight block");
#pragma unroll
    for (int k = 0; k < PERF; ++k) r[k] = reinterpret_cast<const u32x4*>(src)[threadIdx.x + k * NTH];
    if constexpr (REM > 0 && REM * 4 <= NTH) {  // (branch-free: the clamped re-read is not stored)
      rd = reinterpret_cast<const uint32_t*>(src + PERF * NTH * 8)[min((int)threadIdx.x, REM * 4 - 1)];
    } else if constexpr (REM > 0) {
      rq = reinterpret_cast<const u32x4*>(src)[PERF * NTH + min((int)threadIdx.x, REM - 1)];
    }
  }
  template <int NH>
  __device__ __forceinline__ void commit(_Float16* wb) const {
    constexpr int NC = NH / 8, PERF = NC / NTH, REM = NC % NTH;
#pragma unroll
    for (int k = 0; k < PERF; ++k) reinterpret_cast<u32x4*>(wb)[threadIdx.x + k * NTH] = r[k];
    if constexpr (REM > 0 && REM * 4 <= NTH) {
      if ((int)threadIdx.x < REM * 4) reinterpret_cast<uint32_t*>(wb + PERF * NTH * 8)[threadIdx.x] = rd;
    } else if constexpr (REM > 0) {
      if ((int)threadIdx.x < REM) reinterpret_cast<u32x4*>(wb)[PERF * NTH + threadIdx.x] = rq;
    }
  }
};
using WStage = WStageT<kHThreads>;

// offset (halves) of this lane's 8 K-elements of k-step s inside the receptive field of a pixel
template <int CIN, int CS, int WP>
__device__ __forceinline__ int k_offset(int s, int g, int part) {
  int tap;
  int ch = 0;
  if (CIN == 3) {
    tap = 8 * s + 2 * g + part;
  } else {
    constexpr int cpg = CIN / 8, tpk = 32 / CIN;
    tap = s * tpk + g / cpg;
    ch = 8 * (g % cpg);
  }
  if (tap >= 9) tap = 0;  // zero weights: any in-bounds pixel
  return ((tap / 3) * WP + tap % 3) * CS + ch;
}

__device__ __forceinline__ h4 to_h4(float a, float b, float c, float d) {
  return h4{(_Float16)a, (_Float16)b, (_Float16)c, (_Float16)d};
}

// fmaf((float)x.lo / x.hi, s, t) as one v_fma_mix_f32 (the f16 operand is converted inside the instruction, one
// rounding -- fmaf's value; the compiler picks the same instruction for that pattern when it does not pair the
// fmas into v_pk_fma_f32, which then needs a separate conversion per element)
__device__ __forceinline__ float fma_mix_lo(h2 x, float s, float t) {
  float r;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(x), "v"(s), "v"(t));
  return r;
}
__device__ __forceinline__ float fma_mix_hi(h2 x, float s, float t) {
  float r;
  asm("v_fma_mix_f32 %0, %1, %2, %3 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(x), "v"(s), "v"(t));
  return r;
}
__device__ __forceinline__ h2 lo2(h4 v) { return __builtin_shufflevector(v, v, 0, 1); }
__device__ __forceinline__ h2 hi2(h4 v) { return __builtin_shufflevector(v, v, 2, 3); }
// ReLU after the f16 rounding (two v_pk_max_f16): the value of rounding relu(x) (a negative x gives -0 or +0)
__device__ __forceinline__ h4 relu_h4(h4 v) { return __builtin_elementwise_max(v, h4{0, 0, 0, 0}); }

// T <- BN(X) (optionally ReLU): X [H][H][C] f16 -> padded image [H+2][H+2][CS]; BORDER: zero border.
template <int C, int H, bool RELU, bool BORDER, int NTH = kHThreads>
__device__ __forceinline__ void to_padded_h(const _Float16* X, _Float16* T, const float* sc, const float* sh) {
  constexpr int CS = Pix<C>::CS, WP = H + 2, G = C / 8;
  static_assert(NTH % G == 0, "a thread keeps one 8-channel group");
  constexpr int PPI = NTH / G, NP = H * H, IT = (NP + PPI - 1) / PPI;
  const int cg = threadIdx.x % G;
  float scv[8], shv[8];  // this thread's channels: loaded once, not per pixel
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    scv[k] = sc[8 * cg + k];
    shv[k] = sh[8 * cg + k];
  }
#pragma unroll
  for (int it = 0; it < IT; ++it) {
    const int pix = threadIdx.x / G + it * PPI;
    if (NP % PPI != 0 && pix >= NP) break;
    const int y = pix / H, x = pix % H;
    const h8 v = *reinterpret_cast<const h8*>(X + xidx<C>(pix, 8 * cg));
    const h2 p[4] = {__builtin_shufflevector(v, v, 0, 1), __builtin_shufflevector(v, v, 2, 3),
                     __builtin_shufflevector(v, v, 4, 5), __builtin_shufflevector(v, v, 6, 7)};
    h4 o[2];
#pragma unroll
    for (int hq = 0; hq < 2; ++hq) {
      const int k = 4 * hq;
      o[hq] = to_h4(fma_mix_lo(p[2 * hq], scv[k], shv[k]), fma_mix_hi(p[2 * hq], scv[k + 1], shv[k + 1]),
                    fma_mix_lo(p[2 * hq + 1], scv[k + 2], shv[k + 2]), fma_mix_hi(p[2 * hq + 1], scv[k + 3], shv[k + 3]));
      if (RELU) o[hq] = relu_h4(o[hq]);
    }
    *reinterpret_cast<h8*>(T + tidx<C>((y + 1) * WP + x + 1, 8 * cg)) = __builtin_shufflevector(o[0], o[1], 0, 1, 2, 3, 4, 5, 6, 7);
  }
  if (BORDER) {
    const h8 z = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int i = threadIdx.x; i < 4 * (H + 1) * G; i += NTH) {
      const int cg = i % G, r = i / G, side = r / (H + 1), k = r - side * (H + 1);
      const int pix = side == 0 ? k : side == 1 ? (H + 1) * WP + 1 + k : side == 2 ? (k + 1) * WP : k * WP + WP - 1;
      *reinterpret_cast<h8*>(T + pix * CS + 8 * cg) = z;
    }
  }
}

// Zero border of a padded image [H+2][H+2][CS] (the interior is written by a conv epilogue).
template <int C, int H>
__device__ __forceinline__ void zero_border_h(_Float16* T) {  // (kHThreads = conv_kernel_h2<512>'s block too)
  constexpr int CS = Pix<C>::CS, WP = H + 2, G = C / 8;
  const h8 z = {0, 0, 0, 0, 0, 0, 0, 0};
  for (int i = threadIdx.x; i < 4 * (H + 1) * G; i += kHThreads) {
    const int cg = i % G, r = i / G, side = r / (H + 1), k = r - side * (H + 1);
    const int pix = side == 0 ? k : side == 1 ? (H + 1) * WP + 1 + k : side == 2 ? (k + 1) * WP : k * WP + WP - 1;
    *reinterpret_cast<h8*>(T + pix * CS + 8 * cg) = z;
  }
}

// =====================================================================================================
// conv_kernel_h2: the fp16 conv stack, one env per 8-wave workgroup, TWO workgroups per CU (<= 80 KiB LDS, <= 128
// VGPRs: 4 waves per SIMD -- the register file, not the LDS, is what admits no third workgroup).  One env's ~36
// barrier-separated phases per step (entry convs, pools, BN passes, epilogues) overlap the other workgroup's MFMA
// phases.  The stage-1 frame is generated per 16-row entry band (double-buffered: band b+1's rows are made during
// band b's pool phase); the stage entries pool in registers (below); residual convs are single-buffered (conv ->
// accumulators -> barrier -> in-place epilogue); the stage-2 entry writes its pooled rows into the dead rows of its
// own input image; WB is placed per stage (2,560 halves beside X1 in stage 1, 9,216 after X1 dies).
// LDS map (halves, R = arena after the BN / bias tables; every buffer below R + 38,080):
//   stage 1 entry : FB0 | FB1 | EX1 (kH3*) | X1 [18496, 34880) | WB_A [34880, 37440)
//   stage 1 res   : T1 [0, 18496) | X1 | WB_A
//   stage 2 entry : T1 (X2 into [0, 8192) band by band) | EX2 | WB_B [27712, 36928)
//   stage 2 res   : X2 [0, 8192) | T2 [8192, 18560) | WB_B
//   stage 3 entry : X3 [0, 2048) | T2 | EX3 | WB_B
//   stage 3 res   : X3 | T3 [2048, 5248) | WB_B
// =====================================================================================================
constexpr int kH2Arena = 38080;                           // halves
constexpr int kH2X1 = 18496, kH2WBA = 34880, kH2WBB = 27712, kH2T2 = 8192, kH2T3 = 2048;
constexpr int kH2LdsBytes = 3 * kBnTab * 4 + kH2Arena * 2;
static_assert(kH2LdsBytes <= 80 * 1024, "two conv_kernel_h2 workgroups per CU");
static_assert(kH2X1 + 32 * 32 * 16 == kH2WBA && kH2WBA + 2560 <= kH2Arena, "stage 1 map");
static_assert(34 * 34 * 16 <= kH2X1 && kH2WBB + kWB <= kH2Arena, "stage 2 map");
static_assert(16 * 16 * 32 <= kH2T2 && kH2T2 + 18 * 18 * 32 <= kH2WBB, "stage 3 map");
static_assert(8 * 8 * 32 <= kH2T3 && kH2T3 + 10 * 10 * 32 <= kH2T2, "stage 3 res map");
static_assert(3 * kBnTab * 2 >= 34 * 16, "row -1 guard");

// The residual convs in tile-outer order (every K-step of tile i, then tile i + 1): K-outer order keeps 5 pixel
// addresses per tile live at once (80 VGPRs in the stage-1 residual convs, which spilled), tile-outer order keeps
// one tile's.  Dependent MFMAs on one accumulator
// issue back to back (SrcC forwarding of the same opcode), and the other workgroup's waves fill the SIMD.
// STREAM (Cin = 32 at 8 waves, where 72 fragment VGPRs do not fit beside the accumulators under 128): the A
// fragments are read from the LDS weight block ws per K-step (K-outer: both channel tiles' fragments, then every
// tile's B fragment of that step) instead of af -- the same products in the same K order.
// NTA / nt0 (streamed form): the block holds NTA channel tiles, this wave computes tiles nt0 .. nt0 + NT - 1.
// R32 (conv_kernel_h2<512>): the tap-8 remainder runs as one more v_mfma_f32_16x16x32_f16 on the pack's K = 32
// fragment (tap 8 + zeros) chained onto the accumulator -- a K = 16 MFMA takes the same 16-clock slot
// (profiles/r08a_mfma_rate_probe.txt), and the separate accumulator's VALU add (the K = 16 product cannot be chained:
// DESIGN.md 3.4 SrcC) and its registers go.
template <int CIN, int CS, int NT, int TPW, int W, int WP, int MT, int NW, bool STREAM = false, int NTA = NT,
          bool R32 = false>
__device__ __forceinline__ void conv_h2(const _Float16* Tin, const h8 (&af)[KSteps<CIN>::N][NT],
                                        f32x4 (&acc)[TPW][NT], int wave, int lane, int qoff = 0,
                                        const _Float16* ws = nullptr, int nt0 = 0) {
  constexpr int KS = KSteps<CIN>::N, NF = KSteps<CIN>::NF;
  // A wave's tiles are wave + NW i: tile i's pixels are tile 0's shifted by DQ i padded pixels (whole rows),
  // so every read is one of NF per-lane addresses plus an immediate.  The chunk swizzle of q + DQ i is the
  // swizzle of q XOR flip(i) when DQ keeps the swizzle bits carry-free (asserted).
  constexpr int DQ = W >= 16 ? (NW / (W / 16)) * WP : NW * (16 / W) * WP;
  static_assert(W >= 16 ? NW % (W / 16) == 0 : 16 % W == 0, "tile rows");
  static_assert(CIN == 3 || (CIN == 16 && DQ % 4 == 0) || (CIN == 32 && DQ % 8 == 0), "swizzle step");
  auto flip = [](int i) { return CIN == 16 ? ((DQ * i) >> 2) & 1 : (CIN == 32 ? ((DQ * i) >> 1) & 3 : 0); };
  const int g = lane >> 4, m0 = wave * 16 + (lane & 15);
  const int base = (m0 / W) * WP + (m0 % W);  // padded pixel of tap 0, tile 0
  int off[NF], sw[NF];
#pragma unroll
  for (int s = 0; s < NF; ++s) {
    if constexpr (CIN == 3) {
      off[s] = base * CS;
      sw[s] = 0;
    } else {
      constexpr int cpg = CIN / 8, tpk = 32 / CIN;
      const int tap = s * tpk + g / cpg, q = base + (tap / 3) * WP + tap % 3;
      off[s] = q * CS;
      sw[s] = (g % cpg) ^ tsw<CIN>(q + qoff);
    }
  }
  auto live = [&](int i) { return TPW * NW == MT || i < TPW - 1 || wave + NW * i < MT; };  // wave-uniform
  const int qr = base + 2 * WP + 2;  // tap 8
  const int offr = CIN == 3 ? qr * CS : qr * CS + 4 * (g & 1);
  const int swr = CIN == 3 ? 0 : (g >> 1) ^ tsw<CIN>(qr + qoff);
  const int offr32 = qr * CS, swr32 = CIN == 3 ? 0 : (g & 1) ^ tsw<CIN>(qr + qoff);
  (void)offr32, (void)swr32;
  if constexpr (STREAM) {
    static_assert(CIN == 32 || CIN == 16, "streamed fragments: Cin = 16 / 32");
#pragma unroll
    for (int i = 0; i < TPW; ++i)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[i][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NF; ++s) {
      h8 a[NT], b[TPW];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) a[nt] = *reinterpret_cast<const h8*>(ws + (((s * NTA + nt0 + nt) * 64) + lane) * 8);
#pragma unroll
      for (int i = 0; i < TPW; ++i)
        if (live(i)) b[i] = *reinterpret_cast<const h8*>(Tin + DQ * i * CS + off[s] + ((sw[s] ^ flip(i)) << 3));
      // ordering point (as in the tile form): step s's reads are issued before step s-1's products are final,
      // and step s+1's only after -- one step of reads in flight
      if (s > 0) {
#pragma unroll
        for (int i = 0; i < TPW; ++i)
#pragma unroll
          for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(acc[i][nt]));
      }
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        if (!live(i)) continue;
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[nt], b[i], acc[i][nt], 0, 0, 0);
      }
    }
    if constexpr (KSteps<CIN>::kRem) {  // tap 8 on K = 16 (rem_fragment's lane map), added by VALU
      const int src = (lane & 15) + 16 * (g >> 1);
      h4 a[NT];
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        a[nt] = *reinterpret_cast<const h4*>(ws + ((((KS - 1) * NTA + nt0 + nt) * 64) + src) * 8 + 4 * (g & 1));
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        if (!live(i)) continue;
        const h4 b = *reinterpret_cast<const h4*>(Tin + DQ * i * CS + offr + ((swr ^ flip(i)) << 3));
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[i][nt] += __builtin_amdgcn_mfma_f32_16x16x16f16(a[nt], b, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
    }
    return;
  }
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[i][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
    if (live(i)) {
      const _Float16* Ti = Tin + DQ * i * CS;
#pragma unroll
      for (int s = 0; s < NF; ++s) {
        h8 b;
        if constexpr (CIN == 3) {
          const h4 lo = *reinterpret_cast<const h4*>(Ti + off[s] + k_offset<CIN, CS, WP>(s, g, 0));
          const h4 hi = *reinterpret_cast<const h4*>(Ti + off[s] + k_offset<CIN, CS, WP>(s, g, 1));
          b = h8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        } else {
          b = *reinterpret_cast<const h8*>(Ti + off[s] + ((sw[s] ^ flip(i)) << 3));
        }
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[s][nt], b, acc[i][nt], 0, 0, 0);
      }
      if constexpr (KSteps<CIN>::kRem && R32) {  // tap 8 + zeros on K = 32, chained
        static_assert(CIN == 16, "R32: the 16-channel residual convs");
        // lane group g: tap 8's chunk g & 1 (groups 2, 3 meet the fragment's zeros)
        const h8 b = *reinterpret_cast<const h8*>(Ti + offr32 + ((swr32 ^ flip(i)) << 3));
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[KS - 1][nt], b, acc[i][nt], 0, 0, 0);
      } else if constexpr (KSteps<CIN>::kRem) {  // tap 8 on K = 16, added by VALU (conv_h's note)
        const h4 b = *reinterpret_cast<const h4*>(Ti + offr + (CIN == 3 ? 0 : (swr ^ flip(i)) << 3));
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) {
          const h8 w = af[KS - 1][nt];
          acc[i][nt] += __builtin_amdgcn_mfma_f32_16x16x16f16(h4{w[0], w[1], w[2], w[3]}, b, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
        }
      }
    }
    // ordering point: tile i-1's accumulators are final before tile i+1's reads are issued (without it the DAG
    // linearisation issues every tile's reads up front and sinks the MFMAs to the epilogue: spills)
    if (i > 0) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(acc[i - 1][nt]));
    }
  }
}

// x / 255 for an integer-valued x in [0, 255], bit-identical to the IEEE division (checked exhaustively: q = x r,
// one fma residual correction): the synthetic frame's bytes, without the ~10-instruction division sequence.
__device__ __forceinline__ float div255_byte(float x) {
  constexpr float r = 1.0f / 255.0f;
  const float q = x * r;
  return fmaf(fmaf(-q, 255.0f, x), r, q);
}

// padded frame rows [p0 + r0, p0 + kH2FBRows) of this env (policies/impala.py:147 frame / 255, then BN2d(3) with
// this thread's per-channel scale sc / shift sh) into FB [rows][66][4] f16 -- zero outside the 64 x 64 image and
// in the 4th channel slot; conv_kernel_h's values.  Work item = (row, 8-pixel chunk, channel): one hash word (or
// 8 frame floats) -> 8 halves of one channel, spread over all 256 threads.  r0 = 3: the band's first three rows
// are the previous band's last three (prev), copied.
struct FrameBn {  // BN2d(3) of the frame: per-channel scale / shift (scalars: the struct is passed by value)
  float s0, s1, s2, h0, h1, h2;
};
template <int NTH, int FR>
__device__ __forceinline__ void frame_band_h2(_Float16* FB, const _Float16* prev, int r0, int p0, const StepArgs& a,
                                              int64_t env, int e, FrameBn bn) {
  const int nitem = (FR - r0) * 24;
  for (int i = threadIdx.x; i < nitem; i += NTH) {
    const int c = i % 3, w = (i / 3) & 7, r = r0 + i / 24, y = p0 + r - 1;  // image row of padded row p0 + r
    _Float16 o[8];
    if (y >= 0 && y < 64) {
      float fv[8];
      if (a.frames) {
        const float* fr = a.frames + (a.shared_frames ? (int64_t)e : env) * kFramePix + c * 4096 + y * 64 + w * 8;
#pragma unroll
        for (int j = 0; j < 8; ++j) fv[j] = fr[j] / 255.0f;
      } else {
        const uint64_t gid = (uint64_t)(a.lane_offset * a.envs + env);
        const uint64_t word = (uint64_t)(c * 512 + y * 8 + w);
        const uint64_t hb = mix64(a.fkey + ((gid << 32) | ((uint64_t)a.t << 11) | word) * kGolden);
#pragma unroll
        for (int j = 0; j < 8; ++j) fv[j] = div255_byte((float)((uint32_t)(hb >> (8 * j)) & 255u));
      }
      const float s_ = c == 0 ? bn.s0 : (c == 1 ? bn.s1 : bn.s2), h_ = c == 0 ? bn.h0 : (c == 1 ? bn.h1 : bn.h2);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (_Float16)fmaf(fv[j], s_, h_);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (_Float16)0.f;
    }
    _Float16* d = FB + (r * 66 + 1 + w * 8) * 4 + c;
    if (c == 2) {  // channel 2 and the zero 4th slot in one 4-byte store
#pragma unroll
      for (int j = 0; j < 8; ++j) *reinterpret_cast<h2*>(d + 4 * j) = h2{o[j], (_Float16)0.f};
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) d[4 * j] = o[j];
    }
  }
  // the two pad columns of every generated row, and the overlap rows
  const int npad = (FR - r0) * 2, ncopy = r0 * 66 * 4 / 8;
  for (int i = NTH - 1 - threadIdx.x; i < npad + ncopy; i += NTH) {
    if (i < npad)
      *reinterpret_cast<h4*>(FB + ((r0 + (i >> 1)) * 66 + (i & 1) * 65) * 4) = h4{0, 0, 0, 0};
    else
      reinterpret_cast<uint4*>(FB)[i - npad] = reinterpret_cast<const uint4*>(prev + (FR - r0) * 66 * 4)[i - npad];
  }
}

// -----------------------------------------------------------------------------------------------------
// Stage entries with the max pool in registers (conv_kernel_h2<512>; docs/DESIGN_LOG.md 3.4 "r07 entries").
// A band is 16 conv rows; wave w owns band rows 2w and 2w + 1, all their pixels, all output channels.  The 3 x 3 /
// stride-2 pool then needs no image of the conv output: horizontally the window's three columns are in
// neighbouring lanes (DPP), vertically pooled row w is max(row 2w - 1, 2w, 2w + 1) -- rows 2w, 2w + 1 are the
// wave's own, row 2w - 1 is wave w - 1's second row, handed over through a small exchange slot (EX) across the
// band's one barrier (wave 0 takes the previous band's wave-7 slot).  Per band: conv, pool, export, barrier,
// import, X store -- one barrier instead of conv / S store / barrier / pool / barrier, and no S image.
// Values: max commutes with the monotone f16(f32(v + b)) of the S store, so pooling the f32 sums and adding the
// bias after is conv_kernel_h's f16 pool output bit for bit.
// -----------------------------------------------------------------------------------------------------
constexpr int kH3FR = 18;                              // padded frame rows per stage-1 band (16 conv rows + 2)
constexpr int kH3FB = kH3FR * 66 * 4;                  // halves
// stage 1: FB0 | pad pixel | FB1 | pad pixel | EX (16 slots x 512).  The pad pixels (zeroed per env) are what the
// last buffer row's column-66 read of conv_band_s1's tap pairs (kx 2, 3 = zero weight) meets: finite zeros
constexpr int kH3FB0 = 0, kH3FB1 = kH3FB + 8, kH3EX1 = 2 * kH3FB + 16;
constexpr int kH3EX2 = 18560, kH3EX3 = 18560;          // stages 2 / 3: EX after T2's extent
static_assert(kH3EX1 + 16 * 512 <= kH2X1, "stage 1 h3 map");
static_assert(kH3EX2 + 16 * 512 <= kH2WBB && kH3EX3 + 8 * 256 <= kH2WBB, "stage 2/3 h3 map");

template <int CTRL>
__device__ __forceinline__ float dpp_f(float old, float src) {  // src from the DPP lane; invalid source: old
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(__builtin_bit_cast(int, old), __builtin_bit_cast(int, src),
                                                               CTRL, 0xF, 0xF, false));
}
constexpr int kDppShl1 = 0x101, kDppShr1 = 0x111, kDppRor1 = 0x121;

// Stage-1 band conv (Cin 3 -> 16 at 64 x 64) in even / odd pixel tiles: tile i = (rho = i >> 2, k = (i >> 1) & 1,
// par = i & 1) holds, in lane l, the 16 channels of pixel x = 2 (16 k + l) + par of band row 2 wave + rho -- so a
// pooled pixel's three columns 2p - 1, 2p, 2p + 1 are in one lane (even, odd tile) and its left neighbour (odd tile,
// one lane down).  FBb: the band's padded frame rows [18][66][4].
// K order (s1_frag): every lane group's two taps of a K-step are horizontally adjacent, (ky, kx0) and (ky, kx0 + 1),
// so a lane's B fragment is 16 contiguous bytes (one ds_read2_b64 into the operand registers, no assembly moves):
// K-step 0 = groups (0,0)(0,1) | (1,0)(1,1) | (2,0)(2,1) | (0,2)(0,3); K-step 1 = (1,2)(1,3) | (2,2)(2,3) | - | -.
// Column-3 taps and the empty groups carry zero weights (their B reads are finite pixels: pads and the buffers' pad
// pixel).  Both K-steps chain on one accumulator (same opcode).
__device__ __forceinline__ void s1_tap(int s, int g, int& ky, int& kx0) {
  if (s == 0) {
    ky = g < 3 ? g : 0;
    kx0 = g < 3 ? 0 : 2;
  } else {
    ky = g == 1 ? 2 : 1;
    kx0 = 2;
  }
}
// A fragments in that order, gathered per lane from the pack's K order (conv_h's: group g holds taps 2g, 2g + 1 of
// K-step t / 8; tap 8 in K-step 1, group 0)
__device__ __forceinline__ void s1_frag(const _Float16* __restrict__ w, h8 (&af)[2], int lane) {
  const int g = lane >> 4, m = lane & 15;
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    int ky, kx0;
    s1_tap(s, g, ky, kx0);
    h4 part[2];
#pragma unroll
    for (int pp = 0; pp < 2; ++pp) {
      const int kx = kx0 + pp, t = 3 * ky + kx;
      const bool valid = kx <= 2 && (s == 0 || g < 2);
      const int tt = valid ? t : 0;
      const h4 v = *reinterpret_cast<const h4*>(w + (((tt >> 3) * 64) + m + 16 * ((tt & 7) >> 1)) * 8 + 4 * (tt & 1));
      part[pp] = valid ? v : h4{0, 0, 0, 0};
    }
    af[s] = h8{part[0][0], part[0][1], part[0][2], part[0][3], part[1][0], part[1][1], part[1][2], part[1][3]};
  }
}
__device__ __forceinline__ void conv_band_s1(const _Float16* FBb, const h8 (&af)[2], f32x4 (&acc)[8], int wave, int lane) {
  constexpr int WP = 66, CS = 4;
  const int g = lane >> 4, l = lane & 15;
  const _Float16* p = FBb + (2 * wave * WP + 2 * l) * CS;
  int o[2];
#pragma unroll
  for (int s = 0; s < 2; ++s) {
    int ky, kx0;
    s1_tap(s, g, ky, kx0);
    o[s] = (ky * WP + kx0) * CS;
  }
  // two halves of 4 tiles (the second half's reads in flight under the first half's MFMAs, not all 16 up front)
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    h8 b[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * hf + j, off = ((i >> 2) * WP + 32 * ((i >> 1) & 1) + (i & 1)) * CS;
#pragma unroll
      for (int s = 0; s < 2; ++s) {  // 16 contiguous bytes at 8-byte alignment: two b64 halves
        const h4 lo = *reinterpret_cast<const h4*>(p + off + o[s]);
        const h4 hi = *reinterpret_cast<const h4*>(p + off + o[s] + 4);
        b[j][s] = __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
      }
    }
    if (hf > 0) {
#pragma unroll
      for (int j = 0; j < 4; ++j) asm volatile("" : "+v"(acc[j]));
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[4 * hf + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[0], b[j][0], f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[4 * hf + j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[1], b[j][1], acc[4 * hf + j], 0, 0, 0);
  }
}

// Band conv of stages 2 / 3 (Cin 16 / 32, Cout 32, H = 32 / 16) in natural tiles: tile i = (rho = i / TR, k = i % TR),
// lane l = pixel x = 16 k + l of band row 2 wave + rho (TR = H / 16 tiles per row), A fragments streamed from the LDS
// weight block ws per K-step (conv_h2 STREAM: the same products in the same K order).  Tin: the whole padded input
// image, r0: the band's first conv row.
template <int CIN, int H>
__device__ __forceinline__ void conv_band_nat(const _Float16* Tin, int r0, const _Float16* ws,
                                              f32x4 (&acc)[2 * (H / 16)][2], int wave, int lane) {
  constexpr int CS = Pix<CIN>::CS, WP = H + 2, NT = 2, TR = H / 16, NTL = 2 * TR, KS = KSteps<CIN>::N;
  constexpr int NF = KSteps<CIN>::NF, cpg = CIN / 8, tpk = 32 / CIN;
  const int g = lane >> 4, l = lane & 15;
  const int qb = (r0 + 2 * wave) * WP + l;  // padded pixel of tap 0, row rho = 0, k = 0
#pragma unroll
  for (int i = 0; i < NTL; ++i)
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) acc[i][nt] = f32x4{0.f, 0.f, 0.f, 0.f};
  // +16 pixels (tile k + 1) leaves the swizzle bits (bit 2 at 16 channels, bits 1-2 at 32) unchanged: one address
  // per (rho, K-step), k as an immediate
#pragma unroll
  for (int s = 0; s < NF; ++s) {
    const int tap = s * tpk + g / cpg, tq = (tap / 3) * WP + tap % 3;
    h8 a[NT], b[NTL];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) a[nt] = *reinterpret_cast<const h8*>(ws + (((s * NT + nt) * 64) + lane) * 8);
#pragma unroll
    for (int rho = 0; rho < 2; ++rho) {
      const int q = qb + rho * WP + tq;
      const _Float16* pa = Tin + q * CS + (((g % cpg) ^ tsw<CIN>(q)) << 3);
#pragma unroll
      for (int k = 0; k < TR; ++k) b[rho * TR + k] = *reinterpret_cast<const h8*>(pa + 16 * k * CS);
    }
    if (s > 0) {  // one K-step of reads in flight (conv_h2 STREAM's ordering point)
#pragma unroll
      for (int i = 0; i < NTL; ++i)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt) asm volatile("" : "+v"(acc[i][nt]));
    }
#pragma unroll
    for (int i = 0; i < NTL; ++i)
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) acc[i][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[nt], b[i], acc[i][nt], 0, 0, 0);
  }
  if constexpr (KSteps<CIN>::kRem) {  // tap 8 + zeros on K = 32 (the pack's fragment), chained
    h8 a[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) a[nt] = *reinterpret_cast<const h8*>(ws + ((((KS - 1) * NT + nt) * 64) + lane) * 8);
#pragma unroll
    for (int rho = 0; rho < 2; ++rho) {
      const int q = qb + rho * WP + 2 * WP + 2;
      const _Float16* pa = Tin + q * CS + (((g & 1) ^ tsw<CIN>(q)) << 3);
#pragma unroll
      for (int k = 0; k < TR; ++k) {
        const h8 b = *reinterpret_cast<const h8*>(pa + 16 * k * CS);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[rho * TR + k][nt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a[nt], b, acc[rho * TR + k][nt], 0, 0, 0);
      }
    }
  } else if constexpr (KSteps<CIN>::kRem) {  // tap 8 on K = 16 (rem_fragment's lane map), added by VALU
    const int src = l + 16 * (g >> 1);
    h4 a[NT];
#pragma unroll
    for (int nt = 0; nt < NT; ++nt) a[nt] = *reinterpret_cast<const h4*>(ws + ((((KS - 1) * NT + nt) * 64) + src) * 8 + 4 * (g & 1));
#pragma unroll
    for (int rho = 0; rho < 2; ++rho) {
      const int q = qb + rho * WP + 2 * WP + 2;
      const _Float16* pa = Tin + q * CS + (((g >> 1) ^ tsw<CIN>(q)) << 3) + 4 * (g & 1);
#pragma unroll
      for (int k = 0; k < TR; ++k) {
        const h4 b = *reinterpret_cast<const h4*>(pa + 16 * k * CS);
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
          acc[rho * TR + k][nt] += __builtin_amdgcn_mfma_f32_16x16x16f16(a[nt], b, f32x4{0.f, 0.f, 0.f, 0.f}, 0, 0, 0);
      }
    }
  }
}

// Horizontal 3-wide / stride-2 max of one row value v (natural tiles: lane l = pixel 16 k + l): valid in even lanes
// (pooled pixel 8 k + l / 2); vp = the row's previous tile (k > 0), whose lane 15 is column 16 k - 1.
__device__ __forceinline__ float hpool_nat(float v, float vp, bool first) {
  const float r = dpp_f<kDppShl1>(v, v);                     // column + 1 (lane 15: itself)
  const float l0 = first ? v : dpp_f<kDppRor1>(v, vp);       // lane 0: column - 1 from the previous tile
  const float lf = dpp_f<kDppShr1>(l0, v);                   // column - 1
  return fmaxf(fmaxf(v, r), lf);
}

// Pool, export, barrier, import, X store of one band (both tile forms).  P: this wave's two rows' horizontal pools
// combined, B: its second row's; both + bias, rounded to f16.  Pooled row = 8 band + wave.
// relu(BN(x)) of 4 channels into the next conv's padded image T (to_padded_h's arithmetic: v_fma_mix_f32 on the f16
// value, rounded, ReLU on f16); sc / sh: the BN table row
template <int C, int HO>
__device__ __forceinline__ void t_store_h3(_Float16* T, h4 x, int pr, int px, int ch, const float* sc, const float* sh) {
  const h2 lo = lo2(x), hi = hi2(x);
  const h4 t = to_h4(fma_mix_lo(lo, sc[ch], sh[ch]), fma_mix_hi(lo, sc[ch + 1], sh[ch + 1]), fma_mix_lo(hi, sc[ch + 2], sh[ch + 2]),
                     fma_mix_hi(hi, sc[ch + 3], sh[ch + 3]));
  *reinterpret_cast<h4*>(T + tidx<C>((pr + 1) * (HO + 2) + px + 1, ch)) = relu_h4(t);
}

// Exchange-slot entry (halves) of 4 channels ch .. ch + 3 of pooled pixel p (PX pooled pixels per row): channel-group-
// major, so a 16-lane group's b64 stores (one channel group, 16 consecutive pixels) are contiguous; with 32 pixels the
// odd groups flip pixel bit 4, so the b64 reads' 32-lane groups (channel groups 2j, 2j + 1) use disjoint banks
// (tools/lds_model/h3_model.py: pixel-major slots were 4-way on the stores).
template <int PX>
__device__ __forceinline__ int ex_idx(int p, int ch) {
  const int cg = ch >> 2;
  return (cg * PX + (PX >= 32 ? p ^ ((cg & 1) << 4) : p)) * 4;
}

// T: also write relu(BN(pooled)) into the next conv's padded image (sc / sh: its BN row), or nullptr
template <int COUT, int H, bool EO, int NV>
__device__ __forceinline__ void band_out_h3(const h4 (&P)[NV], const h4 (&Bx)[NV], h4 (&prev)[NV], _Float16* X,
                                            _Float16* EX, int band, int wave, int lane, _Float16* T = nullptr,
                                            const float* sc = nullptr, const float* sh = nullptr) {
  constexpr int SLOT = (H / 2) * COUT, NT = COUT / 16;
  const int g = lane >> 4, l = lane & 15;
  const bool st_lane = EO || (l & 1) == 0;
  // v = (k, nt): pooled pixel p(k) = EO ? 16 k + l : 8 k + l / 2, channels nt * 16 + 4 g
  auto pix = [&](int v) { return EO ? 16 * (v / NT) + l : 8 * (v / NT) + (l >> 1); };
  auto chn = [&](int v) { return (v % NT) * 16 + 4 * g; };
  _Float16* ex = EX + ((band & 1) * 8 + wave) * SLOT;
  if (st_lane) {
#pragma unroll
    for (int v = 0; v < NV; ++v) *reinterpret_cast<h4*>(ex + ex_idx<H / 2>(pix(v), chn(v))) = Bx[v];
  }
  __syncthreads();
  h4 o[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) o[v] = P[v];
  if (wave > 0) {
    const _Float16* ei = EX + ((band & 1) * 8 + wave - 1) * SLOT;
#pragma unroll
    for (int v = 0; v < NV; ++v) o[v] = __builtin_elementwise_max(o[v], *reinterpret_cast<const h4*>(ei + ex_idx<H / 2>(pix(v), chn(v))));
  } else if (band > 0) {
#pragma unroll
    for (int v = 0; v < NV; ++v) o[v] = __builtin_elementwise_max(o[v], prev[v]);
  }
  if (st_lane) {
    const int m0 = (8 * band + wave) * (H / 2);
#pragma unroll
    for (int v = 0; v < NV; ++v) *reinterpret_cast<h4*>(X + xidx<COUT>(m0 + pix(v), chn(v))) = o[v];
    if (T) {
#pragma unroll
      for (int v = 0; v < NV; ++v) t_store_h3<COUT, H / 2>(T, o[v], 8 * band + wave, pix(v), chn(v), sc, sh);
    }
  }
}

// wave 0, band > 0: the previous band's wave-7 slot (row 15), read before this band's barrier -- wave 7 rewrites that
// slot two bands later, after this band's barrier
template <int COUT, int H, bool EO, int NV>
__device__ __forceinline__ void band_prev_h3(h4 (&prev)[NV], const _Float16* EX, int band, int wave, int lane) {
  constexpr int SLOT = (H / 2) * COUT, NT = COUT / 16;
  if (wave != 0 || band == 0) return;
  const int g = lane >> 4, l = lane & 15;
  const _Float16* ei = EX + (((band - 1) & 1) * 8 + 7) * SLOT;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const int p = EO ? 16 * (v / NT) + l : 8 * (v / NT) + (l >> 1);
    prev[v] = *reinterpret_cast<const h4*>(ei + ex_idx<H / 2>(p, (v % NT) * 16 + 4 * g));
  }
}

// Stage-1 pool of a band (even / odd tiles, 16 channels): P, Bx per pooled tile k (2 per row)
__device__ __forceinline__ void pool_s1(const f32x4 (&acc)[8], const float (&bz)[1][4], h4 (&P)[2], h4 (&Bx)[2]) {
  float hp[2][2][4];  // [rho][k][channel]
#pragma unroll
  for (int rho = 0; rho < 2; ++rho)
#pragma unroll
    for (int k = 0; k < 2; ++k)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float e = acc[rho * 4 + k * 2][j], o = acc[rho * 4 + k * 2 + 1][j];
        const float l0 = k == 0 ? e : dpp_f<kDppRor1>(e, acc[rho * 4 + (k - 1) * 2 + 1][j]);  // lane 0: column 32 k - 1
        hp[rho][k][j] = fmaxf(fmaxf(e, o), dpp_f<kDppShr1>(l0, o));
      }
#pragma unroll
  for (int k = 0; k < 2; ++k) {
    P[k] = to_h4(fmaxf(hp[0][k][0], hp[1][k][0]) + bz[0][0], fmaxf(hp[0][k][1], hp[1][k][1]) + bz[0][1],
                 fmaxf(hp[0][k][2], hp[1][k][2]) + bz[0][2], fmaxf(hp[0][k][3], hp[1][k][3]) + bz[0][3]);
    Bx[k] = to_h4(hp[1][k][0] + bz[0][0], hp[1][k][1] + bz[0][1], hp[1][k][2] + bz[0][2], hp[1][k][3] + bz[0][3]);
  }
}

// Stage-2 / 3 pool of a band (natural tiles, 32 channels): v = (k, nt)
template <int H>
__device__ __forceinline__ void pool_nat(const f32x4 (&acc)[2 * (H / 16)][2], const float (&bz)[2][4],
                                         h4 (&P)[2 * (H / 16)], h4 (&Bx)[2 * (H / 16)]) {
  constexpr int TR = H / 16;
#pragma unroll
  for (int k = 0; k < TR; ++k)
#pragma unroll
    for (int nt = 0; nt < 2; ++nt) {
      float pv[4], bv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float h0 = hpool_nat(acc[k][nt][j], acc[k > 0 ? k - 1 : 0][nt][j], k == 0);
        const float h1 = hpool_nat(acc[TR + k][nt][j], acc[TR + (k > 0 ? k - 1 : 0)][nt][j], k == 0);
        pv[j] = fmaxf(h0, h1) + bz[nt][j];
        bv[j] = h1 + bz[nt][j];
      }
      P[k * 2 + nt] = to_h4(pv[0], pv[1], pv[2], pv[3]);
      Bx[k * 2 + nt] = to_h4(bv[0], bv[1], bv[2], bv[3]);
    }
}

// Two residual blocks, single-buffered (conv -> accumulators -> barrier -> in-place epilogue); the arithmetic
// of res_blocks_h.  af holds block 0's conv0 on entry and st the issued copy of its conv1.  WB protocol: a
// commit only after a barrier that follows every wave's fragment load of the previous block.  On exit T holds
// the next stage's input (or the features are written, LAST), and st holds the issued next-stage block (NEXTH
// halves; committed by the caller, whose WB may differ).
template <int NTH, int C, int H, int LAST, int NEXTH>
__device__ __forceinline__ void res_blocks_h2(_Float16* T, _Float16* X, h8 (&af)[KSteps<C>::N][C / 16],
                                              const _Float16* __restrict__ hp, const Layout& L, int stage,
                                              const float* bsc, const float* bsh, const float* bcb, int wave, int lane,
                                              float* __restrict__ out, WStageT<NTH>& st, _Float16* wb,
                                              const _Float16* __restrict__ next_w, const StepArgs& a, int stamp) {
  constexpr int CS = Pix<C>::CS, WP = H + 2, NTA = C / 16, MT = H * H / 16, NWA = NTH / 64;
  constexpr bool ST = NTH >= 512 && C == 32;  // A fragments streamed from wb (conv_h2 STREAM); af unused
  constexpr bool R32 = NTH >= 512 && C == 16;  // tap 8 as a chained K = 32 MFMA (conv_h2 R32)
  // SPLIT (8 x 8 stage at 8 waves: 4 pixel tiles x 2 channel tiles): wave = (pixel tile w % 4, channel tile w / 4), so
  // every wave runs one MFMA per K-step and streams only its own channel tile's A fragments (without it waves 4-7
  // had no tile but still read both channel tiles' fragments)
  constexpr int SPLIT = ST && MT * NTA == NWA ? NTA : 1;
  static_assert(SPLIT == 1 || (MT == 4 && NTA == 2), "split map");
  constexpr int NT = NTA / SPLIT, NW = NWA / SPLIT;
  const int nt0 = SPLIT > 1 ? (wave / NW) * NT : 0;
  wave = SPLIT > 1 ? wave % NW : wave;
  constexpr int TPW = (MT + NW - 1) / NW, WH = kBlockHalves<C, C / 16>;
  // conv_h2's fragment argument (unread in the streamed form, which every SPLIT > 1 instance is)
  auto& afw = reinterpret_cast<h8 (&)[KSteps<C>::N][NT]>(af);
  // Epilogue addresses: tile i's pixels are tile 0's + 16 NW i (X, S: the chunk swizzle is unchanged by that
  // step) and padded pixel + DQ i (T: the swizzle flips by tflip(i), conv_h2's step) -- per-lane bases + immediates.
  constexpr int DQ = H >= 16 ? (NW / (H / 16)) * WP : NW * (16 / H) * WP;
  static_assert((C == 16 && DQ % 4 == 0 && (16 * NW) % 16 == 0) || (C == 32 && DQ % 8 == 0 && (16 * NW) % 16 == 0),
                "epilogue address steps");
  auto tflip = [](int i) { return C == 16 ? ((DQ * i) >> 2) & 1 : 0; };
  const int cl = 4 * (lane >> 4), m0 = wave * 16 + (lane & 15), q0 = (m0 / H + 1) * WP + (m0 % H) + 1;
  int xb[NT], tb[NT][2];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) {
    const int ch0 = (nt0 + nt) * 16 + cl;
    xb[nt] = xidx<C>(m0, ch0);
    tb[nt][0] = tidx<C>(q0, ch0);
    tb[nt][1] = q0 * CS + ((((ch0 >> 3) ^ tsw<C>(q0)) ^ 1) << 3) + (ch0 & 7);
  }
  // f(i, nt, x offset, T offset, m, v) over this wave's live tiles
  auto epilogue = [&](const f32x4 (&acc)[TPW][NT], auto&& f) {
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      if (!(TPW * NW == MT || wave + NW * i < MT)) continue;  // wave-uniform
#pragma unroll
      for (int nt = 0; nt < NT; ++nt)
        f(nt, xb[nt] + 16 * NW * i * C, tb[nt][tflip(i)] + DQ * i * CS, m0 + 16 * NW * i, acc[i][nt]);
    }
  };
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int i0 = stage * 5 + 1 + 2 * r, i1 = i0 + 1;
    const int inext = r == 0 ? i1 + 1 : (stage + 1) * 5;
    // epilogue constants are read from the tables after each conv's barrier (not held across the MFMA loop:
    // 4 waves carry twice conv_kernel_h's tiles per wave, and the registers go to accumulators)
    float b0[NT][4], s1[NT][4], t1[NT][4], b1[NT][4], s2[NT][4], t2[NT][4];
    f32x4 acc[TPW][NT];
    // ---- conv0: T -> T (relu(bn1(. + b0))) ----
    conv_h2<C, CS, NT, TPW, H, WP, MT, NW, ST, NTA, R32>(T, afw, acc, wave, lane, 0, wb, nt0);
    __syncthreads();  // every wave has read T
    FDR_STAMP(a, stamp + 4 * r);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ch = (nt0 + nt) * 16 + cl + k;
        b0[nt][k] = bcb[i0 * 32 + ch];
        s1[nt][k] = bsc[i1 * 32 + ch];
        t1[nt][k] = bsh[i1 * 32 + ch];
      }
    epilogue(acc, [&](int nt, int, int to, int, f32x4 v) {
      float o[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) o[k] = fmaf(v[k] + b0[nt][k], s1[nt][k], t1[nt][k]);
      *reinterpret_cast<h4*>(T + to) = relu_h4(to_h4(o[0], o[1], o[2], o[3]));
    });
    st.template commit<WH>(wb);  // conv i1 (every wave loaded conv i0's fragments before the barrier above)
    __syncthreads();
    FDR_STAMP(a, stamp + 4 * r + 1);
    if constexpr (!ST) load_af_lds<C, NT, R32>(wb, af, lane);
    if (r == 0) {
      st.template issue<WH>(hp + L.conv_h[i1 + 1]);  // block 1 conv0 (committed after the next barrier)
    } else if constexpr (NEXTH > 0) {
      st.template issue<NEXTH>(next_w);
    }
    // ---- conv1: T -> X += . + b1; T <- bn(X) (relu before a block) ----
    conv_h2<C, CS, NT, TPW, H, WP, MT, NW, ST, NTA, R32>(T, afw, acc, wave, lane, 0, wb, nt0);
    __syncthreads();
    FDR_STAMP(a, stamp + 4 * r + 2);
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int ch = (nt0 + nt) * 16 + cl + k;
        b1[nt][k] = bcb[i1 * 32 + ch];
        s2[nt][k] = (r == 1 && LAST) ? 0.f : bsc[inext * 32 + ch];
        t2[nt][k] = (r == 1 && LAST) ? 0.f : bsh[inext * 32 + ch];
      }
    epilogue(acc, [&](int nt, int xo_, int to, int m, f32x4 v) {
      const h4 xo = *reinterpret_cast<const h4*>(X + xo_);
      // x' = f16((v + b1) + x) and the next BN of x' on v_fma_mix_f32 (x * 1 + s is the f32 add, exact)
      const h2 xl = lo2(xo), xh = hi2(xo);
      const h4 xn = to_h4(fma_mix_lo(xl, 1.f, v[0] + b1[nt][0]), fma_mix_hi(xl, 1.f, v[1] + b1[nt][1]),
                          fma_mix_lo(xh, 1.f, v[2] + b1[nt][2]), fma_mix_hi(xh, 1.f, v[3] + b1[nt][3]));
      if (r == 1 && LAST) {
#pragma unroll
        for (int k = 0; k < 4; ++k) out[((nt0 + nt) * 16 + cl + k) * H * H + m] = relu((float)xn[k]);  // flatten (C,H,W)
      } else {
        if (r == 0) *reinterpret_cast<h4*>(X + xo_) = xn;
        const h2 nl = lo2(xn), nh = hi2(xn);
        const h4 t = to_h4(fma_mix_lo(nl, s2[nt][0], t2[nt][0]), fma_mix_hi(nl, s2[nt][1], t2[nt][1]),
                           fma_mix_lo(nh, s2[nt][2], t2[nt][2]), fma_mix_hi(nh, s2[nt][3], t2[nt][3]));
        *reinterpret_cast<h4*>(T + to) = r == 0 ? relu_h4(t) : t;
      }
    });
    if (r == 0) st.template commit<WH>(wb);  // block 1 conv0 (af of conv1 loaded before the barrier above)
    __syncthreads();
    FDR_STAMP(a, stamp + 4 * r + 3);
    if (r == 0) {
      if constexpr (!ST) load_af_lds<C, NT, R32>(wb, af, lane);
      st.template issue<WH>(hp + L.conv_h[i1 + 2]);  // block 1 conv1 (committed after the next barrier)
    }
  }
}

#ifdef FDR_H3_FINE  // diagnostics build: clocks inside the h3 entry bands (dbg[64..])
#define FDR_FINE_STAMP(a, k) FDR_STAMP(a, k)
#else
#define FDR_FINE_STAMP(a, k) \
  do {                       \
  } while (0)
#endif
// The conv stack after the BN / bias tables' inputs are in hand: frame band 0, the tables into LDS (store_tables), the
// first barrier, the three stages.  Shared by both table sources of conv_kernel_h2.
template <int NTH, class StoreTables>
__device__ __forceinline__ void conv_body_h2(const Layout& L, const StepArgs& a, int lane, int e, int64_t env, int wave,
                                             int ln, const _Float16* hp, unsigned char* smem, FrameBn fbn,
                                             const h8 (&af3n)[2], WStageT<NTH>& st, StoreTables&& store_tables) {
  float* bsc = reinterpret_cast<float*>(smem);
  float* bsh = bsc + kBnTab;
  float* bcb = bsh + kBnTab;  // conv biases [15][32]
  _Float16* R = reinterpret_cast<_Float16*>(smem + 3 * kBnTab * 4);  // the tables double as row -1's guard
  (void)lane;
  auto FB3 = [&](int k) { return R + ((k & 1) ? kH3FB1 : kH3FB0); };
  frame_band_h2<NTH, kH3FR>(FB3(0), nullptr, 0, 0, a, env, e, fbn);
  if (threadIdx.x < 2)  // the frame buffers' pad pixels (conv_band_s1)
    *reinterpret_cast<h4*>(R + (threadIdx.x ? kH3FB1 : kH3FB0) + kH3FB) = h4{0, 0, 0, 0};
  store_tables();
  __syncthreads();
  FDR_STAMP(a, 1);

  // ---- stage 1: entry (3 -> 16 at 64 x 64, pooled to 32 x 32) in 4 bands of 16 rows, pool in registers ----
  {
    for (int bd = 0; bd < 4; ++bd) {
      h4 prev[2], P[2], Bx[2];
      f32x4 acc[8];
      conv_band_s1(FB3(bd), af3n, acc, wave, ln);
      FDR_FINE_STAMP(a, 64 + 4 * bd);
      if (bd + 1 < 4) frame_band_h2<NTH, kH3FR>(FB3(bd + 1), FB3(bd), 2, 16 * (bd + 1), a, env, e, fbn);
      FDR_FINE_STAMP(a, 65 + 4 * bd);
      float bz[1][4];  // (from the LDS table here, not held across the conv)
#pragma unroll
      for (int k = 0; k < 4; ++k) bz[0][k] = bcb[0 * 32 + 4 * (ln >> 4) + k];
      pool_s1(acc, bz, P, Bx);
      FDR_FINE_STAMP(a, 66 + 4 * bd);
      band_prev_h3<16, 64, true>(prev, R + kH3EX1, bd, wave, ln);
      if (bd == 0) st.template commit<kBlockHalves<16, 1>>(R + kH2WBA);
      band_out_h3<16, 64, true>(P, Bx, prev, R + kH2X1, R + kH3EX1, bd, wave, ln);
      FDR_STAMP(a, 2 + bd);
    }
    __syncthreads();
    FDR_STAMP(a, 6);
  }
  // ---- stage 1 residual blocks (16 ch, 32 x 32) ----
  {
    h8 af[KSteps<16>::N][1];
    load_af_lds<16, 1, true>(R + kH2WBA, af, ln);
    st.template issue<kBlockHalves<16, 1>>(hp + L.conv_h[2]);
    to_padded_h<16, 32, true, true, NTH>(R + kH2X1, R, bsc + 1 * 32, bsh + 1 * 32);
    __syncthreads();
    FDR_STAMP(a, 18);
    res_blocks_h2<NTH, 16, 32, 0, kBlockHalves<16, 2>>(R, R + kH2X1, af, hp, L, 0, bsc, bsh, bcb, wave, ln, nullptr, st,
                                                  R + kH2WBA, hp + L.conv_h[5], a, 19);
    st.template commit<kBlockHalves<16, 2>>(R + kH2WBB);  // X1 is dead: the stage-2 entry block goes to WB_B
    __syncthreads();
  }
  // ---- stage 2: entry (16 -> 32 at 32 x 32, pooled to 16 x 16) in 2 bands of 16 rows, pool in registers; X2 into
  // T1's consumed rows (band 1 reads padded rows 16..33, past X2's first half) ----
  {
    // conv 6's weight block is requested after band 1's conv, once the accumulators are pooled (r10: issued before
    // the two bands, its 9 staging VGPRs lived across both bands' convs -- one 16-B chunk spilled, the kernel's only
    // scratch traffic, 33.5 MB written + read per launch)
    for (int bd = 0; bd < 2; ++bd) {
      h4 prev[4], P[4], Bx[4];
      f32x4 acc[4][2];
      conv_band_nat<16, 32>(R, 16 * bd, R + kH2WBB, acc, wave, ln);
      FDR_FINE_STAMP(a, 80 + 4 * bd);
      float bz[2][4];
#pragma unroll
      for (int nt = 0; nt < 2; ++nt)
#pragma unroll
        for (int k = 0; k < 4; ++k) bz[nt][k] = bcb[5 * 32 + nt * 16 + 4 * (ln >> 4) + k];
      pool_nat<32>(acc, bz, P, Bx);
      if (bd == 1) st.template issue<kBlockHalves<32, 2>>(hp + L.conv_h[6]);
      FDR_FINE_STAMP(a, 81 + 4 * bd);
      band_prev_h3<32, 32, false>(prev, R + kH3EX2, bd, wave, ln);
      // (barrier inside).  Band 1 also writes T2 = relu(BN(X2)) of its rows: T2 lies over T1's rows 15.., which band
      // 1's conv read before that barrier
      band_out_h3<32, 32, false>(P, Bx, prev, R, R + kH3EX2, bd, wave, ln, bd == 1 ? R + kH2T2 : nullptr,
                                 bsc + 6 * 32, bsh + 6 * 32);
      if (bd == 1) st.template commit<kBlockHalves<32, 2>>(R + kH2WBB);   // every wave is past conv 5's reads
      FDR_STAMP(a, 28 + bd);
    }
    // band 0's rows of T2 from the wave's own X2 row (its own stores: no barrier), and T2's zero border
    if ((ln & 1) == 0) {
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int px = 8 * (v >> 1) + ((ln & 15) >> 1), ch = (v & 1) * 16 + 4 * (ln >> 4);
        t_store_h3<32, 16>(R + kH2T2, *reinterpret_cast<const h4*>(R + xidx<32>(wave * 16 + px, ch)), wave, px, ch,
                           bsc + 6 * 32, bsh + 6 * 32);
      }
    }
    zero_border_h<32, 16>(R + kH2T2);
    __syncthreads();  // X2, T2 complete
    FDR_STAMP(a, 30);
  }
  // ---- stage 2 residual blocks (32 ch, 16 x 16) ----
  {
    h8 af[KSteps<32>::N][2];  // (unread: the 32-channel convs stream their A fragments from WB)
    st.template issue<kBlockHalves<32, 2>>(hp + L.conv_h[7]);
    res_blocks_h2<NTH, 32, 16, 0, kBlockHalves<32, 2>>(R + kH2T2, R, af, hp, L, 1, bsc, bsh, bcb, wave, ln, nullptr, st,
                                                  R + kH2WBB, hp + L.conv_h[10], a, 37);
    st.template commit<kBlockHalves<32, 2>>(R + kH2WBB);
    __syncthreads();
  }
  // ---- stage 3: entry (32 -> 32 at 16 x 16, pooled to 8 x 8): one band of 16 rows, pool in registers ----
  {
    st.template issue<kBlockHalves<32, 2>>(hp + L.conv_h[11]);
    h4 prev[2], P[2], Bx[2];
    f32x4 acc[2][2];
    conv_band_nat<32, 16>(R + kH2T2, 0, R + kH2WBB, acc, wave, ln);
    float bz[2][4];
#pragma unroll
    for (int nt = 0; nt < 2; ++nt)
#pragma unroll
      for (int k = 0; k < 4; ++k) bz[nt][k] = bcb[10 * 32 + nt * 16 + 4 * (ln >> 4) + k];
    pool_nat<16>(acc, bz, P, Bx);
    band_out_h3<32, 16, false>(P, Bx, prev, R, R + kH3EX3, 0, wave, ln, R + kH2T3, bsc + 11 * 32, bsh + 11 * 32);
    zero_border_h<32, 8>(R + kH2T3);
    st.template commit<kBlockHalves<32, 2>>(R + kH2WBB);
    FDR_STAMP(a, 45);
    __syncthreads();  // X3, T3 complete
    FDR_STAMP(a, 46);
  }
  // ---- stage 3 residual blocks (32 ch, 8 x 8) -> features ----
  {
    h8 af[KSteps<32>::N][2];
    st.template issue<kBlockHalves<32, 2>>(hp + L.conv_h[12]);
    res_blocks_h2<NTH, 32, 8, 1, 0>(R + kH2T3, R, af, hp, L, 2, bsc, bsh, bcb, wave, ln, a.feat + env * kFeat, st,
                               R + kH2WBB, nullptr, a, 50);
  }
}

template <int NTH>
__global__ __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(NTH / 128))) void conv_kernel_h2(Layout L, StepArgs a) {
  static_assert(NTH == kHThreads, "8 waves (zero_border_h's thread count; the h3 entries' band rows)");
  __shared__ __attribute__((aligned(16))) unsigned char smem[kH2LdsBytes];
  const int b = blockIdx.x, xcd = b & 7, slot = b >> 3;
  const int lane = (slot / a.envs) * 8 + xcd, e = slot % a.envs;
  if (lane >= a.n_lanes) return;
  FDR_STAMP(a, 0);
#ifdef FDR_WG_TIMELINE  // diagnostics build: every workgroup's start / end (s_memrealtime, 100 MHz) and HW_ID / XCC_ID
  if (a.dbg && threadIdx.x == 0) {
    a.dbg[256 + 4 * b] = wall_clock64();
    a.dbg[256 + 4 * b + 2] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 4);
    a.dbg[256 + 4 * b + 3] = (uint64_t)__builtin_amdgcn_s_getreg((31 << 11) | 20);
  }
#endif
  // wave index in an SGPR: every wave-uniform tile / address term derived from it stays scalar (VGPR pressure)
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), ln = threadIdx.x & 63;
  const int64_t env = (int64_t)lane * a.envs + e;
  const float* pk = a.pack + (int64_t)lane * a.pack_stride;
  const _Float16* hp = a.hpack + (int64_t)lane * a.hpack_stride;
  float* bsc = reinterpret_cast<float*>(smem);
  float* bsh = bsc + kBnTab;
  float* bcb = bsh + kBnTab;  // conv biases [15][32]

  // BN / bias tables: with a.bntab (the rollout) the lane's tables were folded once per rollout by bn_table_kernel
  // and are copied here (one 16-B load per thread, L2-resident: the lane's E envs read the same 5.6 KB); otherwise
  // folded here, two entries per thread: their inputs are loaded first, the first frame band (which folds BN2d(3)
  // per thread from the same inputs) covers the latency, then the tables are written.  The weight block of the
  // first residual conv is issued now and committed in the first pool phase.
  if (a.bntab) {
    constexpr int kQ = 3 * kBnTab / 4;  // float4s of the three tables
    static_assert(kQ <= NTH, "one float4 per thread");
    const float4* src = reinterpret_cast<const float4*>(a.bntab + (int64_t)lane * 3 * kBnTab);
    const float4 v = src[min((int)threadIdx.x, kQ - 1)];
    const float f0 = a.bntab[(int64_t)lane * 3 * kBnTab + 0], f1 = a.bntab[(int64_t)lane * 3 * kBnTab + 1],
                f2 = a.bntab[(int64_t)lane * 3 * kBnTab + 2];
    const float g0 = a.bntab[(int64_t)lane * 3 * kBnTab + kBnTab], g1 = a.bntab[(int64_t)lane * 3 * kBnTab + kBnTab + 1],
                g2 = a.bntab[(int64_t)lane * 3 * kBnTab + kBnTab + 2];
    h8 af3n[2];
    s1_frag(hp + L.conv_h[0], af3n, ln);
    WStageT<NTH> st;
    st.template issue<kBlockHalves<16, 1>>(hp + L.conv_h[1]);
    conv_body_h2<NTH>(L, a, lane, e, env, wave, ln, hp, smem, FrameBn{f0, f1, f2, g0, g1, g2}, af3n, st, [&]() {
      if ((int)threadIdx.x < kQ) reinterpret_cast<float4*>(bsc)[threadIdx.x] = v;
    });
    return;
  }
  constexpr int kTabIt = (kBnTab + NTH - 1) / NTH;
  float rm[kTabIt], rv[kTabIt], bnw[kTabIt], bnb[kTabIt], cbv[kTabIt];
  // Branch-free (r11): every load unconditional from an in-bounds address, the unused values selected away after.
  // A conditional load ends its basic block with s_waitcnt vmcnt(0), and the layout offsets were read per lane from
  // the kernel argument block -- together 4-5 serialised global round trips in this phase (r11 probe of the same
  // table in conv_s3_kernel: 3.3-3.9 K clocks); the offsets are now scalar loads (the wave's two table rows).
  {
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hi = (threadIdx.x >> 5) & 1;
    const float* bmp = a.bn_mean ? a.bn_mean : pk;  // a valid address either way
    const float* bvp = a.bn_var ? a.bn_var : pk;
#pragma unroll
    for (int k = 0; k < kTabIt; ++k) {
      const int bi = threadIdx.x + k * NTH, bidx = bi >> 5, bch = bi & 31;
      const int r0 = min((wv * 64 + k * NTH) >> 5, kConvs - 1), r1 = min(r0 + 1, kConvs - 1);  // wave-uniform rows
      auto pick = [&](const int32_t* arr) { return hi ? arr[r1] : arr[r0]; };
      const bool has_bn = bi < kBnTab && bch < (bidx == 0 ? 3 : (bidx == 5 ? 16 : (bidx < 5 ? 16 : 32)));
      const bool has_cb = bi < kBnTab && bch < (bidx < 5 ? 16 : 32);
      const int so = pick(L.bn_stat) + bch;
      const float m_ = bmp[so], v_ = bvp[so], w_ = pk[pick(L.bn_w) + bch], b_ = pk[pick(L.bn_b) + bch],
                  c_ = pk[pick(L.conv_b) + bch];
      rm[k] = has_bn && a.bn_mean ? m_ : 0.f;
      rv[k] = has_bn && a.bn_var ? v_ : 1.f;
      bnw[k] = has_bn ? w_ : 0.f;
      bnb[k] = has_bn ? b_ : 0.f;
      cbv[k] = has_cb ? c_ : 0.f;
    }
  }
  h8 af3n[2];  // conv_band_s1's K order
  s1_frag(hp + L.conv_h[0], af3n, ln);
  WStageT<NTH> st;
  st.template issue<kBlockHalves<16, 1>>(hp + L.conv_h[1]);
  float fsc[3], fsh[3];  // BN2d(3) of the frame, per thread (table entries 0..2)
#pragma unroll
  for (int c = 0; c < 3; ++c) {
    const float m_ = (a.bn_mean ? a.bn_mean : pk)[L.bn_stat[0] + c], v_ = (a.bn_var ? a.bn_var : pk)[L.bn_stat[0] + c];
    const float m = a.bn_mean ? m_ : 0.f, v = a.bn_var ? v_ : 1.f;
    fsc[c] = pk[L.bn_w[0] + c] * (1.f / sqrtf(v + kBnEps));
    fsh[c] = pk[L.bn_b[0] + c] - m * fsc[c];
  }
  const FrameBn fbn{fsc[0], fsc[1], fsc[2], fsh[0], fsh[1], fsh[2]};
  conv_body_h2<NTH>(L, a, lane, e, env, wave, ln, hp, smem, fbn, af3n, st, [&]() {
#pragma unroll
    for (int k = 0; k < kTabIt; ++k) {
      const int bi = threadIdx.x + k * NTH, bidx = bi >> 5, bch = bi & 31;
      if (bi >= kBnTab) break;
      const bool has_bn = bch < (bidx == 0 ? 3 : (bidx == 5 ? 16 : (bidx < 5 ? 16 : 32)));
      const float sc = has_bn ? bnw[k] * (1.f / sqrtf(rv[k] + kBnEps)) : 0.f;
      bsc[bi] = sc;
      bsh[bi] = has_bn ? bnb[k] - rm[k] * sc : 0.f;
      bcb[bi] = cbv[k];
    }
  });
#ifdef FDR_WG_TIMELINE
  __syncthreads();
  if (a.dbg && threadIdx.x == 0) a.dbg[256 + 4 * b + 1] = wall_clock64();
#endif
}
template __global__ void conv_kernel_h2<kHThreads>(Layout, StepArgs);

// The folded BN / bias tables of each lane (conv_kernel_h2's in-kernel folding, the same formulas): theta' and the
// running statistics are constant over a rollout, so they are folded once here instead of by every conv workgroup
// of every step.  tab [lane][scale kBnTab | shift kBnTab | conv bias kBnTab], row = conv index, 32 channels a row.
__global__ __launch_bounds__(256) void bn_table_kernel(Layout L, StepArgs a, float* tab) {
  const int lane = blockIdx.x;
  const float* pk = a.pack + (int64_t)lane * a.pack_stride;
  float* t = tab + (int64_t)lane * 3 * kBnTab;
  for (int bi = threadIdx.x; bi < kBnTab; bi += blockDim.x) {
    const int bidx = bi >> 5, bch = bi & 31;
    const bool has_bn = bch < (bidx == 0 ? 3 : (bidx == 5 ? 16 : (bidx < 5 ? 16 : 32)));
    const bool has_cb = bch < (bidx < 5 ? 16 : 32);
    const float rm = has_bn && a.bn_mean ? a.bn_mean[L.bn_stat[bidx] + bch] : 0.f;
    const float rv = has_bn && a.bn_var ? a.bn_var[L.bn_stat[bidx] + bch] : 1.f;
    const float bnw = has_bn ? pk[L.bn_w[bidx] + bch] : 0.f, bnb = has_bn ? pk[L.bn_b[bidx] + bch] : 0.f;
    const float sc = has_bn ? bnw * (1.f / sqrtf(rv + kBnEps)) : 0.f;
    t[bi] = sc;
    t[kBnTab + bi] = has_bn ? bnb - rm * sc : 0.f;
    t[2 * kBnTab + bi] = has_cb ? pk[L.conv_b[bidx] + bch] : 0.f;
  }
}

// ---- core (fc + LSTM + head) with f16 weights ------------------------------------------------------
template <int E, int MODE>
__global__ __launch_bounds__(kCoreThreads) __attribute__((amdgpu_waves_per_eu(E <= 4 ? 4 : 1))) void core_kernel_h(
    Layout L, StepArgs a) {  // E <= 4: <= 128 VGPRs -> 4 lanes per CU (the LDS allows 4)
  // xw: xs [2048][E] -> fc partials [8][256][E] -> gates [x|h][1024][E], phases separated by
  // barriers.  The core input lives in xw's second half between the fc and the gate writes, the
  // logits at xw's start after the gates are consumed: 36 KiB per workgroup -> 4 lanes per CU, so
  // 1024 lanes run in one round (at 41 KiB only 3 fit).
  __shared__ float xw[kFeat * E];
  __shared__ float hs[kHid * E];
  float* cis = xw + kFeat * E / 2;
  float* logit = xw;
  static_assert(kCoreIn * E <= kFeat * E / 2 && E * kMaxAct <= kFeat * E, "core LDS aliasing");
  const int lane = blockIdx.x, j = threadIdx.x;
  const float* pk = a.pack + (int64_t)lane * a.pack_stride;
  const _Float16* hp = a.hpack + (int64_t)lane * a.hpack_stride;
  const int64_t e0 = (int64_t)lane * E;
  const int A = a.n_act;

  if constexpr (!seq_mode(MODE)) {
    for (int k = j; k < kFeat; k += kCoreThreads) {
      const float rm = a.bn_mean ? a.bn_mean[L.bn_stat[15] + k] : 0.f;
      const float rv = a.bn_var ? a.bn_var[L.bn_stat[15] + k] : 1.f;
      const float sc = pk[L.bn_w[15] + k] * (1.f / sqrtf(rv + kBnEps));
      const float sh = fmaf(-rm, sc, pk[L.bn_b[15] + k]);
#pragma unroll
      for (int e = 0; e < E; ++e) xw[k * E + e] = fmaf(a.feat[(e0 + e) * kFeat + k], sc, sh);
    }
    __syncthreads();
    // fc: thread = (8 columns, one of 8 K-slices of 256 rows); f16 W^T rows, 16 B per lane
    const int c8 = j & 31, ks = j >> 5;
    float acc[8][E];
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) acc[c][e] = 0.f;
    const h8* w8 = reinterpret_cast<const h8*>(hp + L.fc_wt_h) + c8;
#pragma unroll FDR_CORE_UNROLL_H
    for (int k = ks * 256; k < ks * 256 + 256; ++k) {
      const h8 w = ld_stream(w8 + (int64_t)k * (kHid / 8));
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float x = xw[k * E + e];
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c][e] = fmaf((float)w[c], x, acc[c][e]);
      }
    }
    __syncthreads();
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) xw[(ks * kHid + 8 * c8 + c) * E + e] = acc[c][e];
    __syncthreads();
    const float bj = pk[L.fc_b + j];
    float yv[E];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      float y = 0.f;
#pragma unroll
      for (int q = 0; q < 8; ++q) y += xw[(q * kHid + j) * E + e];
      yv[e] = relu(y + bj);
    }
    __syncthreads();  // every partial read before cis (inside xw) is written
#pragma unroll
    for (int e = 0; e < E; ++e) cis[j * E + e] = yv[e];
    if (j < E) {
      const float r = MODE == kForward ? (a.reward_in ? a.reward_in[e0 + j] : 0.f) : a.rprev[e0 + j];
      cis[kHid * E + j] = fminf(fmaxf(r, -1.f), 1.f);
    }
    if (MODE == kRollout && a.ci) {
      __syncthreads();
      float* dst = a.ci + ((int64_t)a.t * a.n_lanes * E + e0) * kCoreIn;
      for (int i = j; i < kCoreIn * E; i += kCoreThreads) {
        const int e = i / kCoreIn, k = i - e * kCoreIn;
        dst[i] = cis[k * E + e];
      }
    }
  } else if (!a.gx) {
    const float* src = a.ci + ((int64_t)a.t * a.n_lanes * E + e0) * kCoreIn;
    for (int i = j; i < kCoreIn * E; i += kCoreThreads) {
      const int e = i / kCoreIn, k = i - e * kCoreIn;
      cis[k * E + e] = src[i];
    }
  }
  float cj[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const float nd = (MODE == kForward && a.notdone) ? a.notdone[e0 + e] : 1.f;
    hs[j * E + e] = nd * a.h[(e0 + e) * kHid + j];
    cj[e] = nd * a.c[(e0 + e) * kHid + j];
  }
  __syncthreads();
  if (seq_mode(MODE) && a.gx) {
    // replay with x W_ih^T precomputed (lstm_xproj_kernel<true>): all 256 threads stream W_hh^T,
    // 4 columns each (the same per-column fma chain as below, twice the waves in flight)
    typedef _Float16 h4v __attribute__((ext_vector_type(4)));
    float acc[4][E];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) acc[c][e] = 0.f;
    const h4v* w4 = reinterpret_cast<const h4v*>(hp + L.lstm_wt_h) + j;
#pragma unroll FDR_CORE_UNROLL
    for (int k = 0; k < kHid; ++k) {
      const h4v w = ld_stream(w4 + (int64_t)(kCoreIn + k) * (kGates / 4));
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float x = hs[k * E + e];
#pragma unroll
        for (int c = 0; c < 4; ++c) acc[c][e] = fmaf((float)w[c], x, acc[c][e]);
      }
    }
    const float4* g4 = reinterpret_cast<const float4*>(a.gx + ((int64_t)(a.t - a.gx_t0) * a.n_lanes * E + e0) * kGates);
    float4 gv[E];
#pragma unroll
    for (int e = 0; e < E; ++e) gv[e] = ld_stream(g4 + (int64_t)e * (kGates / 4) + j);
    __syncthreads();  // every read of hs (inside xw) is done before the gates overwrite it
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float gx4[4] = {gv[e].x, gv[e].y, gv[e].z, gv[e].w};
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        xw[(4 * j + c) * E + e] = gx4[c];
        xw[(kGates + 4 * j + c) * E + e] = acc[c][e];
      }
    }
  } else {  // gates: threads 0..127 stream W_ih^T (x part), 128..255 W_hh^T (h part), 8 columns each
    const int cg = j & 127, part = j >> 7;
    float acc[8][E];
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) acc[c][e] = 0.f;
    const int k_lo = part ? kCoreIn : 0, k_n = part ? kHid : kCoreIn;
    const float* xin = part ? hs : cis;
    const h8* w8 = reinterpret_cast<const h8*>(hp + L.lstm_wt_h) + cg;
#pragma unroll FDR_CORE_UNROLL_H
    for (int k = 0; k < k_n; ++k) {
      const h8 w = ld_stream(w8 + (int64_t)(k_lo + k) * (kGates / 8));
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float x = xin[k * E + e];
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c][e] = fmaf((float)w[c], x, acc[c][e]);
      }
    }
    __syncthreads();  // every read of cis (inside xw) is done before the gates overwrite it
#pragma unroll
    for (int c = 0; c < 8; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) xw[(part * kGates + 8 * cg + c) * E + e] = acc[c][e];
  }
  __syncthreads();
  float hj[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    float pre[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int col = g * kHid + j;
      pre[g] = (xw[col * E + e] + pk[L.lstm_bih + col]) + (xw[(kGates + col) * E + e] + pk[L.lstm_bhh + col]);
    }
    const float gi = sigm(pre[0]), gf = sigm(pre[1]), gg = tanhf(pre[2]), go = sigm(pre[3]);
    cj[e] = fmaf(gf, cj[e], gi * gg);  // explicit: the same rounding in every core form
    hj[e] = go * tanhf(cj[e]);
    a.h[(e0 + e) * kHid + j] = hj[e];
    a.c[(e0 + e) * kHid + j] = cj[e];
  }
  {
    const float rm = a.bn_mean ? a.bn_mean[L.bn_stat[16] + j] : 0.f;
    const float rv = a.bn_var ? a.bn_var[L.bn_stat[16] + j] : 1.f;
    const float sc = pk[L.bn_w[16] + j] * (1.f / sqrtf(rv + kBnEps));
    const float sh = fmaf(-rm, sc, pk[L.bn_b[16] + j]);
#pragma unroll
    for (int e = 0; e < E; ++e) hs[j * E + e] = fmaf(hj[e], sc, sh);
  }
  __syncthreads();
  if (j < A * E) {  // head in f32 (A x 256, tiny)
    const int ai = j / E, e = j - ai * E;
    const float* w = pk + L.head_w + ai * kHid;
    float s = 0.f;
    for (int k = 0; k < kHid; ++k) s = fmaf(w[k], hs[k * E + e], s);
    logit[e * kMaxAct + ai] = s + pk[L.head_b + ai];
  }
  __syncthreads();
  if (j < E) core_finish<E, MODE>(a, logit, lane, j);
}

// ---- MFMA form of the fp16 pair core step (ctx core_mfma, the default) ---------------------------------------
// The pair's lanes share theta and sigma-eps E, so each GEMM of the step is  W_l x = theta x + s_l (E x):
// one v_mfma_f32_16x16x32_f16 of theta's A fragment against the B fragment X (the pair's 2E envs as columns,
// repeated to 16) and one of E's fragment against S X (the columns of the minus lane sign-flipped), chained
// into ONE f32 accumulator per 16-column tile.  The VALU form (core_kernel_hp) issues 96 VALU instructions per
// 32 streamed bytes and leaves the HBM stream latency-bound at 2 waves/SIMD; here the VALU work is gone and
// the weights stream through a 4-deep register ring (the images hold the A fragments in HBM order, 1 KB per
// wave-load).  Activations x, the fc output and h are rounded to f16 as the B operand (fp16 tolerance).

// MFMA images of n half packs: block (k-step, 256-column quarter) of W^T -> LDS -> fragments [ks][nt][l][8].
__global__ __launch_bounds__(256) void mfma_image_kernel(Layout L, const _Float16* src, int64_t src_stride,
                                                          _Float16* dst) {
  constexpr int TP = 256 + 8;  // LDS tile pitch (halves)
  __shared__ __attribute__((aligned(16))) _Float16 tile[32 * TP];
  const int b = blockIdx.x, t = threadIdx.x;
  const bool fc = b < kFcKS;
  const int ks = fc ? b : (b - kFcKS) >> 2, q = fc ? 0 : (b - kFcKS) & 3;
  const int ncol = fc ? kHid : kGates, nt_n = fc ? kFcNT : kGateNT, krows = fc ? kFeat : kGateK;
  const _Float16* s = src + (int64_t)blockIdx.y * src_stride + (fc ? L.fc_wt_h : L.lstm_wt_h);
  _Float16* d = dst + (int64_t)blockIdx.y * kMImg + (fc ? 0 : kFcImg);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = t + 256 * i, r = idx >> 5, cc = idx & 31, k = 32 * ks + r;
    h8 v = h8{0, 0, 0, 0, 0, 0, 0, 0};
    if (k < krows) v = *reinterpret_cast<const h8*>(s + (int64_t)k * ncol + 256 * q + 8 * cc);
    *reinterpret_cast<h8*>(tile + r * TP + 8 * cc) = v;
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int idx = t + 256 * i, nt = idx >> 6, l = idx & 63;
    h8 v;
#pragma unroll
    for (int jj = 0; jj < 8; ++jj) v[jj] = tile[(8 * (l >> 4) + jj) * TP + 16 * nt + (l & 15)];
    *reinterpret_cast<h8*>(d + (((int64_t)ks * nt_n + 16 * q + nt) * 64 + l) * 8) = v;
  }
}

// ---- Two pairs per workgroup (ctx core_mfma = 2, the default) ------------------------------------------------------
// theta's fragment of a k-step is the same for every pair, yet core_kernel_hpm loads it once per pair from L2 next to
// the pair's streamed E (the probe build without those loads ran the launch 16 % faster: 0.237 -> 0.199 ms at config
// 5).  Here a workgroup of 8 waves takes two pairs -- 4 lanes, their 4E envs as the B columns -- and issues per
// 16-column tile and k-step  theta x X,  E_0 x (S X masked to pair 0's columns),  E_1 x (S X masked to pair 1's):
// three MFMAs for two pairs where the one-pair form issues four, theta read once for both.  A masked column adds
// exact zeros, so every accumulator sees core_kernel_hpm's products in its order: the two forms agree bit for bit.
template <int NQ, class Frag>
struct MfmaRing2 {
  static constexpr int D = 4;
  static_assert(NQ % D == 0, "ring depth divides the step count");
  const _Float16* thm;
  const _Float16* ep0;
  const _Float16* ep1;
  Frag frag;
  h8 rt[D][2], ra[D][2], rb[D][2];
  __device__ __forceinline__ void issue(int q, h8 (&t)[2], h8 (&ea)[2], h8 (&eb)[2]) {
    const int64_t o = frag(q);
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) {
      t[jt] = *reinterpret_cast<const h8*>(thm + o + 512 * jt);
      ea[jt] = ld_stream(reinterpret_cast<const h8*>(ep0 + o + 512 * jt));
      eb[jt] = ld_stream(reinterpret_cast<const h8*>(ep1 + o + 512 * jt));
    }
  }
  __device__ __forceinline__ void prime() {
#pragma unroll
    for (int u = 0; u < D - 1; ++u) issue(u, rt[u], ra[u], rb[u]);
  }
  template <class Mma>
  __device__ __forceinline__ void run(Mma&& mma) {
#pragma unroll 1
    for (int q0 = 0; q0 < NQ; q0 += D) {
#pragma unroll
      for (int u = 0; u < D; ++u) {
        const int q = q0 + u;
        const int v = (u + D - 1) % D;
        issue(min(q + D - 1, NQ - 1), rt[v], ra[v], rb[v]);  // past the end: a re-read
        __builtin_amdgcn_sched_barrier(0);
        mma(q, rt[u], ra[u], rb[u]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
};
template <int NQ, class Frag>
__device__ __forceinline__ MfmaRing2<NQ, Frag> mfma_ring2(const _Float16* thm, const _Float16* ep0, const _Float16* ep1,
                                                          Frag f) {
  return MfmaRing2<NQ, Frag>{thm, ep0, ep1, f};
}

// The head logits of a workgroup's NE envs (policies/impala.py:122): logit[e][ai] = b[ai] + sum_k W[ai][k] hs[k][e],
// split over the 512 threads -- P parts of 256 / P inputs each, the parts added in part order (P = 8 at A * NE <= 64).
// (One wave walking the 256 dependent FMAs per logit left the other seven waiting at the next barrier.)
template <int E, int NE>
__device__ __forceinline__ void head_split(const float* pack, int64_t pack_stride, int l0, const Layout& L, int A,
                                           const float* hs, float* part, float* logit) {
  const int j = threadIdx.x, nl = A * NE;
  const int parts = nl <= 64 ? 8 : (nl <= 128 ? 4 : (nl <= 256 ? 2 : 1));
  const int kn = kHid / parts;
  if (j < parts * nl) {
    const int pi = j / nl, r = j - pi * nl, ai = r / NE, e = r - ai * NE;
    const float* wh = pack + (int64_t)(l0 + e / E) * pack_stride + L.head_w + ai * kHid + pi * kn;
    const float* hp = hs + (pi * kn) * NE + e;
    float s = 0.f;
    for (int k = 0; k < kn; ++k) s = fmaf(wh[k], hp[k * NE], s);
    part[j] = s;
  }
  __syncthreads();
  if (j < nl) {
    const int ai = j / NE, e = j - ai * NE;
    float s = part[j];
    for (int pi = 1; pi < parts; ++pi) s += part[pi * nl + j];
    logit[e * kMaxAct + ai] = s + pack[(int64_t)(l0 + e / E) * pack_stride + L.head_b + ai];
  }
}

template <int E, int MODE>
__global__ __launch_bounds__(2 * kCoreThreads) __attribute__((amdgpu_waves_per_eu(2))) void core_kernel_hpm2(
    Layout L, StepArgs a) {
  constexpr int E2 = 2 * E, NE = 4 * E;  // envs of a pair / of the workgroup's 4 lanes
  // the rollout step only: the sequence modes run whole chunks per launch (replay_chunk_hpm2 below)
  static_assert(MODE == kRollout, "core_kernel_hpm2 is the rollout step");
  constexpr bool kRep = false;
  constexpr int kKs0 = kRep ? kCoreIn / 32 : 0, kNks = kGateKS - kKs0;
  static_assert(NE <= 16 && (NE & (NE - 1)) == 0, "the workgroup's envs are the B operand's columns (mod NE)");
  constexpr int XP = kFeat + 16, GP = kGateKS * 32 + 16;  // f16 pitches, as core_kernel_hpm
  constexpr int kXBytes = NE * XP * 2, kGBytes = kGates * NE * 4;
  __shared__ __attribute__((aligned(16))) char xg[kXBytes > kGBytes ? kXBytes : kGBytes];
  __shared__ __attribute__((aligned(16))) _Float16 gh[NE * GP];
  __shared__ float hs[kHid * NE];
  __shared__ float logit[NE * kMaxAct];
  __shared__ float hpart[2 * kCoreThreads];  // head_split's partial sums
  __shared__ float bsum[4 * kGates];               // b_ih + b_hh of the 4 lanes
  _Float16* xh = reinterpret_cast<_Float16*>(xg);
  float* gates = reinterpret_cast<float*>(xg);
  const int j = threadIdx.x, w = j >> 6, l = j & 63;
  const int u = j & (kHid - 1), hf = j >> 8;       // cell / BN roles: hidden unit u of pair hf's envs
  const int l0 = 4 * blockIdx.x;
  auto pkl = [&](int li) { return a.pack + (int64_t)(l0 + li) * a.pack_stride; };
  const _Float16* ep0 = a.epm + (int64_t)(2 * blockIdx.x) * kMImg;
  const _Float16* ep1 = ep0 + kMImg;
  // wave w: fc column tiles 2w, 2w + 1; gate column tiles 8w .. 8w + 7, two at a time
  auto fc_ring = mfma_ring2<kFcKS>(a.thm, ep0, ep1, [w, l](int q) { return ((int64_t)(q * kFcNT + 2 * w) * 64 + l) * 8; });
  auto gate_ring = mfma_ring2<4 * kNks>(a.thm + kFcImg, ep0 + kFcImg, ep1 + kFcImg, [w, l](int q) {
    const int g = q / kNks, ks = kKs0 + q - g * kNks;
    return ((int64_t)(ks * kGateNT + 8 * w + 2 * g) * 64 + l) * 8;
  });
  if constexpr (kRep)
    gate_ring.prime();
  else
    fc_ring.prime();
  const int64_t e0 = (int64_t)l0 * E;
  const int ep_ = hf * E2;  // this thread's first env in the workgroup (cell / BN roles)
  float gxv[kRep ? E2 : 1][4];
  if constexpr (kRep) {
    const float* g = a.gx + ((int64_t)(a.t - a.gx_t0) * a.n_lanes * E + e0 + ep_) * kGates + u;
#pragma unroll
    for (int e = 0; e < E2; ++e)
#pragma unroll
      for (int q = 0; q < 4; ++q) gxv[e][q] = g[(int64_t)e * kGates + q * kHid];
  }
  const int8_t* sgp = a.sign ? a.sign + l0 : reinterpret_cast<const int8_t*>(a.pack);  // branch-free
  const int8_t sg0 = sgp[0], sg1 = sgp[1], sg2 = sgp[2], sg3 = sgp[3];
  const int A = a.n_act;
  // this lane's B column: env benv of the workgroup (lane bl, pair bl / 2); S X flips the minus lanes' columns and
  // the two E operands see only their own pair's columns
  const int benv = (l & 15) & (NE - 1), bl = benv / E;
  const int8_t bsg = bl == 0 ? sg0 : (bl == 1 ? sg1 : (bl == 2 ? sg2 : sg3));
  const unsigned smask = (a.sign && bsg < 0) ? 0x80008000u : 0u;
  const unsigned zmask = (a.sign && bsg == 0) ? 0u : ~0u;  // a sign-0 (unperturbed) lane: E adds exact zeros
  const unsigned ma = (bl < 2 ? ~0u : 0u) & zmask, mb = (bl < 2 ? 0u : ~0u) & zmask;
  auto bfrag = [&](const _Float16* rowp, int k0, h8& x, h8& xa, h8& xb) {
    x = *reinterpret_cast<const h8*>(rowp + k0 + 8 * (l >> 4));
    const u32x4 sx = __builtin_bit_cast(u32x4, x) ^ u32x4{smask, smask, smask, smask};
    xa = __builtin_bit_cast(h8, sx & u32x4{ma, ma, ma, ma});
    xb = __builtin_bit_cast(h8, sx & u32x4{mb, mb, mb, mb});
  };

  float cj[E2];
#pragma unroll
  for (int e = 0; e < E2; ++e) {
    gh[(ep_ + e) * GP + kCoreIn + u] = (_Float16)a.h[(e0 + ep_ + e) * kHid + u];
    cj[e] = a.c[(e0 + ep_ + e) * kHid + u];
  }
  for (int i = j; i < NE * (GP - kGateK); i += 2 * kCoreThreads) {
    const int e = i / (GP - kGateK);
    gh[e * GP + kGateK + i - e * (GP - kGateK)] = (_Float16)0.f;
  }
#pragma unroll
  for (int it = 0; it < 4 * kGates / (2 * kCoreThreads); ++it) {
    const int i = j + it * 2 * kCoreThreads, li = i / kGates, col = i & (kGates - 1);
    const float* pk = pkl(li);
    bsum[i] = pk[L.lstm_bih + col] + pk[L.lstm_bhh + col];
  }
  if constexpr (kRep) {
    if (j < NE) gh[j * GP + kHid] = (_Float16)0.f;  // W_ih's reward row: its product is inside a.gx
  } else {
  float4 fcb[2];
#pragma unroll
  for (int jt = 0; jt < 2; ++jt)
    fcb[jt] = *reinterpret_cast<const float4*>(pkl(bl) + L.fc_b + 16 * (2 * w + jt) + 4 * (l >> 4));
  const bool has_m = a.bn_mean != nullptr, has_v = a.bn_var != nullptr;
  const float* bmp = has_m ? a.bn_mean + L.bn_stat[15] : a.pack;
  const float* bvp = has_v ? a.bn_var + L.bn_stat[15] : a.pack;
  typedef _Float16 h4v __attribute__((ext_vector_type(4)));
  static_assert(kFeat == 4 * 2 * kCoreThreads, "BN1d prologue: 4 features per thread");
  {
    const int k = 4 * j;
    float rm[4], rv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const float rmv = bmp[k + c], rvv = bvp[k + c];
      rm[c] = has_m ? rmv : 0.f;
      rv[c] = has_v ? rvv : 1.f;
    }
    float4 f[NE];
#pragma unroll
    for (int e = 0; e < NE; ++e) f[e] = *reinterpret_cast<const float4*>(a.feat + (e0 + e) * kFeat + k);
#pragma unroll
    for (int li = 0; li < 4; ++li) {
      const float* pk = pkl(li);
      const float4 w4 = *reinterpret_cast<const float4*>(pk + L.bn_w[15] + k);
      const float4 b4 = *reinterpret_cast<const float4*>(pk + L.bn_b[15] + k);
      float sc[4], sh[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        sc[c] = w4[c] * (1.f / sqrtf(rv[c] + kBnEps));
        sh[c] = b4[c] - rm[c] * sc[c];
      }
#pragma unroll
      for (int e = li * E; e < li * E + E; ++e)
        *reinterpret_cast<h4v*>(xh + e * XP + k) =
            h4v{(_Float16)fmaf(f[e][0], sc[0], sh[0]), (_Float16)fmaf(f[e][1], sc[1], sh[1]),
                (_Float16)fmaf(f[e][2], sc[2], sh[2]), (_Float16)fmaf(f[e][3], sc[3], sh[3])};
    }
  }
  float* ci = a.ci ? a.ci + ((int64_t)a.t * a.n_lanes * E + e0) * kCoreIn : nullptr;
  {
    const float r = fminf(fmaxf(a.rprev[e0 + (j & (NE - 1))], -1.f), 1.f);  // every thread loads: no branch
    if (j < NE) {
      gh[j * GP + kHid] = (_Float16)r;
      if (ci) ci[j * kCoreIn + kHid] = r;
    }
  }
  __syncthreads();
  {  // fc
    f32x4 acc[2];
#pragma unroll
    for (int jt = 0; jt < 2; ++jt) acc[jt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const _Float16* xrow = xh + benv * XP;
    fc_ring.run([&](int q, const h8 (&tf)[2], const h8 (&fa)[2], const h8 (&fb)[2]) {
      h8 x, xa, xb;
      bfrag(xrow, 32 * q, x, xa, xb);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(tf[jt], x, acc[jt], 0, 0, 0);
        acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[jt], xa, acc[jt], 0, 0, 0);
        acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[jt], xb, acc[jt], 0, 0, 0);
      }
    });
    gate_ring.prime();
    if ((l & 15) < NE) {
      const int e = l & 15;
#pragma unroll
      for (int jt = 0; jt < 2; ++jt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int n = 16 * (2 * w + jt) + 4 * (l >> 4) + i;
          const float y = relu(acc[jt][i] + fcb[jt][i]);
          gh[e * GP + n] = (_Float16)y;
          if (ci) ci[e * kCoreIn + n] = y;
        }
    }
  }
  }  // !kRep
  __syncthreads();
  if (a.ci16) {  // the gate rows' x part as f16 core inputs for the replay's x W_ih^T (zero beyond kCoreIn)
    constexpr int kR8 = kCiPitch / 8;
    _Float16* dst = a.ci16 + ((int64_t)a.t * a.n_lanes * E + e0) * kCiPitch;
    for (int i = j; i < NE * kR8; i += 2 * kCoreThreads) {
      const int e = i / kR8, k8 = 8 * (i - e * kR8);
      h8 v = *reinterpret_cast<const h8*>(gh + e * GP + k8);
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = k8 + q < kCoreIn ? v[q] : (_Float16)0.f;
      *reinterpret_cast<h8*>(dst + e * kCiPitch + k8) = v;
    }
  }
  {  // gates
    f32x4 acc[2];
    const _Float16* grow = gh + benv * GP;
    gate_ring.run([&](int q, const h8 (&tf)[2], const h8 (&fa)[2], const h8 (&fb)[2]) {
      const int g = q / kNks, ks = kKs0 + q - g * kNks;
      if (ks == kKs0)
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) acc[jt] = f32x4{0.f, 0.f, 0.f, 0.f};
      h8 x, xa, xb;
      bfrag(grow, 32 * ks, x, xa, xb);
#pragma unroll
      for (int jt = 0; jt < 2; ++jt) {
        acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(tf[jt], x, acc[jt], 0, 0, 0);
        acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[jt], xa, acc[jt], 0, 0, 0);
        acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[jt], xb, acc[jt], 0, 0, 0);
      }
      if (ks == kGateKS - 1 && (l & 15) < NE) {
#pragma unroll
        for (int jt = 0; jt < 2; ++jt)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            gates[(16 * (8 * w + 2 * g + jt) + 4 * (l >> 4) + i) * NE + (l & 15)] = acc[jt][i];
      }
    });
  }
  __syncthreads();
  float hj[E2];
#pragma unroll
  for (int e = 0; e < E2; ++e) {
    const int we = ep_ + e;  // the env in the workgroup; its lane we / E
    float pre[4];
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int col = g * kHid + u;
      pre[g] = gates[col * NE + we] + bsum[(we / E) * kGates + col];
      if constexpr (kRep) pre[g] += gxv[e][g];
    }
    auto sg = [](float x) { return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x)); };
    const float gi = sg(pre[0]), gf = sg(pre[1]), gg = tanh_fast(pre[2]), go = sg(pre[3]);
    cj[e] = fmaf(gf, cj[e], gi * gg);  // explicit: the same rounding in every core form
    hj[e] = go * tanh_fast(cj[e]);
    a.h[(e0 + we) * kHid + u] = hj[e];
    a.c[(e0 + we) * kHid + u] = cj[e];
  }
  {
    const float rmv = (a.bn_mean ? a.bn_mean + L.bn_stat[16] : a.pack)[u];  // branch-free
    const float rvv = (a.bn_var ? a.bn_var + L.bn_stat[16] : a.pack)[u];
    const float rm = a.bn_mean ? rmv : 0.f, rv = a.bn_var ? rvv : 1.f;
#pragma unroll
    for (int h2i = 0; h2i < 2; ++h2i) {  // the pair's two lanes
      const float* pk = pkl(2 * hf + h2i);
      const float sc = pk[L.bn_w[16] + u] * (1.f / sqrtf(rv + kBnEps));
      const float sh = fmaf(-rm, sc, pk[L.bn_b[16] + u]);
#pragma unroll
      for (int e = 0; e < E; ++e) hs[u * NE + ep_ + h2i * E + e] = fmaf(hj[h2i * E + e], sc, sh);
    }
  }
  __syncthreads();
  head_split<E, NE>(a.pack, a.pack_stride, l0, L, A, hs, hpart, logit);
  __syncthreads();
  if (j < NE) core_finish<E, MODE>(a, logit + (j / E) * E * kMaxAct, l0 + j / E, j % E);
}
template __global__ void core_kernel_hpm2<1, kRollout>(Layout, StepArgs);
template __global__ void core_kernel_hpm2<2, kRollout>(Layout, StepArgs);
template __global__ void core_kernel_hpm2<4, kRollout>(Layout, StepArgs);

// ---- The entropy replay of a whole chunk per launch (ctx core_mfma = 2) -----------------------------------------------
// A per-step replay launch (two pairs per workgroup) streamed the pairs' W_hh images in ~38 us of its ~62 at config 5
// and spent the rest on its prologue (h / c / biases / signs) and epilogue (cell, BN1d, head, entropy).  The pairs'
// sequences are independent, so one workgroup runs every step of the chunk for its two pairs: the prologue runs once,
// h / c / the entropy sums stay in registers, and the next step's first fragments load under the epilogue (the
// weights do not depend on h).  Each step is core_kernel_hpm<E, kReplay>'s arithmetic in its order: bitwise equal to
// the one-pair form (core_mfma 1) over whole episodes.
template <int E, int MODE>
__global__ __launch_bounds__(2 * kCoreThreads) __attribute__((amdgpu_waves_per_eu(2))) void replay_chunk_hpm2(
    Layout L, StepArgs a, int t0, int tc) {
  static_assert(MODE == kReplay || MODE == kStrategy, "sequence modes");
  constexpr int E2 = 2 * E, NE = 4 * E;
  constexpr int kKs0 = kCoreIn / 32, kNks = kGateKS - kKs0, NQ = 4 * kNks;
  static_assert(NE <= 16 && (NE & (NE - 1)) == 0, "the workgroup's envs are the B operand's columns (mod NE)");
  constexpr int GP = kGateKS * 32 + 16;
  __shared__ __attribute__((aligned(16))) float gates[kGates * NE];
  __shared__ __attribute__((aligned(16))) _Float16 gh[NE * GP];
  __shared__ float hs[kHid * NE];
  __shared__ float logit[NE * kMaxAct];
  __shared__ float hpart[2 * kCoreThreads];  // head_split's partial sums
  __shared__ float bsum[4 * kGates];
  const int j = threadIdx.x, w = j >> 6, l = j & 63;
  const int u = j & (kHid - 1), hf = j >> 8;
  const int l0 = 4 * blockIdx.x;
  auto pkl = [&](int li) { return a.pack + (int64_t)(l0 + li) * a.pack_stride; };
  const _Float16* ep0 = a.epm + (int64_t)(2 * blockIdx.x) * kMImg;
  const _Float16* ep1 = ep0 + kMImg;
  auto ring = mfma_ring2<NQ>(a.thm + kFcImg, ep0 + kFcImg, ep1 + kFcImg, [w, l](int q) {
    const int g = q / kNks, ks = kKs0 + q - g * kNks;
    return ((int64_t)(ks * kGateNT + 8 * w + 2 * g) * 64 + l) * 8;
  });
  ring.prime();
  const int64_t e0 = (int64_t)l0 * E;
  const int ep_ = hf * E2;
  const int8_t* sgp = a.sign ? a.sign + l0 : reinterpret_cast<const int8_t*>(a.pack);  // branch-free
  const int8_t sg0 = sgp[0], sg1 = sgp[1], sg2 = sgp[2], sg3 = sgp[3];
  const int A = a.n_act;
  const int benv = (l & 15) & (NE - 1), bl = benv / E;
  const int8_t bsg = bl == 0 ? sg0 : (bl == 1 ? sg1 : (bl == 2 ? sg2 : sg3));
  const unsigned smask = (a.sign && bsg < 0) ? 0x80008000u : 0u;
  const unsigned zmask = (a.sign && bsg == 0) ? 0u : ~0u;
  const unsigned ma = (bl < 2 ? ~0u : 0u) & zmask, mb = (bl < 2 ? 0u : ~0u) & zmask;
  auto bfrag = [&](const _Float16* rowp, int k0, h8& x, h8& xa, h8& xb) {
    x = *reinterpret_cast<const h8*>(rowp + k0 + 8 * (l >> 4));
    const u32x4 sx = __builtin_bit_cast(u32x4, x) ^ u32x4{smask, smask, smask, smask};
    xa = __builtin_bit_cast(h8, sx & u32x4{ma, ma, ma, ma});
    xb = __builtin_bit_cast(h8, sx & u32x4{mb, mb, mb, mb});
  };
  float cj[E2], hj[E2];
#pragma unroll
  for (int e = 0; e < E2; ++e) {
    gh[(ep_ + e) * GP + kCoreIn + u] = (_Float16)a.h[(e0 + ep_ + e) * kHid + u];
    cj[e] = a.c[(e0 + ep_ + e) * kHid + u];
    hj[e] = 0.f;
  }
  for (int i = j; i < NE * (GP - kGateK); i += 2 * kCoreThreads) {
    const int e = i / (GP - kGateK);
    gh[e * GP + kGateK + i - e * (GP - kGateK)] = (_Float16)0.f;
  }
#pragma unroll
  for (int it = 0; it < 4 * kGates / (2 * kCoreThreads); ++it) {
    const int i = j + it * 2 * kCoreThreads, li = i / kGates, col = i & (kGates - 1);
    const float* pk = pkl(li);
    bsum[i] = pk[L.lstm_bih + col] + pk[L.lstm_bhh + col];
  }
  if (j < NE) gh[j * GP + kHid] = (_Float16)0.f;  // W_ih's reward row: its product is inside a.gx
  // head BN1d of unit u for the pair's two lanes (constant over the chunk)
  float bsc[2], bsh[2];
  {
    const float rmv = (a.bn_mean ? a.bn_mean + L.bn_stat[16] : a.pack)[u];  // branch-free
    const float rvv = (a.bn_var ? a.bn_var + L.bn_stat[16] : a.pack)[u];
    const float rm = a.bn_mean ? rmv : 0.f, rv = a.bn_var ? rvv : 1.f;
#pragma unroll
    for (int h2i = 0; h2i < 2; ++h2i) {
      const float* pk = pkl(2 * hf + h2i);
      bsc[h2i] = pk[L.bn_w[16] + u] * (1.f / sqrtf(rv + kBnEps));
      bsh[h2i] = fmaf(-rm, bsc[h2i], pk[L.bn_b[16] + u]);
    }
  }
  // thread j < NE: env j's entropy sum, continued from a.ent in the per-step kernel's order and stored at the end
  double ent = MODE == kReplay ? a.ent[e0 + (j & (NE - 1))] : 0.0;
  for (int s = 0; s < tc; ++s) {
    const int t = t0 + s;
    float gxv[E2][4];
    {
      const float* g = a.gx + ((int64_t)(t - a.gx_t0) * a.n_lanes * E + e0 + ep_) * kGates + u;
#pragma unroll
      for (int e = 0; e < E2; ++e)
#pragma unroll
        for (int q = 0; q < 4; ++q) gxv[e][q] = g[(int64_t)e * kGates + q * kHid];
    }
    __syncthreads();  // gh holds h_(t-1) (the prologue or the previous step's cell phase)
    {
      f32x4 acc[2];
      const _Float16* grow = gh + benv * GP;
      ring.run([&](int q, const h8 (&tf)[2], const h8 (&fa)[2], const h8 (&fb)[2]) {
        const int g = q / kNks, ks = kKs0 + q - g * kNks;
        if (ks == kKs0)
#pragma unroll
          for (int jt = 0; jt < 2; ++jt) acc[jt] = f32x4{0.f, 0.f, 0.f, 0.f};
        h8 x, xa, xb;
        bfrag(grow, 32 * ks, x, xa, xb);
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
          acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(tf[jt], x, acc[jt], 0, 0, 0);
          acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fa[jt], xa, acc[jt], 0, 0, 0);
          acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(fb[jt], xb, acc[jt], 0, 0, 0);
        }
        if (ks == kGateKS - 1 && (l & 15) < NE) {
#pragma unroll
          for (int jt = 0; jt < 2; ++jt)
#pragma unroll
            for (int i = 0; i < 4; ++i)
              gates[(16 * (8 * w + 2 * g + jt) + 4 * (l >> 4) + i) * NE + (l & 15)] = acc[jt][i];
        }
      });
    }
    if (s + 1 < tc) ring.prime();  // the next step's first fragments, under this step's epilogue
    __syncthreads();
#pragma unroll
    for (int e = 0; e < E2; ++e) {
      const int we = ep_ + e;
      float pre[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int col = g * kHid + u;
        pre[g] = gates[col * NE + we] + bsum[(we / E) * kGates + col];
        pre[g] += gxv[e][g];
      }
      auto sg = [](float x) { return __builtin_amdgcn_rcpf(1.f + __builtin_amdgcn_exp2f(-1.44269504088896341f * x)); };
      const float gi = sg(pre[0]), gf = sg(pre[1]), gg = tanh_fast(pre[2]), go = sg(pre[3]);
      cj[e] = fmaf(gf, cj[e], gi * gg);  // explicit: the same rounding in every core form
      hj[e] = go * tanh_fast(cj[e]);
      gh[we * GP + kCoreIn + u] = (_Float16)hj[e];  // the next step's B rows (read after its first barrier)
    }
#pragma unroll
    for (int h2i = 0; h2i < 2; ++h2i)
#pragma unroll
      for (int e = 0; e < E; ++e) hs[u * NE + ep_ + h2i * E + e] = fmaf(hj[h2i * E + e], bsc[h2i], bsh[h2i]);
    __syncthreads();
    head_split<E, NE>(a.pack, a.pack_stride, l0, L, A, hs, hpart, logit);
    __syncthreads();
    if (j < NE) core_finish<E, MODE>(a, logit + (j / E) * E * kMaxAct, l0 + j / E, j % E, false, &ent, t);
  }
#pragma unroll
  for (int e = 0; e < E2; ++e) {
    a.h[(e0 + ep_ + e) * kHid + u] = hj[e];
    a.c[(e0 + ep_ + e) * kHid + u] = cj[e];
  }
  if (MODE == kReplay && j < NE) a.ent[e0 + j] = ent;
}
template __global__ void replay_chunk_hpm2<1, kReplay>(Layout, StepArgs, int, int);
template __global__ void replay_chunk_hpm2<2, kReplay>(Layout, StepArgs, int, int);
template __global__ void replay_chunk_hpm2<4, kReplay>(Layout, StepArgs, int, int);
template __global__ void replay_chunk_hpm2<1, kStrategy>(Layout, StepArgs, int, int);

// Entropy replay, input projection of one chunk in the fp16 pair form on MFMA: gx = theta X + s (E X) with the
// gate images' k-steps 0 .. 8 (rows 0 .. 287 = W_ih^T's 257 rows; X is zero beyond k = 256) -- the per-lane
// f32 GEMM (lstm_xproj_kernel<true>) ran at the f32 MFMA rate and re-read each lane's W_ih per row block.
// A workgroup = (pair, group of 4 column tiles): it holds the group's theta / E fragments in LDS (72 KiB) and its 4
// waves take the pair's row tiles (rows = (t, env of the pair), B columns; X rounded to f16).  XCD-aware grid
// (xproj_grid): the kGateNT / 4 = 16 workgroups of a pair are dispatched together onto ONE XCD, so the pair's chunk of
// core inputs (64 steps x 2E envs x 257 f32, 0.5 MB) is fetched from HBM once and re-read from that XCD's L2 by the
// other 15 (with the pair as the fast grid index the 16 readers were ~n_pairs workgroups apart: 16 HBM reads).
constexpr int kXprojGroups = kGateNT / 4;
template <int E, bool H16>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void xproj_pair_kernel(Layout L, StepArgs a, int t0,
                                                                                            int tc, float* __restrict__ gx) {
  constexpr int E2 = 2 * E, KS = (kCoreIn + 31) / 32;
  __shared__ h8 af[2][KS][4][64];
  const int b = blockIdx.x, xcd = b & 7, slot = b >> 3;
  const int pr = (slot / kXprojGroups) * 8 + xcd, nt0 = 4 * (slot % kXprojGroups);
  if (2 * pr >= a.n_lanes) return;  // (the grid rounds the pairs up to a multiple of 8)
  const int tid = threadIdx.x, w = tid >> 6, l = tid & 63;
  const _Float16* src[2] = {a.thm + kFcImg, a.epm + (int64_t)pr * kMImg + kFcImg};
  for (int i = tid; i < 2 * KS * 4 * 64; i += 256) {
    const int sidx = i / (KS * 256), rem = i - sidx * (KS * 256), ks = rem >> 8, jt = (rem >> 6) & 3, ll = rem & 63;
    af[sidx][ks][jt][ll] = *reinterpret_cast<const h8*>(src[sidx] + (((int64_t)ks * kGateNT + nt0 + jt) * 64 + ll) * 8);
  }
  const int l0 = 2 * pr;
  const bool neg0 = a.sign && a.sign[l0] < 0, neg1 = a.sign && a.sign[l0 + 1] < 0;
  const bool zero0 = a.sign && a.sign[l0] == 0, zero1 = a.sign && a.sign[l0 + 1] == 0;
  const int64_t e0 = (int64_t)l0 * E, ne = (int64_t)a.n_lanes * E;
  const int rows = tc * E2;
  __syncthreads();
  for (int rt = w; rt < (rows + 15) / 16; rt += 4) {
    const int row = rt * 16 + (l & 15);  // this lane's B column
    const bool ok = row < rows;
    const int rr = ok ? row : 0, t = rr / E2, env = rr - t * E2;
    const float* xr = H16 ? nullptr : a.ci + ((int64_t)(t0 + t) * ne + e0 + env) * kCoreIn;
    const _Float16* xr16 = H16 ? a.ci16 + ((int64_t)(t0 + t) * ne + e0 + env) * kCiPitch + 8 * (l >> 4) : nullptr;
    const unsigned smask = (env < E ? neg0 : neg1) ? 0x80008000u : 0u;
    const unsigned zmask = (env < E ? zero0 : zero1) ? 0u : ~0u;  // sign-0 lane: E X = 0
    f32x4 acc[4];
#pragma unroll
    for (int jt = 0; jt < 4; ++jt) acc[jt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 3
    for (int ks = 0; ks < KS; ++ks) {
      h8 x;
      if constexpr (H16) {  // the rollout's f16 rows (zero beyond kCoreIn); a dead row reads row 0 and is dropped
        const h8 v = *reinterpret_cast<const h8*>(xr16 + 32 * ks);
        const unsigned okm = ok ? ~0u : 0u;
        x = __builtin_bit_cast(h8, __builtin_bit_cast(u32x4, v) & u32x4{okm, okm, okm, okm});
      } else {
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          const int k = 32 * ks + 8 * (l >> 4) + i;
          const float v = xr[k < kCoreIn ? k : 0];  // branch-free: the clamped load is discarded
          x[i] = (_Float16)(ok && k < kCoreIn ? v : 0.f);
        }
      }
      u32x4 u = __builtin_bit_cast(u32x4, x);
      u = (u ^ u32x4{smask, smask, smask, smask}) & u32x4{zmask, zmask, zmask, zmask};
      const h8 sx = __builtin_bit_cast(h8, u);
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) {
        acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[0][ks][jt][l], x, acc[jt], 0, 0, 0);
        acc[jt] = __builtin_amdgcn_mfma_f32_16x16x32_f16(af[1][ks][jt][l], sx, acc[jt], 0, 0, 0);
      }
    }
    if (ok) {  // lane: gate columns 16 (nt0 + jt) + 4 (l >> 4) .. +3 of its row
      float* dst = gx + ((int64_t)t * ne + e0 + env) * kGates + 16 * nt0 + 4 * (l >> 4);
#pragma unroll
      for (int jt = 0; jt < 4; ++jt) *reinterpret_cast<f32x4*>(dst + 16 * jt) = acc[jt];
    }
  }
}
template __global__ void xproj_pair_kernel<1, false>(Layout, StepArgs, int, int, float*);
template __global__ void xproj_pair_kernel<1, true>(Layout, StepArgs, int, int, float*);
template __global__ void xproj_pair_kernel<2, true>(Layout, StepArgs, int, int, float*);
template __global__ void xproj_pair_kernel<4, true>(Layout, StepArgs, int, int, float*);

template __global__ void core_kernel_h<1, kRollout>(Layout, StepArgs);
template __global__ void core_kernel_h<1, kReplay>(Layout, StepArgs);
template __global__ void core_kernel_h<1, kForward>(Layout, StepArgs);
template __global__ void core_kernel_h<1, kStrategy>(Layout, StepArgs);
template __global__ void core_kernel_h<2, kRollout>(Layout, StepArgs);
template __global__ void core_kernel_h<2, kReplay>(Layout, StepArgs);
template __global__ void core_kernel_h<4, kRollout>(Layout, StepArgs);
template __global__ void core_kernel_h<4, kReplay>(Layout, StepArgs);
template __global__ void core_kernel_h<8, kRollout>(Layout, StepArgs);
template __global__ void core_kernel_h<8, kReplay>(Layout, StepArgs);


}  // namespace impala
}  // namespace fdr
