// fdr_impala.hip -- ImpalaPolicy rollouts (policies/impala.py:8-186) on gfx950.
//
// Per rollout:   prep    theta'_l = fl32(theta + fl32(sigma * s_l * eps_l)) gathered once into a
//                        per-lane pack laid out for the kernels (+ |lambda_l|^2 partials)
// Per step t:    conv    one workgroup per (lane, env): synthetic frame -> 15 convs on f32 MFMA
//                        (v_mfma_f32_16x16x4_f32), activations LDS-resident, -> relu'd 2048 feature
//                core    one workgroup per lane (E envs): BN1d + fc + ReLU, LSTM cell, BN1d + head,
//                        softmax, action, synthetic reward, return
// After T steps: replay  the reference's entropy pass (worker/agent.py:60-66): the visited obs
//                        replayed through the LSTM from the end-of-episode state
//                finish  jiggle, mean entropy, steps, |lambda|^2
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cfloat>
#include <cmath>
#include <vector>

#include "fdr_impala.h"

namespace fdr {
namespace impala {

typedef float f32x4 __attribute__((ext_vector_type(4)));

constexpr int kCh[3] = {16, 32, 32};
constexpr uint64_t kFrameSalt = 0x4652414D45533031ull;  // oracle/impala.py FRAME_SALT
constexpr uint64_t kRewardSalt = 0x5245574152443031ull; // oracle/impala.py REWARD_SALT

// ------------------------------------------------------------------------------------------
// Host: pack layout.  Walks the reference's parameters() order (feat_convs, resnet1, resnet2,
// fc, core, policy -- policies/impala.py:60-119) and assigns every tensor a pack section.
// Conv / BN index = stage * 5 + part, part 0 = stage entry, 1/2 = resnet1 bn0+conv0 / bn1+conv1,
// 3/4 = resnet2; BN 15 = fc BN1d, 16 = head BN1d.  Running stats follow modules() order, which
// is the same walk.
// ------------------------------------------------------------------------------------------
static int64_t round_up(int64_t v, int64_t m) { return (v + m - 1) / m * m; }

bool make_layout(int n_act, Layout* L) {
  if (n_act < 1 || n_act > kMaxAct) return false;
  *L = Layout{};
  L->n_act = n_act;
  int32_t dst = 0, src = 0, stat = 0;
  auto add = [&](int32_t kind, int32_t len, int32_t a, int32_t b, int32_t src_len) {
    dst = (int32_t)round_up(dst, 16);  // 64-byte aligned sections: float4 streaming in the core kernel
    Section& s = L->sec[L->n_sections++];
    s = Section{dst, len, src, kind, a, b};
    const int32_t at = dst;
    dst += len;
    src += src_len;
    return at;
  };
  auto bn = [&](int idx, int ch) {
    L->bn_w[idx] = add(kCopy, 2 * ch, 0, 0, 2 * ch);  // weight then bias, contiguous in theta
    L->bn_b[idx] = L->bn_w[idx] + ch;
    L->bn_stat[idx] = stat;
    stat += ch;
  };
  auto conv = [&](int idx, int cin, int cout) {
    const int kpad = (int)round_up(9 * cin, 4);
    L->conv_w[idx] = add(kConvFrag, kpad * cout, cin, cout, 9 * cin * cout);
    L->conv_b[idx] = add(kCopy, cout, 0, 0, cout);
  };
  int cin = 3;
  for (int s = 0; s < 3; ++s) {  // feat_convs[s]: BN2d(cin), Conv2d(cin -> c)
    bn(s * 5, cin);
    conv(s * 5, cin, kCh[s]);
    cin = kCh[s];
  }
  for (int r = 0; r < 2; ++r)    // resnet1[s], resnet2[s]: (BN, ReLU, Conv) x 2
    for (int s = 0; s < 3; ++s)
      for (int j = 0; j < 2; ++j) {
        const int idx = s * 5 + 1 + 2 * r + j;
        bn(idx, kCh[s]);
        conv(idx, kCh[s], kCh[s]);
      }
  bn(15, kFeat);                                                   // fc[0] BatchNorm1d(2048)
  L->fc_wt = add(kTranspose, kFeat * kHid, kHid, kFeat, kFeat * kHid);  // fc[1].weight -> W^T
  L->fc_b = add(kCopy, kHid, 0, 0, kHid);
  L->lstm_wt = add(kTranspose, kCoreIn * kGates, kGates, kCoreIn, kCoreIn * kGates);  // W_ih^T
  add(kTranspose, kHid * kGates, kGates, kHid, kHid * kGates);                        // W_hh^T
  L->lstm_bih = add(kCopy, 2 * kGates, 0, 0, 2 * kGates);  // b_ih, b_hh
  L->lstm_bhh = L->lstm_bih + kGates;
  bn(16, kHid);                                                    // policy[0] BatchNorm1d(256)
  L->head_w = add(kCopy, n_act * kHid + n_act, 0, 0, n_act * kHid + n_act);  // weight, bias
  L->head_b = L->head_w + n_act * kHid;
  L->P = src;
  L->pack = round_up(dst, 64);
  L->n_bn_stats = stat;

  // half pack: walk the same source offsets again
  int32_t hdst = 0;
  auto hadd = [&](int32_t kind, int32_t len, int32_t a, int32_t b, int32_t s0) {
    hdst = (int32_t)round_up(hdst, 64);
    Section& h = L->hsec[L->n_hsections++];
    h = Section{hdst, len, s0, kind, a, b};
    const int32_t at = hdst;
    hdst += len;
    return at;
  };
  for (int i = 0; i < L->n_sections; ++i) {
    const Section& q = L->sec[i];
    if (q.kind == kConvFrag) {
      const int cin = q.a, cout = q.b;
      const int ks = cin == 3 ? 2 : (9 * cin + 31) / 32;      // k-steps of 32
      const int idx = [&] { for (int c = 0; c < kConvs; ++c) if (L->conv_w[c] == q.dst) return c; return -1; }();
      L->conv_h[idx] = hadd(kConvFragH, ks * (cout / 16) * 64 * 8, cin, cout, q.src);
    } else if (q.kind == kTranspose) {
      const int32_t at = hadd(kTranspose, q.len, q.a, q.b, q.src);
      if (q.dst == L->fc_wt) L->fc_wt_h = at;
      if (q.dst == L->lstm_wt) L->lstm_wt_h = at;
    }
  }
  L->hpack = round_up(hdst, 64);
  return true;
}

constexpr int kPrepThreads = 256;
constexpr int kPrepPer = 4;
constexpr int kPrepSpan = kPrepThreads * kPrepPer;

bool pair_core_supported(int envs) { return envs == 1 || envs == 2 || envs == 4; }

Plan plan(const Layout& L, int n_lanes, int envs, int T, bool entropy, bool fp16, bool pairs) {
  Plan p{};
  const int64_t ne = (int64_t)n_lanes * envs;
  int64_t o = 0;
  auto take = [&](int64_t bytes) { const int64_t at = o; o += round_up(std::max<int64_t>(bytes, 0), 256); return at; };
  p.nblk = prep_blocks(L);
  p.pack = take((int64_t)n_lanes * L.pack * 4);
  p.hpack = take(fp16 ? (int64_t)n_lanes * L.hpack * 2 : 0);
  p.feat = take(ne * kFeat * 4);
  p.h = take(ne * kHid * 4);
  p.c = take(ne * kHid * 4);
  p.rprev = take(ne * 4);
  p.ci = take(entropy ? (int64_t)T * ne * kCoreIn * 4 : 0);
  p.gx = take(entropy ? (int64_t)std::min(T, kReplayChunk) * ne * kGates * 4 : 0);
  p.n2 = take((int64_t)n_lanes * p.nblk * 8);
  const bool pr = pairs && pair_core_supported(envs);
  const int64_t plen = fp16 ? L.hpack * 2 : L.pack * 4;  // one (half) pack in bytes
  p.zeros = take(pr ? L.P * 4 : 0);
  p.thpack = take(pr ? plen : 0);
  p.epack = take(pr ? (int64_t)(n_lanes / 2) * plen : 0);
  p.idxe = take(pr ? (int64_t)(n_lanes / 2) * 8 : 0);
  p.n2x = take(pr && !fp16 ? (int64_t)(n_lanes / 2 + 1) * p.nblk * 8 : 0);  // the f32 pack kernels' n2 partials
  p.mimg = take(pr && fp16 ? (int64_t)(n_lanes / 2 + 1) * kMImg * 2 : 0);  // theta's + the pairs' MFMA images
  p.bntab = take(fp16 ? (int64_t)n_lanes * 3 * kBnTab * 4 : 0);       // the conv stack's folded BN / bias tables
  p.total = o;
  return p;
}

// ------------------------------------------------------------------------------------------
// prep: pack[lane][j] = theta'_lane[src(j)]  (fl32(theta + fl32(sigma * +-eps)), no contraction)
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ int64_t section_src(const Section& s, int32_t u) {
  if (s.kind == kCopy) return (int64_t)s.src + u;
  if (s.kind == kTranspose) {  // pack = W^T: u = k * rows + r  ->  W[r][k]
    const int32_t k = u / s.a, r = u - k * s.a;
    return (int64_t)s.src + (int64_t)r * s.b + k;
  }
  if (s.kind == kConvFragH) {
    // f16 A-fragment (v_mfma_f32_16x16x32_f16, weights as A): u = ((kstep * NT + nt) * 64 + l) * 8 + jj,
    // A[i = nt*16 + (l & 15)][k = 8 (l >> 4) + jj].  K order per k-step of 32: Cin % 8 == 0 -> lane group
    // g = l >> 4 holds 8 consecutive channels of one tap (taps per k-step 32 / Cin); Cin = 3 (frame image
    // with 4 channel slots) -> group g holds taps 8 kstep + 2g, +1 with 4 channel slots each.
    const int32_t cin = s.a, nt_n = s.b / 16;
    const int32_t jj = u & 7, l = (u >> 3) & 63, rest = u >> 9;
    const int32_t nt = rest % nt_n, ks = rest / nt_n;
    const int32_t i = nt * 16 + (l & 15), g = l >> 4;
    int32_t tap, ci;
    if (cin == 3) {
      tap = 8 * ks + 2 * g + (jj >> 2);
      ci = jj & 3;
      if (ci >= 3) return -1;
    } else {
      const int32_t cpg = cin / 8, tpk = 32 / cin;
      tap = ks * tpk + g / cpg;
      ci = 8 * (g % cpg) + jj;
    }
    if (tap >= 9) return -1;
    return (int64_t)s.src + ((int64_t)i * cin + ci) * 9 + tap;
  }
  // conv B-fragment (v_mfma_f32_16x16x4_f32): u = (kstep * NT + nt) * 64 + l; B[k][n] with
  // k = 4 * kstep + (l >> 4), n = nt * 16 + (l & 15).  K order: Cin % 4 == 0 -> tap-major,
  // cin = 4 * (kstep % (Cin/4)) + (l >> 4); Cin = 3 -> k = tap * 3 + cin, zero-padded to 28.
  const int32_t cin = s.a & 255, cout = s.b, nt_n = cout / 16;
  const int32_t ntaps = (s.a >> 8) ? (s.a >> 8) : 9;  // AtariPolicy convs: 8x8 / 4x4 kernels
  const int32_t ks = u / (nt_n * 64), rem = u - ks * nt_n * 64;
  const int32_t nt = rem >> 6, l = rem & 63;
  const int32_t n = nt * 16 + (l & 15);
  int32_t tap, ci;
  if ((cin & 3) == 0) {
    const int32_t q = cin >> 2;
    tap = ks / q;
    ci = 4 * (ks - tap * q) + (l >> 4);
  } else {
    const int32_t k = 4 * ks + (l >> 4);
    if (k >= 9 * cin) return -1;
    tap = k / cin;
    ci = k - tap * cin;
  }
  if (tap >= ntaps) return -1;
  return (int64_t)s.src + ((int64_t)n * cin + ci) * ntaps + tap;
}

template <typename OUT>
__global__ __launch_bounds__(kPrepThreads) void prep_kernel(Layout L, LanesArgs lanes, OUT* __restrict__ pack,
                                                            double* __restrict__ n2_part, int half, int n2_slots) {
  const int lane = blockIdx.y;
  ParamSrc src = lanes.src(lane);
  const int64_t j0 = (int64_t)blockIdx.x * kPrepSpan + threadIdx.x;
  const int64_t len = half ? L.hpack : L.pack;
  const Section* sec = half ? L.hsec : L.sec;
  const int nsec = half ? L.n_hsections : L.n_sections;
  OUT* out = pack + (int64_t)lane * len;
  const bool bad = src.n2 != src.n2;  // out-of-range table offset: NaN norm, unperturbed lane
  src.n2 = 0.0;
  {  // a block entirely inside one transposed section has nothing to do (prep_transpose_kernel)
    const int64_t b0 = (int64_t)blockIdx.x * kPrepSpan, b1 = b0 + kPrepSpan - 1;
    int lo = 0, hi = nsec - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (sec[mid].dst <= b0) lo = mid; else hi = mid - 1;
    }
    if (sec[lo].kind == kTranspose && b0 >= sec[lo].dst && b1 < (int64_t)sec[lo].dst + sec[lo].len) {
      if (!half && threadIdx.x == 0) n2_part[(int64_t)lane * n2_slots + blockIdx.x] = bad ? __builtin_nan("") : 0.0;
      return;
    }
  }
#pragma unroll
  for (int i = 0; i < kPrepPer; ++i) {
    const int64_t j = j0 + (int64_t)i * kPrepThreads;
    if (j >= len) break;
    int lo = 0, hi = nsec - 1;  // last section with dst <= j
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (sec[mid].dst <= j) lo = mid; else hi = mid - 1;
    }
    const Section& s = sec[lo];
    const int32_t u = (int32_t)(j - s.dst);
    if (s.kind == kTranspose && j >= s.dst && u < s.len) continue;  // prep_transpose_kernel's part
    const int64_t p = (j >= s.dst && u < s.len) ? section_src(s, u) : -1;
    out[j] = (OUT)(p >= 0 ? (half ? src.get_nocount(p) : src.get(p)) : 0.f);
  }
  if (half) return;
  double n2 = src.n2;
  // block reduce (deterministic): wave sums, then wave 0
  __shared__ double red[kPrepThreads / kWave];
  n2 = wave_sum(n2);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = n2;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < kPrepThreads / kWave; ++w) t += red[w];
    n2_part[(int64_t)lane * n2_slots + blockIdx.x] = bad ? __builtin_nan("") : t;
  }
}

// Transposed sections (fc W^T, [W_ih | W_hh]^T: 90 % of the pack) through a 64 x 64 LDS tile: theta and
// the lane's noise-table slice are read along W's rows (coalesced) and W^T is written along its rows
// (coalesced) -- the element-order gather of prep_kernel read them at a 4-8 KB stride (one 64-B
// line per 4-byte element).  Same values (fl32(theta +- fl32(sigma eps))) and the same n2 terms.
constexpr int kTT = 64;  // transpose tile edge
__host__ __device__ inline int transpose_tiles(const Section& s) { return ((s.a + kTT - 1) / kTT) * ((s.b + kTT - 1) / kTT); }

// write = 0: the f32 call's n2 partials only (the same reads and reduce order, no tile, no stores) -- for fp16 calls,
// whose kernels take these weights from the half pack / the pair images
template <class OUT>
__global__ __launch_bounds__(256) void prep_transpose_kernel(Layout L, LanesArgs lanes, OUT* __restrict__ pack,
                                                             double* __restrict__ n2_part, int half, int n2_slot0,
                                                             int n2_slots, int write) {
  __shared__ float tile[kTT][kTT + 1];
  __shared__ double red[256 / kWave];
  const int lane = blockIdx.y;
  ParamSrc src = lanes.src(lane);
  const bool bad = src.n2 != src.n2;
  src.n2 = 0.0;
  const Section* sec = half ? L.hsec : L.sec;
  const int nsec = half ? L.n_hsections : L.n_sections;
  int t = blockIdx.x, si = 0;
  for (; si < nsec; ++si) {
    if (sec[si].kind != kTranspose) continue;
    const int n = transpose_tiles(sec[si]);
    if (t < n) break;
    t -= n;
  }
  const Section s = sec[si];
  const int tr = (s.a + kTT - 1) / kTT;
  const int r0 = (t % tr) * kTT, k0 = (t / tr) * kTT;
  OUT* out = pack + (int64_t)lane * (half ? L.hpack : L.pack) + s.dst;
#pragma unroll
  for (int m = 0; m < kTT * kTT / 256; ++m) {  // W[r][k] along k
    const int e = threadIdx.x + 256 * m, i = e / kTT, jj = e % kTT, r = r0 + i, k = k0 + jj;
    float v = 0.f;
    if (r < s.a && k < s.b) {
      const int64_t p = (int64_t)s.src + (int64_t)r * s.b + k;
      v = half ? src.get_nocount(p) : src.get(p);
    }
    if (write) tile[jj][i] = v;
  }
  if (write) {
    __syncthreads();
#pragma unroll
    for (int m = 0; m < kTT * kTT / 256; ++m) {  // W^T[k][r] along r
      const int e = threadIdx.x + 256 * m, jj = e / kTT, i = e % kTT, r = r0 + i, k = k0 + jj;
      if (r < s.a && k < s.b) out[(int64_t)k * s.a + r] = (OUT)tile[jj][i];
    }
  }
  if (half) return;
  double n2 = wave_sum(src.n2);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = n2;
  __syncthreads();
  if (threadIdx.x == 0) {
    double tot = 0.0;
    for (int w = 0; w < 256 / kWave; ++w) tot += red[w];
    n2_part[(int64_t)lane * n2_slots + n2_slot0 + blockIdx.x] = bad ? __builtin_nan("") : tot;
  }
}

static int generic_prep_blocks(const Layout& L, bool half) {
  return (int)(((half ? L.hpack : L.pack) + kPrepSpan - 1) / kPrepSpan);
}
static int transpose_prep_tiles(const Layout& L, bool half) {
  const Section* sec = half ? L.hsec : L.sec;
  const int nsec = half ? L.n_hsections : L.n_sections;
  int n = 0;
  for (int i = 0; i < nsec; ++i)
    if (sec[i].kind == kTranspose) n += transpose_tiles(sec[i]);
  return n;
}

// theta' pack (half = 0, f32, with the per-lane n2 partials) or half pack (half = 1, f16).  The transposed sections
// (fc W^T, [W_ih | W_hh]^T: 90 % of the pack) by tmode: kTrFull written; kTrNorm not written, n2 partials only (an
// fp16 call's f32 pack: its kernels read those weights from the half pack or the pair images); kTrSkip nothing
// (an fp16 call's f32 pack when n2 is not wanted, or its half pack under the pair core).  copies = false (half packs
// only: no n2): the other sections are not written either -- the pairs' sigma-eps packs that feed only the MFMA images
enum TransposedMode { kTrFull = 0, kTrNorm = 1, kTrSkip = 2 };
template <class OUT>
static void launch_pack(const Layout& L, const LanesArgs& lanes, OUT* pack, double* n2, int n_lanes, int half,
                        hipStream_t stream, TransposedMode tmode = kTrFull, bool copies = true) {
  const int g = generic_prep_blocks(L, half != 0), tt = tmode == kTrSkip ? 0 : transpose_prep_tiles(L, half != 0);
  const int slots = prep_blocks(L);
  if (copies || !half)
    hipLaunchKernelGGL(prep_kernel<OUT>, dim3(g, n_lanes), dim3(kPrepThreads), 0, stream, L, lanes, pack, n2, half,
                       slots);
  if (tt > 0)
    hipLaunchKernelGGL(prep_transpose_kernel<OUT>, dim3(tt, n_lanes), dim3(256), 0, stream, L, lanes, pack, n2, half,
                       generic_prep_blocks(L, false), slots, tmode == kTrFull ? 1 : 0);
}

// ------------------------------------------------------------------------------------------
// conv stack: one workgroup (8 waves) per (lane, env); everything between the frame and the
// 2048-feature stays in LDS (all 160 KiB; floats):
//   [guard 128][TE 23,488: padded input image T of the current conv + band scratch S][X 16,384]
//   [BN scale/shift 960]
// Padded planes are strided so the 4 lane groups of an MFMA A-read (4 input channels) start 16
// banks apart: plane % 64 == 16 (32x32 and 16x16 stages) -> conflict-free ds_read_b32.
// ------------------------------------------------------------------------------------------
constexpr int kConvThreads = 512;
constexpr int kGuard = 128;          // padded rows above T: the band of conv row -1 reads them
constexpr int kTE = 23488;
constexpr int kRX = 16 * 32 * 32;
constexpr int kConvLds = kGuard + kTE + kRX + 2 * kBnTab;  // 40,960 floats = 160 KiB
constexpr int kBand = 9;             // conv rows per entry-conv band: 4 pooled rows + 1 shared row

template <int H>
struct Plane {  // padded [H+2][H+2] image, bank-staggered plane stride
  static constexpr int WP = H + 2;
  static constexpr int RAW = WP * WP;
  static constexpr int P = H == 64 ? RAW : RAW + ((16 - RAW % 64) % 64 + 64) % 64 + (H == 8 ? 2 : 0);
};
static_assert(Plane<32>::P == 1168 && Plane<16>::P == 336 && Plane<8>::P == 146, "plane strides");

// Channel skew of a padded plane (words), for the strides = 16 (mod 32) banks.  ds_write_b32 banks are
// (a/4) mod 32 over 32-lane halves: an epilogue store of one M-tile (lanes: 16 channels x 2 pixel
// quads) then hits 4 banks in 32 without the skew, an 8-way conflict (r05 PMC: SQ_LDS_BANK_CONFLICT
// 15 % of the conv kernel's cycles).  With bits (c>>1)&1 -> 8 and (c>>2)&3 -> 0..3 the 32 lanes land on 32
// banks.  An MFMA A-read takes channels 4q + g (g = lane >> 4): its skew (g>>1) 8 + (q & 3) is uniform
// per 32-lane half, so the reads stay conflict-free.
template <int PLANE>
__device__ __forceinline__ constexpr int cskew(int c) {
  return PLANE % 32 == 16 ? ((c >> 1) & 1) * 8 + ((c >> 2) & 3) : 0;
}
constexpr int kSkewPad = 16;  // room for the last plane's skew (<= 11) before the next region

// X [C][H][H] with a per-channel XOR on bits 2-5 of the pixel index (HH >= 64): the residual read-modify-
// write of an epilogue (lane: channel n, 4 pixels) goes from 16 channels on one 4-bank group to 16
// distinct groups (ds_read_b128 / ds_write_b128 conflict-free); pool writes and the float4 reads of
// to_padded stay contiguous.
template <int HH>
__device__ __forceinline__ int xpos(int c, int m) {
  static_assert(HH >= 64, "swizzle spans 64 pixels");
  return c * HH + (m ^ ((c & 15) << 2));
}

static_assert(16 * Plane<32>::P + kSkewPad <= kTE && 3 * Plane<64>::P + 16 * kBand * 65 <= kTE, "LDS plan");
static_assert(16 * Plane<32>::P + kSkewPad + 32 * kBand * 33 + 32 * 16 * 16 <= kTE + kRX, "LDS plan, stage 2");
static_assert(32 * Plane<16>::P + kSkewPad + 32 * 17 * 17 + 32 * 8 * 8 <= kTE + kRX, "LDS plan, stage 3");


// B fragments of one conv for this wave's N-tile: bf[s] = B[k = 4s + (lane >> 4)][n], one VGPR each.
template <int CIN, int NT>
__device__ __forceinline__ void load_frag(const float* __restrict__ wf, float (&bf)[(9 * CIN + 3) / 4], int wave,
                                          int lane) {
  constexpr int KS = (9 * CIN + 3) / 4;
  const int nt = wave % NT;
#pragma unroll
  for (int s = 0; s < KS; ++s) bf[s] = wf[(s * NT + nt) * 64 + lane];
}

// acc[i] (tile q = wave + 8 i) = A_tile(q) * B over K = 9 * CIN on v_mfma_f32_16x16x4_f32, A gathered
// from the padded LDS image Tin ([CIN][*][WP] with plane stride PLANE, row 0 = padded row of output
// row 0).  M-tile = 16 consecutive output pixels (row-major, width W).
template <int CIN, int NT, int TPW, int W, int WP, int PLANE, int MT>
__device__ __forceinline__ void conv_mfma(const float* Tin, const float (&bf)[(9 * CIN + 3) / 4], f32x4 (&acc)[TPW],
                                          int wave, int lane) {
  constexpr int KS = (9 * CIN + 3) / 4;
  int base[TPW];
  const int g = lane >> 4;
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    int mt = (wave + 8 * i) / NT;
    mt = mt < MT ? mt : MT - 1;
    const int m = mt * 16 + (lane & 15);
    base[i] = (m / W) * WP + (m % W);
    acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  }
  if constexpr ((CIN & 3) == 0) {
#pragma unroll
    for (int i = 0; i < TPW; ++i) base[i] += g * PLANE + cskew<PLANE>(g);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int tap = s / (CIN / 4), q = s % (CIN / 4);
      const int off = 4 * q * PLANE + cskew<PLANE>(4 * q) + (tap / 3) * WP + (tap % 3);
#pragma unroll
      for (int i = 0; i < TPW; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(Tin[base[i] + off], bf[s], acc[i], 0, 0, 0);
    }
  } else {
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int k = 4 * s + g;
      const int tap = k / CIN, ci = k - tap * CIN;
      const int off = k < 9 * CIN ? ci * PLANE + cskew<PLANE>(ci) + (tap / 3) * WP + (tap % 3) : 0;  // pad k: weight 0
#pragma unroll
      for (int i = 0; i < TPW; ++i)
        acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(Tin[base[i] + off], bf[s], acc[i], 0, 0, 0);
    }
  }
}

// Visit the outputs of conv_mfma: f(n, m, v) for channel n, output pixel m (row-major, width W).
template <int NT, int TPW, int MT, typename F>
__device__ __forceinline__ void conv_out(const f32x4 (&acc)[TPW], int wave, int lane, F f) {
  const int n = (wave % NT) * 16 + (lane & 15);
#pragma unroll
  for (int i = 0; i < TPW; ++i) {
    const int q = wave + 8 * i;
    if (q / NT >= MT) continue;
    const int m0 = (q / NT) * 16 + (lane >> 4) * 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) f(n, m0 + r, acc[i][r]);
  }
}

// T <- BN(X) (optionally ReLU) into the padded image [C][H+2][H+2] (plane stride Plane<H>::P).
// BORDER: also write the zero border (needed when T last held another layout).
template <int C, int H, bool RELU, bool BORDER>
__device__ __forceinline__ void to_padded(const float* X, float* T, const float* sc, const float* sh) {
  constexpr int WP = Plane<H>::WP, PL = Plane<H>::P, LH = H == 64 ? 6 : (H == 32 ? 5 : (H == 16 ? 4 : 3));
  // interior, 4 consecutive x per thread (one ds_read_b128 of X)
  for (int i = threadIdx.x; i < C * H * H / 4; i += kConvThreads) {
    const int e = 4 * i, ch = e >> (2 * LH), y = (e >> LH) & (H - 1), x = e & (H - 1);
    const float4 v = *reinterpret_cast<const float4*>(X + xpos<H * H>(ch, e & (H * H - 1)));
    const float a = sc[ch], b = sh[ch];
    float o0 = fmaf(v.x, a, b), o1 = fmaf(v.y, a, b), o2 = fmaf(v.z, a, b), o3 = fmaf(v.w, a, b);
    if (RELU) { o0 = relu(o0); o1 = relu(o1); o2 = relu(o2); o3 = relu(o3); }
    float* d = T + ch * PL + cskew<PL>(ch) + (y + 1) * WP + x + 1;
    d[0] = o0; d[1] = o1; d[2] = o2; d[3] = o3;
  }
  if (BORDER) {  // 4 (H + 1) border cells per plane
    for (int i = threadIdx.x; i < C * 4 * (H + 1); i += kConvThreads) {
      const int ch = i / (4 * (H + 1)), r = i - ch * 4 * (H + 1), side = r / (H + 1), k = r - side * (H + 1);
      const int off = side == 0 ? k : side == 1 ? (H + 1) * WP + 1 + k : side == 2 ? (k + 1) * WP : k * WP + WP - 1;
      T[ch * PL + cskew<PL>(ch) + off] = 0.f;
    }
  }
}

// Stage entry: X <- maxpool3s2p1(conv3x3(T) + b) in bands of BR-1 new conv rows (8 b .. 8 b + 7 for
// BR = 9) through the scratch S [COUT][BR][1 + H], a RING of conv rows: conv row g lives in slot
// (g + 1) mod BR, so a band's pool window (rows 8 b - 1 .. 8 b + 7) is the previous band's last row
// plus the new ones -- no row is computed twice and every band is (BR-1) H / 16 tiles (a multiple
// of the 8 waves).  Column -1 of S is -inf (the pool's left pad) and conv row -1 (slot 0 before
// band 0) is -inf, so the pool is branch-free and separable -- one thread per (channel, pooled
// column): BR horizontal max3, then vertical max3.  The B fragments are loaded by the caller and
// reused by every band.
template <int CIN, int COUT, int H, int PLANE, int BR>
__device__ __forceinline__ void stage_entry(const float* T, float* S, float* X, const float (&bf)[(9 * CIN + 3) / 4],
                                            const float* __restrict__ bias, int wave, int lane, const StepArgs& a,
                                            int kst) {
  constexpr int WP = H + 2, NT = COUT / 16, NR = BR - 1, MT = NR * H / 16, PRB = NR / 2;
  constexpr int TPW = (MT * NT + 7) / 8, HO = H / 2, SW = H + 1;
  static_assert((NR * H) % 16 == 0 && H % NR == 0 && NR % 2 == 0, "band shape");
  const float bn_ = bias[(wave % NT) * 16 + (lane & 15)];
  uint64_t t_conv = 0, t_pool = 0, t0 = a.dbg ? clock64() : 0;  // diagnostics (fdr_impala_debug_clock)
  // H = 64: a scratch row holds the even columns, the pad (column -1), then the odd columns, so the pool's
  // reads of columns 2px-1, 2px, 2px+1 are unit-stride across the 32 lanes of one channel (interleaved: stride
  // 2, 2-way conflicts; stage-1 pool 10.2 K -> 7.5 K clocks).  H <= 32: the pad first, then columns in order --
  // a 32-lane half spans 2+ channels whose odd channel stride puts them on the other bank parity.
  constexpr bool DI = HO >= 32;
  constexpr int PAD = DI ? HO : 0;
  auto col = [](int x) { return DI ? ((x & 1) ? HO + 1 + (x >> 1) : (x >> 1)) : 1 + x; };
  for (int i = threadIdx.x; i < COUT * BR; i += kConvThreads) S[i * SW + PAD] = -FLT_MAX;  // pad column
  for (int i = threadIdx.x; i < COUT * H; i += kConvThreads)                              // conv row -1
    S[(i / H) * BR * SW + col(i % H)] = -FLT_MAX;
  for (int b = 0; b < H / NR; ++b) {
    const int rot = (NR * b) % BR;  // slot of conv row NR b - 1
    auto slot = [&](int r) { return rot + r >= BR ? rot + r - BR : rot + r; };  // conv row NR b - 1 + r
    f32x4 acc[TPW];
    conv_mfma<CIN, NT, TPW, H, WP, PLANE, MT>(T + NR * b * WP, bf, acc, wave, lane);
    conv_out<NT, TPW, MT>(acc, wave, lane, [&](int n, int m, float v) {
      const int r = m / H, x = m % H;
      S[(n * BR + slot(r + 1)) * SW + col(x)] = v + bn_;
    });
    __syncthreads();
    if (a.dbg) {
      const uint64_t t1 = clock64();
      t_conv += t1 - t0;
      t0 = t1;
    }
    for (int i = threadIdx.x; i < COUT * HO; i += kConvThreads) {
      const int ch = i / HO, px = i - ch * HO;
      // columns 2px-1, 2px, 2px+1
      const float* sc = S + ch * BR * SW + (DI ? px : 2 * px);
      constexpr int c0 = DI ? HO : 0, c1 = DI ? 0 : 1, c2 = DI ? HO + 1 : 2;
      float hm[BR];
#pragma unroll
      for (int r = 0; r < BR; ++r) {  // conv row NR b - 1 + r
        const int sl = slot(r);
        hm[r] = fmaxf(fmaxf(sc[sl * SW + c0], sc[sl * SW + c1]), sc[sl * SW + c2]);
      }
#pragma unroll
      for (int pr = 0; pr < PRB; ++pr)
        X[xpos<HO * HO>(ch, (PRB * b + pr) * HO + px)] = fmaxf(fmaxf(hm[2 * pr], hm[2 * pr + 1]), hm[2 * pr + 2]);
    }
    __syncthreads();
    if (a.dbg) {
      const uint64_t t1 = clock64();
      t_pool += t1 - t0;
      t0 = t1;
    }
  }
  if (a.dbg && blockIdx.x == 0 && threadIdx.x == 0) {  // summed over the bands
    a.dbg[kst] = t_conv;
    a.dbg[kst + 1] = t_pool;
  }
}

// Two residual blocks (policies/impala.py:77-105, 152-157) on X [C][H][H], T [C][H+2][H+2] as the conv
// input.  On entry T must hold relu(bn0(X)) of block 0 with a zero border, and bf the B fragments of
// block 0's first conv.  Every BN (+ReLU) that follows a conv is fused into that conv's epilogue:
//   block 0 conv1 epilogue: X <- X + conv + b; T <- relu(bn0_block1(X))
//   block 1 conv1 epilogue: LAST == 0: T <- bn_entry(stage+1)(X + conv + b)  (the next stage's input,
//                           same padded geometry); LAST == 1: out <- relu(X + conv + b) (the features)
// Weights of the next conv are fetched right after the MFMAs that last read bf, ahead of the barrier.
template <int C, int H, int LAST>
__device__ __forceinline__ void res_blocks(float* T, float* X, float (&bf)[(9 * C + 3) / 4], const float* __restrict__ pk,
                                           const Layout& L, int stage, const float* bsc, const float* bsh, int wave,
                                           int lane, const StepArgs& a, int k0, float* __restrict__ out) {
  constexpr int WP = H + 2, PLANE = Plane<H>::P, NT = C / 16, MT = H * H / 16;
  constexpr int TPW = (MT * NT + 7) / 8;
  const int n_ = (wave % NT) * 16 + (lane & 15);
  auto tpos = [&](int n, int m) { return n * PLANE + cskew<PLANE>(n) + (m / H + 1) * WP + (m % H) + 1; };
#pragma unroll
  for (int r = 0; r < 2; ++r) {
    const int i0 = stage * 5 + 1 + 2 * r, i1 = i0 + 1;
    FDR_STAMP(a, k0 + 4 * r);
    f32x4 acc[TPW];
    conv_mfma<C, NT, TPW, H, WP, PLANE, MT>(T, bf, acc, wave, lane);
    const float b0 = pk[L.conv_b[i0] + n_], s1 = bsc[i1 * 32 + n_], h1 = bsh[i1 * 32 + n_];
    load_frag<C, NT>(pk + L.conv_w[i1], bf, wave, lane);
    __syncthreads();  // every wave is done reading T
    FDR_STAMP(a, k0 + 4 * r + 1);
    conv_out<NT, TPW, MT>(acc, wave, lane, [&](int n, int m, float v) { T[tpos(n, m)] = relu(fmaf(v + b0, s1, h1)); });
    __syncthreads();
    FDR_STAMP(a, k0 + 4 * r + 2);
    conv_mfma<C, NT, TPW, H, WP, PLANE, MT>(T, bf, acc, wave, lane);
    const float b1 = pk[L.conv_b[i1] + n_];
    // BN that consumes this block's output: block 1's bn0, or the next stage's entry BN
    const int inext = r == 0 ? i1 + 1 : (stage + 1) * 5;
    const float s2 = (r == 1 && LAST) ? 0.f : bsc[inext * 32 + n_];
    const float h2 = (r == 1 && LAST) ? 0.f : bsh[inext * 32 + n_];
    __syncthreads();  // every wave is done reading T
    FDR_STAMP(a, k0 + 4 * r + 3);
    if (r == 0) {
      // two passes over the accumulators (X update, then T) keep the live set small
#pragma unroll
      for (int i = 0; i < TPW; ++i) {
        const int q = wave + 8 * i;
        if (q / NT >= MT) continue;
        const int m0 = (q / NT) * 16 + (lane >> 4) * 4;
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int xp = xpos<H * H>(n_, m0) + rr;  // the swizzle keeps the 4 pixels contiguous
          const float xn = (acc[i][rr] + b1) + X[xp];
          X[xp] = xn;
          acc[i][rr] = xn;
        }
      }
      conv_out<NT, TPW, MT>(acc, wave, lane, [&](int n, int m, float v) { T[tpos(n, m)] = relu(fmaf(v, s2, h2)); });
      load_frag<C, NT>(pk + L.conv_w[i1 + 1], bf, wave, lane);  // block 1's first conv
    } else if (!LAST) {
      conv_out<NT, TPW, MT>(acc, wave, lane, [&](int n, int m, float v) {
        T[tpos(n, m)] = fmaf((v + b1) + X[xpos<H * H>(n, m)], s2, h2);
      });
    } else {
      conv_out<NT, TPW, MT>(acc, wave, lane, [&](int n, int m, float v) {
        out[n * H * H + m] = relu((v + b1) + X[xpos<H * H>(n, m)]);   // flatten (C, H, W), impala.py:159-160
      });
    }
    __syncthreads();
  }
}

__global__ __launch_bounds__(kConvThreads) void conv_kernel(Layout L, StepArgs a) {
  __shared__ float lds[kConvLds];
  // XCD-aware: the E workgroups of one lane run on one XCD, back to back (shared weights in L2)
  const int b = blockIdx.x, xcd = b & 7, slot = b >> 3;
  const int lane = (slot / a.envs) * 8 + xcd, e = slot % a.envs;
  if (lane >= a.n_lanes) return;
  const int wave = threadIdx.x >> 6, ln = threadIdx.x & 63;
  const int64_t env = (int64_t)lane * a.envs + e;
  const float* pk = a.pack + (int64_t)lane * a.pack_stride;
  float* T = lds + kGuard;
  float* X = T + kTE;
  float* bsc = X + kRX;
  float* bsh = bsc + kBnTab;
  constexpr int FW = 66, FPLANE = Plane<64>::P;

  float bf3[7];
  load_frag<3, 1>(pk + L.conv_w[0], bf3, wave, ln);
  FDR_STAMP(a, 0);
  // eval-mode BN folded per channel: y = x * (w / sqrt(rv + eps)) + (b - rm * scale).  Branch-free (r11, as
  // conv_kernel_h2's table): every load unconditional from a valid address, the unused values selected away after,
  // the layout offsets as scalar loads of the wave's two table rows -- a conditional load ends its basic block
  // with a full vmcnt wait, and the per-lane offset reads were a dependent round trip of their own
  static_assert(kBnTab <= kConvThreads, "one table entry per thread");
  {
    const int i = threadIdx.x, idx = i >> 5, ch = i & 31;
    const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), hi = (threadIdx.x >> 5) & 1;
    const int r0 = min(2 * wv, kConvs - 1), r1 = min(2 * wv + 1, kConvs - 1);  // wave-uniform rows
    auto pick = [&](const int32_t* arr) { return hi ? arr[r1] : arr[r0]; };
    const float* bmp = a.bn_mean ? a.bn_mean : pk;
    const float* bvp = a.bn_var ? a.bn_var : pk;
    const int so = pick(L.bn_stat) + ch;
    const float rm_ = bmp[so], rv_ = bvp[so], w_ = pk[pick(L.bn_w) + ch], b_ = pk[pick(L.bn_b) + ch];
    const int nch = idx == 0 ? 3 : (idx == 5 ? 16 : (idx < 5 ? 16 : 32));
    const bool live = i < kBnTab && ch < nch;
    const float rm = a.bn_mean ? rm_ : 0.f, rv = a.bn_var ? rv_ : 1.f;
    const float inv = 1.f / sqrtf(rv + kBnEps);
    const float sc = live ? w_ * inv : 0.f;
    const float sh = live ? b_ - rm * sc : 0.f;
    if (i < kBnTab) {
      bsc[i] = sc;
      bsh[i] = sh;
    }
  }
  for (int i = threadIdx.x; i < kGuard + 3 * FPLANE; i += kConvThreads) lds[i] = 0.f;
  __syncthreads();
  FDR_STAMP(a, 1);

  // ---- frame (policies/impala.py:147: frame / 255) -> BN2d(3) -> padded [3][66][66] ----
  if (a.frames) {
    const float* fr = a.frames + (a.shared_frames ? (int64_t)e : env) * kFramePix;
    for (int p = threadIdx.x; p < kFramePix; p += kConvThreads) {
      const int ch = p >> 12, y = (p >> 6) & 63, x = p & 63;
      T[ch * FPLANE + (y + 1) * FW + x + 1] = fmaf(fr[p] / 255.0f, bsc[ch], bsh[ch]);
    }
  } else {
    const uint64_t gid = (uint64_t)(a.lane_offset * a.envs + env);
    for (int w = threadIdx.x; w < kFramePix / 8; w += kConvThreads) {
      const uint64_t ctr = (gid << 32) | ((uint64_t)a.t << 11) | (uint64_t)w;
      const uint64_t hb = mix64(a.fkey + ctr * kGolden);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int p = 8 * w + j, ch = p >> 12, y = (p >> 6) & 63, x = p & 63;
        const float v = (float)((uint32_t)(hb >> (8 * j)) & 255u);
        T[ch * FPLANE + (y + 1) * FW + x + 1] = fmaf(v / 255.0f, bsc[ch], bsh[ch]);
      }
    }
  }
  __syncthreads();
  FDR_STAMP(a, 2);

  // ---- stage 1: conv 3->16 @64x64, pool -> X1 [16][32][32], residual blocks ----
  stage_entry<3, 16, 64, FPLANE, kBand>(T, T + 3 * FPLANE, X, bf3, pk + L.conv_b[0], wave, ln, a, 40);
  {
    float bf[36];
    load_frag<16, 1>(pk + L.conv_w[1], bf, wave, ln);
    to_padded<16, 32, true, true>(X, T, bsc + 1 * 32, bsh + 1 * 32);
    __syncthreads();
    FDR_STAMP(a, 3);
    res_blocks<16, 32, 0>(T, X, bf, pk, L, 0, bsc, bsh, wave, ln, a, 4, nullptr);  // ends with T = BN5(X1)
  }
  // ---- stage 2: conv 16->32 @32x32 (S2 after T, over the dead X1), pool -> X2 [32][16][16] ----
  float* X2 = T + 16 * Plane<32>::P + kSkewPad + 32 * kBand * 33;
  {
    float bf[36];
    load_frag<16, 2>(pk + L.conv_w[5], bf, wave, ln);
    FDR_STAMP(a, 12);
    stage_entry<16, 32, 32, Plane<32>::P, kBand>(T, T + 16 * Plane<32>::P + kSkewPad, X2, bf, pk + L.conv_b[5], wave, ln, a, 48);
  }
  {
    float bf[72];
    load_frag<32, 2>(pk + L.conv_w[6], bf, wave, ln);
    to_padded<32, 16, true, true>(X2, T, bsc + 6 * 32, bsh + 6 * 32);
    __syncthreads();
    FDR_STAMP(a, 13);
    res_blocks<32, 16, 0>(T, X2, bf, pk, L, 1, bsc, bsh, wave, ln, a, 14, nullptr);  // ends with T = BN10(X2)
  }
  // ---- stage 3: conv 32->32 @16x16 in one 17-row band, pool -> X3 [32][8][8] ----
  float* X3 = T + 32 * Plane<16>::P + kSkewPad + 32 * 17 * 17;
  {
    float bf[72];
    load_frag<32, 2>(pk + L.conv_w[10], bf, wave, ln);
    FDR_STAMP(a, 22);
    stage_entry<32, 32, 16, Plane<16>::P, 17>(T, T + 32 * Plane<16>::P + kSkewPad, X3, bf, pk + L.conv_b[10], wave, ln, a, 56);
  }
  {
    float bf[72];
    load_frag<32, 2>(pk + L.conv_w[11], bf, wave, ln);
    to_padded<32, 8, true, true>(X3, T, bsc + 11 * 32, bsh + 11 * 32);
    __syncthreads();
    FDR_STAMP(a, 23);
    // ---- relu + flatten (C, H, W) fused into the last epilogue (policies/impala.py:159-160) ----
    res_blocks<32, 8, 1>(T, X3, bf, pk, L, 2, bsc, bsh, wave, ln, a, 24, a.feat + env * kFeat);
  }
  FDR_STAMP(a, 32);
}

// ------------------------------------------------------------------------------------------
// core: one workgroup (256 threads) per lane, E envs.  Thread j owns fc unit j and LSTM unit j
// (gate rows j, 256+j, 512+j, 768+j), so the cell update is thread-local; weights stream from the
// pack as coalesced rows of W^T, activations are LDS broadcasts.
// ------------------------------------------------------------------------------------------


template <int E, int MODE>
__global__ __launch_bounds__(kCoreThreads) void core_kernel(Layout L, StepArgs a) {
  // xw: the BN'd features xs [2048][E] during the fc, then the fc partial sums [4][256][E] (first
  // half), then the LSTM gate pre-activations [1024][E] (first half) -- each phase separated by a
  // barrier.  The core input, h and the logits live in xw's second half once the features are dead:
  // 32 KiB per workgroup, so 5 lanes fit a CU and 1024 lanes run in one round (at 41 KiB only 3 did).
  __shared__ float xw[kFeat * E];
  float* cis = xw + kFeat * E / 2;   // core input, [k][e]
  float* hs = cis + kCoreIn * E;     // h (then BN(h')), [k][e]
  float* logit = hs + kHid * E;      // [e][kMaxAct]
  static_assert(kFeat * E / 2 + (kCoreIn + kHid) * E + E * kMaxAct <= kFeat * E, "core LDS aliasing");
  const int lane = blockIdx.x, j = threadIdx.x;
  const float* pk = a.pack + (int64_t)lane * a.pack_stride;
  const int64_t e0 = (int64_t)lane * E;
  const int A = a.n_act;
  const int c4 = j & 63, wq = j >> 6;  // float4 column group, wave index

  if constexpr (!seq_mode(MODE)) {
    for (int k = j; k < kFeat; k += kCoreThreads) {
      const float rmv = (a.bn_mean ? a.bn_mean + L.bn_stat[15] : a.pack)[k];  // branch-free
      const float rvv = (a.bn_var ? a.bn_var + L.bn_stat[15] : a.pack)[k];
      const float rm = a.bn_mean ? rmv : 0.f, rv = a.bn_var ? rvv : 1.f;
      const float sc = pk[L.bn_w[15] + k] * (1.f / sqrtf(rv + kBnEps));
      const float sh = fmaf(-rm, sc, pk[L.bn_b[15] + k]);
#pragma unroll
      for (int e = 0; e < E; ++e) xw[k * E + e] = fmaf(a.feat[(e0 + e) * kFeat + k], sc, sh);
    }
    __syncthreads();
    // fc (2048 -> 256): wave wq streams rows [512 wq, 512 wq + 512) of W^T as float4 (1 KiB / wave-load)
    float acc[4][E];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) acc[c][e] = 0.f;
    const float4* w4 = reinterpret_cast<const float4*>(pk + L.fc_wt) + c4;
#pragma unroll FDR_CORE_UNROLL
    for (int k = wq * (kFeat / 4); k < (wq + 1) * (kFeat / 4); ++k) {
      const float4 w = ld_stream(w4 + (int64_t)k * (kHid / 4));
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float x = xw[k * E + e];
        acc[0][e] = fmaf(w.x, x, acc[0][e]);
        acc[1][e] = fmaf(w.y, x, acc[1][e]);
        acc[2][e] = fmaf(w.z, x, acc[2][e]);
        acc[3][e] = fmaf(w.w, x, acc[3][e]);
      }
    }
    __syncthreads();  // xs is dead
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) xw[(wq * kHid + 4 * c4 + c) * E + e] = acc[c][e];
    __syncthreads();
    const float bj = pk[L.fc_b + j];
#pragma unroll
    for (int e = 0; e < E; ++e) {
      const float y = ((xw[j * E + e] + xw[(kHid + j) * E + e]) + xw[(2 * kHid + j) * E + e]) + xw[(3 * kHid + j) * E + e];
      cis[j * E + e] = relu(y + bj);
    }
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

  // LSTM gates (torch order i, f, g, o): thread j streams columns 4j .. 4j+3 of [W_ih | W_hh]^T, so
  // wave wq computes gate wq; gates = (W_ih x + b_ih) + (W_hh h + b_hh)
  {
    float ax[4][E], ah[4][E];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) ax[c][e] = ah[c][e] = 0.f;
    const float4* wl = reinterpret_cast<const float4*>(pk + L.lstm_wt) + j;
    if (seq_mode(MODE) && a.gx) {  // x W_ih^T precomputed by lstm_xproj_kernel (same fma chain)
      const float4* g4 = reinterpret_cast<const float4*>(a.gx + ((int64_t)(a.t - a.gx_t0) * a.n_lanes * E + e0) * kGates);
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float4 g = ld_stream(g4 + (int64_t)e * (kGates / 4) + j);
        ax[0][e] = g.x;
        ax[1][e] = g.y;
        ax[2][e] = g.z;
        ax[3][e] = g.w;
      }
    } else {
#pragma unroll FDR_CORE_UNROLL
      for (int k = 0; k < kCoreIn; ++k) {
        const float4 w = ld_stream(wl + (int64_t)k * (kGates / 4));
#pragma unroll
        for (int e = 0; e < E; ++e) {
          const float x = cis[k * E + e];
          ax[0][e] = fmaf(w.x, x, ax[0][e]);
          ax[1][e] = fmaf(w.y, x, ax[1][e]);
          ax[2][e] = fmaf(w.z, x, ax[2][e]);
          ax[3][e] = fmaf(w.w, x, ax[3][e]);
        }
      }
    }
#pragma unroll FDR_CORE_UNROLL
    for (int k = 0; k < kHid; ++k) {
      const float4 w = ld_stream(wl + (int64_t)(kCoreIn + k) * (kGates / 4));
#pragma unroll
      for (int e = 0; e < E; ++e) {
        const float x = hs[k * E + e];
        ah[0][e] = fmaf(w.x, x, ah[0][e]);
        ah[1][e] = fmaf(w.y, x, ah[1][e]);
        ah[2][e] = fmaf(w.z, x, ah[2][e]);
        ah[3][e] = fmaf(w.w, x, ah[3][e]);
      }
    }
    const float4 bi = reinterpret_cast<const float4*>(pk + L.lstm_bih)[j];
    const float4 bh = reinterpret_cast<const float4*>(pk + L.lstm_bhh)[j];
    const float bif[4] = {bi.x, bi.y, bi.z, bi.w}, bhf[4] = {bh.x, bh.y, bh.z, bh.w};
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < E; ++e) xw[(4 * j + c) * E + e] = (ax[c][e] + bif[c]) + (ah[c][e] + bhf[c]);
  }
  __syncthreads();  // gates complete; all reads of the old h are done
  float hj[E];
#pragma unroll
  for (int e = 0; e < E; ++e) {
    const float gi = sigm(xw[j * E + e]);
    const float gf = sigm(xw[(kHid + j) * E + e]);
    const float gg = tanhf(xw[(2 * kHid + j) * E + e]);
    const float go = sigm(xw[(3 * kHid + j) * E + e]);
    cj[e] = fmaf(gf, cj[e], gi * gg);  // explicit: the same rounding in every core form
    hj[e] = go * tanhf(cj[e]);
    a.h[(e0 + e) * kHid + j] = hj[e];
    a.c[(e0 + e) * kHid + j] = cj[e];
  }
  {
    const float rmv = (a.bn_mean ? a.bn_mean + L.bn_stat[16] : pk)[j];  // branch-free (see conv_kernel's table)
    const float rvv = (a.bn_var ? a.bn_var + L.bn_stat[16] : pk)[j];
    const float rm = a.bn_mean ? rmv : 0.f, rv = a.bn_var ? rvv : 1.f;
    const float sc = pk[L.bn_w[16] + j] * (1.f / sqrtf(rv + kBnEps));
    const float sh = fmaf(-rm, sc, pk[L.bn_b[16] + j]);
#pragma unroll
    for (int e = 0; e < E; ++e) hs[j * E + e] = fmaf(hj[e], sc, sh);
  }
  __syncthreads();
  if (j < A * E) {  // policy head Linear(256 -> A) (policies/impala.py:122, 184)
    const int ai = j / E, e = j - ai * E;
    const float* w = pk + L.head_w + ai * kHid;
    float s = 0.f;
    for (int k = 0; k < kHid; ++k) s = fmaf(w[k], hs[k * E + e], s);
    logit[e * kMaxAct + ai] = s + pk[L.head_b + ai];
  }
  __syncthreads();
  if (j < E) core_finish<E, MODE>(a, logit, lane, j);
}

// ------------------------------------------------------------------------------------------
// Pair form of the f32 rollout core step (fdr_impala_desc.pairs).  Lanes 2p, 2p+1 of an antithetic pair
// share their table offset: their fc / LSTM weights are fl32(theta + s_l fl32(sigma eps)).  One workgroup
// per pair streams the pair's fl32(sigma eps) pack once from HBM and theta's pack (read by every workgroup:
// L2 / MALL) and forms w = fl32(theta + s_l E) in registers -- the per-lane pack's value bit for bit (an fma
// with s = +-1 rounds theta +- E once), so every env sees core_kernel's exact fma chains; half its HBM bytes.
// The pair's 2E envs are contiguous, biases / BN / head are each lane's own pack.
// ------------------------------------------------------------------------------------------
template <int E>
__global__ __launch_bounds__(kCoreThreads) void core_kernel_p(Layout L, StepArgs a) {
  constexpr int E2 = 2 * E;
  __shared__ float xw[kFeat * E2];
  float* cis = xw + kFeat * E2 / 2;
  float* hs = cis + kCoreIn * E2;
  float* logit = hs + kHid * E2;
  static_assert(kFeat * E2 / 2 + (kCoreIn + kHid) * E2 + E2 * kMaxAct <= kFeat * E2, "core LDS aliasing");
  const int pr = blockIdx.x, j = threadIdx.x;
  const int l0 = 2 * pr;
  const float* pk0 = a.pack + (int64_t)l0 * a.pack_stride;
  const float* pk1 = pk0 + a.pack_stride;
  // branch-free sign loads (a conditional load ends its block with a full vmcnt wait)
  const int8_t* sgp = a.sign ? a.sign + l0 : reinterpret_cast<const int8_t*>(pk0);
  const int8_t sg0v = sgp[0], sg1v = sgp[1];
  const float sg0 = a.sign ? (float)sg0v : 1.f, sg1 = a.sign ? (float)sg1v : 1.f;
  const float* ep = a.ep32 + (int64_t)pr * a.ep_stride;
  const int64_t e0 = (int64_t)l0 * E;
  const int A = a.n_act;
  const int c4 = j & 63, wq = j >> 6;
  auto pkof = [&](int e) { return e < E ? pk0 : pk1; };
  // one streamed float4 row: w = fl32(theta + s_l E) per lane, then each env's fma chain of core_kernel
  auto accum = [&](float (&acc)[4][E2], float4 t, float4 d, const float* x) {
    const float tp[4] = {fmaf(sg0, d.x, t.x), fmaf(sg0, d.y, t.y), fmaf(sg0, d.z, t.z), fmaf(sg0, d.w, t.w)};
    const float tm[4] = {fmaf(sg1, d.x, t.x), fmaf(sg1, d.y, t.y), fmaf(sg1, d.z, t.z), fmaf(sg1, d.w, t.w)};
#pragma unroll
    for (int e = 0; e < E2; ++e) {
      const float xv = x[e];
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c][e] = fmaf(e < E ? tp[c] : tm[c], xv, acc[c][e]);
    }
  };

  // branch-free BN1d loads (a conditional load ends its block with a full vmcnt wait; without running
  // statistics the loads read the pack and the values are replaced by 0 / 1) -- the same values
  const bool has_m = a.bn_mean != nullptr, has_v = a.bn_var != nullptr;
  const float* bmp = has_m ? a.bn_mean + L.bn_stat[15] : pk0;
  const float* bvp = has_v ? a.bn_var + L.bn_stat[15] : pk0;
#pragma unroll
  for (int it = 0; it < kFeat / kCoreThreads; ++it) {
    const int k = j + it * kCoreThreads;
    const float rmv = bmp[k], rvv = bvp[k];
    const float rm = has_m ? rmv : 0.f, rv = has_v ? rvv : 1.f;
#pragma unroll
    for (int hf = 0; hf < 2; ++hf) {
      const float* pk = hf ? pk1 : pk0;
      const float sc = pk[L.bn_w[15] + k] * (1.f / sqrtf(rv + kBnEps));
      const float sh = fmaf(-rm, sc, pk[L.bn_b[15] + k]);
#pragma unroll
      for (int e = 0; e < E; ++e) xw[k * E2 + hf * E + e] = fmaf(a.feat[(e0 + hf * E + e) * kFeat + k], sc, sh);
    }
  }
  __syncthreads();
  {
    float acc[4][E2];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < E2; ++e) acc[c][e] = 0.f;
    const float4* t4 = reinterpret_cast<const float4*>(a.th32 + L.fc_wt) + c4;
    const float4* d4 = reinterpret_cast<const float4*>(ep + L.fc_wt) + c4;
#pragma unroll FDR_CORE_UNROLL
    for (int k = wq * (kFeat / 4); k < (wq + 1) * (kFeat / 4); ++k)
      accum(acc, t4[(int64_t)k * (kHid / 4)], ld_stream(d4 + (int64_t)k * (kHid / 4)), xw + k * E2);
    __syncthreads();  // xs is dead
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < E2; ++e) xw[(wq * kHid + 4 * c4 + c) * E2 + e] = acc[c][e];
  }
  __syncthreads();
#pragma unroll
  for (int e = 0; e < E2; ++e) {
    const float y = ((xw[j * E2 + e] + xw[(kHid + j) * E2 + e]) + xw[(2 * kHid + j) * E2 + e]) +
                    xw[(3 * kHid + j) * E2 + e];
    cis[j * E2 + e] = relu(y + pkof(e)[L.fc_b + j]);
  }
  if (j < E2) cis[kHid * E2 + j] = fminf(fmaxf(a.rprev[e0 + j], -1.f), 1.f);
  if (a.ci) {
    __syncthreads();
    float* dst = a.ci + ((int64_t)a.t * a.n_lanes * E + e0) * kCoreIn;
    for (int i = j; i < kCoreIn * E2; i += kCoreThreads) {
      const int e = i / kCoreIn, k = i - e * kCoreIn;
      dst[i] = cis[k * E2 + e];
    }
  }
  float cj[E2];
#pragma unroll
  for (int e = 0; e < E2; ++e) {
    hs[j * E2 + e] = a.h[(e0 + e) * kHid + j];
    cj[e] = a.c[(e0 + e) * kHid + j];
  }
  __syncthreads();
  {
    float ax[4][E2], ah[4][E2];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < E2; ++e) ax[c][e] = ah[c][e] = 0.f;
    const float4* tl = reinterpret_cast<const float4*>(a.th32 + L.lstm_wt) + j;
    const float4* dl = reinterpret_cast<const float4*>(ep + L.lstm_wt) + j;
#pragma unroll FDR_CORE_UNROLL
    for (int k = 0; k < kCoreIn; ++k)
      accum(ax, tl[(int64_t)k * (kGates / 4)], ld_stream(dl + (int64_t)k * (kGates / 4)), cis + k * E2);
#pragma unroll FDR_CORE_UNROLL
    for (int k = 0; k < kHid; ++k)
      accum(ah, tl[(int64_t)(kCoreIn + k) * (kGates / 4)], ld_stream(dl + (int64_t)(kCoreIn + k) * (kGates / 4)),
            hs + k * E2);
    const float4 bi0 = reinterpret_cast<const float4*>(pk0 + L.lstm_bih)[j];
    const float4 bh0 = reinterpret_cast<const float4*>(pk0 + L.lstm_bhh)[j];
    const float4 bi1 = reinterpret_cast<const float4*>(pk1 + L.lstm_bih)[j];
    const float4 bh1 = reinterpret_cast<const float4*>(pk1 + L.lstm_bhh)[j];
    const float bif0[4] = {bi0.x, bi0.y, bi0.z, bi0.w}, bhf0[4] = {bh0.x, bh0.y, bh0.z, bh0.w};
    const float bif1[4] = {bi1.x, bi1.y, bi1.z, bi1.w}, bhf1[4] = {bh1.x, bh1.y, bh1.z, bh1.w};
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < E2; ++e)
        xw[(4 * j + c) * E2 + e] = (ax[c][e] + (e < E ? bif0[c] : bif1[c])) + (ah[c][e] + (e < E ? bhf0[c] : bhf1[c]));
  }
  __syncthreads();
  float hj[E2];
#pragma unroll
  for (int e = 0; e < E2; ++e) {
    const float gi = sigm(xw[j * E2 + e]);
    const float gf = sigm(xw[(kHid + j) * E2 + e]);
    const float gg = tanhf(xw[(2 * kHid + j) * E2 + e]);
    const float go = sigm(xw[(3 * kHid + j) * E2 + e]);
    cj[e] = fmaf(gf, cj[e], gi * gg);  // explicit: the same rounding in every core form
    hj[e] = go * tanhf(cj[e]);
    a.h[(e0 + e) * kHid + j] = hj[e];
    a.c[(e0 + e) * kHid + j] = cj[e];
  }
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    const float* pk = hf ? pk1 : pk0;
    const float rmv = (a.bn_mean ? a.bn_mean + L.bn_stat[16] : pk)[j];  // branch-free (see conv_kernel's table)
    const float rvv = (a.bn_var ? a.bn_var + L.bn_stat[16] : pk)[j];
    const float rm = a.bn_mean ? rmv : 0.f, rv = a.bn_var ? rvv : 1.f;
    const float sc = pk[L.bn_w[16] + j] * (1.f / sqrtf(rv + kBnEps));
    const float sh = fmaf(-rm, sc, pk[L.bn_b[16] + j]);
#pragma unroll
    for (int e = 0; e < E; ++e) hs[j * E2 + hf * E + e] = fmaf(hj[hf * E + e], sc, sh);
  }
  __syncthreads();
  if (j < A * E2) {
    const int ai = j / E2, e = j - ai * E2;
    const float* pk = pkof(e);
    const float* w = pk + L.head_w + ai * kHid;
    float s = 0.f;
    for (int k = 0; k < kHid; ++k) s = fmaf(w[k], hs[k * E2 + e], s);
    logit[e * kMaxAct + ai] = s + pk[L.head_b + ai];
  }
  __syncthreads();
  if (j < E2) core_finish<E, kRollout>(a, logit + (j >= E ? E * kMaxAct : 0), l0 + (j >= E ? 1 : 0), j % E);
}
// Replay (entropy pass) in the pair form: the x W_ih^T half of the gates comes precomputed per env
// (lstm_xproj_kernel, a.gx), the W_hh h half streams theta + s_l fl32(sigma eps) for the pair -- the same
// values and fma chains as core_kernel<E, kReplay> (bit-identical), half its W_hh bytes.
template <int E>
__global__ __launch_bounds__(kCoreThreads) void core_kernel_pr(Layout L, StepArgs a) {
  constexpr int E2 = 2 * E;
  __shared__ float xw[kGates * E2 + kHid * E2 + E2 * kMaxAct];
  float* hs = xw + kGates * E2;
  float* logit = hs + kHid * E2;
  const int pr = blockIdx.x, j = threadIdx.x;
  const int l0 = 2 * pr;
  const float* pk0 = a.pack + (int64_t)l0 * a.pack_stride;
  const float* pk1 = pk0 + a.pack_stride;
  const float sg0 = a.sign ? (float)a.sign[l0] : 1.f, sg1 = a.sign ? (float)a.sign[l0 + 1] : 1.f;
  const float* ep = a.ep32 + (int64_t)pr * a.ep_stride;
  const int64_t e0 = (int64_t)l0 * E;
  const int A = a.n_act;
  float cj[E2];
#pragma unroll
  for (int e = 0; e < E2; ++e) {
    hs[j * E2 + e] = a.h[(e0 + e) * kHid + j];
    cj[e] = a.c[(e0 + e) * kHid + j];
  }
  __syncthreads();
  {
    float ah[4][E2];
#pragma unroll
    for (int c = 0; c < 4; ++c)
#pragma unroll
      for (int e = 0; e < E2; ++e) ah[c][e] = 0.f;
    const float4* tl = reinterpret_cast<const float4*>(a.th32 + L.lstm_wt) + j;
    const float4* dl = reinterpret_cast<const float4*>(ep + L.lstm_wt) + j;
#pragma unroll FDR_CORE_UNROLL
    for (int k = 0; k < kHid; ++k) {
      const float4 t = tl[(int64_t)(kCoreIn + k) * (kGates / 4)];
      const float4 d = ld_stream(dl + (int64_t)(kCoreIn + k) * (kGates / 4));
      const float tp[4] = {fmaf(sg0, d.x, t.x), fmaf(sg0, d.y, t.y), fmaf(sg0, d.z, t.z), fmaf(sg0, d.w, t.w)};
      const float tm[4] = {fmaf(sg1, d.x, t.x), fmaf(sg1, d.y, t.y), fmaf(sg1, d.z, t.z), fmaf(sg1, d.w, t.w)};
#pragma unroll
      for (int e = 0; e < E2; ++e) {
        const float xv = hs[k * E2 + e];
#pragma unroll
        for (int c = 0; c < 4; ++c) ah[c][e] = fmaf(e < E ? tp[c] : tm[c], xv, ah[c][e]);
      }
    }
    const float4* g4 = reinterpret_cast<const float4*>(a.gx + ((int64_t)(a.t - a.gx_t0) * a.n_lanes * E + e0) * kGates);
    const float4 bi0 = reinterpret_cast<const float4*>(pk0 + L.lstm_bih)[j];
    const float4 bh0 = reinterpret_cast<const float4*>(pk0 + L.lstm_bhh)[j];
    const float4 bi1 = reinterpret_cast<const float4*>(pk1 + L.lstm_bih)[j];
    const float4 bh1 = reinterpret_cast<const float4*>(pk1 + L.lstm_bhh)[j];
    const float bif0[4] = {bi0.x, bi0.y, bi0.z, bi0.w}, bhf0[4] = {bh0.x, bh0.y, bh0.z, bh0.w};
    const float bif1[4] = {bi1.x, bi1.y, bi1.z, bi1.w}, bhf1[4] = {bh1.x, bh1.y, bh1.z, bh1.w};
#pragma unroll
    for (int e = 0; e < E2; ++e) {
      const float4 g = ld_stream(g4 + (int64_t)e * (kGates / 4) + j);
      const float gxv[4] = {g.x, g.y, g.z, g.w};
#pragma unroll
      for (int c = 0; c < 4; ++c)
        xw[(4 * j + c) * E2 + e] = (gxv[c] + (e < E ? bif0[c] : bif1[c])) + (ah[c][e] + (e < E ? bhf0[c] : bhf1[c]));
    }
  }
  __syncthreads();
  float hj[E2];
#pragma unroll
  for (int e = 0; e < E2; ++e) {
    const float gi = sigm(xw[j * E2 + e]);
    const float gf = sigm(xw[(kHid + j) * E2 + e]);
    const float gg = tanhf(xw[(2 * kHid + j) * E2 + e]);
    const float go = sigm(xw[(3 * kHid + j) * E2 + e]);
    cj[e] = fmaf(gf, cj[e], gi * gg);  // explicit: the same rounding in every core form
    hj[e] = go * tanhf(cj[e]);
    a.h[(e0 + e) * kHid + j] = hj[e];
    a.c[(e0 + e) * kHid + j] = cj[e];
  }
  __syncthreads();  // every read of hs is done before BN(h') overwrites it
#pragma unroll
  for (int hf = 0; hf < 2; ++hf) {
    const float* pk = hf ? pk1 : pk0;
    const float rmv = (a.bn_mean ? a.bn_mean + L.bn_stat[16] : pk)[j];  // branch-free (see conv_kernel's table)
    const float rvv = (a.bn_var ? a.bn_var + L.bn_stat[16] : pk)[j];
    const float rm = a.bn_mean ? rmv : 0.f, rv = a.bn_var ? rvv : 1.f;
    const float sc = pk[L.bn_w[16] + j] * (1.f / sqrtf(rv + kBnEps));
    const float sh = fmaf(-rm, sc, pk[L.bn_b[16] + j]);
#pragma unroll
    for (int e = 0; e < E; ++e) hs[j * E2 + hf * E + e] = fmaf(hj[hf * E + e], sc, sh);
  }
  __syncthreads();
  if (j < A * E2) {
    const int ai = j / E2, e = j - ai * E2;
    const float* pk = e < E ? pk0 : pk1;
    const float* w = pk + L.head_w + ai * kHid;
    float s = 0.f;
    for (int k = 0; k < kHid; ++k) s = fmaf(w[k], hs[k * E2 + e], s);
    logit[e * kMaxAct + ai] = s + pk[L.head_b + ai];
  }
  __syncthreads();
  if (j < E2) core_finish<E, kReplay>(a, logit + (j >= E ? E * kMaxAct : 0), l0 + (j >= E ? 1 : 0), j % E);
}
template __global__ void core_kernel_pr<1>(Layout, StepArgs);
template __global__ void core_kernel_pr<2>(Layout, StepArgs);
template __global__ void core_kernel_pr<4>(Layout, StepArgs);

template __global__ void core_kernel_p<1>(Layout, StepArgs);
template __global__ void core_kernel_p<2>(Layout, StepArgs);
template __global__ void core_kernel_p<4>(Layout, StepArgs);

__global__ void init_kernel(int64_t n_env, float* h, float* c, float* rprev, double* ret, double* ent) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (h && i < n_env * kHid) { h[i] = 0.f; c[i] = 0.f; }
  if (i < n_env) {
    if (rprev) rprev[i] = 0.f;
    ret[i] = 0.0;
    ent[i] = 0.0;
  }
}

// n2 partial slots per lane: the generic prep blocks, then the transpose tiles
int prep_blocks(const Layout& L) { return generic_prep_blocks(L, false) + transpose_prep_tiles(L, false); }

int launch_prep(const Layout& L, const LanesArgs& lanes, float* pack, double* n2_part, int n_lanes,
                hipStream_t stream) {
  launch_pack<float>(L, lanes, pack, n2_part, n_lanes, 0, stream);
  return check_launch("prep_kernel");
}

__global__ void finish_kernel(int n_lanes, int envs, int T, int entropy, int jiggle, uint64_t akey,
                              int64_t lane_offset, const double* n2_part, int nblk, double* ret,
                              double* ent, int32_t* steps, double* norm2) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < (int64_t)n_lanes * envs) {
    const uint64_t gid = (uint64_t)(lane_offset * envs + i);
    if (jiggle) ret[i] += (hash_ctr(akey, gid, kJiggleT, 15) & 1ull) ? 1e-12 : -1e-12;
    if (ent) ent[i] = entropy ? ent[i] / (double)T : 0.0;
    if (steps) steps[i] = T;
  }
  if (i < n_lanes && norm2) {
    double s = 0.0;
    for (int b = 0; b < nblk; ++b) s += n2_part[i * nblk + b];
    norm2[i] = s;
  }
}

// Opt-in phase timing (fdr_ctx_impala_profile): HIP events between the launches of the step loop, so
// a caller (bench.py) can attribute the rollout's time to conv / core / replay kernels live.  One
// Profile per context.
struct Profile {
  bool on = false;
  std::vector<hipEvent_t> ev;
  int used = 0, T = 0, entropy = 0;
  hipEvent_t next() {
    if (used == (int)ev.size()) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return nullptr;
      ev.push_back(e);
    }
    return ev[used++];
  }
};

void destroy_profile(Profile* p) {
  if (!p) return;
  for (hipEvent_t e : p->ev) (void)hipEventDestroy(e);
  delete p;
}

static void mark(Profile* p, hipStream_t s) {
  if (p && p->on) {
    hipEvent_t e = p->next();
    if (e) (void)hipEventRecord(e, s);
  }
}

int set_profile(Context& ctx, int on) {
  if (!ctx.prof) ctx.prof = new Profile();
  ctx.prof->on = on != 0;
  ctx.prof->used = 0;
  return FDR_OK;
}

int read_profile(Context& ctx, double* out) {
  out[0] = out[1] = out[2] = 0.0;
  Profile* p = ctx.prof;
  if (!p) return set_error(FDR_ERR_INVALID, "no profiled impala rollout");
  const int need = 2 * p->T + 1 + (p->entropy ? p->T : 0);
  if (!p->on || p->used < need) return set_error(FDR_ERR_INVALID, "no profiled impala rollout");
  if (hipEventSynchronize(p->ev[need - 1]) != hipSuccess) return set_error(FDR_ERR_HIP, "event sync failed");
  auto ms = [](hipEvent_t a, hipEvent_t b) { float v = 0.f; (void)hipEventElapsedTime(&v, a, b); return (double)v; };
  for (int t = 0; t < p->T; ++t) {
    out[0] += ms(p->ev[2 * t], p->ev[2 * t + 1]);
    out[1] += ms(p->ev[2 * t + 1], p->ev[2 * t + 2]);
  }
  for (int t = 0; p->entropy && t < p->T; ++t)
    out[2] += ms(p->ev[2 * p->T + t], p->ev[2 * p->T + t + 1]);
  return FDR_OK;
}

// ------------------------------------------------------------------------------------------
// Entropy replay, input projection.  The reference's get_entropy runs the stored core inputs through
// the LSTM as ONE sequence (policies/impala.py:21-22, 166-182); the x W_ih^T half of every step's gates
// does not depend on h, so -- as torch's LSTM does -- it is one GEMM per lane over a chunk of steps:
// G[(t, e)][n] = sum_k x_(t,e)[k] W_ih^T[k][n] on v_mfma_f32_16x16x4_f32.  An f32 MFMA is a k-ordered
// fma chain, so G is bit-identical to the k-loop the replay kernel ran, while W_ih is read once per
// 64 rows instead of once per step (the replay then streams W_hh only).  fp16 mode reads the f16
// W_ih^T (exact in f32), as its replay did.
// Workgroup: 64 rows x 256 gate columns, 4 waves x (4 x 4) 16x16 tiles; K in LDS chunks of 32.
// ------------------------------------------------------------------------------------------
template <bool HALF>
__global__ __launch_bounds__(256) void lstm_xproj_kernel(Layout L, StepArgs a, int t0, int tc, float* __restrict__ gx) {
  constexpr int KC = 32, NKC = (kCoreIn + KC - 1) / KC, XP = 80, WP = 256 + 16;  // pads: conflict-free reads
  __shared__ float xs[KC * XP];  // [k][row]
  __shared__ float ws[KC * WP];  // [k][col]
  const int lane = blockIdx.x, E = a.envs, rows = tc * E;
  const int row0 = blockIdx.y * 64, n0 = blockIdx.z * 256;
  const int tid = threadIdx.x, wave = tid >> 6, ln = tid & 63, g = ln >> 4, r = ln & 15;
  const int64_t ne = (int64_t)a.n_lanes * E;
  f32x4 acc[4][4];
#pragma unroll
  for (int ti = 0; ti < 4; ++ti)
#pragma unroll
    for (int tj = 0; tj < 4; ++tj) acc[ti][tj] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int kc = 0; kc < NKC; ++kc) {
    const int k0 = kc * KC;
#pragma unroll
    for (int m = 0; m < 8; ++m) {  // X tile: row-contiguous global reads (32 k of one row per half-wave)
      const int i = tid + 256 * m, row = i >> 5, k = i & 31;
      const int q = row0 + row;
      float v = 0.f;
      if (q < rows && k0 + k < kCoreIn) {
        const int64_t t = t0 + q / E, e = q % E;
        v = a.ci[((t * a.n_lanes + lane) * E + e) * kCoreIn + k0 + k];
      }
      xs[k * XP + row] = v;
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {  // W_ih^T tile [32 k][256 cols]
      const int i = tid + 256 * m, k = i >> 6, c4 = i & 63;
      float4 w = float4{0.f, 0.f, 0.f, 0.f};
      if (k0 + k < kCoreIn) {
        if constexpr (HALF) {
          typedef _Float16 h4v __attribute__((ext_vector_type(4)));
          const h4v hv = *reinterpret_cast<const h4v*>(a.hpack + (int64_t)lane * a.hpack_stride + L.lstm_wt_h +
                                                        (int64_t)(k0 + k) * kGates + n0 + 4 * c4);
          w = float4{(float)hv[0], (float)hv[1], (float)hv[2], (float)hv[3]};
        } else {
          w = *reinterpret_cast<const float4*>(a.pack + (int64_t)lane * a.pack_stride + L.lstm_wt +
                                               (int64_t)(k0 + k) * kGates + n0 + 4 * c4);
        }
      }
      *reinterpret_cast<float4*>(ws + k * WP + 4 * c4) = w;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < KC / 4; ++s) {
      const int k = 4 * s + g;
      float av[4], bv[4];
#pragma unroll
      for (int ti = 0; ti < 4; ++ti) av[ti] = xs[k * XP + 16 * ti + r];
#pragma unroll
      for (int tj = 0; tj < 4; ++tj) bv[tj] = ws[k * WP + 64 * wave + 16 * tj + r];
#pragma unroll
      for (int ti = 0; ti < 4; ++ti)
#pragma unroll
        for (int tj = 0; tj < 4; ++tj) acc[ti][tj] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ti], bv[tj], acc[ti][tj], 0, 0, 0);
    }
    __syncthreads();
  }
#pragma unroll
  for (int ti = 0; ti < 4; ++ti)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int q = row0 + 16 * ti + 4 * g + v;
      if (q >= rows) continue;
      float* dst = gx + ((int64_t)(q / E) * ne + (int64_t)lane * E + q % E) * kGates + n0 + 64 * wave + r;
#pragma unroll
      for (int tj = 0; tj < 4; ++tj) dst[16 * tj] = acc[ti][tj][v];
    }
}

// the pairs' table offsets idx[2p] (fdr_impala_desc.pairs: idx[2p] == idx[2p+1] by contract)
// idxe[p] = the pair's shared offset.  A pair whose lanes disagree (fdr_impala_desc.pairs violated) would run lane
// 2p + 1 on lane 2p's noise: both lanes' norms are poisoned with NaN instead (slot 0 of their n2 partials, written by
// the lanes' pack kernels before this launch), as for an out-of-range offset.
__global__ void pair_offsets_kernel(const int64_t* __restrict__ idx, int n_pairs, int64_t* __restrict__ idxe,
                                    double* __restrict__ n2, int nblk) {
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= n_pairs) return;
  const int64_t o0 = idx[2 * p], o1 = idx[2 * p + 1];
  idxe[p] = o0;
  if (o0 != o1) {
    n2[(int64_t)(2 * p) * nblk] = __builtin_nan("");
    n2[(int64_t)(2 * p + 1) * nblk] = __builtin_nan("");
  }
}

// the fp16 conv stack over grid workgroups (one per env, XCD-interleaved lanes)
static void launch_conv_h(int grid, const Layout& L, const StepArgs& a, hipStream_t stream) {
  hipLaunchKernelGGL((conv_kernel_h2<kHThreads>), dim3(grid), dim3(kHThreads), 0, stream, L, a);
}

template <int E>
static int launch_steps(const Context& ctx, const Layout& L, StepArgs a, int entropy, hipStream_t stream) {
  const int conv_grid = (a.n_lanes + 7) / 8 * 8 * a.envs;
  const bool h = a.hpack != nullptr;
  Profile* prof = ctx.prof;
  if (prof) {
    prof->used = 0;
    prof->T = a.T;
    prof->entropy = entropy;
  }
  mark(prof, stream);
  for (int t = 0; t < a.T; ++t) {
    a.t = t;
    if (h)
      launch_conv_h(conv_grid, L, a, stream);
    else
      hipLaunchKernelGGL(conv_kernel, dim3(conv_grid), dim3(kConvThreads), 0, stream, L, a);
    mark(prof, stream);
    bool pair_done = false;
    if constexpr (E <= 4) {
      if (h && a.epm) {  // (launch_rollout builds the images only for n_lanes % 4 == 0)
        hipLaunchKernelGGL((core_kernel_hpm2<E, kRollout>), dim3(a.n_lanes / 4), dim3(2 * kCoreThreads), 0, stream, L,
                           a);
        pair_done = true;
      } else if (!h && a.ep32) {
        hipLaunchKernelGGL((core_kernel_p<E>), dim3(a.n_lanes / 2), dim3(kCoreThreads), 0, stream, L, a);
        pair_done = true;
      }
    }
    if (pair_done) {
    } else if (h)
      hipLaunchKernelGGL((core_kernel_h<E, kRollout>), dim3(a.n_lanes), dim3(kCoreThreads), 0, stream, L, a);
    else
      hipLaunchKernelGGL((core_kernel<E, kRollout>), dim3(a.n_lanes), dim3(kCoreThreads), 0, stream, L, a);
    mark(prof, stream);
  }
  float* gx = const_cast<float*>(a.gx);
  a.gx = nullptr;
  if (entropy)
    for (int t0 = 0; t0 < a.T; t0 += kReplayChunk) {
      const int tc = std::min(kReplayChunk, a.T - t0);
      if (ctx.replay_gemm && gx) {
        const dim3 grid(a.n_lanes, (tc * E + 63) / 64, kGates / 256);
        bool pair_xproj = false;
        if constexpr (E <= 4) {
          if (h && a.epm) {  // fp16 pair form on MFMA: theta X + s (E X) from the gate images
            hipLaunchKernelGGL((xproj_pair_kernel<E, true>), xproj_grid(a.n_lanes), dim3(256), 0, stream, L, a,
                               t0, tc, gx);
            pair_xproj = true;
          }
        }
        if (pair_xproj) {
        } else if (h)
          hipLaunchKernelGGL(lstm_xproj_kernel<true>, grid, dim3(256), 0, stream, L, a, t0, tc, gx);
        else
          hipLaunchKernelGGL(lstm_xproj_kernel<false>, grid, dim3(256), 0, stream, L, a, t0, tc, gx);
        a.gx = gx;
        a.gx_t0 = t0;
      }
      if constexpr (E <= 4) {
        if (a.gx && h && a.epm) {  // the whole chunk in one launch
          hipLaunchKernelGGL((replay_chunk_hpm2<E, kReplay>), dim3(a.n_lanes / 4), dim3(2 * kCoreThreads), 0, stream, L,
                             a, t0, tc);
          for (int t = t0; t < t0 + tc; ++t) mark(prof, stream);  // the profiler's per-step marks
          continue;
        }
      }
      for (int t = t0; t < t0 + tc; ++t) {
        a.t = t;
        bool pair_done = false;
        if constexpr (E <= 4) {
          if (a.gx && !h && a.ep32) {
            hipLaunchKernelGGL((core_kernel_pr<E>), dim3(a.n_lanes / 2), dim3(kCoreThreads), 0, stream, L, a);
            pair_done = true;
          }
        }
        if (pair_done) {
        } else if (h)
          hipLaunchKernelGGL((core_kernel_h<E, kReplay>), dim3(a.n_lanes), dim3(kCoreThreads), 0, stream, L, a);
        else
          hipLaunchKernelGGL((core_kernel<E, kReplay>), dim3(a.n_lanes), dim3(kCoreThreads), 0, stream, L, a);
        mark(prof, stream);
      }
    }
  return check_launch("impala step kernels");
}

int launch_rollout(const RolloutCall& c, void* ws, int64_t ws_bytes, hipStream_t stream) {
  const Layout& L = *c.layout;
  const Plan p = plan(L, c.n_lanes, c.envs, c.T, c.entropy != 0, c.fp16 != 0, c.pairs != 0);
  if (!ws || ws_bytes < p.total) return set_error(FDR_ERR_WORKSPACE, "impala workspace too small");
  if (c.n_lanes == 0) return FDR_OK;
  char* w = static_cast<char*>(ws);
  StepArgs a{};
  a.pack = reinterpret_cast<float*>(w + p.pack);
  a.pack_stride = L.pack;
  a.bn_mean = c.bn_mean;
  a.bn_var = c.bn_var;
  a.n_lanes = c.n_lanes;
  a.envs = c.envs;
  a.n_act = L.n_act;
  a.T = c.T;
  a.lane_offset = c.lanes.lane_offset;
  a.fkey = mix64(c.env_seed ^ kFrameSalt);
  a.rkey = mix64(c.env_seed ^ kRewardSalt);
  a.akey = mix64(c.seed);
  a.feat = reinterpret_cast<float*>(w + p.feat);
  a.h = reinterpret_cast<float*>(w + p.h);
  a.c = reinterpret_cast<float*>(w + p.c);
  a.rprev = reinterpret_cast<float*>(w + p.rprev);
  a.ci = c.entropy ? reinterpret_cast<float*>(w + p.ci) : nullptr;
  a.gx = c.entropy ? reinterpret_cast<float*>(w + p.gx) : nullptr;  // launch_steps hands it to the replay
  a.ret = c.ret;
  a.ent = c.ent;
  a.actions = c.actions;
  a.probs = c.probs;
  a.deterministic = c.lanes.deterministic;
  a.dbg = c.ctx->debug_clock;
  double* n2 = reinterpret_cast<double*>(w + p.n2);

  // fp16: the MFMA pair core takes two pairs per workgroup (n_lanes % 4 == 0); other lane counts run per lane
  const bool pair_core = c.pairs && pair_core_supported(c.envs) && c.lanes.table && c.lanes.base_stride == 0 &&
                         c.n_lanes >= 2 && (!c.fp16 || c.n_lanes % 4 == 0);
  launch_pack<float>(L, c.lanes, const_cast<float*>(a.pack), n2, c.n_lanes, 0, stream, c.fp16 ? kTrNorm : kTrFull);
  if (c.fp16) {
    a.hpack = reinterpret_cast<_Float16*>(w + p.hpack);
    a.hpack_stride = L.hpack;
    // the per-lane half pack's fc / LSTM weights are read only off the MFMA pair path: core_kernel_h (no pair core),
    // lstm_xproj_kernel (pair core on VALU) and core_kernel_h<kReplay> (replay without the gate GEMM)
    const bool pair_images = pair_core && (!c.entropy || c.ctx->replay_gemm);
    launch_pack<_Float16>(L, c.lanes, a.hpack, n2, c.n_lanes, 1, stream, pair_images ? kTrSkip : kTrFull);
  }
  if (pair_core) {
    // the pair form's operands, built by the same pack kernels: theta's pack (no table: theta' = theta) and
    // per pair fl32(sigma eps) (a zero base, sign +1: fl32(0 + fl32(sigma eps))) -- f16 in fp16 mode
    const int np = c.n_lanes / 2;
    float* zeros = reinterpret_cast<float*>(w + p.zeros);
    int64_t* idxe = reinterpret_cast<int64_t*>(w + p.idxe);
    (void)hipMemsetAsync(zeros, 0, (size_t)L.P * 4, stream);
    hipLaunchKernelGGL(pair_offsets_kernel, dim3((np + 255) / 256), dim3(256), 0, stream, c.lanes.idx, np, idxe, n2,
                       p.nblk);
    LanesArgs lt = c.lanes;
    lt.table = nullptr;
    LanesArgs le = c.lanes;
    le.base = zeros;
    le.base_stride = 0;
    le.idx = idxe;
    le.sign = nullptr;
    if (c.fp16) {
      _Float16* th = reinterpret_cast<_Float16*>(w + p.thpack);
      _Float16* ep = reinterpret_cast<_Float16*>(w + p.epack);
      launch_pack<_Float16>(L, lt, th, n2, 1, 1, stream);
      // under the MFMA core only the images read the pairs' packs (their transposed sections)
      launch_pack<_Float16>(L, le, ep, n2, np, 1, stream, kTrFull, false);
      a.th = th;
      a.ep = ep;
      a.ep_stride = L.hpack;
      if (c.entropy && c.ctx->replay_gemm) {  // core inputs as f16 rows for xproj_pair_kernel<E, true> (the ci space)
        a.ci16 = reinterpret_cast<_Float16*>(a.ci);
        a.ci = nullptr;
      }
      {  // MFMA-fragment images of theta's and the pairs' fc / LSTM weights
        _Float16* im = reinterpret_cast<_Float16*>(w + p.mimg);
        const unsigned nb = kFcKS + 4 * kGateKS;
        hipLaunchKernelGGL(mfma_image_kernel, dim3(nb, 1), dim3(256), 0, stream, L, th, (int64_t)0, im);
        hipLaunchKernelGGL(mfma_image_kernel, dim3(nb, np), dim3(256), 0, stream, L, ep, (int64_t)L.hpack, im + kMImg);
        a.thm = im;
        a.epm = im + kMImg;
      }
    } else {  // f32: w = fl32(theta +- fl32(sigma eps)) in registers is the pack's value bit for bit
      float* th = reinterpret_cast<float*>(w + p.thpack);
      float* ep = reinterpret_cast<float*>(w + p.epack);
      double* n2x = reinterpret_cast<double*>(w + p.n2x);  // these packs' norms are not the lanes'
      launch_pack<float>(L, lt, th, n2x, 1, 0, stream);
      launch_pack<float>(L, le, ep, n2x + p.nblk, np, 0, stream);
      a.th32 = th;
      a.ep32 = ep;
      a.ep_stride = L.pack;
    }
    a.sign = c.lanes.sign;
  }
  if (c.fp16) {  // the lanes' BN / bias tables, folded once per rollout (r12: conv launch -1.4 %, same box)
    float* tab = reinterpret_cast<float*>(w + p.bntab);
    hipLaunchKernelGGL(bn_table_kernel, dim3(c.n_lanes), dim3(256), 0, stream, L, a, tab);
    a.bntab = tab;
  }
  const int64_t ne = (int64_t)c.n_lanes * c.envs;
  hipLaunchKernelGGL(init_kernel, dim3((unsigned)((ne * kHid + 255) / 256)), dim3(256), 0, stream, ne, a.h, a.c,
                     a.rprev, a.ret, a.ent);
  int rc = check_launch("impala prep/init");
  if (rc) return rc;
  switch (c.envs) {
    case 1: rc = launch_steps<1>(*c.ctx, L, a, c.entropy, stream); break;
    case 2: rc = launch_steps<2>(*c.ctx, L, a, c.entropy, stream); break;
    case 4: rc = launch_steps<4>(*c.ctx, L, a, c.entropy, stream); break;
    case 8: rc = launch_steps<8>(*c.ctx, L, a, c.entropy, stream); break;
    default: return set_error(FDR_ERR_UNSUPPORTED, "envs_per_lane must be 1, 2, 4 or 8");
  }
  if (rc) return rc;
  const int64_t nmax = std::max<int64_t>(ne, c.n_lanes);
  hipLaunchKernelGGL(finish_kernel, dim3((unsigned)((nmax + 255) / 256)), dim3(256), 0, stream, c.n_lanes, c.envs,
                     c.T, c.entropy, c.jiggle, a.akey, c.lanes.lane_offset, n2, p.nblk, c.ret, c.ent, c.steps,
                     c.norm2);
  return check_launch("impala finish");
}

int64_t forward_workspace_bytes(const Layout& L, int n_envs, bool fp16) {
  const Plan p = plan(L, 1, std::max(n_envs, 0), 0, false, fp16);
  return p.total;
}

int launch_forward(const ForwardCall& c, void* ws, int64_t ws_bytes, hipStream_t stream) {
  const Layout& L = *c.layout;
  const Plan p = plan(L, 1, c.n_envs, 0, false, c.fp16 != 0);
  if (!ws || ws_bytes < p.total) return set_error(FDR_ERR_WORKSPACE, "impala forward workspace too small");
  if (c.n_envs == 0) return FDR_OK;
  char* w = static_cast<char*>(ws);
  LanesArgs lanes{};
  lanes.base = c.theta;
  StepArgs a{};
  a.pack = reinterpret_cast<float*>(w + p.pack);
  a.pack_stride = 0;  // every env shares the one pack
  a.bn_mean = c.bn_mean;
  a.bn_var = c.bn_var;
  a.n_lanes = c.n_envs;
  a.envs = 1;
  a.n_act = L.n_act;
  a.frames = c.frames;
  a.feat = c.feat_out ? c.feat_out : reinterpret_cast<float*>(w + p.feat);
  a.h = c.h;
  a.c = c.c;
  a.probs = c.probs;
  a.reward_in = c.reward;
  a.notdone = c.notdone;
  launch_pack<float>(L, lanes, const_cast<float*>(a.pack), reinterpret_cast<double*>(w + p.n2), 1, 0, stream);
  if (c.fp16) {
    a.hpack = reinterpret_cast<_Float16*>(w + p.hpack);
    a.hpack_stride = 0;
    launch_pack<_Float16>(L, lanes, a.hpack, reinterpret_cast<double*>(w + p.n2), 1, 1, stream);
  }
  if (c.fp16) {
    launch_conv_h((c.n_envs + 7) / 8 * 8, L, a, stream);
    hipLaunchKernelGGL((core_kernel_h<1, kForward>), dim3(c.n_envs), dim3(kCoreThreads), 0, stream, L, a);
  } else {
    hipLaunchKernelGGL(conv_kernel, dim3((c.n_envs + 7) / 8 * 8), dim3(kConvThreads), 0, stream, L, a);
    hipLaunchKernelGGL((core_kernel<1, kForward>), dim3(c.n_envs), dim3(kCoreThreads), 0, stream, L, a);
  }
  return check_launch("impala forward");
}


// ------------------------------------------------------------------------------------------
// get_strategy over a probe set zeta (policies/impala.py:24-27 -> ImpalaCNN.forward :136-186): the Z
// stacked obs are ONE batch_first LSTM sequence per lane (B = 1, T = Z), so per lane the conv stack runs
// on Z shared frames (conv kernel, shared_frames), the fc is one GEMM over the Z feature rows
// (fc_rows_kernel below), the LSTM input projection one GEMM per 64-step chunk (lstm_xproj_kernel) and
// the recurrence + head one core-kernel launch per step (kStrategy: probabilities out).
// ------------------------------------------------------------------------------------------
// ci[z][lane][0:256] = relu(BN1d(feat_(lane, z)) W_fc^T + b_fc), ci[z][lane][256] = clamp(reward_z, -1, 1)
// (policies/impala.py:161-164) on v_mfma_f32_16x16x4_f32: 64 rows x 256 columns per workgroup, K = 2048
// in LDS chunks of 32 with the eval-mode BN folded into the X-tile load.  fp16 mode reads the f16 W^T.
template <bool HALF>
__global__ __launch_bounds__(256) void fc_rows_kernel(Layout L, StepArgs a, int z0, int zc) {
  constexpr int KC = 32, XP = 80, WP = 256 + 16;
  __shared__ float xs[KC * XP];  // [k][row]
  __shared__ float ws[KC * WP];  // [k][col]
  const int lane = blockIdx.x, row0 = blockIdx.y * 64;
  const int tid = threadIdx.x, wave = tid >> 6, ln = tid & 63, g = ln >> 4, r = ln & 15;
  const float* pk = a.pack + (int64_t)lane * a.pack_stride;
  f32x4 acc[4][4];
#pragma unroll
  for (int ti = 0; ti < 4; ++ti)
#pragma unroll
    for (int tj = 0; tj < 4; ++tj) acc[ti][tj] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int k0 = 0; k0 < kFeat; k0 += KC) {
    const int kk = k0 + (tid & 31);  // every X element this thread loads has this k
    const float rmv = (a.bn_mean ? a.bn_mean + L.bn_stat[15] : a.pack)[kk];  // branch-free
    const float rvv = (a.bn_var ? a.bn_var + L.bn_stat[15] : a.pack)[kk];
    const float rm = a.bn_mean ? rmv : 0.f, rv = a.bn_var ? rvv : 1.f;
    const float sc = pk[L.bn_w[15] + kk] * (1.f / sqrtf(rv + kBnEps));
    const float sh = fmaf(-rm, sc, pk[L.bn_b[15] + kk]);
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int i = tid + 256 * m, row = i >> 5, q = row0 + row;
      xs[(i & 31) * XP + row] = q < zc ? fmaf(a.feat[((int64_t)lane * zc + q) * kFeat + kk], sc, sh) : 0.f;
    }
#pragma unroll
    for (int m = 0; m < 8; ++m) {
      const int i = tid + 256 * m, k = i >> 6, c4 = i & 63;
      float4 w;
      if constexpr (HALF) {
        typedef _Float16 h4v __attribute__((ext_vector_type(4)));
        const h4v hv = *reinterpret_cast<const h4v*>(a.hpack + (int64_t)lane * a.hpack_stride + L.fc_wt_h +
                                                      (int64_t)(k0 + k) * kHid + 4 * c4);
        w = float4{(float)hv[0], (float)hv[1], (float)hv[2], (float)hv[3]};
      } else {
        w = *reinterpret_cast<const float4*>(pk + L.fc_wt + (int64_t)(k0 + k) * kHid + 4 * c4);
      }
      *reinterpret_cast<float4*>(ws + k * WP + 4 * c4) = w;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < KC / 4; ++s) {
      const int k = 4 * s + g;
      float av[4], bv[4];
#pragma unroll
      for (int ti = 0; ti < 4; ++ti) av[ti] = xs[k * XP + 16 * ti + r];
#pragma unroll
      for (int tj = 0; tj < 4; ++tj) bv[tj] = ws[k * WP + 64 * wave + 16 * tj + r];
#pragma unroll
      for (int ti = 0; ti < 4; ++ti)
#pragma unroll
        for (int tj = 0; tj < 4; ++tj) acc[ti][tj] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[ti], bv[tj], acc[ti][tj], 0, 0, 0);
    }
    __syncthreads();
  }
  float bias[4];
#pragma unroll
  for (int tj = 0; tj < 4; ++tj) bias[tj] = pk[L.fc_b + 64 * wave + 16 * tj + r];
#pragma unroll
  for (int ti = 0; ti < 4; ++ti)
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int q = row0 + 16 * ti + 4 * g + v;
      if (q >= zc) continue;
      float* dst = a.ci + ((int64_t)(z0 + q) * a.n_lanes + lane) * kCoreIn + 64 * wave + r;
#pragma unroll
      for (int tj = 0; tj < 4; ++tj) dst[16 * tj] = relu(acc[ti][tj][v] + bias[tj]);
    }
  if (blockIdx.y == 0 && tid < zc) {
    const float rw = a.reward_in ? a.reward_in[z0 + tid] : 0.f;
    a.ci[((int64_t)(z0 + tid) * a.n_lanes + lane) * kCoreIn + kHid] = fminf(fmaxf(rw, -1.f), 1.f);
  }
}

namespace {
struct StratPlan {
  int64_t pack, hpack, feat, ci, gx, h, c, n2, zeros, thpack, epack, idxe, mimg, total;
  int nblk;
};
// pairs (fp16): theta's half pack, one sigma-eps half pack per pair and their MFMA images, as the rollout's pair form
StratPlan strat_plan(const Layout& L, int n_lanes, int Z, bool fp16, bool pairs = false) {
  StratPlan p{};
  int64_t o = 0;
  auto take = [&](int64_t bytes) { const int64_t at = o; o += round_up(std::max<int64_t>(bytes, 0), 256); return at; };
  const int zc = std::min(Z, kReplayChunk);
  p.nblk = prep_blocks(L);
  p.pack = take((int64_t)n_lanes * L.pack * 4);
  p.hpack = take(fp16 ? (int64_t)n_lanes * L.hpack * 2 : 0);
  p.feat = take((int64_t)n_lanes * zc * kFeat * 4);
  p.ci = take((int64_t)Z * n_lanes * kCoreIn * 4);
  p.gx = take((int64_t)zc * n_lanes * kGates * 4);
  p.h = take((int64_t)n_lanes * kHid * 4);
  p.c = take((int64_t)n_lanes * kHid * 4);
  p.n2 = take((int64_t)n_lanes * p.nblk * 8);
  const bool pr = pairs && fp16;
  p.zeros = take(pr ? L.P * 4 : 0);
  p.thpack = take(pr ? L.hpack * 2 : 0);
  p.epack = take(pr ? (int64_t)(n_lanes / 2) * L.hpack * 2 : 0);
  p.idxe = take(pr ? (int64_t)(n_lanes / 2) * 8 : 0);
  p.mimg = take(pr ? (int64_t)(n_lanes / 2 + 1) * kMImg * 2 : 0);
  p.total = o;
  return p;
}
}  // namespace

int64_t strategies_workspace_bytes(const Layout& L, int n_lanes, int n_states, bool fp16, bool pairs) {
  return strat_plan(L, n_lanes, n_states, fp16, pairs).total;
}

// The pair form ran lane 2p + 1 on lane 2p's noise: a pair whose offsets differ has no defined result, so both lanes'
// probabilities become NaN (the rollout's pair form poisons their norms the same way, pair_offsets_kernel)
__global__ void poison_pair_probs_kernel(const int64_t* __restrict__ idx, int64_t per_lane, float* __restrict__ probs) {
  const int p = blockIdx.x;
  if (idx[2 * p] == idx[2 * p + 1]) return;
  float* q = probs + (int64_t)2 * p * per_lane;
  for (int64_t e = threadIdx.x; e < 2 * per_lane; e += blockDim.x) q[e] = __builtin_nanf("");
}

int launch_strategies(const StrategiesCall& c, void* ws, int64_t ws_bytes, hipStream_t stream) {
  const Layout& L = *c.layout;
  const int Z = c.n_states;
  const StratPlan p = strat_plan(L, c.n_lanes, Z, c.fp16 != 0, c.pairs != 0);
  if (!ws || ws_bytes < p.total) return set_error(FDR_ERR_WORKSPACE, "impala strategies workspace too small");
  if (c.n_lanes == 0 || Z == 0) return FDR_OK;
  char* w = static_cast<char*>(ws);
  const bool half = c.fp16 != 0;
  StepArgs a{};
  a.pack = reinterpret_cast<float*>(w + p.pack);
  a.pack_stride = L.pack;
  a.bn_mean = c.bn_mean;
  a.bn_var = c.bn_var;
  a.n_lanes = c.n_lanes;
  a.n_act = L.n_act;
  a.T = Z;
  a.shared_frames = 1;
  a.reward_in = c.reward;
  a.feat = reinterpret_cast<float*>(w + p.feat);
  a.ci = reinterpret_cast<float*>(w + p.ci);
  a.h = c.h ? c.h : reinterpret_cast<float*>(w + p.h);
  a.c = c.c ? c.c : reinterpret_cast<float*>(w + p.c);
  a.probs = c.probs;
  double* n2 = reinterpret_cast<double*>(w + p.n2);
  launch_pack<float>(L, c.lanes, const_cast<float*>(a.pack), n2, c.n_lanes, 0, stream, half ? kTrSkip : kTrFull);
  if (half) {
    a.hpack = reinterpret_cast<_Float16*>(w + p.hpack);
    a.hpack_stride = L.hpack;
    launch_pack<_Float16>(L, c.lanes, a.hpack, n2, c.n_lanes, 1, stream);
  }
  // antithetic pairs (fp16): the recurrence streams each pair's sigma-eps image once (replay_chunk_hpm2<1, kStrategy>,
  // x W_ih^T by xproj_pair_kernel), as the rollout's pair form -- conv and fc stay per lane (per-lane half pack)
  const bool pair_form = half && c.pairs && c.n_lanes % 4 == 0 && c.lanes.table &&
                         c.lanes.base_stride == 0;
  if (pair_form) {
    const int np = c.n_lanes / 2;
    float* zeros = reinterpret_cast<float*>(w + p.zeros);
    int64_t* idxe = reinterpret_cast<int64_t*>(w + p.idxe);
    _Float16* th = reinterpret_cast<_Float16*>(w + p.thpack);
    _Float16* ep = reinterpret_cast<_Float16*>(w + p.epack);
    _Float16* im = reinterpret_cast<_Float16*>(w + p.mimg);
    (void)hipMemsetAsync(zeros, 0, (size_t)L.P * 4, stream);
    hipLaunchKernelGGL(pair_offsets_kernel, dim3((np + 255) / 256), dim3(256), 0, stream, c.lanes.idx, np, idxe, n2,
                       p.nblk);
    LanesArgs lt = c.lanes;
    lt.table = nullptr;
    LanesArgs le = c.lanes;
    le.base = zeros;
    le.base_stride = 0;
    le.idx = idxe;
    le.sign = nullptr;
    launch_pack<_Float16>(L, lt, th, n2, 1, 1, stream);
    launch_pack<_Float16>(L, le, ep, n2, np, 1, stream, kTrFull, false);  // feeds only the images
    const unsigned nb = kFcKS + 4 * kGateKS;
    hipLaunchKernelGGL(mfma_image_kernel, dim3(nb, 1), dim3(256), 0, stream, L, th, (int64_t)0, im);
    hipLaunchKernelGGL(mfma_image_kernel, dim3(nb, np), dim3(256), 0, stream, L, ep, (int64_t)L.hpack, im + kMImg);
    a.thm = im;
    a.epm = im + kMImg;
    a.sign = c.lanes.sign;
  }
  if (!c.h || !c.c) {  // the reset state (worker/agent.py:66 resets the policy before compute_novelty)
    if (hipMemsetAsync(a.h, 0, (size_t)c.n_lanes * kHid * 4, stream) != hipSuccess ||
        hipMemsetAsync(a.c, 0, (size_t)c.n_lanes * kHid * 4, stream) != hipSuccess)
      return set_error(FDR_ERR_HIP, "memset of the initial LSTM state failed");
  }
  for (int z0 = 0; z0 < Z; z0 += kReplayChunk) {
    const int zc = std::min(kReplayChunk, Z - z0);
    a.envs = zc;
    a.frames = c.frames + (int64_t)z0 * kFramePix;
    const int conv_grid = (c.n_lanes + 7) / 8 * 8 * zc;
    if (half)
      launch_conv_h(conv_grid, L, a, stream);
    else
      hipLaunchKernelGGL(conv_kernel, dim3(conv_grid), dim3(kConvThreads), 0, stream, L, a);
    const dim3 grid(c.n_lanes, (zc + 63) / 64);
    if (half)
      hipLaunchKernelGGL(fc_rows_kernel<true>, grid, dim3(256), 0, stream, L, a, z0, zc);
    else
      hipLaunchKernelGGL(fc_rows_kernel<false>, grid, dim3(256), 0, stream, L, a, z0, zc);
  }
  a.envs = 1;
  float* gx = reinterpret_cast<float*>(w + p.gx);
  for (int t0 = 0; t0 < Z; t0 += kReplayChunk) {
    const int tc = std::min(kReplayChunk, Z - t0);
    const dim3 grid(c.n_lanes, (tc + 63) / 64, kGates / 256);
    a.gx = nullptr;
    if (pair_form)
      hipLaunchKernelGGL((xproj_pair_kernel<1, false>), xproj_grid(c.n_lanes), dim3(256), 0, stream, L, a, t0, tc,
                         gx);
    else if (half)
      hipLaunchKernelGGL(lstm_xproj_kernel<true>, grid, dim3(256), 0, stream, L, a, t0, tc, gx);
    else
      hipLaunchKernelGGL(lstm_xproj_kernel<false>, grid, dim3(256), 0, stream, L, a, t0, tc, gx);
    a.gx = gx;
    a.gx_t0 = t0;
    if (pair_form) {  // the chunk's sequence steps in one launch
      hipLaunchKernelGGL((replay_chunk_hpm2<1, kStrategy>), dim3(c.n_lanes / 4), dim3(2 * kCoreThreads), 0, stream, L, a,
                         t0, tc);
      continue;
    }
    for (int t = t0; t < t0 + tc; ++t) {
      a.t = t;
      if (half)
        hipLaunchKernelGGL((core_kernel_h<1, kStrategy>), dim3(c.n_lanes), dim3(kCoreThreads), 0, stream, L, a);
      else
        hipLaunchKernelGGL((core_kernel<1, kStrategy>), dim3(c.n_lanes), dim3(kCoreThreads), 0, stream, L, a);
    }
  }
  if (pair_form)
    hipLaunchKernelGGL(poison_pair_probs_kernel, dim3(c.n_lanes / 2), dim3(256), 0, stream, c.lanes.idx,
                       (int64_t)Z * L.n_act, c.probs);
  return check_launch("impala strategies");
}

// ------------------------------------------------------------------------------------------
// The synthetic frame env's observations outside a rollout (eval states / the probe set zeta,
// run_sequential.py:142-143, 198-213): frame_t of env `env_id` (the conv kernel's generator) and, given
// the actions taken, the reward each step returns.  One workgroup per step.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void env_frames_kernel(uint64_t fkey, uint64_t rkey, int n_act, uint64_t env_id,
                                                         int t0, const int32_t* actions, float* frames,
                                                         float* reward) {
  const int i = blockIdx.x, t = t0 + i;
  float* fr = frames + (int64_t)i * kFramePix;
  for (int w = threadIdx.x; w < kFramePix / 8; w += blockDim.x) {
    const uint64_t hb = mix64(fkey + ((env_id << 32) | ((uint64_t)t << 11) | (uint64_t)w) * kGolden);
#pragma unroll
    for (int j = 0; j < 8; ++j) fr[8 * w + j] = (float)((uint32_t)(hb >> (8 * j)) & 255u);
  }
  if (threadIdx.x == 0 && reward) {
    float r = 0.f;
    if (actions) {
      const int tgt = (int)((mix64(rkey + ((env_id << 32) | ((uint64_t)t << 11)) * kGolden) >> 40) % (uint64_t)n_act);
      const int act = actions[i];
      r = act == tgt ? 1.f : (act == (tgt + 1) % n_act ? -1.f : 0.f);
    }
    reward[i] = r;
  }
}

int launch_env_frames(uint64_t env_seed, int n_act, uint64_t env_id, int t0, int n, const int32_t* actions,
                      float* frames, float* reward, hipStream_t stream) {
  if (n == 0) return FDR_OK;
  hipLaunchKernelGGL(env_frames_kernel, dim3(n), dim3(256), 0, stream, mix64(env_seed ^ kFrameSalt),
                     mix64(env_seed ^ kRewardSalt), n_act, env_id, t0, actions, frames, reward);
  return check_launch("impala env frames");
}

}  // namespace impala
}  // namespace fdr
