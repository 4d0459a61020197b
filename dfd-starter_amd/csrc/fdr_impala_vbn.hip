// ImpalaPolicy.compute_vbn (policies/impala.py:12-16) on the device: one train-mode pass of the VBN buffer
// (run_sequential.py:156-157, :198-213) through the ImpalaCNN, layer by layer.
//
// Train-mode BatchNorm couples every sample of the buffer: a BN layer can normalise only once the batch
// statistics of its whole input are known, so the pass is a sequence of (statistics -> BN-fused layer) launches
// over the [n, C, H, W] activations (NCHW, f32, HBM), not the per-env fused stack of the rollout kernels:
//   stats_kernel     per-channel f64 sum / sum of squares over n x H x W (grid C x blocks), partials
//   finalize_kernel  mean, biased var -> the affine BN terms torch's CPU kernel uses (alpha = w / sqrt(var + eps),
//                    beta = b - mean alpha) and the running-stat update (unbiased var, momentum)
//   conv_kernel      BN (+ ReLU) applied while a 16 x 16 tile and its halo are staged in LDS (zero padding AFTER the
//                    BN, as Conv2d pads its input), 3 x 3 conv + bias (+ residual) with COUT accumulators per thread
//   pool_kernel      MaxPool2d(3, 2, 1) (-inf padding)
//   fc / gx kernels  BatchNorm1d(2048) over the n rows -> Linear + ReLU -> cat(clamped reward); x W_ih^T + b_ih
//   lstm_seq_kernel  the batch_first LSTM over the n obs as ONE sequence (B = 1, T = n) from the carried state, zeroed
//                    iff the first obs is done (impala.py:165-176); the end state is written back (:184)
// then the head BatchNorm1d(256)'s statistics over the n hidden states.  Off the hot path (once per epoch); parity:
// tests/test_gpu_impala_vbn.py against the reference's own compute_vbn (tests/golden/g14_impala_vbn.npz).
//
// AtariPolicy.compute_vbn (policies/policy.py:31-34 on atari.py:36-51) is the same statistics -> BN-fused layer chain
// over its three BNs (atari::launch_vbn at the end of this file): conv 4->16 k8 s4, BN2d(16), ReLU, conv 16->32 k4 s2,
// BN2d(32), ReLU, Linear 2592->256, BN1d(256) -- the head after it feeds no statistic.  Parity: G16.
#include <cfloat>

#include "fdr_impala.h"

namespace fdr {
namespace impala {
namespace {

constexpr int kCh[3] = {16, 32, 32};
constexpr int kStatBlocks = 64;  // max blocks per channel of stats_kernel
constexpr int kFcRows = 8;       // buffer rows per workgroup of the fc / gx kernels

// Theta offsets (reference parameters() order) of every weight the pass reads, from the Layout's sections.
struct VbnParams {
  int64_t bn_w[kBns];       // weight; bias follows (+ channels)
  int64_t conv_w[kConvs], conv_b[kConvs];
  int64_t fc_w, fc_b, w_ih, w_hh, b_ih, b_hh;
};

int64_t src_of(const Layout& L, int32_t dst) {
  for (int i = 0; i < L.n_sections; ++i)
    if (L.sec[i].dst == dst) return L.sec[i].src;
  return -1;
}

bool vbn_params(const Layout& L, VbnParams* p) {
  for (int k = 0; k < kBns; ++k) p->bn_w[k] = src_of(L, L.bn_w[k]);
  for (int k = 0; k < kConvs; ++k) {
    p->conv_w[k] = src_of(L, L.conv_w[k]);
    p->conv_b[k] = src_of(L, L.conv_b[k]);
  }
  p->fc_w = src_of(L, L.fc_wt);
  p->fc_b = src_of(L, L.fc_b);
  p->w_ih = src_of(L, L.lstm_wt);
  p->w_hh = p->w_ih + (int64_t)kGates * kCoreIn;  // the section after W_ih (impala.py:118, nn.LSTM order)
  p->b_ih = src_of(L, L.lstm_bih);
  p->b_hh = p->b_ih + kGates;
  for (int k = 0; k < kBns; ++k)
    if (p->bn_w[k] < 0) return false;
  for (int k = 0; k < kConvs; ++k)
    if (p->conv_w[k] < 0 || p->conv_b[k] < 0) return false;
  return p->fc_w >= 0 && p->fc_b >= 0 && p->w_ih >= 0 && p->b_ih >= 0;
}

// x[i][c][p] (relu'd if RELU; / div for the raw frames) partial sums over samples [b * per, (b + 1) * per)
__global__ __launch_bounds__(256) void stats_kernel(const float* __restrict__ X, int n, int C, int HW, int relu,
                                                    float div, double* __restrict__ part) {
  const int c = blockIdx.x, b = blockIdx.y, nb = gridDim.y;
  const int per = (n + nb - 1) / nb;
  const int i0 = b * per, i1 = min(n, i0 + per);
  double s = 0.0, q = 0.0;
  const int64_t cnt = i1 > i0 ? (int64_t)(i1 - i0) * HW : 0;
  for (int64_t e = threadIdx.x; e < cnt; e += 256) {
    const int64_t i = i0 + e / HW, p = e % HW;
    float v = X[(i * C + c) * HW + p];
    if (div != 1.f) v = v / div;
    if (relu) v = v > 0.f ? v : 0.f;
    s += (double)v;
    q += (double)v * (double)v;
  }
  s = wave_sum(s);
  q = wave_sum(q);
  __shared__ double red[2][4];
  if ((threadIdx.x & 63) == 0) {
    red[0][threadIdx.x >> 6] = s;
    red[1][threadIdx.x >> 6] = q;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    part[((int64_t)c * nb + b) * 2 + 0] = red[0][0] + red[0][1] + red[0][2] + red[0][3];
    part[((int64_t)c * nb + b) * 2 + 1] = red[1][0] + red[1][1] + red[1][2] + red[1][3];
  }
}

// torch CPU train-mode BN (double accumulation): mean, var_sum; invstd = 1 / sqrt(var_sum / N + eps);
// running_mean = m * mean + (1 - m) * rm, running_var = m * var_sum / (N - 1) + (1 - m) * rv
__global__ void finalize_kernel(int C, int nb, int64_t N, const double* __restrict__ part,
                                const float* __restrict__ w, const float* __restrict__ bias, float momentum,
                                float* __restrict__ rm, float* __restrict__ rv, float* __restrict__ scale,
                                float* __restrict__ shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double s = 0.0, q = 0.0;
  for (int b = 0; b < nb; ++b) {
    s += part[((int64_t)c * nb + b) * 2 + 0];
    q += part[((int64_t)c * nb + b) * 2 + 1];
  }
  const double mean = s / (double)N;
  double var_sum = q - s * mean;
  var_sum = var_sum > 0.0 ? var_sum : 0.0;
  const float invstd = (float)(1.0 / sqrt(var_sum / (double)N + (double)kBnEps));
  const float alpha = invstd * w[c];
  scale[c] = alpha;
  shift[c] = bias[c] - (float)mean * alpha;
  const double m = (double)momentum;
  rm[c] = (float)(m * mean + (1.0 - m) * (double)rm[c]);
  rv[c] = (float)(m * (var_sum / (double)(N - 1)) + (1.0 - m) * (double)rv[c]);
}

// Y[i][co][y][x] = bias[co] + sum_{ci,ky,kx} W[co][ci][ky][kx] * pad(act(BN(X)))[i][ci][y+ky-1][x+kx-1] (+ R)
template <int CIN, int COUT, int H>
__global__ __launch_bounds__(256) void conv_kernel(const float* __restrict__ X, const float* __restrict__ scale,
                                                   const float* __restrict__ shift, int relu, float div,
                                                   const float* __restrict__ W, const float* __restrict__ bias,
                                                   const float* R, float* Y) {
  constexpr int TW = H < 16 ? H : 16, TP = TW + 2, TPW = TP + 1;  // a TW x TW tile per workgroup of TW^2 threads
  constexpr int TILES = H / TW, NT = TW * TW;
  __shared__ float tin[CIN][TP][TPW];
  __shared__ float ws[CIN * 9][COUT];  // [ci][k][co]: the COUT weights of one (ci, k) are contiguous
  const int i = blockIdx.y;
  const int ty0 = (blockIdx.x / TILES) * TW, tx0 = (blockIdx.x % TILES) * TW;
  const int tid = threadIdx.x;
  for (int e = tid; e < COUT * CIN * 9; e += NT) {
    const int co = e / (CIN * 9), r = e % (CIN * 9);
    ws[r][co] = W[e];
  }
  const float* xi = X + (int64_t)i * CIN * H * H;
  for (int e = tid; e < CIN * TP * TP; e += NT) {
    const int ci = e / (TP * TP), r = e % (TP * TP);
    const int yy = r / TP, xx = r % TP;
    const int gy = ty0 + yy - 1, gx = tx0 + xx - 1;
    float v = 0.f;
    if (gy >= 0 && gy < H && gx >= 0 && gx < H) {
      v = xi[((int64_t)ci * H + gy) * H + gx];
      if (div != 1.f) v = v / div;
      v = v * scale[ci] + shift[ci];
      if (relu) v = v > 0.f ? v : 0.f;
    }
    tin[ci][yy][xx] = v;
  }
  __syncthreads();
  const int ty = tid / TW, tx = tid % TW;
  float acc[COUT];
#pragma unroll
  for (int co = 0; co < COUT; ++co) acc[co] = 0.f;
  for (int ci = 0; ci < CIN; ++ci)
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const float v = tin[ci][ty + k / 3][tx + k % 3];
      const float* wk = ws[ci * 9 + k];
#pragma unroll
      for (int co = 0; co < COUT; ++co) acc[co] = fmaf(wk[co], v, acc[co]);
    }
  const int y = ty0 + ty, x = tx0 + tx;
#pragma unroll
  for (int co = 0; co < COUT; ++co) {
    const int64_t o = (((int64_t)i * COUT + co) * H + y) * H + x;
    float v = acc[co] + bias[co];
    if (R) v = v + R[o];
    Y[o] = v;
  }
}

// MaxPool2d(kernel 3, stride 2, padding 1): [n][C][H][H] -> [n][C][H/2][H/2]
__global__ void pool_kernel(const float* __restrict__ X, int64_t total, int H, float* __restrict__ Y) {
  const int64_t o = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (o >= total) return;
  const int Ho = H / 2;
  const int x = (int)(o % Ho), y = (int)((o / Ho) % Ho);
  const int64_t plane = o / ((int64_t)Ho * Ho);
  const float* xp = X + plane * H * H;
  float m = -FLT_MAX;
  bool any = false;
  for (int dy = -1; dy <= 1; ++dy)
    for (int dx = -1; dx <= 1; ++dx) {
      const int yy = 2 * y + dy, xx = 2 * x + dx;
      if (yy < 0 || yy >= H || xx < 0 || xx >= H) continue;
      const float v = xp[yy * H + xx];
      m = any ? fmaxf(m, v) : v;
      any = true;
    }
  Y[o] = m;
}

// WT[k][j] = W[j][k]  (rows x cols -> cols x rows), coalesced reads of the streamed weights below
__global__ void transpose_kernel(const float* __restrict__ W, int rows, int cols, float* __restrict__ WT) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (int64_t)rows * cols) return;
  const int j = (int)(e / cols), k = (int)(e % cols);
  WT[(int64_t)k * rows + j] = W[e];
}

// CI[i] = [relu(fc_b + BN1d(relu(X[i])) fc_w^T) | clamp(reward[i], -1, 1)]  (impala.py:159-164)
__global__ __launch_bounds__(256) void fc_kernel(const float* __restrict__ X, int n, const float* __restrict__ scale,
                                                 const float* __restrict__ shift, const float* __restrict__ WT,
                                                 const float* __restrict__ b, const float* __restrict__ reward,
                                                 float* __restrict__ CI) {
  __shared__ float xs[kFcRows][kFeat];
  const int i0 = blockIdx.x * kFcRows, tid = threadIdx.x;
  for (int e = tid; e < kFcRows * kFeat; e += 256) {
    const int r = e / kFeat, k = e % kFeat;
    float v = 0.f;
    if (i0 + r < n) {
      v = X[(int64_t)(i0 + r) * kFeat + k];
      v = v > 0.f ? v : 0.f;
      v = v * scale[k] + shift[k];
    }
    xs[r][k] = v;
  }
  __syncthreads();
  float acc[kFcRows];
#pragma unroll
  for (int r = 0; r < kFcRows; ++r) acc[r] = 0.f;
  for (int k = 0; k < kFeat; ++k) {
    const float w = WT[(int64_t)k * kHid + tid];
#pragma unroll
    for (int r = 0; r < kFcRows; ++r) acc[r] = fmaf(w, xs[r][k], acc[r]);
  }
  for (int r = 0; r < kFcRows; ++r) {
    if (i0 + r >= n) break;
    const float v = acc[r] + b[tid];
    CI[(int64_t)(i0 + r) * kCoreIn + tid] = v > 0.f ? v : 0.f;
    if (tid == 0) {
      const float rw = reward ? reward[i0 + r] : 0.f;
      CI[(int64_t)(i0 + r) * kCoreIn + kHid] = fminf(fmaxf(rw, -1.f), 1.f);
    }
  }
}

// GX[i][g] = CI[i] W_ih[g]^T + b_ih[g]; grid (rows / kFcRows, kGates / 256)
__global__ __launch_bounds__(256) void gx_kernel(const float* __restrict__ CI, int n, const float* __restrict__ WT,
                                                 const float* __restrict__ b, float* __restrict__ GX) {
  __shared__ float xs[kFcRows][kCoreIn];
  const int i0 = blockIdx.x * kFcRows, g = blockIdx.y * 256 + threadIdx.x;
  for (int e = threadIdx.x; e < kFcRows * kCoreIn; e += 256) {
    const int r = e / kCoreIn, k = e % kCoreIn;
    xs[r][k] = i0 + r < n ? CI[(int64_t)(i0 + r) * kCoreIn + k] : 0.f;
  }
  __syncthreads();
  float acc[kFcRows];
#pragma unroll
  for (int r = 0; r < kFcRows; ++r) acc[r] = 0.f;
  for (int k = 0; k < kCoreIn; ++k) {
    const float w = WT[(int64_t)k * kGates + g];
#pragma unroll
    for (int r = 0; r < kFcRows; ++r) acc[r] = fmaf(w, xs[r][k], acc[r]);
  }
  for (int r = 0; r < kFcRows && i0 + r < n; ++r) GX[(int64_t)(i0 + r) * kGates + g] = acc[r] + b[g];
}

__device__ __forceinline__ float sigmoid_ref(float x) { return 1.f / (1.f + expf(-x)); }

// The LSTM over the n obs as one sequence (one workgroup, thread g = gate row; gate order i, f, g, o).
__global__ __launch_bounds__(1024) void lstm_seq_kernel(const float* __restrict__ GX, int n,
                                                        const float* __restrict__ WT_hh, const float* __restrict__ b_hh,
                                                        float* h, float* c, int first_done, float* __restrict__ HS) {
  __shared__ float hs[kHid];
  __shared__ float gs[kGates];
  const int g = threadIdx.x;
  float cr = 0.f;
  if (g < kHid) {
    const float h0 = h && !first_done ? h[g] : 0.f;
    cr = c && !first_done ? c[g] : 0.f;
    hs[g] = h0;
  }
  __syncthreads();
  for (int t = 0; t < n; ++t) {
    float acc = 0.f;
    for (int k = 0; k < kHid; ++k) acc = fmaf(WT_hh[(int64_t)k * kGates + g], hs[k], acc);
    gs[g] = GX[(int64_t)t * kGates + g] + (acc + b_hh[g]);
    __syncthreads();
    if (g < kHid) {
      const float ig = sigmoid_ref(gs[g]), fg = sigmoid_ref(gs[kHid + g]);
      const float gg = tanhf(gs[2 * kHid + g]), og = sigmoid_ref(gs[3 * kHid + g]);
      cr = fg * cr + ig * gg;
      const float hv = og * tanhf(cr);
      HS[(int64_t)t * kHid + g] = hv;
      hs[g] = hv;
    }
    __syncthreads();
  }
  if (g < kHid) {
    if (h) h[g] = hs[g];
    if (c) c[g] = cr;
  }
}

struct VbnPlan {
  int64_t A, X, Y, CI, GX, HS, WTfc, WTih, WThh, part, scale, shift, total;
};

VbnPlan vbn_plan(int n) {
  VbnPlan p{};
  int64_t off = 0;
  auto take = [&](int64_t bytes) {
    const int64_t at = off;
    off += (bytes + 255) / 256 * 256;
    return at;
  };
  p.A = take((int64_t)n * kCh[0] * 64 * 64 * 4);
  p.X = take((int64_t)n * kCh[0] * 32 * 32 * 4);
  p.Y = take((int64_t)n * kCh[0] * 32 * 32 * 4);
  p.CI = take((int64_t)n * kCoreIn * 4);
  p.GX = take((int64_t)n * kGates * 4);
  p.HS = take((int64_t)n * kHid * 4);
  p.WTfc = take((int64_t)kFeat * kHid * 4);
  p.WTih = take((int64_t)kCoreIn * kGates * 4);
  p.WThh = take((int64_t)kHid * kGates * 4);
  p.part = take((int64_t)kFeat * kStatBlocks * 2 * 8);
  p.scale = take((int64_t)kFeat * 4);
  p.shift = take((int64_t)kFeat * 4);
  p.total = off;
  return p;
}

template <int CIN, int COUT, int H>
void conv(const float* X, const float* sc, const float* sh, int relu, float div, const float* W, const float* b,
          const float* R, float* Y, int n, hipStream_t s) {
  constexpr int TW = H < 16 ? H : 16;
  hipLaunchKernelGGL((conv_kernel<CIN, COUT, H>), dim3((H / TW) * (H / TW), n), dim3(TW * TW), 0, s, X, sc, sh, relu,
                     div, W, b, R, Y);
}

}  // namespace

int64_t vbn_workspace_bytes(int n) { return n < 0 ? -1 : vbn_plan(n).total; }

int launch_vbn(const VbnCall& a, void* ws, int64_t ws_bytes, hipStream_t s) {
  const Layout& L = *a.layout;
  const int n = a.n;
  VbnParams P;
  if (!vbn_params(L, &P)) return set_error(FDR_ERR_INVALID, "impala layout has no theta offset for a layer");
  const VbnPlan pl = vbn_plan(n);
  if (!ws || ws_bytes < pl.total) return set_error(FDR_ERR_WORKSPACE, "impala bn refresh workspace too small");
  char* base = static_cast<char*>(ws);
  float* A = reinterpret_cast<float*>(base + pl.A);
  float* X = reinterpret_cast<float*>(base + pl.X);
  float* Y = reinterpret_cast<float*>(base + pl.Y);
  float* CI = reinterpret_cast<float*>(base + pl.CI);
  float* GX = reinterpret_cast<float*>(base + pl.GX);
  float* HS = reinterpret_cast<float*>(base + pl.HS);
  float* WTfc = reinterpret_cast<float*>(base + pl.WTfc);
  float* WTih = reinterpret_cast<float*>(base + pl.WTih);
  float* WThh = reinterpret_cast<float*>(base + pl.WThh);
  double* part = reinterpret_cast<double*>(base + pl.part);
  float* sc = reinterpret_cast<float*>(base + pl.scale);
  float* sh = reinterpret_cast<float*>(base + pl.shift);
  const float* th = a.theta;
  const int nb = n < kStatBlocks ? n : kStatBlocks;

  // statistics of layer k's input [n][C][HW] (relu'd first only for the fc BN: relu(x).view -> fc, impala.py:159-161;
  // the residual blocks' ReLU follows their BN) -> running stats + the affine BN terms in sc / sh
  auto bn_stats = [&](int k, const float* in, int C, int HW, int relu, float div) {
    hipLaunchKernelGGL(stats_kernel, dim3(C, nb), dim3(256), 0, s, in, n, C, HW, relu, div, part);
    const float* w = th + P.bn_w[k];
    hipLaunchKernelGGL(finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, C, nb, (int64_t)n * HW, part, w,
                       w + C, a.momentum, a.bn_mean + L.bn_stat[k], a.bn_var + L.bn_stat[k], sc, sh);
  };
  auto pool = [&](const float* in, int C, int H, float* out) {
    const int64_t total = (int64_t)n * C * (H / 2) * (H / 2);
    hipLaunchKernelGGL(pool_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, s, in, total, H, out);
  };
  auto cw = [&](int k) { return th + P.conv_w[k]; };
  auto cb = [&](int k) { return th + P.conv_b[k]; };

  // stage 0: frames / 255 (impala.py:148), 3 -> 16 channels at 64 x 64
  bn_stats(0, a.frames, 3, 64 * 64, 0, 255.f);
  conv<3, 16, 64>(a.frames, sc, sh, 0, 255.f, cw(0), cb(0), nullptr, A, n, s);
  pool(A, 16, 64, X);
  for (int r = 0; r < 2; ++r) {
    const int k0 = 1 + 2 * r, k1 = k0 + 1;
    bn_stats(k0, X, 16, 32 * 32, 0, 1.f);
    conv<16, 16, 32>(X, sc, sh, 1, 1.f, cw(k0), cb(k0), nullptr, Y, n, s);
    bn_stats(k1, Y, 16, 32 * 32, 0, 1.f);
    conv<16, 16, 32>(Y, sc, sh, 1, 1.f, cw(k1), cb(k1), X, X, n, s);
  }
  // stage 1: 16 -> 32 channels at 32 x 32, pooled to 16 x 16
  bn_stats(5, X, 16, 32 * 32, 0, 1.f);
  conv<16, 32, 32>(X, sc, sh, 0, 1.f, cw(5), cb(5), nullptr, A, n, s);
  pool(A, 32, 32, X);
  for (int r = 0; r < 2; ++r) {
    const int k0 = 6 + 2 * r, k1 = k0 + 1;
    bn_stats(k0, X, 32, 16 * 16, 0, 1.f);
    conv<32, 32, 16>(X, sc, sh, 1, 1.f, cw(k0), cb(k0), nullptr, Y, n, s);
    bn_stats(k1, Y, 32, 16 * 16, 0, 1.f);
    conv<32, 32, 16>(Y, sc, sh, 1, 1.f, cw(k1), cb(k1), X, X, n, s);
  }
  // stage 2: 32 -> 32 channels at 16 x 16, pooled to 8 x 8
  bn_stats(10, X, 32, 16 * 16, 0, 1.f);
  conv<32, 32, 16>(X, sc, sh, 0, 1.f, cw(10), cb(10), nullptr, A, n, s);
  pool(A, 32, 16, X);
  for (int r = 0; r < 2; ++r) {
    const int k0 = 11 + 2 * r, k1 = k0 + 1;
    bn_stats(k0, X, 32, 8 * 8, 0, 1.f);
    conv<32, 32, 8>(X, sc, sh, 1, 1.f, cw(k0), cb(k0), nullptr, Y, n, s);
    bn_stats(k1, Y, 32, 8 * 8, 0, 1.f);
    conv<32, 32, 8>(Y, sc, sh, 1, 1.f, cw(k1), cb(k1), X, X, n, s);
  }
  // fc: BatchNorm1d(2048) of relu(x).view(n, -1) (C, H, W order == NCHW), Linear, ReLU, reward column
  hipLaunchKernelGGL(transpose_kernel, dim3(kHid * kFeat / 256), dim3(256), 0, s, th + P.fc_w, kHid, kFeat, WTfc);
  hipLaunchKernelGGL(transpose_kernel, dim3(kGates * kCoreIn / 256 + 1), dim3(256), 0, s, th + P.w_ih, kGates, kCoreIn,
                     WTih);
  hipLaunchKernelGGL(transpose_kernel, dim3(kGates * kHid / 256), dim3(256), 0, s, th + P.w_hh, kGates, kHid, WThh);
  bn_stats(15, X, kFeat, 1, 1, 1.f);
  const int rows = (n + kFcRows - 1) / kFcRows;
  hipLaunchKernelGGL(fc_kernel, dim3(rows), dim3(256), 0, s, X, n, sc, sh, WTfc, th + P.fc_b, a.reward, CI);
  hipLaunchKernelGGL(gx_kernel, dim3(rows, kGates / 256), dim3(256), 0, s, CI, n, WTih, th + P.b_ih, GX);
  hipLaunchKernelGGL(lstm_seq_kernel, dim3(1), dim3(1024), 0, s, GX, n, WThh, th + P.b_hh, a.h, a.c, a.first_done, HS);
  // head BatchNorm1d(256) over the n hidden states (its logits feed no statistic)
  bn_stats(16, HS, kHid, 1, 0, 1.f);
  return check_launch("impala bn refresh");
}

}  // namespace impala

namespace atari {
namespace {

using impala::finalize_kernel;
using impala::kFcRows;
using impala::stats_kernel;
using impala::transpose_kernel;

constexpr int kA1 = 16, kA2 = 32, kO1 = 20, kO2 = 9, kAFeat = kA2 * kO2 * kO2, kAFc = 256;
// theta offsets in the reference's parameters() order (atari.py:36-51): conv1 w [16][4][8][8], b; BN2d(16) w, b;
// conv2 w [32][16][4][4], b; BN2d(32) w, b; fc w [256][2592], b; BN1d(256) w, b; head
constexpr int64_t kC1w = 0, kC1b = kC1w + kA1 * 4 * 64, kBn1 = kC1b + kA1, kC2w = kBn1 + 2 * kA1,
                  kC2b = kC2w + kA2 * kA1 * 16, kBn2 = kC2b + kA2, kFcw = kBn2 + 2 * kA2,
                  kFcb = kFcw + (int64_t)kAFc * kAFeat, kBn3 = kFcb + kAFc;

// Y[i][co][oy][ox] = b[co] + sum_{ci,ky,kx} W[co][ci][ky][kx] * act(X[i][ci][S oy + ky][S ox + kx])  (no padding);
// act = relu(scale[ci] x + shift[ci]) (the previous layer's train-mode BN) when BNIN, else the raw input
template <int CIN, int COUT, int K, int S, int HI, int HO, bool BNIN>
__global__ __launch_bounds__(256) void sconv_kernel(const float* __restrict__ X, const float* __restrict__ scale,
                                                    const float* __restrict__ shift, const float* __restrict__ W,
                                                    const float* __restrict__ b, float* __restrict__ Y, int64_t total) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= total) return;
  const int ox = (int)(e % HO), oy = (int)((e / HO) % HO), co = (int)((e / (HO * HO)) % COUT);
  const int64_t i = e / ((int64_t)HO * HO * COUT);
  float acc = 0.f;
  for (int ci = 0; ci < CIN; ++ci) {
    const float* xp = X + ((i * CIN + ci) * HI + S * oy) * HI + S * ox;
    const float* wp = W + ((int64_t)co * CIN + ci) * K * K;
    const float sc = BNIN ? scale[ci] : 1.f, sh = BNIN ? shift[ci] : 0.f;
#pragma unroll
    for (int ky = 0; ky < K; ++ky)
#pragma unroll
      for (int kx = 0; kx < K; ++kx) {
        float v = xp[ky * HI + kx];
        if (BNIN) v = fmaxf(fmaf(v, sc, sh), 0.f);
        acc = fmaf(wp[ky * K + kx], v, acc);
      }
  }
  Y[e] = acc + b[co];
}

// F[i][o] = fc_b[o] + sum_k fc_w[o][k] relu(BN2d(X2))[i][k]  (k = c * 81 + p: the C, H, W flatten of atari.py:47)
__global__ __launch_bounds__(256) void afc_kernel(const float* __restrict__ X, int n, const float* __restrict__ scale,
                                                  const float* __restrict__ shift, const float* __restrict__ WT,
                                                  const float* __restrict__ b, float* __restrict__ F) {
  __shared__ float xs[kFcRows][kAFeat];
  const int i0 = blockIdx.x * kFcRows, tid = threadIdx.x;
  for (int e = tid; e < kFcRows * kAFeat; e += 256) {
    const int r = e / kAFeat, k = e % kAFeat, c = k / (kO2 * kO2);
    xs[r][k] = i0 + r < n ? fmaxf(fmaf(X[(int64_t)(i0 + r) * kAFeat + k], scale[c], shift[c]), 0.f) : 0.f;
  }
  __syncthreads();
  float acc[kFcRows];
#pragma unroll
  for (int r = 0; r < kFcRows; ++r) acc[r] = 0.f;
  for (int k = 0; k < kAFeat; ++k) {
    const float w = WT[(int64_t)k * kAFc + tid];
#pragma unroll
    for (int r = 0; r < kFcRows; ++r) acc[r] = fmaf(w, xs[r][k], acc[r]);
  }
  for (int r = 0; r < kFcRows && i0 + r < n; ++r) F[(int64_t)(i0 + r) * kAFc + tid] = acc[r] + b[tid];
}

struct AVbnPlan {
  int64_t X1, X2, F, WT, part, scale, shift, total;
};

AVbnPlan avbn_plan(int n) {
  AVbnPlan p{};
  int64_t off = 0;
  auto take = [&](int64_t bytes) {
    const int64_t at = off;
    off += (bytes + 255) / 256 * 256;
    return at;
  };
  p.X1 = take((int64_t)n * kA1 * kO1 * kO1 * 4);
  p.X2 = take((int64_t)n * kAFeat * 4);
  p.F = take((int64_t)n * kAFc * 4);
  p.WT = take((int64_t)kAFeat * kAFc * 4);
  p.part = take((int64_t)kAFc * impala::kStatBlocks * 2 * 8);
  p.scale = take((int64_t)kAFc * 4);
  p.shift = take((int64_t)kAFc * 4);
  p.total = off;
  return p;
}

}  // namespace

int64_t vbn_workspace_bytes(int n) { return n < 0 ? -1 : avbn_plan(n).total; }

int launch_vbn(const float* theta, int n, const float* frames, float momentum, float* bn_mean, float* bn_var, void* ws,
               int64_t ws_bytes, hipStream_t s) {
  const AVbnPlan pl = avbn_plan(n);
  if (!ws || ws_bytes < pl.total) return set_error(FDR_ERR_WORKSPACE, "atari bn refresh workspace too small");
  char* base = static_cast<char*>(ws);
  float* X1 = reinterpret_cast<float*>(base + pl.X1);
  float* X2 = reinterpret_cast<float*>(base + pl.X2);
  float* F = reinterpret_cast<float*>(base + pl.F);
  float* WT = reinterpret_cast<float*>(base + pl.WT);
  double* part = reinterpret_cast<double*>(base + pl.part);
  float* sc = reinterpret_cast<float*>(base + pl.scale);
  float* sh = reinterpret_cast<float*>(base + pl.shift);
  const float* th = theta;
  const int nb = n < impala::kStatBlocks ? n : impala::kStatBlocks;
  // statistics of a BN's input [n][C][HW] -> its running stats (at `at` in the flat [16 | 32 | 256]) + sc / sh
  auto bn_stats = [&](const float* in, int C, int HW, int64_t w, int at) {
    hipLaunchKernelGGL(stats_kernel, dim3(C, nb), dim3(256), 0, s, in, n, C, HW, 0, 1.f, part);
    hipLaunchKernelGGL(finalize_kernel, dim3((C + 255) / 256), dim3(256), 0, s, C, nb, (int64_t)n * HW, part, th + w,
                       th + w + C, momentum, bn_mean + at, bn_var + at, sc, sh);
  };
  auto grid = [](int64_t total) { return dim3((unsigned)((total + 255) / 256)); };
  const int64_t t1 = (int64_t)n * kA1 * kO1 * kO1, t2 = (int64_t)n * kAFeat;
  hipLaunchKernelGGL((sconv_kernel<4, kA1, 8, 4, 84, kO1, false>), grid(t1), dim3(256), 0, s, frames, nullptr, nullptr,
                     th + kC1w, th + kC1b, X1, t1);
  bn_stats(X1, kA1, kO1 * kO1, kBn1, 0);
  hipLaunchKernelGGL((sconv_kernel<kA1, kA2, 4, 2, kO1, kO2, true>), grid(t2), dim3(256), 0, s, X1, sc, sh, th + kC2w,
                     th + kC2b, X2, t2);
  bn_stats(X2, kA2, kO2 * kO2, kBn2, kA1);
  hipLaunchKernelGGL(transpose_kernel, dim3(kAFc * kAFeat / 256), dim3(256), 0, s, th + kFcw, kAFc, kAFeat, WT);
  hipLaunchKernelGGL(afc_kernel, dim3((n + kFcRows - 1) / kFcRows), dim3(256), 0, s, X2, n, sc, sh, WT, th + kFcb, F);
  bn_stats(F, kAFc, 1, kBn3, kA1 + kA2);
  return check_launch("atari bn refresh");
}

}  // namespace atari
}  // namespace fdr
