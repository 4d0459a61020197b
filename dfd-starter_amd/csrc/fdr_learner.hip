// fdr_learner.hip -- perturbation batch, FD weighting, noise-weighted gradient reduce, DSGD.
//
// All of these are HBM-bound integer/byte-indexed streams (DESIGN.md "Learner kernels"):
//   perturb       reads P floats of theta (L2-resident) + n*P table floats, writes n*P
//   fd_weights    one workgroup, N rewards (a few KB)
//   fd_grad       reads n_dirs * P table floats once (dword loads: table offsets are arbitrary,
//                 so rows are only 4-B aligned), f64 column partial sums per row-chunk, then a
//                 fixed-order chunk reduce -> deterministic result independent of launch shape
//   dsgd          two passes over P (norm partials, then update + update-norm partials)
#include <hip/hip_runtime.h>

#include <cmath>

#include "fdr_common.h"
#include "fdr_internal.h"

namespace fdr {

// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void perturb_kernel(const float* __restrict__ theta, int64_t P,
                                                       const float* __restrict__ table, int64_t max_idx,
                                                       const int64_t* __restrict__ idx,
                                                       const int8_t* __restrict__ sign, float sigma,
                                                       float* __restrict__ out) {
#pragma clang fp contract(off)
  const int l = blockIdx.y;
  const int s = sign ? sign[l] : 1;
  const int64_t off = idx[l];
  const bool bad = off < 0 || off > max_idx;  // never dereference an out-of-range offset
  const float* eps = table + (bad ? 0 : off);
  float* o = out + (int64_t)l * P;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P;
       p += (int64_t)gridDim.x * blockDim.x) {
    const float t = theta[p];
    if (bad) {
      o[p] = __builtin_nanf("");
      continue;
    }
    const float st = sigma * eps[p];
    o[p] = s > 0 ? t + st : (s < 0 ? t - st : t);
  }
}

int launch_perturb(const float* theta, int64_t P, const float* table, int64_t table_size,
                   const int64_t* idx, const int8_t* sign, int n, float sigma, float* out,
                   hipStream_t stream) {
  const int bx = (int)std::min<int64_t>((P + 255) / 256, 64);
  hipLaunchKernelGGL(perturb_kernel, dim3(bx, n), dim3(256), 0, stream, theta, P, table,
                     table_size - P, idx, sign, sigma, out);
  return check_launch("perturb_kernel");
}

// ------------------------------------------------------------------------------------------
// FD weighting: one 1024-thread workgroup.  Deterministic tree sums in f64.
// ------------------------------------------------------------------------------------------
__device__ double block_sum_1024(double v, double* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, j = threadIdx.x & 63;
  __syncthreads();
  if (j == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < (int)(blockDim.x >> 6); ++i) s += red[i];
  return s;
}

__global__ __launch_bounds__(1024) void fd_weights_kernel(const double* __restrict__ r_all, int n_all,
                                                           double pr, int lo, int n_local,
                                                           const int8_t* __restrict__ sign,
                                                           const double* __restrict__ n2, int lpd,
                                                           float sigma, double* __restrict__ coef) {
  __shared__ double red[16];
  double s = 0.0;
  for (int i = threadIdx.x; i < n_all; i += blockDim.x) s += r_all[i] - pr;
  const double mean = block_sum_1024(s, red) / (double)n_all;
  double q = 0.0;
  for (int i = threadIdx.x; i < n_all; i += blockDim.x) {
    const double d = (r_all[i] - pr) - mean;
    q += d * d;
  }
  const double var = block_sum_1024(q, red) / (double)n_all;
  const double sd = sqrt(var);
  const int n_dirs = n_local / lpd;
  for (int d = threadIdx.x; d < n_dirs; d += blockDim.x) {
    double c = 0.0;
    for (int k = 0; k < lpd; ++k) {
      const int i = d * lpd + k;
      const int sg = sign[i];
      if (sg == 0) continue;
      const double x = r_all[lo + i] - pr;
      const double z = sd == 0.0 ? x : (x - mean) / sd;  // utils/math_helpers.py:127-134
      c += z * (double)sg * (double)sigma / n2[i];
    }
    coef[d] = c;
  }
}

int launch_fd_weights(const double* r_all, int n_all, double pr, int lo, int n_local,
                      const int8_t* sign, const double* n2, int lpd, float sigma, double* coef,
                      hipStream_t stream) {
  hipLaunchKernelGGL(fd_weights_kernel, dim3(1), dim3(1024), 0, stream, r_all, n_all, pr, lo,
                     n_local, sign, n2, lpd, sigma, coef);
  return check_launch("fd_weights_kernel");
}

// ------------------------------------------------------------------------------------------
// Noise-weighted gradient: g[p] = sum_d coef[d] * table[idx[d] + p]
// ------------------------------------------------------------------------------------------
constexpr int kGradThreads = 256;  // one column per thread: a wave reads 256 contiguous bytes per row
constexpr int kGradMinRows = 64;   // rows per chunk: bounds the partial slabs to n_dirs/64 * P * 8 B

struct GradPlan {
  int col_blocks, rows_per_chunk, n_chunks;
};
static GradPlan grad_plan(int n_dirs, int64_t P) {
  GradPlan g;
  g.col_blocks = (int)((P + kGradThreads - 1) / kGradThreads);
  // aim for ~1024 workgroups (4 per CU) without letting the slab count explode
  const int target_chunks = std::max(1, 1024 / std::max(1, g.col_blocks));
  g.rows_per_chunk = std::max(kGradMinRows, (n_dirs + target_chunks - 1) / target_chunks);
  g.n_chunks = (n_dirs + g.rows_per_chunk - 1) / g.rows_per_chunk;
  return g;
}

int64_t grad_workspace_bytes(int n_dirs, int64_t P) {
  if (n_dirs <= 0 || P <= 0) return 0;
  const GradPlan g = grad_plan(n_dirs, P);
  return (int64_t)g.n_chunks * P * (int64_t)sizeof(double);
}

__global__ __launch_bounds__(kGradThreads) void fd_grad_partial_kernel(
    const float* __restrict__ table, int64_t max_idx, const int64_t* __restrict__ idx,
    const double* __restrict__ coef, int n_dirs, int64_t P, int rows_per_chunk,
    double* __restrict__ partial) {
  const int64_t c = (int64_t)blockIdx.x * kGradThreads + threadIdx.x;
  const int chunk = blockIdx.y;
  const int d0 = chunk * rows_per_chunk;
  const int d1 = min(n_dirs, d0 + rows_per_chunk);
  const bool ok = c < P;
  const int64_t cc = ok ? c : 0;
  // an out-of-range offset reads row 0 with a NaN weight: the gradient is poisoned, never a fault
  auto row = [&](int dd, double& w) {
    const int64_t off = idx[dd];
    const bool bad = off < 0 || off > max_idx;
    w = bad ? __builtin_nan("") : coef[dd];
    return table + (bad ? 0 : off);
  };
  double acc0 = 0.0, acc1 = 0.0;
  int d = d0;
  for (; d + 4 <= d1; d += 4) {  // four rows in flight
    double w0, w1, w2, w3;
    const float v0 = row(d, w0)[cc], v1 = row(d + 1, w1)[cc];
    const float v2 = row(d + 2, w2)[cc], v3 = row(d + 3, w3)[cc];
    acc0 = fma(w0, (double)v0, acc0);
    acc1 = fma(w1, (double)v1, acc1);
    acc0 = fma(w2, (double)v2, acc0);
    acc1 = fma(w3, (double)v3, acc1);
  }
  for (; d < d1; ++d) {
    double w;
    const float v = row(d, w)[cc];
    acc0 = fma(w, (double)v, acc0);
  }
  if (ok) partial[(int64_t)chunk * P + c] = acc0 + acc1;
}

__global__ __launch_bounds__(256) void fd_grad_reduce_kernel(const double* __restrict__ partial,
                                                              int n_chunks, int64_t P,
                                                              double* __restrict__ g) {
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P;
       p += (int64_t)gridDim.x * blockDim.x) {
    double s = 0.0;
    for (int c = 0; c < n_chunks; ++c) s += partial[(int64_t)c * P + p];
    g[p] = s;
  }
}

int launch_fd_grad(const float* table, int64_t table_size, const int64_t* idx, const double* coef,
                   int n_dirs, int64_t P, double* g, void* ws, int64_t ws_bytes, hipStream_t stream) {
  const GradPlan pl = grad_plan(n_dirs, P);
  if (ws_bytes < grad_workspace_bytes(n_dirs, P) || ws == nullptr)
    return set_error(FDR_ERR_WORKSPACE, "fd_grad workspace too small");
  double* partial = static_cast<double*>(ws);
  hipLaunchKernelGGL(fd_grad_partial_kernel, dim3(pl.col_blocks, pl.n_chunks), dim3(kGradThreads), 0,
                     stream, table, table_size - P, idx, coef, n_dirs, P, pl.rows_per_chunk, partial);
  int rc = check_launch("fd_grad_partial_kernel");
  if (rc) return rc;
  const int rb = (int)std::min<int64_t>((P + 255) / 256, 2048);
  hipLaunchKernelGGL(fd_grad_reduce_kernel, dim3(rb), dim3(256), 0, stream, partial, pl.n_chunks, P, g);
  return check_launch("fd_grad_reduce_kernel");
}

// ------------------------------------------------------------------------------------------
// Delayed returns (learner/finite_differences.py:66-73, 80-114): the perturbation of return i is
//   lambda_i[p] = fl32( sign_i * fl32(sigma * eps_i[p]) + D_{slot_i}[p] ),  D = dist_map[epoch_i]
// (theta of that epoch minus the current theta; slot < 0: current epoch, D = 0).  Norms and the
// gradient g = sum_i coef_i * lambda_i run over returns, in the fd_grad tiling, f64 accumulation.
// ------------------------------------------------------------------------------------------

__global__ __launch_bounds__(256) void lambda_norm_kernel(LambdaRow R, double* __restrict__ n2) {
  const int i = blockIdx.x;
  bool bad;
  const float* e = R.eps(i, bad);
  const float* d = R.dr(i);
  const int sg = R.sign ? (int)R.sign[i] : 1;
  double acc = 0.0;
  for (int64_t p = threadIdx.x; p < R.P; p += 256) {
    const double v = R.value(e, d, sg, p);
    acc = fma(v, v, acc);
  }
  __shared__ double red[256 / kWave];
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0.0;
    for (int w = 0; w < 256 / kWave; ++w) t += red[w];
    n2[i] = bad ? __builtin_nan("") : t;
  }
}

__global__ __launch_bounds__(kGradThreads) void lambda_grad_partial_kernel(LambdaRow R, const double* __restrict__ coef,
                                                                          int n, int rows_per_chunk,
                                                                          double* __restrict__ partial) {
  const int64_t c = (int64_t)blockIdx.x * kGradThreads + threadIdx.x;
  const int chunk = blockIdx.y;
  const int d0 = chunk * rows_per_chunk, d1 = min(n, d0 + rows_per_chunk);
  const bool ok = c < R.P;
  const int64_t cc = ok ? c : 0;
  double acc0 = 0.0, acc1 = 0.0;
  int i = d0;
  for (; i + 2 <= d1; i += 2) {
    bool b0, b1;
    const float* e0 = R.eps(i, b0);
    const float* e1 = R.eps(i + 1, b1);
    const float v0 = R.value(e0, R.dr(i), R.sign ? (int)R.sign[i] : 1, cc);
    const float v1 = R.value(e1, R.dr(i + 1), R.sign ? (int)R.sign[i + 1] : 1, cc);
    acc0 = fma(b0 ? __builtin_nan("") : coef[i], (double)v0, acc0);
    acc1 = fma(b1 ? __builtin_nan("") : coef[i + 1], (double)v1, acc1);
  }
  for (; i < d1; ++i) {
    bool b;
    const float* e = R.eps(i, b);
    const float v = R.value(e, R.dr(i), R.sign ? (int)R.sign[i] : 1, cc);
    acc0 = fma(b ? __builtin_nan("") : coef[i], (double)v, acc0);
  }
  if (ok) partial[(int64_t)chunk * R.P + c] = acc0 + acc1;
}

int launch_lambda_norms(const LambdaRow& R, int n, double* n2, hipStream_t stream) {
  if (n == 0) return FDR_OK;
  hipLaunchKernelGGL(lambda_norm_kernel, dim3(n), dim3(256), 0, stream, R, n2);
  return check_launch("lambda_norm_kernel");
}

int launch_lambda_grad(const LambdaRow& R, const double* coef, int n, double* g, void* ws, int64_t ws_bytes,
                       hipStream_t stream) {
  const GradPlan pl = grad_plan(n, R.P);
  if (ws_bytes < grad_workspace_bytes(n, R.P) || ws == nullptr)
    return set_error(FDR_ERR_WORKSPACE, "fd_grad workspace too small");
  double* partial = static_cast<double*>(ws);
  hipLaunchKernelGGL(lambda_grad_partial_kernel, dim3(pl.col_blocks, pl.n_chunks), dim3(kGradThreads), 0, stream,
                     R, coef, n, pl.rows_per_chunk, partial);
  int rc = check_launch("lambda_grad_partial_kernel");
  if (rc) return rc;
  const int rb = (int)std::min<int64_t>((R.P + 255) / 256, 2048);
  hipLaunchKernelGGL(fd_grad_reduce_kernel, dim3(rb), dim3(256), 0, stream, partial, pl.n_chunks, R.P, g);
  return check_launch("fd_grad_reduce_kernel");
}

// ------------------------------------------------------------------------------------------
// DSGD (dsgd/dynamic_sgd.py:19-39)
// ------------------------------------------------------------------------------------------
constexpr int kDsgdBlocks = 256;
int64_t dsgd_workspace_bytes(int64_t) { return (int64_t)(2 * kDsgdBlocks + 8) * sizeof(double); }

__device__ double block_sum_256(double v, double* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, j = threadIdx.x & 63;
  if (j == 0) red[w] = v;
  __syncthreads();
  const double s = red[0] + red[1] + red[2] + red[3];
  __syncthreads();
  return s;
}

__global__ __launch_bounds__(256) void dsgd_norm_kernel(const double* __restrict__ g, int64_t P,
                                                         double* __restrict__ part) {
  __shared__ double red[4];
  double s = 0.0;
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P;
       p += (int64_t)gridDim.x * blockDim.x) {
    const float gr = (float)(-g[p]);  // set_grad_from_flat casts to f32 (policy.py:68)
    s += (double)gr * (double)gr;
  }
  s = block_sum_256(s, red);
  if (threadIdx.x == 0) part[blockIdx.x] = s;
}

__global__ __launch_bounds__(256) void dsgd_apply_kernel(float* __restrict__ theta,
                                                          const double* __restrict__ g, int64_t P,
                                                          double lr, double lr_scale,
                                                          double* __restrict__ part) {
#pragma clang fp contract(off)
  __shared__ double red[4];
  // every block re-reduces the norm partials in the same fixed order -> identical coef
  double ss = 0.0;
  for (int i = 0; i < (int)gridDim.x; ++i) ss += part[i];
  const float norm = (float)sqrt(ss);  // flat_grad.norm().item() (dynamic_sgd.py:27)
  double s = 0.0;
  if (norm > 0.f) {
    const double coef = lr * sqrt((double)P) * lr_scale / (double)norm;  // dynamic_sgd.py:30,51
    const float c32 = (float)coef;
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P;
         p += (int64_t)gridDim.x * blockDim.x) {
      const float gr = (float)(-g[p]);
      const float old = theta[p];
      const float nw = old - c32 * gr;  // p.sub_(coef * grad_slice) (dynamic_sgd.py:36)
      theta[p] = nw;
      const float dd = old - nw;
      s += (double)dd * (double)dd;
    }
  }
  s = block_sum_256(s, red);
  if (threadIdx.x == 0) part[gridDim.x + blockIdx.x] = s;
  if (blockIdx.x == 0 && threadIdx.x == 0) part[2 * gridDim.x] = (double)norm;
}

__global__ void dsgd_final_kernel(const double* __restrict__ part, int nb, double* __restrict__ out) {
  if (threadIdx.x == 0) {
    double s = 0.0;
    for (int i = 0; i < nb; ++i) s += part[nb + i];
    out[0] = sqrt(s);
    out[1] = part[2 * nb];
  }
}

int launch_dsgd(float* theta, const double* g, int64_t P, double lr, double lr_scale, double* out,
                void* ws, int64_t ws_bytes, hipStream_t stream) {
  if (ws == nullptr || ws_bytes < dsgd_workspace_bytes(P))
    return set_error(FDR_ERR_WORKSPACE, "dsgd workspace too small");
  double* part = static_cast<double*>(ws);
  const int nb = (int)std::min<int64_t>(kDsgdBlocks, (P + 255) / 256);
  hipLaunchKernelGGL(dsgd_norm_kernel, dim3(nb), dim3(256), 0, stream, g, P, part);
  int rc = check_launch("dsgd_norm_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(dsgd_apply_kernel, dim3(nb), dim3(256), 0, stream, theta, g, P, lr, lr_scale, part);
  rc = check_launch("dsgd_apply_kernel");
  if (rc) return rc;
  hipLaunchKernelGGL(dsgd_final_kernel, dim3(1), dim3(64), 0, stream, part, nb, out);
  return check_launch("dsgd_final_kernel");
}

}  // namespace fdr

namespace fdr {

// ------------------------------------------------------------------------------------------
// Strategy distances / novelty (utils/math_helpers.py:147-222, strategy/*): one 256-thread block
// per strategy i holds it in LDS; each wave walks archive entries h = w, w+4, ..., its lanes over
// the probe states z, f64 accumulation, fixed reduction order.  d[i][h] = mean_z term(a_iz, b_hz).
// ------------------------------------------------------------------------------------------
constexpr int kNovThreads = 256;
constexpr int kNovMaxZD = 8192;  // floats of one strategy held in LDS (32 KiB)

__global__ __launch_bounds__(kNovThreads) void strategy_dist_kernel(const float* __restrict__ S, const float* __restrict__ B,
                                                                   int H, int Z, int D, int kind, double* __restrict__ dists,
                                                                   double* __restrict__ min_d, int32_t* __restrict__ arg) {
  __shared__ float a[kNovMaxZD];
  __shared__ double wmin[kNovThreads / kWave];
  __shared__ int warg[kNovThreads / kWave];
  const int i = blockIdx.x, wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int ZD = Z * D;
  for (int t = threadIdx.x; t < ZD; t += kNovThreads) a[t] = S[(int64_t)i * ZD + t];
  __syncthreads();
  double best = __builtin_inf();
  int best_h = -1;
  const int k = D / 2;
  for (int h = wave; h < H; h += kNovThreads / kWave) {
    const float* b = B + (int64_t)h * ZD;
    double acc = 0.0;
    for (int z = lane; z < Z; z += kWave) {
      const float* az = a + z * D;
      const float* bz = b + z * D;
      double term = 0.0;
      if (kind == FDR_DIST_TVD) {
        for (int d = 0; d < D; ++d) term += fabs((double)az[d] - (double)bz[d]);
      } else if (kind == FDR_DIST_L2) {
        for (int d = 0; d < D; ++d) { const double df = (double)bz[d] - (double)az[d]; term += df * df; }
        term = sqrt(term);
      } else {  // FDR_DIST_W2: [mean | std]
        for (int d = 0; d < k; ++d) {
          const double dm = (double)az[d] - (double)bz[d];
          const double s1 = az[k + d], s2 = bz[k + d];
          term += dm * dm + (s1 + s2 - 2.0 * sqrt(s1 * s2));
        }
      }
      acc += term;
    }
    acc = wave_sum(acc) / (double)Z;
    if (dists && lane == 0) dists[(int64_t)i * H + h] = acc;
    if (acc < best) { best = acc; best_h = h; }  // h increases: first minimum kept
  }
  if (lane == 0) { wmin[wave] = best; warg[wave] = best_h; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double m = __builtin_inf();
    int am = -1;
    for (int w = 0; w < kNovThreads / kWave; ++w)
      if (warg[w] >= 0 && (wmin[w] < m || (wmin[w] == m && warg[w] < am))) { m = wmin[w]; am = warg[w]; }
    if (min_d) min_d[i] = m;
    if (arg) arg[i] = am;
  }
}

int launch_strategy_dist(const float* S, int n, const float* B, int H, int Z, int D, int kind, double* dists,
                         double* min_d, int32_t* arg, hipStream_t stream) {
  if ((int64_t)Z * D > kNovMaxZD) return set_error(FDR_ERR_UNSUPPORTED, "Z * D exceeds 8192");
  if (n == 0) return FDR_OK;
  hipLaunchKernelGGL(strategy_dist_kernel, dim3(n), dim3(kNovThreads), 0, stream, S, B, H, Z, D, kind, dists, min_d, arg);
  return check_launch("strategy_dist_kernel");
}

}  // namespace fdr

namespace fdr {

// ------------------------------------------------------------------------------------------
// BatchNorm running-stat refresh of the DiscretePolicy (policies/policy.py:31-34 compute_vbn,
// policies/discrete.py:34-48): one train-mode pass of the buffer; each BN normalises with its batch
// statistics (biased variance) and folds mean / unbiased variance into its running stats.
// ------------------------------------------------------------------------------------------
constexpr float kVbnEps = 1e-5f;

__global__ __launch_bounds__(256) void col_stats_kernel(const float* __restrict__ X, int n, int C,
                                                        double* __restrict__ mean, double* __restrict__ var) {
  const int c = blockIdx.x;
  __shared__ double red[256 / kWave];
  __shared__ double mu;
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += X[(int64_t)i * C + c];
  s = wave_sum(s);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) mu = (red[0] + red[1] + red[2] + red[3]) / n;
  __syncthreads();
  double q = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    const double d = X[(int64_t)i * C + c] - mu;
    q = fma(d, d, q);
  }
  q = wave_sum(q);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = q;
  __syncthreads();
  if (threadIdx.x == 0) {
    mean[c] = mu;
    var[c] = (red[0] + red[1] + red[2] + red[3]) / n;  // biased: what train-mode BN normalises with
  }
}

// Y[i][j] = relu(b_j + sum_k W[j][k] * BN_batch(X[i][k]))
__global__ __launch_bounds__(256) void bn_linear_relu_kernel(const float* __restrict__ X, int n, int Cin,
                                                             const double* __restrict__ mean, const double* __restrict__ var,
                                                             const float* __restrict__ bw, const float* __restrict__ bb,
                                                             const float* __restrict__ W, const float* __restrict__ b,
                                                             int Cout, float* __restrict__ Y) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= (int64_t)n * Cout) return;
  const int i = (int)(t / Cout), j = (int)(t % Cout);
  float acc = b[j];
  for (int k = 0; k < Cin; ++k) {
    const float inv = 1.f / sqrtf((float)var[k] + kVbnEps);
    const float xn = ((X[(int64_t)i * Cin + k] - (float)mean[k]) * inv) * bw[k] + bb[k];
    acc = fmaf(W[j * Cin + k], xn, acc);
  }
  Y[t] = acc > 0.f ? acc : 0.f;
}

__global__ void bn_running_update_kernel(int C, int n, float momentum, const double* __restrict__ mean,
                                         const double* __restrict__ var, float* __restrict__ rm,
                                         float* __restrict__ rv) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float unb = (float)(var[c] * (double)n / (double)(n - 1));
  rm[c] = momentum * (float)mean[c] + (1.f - momentum) * rm[c];
  rv[c] = momentum * unb + (1.f - momentum) * rv[c];
}

int64_t bn_refresh_workspace_bytes(int n) { return (int64_t)n * 64 * 4 * 2 + 6 * 64 * 8 + 256; }

int launch_bn_refresh(int n_in, const float* theta, const float* x, int n, float momentum, float* rm, float* rv,
                      void* ws, int64_t ws_bytes, hipStream_t stream) {
  if (ws_bytes < bn_refresh_workspace_bytes(n) || !ws) return set_error(FDR_ERR_WORKSPACE, "bn refresh workspace too small");
  constexpr int H = kHidden;
  float* h1 = static_cast<float*>(ws);
  float* h2 = h1 + (int64_t)n * H;
  double* st = reinterpret_cast<double*>(h2 + (int64_t)n * H);  // [3 layers][mean 64 | var 64]
  // theta layout (policies/discrete.py:34-48, parameters() order)
  const float* bn0w = theta;
  const float* bn0b = bn0w + n_in;
  const float* l1w = bn0b + n_in;
  const float* l1b = l1w + H * n_in;
  const float* bn1w = l1b + H;
  const float* bn1b = bn1w + H;
  const float* l2w = bn1b + H;
  const float* l2b = l2w + H * H;
  const float* bn2w = l2b + H;
  (void)bn2w;
  const int nb = (int)(((int64_t)n * H + 255) / 256);
  hipLaunchKernelGGL(col_stats_kernel, dim3(n_in), dim3(256), 0, stream, x, n, n_in, st, st + 64);
  hipLaunchKernelGGL(bn_linear_relu_kernel, dim3(nb), dim3(256), 0, stream, x, n, n_in, st, st + 64, bn0w, bn0b, l1w,
                     l1b, H, h1);
  hipLaunchKernelGGL(col_stats_kernel, dim3(H), dim3(256), 0, stream, h1, n, H, st + 128, st + 192);
  hipLaunchKernelGGL(bn_linear_relu_kernel, dim3(nb), dim3(256), 0, stream, h1, n, H, st + 128, st + 192, bn1w, bn1b,
                     l2w, l2b, H, h2);
  hipLaunchKernelGGL(col_stats_kernel, dim3(H), dim3(256), 0, stream, h2, n, H, st + 256, st + 320);
  hipLaunchKernelGGL(bn_running_update_kernel, dim3(1), dim3(64), 0, stream, n_in, n, momentum, st, st + 64, rm, rv);
  hipLaunchKernelGGL(bn_running_update_kernel, dim3(1), dim3(64), 0, stream, H, n, momentum, st + 128, st + 192,
                     rm + n_in, rv + n_in);
  hipLaunchKernelGGL(bn_running_update_kernel, dim3(1), dim3(64), 0, stream, H, n, momentum, st + 256, st + 320,
                     rm + n_in + H, rv + n_in + H);
  return check_launch("bn refresh kernels");
}

}  // namespace fdr

namespace fdr {

// ------------------------------------------------------------------------------------------
// Fused learner step (fdr_fd_grad_fused / fdr_fd_step): the weighting, the noise-weighted gradient and
// its chunk combine in ONE launch -- and, single-process with P <= 65536, DSGD in the same launch.
//
// fd_grad_fused_kernel, grid (column blocks of 256, row chunks), 256 threads:
//   1. the chunk's first 64 table rows are requested up front (they do not depend on the weights);
//   2. meanwhile the workgroup forms the weights of ITS directions: the z-score statistics over all
//      rewards (f64, the same fixed-order tree in every workgroup, so all agree bit for bit), or
//      precomputed centred-rank weights, or the raw moments form; coefficients in LDS (NaN for a row
//      whose table offset is out of range: the gradient is poisoned, the table never over-read);
//   3. f64 column sums over the chunk's rows;
//   4. chunk partials are combined in the same launch: slab store -> agent-scope release -> ticket on
//      the column block's counter; the last arriver acquires and sums the slabs in chunk order
//      (deterministic and placement-independent: cdna_hip_programming.md Guideline 16, counter form)
//      and resets the counter;
//   5. (fdr_fd_step) each column block's owner publishes sum fl32(-g)^2 of its columns and takes a
//      ticket on the DSGD counter; the last owner forms ||fl32(-g)|| in column-block order and applies
//      the update to all of theta (dynamic_sgd.py:19-39), then ||d theta||.
// Counters must be zero before the first launch on a workspace (the caller zeroes the leading counter
// block once); every launch leaves them zero.
// ------------------------------------------------------------------------------------------
constexpr int kFusedRows = 64;       // table rows per pass: loads in flight per thread
constexpr int kFusedMaxRows = 1024;  // directions per chunk (LDS coefficient arrays)

struct FdArgs {
  const float* table;
  int64_t max_idx;
  const int64_t* idx;    // per LOCAL lane [n_dirs * lpd]; direction d's row starts at idx[d * lpd]
  int n_dirs;
  int64_t P;
  const double* r_all;   // [n_all]; MOMENTS: the local lanes' rewards only
  int n_all;             // lanes over all ranks
  double pr;
  int lo;                // this rank's first global lane
  const int8_t* sign;    // [n_dirs * lpd] (local lanes)
  const double* n2;      // [n_dirs * lpd]
  const double* w;       // centred-rank weights of the local lanes
  int lpd;
  float sigma;
  int rows_per_chunk, n_chunks, col_blocks;
  double* partial;       // [n_chunks][P] (x2 in MOMENTS mode)
  unsigned* cnt;         // [col_blocks] chunk tickets, [col_blocks] the DSGD ticket
  double* out;           // g [P]; MOMENTS: [A | B | n_local | r' slots [n_all]]
  double* gsq;           // [col_blocks] sum fl32(-g)^2 per column block (fdr_fd_step), or NULL
};

// handed-off payload is stored write-through (sc1: an agent-scope relaxed atomic store), so the ticket needs
// no release fence (cdna_hip_programming.md Guideline 16 R1)
__device__ __forceinline__ void store_wt(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), __builtin_bit_cast(unsigned long long, v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void publish_and_ticket(unsigned* cnt, unsigned need, int* s_flag) {
  // every storing wave drains its sc1 stores, the workgroup meets, ONE lane takes the ticket
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    const unsigned prev = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = prev == need - 1;
    if (last) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    *s_flag = last;
  }
  __syncthreads();
}

// sum over k < n of base[k * stride] in k order, 16 loads in flight
__device__ __forceinline__ double sum_slabs(const double* base, int64_t stride, int n) {
  double s = 0.0;
  int k = 0;
  for (; k + 16 <= n; k += 16) {
    double v[16];
#pragma unroll
    for (int e = 0; e < 16; ++e) v[e] = base[(int64_t)(k + e) * stride];
#pragma unroll
    for (int e = 0; e < 16; ++e) s += v[e];
  }
  for (; k < n; ++k) s += base[(int64_t)k * stride];
  return s;
}

template <int MODE>
__global__ __launch_bounds__(256) void fd_grad_fused_kernel(FdArgs a) {
  __shared__ double cA[kFusedMaxRows];
  __shared__ double cB[MODE == FDR_WEIGHT_MOMENTS ? kFusedMaxRows : 1];
  __shared__ double red[4];
  __shared__ int s_flag;
  const int tid = threadIdx.x;
  const int chunk = blockIdx.y, cb = blockIdx.x;
  const int d0 = chunk * a.rows_per_chunk, d1 = min(a.n_dirs, d0 + a.rows_per_chunk);
  const int64_t P = a.P;
  const int64_t col = (int64_t)cb * 256 + tid;
  const bool ok = col < P;
  const int64_t cc = ok ? col : 0;
  auto row_off = [&](int d) {
    const int64_t off = a.idx[(int64_t)d * a.lpd];
    return (off < 0 || off > a.max_idx) ? (int64_t)-1 : off;
  };
  float v[kFusedRows];
  // Row offsets: lane l of every wave loads row r0 + l's offset (one vector load; clamped into the chunk,
  // an invalid offset reads row 0 -- its coefficient is NaN) and the pass takes row r's through
  // v_readlane, so the table address is scalar base + column.  (Per-row scalar loads were each followed
  // by an lgkmcnt(0) wait: 64 dependent round trips before the last row was even requested.)
  auto row_offsets = [&](int r0) {
    int64_t off = a.idx[(int64_t)min(r0 + (tid & 63), d1 - 1) * a.lpd];
    return (off < 0 || off > a.max_idx) ? (int64_t)0 : off;
  };
  auto load_pass = [&](int r0, int64_t offl) {
    const unsigned lo = (unsigned)offl, hi = (unsigned)((uint64_t)offl >> 32);
#pragma unroll
    for (int r = 0; r < kFusedRows; ++r) {
      const int64_t o = (int64_t)(((uint64_t)(unsigned)__builtin_amdgcn_readlane((int)hi, r) << 32) |
                                  (unsigned)__builtin_amdgcn_readlane((int)lo, r));
      const float x = a.table[o + cc];  // unconditional (rows past the chunk repeat its last row): no branch
      v[r] = r0 + r < d1 ? x : 0.f;
    }
  };
  const int64_t off0 = row_offsets(d0);  // first in the vmcnt order: the table loads wait only for it
  // Load order matters: vmcnt retires loads in issue order, so the statistics' inputs are requested
  // BEFORE the chunk's 64 table rows -- consuming them then waits only for themselves, and the table
  // rows stay in flight through the statistics (issued after the rows, they would wait for all 64).
  // this thread's first direction's per-lane inputs
  constexpr int kMaxLpd = 4;
  const int dmine = d0 + tid;
  // Branch-free (clamped indices, selects): a load under a condition ends its basic block with a full
  // vmcnt(0) wait, which serialised these ~30 loads into as many L2 round trips (measured: the kernel's
  // 24 us vs 10.5 us for the bare 50 MB stream, tools/learner_bench.py).
  double xin[kMaxLpd], vin[kMaxLpd];
  const int roff = MODE == FDR_WEIGHT_MOMENTS ? 0 : a.lo;  // MOMENTS: r_all holds the local lanes only
  {
    const int nloc = max(1, (d1 - d0) * a.lpd);  // this chunk's local lanes: [d0 * lpd, d1 * lpd)
    int sg[kMaxLpd];
    double n2v[kMaxLpd], xv[kMaxLpd];
#pragma unroll
    for (int k = 0; k < kMaxLpd; ++k) {
      const int i = d0 * a.lpd + min((dmine - d0) * a.lpd + k, nloc - 1);
      sg[k] = a.sign[i];
      n2v[k] = a.n2[i];
      if constexpr (MODE == FDR_WEIGHT_CENTERED_RANK) xv[k] = a.w[i];
      else xv[k] = a.r_all[roff + i];
    }
#pragma unroll
    for (int k = 0; k < kMaxLpd; ++k) {
      // computed unconditionally (an unused lane's 0/0 is selected away): a division under the condition
      // lets the compiler sink the n2 load into the branch, behind a vmcnt(0)
      const double q = (double)sg[k] * (double)a.sigma / n2v[k];
      const bool use = dmine < d1 && k < a.lpd && sg[k] != 0;
      vin[k] = use ? q : 0.0;
      xin[k] = use ? (MODE == FDR_WEIGHT_CENTERED_RANK ? xv[k] : xv[k] - a.pr) : 0.0;
    }
  }
  double mean = 0.0, sd = 0.0;
  // one load pass, the values kept in registers for the second (same per-thread order as a reload)
  constexpr int kR = MODE == FDR_WEIGHT_ZSCORE ? 16 : 1;
  double xr[kR];
  if constexpr (MODE == FDR_WEIGHT_ZSCORE) {
#pragma unroll
    for (int k = 0; k < kR; ++k) xr[k] = a.r_all[min(tid + 256 * k, a.n_all - 1)];  // clamped: no branches
#pragma unroll
    for (int k = 0; k < kR; ++k) xr[k] = tid + 256 * k < a.n_all ? xr[k] - a.pr : 0.0;
  }
  load_pass(d0, off0);  // the table rows: in flight from here through the statistics and the coefficients
  if constexpr (MODE == FDR_WEIGHT_ZSCORE) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < kR; ++k)
      if (tid + 256 * k < a.n_all) s += xr[k];
    for (int i = tid + 256 * kR; i < a.n_all; i += 256) s += a.r_all[i] - a.pr;
    mean = block_sum_256(s, red) / (double)a.n_all;
    double q = 0.0;
#pragma unroll
    for (int k = 0; k < kR; ++k)
      if (tid + 256 * k < a.n_all) {
        const double d = xr[k] - mean;
        q += d * d;
      }
    for (int i = tid + 256 * kR; i < a.n_all; i += 256) {
      const double d = (a.r_all[i] - a.pr) - mean;
      q += d * d;
    }
    sd = sqrt(block_sum_256(q, red) / (double)a.n_all);
  }
  auto weight = [&](double x) {
    if constexpr (MODE == FDR_WEIGHT_ZSCORE) return sd == 0.0 ? x : (x - mean) / sd;  // math_helpers.py:127-134
    else return x;
  };
  // MOMENTS: c = sum_k (r'_k - r'_0) v_k + r'_0 b, b = sum_k v_k -- the same value in real arithmetic, but an
  // antithetic pair (v_1 = -v_0, so b = 0 exactly) gives c = (r'_1 - r'_0) v_1 with the difference exact
  // (Sterbenz) instead of r'_0 v_0 + r'_1 v_1, whose products cancel when the returns are near-constant
  if (dmine < d1 && a.lpd <= kMaxLpd) {
    double c = 0.0, b = 0.0;
    const double x0 = MODE == FDR_WEIGHT_MOMENTS ? xin[0] : 0.0;
#pragma unroll
    for (int k = 0; k < kMaxLpd; ++k)
      if (k < a.lpd && vin[k] != 0.0) {
        c += weight(xin[k] - x0) * vin[k];
        b += vin[k];
      }
    if constexpr (MODE == FDR_WEIGHT_MOMENTS) c = fma(x0, b, c);
    if (row_off(dmine) < 0) c = b = __builtin_nan("");
    cA[dmine - d0] = c;
    if constexpr (MODE == FDR_WEIGHT_MOMENTS) cB[dmine - d0] = b;
  }
  for (int d = d0 + tid + (a.lpd <= kMaxLpd ? 256 : 0); d < d1; d += 256) {  // further directions of this thread
    double c = 0.0, b = 0.0, x0 = 0.0;
    for (int k = 0; k < a.lpd; ++k) {
      const int i = d * a.lpd + k;
      const int sg = a.sign[i];
      if (sg == 0) continue;
      const double vi = (double)sg * (double)a.sigma / a.n2[i];
      double x;
      if constexpr (MODE == FDR_WEIGHT_CENTERED_RANK) x = a.w[i];
      else x = a.r_all[roff + i] - a.pr;
      if (MODE == FDR_WEIGHT_MOMENTS && k == 0) x0 = x;  // as above
      c += weight(x - x0) * vi;
      b += vi;
    }
    if constexpr (MODE == FDR_WEIGHT_MOMENTS) c = fma(x0, b, c);
    if (row_off(d) < 0) c = b = __builtin_nan("");
    cA[d - d0] = c;
    if constexpr (MODE == FDR_WEIGHT_MOMENTS) cB[d - d0] = b;
  }
  __syncthreads();

  double acc0 = 0.0, acc1 = 0.0, bcc0 = 0.0, bcc1 = 0.0;
  for (int r0 = d0; r0 < d1; r0 += kFusedRows) {
    if (r0 != d0) load_pass(r0, row_offsets(r0));
#pragma unroll
    for (int r = 0; r < kFusedRows; r += 2) {
      if (r0 + r < d1) {
        acc0 = fma(cA[r0 + r - d0], (double)v[r], acc0);
        if constexpr (MODE == FDR_WEIGHT_MOMENTS) bcc0 = fma(cB[r0 + r - d0], (double)v[r], bcc0);
      }
      if (r0 + r + 1 < d1) {
        acc1 = fma(cA[r0 + r + 1 - d0], (double)v[r + 1], acc1);
        if constexpr (MODE == FDR_WEIGHT_MOMENTS) bcc1 = fma(cB[r0 + r + 1 - d0], (double)v[r + 1], bcc1);
      }
    }
  }
  const double ga = acc0 + acc1, gb = bcc0 + bcc1;

  bool owner = true;  // this workgroup holds the final g of its column block
  double gfin = ga;
  if (a.n_chunks == 1) {
    if (ok) {
      store_wt(a.out + col, ga);
      if constexpr (MODE == FDR_WEIGHT_MOMENTS) a.out[P + col] = gb;
    }
  } else {
    if (ok) {
      store_wt(a.partial + (int64_t)chunk * P + col, ga);
      if constexpr (MODE == FDR_WEIGHT_MOMENTS) store_wt(a.partial + ((int64_t)a.n_chunks + chunk) * P + col, gb);
    }
    publish_and_ticket(a.cnt + cb, (unsigned)a.n_chunks, &s_flag);
    owner = s_flag != 0;
    if (owner) {
      double sa = 0.0, sb = 0.0;
      if (ok) {
        sa = sum_slabs(a.partial + col, P, a.n_chunks);
        store_wt(a.out + col, sa);  // read by the DSGD workgroup of fdr_fd_step
        if constexpr (MODE == FDR_WEIGHT_MOMENTS) {
          sb = sum_slabs(a.partial + (int64_t)a.n_chunks * P + col, P, a.n_chunks);
          a.out[P + col] = sb;
        }
      }
      gfin = sa;
      if (tid == 0) __hip_atomic_store(a.cnt + cb, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  if constexpr (MODE == FDR_WEIGHT_MOMENTS) {
    if (cb == 0 && chunk == 0) {
      // [n_local | r' slots]: this rank's r' at its global lanes, 0 elsewhere -- the all-reduce's sum is then
      // every rank's r' (x + 0 = x exactly) and the lane count, from which the DSGD launch forms the z-score
      // statistics in two passes as standardize_arr does (a one-pass sum r'^2 / n - m^2 cancels when the
      // returns are near-constant)
      const int n_local = a.n_dirs * a.lpd;
      double* slots = a.out + 2 * P + 1;
      for (int i = tid; i < a.n_all; i += 256) {
        const int k = i - a.lo;
        slots[i] = (k >= 0 && k < n_local) ? a.r_all[k] - a.pr : 0.0;
      }
      if (tid == 0) a.out[2 * P] = (double)n_local;
    }
  } else {
    if (a.gsq && owner) {  // fdr_fd_step: this column block's sum fl32(-g)^2 for the DSGD launch
      const float gr = ok ? (float)(-gfin) : 0.f;  // set_grad_from_flat casts to f32 (policy.py:68)
      const double part = block_sum_256((double)gr * (double)gr, red);
      if (tid == 0) a.gsq[cb] = part;
    }
  }
}

// DSGD after fd_grad_fused (fdr_fd_step): one 256-column block per workgroup.  Every workgroup forms
// ||fl32(-g)|| from the per-column-block partials in the same order, updates its columns
// (dynamic_sgd.py:19-39), writes theta_new to the history slot (the learner's policy_history,
// finite_differences.py:75-78) and its sum of squared updates; the last workgroup (ticket) forms ||d theta||.
__global__ __launch_bounds__(256) void dsgd_apply_cb_kernel(float* __restrict__ theta, const double* __restrict__ g,
                                                            int64_t P, const double* __restrict__ gsq, int col_blocks,
                                                            double lr, double lr_scale, float* __restrict__ hist,
                                                            double* __restrict__ upart, unsigned* __restrict__ cnt,
                                                            double* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ double red[4];
  __shared__ double gs[256];
  __shared__ int s_flag;
  const int tid = threadIdx.x, cb = blockIdx.x;
  const int64_t p = (int64_t)cb * 256 + tid;
  const double gv = p < P ? g[p] : 0.0;
  const float old = p < P ? theta[p] : 0.f;
  double ss = 0.0;
  for (int k0 = 0; k0 < col_blocks; k0 += 256) {
    __syncthreads();
    if (k0 + tid < col_blocks) gs[tid] = gsq[k0 + tid];
    __syncthreads();
    for (int k = 0; k < min(256, col_blocks - k0); ++k) ss += gs[k];
  }
  const float norm = (float)sqrt(ss);  // flat_grad.norm().item() (dynamic_sgd.py:27)
  double u = 0.0;
  float nw = old;
  if (norm > 0.f) {
    const double coef = lr * sqrt((double)P) * lr_scale / (double)norm;  // dynamic_sgd.py:30,51
    const float c32 = (float)coef;
    const float g32 = (float)(-gv);
    nw = old - c32 * g32;  // p.sub_(coef * grad_slice) (dynamic_sgd.py:36)
    const float dd = old - nw;
    u = p < P ? (double)dd * (double)dd : 0.0;
  }
  if (p < P) {
    theta[p] = nw;
    if (hist) hist[p] = nw;
  }
  u = block_sum_256(u, red);
  if (tid == 0) store_wt(upart + cb, u);
  publish_and_ticket(cnt, (unsigned)col_blocks, &s_flag);
  if (s_flag) {
    double t = 0.0;
    for (int k0 = 0; k0 < col_blocks; k0 += 256) {
      __syncthreads();
      if (k0 + tid < col_blocks) gs[tid] = upart[k0 + tid];
      __syncthreads();
      for (int k = 0; k < min(256, col_blocks - k0); ++k) t += gs[k];
    }
    if (tid == 0) {
      out[0] = sqrt(t);
      out[1] = (double)norm;
      __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

struct FusedPlan {
  int col_blocks, rows_per_chunk, n_chunks;
};
static FusedPlan fused_plan(int n_dirs, int64_t P) {
  FusedPlan f;
  f.col_blocks = (int)((P + 255) / 256);
  const int target_chunks = std::max(1, 1024 / std::max(1, f.col_blocks));
  const int rows = std::max(kFusedRows, (n_dirs + target_chunks - 1) / target_chunks);
  f.rows_per_chunk = std::min(kFusedMaxRows, (rows + kFusedRows - 1) / kFusedRows * kFusedRows);
  f.n_chunks = std::max(1, (n_dirs + f.rows_per_chunk - 1) / f.rows_per_chunk);
  return f;
}

// workspace: [counters: col_blocks + 1 u32, padded to 256 B][gsq][update partials][rank weights][partial slabs]
static int64_t pad256(int64_t b) { return (b + 255) / 256 * 256; }
int64_t fused_counter_bytes(int n_dirs, int64_t P) {
  const FusedPlan f = fused_plan(std::max(1, n_dirs), P);
  return pad256((int64_t)(f.col_blocks + 1) * 4);
}
int64_t fused_workspace_bytes(int n_dirs, int n_local, int64_t P, int mode) {
  if (n_dirs < 0 || P <= 0) return -1;
  const FusedPlan f = fused_plan(std::max(1, n_dirs), P);
  const int64_t slabs = f.n_chunks > 1 ? (int64_t)f.n_chunks * P * 8 * (mode == FDR_WEIGHT_MOMENTS ? 2 : 1) : 0;
  return fused_counter_bytes(n_dirs, P) + 2 * pad256((int64_t)f.col_blocks * 8) +
         pad256((int64_t)std::max(0, n_local) * 8) + slabs;
}

// centred rank (build extension; the standard ES transform): rank of r_i among all n_all returns,
// ties broken by lane index; w_i = rank_i / (n_all - 1) - 0.5.  Each thread counts over LDS tiles.
__global__ __launch_bounds__(256) void rank_weights_kernel(const double* __restrict__ r_all, int n_all, int lo,
                                                           int n_local, double* __restrict__ w) {
  __shared__ double tile[2048];
  const int i = blockIdx.x * 256 + threadIdx.x;
  const int gi = lo + (i < n_local ? i : 0);
  const double ri = r_all[gi];
  int rank = 0;
  for (int t0 = 0; t0 < n_all; t0 += 2048) {
    const int tn = min(2048, n_all - t0);
    __syncthreads();
    for (int k = threadIdx.x; k < tn; k += 256) tile[k] = r_all[t0 + k];
    __syncthreads();
    for (int k = 0; k < tn; ++k) {
      const double rk = tile[k];
      rank += (rk < ri || (rk == ri && t0 + k < gi)) ? 1 : 0;
    }
  }
  if (i < n_local) w[i] = n_all > 1 ? (double)rank / (double)(n_all - 1) - 0.5 : 0.0;
}

int launch_fd_grad_fused(const float* table, int64_t table_size, const int64_t* idx, int n_dirs, int64_t P,
                         const double* r_all, int n_all, double pr, int lo, const int8_t* sign, const double* n2,
                         int lpd, float sigma, int mode, double* out, float* theta, double lr, double lr_scale,
                         float* hist, double* dsgd_out, void* ws, int64_t ws_bytes, hipStream_t stream) {
  const int n_local = n_dirs * lpd;
  if (!ws || ws_bytes < fused_workspace_bytes(n_dirs, n_local, P, mode))
    return set_error(FDR_ERR_WORKSPACE, "fd_grad_fused workspace too small");
  const FusedPlan f = fused_plan(n_dirs, P);
  char* w = static_cast<char*>(ws);
  const int64_t cnt_b = fused_counter_bytes(n_dirs, P);
  const int64_t cb_b = pad256((int64_t)f.col_blocks * 8);
  const int64_t w_b = pad256((int64_t)n_local * 8);
  FdArgs a{};
  a.table = table;
  a.max_idx = table_size - P;
  a.idx = idx;
  a.n_dirs = n_dirs;
  a.P = P;
  a.r_all = r_all;
  a.n_all = n_all;
  a.pr = pr;
  a.lo = lo;
  a.sign = sign;
  a.n2 = n2;
  a.lpd = lpd;
  a.sigma = sigma;
  a.rows_per_chunk = f.rows_per_chunk;
  a.n_chunks = f.n_chunks;
  a.col_blocks = f.col_blocks;
  a.cnt = reinterpret_cast<unsigned*>(w);
  double* gsq = reinterpret_cast<double*>(w + cnt_b);
  double* upart = reinterpret_cast<double*>(w + cnt_b + cb_b);
  a.gsq = theta ? gsq : nullptr;
  a.w = reinterpret_cast<double*>(w + cnt_b + 2 * cb_b);
  a.partial = reinterpret_cast<double*>(w + cnt_b + 2 * cb_b + w_b);
  a.out = out;
  const dim3 grid(f.col_blocks, f.n_chunks);
  switch (mode) {
    case FDR_WEIGHT_ZSCORE:
      hipLaunchKernelGGL(fd_grad_fused_kernel<FDR_WEIGHT_ZSCORE>, grid, dim3(256), 0, stream, a);
      break;
    case FDR_WEIGHT_CENTERED_RANK:
      hipLaunchKernelGGL(rank_weights_kernel, dim3((n_local + 255) / 256), dim3(256), 0, stream, r_all, n_all, lo,
                         n_local, const_cast<double*>(a.w));
      hipLaunchKernelGGL(fd_grad_fused_kernel<FDR_WEIGHT_CENTERED_RANK>, grid, dim3(256), 0, stream, a);
      break;
    case FDR_WEIGHT_MOMENTS:
      if (theta) return set_error(FDR_ERR_INVALID, "the moments form is reduced across ranks before DSGD");
      hipLaunchKernelGGL(fd_grad_fused_kernel<FDR_WEIGHT_MOMENTS>, grid, dim3(256), 0, stream, a);
      break;
    default:
      return set_error(FDR_ERR_INVALID, "unknown weighting mode");
  }
  int rc = check_launch("fd_grad_fused_kernel");
  if (rc || !theta) return rc;
  hipLaunchKernelGGL(dsgd_apply_cb_kernel, dim3(f.col_blocks), dim3(256), 0, stream, theta, out, P, gsq, f.col_blocks,
                     lr, lr_scale, hist, upart, a.cnt + f.col_blocks, dsgd_out);
  return check_launch("dsgd_apply_cb_kernel");
}

int launch_rank_weights(const double* r_all, int n_all, int lo, int n_local, double* w, hipStream_t stream) {
  if (n_local == 0) return FDR_OK;
  hipLaunchKernelGGL(rank_weights_kernel, dim3((n_local + 255) / 256), dim3(256), 0, stream, r_all, n_all, lo, n_local,
                     w);
  return check_launch("rank_weights_kernel");
}

// ------------------------------------------------------------------------------------------
// Fused DSGD (P <= kDsgdFusedMaxP): ONE 1024-thread workgroup does the norm of fl32(-g), the update
// and ||d theta|| (dynamic_sgd.py:19-39) with barriers only.  src = g, or (moments form) the summed
// [A | B | sum r' | sum r'^2 | n] from which g = (A - m B) / sd (z-score identity), also
// written to g_out.  Same per-element arithmetic and the same f32 norm as the 3-kernel path.
// ------------------------------------------------------------------------------------------
constexpr int64_t kDsgdFusedMaxP = 1 << 16;

__device__ __forceinline__ double grad_elem(const double* src, int64_t P, int64_t p, bool mom, double m, double sd) {
  if (!mom) return src[p];
  const double A = src[p], B = src[P + p];
  return sd == 0.0 ? A : (A - m * B) / sd;  // standardize_arr returns its input unchanged when std == 0
}

__device__ double block_sum_1024x(double v, double* red);

// z-score statistics of the summed moments [A | B | n | r'_0 .. r'_{n-1}]: mean and population std of all
// ranks' r' in two f64 passes (utils/math_helpers.py:127-134), by a 1024-thread workgroup in a fixed order
__device__ void moment_stats_1024(const double* src, int64_t P, double* red, double& m, double& sd) {
  const int n = (int)src[2 * P];
  const double* r = src + 2 * P + 1;
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) s += r[i];
  m = block_sum_1024x(s, red) / (double)n;
  double q = 0.0;
  for (int i = threadIdx.x; i < n; i += 1024) {
    const double d = r[i] - m;
    q += d * d;
  }
  sd = sqrt(block_sum_1024x(q, red) / (double)n);
}

__device__ double block_sum_1024x(double v, double* red) {
  v = wave_sum(v);
  const int w = threadIdx.x >> 6, j = threadIdx.x & 63;
  __syncthreads();
  if (j == 0) red[w] = v;
  __syncthreads();
  double s = 0.0;
  for (int i = 0; i < 16; ++i) s += red[i];
  return s;
}

__global__ __launch_bounds__(1024) void dsgd_fused_kernel(float* __restrict__ theta, const double* __restrict__ src,
                                                          int64_t P, int mom, double lr, double lr_scale,
                                                          double* __restrict__ g_out, double* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ double red[16];
  double m = 0.0, sd = 0.0;
  if (mom) moment_stats_1024(src, P, red, m, sd);
  double s = 0.0;
  for (int64_t p = threadIdx.x; p < P; p += 1024) {
    const double g = grad_elem(src, P, p, mom, m, sd);
    if (mom && g_out) g_out[p] = g;
    const float gr = (float)(-g);
    s += (double)gr * (double)gr;
  }
  const float norm = (float)sqrt(block_sum_1024x(s, red));
  double u = 0.0;
  if (norm > 0.f) {
    const double coef = lr * sqrt((double)P) * lr_scale / (double)norm;
    const float c32 = (float)coef;
    for (int64_t p = threadIdx.x; p < P; p += 1024) {
      const float gr = (float)(-grad_elem(src, P, p, mom, m, sd));
      const float old = theta[p];
      const float nw = old - c32 * gr;
      theta[p] = nw;
      const float dd = old - nw;
      u += (double)dd * (double)dd;
    }
  }
  u = block_sum_1024x(u, red);
  if (threadIdx.x == 0) {
    out[0] = sqrt(u);
    out[1] = (double)norm;
  }
}

// multi-block path for large P (ImpalaPolicy): the statistics once, then g = (A - m B) / sd
__global__ __launch_bounds__(1024) void moment_stats_kernel(const double* __restrict__ src, int64_t P,
                                                            double* __restrict__ stats) {
  __shared__ double red[16];
  double m, sd;
  moment_stats_1024(src, P, red, m, sd);
  if (threadIdx.x == 0) {
    stats[0] = m;
    stats[1] = sd;
  }
}

__global__ __launch_bounds__(256) void moments_to_grad_kernel(const double* __restrict__ src, int64_t P,
                                                              const double* __restrict__ stats,
                                                              double* __restrict__ g) {
  const double m = stats[0], sd = stats[1];
  for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < P; p += (int64_t)gridDim.x * blockDim.x)
    g[p] = grad_elem(src, P, p, true, m, sd);
}

int launch_dsgd_ex(float* theta, const double* src, int mom, int64_t P, double lr, double lr_scale, double* g_out,
                   double* out, void* ws, int64_t ws_bytes, hipStream_t stream) {
  if (P <= kDsgdFusedMaxP) {
    hipLaunchKernelGGL(dsgd_fused_kernel, dim3(1), dim3(1024), 0, stream, theta, src, P, mom, lr, lr_scale, g_out, out);
    return check_launch("dsgd_fused_kernel");
  }
  const double* g = src;
  if (mom) {
    if (!g_out) return set_error(FDR_ERR_INVALID, "moments form needs g_out for large P");
    if (ws == nullptr || ws_bytes < dsgd_workspace_bytes(P))
      return set_error(FDR_ERR_WORKSPACE, "dsgd workspace too small");
    double* stats = static_cast<double*>(ws) + 2 * kDsgdBlocks + 2;  // past launch_dsgd's partials
    hipLaunchKernelGGL(moment_stats_kernel, dim3(1), dim3(1024), 0, stream, src, P, stats);
    int rc = check_launch("moment_stats_kernel");
    if (rc) return rc;
    const int rb = (int)std::min<int64_t>((P + 255) / 256, 2048);
    hipLaunchKernelGGL(moments_to_grad_kernel, dim3(rb), dim3(256), 0, stream, src, P, stats, g_out);
    rc = check_launch("moments_to_grad_kernel");
    if (rc) return rc;
    g = g_out;
  }
  return launch_dsgd(theta, g, P, lr, lr_scale, out, ws, ws_bytes, stream);
}

}  // namespace fdr
