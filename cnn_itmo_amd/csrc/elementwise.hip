#include <cstdlib>
// HBM-bound kernels of the U-Net step: BatchNormalization (train/infer, fwd/bwd),
// ReLU gradient, Dropout, MaxPooling2D fwd/bwd, the sigmoid head with MSE loss
// and 'accuracy', RMSprop, weight preparation, first-layer packing and the
// deterministic column reductions.  All accesses are 16-byte NHWC vectors;
// every reduction writes per-block partial rows that a fixed-order fp64 pass
// folds, so results are bitwise reproducible run to run.
#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>

#include "common.h"

// ----------------------------------------------------------------------------
// Error plumbing (thread-local message for cnnitmo_last_error).
// ----------------------------------------------------------------------------
static thread_local char g_err[512];
void cnnitmo_set_error(const char* fmt, ...) {
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(g_err, sizeof(g_err), fmt, ap);
  va_end(ap);
}
int cnnitmo_check_launch(const char* what) {
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    cnnitmo_set_error("%s: launch failed: %s", what, hipGetErrorString(e));
    return CNNITMO_ELAUNCH;
  }
  return CNNITMO_OK;
}
extern "C" const char* cnnitmo_last_error(void) { return g_err; }
// 2: CNNITMO_CONSUMER_ROWS 16 -> 64 (query it with cnnitmo_consumer_rows) and cnnitmo_bn_apply's
//    scale / shift must be 16-byte aligned
extern "C" int cnnitmo_version(void) { return 2; }
extern "C" int cnnitmo_consumer_rows(void) { return CNNITMO_CONSUMER_ROWS; }

static inline int grid_for(long work, int per_block = 256, int cap = 8192) {
  long b = (work + per_block - 1) / per_block;
  return (int)std::max(1L, std::min<long>(b, cap));
}

// ----------------------------------------------------------------------------
// Column reduction: part [rows][cols] fp32 -> ws [G][cols] fp64 (stage 1).
// ----------------------------------------------------------------------------
static constexpr int RED_GMAX = 1024;  // stage-1 row groups (max)
static inline int red_groups(long rows) { return (int)std::max(1L, std::min<long>(RED_GMAX, rows / 16)); }

// grid (ceil(cols/64), G); block = 64 columns x 4 row lanes; fixed-order fp64 sums.
__global__ void colsum_stage1(const float* __restrict__ part, long rows, int cols,
                              double* __restrict__ ws) {
  const int G = gridDim.y, g = blockIdx.y;
  const long per = (rows + G - 1) / G;
  const long r0 = (long)g * per, r1 = std::min(rows, r0 + per);
  const int cl = threadIdx.x & 63, rl = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + cl;
  double s = 0.0;
  if (c < cols)
    for (long r = r0 + rl; r < r1; r += 4) s += part[(size_t)r * cols + c];
  __shared__ double red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  if (rl == 0 && c < cols)
    ws[(size_t)g * cols + c] = ((red[cl] + red[cl + 64]) + red[cl + 128]) + red[cl + 192];
}

static int colsum_stage1_launch(const float* part, long rows, int cols, void* ws, hipStream_t s) {
  const int G = red_groups(rows);
  hipLaunchKernelGGL(colsum_stage1, dim3((cols + 63) / 64, G), dim3(256), 0, s, part, rows, cols,
                     (double*)ws);
  return G;
}

// Fold the G stage-1 rows of one column with a whole wave (fixed-order tree:
// deterministic).  Every lane returns the total.  Finalize kernels run one
// 64-lane wave per output column (256-thread blocks = 4 columns).
__device__ __forceinline__ double fold(const double* ws, int G, int cols, int col) {
  const int lane = threadIdx.x & 63;
  double s = 0.0;
  for (int g = lane; g < G; g += 64) s += ws[(size_t)g * cols + col];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  return s;
}
__device__ __forceinline__ int wave_col() { return blockIdx.x * 4 + (threadIdx.x >> 6); }
static inline int wave_grid(int ncols) { return (ncols + 3) / 4; }

extern "C" size_t cnnitmo_reduce_workspace_bytes(long rows, int cols) {
  return (size_t)red_groups(rows) * cols * sizeof(double);
}

__global__ void colsum_final(const double* __restrict__ ws, int G, int cols, int groups,
                             float* __restrict__ out) {
  const int c = wave_col();
  const int C = cols / groups;
  if (c >= C) return;
  double s = 0.0;
  for (int gr = 0; gr < groups; ++gr) s += fold(ws, G, cols, gr * C + c);
  if ((threadIdx.x & 63) == 0) out[c] = (float)s;
}

extern "C" int cnnitmo_colsum(const float* part, long rows, int cols, int groups, float* out,
                              void* workspace, void* stream) {
  CNN_REQUIRE(rows > 0 && cols > 0 && groups > 0 && cols % groups == 0, "colsum: bad sizes");
  hipStream_t s = (hipStream_t)stream;
  const int G = colsum_stage1_launch(part, rows, cols, workspace, s);
  const int C = cols / groups;
  hipLaunchKernelGGL(colsum_final, dim3(wave_grid(C)), dim3(256), 0, s,
                     (const double*)workspace, G, cols, groups, out);
  return cnnitmo_check_launch("colsum");
}

// ----------------------------------------------------------------------------
// BatchNormalization forward (training) finalize -- model.py:196,200.
// stat_part [rows][2][groups*C]: (sum r, sum r^2) per GEMM column.
// ----------------------------------------------------------------------------
__global__ void bn_fwd_final_kernel(const double* __restrict__ ws, int G, int C, int groups,
                                    double count, const float* __restrict__ gamma,
                                    const float* __restrict__ beta, float* mm, float* mv,
                                    float momentum, float eps, float* scale, float* shift,
                                    float* smean, float* sinv) {
  const int c = wave_col();
  if (c >= C) return;
  const int cols = 2 * groups * C;
  double s1 = 0.0, s2 = 0.0;
  for (int gr = 0; gr < groups; ++gr) {
    s1 += fold(ws, G, cols, gr * C + c);
    s2 += fold(ws, G, cols, groups * C + gr * C + c);
  }
  const double mean = s1 / count;
  const double var = fmax(s2 / count - mean * mean, 0.0);  // biased (tf.nn.moments)
  const double inv = 1.0 / sqrt(var + (double)eps);
  const double sc = (double)gamma[c] * inv;
  if ((threadIdx.x & 63) != 0) return;
  scale[c] = (float)sc;
  shift[c] = (float)((double)beta[c] - mean * sc);
  smean[c] = (float)mean;
  sinv[c] = (float)inv;
  if (mm && mv) {
    // Keras 2.2.x on TF 1.x takes tf.nn.fused_batch_norm for 4-D NHWC input, whose
    // batch variance output is already Bessel-corrected (n/(n-1)); Keras then
    // multiplies by n/(n-(1+eps)) again before K.moving_average_update:
    // moving = moving*m + v*(1-m) with v = var_biased * n/(n-1) * n/(n-1-eps).
    const double var_u = var * (count / (count - 1.0)) * (count / (count - (1.0 + (double)eps)));
    mm[c] = (float)((double)mm[c] * momentum + mean * (1.0 - momentum));
    mv[c] = (float)((double)mv[c] * momentum + var_u * (1.0 - momentum));
  }
}

extern "C" int cnnitmo_bn_fwd_finalize(const float* stat_part, long rows, int c, int groups,
                                       double count, const float* gamma, const float* beta,
                                       float* moving_mean, float* moving_var, float momentum,
                                       float eps, float* scale, float* shift, float* save_mean,
                                       float* save_invstd, void* workspace, void* stream) {
  CNN_REQUIRE(rows > 0 && c > 0 && groups >= 1 && count > 1.0, "bn_fwd_finalize: bad sizes");
  hipStream_t s = (hipStream_t)stream;
  const int G = colsum_stage1_launch(stat_part, rows, 2 * groups * c, workspace, s);
  hipLaunchKernelGGL(bn_fwd_final_kernel, dim3(wave_grid(c)), dim3(256), 0, s,
                     (const double*)workspace, G, c, groups, count, gamma, beta, moving_mean,
                     moving_var, momentum, eps, scale, shift, save_mean, save_invstd);
  return cnnitmo_check_launch("bn_fwd_finalize");
}

__global__ void bn_infer_kernel(int C, const float* g, const float* b, const float* mm,
                                const float* mv, float eps, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const float sc = g[c] / sqrtf(mv[c] + eps);
  scale[c] = sc;
  shift[c] = b[c] - mm[c] * sc;
}

extern "C" int cnnitmo_bn_infer_coeffs(int c, const float* gamma, const float* beta,
                                       const float* mmean, const float* mvar, float eps,
                                       float* scale, float* shift, void* stream) {
  hipLaunchKernelGGL(bn_infer_kernel, dim3((c + 255) / 256), dim3(256), 0, (hipStream_t)stream, c,
                     gamma, beta, mmean, mvar, eps, scale, shift);
  return cnnitmo_check_launch("bn_infer_coeffs");
}

// y view = r*scale + shift [+ Dropout(0.5)].  One thread = one 16-byte vector.  lg >= 0:
// C / VE = 2^lg and fewer than 2^31 vectors, so the (pixel, channel) split of a vector index
// is a shift and a mask in 32 bits (the 64-bit division cost as much as the hash).
template <typename T>
__global__ void bn_apply_kernel(const T* __restrict__ r, long P, int C, const float* __restrict__ sc,
                                const float* __restrict__ sh, T* __restrict__ y, long y_ld, int y_off,
                                int drop, uint64_t dbase, int lg) {
  constexpr int VE = Vec16<T>::N;
  const int cv = C / VE;
  const long total = P * cv;
  auto one = [&](long p, int c0) {
    float v[VE], a[VE], b[VE];
    Pack16<T>::load(r + (size_t)p * C + c0, v);
#pragma unroll
    for (int e = 0; e < VE; e += 4) {
      const float4 s4 = *reinterpret_cast<const float4*>(sc + c0 + e), h4 = *reinterpret_cast<const float4*>(sh + c0 + e);
      a[e] = s4.x; a[e + 1] = s4.y; a[e + 2] = s4.z; a[e + 3] = s4.w;
      b[e] = h4.x; b[e + 1] = h4.y; b[e + 2] = h4.z; b[e + 3] = h4.w;
    }
    const uint64_t i0 = (uint64_t)p * C + c0;
#pragma unroll
    for (int e = 0; e < VE; ++e) {
      float o = v[e] * a[e] + b[e];
      if (drop) o = dropout_keep(dbase, i0 + e) ? o * 2.f : 0.f;
      v[e] = o;
    }
    Pack16<T>::store(y + (size_t)p * y_ld + y_off + c0, v);
  };
  if (lg >= 0) {
    const unsigned tot = (unsigned)total, msk = (unsigned)cv - 1u;
    for (unsigned i = blockIdx.x * blockDim.x + threadIdx.x; i < tot; i += gridDim.x * blockDim.x)
      one((long)(i >> lg), (int)(i & msk) * VE);
    return;
  }
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const long p = i / cv;
    one(p, (int)(i - p * cv) * VE);
  }
}

extern "C" int cnnitmo_bn_apply(int dtype, const void* r, long p, int c, const float* scale,
                                const float* shift, void* y, int y_ld, int y_off, int flags,
                                uint64_t drop_seed, int drop_layer, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int drop = (flags & CNNITMO_DROPOUT) ? 1 : 0;
  const uint64_t base = dropout_base(drop_seed, (uint64_t)drop_layer);
  CNN_REQUIRE(c % 8 == 0 && y_ld % 8 == 0 && y_off % 8 == 0, "bn_apply: channels must be multiples of 8");
  CNN_REQUIRE((uintptr_t)scale % 16 == 0 && (uintptr_t)shift % 16 == 0, "bn_apply: scale/shift must be 16-byte aligned");
  const int ve = dtype == CNNITMO_BF16 ? 8 : 4, cv = c / ve;
  const int lg = ((cv & (cv - 1)) == 0 && p * cv < (1L << 31)) ? __builtin_ctz((unsigned)cv) : -1;
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL(bn_apply_kernel<bf16>, dim3(grid_for(p * c / 8)), dim3(256), 0, s,
                       (const bf16*)r, p, c, scale, shift, (bf16*)y, (long)y_ld, y_off, drop, base, lg);
  else
    hipLaunchKernelGGL(bn_apply_kernel<float>, dim3(grid_for(p * c / 4)), dim3(256), 0, s,
                       (const float*)r, p, c, scale, shift, (float*)y, (long)y_ld, y_off, drop, base, lg);
  return cnnitmo_check_launch("bn_apply");
}

// ----------------------------------------------------------------------------
// BN backward.  Thread layout: TPP = C/VE threads per pixel row, ROWS = 256/TPP
// pixel rows per block iteration; each thread keeps VE channels of sums.
// ----------------------------------------------------------------------------
static constexpr int BWD_BLOCKS = 1024;

static int bwd_blocks() { return BWD_BLOCKS; }

extern "C" int cnnitmo_bn_bwd_rows(long p, int c) {
  (void)c;
  return (int)std::max<long>(1, std::min<long>(bwd_blocks(), (p + 7) / 8));
}

// VE argmax bytes of one channel chunk in ONE 8- (bf16) or 4-byte (fp32) load
template <int VE>
__device__ __forceinline__ void load_args(const uint8_t* p, uint8_t* arg) {
  if constexpr (VE == 8) {
    const uint2 a2 = *reinterpret_cast<const uint2*>(p);
    __builtin_memcpy(arg, &a2, 8);
  } else {
    const uint32_t a1 = *reinterpret_cast<const uint32_t*>(p);
    __builtin_memcpy(arg, &a1, 4);
  }
}

template <typename T>
__device__ __forceinline__ void load_dy(const T* dy, long dy_ld, int dy_off, long p, int C, int c0,
                                        int drop, uint64_t dbase, float* v) {
  constexpr int VE = Vec16<T>::N;
  Pack16<T>::load(dy + (size_t)p * dy_ld + dy_off + c0, v);
  if (drop) {
#pragma unroll
    for (int e = 0; e < VE; ++e)
      v[e] = dropout_keep(dbase, (uint64_t)p * C + c0 + e) ? v[e] * 2.f : 0.f;
  }
}

// Block-level reduction of per-thread [VE][NS] sums into part[blockIdx.x][NS][C].
template <int VE, int NS>
__device__ void block_reduce_rows(float (&acc)[NS][VE], int C, float* __restrict__ part) {
  __shared__ float red[256 * VE * NS];
  const int tpp = C / VE;
  const int rows = 256 / tpp;
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < NS; ++k)
#pragma unroll
    for (int e = 0; e < VE; ++e) red[(k * 256 + tid) * VE + e] = acc[k][e];
  __syncthreads();
  for (int idx = tid; idx < NS * C; idx += 256) {
    const int k = idx / C, c = idx - k * C;
    const int cv = c / VE, e = c - cv * VE;
    float s = 0.f;
    for (int r = 0; r < rows; ++r) s += red[(k * 256 + r * tpp + cv) * VE + e];
    part[((size_t)blockIdx.x * NS + k) * C + c] = s;
  }
}

template <typename T>
__global__ void bn_bwd_reduce_kernel(const T* __restrict__ dy, long dy_ld, int dy_off,
                                     const T* __restrict__ r, long r_ld, int r_off, long P, int C,
                                     const float* __restrict__ mean, const float* __restrict__ inv,
                                     int drop, uint64_t dbase, float* __restrict__ part) {
  constexpr int VE = Vec16<T>::N;
  const int tpp = C / VE, rows = 256 / tpp;
  const int tid = threadIdx.x;
  const int row = tid / tpp, cv = tid - row * tpp, c0 = cv * VE;
  float acc[2][VE];
#pragma unroll
  for (int e = 0; e < VE; ++e) acc[0][e] = acc[1][e] = 0.f;
  float mu[VE], is[VE];
#pragma unroll
  for (int e = 0; e < VE; ++e) {
    mu[e] = row < rows ? mean[c0 + e] : 0.f;
    is[e] = row < rows ? inv[c0 + e] : 0.f;
  }
  if (row < rows) {
    for (long p = (long)blockIdx.x * rows + row; p < P; p += (long)gridDim.x * rows) {
      float g[VE], rv[VE];
      load_dy<T>(dy, dy_ld, dy_off, p, C, c0, drop, dbase, g);
      Pack16<T>::load(r + (size_t)p * r_ld + r_off + c0, rv);
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        acc[0][e] += g[e];
        acc[1][e] += g[e] * (rv[e] - mu[e]) * is[e];
      }
    }
  }
  block_reduce_rows<VE, 2>(acc, C, part);
}

extern "C" int cnnitmo_bn_bwd_reduce(int dtype, const void* dy, int dy_ld, int dy_off,
                                     const void* r, int r_ld, int r_off, long p, int c, const float* mean,
                                     const float* invstd, int flags, uint64_t drop_seed,
                                     int drop_layer, float* part, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int G = cnnitmo_bn_bwd_rows(p, c);
  const int drop = (flags & CNNITMO_DROPOUT) ? 1 : 0;
  const uint64_t base = dropout_base(drop_seed, (uint64_t)drop_layer);
  const int VE = dtype == CNNITMO_BF16 ? 8 : 4;
  CNN_REQUIRE(c % VE == 0 && c / VE <= 256 && dy_ld % VE == 0 && dy_off % VE == 0 &&
              r_ld % VE == 0 && r_off % VE == 0, "bn_bwd_reduce: unsupported channel count %d", c);
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<bf16>, dim3(G), dim3(256), 0, s, (const bf16*)dy,
                       (long)dy_ld, dy_off, (const bf16*)r, (long)r_ld, r_off, p, c, mean, invstd, drop, base, part);
  else
    hipLaunchKernelGGL(bn_bwd_reduce_kernel<float>, dim3(G), dim3(256), 0, s, (const float*)dy,
                       (long)dy_ld, dy_off, (const float*)r, (long)r_ld, r_off, p, c, mean, invstd, drop, base, part);
  return cnnitmo_check_launch("bn_bwd_reduce");
}

// coef [3][C]: dz = [r>0] * (a*dy - b*r + e)
__global__ void bn_bwd_final_kernel(const double* __restrict__ ws, int G, int C, double count,
                                    const float* __restrict__ gamma, const float* __restrict__ mean,
                                    const float* __restrict__ inv, float* dgamma, float* dbeta,
                                    float* coef) {
  const int c = wave_col();
  if (c >= C) return;
  const double sdy = fold(ws, G, 2 * C, c), sdyr = fold(ws, G, 2 * C, C + c);
  if ((threadIdx.x & 63) != 0) return;
  if (dgamma) dgamma[c] = (float)sdyr;
  if (dbeta) dbeta[c] = (float)sdy;
  const double a = (double)gamma[c] * inv[c];
  const double b = a * inv[c] * sdyr / count;
  const double e = b * mean[c] - a * sdy / count;
  coef[c] = (float)a;
  coef[C + c] = (float)b;
  coef[2 * C + c] = (float)e;
}

extern "C" int cnnitmo_bn_bwd_finalize(const float* part, long rows, int c, double count,
                                       const float* gamma, const float* mean, const float* invstd,
                                       float* dgamma, float* dbeta, float* coef, void* workspace,
                                       void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int G = colsum_stage1_launch(part, rows, 2 * c, workspace, s);
  hipLaunchKernelGGL(bn_bwd_final_kernel, dim3(wave_grid(c)), dim3(256), 0, s,
                     (const double*)workspace, G, c, count, gamma, mean, invstd, dgamma, dbeta, coef);
  return cnnitmo_check_launch("bn_bwd_finalize");
}

// NP = 1: partial sums of dz per channel (bias gradient); NP = 4: split by the
// pixel's (h&1, w&1) parity, i.e. per Conv2DTranspose tap of the producer
// (needed by the folded-BN wgrad correction of the tconv; db = their sum).
// G3: dy is the rank-3 product dy[p][c] = sum_o g3[p][o] * wh[o][c] of the sigmoid
// head's per-pixel output gradient g3 and its [3][C] weights (cnnitmo_head_fwd_bwd_g3),
// formed in fp32 on the fly instead of being read as a C-channel tensor.
template <typename T, int NP, bool ROUTE, bool G3 = false>
__global__ void bn_bwd_apply_kernel(const T* __restrict__ dy, long dy_ld, int dy_off,
                                    const T* __restrict__ r, long r_ld, int r_off, long P, int C,
                                    const float* __restrict__ coef, int nobn, int drop,
                                    uint64_t dbase, T* __restrict__ dz, float* __restrict__ part,
                                    int H, int W, const T* __restrict__ dyp,
                                    const uint8_t* __restrict__ pidx, const float* __restrict__ g3,
                                    const float* __restrict__ wh) {
  constexpr int VE = Vec16<T>::N;
  const int tpp = C / VE, rows = 256 / tpp;
  const int tid = threadIdx.x;
  const int row = tid / tpp, cv = tid - row * tpp, c0 = cv * VE;
  float acc[NP][VE];
  float ca[VE], cb[VE], ce[VE];
  float w3[G3 ? 3 : 1][VE];
#pragma unroll
  for (int e = 0; e < VE; ++e) {
#pragma unroll
    for (int k = 0; k < NP; ++k) acc[k][e] = 0.f;
    if constexpr (G3) {
#pragma unroll
      for (int o = 0; o < 3; ++o) w3[o][e] = row < rows ? wh[o * C + c0 + e] : 0.f;
    }
    const bool ok = row < rows && !nobn;
    ca[e] = ok ? coef[c0 + e] : 1.f;
    cb[e] = ok ? coef[C + c0 + e] : 0.f;
    ce[e] = ok ? coef[2 * C + c0 + e] : 0.f;
  }
  if (row < rows) {
    const int hw = H * W;  // ROUTE / NP 4 index math in 32 bits (checked by the launchers)
    for (long p = (long)blockIdx.x * rows + row; p < P; p += (long)gridDim.x * rows) {
      float g[VE], rv[VE];
      if constexpr (G3) {
        const float q0 = g3[p * 3], q1 = g3[p * 3 + 1], q2 = g3[p * 3 + 2];
#pragma unroll
        for (int e = 0; e < VE; ++e) g[e] = q0 * w3[0][e] + q1 * w3[1][e] + q2 * w3[2][e];
      } else {
        load_dy<T>(dy, dy_ld, dy_off, p, C, c0, drop, dbase, g);
      }
      Pack16<T>::load(r + (size_t)p * r_ld + r_off + c0, rv);
      if constexpr (ROUTE) {  // + the MaxPooling2D gradient routed to this pixel
        const int pi = (int)p;
        const int n = pi / hw, rem = pi - n * hw;
        const int hh = rem / W, ww = rem - hh * W, Ho = H / 2, Wo = W / 2;
        if ((hh >> 1) < Ho && (ww >> 1) < Wo) {
          const long po = ((long)n * Ho + (hh >> 1)) * Wo + (ww >> 1);
          const int k = ((hh & 1) << 1) | (ww & 1);
          float gp[VE];
          Pack16<T>::load(dyp + (size_t)po * C + c0, gp);
          const uint8_t* ip = pidx + (size_t)po * C + c0;
          uint8_t arg[VE];
          if constexpr (VE == 8) {
            const uint2 a2 = *(const uint2*)ip;
            __builtin_memcpy(arg, &a2, 8);
          } else {
            const uint32_t a1 = *(const uint32_t*)ip;
            __builtin_memcpy(arg, &a1, 4);
          }
#pragma unroll
          for (int e = 0; e < VE; ++e) g[e] += arg[e] == k ? gp[e] : 0.f;
        }
      }
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        const float d = rv[e] > 0.f ? (ca[e] * g[e] - cb[e] * rv[e] + ce[e]) : 0.f;
        g[e] = d;
      }
      Pack16<T>::store(dz + (size_t)p * C + c0, g);
      int k = 0;
      if constexpr (NP == 4) {
        const int rem = (int)p % hw;
        const int hh = rem / W, ww = rem - hh * W;
        k = ((hh & 1) << 1) | (ww & 1);
      }
      // bias gradient from the stored (rounded) dz, as the weight gradient sees it
#pragma unroll
      for (int kk = 0; kk < NP; ++kk)
        if (kk == k) {
#pragma unroll
          for (int e = 0; e < VE; ++e) acc[kk][e] += to_f32(from_f32<T>(g[e]));
        }
    }
  }
  block_reduce_rows<VE, NP>(acc, C, part);
}

// (A four-pixel form of this pass -- 2x2 windows, every load issued first, the
// pooled gradient read once per window -- measured no faster: 6.84 vs 6.82 ms/step
// for the routed applies, 4.6 vs 3.9 for the g3 one; profiles/r02e1_*.)

extern "C" int cnnitmo_bn_bwd_apply(int dtype, const void* dy, int dy_ld, int dy_off,
                                    const void* r, int r_ld, int r_off, long p, int c,
                                    const float* coef, int flags, uint64_t drop_seed, int drop_layer,
                                    int h, int w, void* dz, float* part, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int G = cnnitmo_bn_bwd_rows(p, c);
  const int drop = (flags & CNNITMO_DROPOUT) ? 1 : 0;
  const int nobn = (flags & CNNITMO_NO_BN) ? 1 : 0;
  const uint64_t base = dropout_base(drop_seed, (uint64_t)drop_layer);
  const int VE = dtype == CNNITMO_BF16 ? 8 : 4;
  CNN_REQUIRE(c % VE == 0 && c / VE <= 256 && dy_ld % VE == 0 && dy_off % VE == 0 &&
              r_ld % VE == 0 && r_off % VE == 0, "bn_bwd_apply: unsupported channel count %d", c);
  CNN_REQUIRE(nobn || coef, "bn_bwd_apply: missing coefficients");
  const bool par = flags & CNNITMO_PARITY;
  CNN_REQUIRE(!par || (h > 0 && w > 0), "bn_bwd_apply: PARITY needs h, w");
  CNN_REQUIRE(!par || p < (1L << 31), "bn_bwd_apply: too many pixels");
#define BNA(T, NP)                                                                                \
  hipLaunchKernelGGL((bn_bwd_apply_kernel<T, NP, false>), dim3(G), dim3(256), 0, s, (const T*)dy, \
                     (long)dy_ld, dy_off, (const T*)r, (long)r_ld, r_off, p, c, coef, nobn, drop, \
                     base, (T*)dz, part, h, w, nullptr, nullptr, nullptr, nullptr)
  if (dtype == CNNITMO_BF16) {
    if (par) { BNA(bf16, 4); } else { BNA(bf16, 1); }
  } else {
    if (par) { BNA(float, 4); } else { BNA(float, 1); }
  }
#undef BNA
  return cnnitmo_check_launch("bn_bwd_apply");
}

extern "C" int cnnitmo_bn_bwd_apply_pooled(int dtype, const void* dy, int dy_ld, int dy_off, const void* r,
                                           int r_ld, int r_off, int n, int h, int w, int c,
                                           const float* coef, const void* dy_pool, const uint8_t* idx,
                                           void* dz, float* part, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const long p = (long)n * h * w;
  const int G = cnnitmo_bn_bwd_rows(p, c);
  const int VE = dtype == CNNITMO_BF16 ? 8 : 4;
  CNN_REQUIRE(c % 8 == 0 && c / VE <= 256 && dy_ld % 8 == 0 && dy_off % 8 == 0 && r_ld % 8 == 0 &&
              r_off % 8 == 0 && coef && dy_pool && idx, "bn_bwd_apply_pooled: unsupported arguments (c=%d)", c);
  CNN_REQUIRE(p < (1L << 31), "bn_bwd_apply_pooled: too many pixels");
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<bf16, 1, true>), dim3(G), dim3(256), 0, s, (const bf16*)dy,
                       (long)dy_ld, dy_off, (const bf16*)r, (long)r_ld, r_off, p, c, coef, 0, 0, (uint64_t)0,
                       (bf16*)dz, part, h, w, (const bf16*)dy_pool, idx, nullptr, nullptr);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<float, 1, true>), dim3(G), dim3(256), 0, s, (const float*)dy,
                       (long)dy_ld, dy_off, (const float*)r, (long)r_ld, r_off, p, c, coef, 0, 0, (uint64_t)0,
                       (float*)dz, part, h, w, (const float*)dy_pool, idx, nullptr, nullptr);
  return cnnitmo_check_launch("bn_bwd_apply_pooled");
}

extern "C" int cnnitmo_bn_bwd_apply_g3(int dtype, const float* g3, const float* wh, const void* r, int r_ld,
                                       int r_off, long p, int c, const float* coef, void* dz, float* part,
                                       void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int G = cnnitmo_bn_bwd_rows(p, c);
  const int VE = dtype == CNNITMO_BF16 ? 8 : 4;
  CNN_REQUIRE(c % VE == 0 && c / VE <= 256 && r_ld % VE == 0 && r_off % VE == 0 && coef && g3 && wh,
              "bn_bwd_apply_g3: unsupported arguments (c=%d)", c);
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL((bn_bwd_apply_kernel<bf16, 1, false, true>), dim3(G), dim3(256), 0, s, nullptr, 0L,
                       0, (const bf16*)r, (long)r_ld, r_off, p, c, coef, 0, 0, (uint64_t)0, (bf16*)dz, part, 0, 0,
                       nullptr, nullptr, g3, wh);
  else
    hipLaunchKernelGGL((bn_bwd_apply_kernel<float, 1, false, true>), dim3(G), dim3(256), 0, s, nullptr, 0L, 0,
                       (const float*)r, (long)r_ld, r_off, p, c, coef, 0, 0, (uint64_t)0, (float*)dz, part, 0,
                       0, nullptr, nullptr, g3, wh);
  return cnnitmo_check_launch("bn_bwd_apply_g3");
}

// ----------------------------------------------------------------------------
// MaxPooling2D 2x2 s2 -- model.py:210,215,220,227.  Tie rule: first maximum in
// window order (0,0),(0,1),(1,0),(1,1) (strict '>' scan), shared with the oracle.
// ----------------------------------------------------------------------------
template <typename T>
__global__ void maxpool_fwd_kernel(const T* __restrict__ x, long x_ld, int x_off, int N, int H,
                                   int W, int C, T* __restrict__ y, uint8_t* __restrict__ idx,
                                   const float* __restrict__ sc, const float* __restrict__ sh) {
  constexpr int VE = Vec16<T>::N;
  const int Ho = H / 2, Wo = W / 2, cv = C / VE;
  const long total = (long)N * Ho * Wo * cv;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int pi = (int)(i / cv);  // 32-bit index math from here (launcher: < 2^31 pixels)
    const long po = pi;
    const int c0 = (int)(i - po * cv) * VE;
    const int n = pi / (Ho * Wo);
    const int rem = pi - n * (Ho * Wo);
    const int ho = rem / Wo, wo = rem - ho * Wo;
    float best[VE], win[4][VE];
    uint8_t arg[VE];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // the whole window's loads first
      const long pin = ((long)n * H + 2 * ho + (k >> 1)) * W + 2 * wo + (k & 1);
      Pack16<T>::load(x + (size_t)pin * x_ld + x_off + c0, win[k]);
    }
    if (sc) {  // folded BN: pool y = r*s + h (the max of y, whatever the sign of s); once per chunk
      float s8[VE], h8[VE];
      Pack16<float>::load(sc + c0, s8);
      Pack16<float>::load(sh + c0, h8);
      if constexpr (VE == 8) {
        Pack16<float>::load(sc + c0 + 4, s8 + 4);
        Pack16<float>::load(sh + c0 + 4, h8 + 4);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < VE; ++e) win[k][e] = win[k][e] * s8[e] + h8[e];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        if (k == 0 || win[k][e] > best[e]) {
          best[e] = win[k][e];
          arg[e] = (uint8_t)k;
        }
      }
    }
    Pack16<T>::store(y + (size_t)po * C + c0, best);
    if constexpr (VE == 8) {
      uint2 a;
      a.x = arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((uint32_t)arg[3] << 24);
      a.y = arg[4] | (arg[5] << 8) | (arg[6] << 16) | ((uint32_t)arg[7] << 24);
      *reinterpret_cast<uint2*>(idx + (size_t)po * C + c0) = a;
    } else {
      *reinterpret_cast<uint32_t*>(idx + (size_t)po * C + c0) =
          arg[0] | (arg[1] << 8) | (arg[2] << 16) | ((uint32_t)arg[3] << 24);
    }
  }
}

// Rows of pooled pixels per 256-thread block: tpp = C/VE threads per pixel.
template <typename T>
__global__ void maxpool_bwd_kernel(const T* __restrict__ dy, const uint8_t* __restrict__ idx, int H, int W,
                                   long Pp, int C, T* __restrict__ dx, long dx_ld, int dx_off) {
  constexpr int VE = Vec16<T>::N;
  const int tpp = C / VE, rows = 256 / tpp;
  const int row = threadIdx.x / tpp, cv = threadIdx.x - row * tpp, c0 = cv * VE;
  const int Ho = H / 2, Wo = W / 2;
  if (row >= rows) return;
  for (long po = (long)blockIdx.x * rows + row; po < Pp; po += (long)gridDim.x * rows) {
    const int n = (int)po / (Ho * Wo);  // 32-bit index math (launcher: < 2^31 pixels)
    const int rem = (int)po - n * (Ho * Wo);
    const int ho = rem / Wo, wo = rem - ho * Wo;
    float g[VE];
    Pack16<T>::load(dy + (size_t)po * C + c0, g);
    uint8_t arg[VE];
    load_args<VE>(idx + (size_t)po * C + c0, arg);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      bool any = false;
#pragma unroll
      for (int e = 0; e < VE; ++e) any |= arg[e] == k;
      if (!any) continue;
      const long pin = ((long)n * H + 2 * ho + (k >> 1)) * W + 2 * wo + (k & 1);
      T* q = dx + (size_t)pin * dx_ld + dx_off + c0;
      float v[VE];
      Pack16<T>::load(q, v);
#pragma unroll
      for (int e = 0; e < VE; ++e)
        if (arg[e] == k) v[e] += g[e];
      Pack16<T>::store(q, v);
    }
  }
}

// The MaxPooling2D share of the BN-backward sums of a folded pool input (see
// cnnitmo_bn_consumer_sums): sum_p dyp[p] and sum_p dyp[p] * rhat[argmax(p)].
// The 2x2 window of r is read whole (two coalesced pixel pairs) and the argmax
// element selected per channel.
// PRE: r is the pooled r itself ([Pp][C] dense: the producer's epilogue wrote r at the
// window index, cnnitmo_conv3x3_fwd_pool), so no window is read and idx is not needed.
template <typename T, bool PRE = false>
__global__ void pool_bnsums_kernel(const T* __restrict__ dyp, const uint8_t* __restrict__ idx, int H, int W,
                                   long Pp, int C, const T* __restrict__ r, long r_ld, int r_off,
                                   const float* __restrict__ mean, const float* __restrict__ inv,
                                   float* __restrict__ part) {
  constexpr int VE = Vec16<T>::N;
  const int tpp = C / VE, rows = 256 / tpp;
  const int row = threadIdx.x / tpp, cv = threadIdx.x - row * tpp, c0 = cv * VE;
  const int Ho = H / 2, Wo = W / 2;
  float acc[2][VE], mu[VE], is[VE];
#pragma unroll
  for (int e = 0; e < VE; ++e) {
    acc[0][e] = acc[1][e] = 0.f;
    mu[e] = row < rows ? mean[c0 + e] : 0.f;
    is[e] = row < rows ? inv[c0 + e] : 0.f;
  }
  if (row < rows) {
    for (long po = (long)blockIdx.x * rows + row; po < Pp; po += (long)gridDim.x * rows) {
      const int n = (int)po / (Ho * Wo);  // 32-bit index math (launcher: < 2^31 pixels)
      const int rem = (int)po - n * (Ho * Wo);
      const int ho = rem / Wo, wo = rem - ho * Wo;
      float g[VE], rw[4][VE];
      Pack16<T>::load(dyp + (size_t)po * C + c0, g);
      if constexpr (PRE) {
        Pack16<T>::load(r + (size_t)po * C + c0, rw[0]);
#pragma unroll
        for (int e = 0; e < VE; ++e) {
          acc[0][e] += g[e];
          acc[1][e] += g[e] * (rw[0][e] - mu[e]) * is[e];
        }
        continue;
      }
      uint8_t arg[VE];
      load_args<VE>(idx + (size_t)po * C + c0, arg);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const long pin = ((long)n * H + 2 * ho + (k >> 1)) * W + 2 * wo + (k & 1);
        Pack16<T>::load(r + (size_t)pin * r_ld + r_off + c0, rw[k]);
      }
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        const int k = arg[e];
        const float rv = k == 0 ? rw[0][e] : (k == 1 ? rw[1][e] : (k == 2 ? rw[2][e] : rw[3][e]));
        acc[0][e] += g[e];
        acc[1][e] += g[e] * (rv - mu[e]) * is[e];
      }
    }
  }
  block_reduce_rows<VE, 2>(acc, C, part);
}

extern "C" int cnnitmo_pool_bnsums_pooled(int dtype, const void* dyp, const void* pr, int n, int h, int w, int c,
                                          const float* mean, const float* invstd, float* part, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int VE = dtype == CNNITMO_BF16 ? 8 : 4;
  CNN_REQUIRE(c % 8 == 0 && c / VE <= 256 && dyp && pr, "pool_bnsums_pooled: unsupported channel count %d", c);
  const long Pp = (long)n * (h / 2) * (w / 2);
  CNN_REQUIRE(Pp < (1L << 31), "pool_bnsums_pooled: too many pixels");
  const int G = cnnitmo_bn_bwd_rows(Pp, c);
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL((pool_bnsums_kernel<bf16, true>), dim3(G), dim3(256), 0, s, (const bf16*)dyp, nullptr, h, w,
                       Pp, c, (const bf16*)pr, (long)c, 0, mean, invstd, part);
  else
    hipLaunchKernelGGL((pool_bnsums_kernel<float, true>), dim3(G), dim3(256), 0, s, (const float*)dyp, nullptr, h,
                       w, Pp, c, (const float*)pr, (long)c, 0, mean, invstd, part);
  return cnnitmo_check_launch("pool_bnsums_pooled");
}

extern "C" int cnnitmo_maxpool2x2_fwd(int dtype, const void* x, int x_ld, int x_off, int n, int h,
                                      int w, int c, void* y, uint8_t* idx, const float* scale,
                                      const float* shift, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  CNN_REQUIRE(c % 8 == 0 && x_ld % 8 == 0 && x_off % 8 == 0, "maxpool_fwd: channels must be multiples of 8");
  const long work = (long)n * (h / 2) * (w / 2) * c;
  CNN_REQUIRE((long)n * (h / 2) * (w / 2) < (1L << 31), "maxpool_fwd: too many pixels");
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL(maxpool_fwd_kernel<bf16>, dim3(grid_for(work / 8)), dim3(256), 0, s,
                       (const bf16*)x, (long)x_ld, x_off, n, h, w, c, (bf16*)y, idx, scale, shift);
  else
    hipLaunchKernelGGL(maxpool_fwd_kernel<float>, dim3(grid_for(work / 4)), dim3(256), 0, s,
                       (const float*)x, (long)x_ld, x_off, n, h, w, c, (float*)y, idx, scale, shift);
  return cnnitmo_check_launch("maxpool_fwd");
}

extern "C" int cnnitmo_maxpool2x2_bwd(int dtype, const void* dy, const uint8_t* idx, int n, int h, int w,
                                      int c, void* dx, int dx_ld, int dx_off, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int VE = dtype == CNNITMO_BF16 ? 8 : 4;
  CNN_REQUIRE(c % 8 == 0 && dx_ld % 8 == 0 && dx_off % 8 == 0 && c / VE <= 256,
              "maxpool_bwd: channels must be multiples of 8 (at most 1024/2048)");
  const long Pp = (long)n * (h / 2) * (w / 2);
  const int rows = 256 / (c / VE);
  const int G = (int)std::max<long>(1, std::min<long>((Pp + rows - 1) / rows, 8192));
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL(maxpool_bwd_kernel<bf16>, dim3(G), dim3(256), 0, s, (const bf16*)dy, idx, h, w, Pp, c,
                       (bf16*)dx, (long)dx_ld, dx_off);
  else
    hipLaunchKernelGGL(maxpool_bwd_kernel<float>, dim3(G), dim3(256), 0, s, (const float*)dy, idx, h, w, Pp,
                       c, (float*)dx, (long)dx_ld, dx_off);
  return cnnitmo_check_launch("maxpool_bwd");
}

extern "C" int cnnitmo_pool_bnsums(int dtype, const void* dyp, const uint8_t* idx, int n, int h, int w,
                                   int c, const void* r, int r_ld, int r_off, const float* mean,
                                   const float* invstd, float* part, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int VE = dtype == CNNITMO_BF16 ? 8 : 4;
  CNN_REQUIRE(c % 8 == 0 && r_ld % 8 == 0 && r_off % 8 == 0 && c / VE <= 256,
              "pool_bnsums: unsupported channel count %d", c);
  const long Pp = (long)n * (h / 2) * (w / 2);
  CNN_REQUIRE(Pp < (1L << 31), "pool_bnsums: too many pixels");
  const int G = cnnitmo_bn_bwd_rows(Pp, c);
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL(pool_bnsums_kernel<bf16>, dim3(G), dim3(256), 0, s, (const bf16*)dyp, idx, h, w, Pp, c,
                       (const bf16*)r, (long)r_ld, r_off, mean, invstd, part);
  else
    hipLaunchKernelGGL(pool_bnsums_kernel<float>, dim3(G), dim3(256), 0, s, (const float*)dyp, idx, h, w, Pp,
                       c, (const float*)r, (long)r_ld, r_off, mean, invstd, part);
  return cnnitmo_check_launch("pool_bnsums");
}

// ----------------------------------------------------------------------------
// Head: Conv2D(3, 1, activation='sigmoid') + MSE + categorical accuracy
// (model.py:276,281).  LPP = cin/VE lanes share one pixel.
// part row layout: [loss, correct, db0..2, dW[3][cin]]
// ----------------------------------------------------------------------------
static constexpr int HEAD_BLOCKS = 1024;
#ifndef HEAD_U
#define HEAD_U 4
#endif
extern "C" int cnnitmo_head_rows(long p) {
  return (int)std::max<long>(1, std::min<long>(HEAD_BLOCKS, (p + 31) / 32));
}

template <typename T, bool BWD>
__global__ void head_kernel(const T* __restrict__ x, int N, int H, int Hv, int W, int cin,
                            const float* __restrict__ wt, const float* __restrict__ bias,
                            const float* __restrict__ target, float* __restrict__ yhat,
                            T* __restrict__ dx, float inv_numel, float* __restrict__ part,
                            const float* __restrict__ fs, const float* __restrict__ fh,
                            float* __restrict__ g3) {
  constexpr int VE = Vec16<T>::N;
  const int lpp = cin / VE;             // lanes per pixel (power of two <= 64)
  const int ppb = 256 / lpp;            // pixels per block iteration
  const int tid = threadIdx.x, sub = tid % lpp, slot = tid / lpp;
  const int c0 = sub * VE;
  float w[3][VE], wf[3][VE];  // raw (for dx) and BN-folded (for z) weights
  float bfold[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int o = 0; o < 3; ++o)
#pragma unroll
    for (int e = 0; e < VE; ++e) {
      w[o][e] = wt[o * cin + c0 + e];
      wf[o][e] = fs ? w[o][e] * fs[c0 + e] : w[o][e];
      if (fh) bfold[o] += w[o][e] * fh[c0 + e];
    }
#pragma unroll
  for (int o = 0; o < 3; ++o)
    for (int off = lpp >> 1; off > 0; off >>= 1) bfold[o] += __shfl_xor(bfold[o], off, 64);
  const float b0 = bias[0] + bfold[0], b1 = bias[1] + bfold[1], b2 = bias[2] + bfold[2];
  float dwacc[3][VE];
#pragma unroll
  for (int o = 0; o < 3; ++o)
#pragma unroll
    for (int e = 0; e < VE; ++e) dwacc[o][e] = 0.f;
  float lsum = 0.f, corr = 0.f, db[3] = {0.f, 0.f, 0.f};
  const long P = (long)N * H * W;
  const int hw = H * W;
  const bool rowal = W % ppb == 0;
  // HEAD_U pixel slots per lane group per iteration, all their loads issued first:
  // one 16-byte load in flight per lane left this HBM pass at ~2 TB/s
  for (long base0 = (long)blockIdx.x * ppb * HEAD_U; base0 < P; base0 += (long)gridDim.x * ppb * HEAD_U) {
    float v[HEAD_U][VE], tg[HEAD_U][3];
    bool inb[HEAD_U], valid[HEAD_U];
    size_t tix[HEAD_U];
#pragma unroll
    for (int u = 0; u < HEAD_U; ++u) {
      const long base = base0 + (long)u * ppb, p = base + slot;
      inb[u] = p < P;
      if (inb[u]) Pack16<T>::load(x + (size_t)p * cin + c0, v[u]);
      else
#pragma unroll
        for (int e = 0; e < VE; ++e) v[u][e] = 0.f;
      // 32-bit index math (P < 2^31, checked by the launchers); when a block's ppb pixels
      // never straddle a row (W % ppb == 0) it is wave-uniform: one scalar division
      int n, h, wc;
      if (rowal) {
        const int b = (int)base, nb = b / hw, rb = b - nb * hw, hb = rb / W;
        n = nb;
        h = hb;
        wc = rb - hb * W + slot;
      } else {
        n = inb[u] ? (int)p / hw : 0;
        const int rem = inb[u] ? (int)p - n * hw : 0;
        h = rem / W;
        wc = rem - h * W;
      }
      valid[u] = inb[u] && h < Hv;
      tix[u] = (((size_t)n * Hv + h) * W + wc) * 3;
      if (BWD) {
#pragma unroll
        for (int o = 0; o < 3; ++o) tg[u][o] = valid[u] ? target[tix[u] + o] : 0.f;
      }
    }
#pragma unroll
    for (int u = 0; u < HEAD_U; ++u) {
      const long p = base0 + (long)u * ppb + slot;
      float z[3];
#pragma unroll
      for (int o = 0; o < 3; ++o) {
        float s = 0.f;
#pragma unroll
        for (int e = 0; e < VE; ++e) s += v[u][e] * wf[o][e];
        for (int off = lpp >> 1; off > 0; off >>= 1) s += __shfl_xor(s, off, 64);
        z[o] = s;
      }
      z[0] += b0; z[1] += b1; z[2] += b2;
      float yh[3];
#pragma unroll
      for (int o = 0; o < 3; ++o) yh[o] = 1.f / (1.f + expf(-z[o]));
      if (!BWD) {
        if (valid[u] && sub == 0) {
          yhat[tix[u] + 0] = yh[0];
          yhat[tix[u] + 1] = yh[1];
          yhat[tix[u] + 2] = yh[2];
        }
        continue;
      }
      float dz[3] = {0.f, 0.f, 0.f};
      if (valid[u]) {
        const float t0 = tg[u][0], t1 = tg[u][1], t2 = tg[u][2];
        const float e0 = yh[0] - t0, e1 = yh[1] - t1, e2 = yh[2] - t2;
        if (sub == 0) {
          lsum += e0 * e0 + e1 * e1 + e2 * e2;
          const int at = (t1 > t0) ? ((t2 > t1) ? 2 : 1) : ((t2 > t0) ? 2 : 0);
          const int ap = (yh[1] > yh[0]) ? ((yh[2] > yh[1]) ? 2 : 1) : ((yh[2] > yh[0]) ? 2 : 0);
          corr += (at == ap) ? 1.f : 0.f;
        }
        dz[0] = 2.f * e0 * yh[0] * (1.f - yh[0]) * inv_numel;
        dz[1] = 2.f * e1 * yh[1] * (1.f - yh[1]) * inv_numel;
        dz[2] = 2.f * e2 * yh[2] * (1.f - yh[2]) * inv_numel;
      }
      if (sub == 0) {
        db[0] += dz[0]; db[1] += dz[1]; db[2] += dz[2];
      }
#pragma unroll
      for (int e = 0; e < VE; ++e)
#pragma unroll
        for (int o = 0; o < 3; ++o) dwacc[o][e] += dz[o] * v[u][e];
      if (g3) {  // rank-3 input gradient: the consumer forms dz . w itself
        if (inb[u] && sub == 0) {
          g3[p * 3] = dz[0];
          g3[p * 3 + 1] = dz[1];
          g3[p * 3 + 2] = dz[2];
        }
      } else {
        float g[VE];
#pragma unroll
        for (int e = 0; e < VE; ++e) g[e] = dz[0] * w[0][e] + dz[1] * w[1][e] + dz[2] * w[2][e];
        if (inb[u]) Pack16<T>::store(dx + (size_t)p * cin + c0, g);
      }
    }
  }
  if (!BWD) return;
  // reduce: lanes with equal `sub` hold the same channel slice
  __shared__ float red[256][3 * 8 + 5];
#pragma unroll
  for (int o = 0; o < 3; ++o)
#pragma unroll
    for (int e = 0; e < VE; ++e) red[tid][o * VE + e] = dwacc[o][e];
  red[tid][3 * VE + 0] = lsum;
  red[tid][3 * VE + 1] = corr;
  red[tid][3 * VE + 2] = db[0];
  red[tid][3 * VE + 3] = db[1];
  red[tid][3 * VE + 4] = db[2];
  __syncthreads();
  const int ncol = 5 + 3 * cin;
  float* out = part + (size_t)blockIdx.x * ncol;
  for (int k = tid; k < ncol; k += 256) {
    float s = 0.f;
    if (k < 5) {
      for (int t = 0; t < 256; t += lpp) s += red[t][3 * VE + k];
    } else {
      const int q = k - 5, o = q / cin, c = q - o * cin;
      const int sb = c / VE, e = c - sb * VE;
      for (int t = sb; t < 256; t += lpp) s += red[t][o * VE + e];
    }
    out[k] = s;
  }
}

// The same head, one wave per 64 consecutive pixels per iteration, in two layouts:
//   * channel layout (loads, dot products, dW, dx): LPP = cin/VE lanes per pixel, each
//     lane issuing LPP 16-byte loads up front (pixel u*64/LPP + lane/LPP): 1 KB per
//     instruction, LPP KB in flight per wave; the dot products reduced over the LPP
//     lanes with DPP (quad_perm xor 1/2, half-row and row mirrors: VALU, no LDS);
//   * pixel layout (sigmoid, loss, accuracy, dz, target and g3/yhat): lane = pixel,
//     the per-pixel math done once (head_kernel did it on all LPP lanes of a pixel),
//     target / g3 / yhat as 12-byte runs of consecutive lanes.
// z and dz cross between the two through a 1 KB LDS slice per wave (no barrier: one
// wave owns the slice, LDS executes a wave's instructions in order).  Bench shape
// (32 x 1088 x 1920 x 64 bf16, g3 out; tools/probe_elem.py): head_kernel 4.85 ms
// (2.1 TB/s), head2_kernel 2.35 ms (4.3 TB/s; a torch copy of x runs at 4.9 TB/s).
template <int LPP>
__device__ __forceinline__ float lane_group_sum(float v) {
  if constexpr (LPP >= 2) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  if constexpr (LPP >= 4) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  if constexpr (LPP >= 8) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  if constexpr (LPP >= 16) v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}

template <typename T>
__device__ __forceinline__ void unpack16(const uint4& q, float* v) {
  if constexpr (Vec16<T>::N == 8) {
    const bf16x8 b = __builtin_bit_cast(bf16x8, q);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)b[i];
  } else {
    v[0] = __uint_as_float(q.x); v[1] = __uint_as_float(q.y); v[2] = __uint_as_float(q.z); v[3] = __uint_as_float(q.w);
  }
}

// BWD: loss + gradients; G3: the gradient leaves as g3 [P][3] (else dx = dz . W)
template <typename T, int LPP, bool BWD, bool G3>
__global__ __launch_bounds__(256) void head2_kernel(const T* __restrict__ x, int H, int Hv, int W, long P,
                                                    const float* __restrict__ wt, const float* __restrict__ bias,
                                                    const float* __restrict__ target, float* __restrict__ yhat,
                                                    T* __restrict__ dx, float inv_numel, float* __restrict__ part,
                                                    const float* __restrict__ fs, const float* __restrict__ fh,
                                                    float* __restrict__ g3) {
  constexpr int VE = Vec16<T>::N, CIN = LPP * VE, PPI = 64 / LPP;  // pixels per load instruction
  __shared__ float4 zs[4][64];
  __shared__ float red[4][3 * CIN + 5];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int sub = lane % LPP, c0 = sub * VE, pq = lane / LPP;
  float w[3][VE], wf[3][VE], bf[3] = {0.f, 0.f, 0.f};
#pragma unroll
  for (int o = 0; o < 3; ++o) {
#pragma unroll
    for (int e = 0; e < VE; ++e) {
      w[o][e] = BWD && !G3 ? wt[o * CIN + c0 + e] : 0.f;  // (dx only)
      const float wo = wt[o * CIN + c0 + e];
      wf[o][e] = fs ? wo * fs[c0 + e] : wo;
      if (fh) bf[o] += wo * fh[c0 + e];
    }
    bf[o] = lane_group_sum<LPP>(bf[o]);
  }
  const float b0 = bias[0] + bf[0], b1 = bias[1] + bf[1], b2 = bias[2] + bf[2];
  float dwacc[3][VE];
#pragma unroll
  for (int o = 0; o < 3; ++o)
#pragma unroll
    for (int e = 0; e < VE; ++e) dwacc[o][e] = 0.f;
  float lsum = 0.f, corr = 0.f, db0 = 0.f, db1 = 0.f, db2 = 0.f;
  const int hw = H * W;
  const long ngroups = (P + 63) / 64, nw = (long)gridDim.x * 4;
  // a group's x (channel layout) and target (pixel layout) loads, all issued first and
  // branch-free (buffer loads, out-of-range ones read 0).  (Issuing the next group's
  // loads before this group's math measured no faster: 2.35 vs 2.35 ms at the bench
  // shape, where a torch copy of the same bytes runs at 4.9 TB/s.)
  const __amdgpu_buffer_rsrc_t tr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(BWD ? target : nullptr), (short)0, BWD ? (int)(P / hw * Hv * W * 12) : 0, 0x00020000);
  auto fetch = [&](long g, uint4 (&xq)[LPP], float (&tq)[3]) {
    const long b = g * 64;
    const long np_ = P - b < 64 ? (P - b > 0 ? P - b : 0) : 64;
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<T*>(x + (b < P ? b : 0) * CIN), (short)0, (int)np_ * CIN * (int)sizeof(T), 0x00020000);
#pragma unroll
    for (int u = 0; u < LPP; ++u)
      xq[u] = __builtin_bit_cast(uint4, __builtin_amdgcn_raw_buffer_load_b128(
                                            xr, (unsigned)(((u * PPI + pq) * CIN + c0) * sizeof(T)), 0, 0));
    if constexpr (BWD) {
      const int pp = (int)b + lane;
      const bool ok = lane < np_;
      const int n = ok ? pp / hw : 0, rem = ok ? pp - n * hw : 0, h = rem / W, wc = rem - h * W;
      const unsigned off = ok && h < Hv ? (((unsigned)n * Hv + h) * W + wc) * 12u : 0x80000000u;
#pragma unroll
      for (int o = 0; o < 3; ++o) tq[o] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(tr, off + 4 * o, 0, 0));
    }
  };
  uint4 xv[LPP];
  float tv[3] = {0.f, 0.f, 0.f};
  for (long grp = (long)blockIdx.x * 4 + wave; grp < ngroups; grp += nw) {
    fetch(grp, xv, tv);
    const long base = grp * 64;
    const int np = (int)(P - base < 64 ? P - base : 64);
    // pixel layout (32-bit index math: P < 2^31, checked by the launchers)
    const int p = (int)base + lane;
    const bool inb = lane < np;
    const int n = inb ? p / hw : 0, rem = inb ? p - n * hw : 0, h = rem / W, wc = rem - h * W;
    const bool valid = inb && h < Hv;
    const size_t tix = (((size_t)n * Hv + h) * W + wc) * 3;
    const float t0 = tv[0], t1 = tv[1], t2 = tv[2];
#pragma unroll
    for (int u = 0; u < LPP; ++u) {
      float v[VE];
      unpack16<T>(xv[u], v);
      float s0 = 0.f, s1 = 0.f, s2 = 0.f;
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        s0 += v[e] * wf[0][e];
        s1 += v[e] * wf[1][e];
        s2 += v[e] * wf[2][e];
      }
      s0 = lane_group_sum<LPP>(s0);
      s1 = lane_group_sum<LPP>(s1);
      s2 = lane_group_sum<LPP>(s2);
      if (sub == 0) zs[wave][u * PPI + pq] = make_float4(s0, s1, s2, 0.f);
    }
    __builtin_amdgcn_wave_barrier();
    const float4 z = zs[wave][lane];
    const float y0 = 1.f / (1.f + expf(-(z.x + b0)));
    const float y1 = 1.f / (1.f + expf(-(z.y + b1)));
    const float y2 = 1.f / (1.f + expf(-(z.z + b2)));
    if (!BWD) {
      if (valid) {
        yhat[tix] = y0;
        yhat[tix + 1] = y1;
        yhat[tix + 2] = y2;
      }
      __builtin_amdgcn_wave_barrier();
      continue;
    }
    float d0 = 0.f, d1 = 0.f, d2 = 0.f;
    if (valid) {
      const float e0 = y0 - t0, e1 = y1 - t1, e2 = y2 - t2;
      lsum += e0 * e0 + e1 * e1 + e2 * e2;
      const int at = (t1 > t0) ? ((t2 > t1) ? 2 : 1) : ((t2 > t0) ? 2 : 0);
      const int ap = (y1 > y0) ? ((y2 > y1) ? 2 : 1) : ((y2 > y0) ? 2 : 0);
      corr += (at == ap) ? 1.f : 0.f;
      d0 = 2.f * e0 * y0 * (1.f - y0) * inv_numel;
      d1 = 2.f * e1 * y1 * (1.f - y1) * inv_numel;
      d2 = 2.f * e2 * y2 * (1.f - y2) * inv_numel;
    }
    db0 += d0;
    db1 += d1;
    db2 += d2;
    if (G3 && inb) {
      g3[(size_t)p * 3] = d0;
      g3[(size_t)p * 3 + 1] = d1;
      g3[(size_t)p * 3 + 2] = d2;
    }
    zs[wave][lane] = make_float4(d0, d1, d2, 0.f);
    __builtin_amdgcn_wave_barrier();
    // back to the channel layout: dW (and dx = dz . W without g3)
#pragma unroll
    for (int u = 0; u < LPP; ++u) {
      const float4 d = zs[wave][u * PPI + pq];
      float v[VE];
      asm volatile("" : "+v"(xv[u].x), "+v"(xv[u].y), "+v"(xv[u].z), "+v"(xv[u].w));  // unpack again: keeping all LPP*VE floats live costs occupancy
      unpack16<T>(xv[u], v);
#pragma unroll
      for (int e = 0; e < VE; ++e) {
        dwacc[0][e] += d.x * v[e];
        dwacc[1][e] += d.y * v[e];
        dwacc[2][e] += d.z * v[e];
      }
      if (!G3 && u * PPI + pq < np) {
        float g[VE];
#pragma unroll
        for (int e = 0; e < VE; ++e) g[e] = d.x * w[0][e] + d.y * w[1][e] + d.z * w[2][e];
        Pack16<T>::store(dx + (size_t)(base + u * PPI + pq) * CIN + c0, g);
      }
    }
    __builtin_amdgcn_wave_barrier();
  }
  if (!BWD) return;
  // reduce: dW over the lanes of equal `sub`, the scalars over the wave, then the 4 waves
#pragma unroll
  for (int o = 0; o < 3; ++o)
#pragma unroll
    for (int e = 0; e < VE; ++e)
#pragma unroll
      for (int m = LPP; m < 64; m <<= 1) dwacc[o][e] += __shfl_xor(dwacc[o][e], m, 64);
  lsum = wave_sum(lsum);
  corr = wave_sum(corr);
  db0 = wave_sum(db0);
  db1 = wave_sum(db1);
  db2 = wave_sum(db2);
  if (lane < LPP) {
#pragma unroll
    for (int o = 0; o < 3; ++o)
#pragma unroll
      for (int e = 0; e < VE; ++e) red[wave][5 + o * CIN + c0 + e] = dwacc[o][e];
  }
  if (lane == 0) {
    red[wave][0] = lsum;
    red[wave][1] = corr;
    red[wave][2] = db0;
    red[wave][3] = db1;
    red[wave][4] = db2;
  }
  __syncthreads();
  float* out = part + (size_t)blockIdx.x * (5 + 3 * CIN);
  for (int k = tid; k < 5 + 3 * CIN; k += 256) out[k] = red[0][k] + red[1][k] + red[2][k] + red[3][k];
}

// head2_kernel for this dtype / width, or false (head_kernel then)
template <bool BWD>
static bool launch_head2(int dtype, const void* x, int n, int h, int h_valid, int w, int cin, const float* wt,
                         const float* b, const float* target, float* yhat, void* dx, float inv_numel,
                         float* part, const float* scale, const float* shift, float* g3, int G_, hipStream_t s) {
  const long P = (long)n * h * w;
  const int lpp = cin / (dtype == CNNITMO_BF16 ? 8 : 4);
  // 32-bit pixel and target-byte offsets inside the kernel
  if (P >= (1L << 30) || (long)n * h_valid * w * 12 >= (1L << 31)) return false;
#define H2K(T, L, G)                                                                                          \
  hipLaunchKernelGGL((head2_kernel<T, L, BWD, G>), dim3(G_), dim3(256), 0, s, (const T*)x, h, h_valid, w, P, wt, \
                     b, target, yhat, (T*)dx, inv_numel, part, scale, shift, g3)
#define H2(T, L)                  \
  do {                            \
    if (BWD && g3) H2K(T, L, BWD); \
    else H2K(T, L, false);        \
  } while (0)
#define H2L(T)                     \
  switch (lpp) {                   \
    case 2: H2(T, 2); return true;   \
    case 4: H2(T, 4); return true;   \
    case 8: H2(T, 8); return true;   \
    case 16: H2(T, 16); return true; \
    default: return false;           \
  }
  if (dtype == CNNITMO_BF16) {
    H2L(bf16)
  } else {
    H2L(float)
  }
#undef H2L
#undef H2
#undef H2K
}

extern "C" int cnnitmo_head_fwd(int dtype, const void* x, int n, int h, int h_valid, int w, int cin,
                                const float* wt, const float* b, const float* scale,
                                const float* shift, float* yhat, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int VE = dtype == CNNITMO_BF16 ? 8 : 4;
  CNN_REQUIRE(cin % VE == 0 && (cin / VE) <= 64 && ((cin / VE) & (cin / VE - 1)) == 0,
              "head: cin/%d must be a power of two <= 64", VE);
  const long P = (long)n * h * w;
  CNN_REQUIRE(P < (1L << 31), "head: too many pixels");
  const int G = cnnitmo_head_rows(P);
  if (launch_head2<false>(dtype, x, n, h, h_valid, w, cin, wt, b, nullptr, yhat, nullptr, 0.f, nullptr, scale,
                          shift, nullptr, G, s))
    return cnnitmo_check_launch("head_fwd");
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL((head_kernel<bf16, false>), dim3(G), dim3(256), 0, s, (const bf16*)x, n, h,
                       h_valid, w, cin, wt, b, nullptr, yhat, nullptr, 0.f, nullptr, scale, shift, nullptr);
  else
    hipLaunchKernelGGL((head_kernel<float, false>), dim3(G), dim3(256), 0, s, (const float*)x, n, h,
                       h_valid, w, cin, wt, b, nullptr, yhat, nullptr, 0.f, nullptr, scale, shift, nullptr);
  return cnnitmo_check_launch("head_fwd");
}

static int head_fwd_bwd(int dtype, const void* x, int n, int h, int h_valid, int w, int cin, const float* wt,
                        const float* b, const float* scale, const float* shift, const float* target, void* dx,
                        float* g3, float* part, double grad_numel, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int VE = dtype == CNNITMO_BF16 ? 8 : 4;
  CNN_REQUIRE(cin % VE == 0 && (cin / VE) <= 64 && ((cin / VE) & (cin / VE - 1)) == 0,
              "head: cin/%d must be a power of two <= 64", VE);
  const long P = (long)n * h * w;
  CNN_REQUIRE(P < (1L << 31), "head: too many pixels");
  const int G = cnnitmo_head_rows(P);
  const double numel = grad_numel > 0.0 ? grad_numel : (double)n * h_valid * w * 3;
  const float inv_numel = (float)(1.0 / numel);
  if (launch_head2<true>(dtype, x, n, h, h_valid, w, cin, wt, b, target, nullptr, dx, inv_numel, part, scale,
                         shift, g3, G, s))
    return cnnitmo_check_launch("head_fwd_bwd");
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL((head_kernel<bf16, true>), dim3(G), dim3(256), 0, s, (const bf16*)x, n, h,
                       h_valid, w, cin, wt, b, target, nullptr, (bf16*)dx, inv_numel, part, scale, shift, g3);
  else
    hipLaunchKernelGGL((head_kernel<float, true>), dim3(G), dim3(256), 0, s, (const float*)x, n, h,
                       h_valid, w, cin, wt, b, target, nullptr, (float*)dx, inv_numel, part, scale, shift, g3);
  return cnnitmo_check_launch("head_fwd_bwd");
}

extern "C" int cnnitmo_head_fwd_bwd(int dtype, const void* x, int n, int h, int h_valid, int w,
                                    int cin, const float* wt, const float* b, const float* scale,
                                    const float* shift, const float* target, void* dx, float* part,
                                    double grad_numel, void* stream) {
  CNN_REQUIRE(dx, "head_fwd_bwd: null dx");
  return head_fwd_bwd(dtype, x, n, h, h_valid, w, cin, wt, b, scale, shift, target, dx, nullptr, part, grad_numel,
                      stream);
}

extern "C" int cnnitmo_head_fwd_bwd_g3(int dtype, const void* x, int n, int h, int h_valid, int w, int cin,
                                       const float* wt, const float* b, const float* scale, const float* shift,
                                       const float* target, float* g3, float* part, double grad_numel,
                                       void* stream) {
  CNN_REQUIRE(g3, "head_fwd_bwd_g3: null g3");
  return head_fwd_bwd(dtype, x, n, h, h_valid, w, cin, wt, b, scale, shift, target, nullptr, g3, part, grad_numel,
                      stream);
}

// Folded input BN (x = r, y = r*s + h): dW[o][c] = s[c]*sum(dz*r) + h[c]*db[o].
__global__ void head_final_kernel(const double* __restrict__ ws, int G, int cin, double numel,
                                  float* loss_acc, float* dw, float* db, const float* fs,
                                  const float* fh, float* raw) {
  const int ncol = 5 + 3 * cin;
  const int k = wave_col();
  if (k < ncol) {
    const double s = fold(ws, G, ncol, k);
    double dbo = 0.0;
    if (k >= 5 && fh) dbo = fold(ws, G, ncol, 2 + (k - 5) / cin);
    if ((threadIdx.x & 63) != 0) return;
    if (k == 0) loss_acc[0] = (float)(s / numel);
    else if (k == 1) loss_acc[1] = (float)(s / (numel / 3.0));
    else if (k < 5) db[k - 2] = (float)s;
    else {
      const int c = (k - 5) % cin;
      dw[k - 5] = (float)((fs ? s * fs[c] : s) + (fh ? dbo * fh[c] : 0.0));
      if (raw) raw[k - 5] = (float)s;
    }
  }
}

extern "C" int cnnitmo_head_finalize(const float* part, long rows, int cin, double numel,
                                     const float* scale, const float* shift, float* loss_acc,
                                     float* dw, float* db, float* raw_out, void* workspace,
                                     void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const int G = colsum_stage1_launch(part, rows, 5 + 3 * cin, workspace, s);
  hipLaunchKernelGGL(head_final_kernel, dim3(wave_grid(5 + 3 * cin)), dim3(256), 0, s, (const double*)workspace, G, cin,
                     numel, loss_acc, dw, db, scale, shift, raw_out);
  return cnnitmo_check_launch("head_finalize");
}

// ----------------------------------------------------------------------------
// RMSprop (Keras 2.2 defaults; eps outside the sqrt) over one flat buffer.
// ----------------------------------------------------------------------------
__global__ void rmsprop_kernel(float* __restrict__ p, const float* __restrict__ g,
                               float* __restrict__ a, long n, float lr, float rho, float eps,
                               float gs) {
  const long n4 = n / 4;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n4;
       i += (long)gridDim.x * blockDim.x) {
    float4 pv = reinterpret_cast<float4*>(p)[i];
    const float4 gv = reinterpret_cast<const float4*>(g)[i];
    float4 av = reinterpret_cast<float4*>(a)[i];
    float* pp = &pv.x;
    const float* gg = &gv.x;
    float* aa = &av.x;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const float gr = gg[e] * gs;
      aa[e] = rho * aa[e] + (1.f - rho) * gr * gr;
      pp[e] -= lr * gr / (sqrtf(aa[e]) + eps);
    }
    reinterpret_cast<float4*>(p)[i] = pv;
    reinterpret_cast<float4*>(a)[i] = av;
  }
  for (long i = n4 * 4 + blockIdx.x * (long)blockDim.x + threadIdx.x; i < n;
       i += (long)gridDim.x * blockDim.x) {
    const float gr = g[i] * gs;
    a[i] = rho * a[i] + (1.f - rho) * gr * gr;
    p[i] -= lr * gr / (sqrtf(a[i]) + eps);
  }
}

extern "C" int cnnitmo_rmsprop(float* p, const float* g, float* a, long n, float lr, float rho,
                               float eps, float grad_scale, void* stream) {
  CNN_REQUIRE(((uintptr_t)p | (uintptr_t)g | (uintptr_t)a) % 16 == 0, "rmsprop: buffers must be 16-byte aligned");
  hipLaunchKernelGGL(rmsprop_kernel, dim3(grid_for(n / 4 + 1, 256, 2048)), dim3(256), 0,
                     (hipStream_t)stream, p, g, a, n, lr, rho, eps, grad_scale);
  return cnnitmo_check_launch("rmsprop");
}

// ----------------------------------------------------------------------------
// Weight preparation: fp32 master -> dtype copies in the layouts kernels read.
// ----------------------------------------------------------------------------
template <typename T>
__global__ void prep_conv_kernel(const float* __restrict__ w, int cout, int cin, T* __restrict__ wf,
                                 T* __restrict__ wflip) {
  const long total = (long)cout * 9 * cin;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % cin);
    const long t = i / cin;
    const int rs = (int)(t % 9), co = (int)(t / 9);
    const T v = from_f32<T>(w[i]);
    wf[i] = v;
    if (wflip) {  // wflip[ci][2-r][2-s][co] = w[co][r][s][ci]
      const int r = rs / 3, s = rs % 3;
      wflip[((long)ci * 9 + (2 - r) * 3 + (2 - s)) * cout + co] = v;
    }
  }
}

template <typename T>
__global__ void prep_tconv_kernel(const float* __restrict__ k, int cout, int cin, T* __restrict__ kf,
                                  T* __restrict__ kT) {
  const long total = 4L * cout * cin;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total;
       i += (long)gridDim.x * blockDim.x) {
    const int ci = (int)(i % cin);
    const long t = i / cin;
    const int co = (int)(t % cout), tap = (int)(t / cout);
    const T v = from_f32<T>(k[i]);
    kf[i] = v;
    kT[((long)ci * 4 + tap) * cout + co] = v;  // kT[ci][a][b][co]
  }
}

template <typename T>
__global__ void prep_c3_kernel(const float* __restrict__ w, int cout, T* __restrict__ wp) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= cout * 32) return;
  const int co = i / 32, k = i % 32;
  wp[i] = from_f32<T>(k < 27 ? w[co * 27 + k] : 0.f);
}

extern "C" int cnnitmo_prep_conv3x3_weights(int dtype, const float* w, int cout, int cin,
                                            void* w_fwd, void* w_flip, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const long n = (long)cout * 9 * cin;
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL(prep_conv_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, s, w, cout, cin,
                       (bf16*)w_fwd, (bf16*)w_flip);
  else
    hipLaunchKernelGGL(prep_conv_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, w, cout, cin,
                       (float*)w_fwd, (float*)w_flip);
  return cnnitmo_check_launch("prep_conv3x3_weights");
}

extern "C" int cnnitmo_prep_tconv2x2_weights(int dtype, const float* k, int cout, int cin,
                                             void* k_fwd, void* kT, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const long n = 4L * cout * cin;
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL(prep_tconv_kernel<bf16>, dim3(grid_for(n)), dim3(256), 0, s, k, cout, cin,
                       (bf16*)k_fwd, (bf16*)kT);
  else
    hipLaunchKernelGGL(prep_tconv_kernel<float>, dim3(grid_for(n)), dim3(256), 0, s, k, cout, cin,
                       (float*)k_fwd, (float*)kT);
  return cnnitmo_check_launch("prep_tconv2x2_weights");
}

extern "C" int cnnitmo_prep_c3_weights(int dtype, const float* w, int cout, void* w_packed,
                                       void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL(prep_c3_kernel<bf16>, dim3((cout * 32 + 255) / 256), dim3(256), 0, s, w,
                       cout, (bf16*)w_packed);
  else
    hipLaunchKernelGGL(prep_c3_kernel<float>, dim3((cout * 32 + 255) / 256), dim3(256), 0, s, w,
                       cout, (float*)w_packed);
  return cnnitmo_check_launch("prep_c3_weights");
}

// ----------------------------------------------------------------------------
// First-layer packing: x [n][h_valid][w][3] fp32 -> cols [n][h][w][32] dtype.
// ----------------------------------------------------------------------------
// One workgroup per 256-pixel segment of an output row: the three input rows it
// reads ((256+2) pixels x 3 channels each, fp32) are staged in LDS once (coalesced,
// zero outside the image / below h_valid), every thread assembles its pixel's 27
// (+5 zero) values, and the 256 x 32 tile leaves through LDS as lane-linear 16-byte
// stores (4.3 GB of bf16 columns per 1080p b32 step: a pure write stream).
template <typename T>
__global__ __launch_bounds__(256) void im2col_c3_kernel(const float* __restrict__ x, int Hv, int H, int W,
                                                        int segs, T* __restrict__ cols) {
  constexpr int SEG = 256, PW = SEG + 2;
  constexpr int VE = Vec16<T>::N;
  __shared__ float xs[3][PW * 3];
  __shared__ __attribute__((aligned(16))) T tile[SEG * 32];
  const int seg = blockIdx.x % segs;
  const long row = blockIdx.x / segs;  // n * H + h
  const int h = (int)(row % H);
  const long n = row / H;
  const int w0 = seg * SEG;
  for (int i = threadIdx.x; i < 3 * PW * 3; i += SEG) {
    const int r = i / (PW * 3), q = i - r * (PW * 3);
    const int ww = w0 - 1 + q / 3, hh = h + r - 1;
    float v = 0.f;
    if (hh >= 0 && hh < Hv && ww >= 0 && ww < W) v = x[((n * Hv + hh) * W + ww) * 3 + q % 3];
    xs[r][q] = v;
  }
  __syncthreads();
  const int t = threadIdx.x;
  float v[32];
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const int tap = k / 3, c = k - tap * 3;
    v[k] = k < 27 ? xs[tap / 3][(t + tap % 3) * 3 + c] : 0.f;
  }
#pragma unroll
  for (int j = 0; j < 32; j += VE) Pack16<T>::store(tile + t * 32 + j, v + j);
  __syncthreads();
  const int npx = min(SEG, W - w0);
  const uint4* src = reinterpret_cast<const uint4*>(tile);
  uint4* dst = reinterpret_cast<uint4*>(cols + ((size_t)row * W + w0) * 32);
  const int nv = npx * 32 / VE;
  for (int i = t; i < nv; i += SEG) dst[i] = src[i];
}

extern "C" int cnnitmo_im2col_c3(int dtype, const float* x, int n, int h_valid, int h, int w,
                                 void* cols, void* stream) {
  CNN_REQUIRE(h_valid <= h, "im2col_c3: h_valid > h");
  CNN_REQUIRE(n > 0 && h > 0 && w > 0, "im2col_c3: bad shape");
  hipStream_t s = (hipStream_t)stream;
  const int segs = (w + 255) / 256;
  const long blocks = (long)n * h * segs;
  CNN_REQUIRE(blocks < (1L << 31), "im2col_c3: too large");
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL(im2col_c3_kernel<bf16>, dim3((unsigned)blocks), dim3(256), 0, s, x, h_valid, h, w, segs,
                       (bf16*)cols);
  else
    hipLaunchKernelGGL(im2col_c3_kernel<float>, dim3((unsigned)blocks), dim3(256), 0, s, x, h_valid, h, w, segs,
                       (float*)cols);
  return cnnitmo_check_launch("im2col_c3");
}

// ----------------------------------------------------------------------------
// BN folding (training): a consumer of a BN output y = r*s + h (per input
// channel) reads the stored r and folds the affine instead of materialising y.
//   conv3x3: W' = W*s, bias' = b + sum_t u_t, u_t[co] = sum_ci W[co][t][ci] h[ci];
//            zero padding applies to y, so the conv epilogue subtracts u_t for every
//            out-of-bounds tap t of a border pixel via the table
//            border[co] = {Utop, Ubot, Uleft, Uright, u0, u2, u6, u8}.
//   tconv:   K' = K*s, bias'[tap][co] = b[co] + sum_ci K[tap][co][ci] h[ci] (no padding).
// ----------------------------------------------------------------------------
__device__ float block_sum_det(float v, float* red) {
  // deterministic 256-thread tree sum; every thread returns the total
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (t < o) red[t] += red[t + o];
    __syncthreads();
  }
  const float s = red[0];
  __syncthreads();
  return s;
}

template <typename T>
__global__ void fold_conv_kernel(const float* __restrict__ w, const float* __restrict__ b,
                                 const float* __restrict__ s, const float* __restrict__ h, int cout,
                                 int cin, int ntaps, T* __restrict__ wout, float* __restrict__ bout,
                                 float* __restrict__ border) {
  __shared__ float red[256];
  const int co = blockIdx.x;
  float u[9];
#pragma unroll
  for (int t = 0; t < 9; ++t) {  // ntaps == 9
    float acc = 0.f;
    for (int ci = threadIdx.x; ci < cin; ci += blockDim.x) {
      const size_t i = ((size_t)co * ntaps + t) * cin + ci;
      const float wv = w[i];
      wout[i] = from_f32<T>(s ? wv * s[ci] : wv);
      if (h) acc += wv * h[ci];
    }
    u[t] = block_sum_det(acc, red);
  }
  if (threadIdx.x == 0) {
    float bsum = b ? b[co] : 0.f;
#pragma unroll
    for (int t = 0; t < 9; ++t) bsum += u[t];
    bout[co] = bsum;
    if (border && ntaps == 9) {
      float* U = border + (size_t)co * 8;
      U[0] = u[0] + u[1] + u[2];
      U[1] = u[6] + u[7] + u[8];
      U[2] = u[0] + u[3] + u[6];
      U[3] = u[2] + u[5] + u[8];
      U[4] = u[0];
      U[5] = u[2];
      U[6] = u[6];
      U[7] = u[8];
    }
  }
}

extern "C" int cnnitmo_fold_conv3x3(int dtype, const float* w, const float* bias, const float* scale,
                                    const float* shift, int cout, int cin, void* w_out,
                                    float* bias_out, float* border, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL(fold_conv_kernel<bf16>, dim3(cout), dim3(256), 0, s, w, bias, scale, shift, cout,
                       cin, 9, (bf16*)w_out, bias_out, border);
  else
    hipLaunchKernelGGL(fold_conv_kernel<float>, dim3(cout), dim3(256), 0, s, w, bias, scale, shift,
                       cout, cin, 9, (float*)w_out, bias_out, border);
  return cnnitmo_check_launch("fold_conv3x3");
}

// tconv: k [4][cout][cin] viewed as [4*cout rows][cin]: one block per (tap, co)
template <typename T>
__global__ void fold_tconv_kernel(const float* __restrict__ k, const float* __restrict__ b,
                                  const float* __restrict__ s, const float* __restrict__ h, int cout,
                                  int cin, T* __restrict__ kout, float* __restrict__ bout) {
  __shared__ float red[256];
  const int row = blockIdx.x, co = row % cout;
  float acc = 0.f;
  for (int ci = threadIdx.x; ci < cin; ci += blockDim.x) {
    const size_t i = (size_t)row * cin + ci;
    const float kv = k[i];
    kout[i] = from_f32<T>(s ? kv * s[ci] : kv);
    if (h) acc += kv * h[ci];
  }
  const float tot = block_sum_det(acc, red);
  if (threadIdx.x == 0) bout[row] = (b ? b[co] : 0.f) + tot;
}

extern "C" int cnnitmo_fold_tconv2x2(int dtype, const float* k, const float* bias, const float* scale,
                                     const float* shift, int cout, int cin, void* k_out,
                                     float* bias_out, void* stream) {
  hipStream_t s = (hipStream_t)stream;
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL(fold_tconv_kernel<bf16>, dim3(4 * cout), dim3(256), 0, s, k, bias, scale, shift,
                       cout, cin, (bf16*)k_out, bias_out);
  else
    hipLaunchKernelGGL(fold_tconv_kernel<float>, dim3(4 * cout), dim3(256), 0, s, k, bias, scale, shift,
                       cout, cin, (float*)k_out, bias_out);
  return cnnitmo_check_launch("fold_tconv2x2");
}

// Border sums of an output gradient dz [n][h][w][c] for the folded-BN conv
// weight-gradient correction: rows [n*BS_SEG][8][c] of partials (reduce with
// cnnitmo_colsum) = {row 0, row h-1, col 0, col w-1, (0,0), (0,w-1), (h-1,0), (h-1,w-1)}.
constexpr int BS_SEG = 16;
template <typename T>
__global__ void border_sums_kernel(const T* __restrict__ dz, int H, int W, int C,
                                   float* __restrict__ part) {
  const int img = blockIdx.x / BS_SEG, seg = blockIdx.x % BS_SEG;
  const T* base = dz + (size_t)img * H * W * C;
  float* out = part + (size_t)blockIdx.x * 8 * C;
  const int w0 = (int)((long)W * seg / BS_SEG), w1 = (int)((long)W * (seg + 1) / BS_SEG);
  const int h0 = (int)((long)H * seg / BS_SEG), h1 = (int)((long)H * (seg + 1) / BS_SEG);
  for (int c = threadIdx.x; c < C; c += blockDim.x) {
    float top = 0.f, bot = 0.f, lef = 0.f, rig = 0.f;
    for (int w = w0; w < w1; ++w) {
      top += to_f32(base[(size_t)w * C + c]);
      bot += to_f32(base[((size_t)(H - 1) * W + w) * C + c]);
    }
    for (int hh = h0; hh < h1; ++hh) {
      lef += to_f32(base[((size_t)hh * W) * C + c]);
      rig += to_f32(base[((size_t)hh * W + W - 1) * C + c]);
    }
    const bool s0 = seg == 0;
    out[0 * C + c] = top;
    out[1 * C + c] = bot;
    out[2 * C + c] = lef;
    out[3 * C + c] = rig;
    out[4 * C + c] = s0 ? to_f32(base[c]) : 0.f;
    out[5 * C + c] = s0 ? to_f32(base[(size_t)(W - 1) * C + c]) : 0.f;
    out[6 * C + c] = s0 ? to_f32(base[((size_t)(H - 1) * W) * C + c]) : 0.f;
    out[7 * C + c] = s0 ? to_f32(base[((size_t)(H - 1) * W + W - 1) * C + c]) : 0.f;
  }
}

extern "C" int cnnitmo_border_rows(int n) { return n * BS_SEG; }

extern "C" int cnnitmo_border_sums(int dtype, const void* dz, int n, int h, int w, int c, float* part,
                                   void* stream) {
  CNN_REQUIRE(n > 0 && h > 0 && w > 0 && c > 0, "border_sums: empty");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == CNNITMO_BF16)
    hipLaunchKernelGGL(border_sums_kernel<bf16>, dim3(n * BS_SEG), dim3(256), 0, s, (const bf16*)dz, h, w, c, part);
  else
    hipLaunchKernelGGL(border_sums_kernel<float>, dim3(n * BS_SEG), dim3(256), 0, s, (const float*)dz, h, w, c, part);
  return cnnitmo_check_launch("border_sums");
}

// ----------------------------------------------------------------------------
// BN-backward sums without a pass over the activations.  For a BN output v whose
// gradient is the input-gradient of a linear consumer (conv3x3 'same', tconv2x2,
// the 1x1 head), both sums the BN backward needs follow from quantities the
// consumer's weight gradient already produced:
//   sum_q dy[q][ci]             = sum_{co,t} W[co][t][ci] * V[co][t]
//   sum_q dy[q][ci] * rhat[q][ci] = inv[ci] * sum_{co,t} W[co][t][ci] * (raw[co][t][ci] - mean[ci] * V[co][t])
// raw = sum_p dz[p][co] * r[p + off_t][ci] (zero padded) and V[co][t] = the sum of dz
// over the pixels whose tap t lands inside the image (conv: db - border sums;
// tconv: the per-tap parity sums; head: db).  Exact in real arithmetic (the
// dgrad is the transpose of the same linear map), O(weights) work.
// part[0][c] = sum dy, part[1][c] = sum dy * rhat (one row for cnnitmo_bn_bwd_finalize).
// mode 1: conv3x3, w/raw [cout][9][cin_tot], V from db[cout] and border sums bs[8][cout]
// mode 2: tconv2x2, w/raw [4][cout][cin_tot], V = par[4*cout]
// mode 3: head 1x1, w/raw [3][cin_tot], V = db[3]
// ----------------------------------------------------------------------------
__device__ __forceinline__ double conv_v(const float* db, const float* bs, int C, int co, int t) {
  const int r = t / 3, q = t - 3 * r;
  double o = 0.0;
  if (r == 0) o += bs[0 * C + co];
  if (r == 2) o += bs[1 * C + co];
  if (q == 0) o += bs[2 * C + co];
  if (q == 2) o += bs[3 * C + co];
  if (r == 0 && q == 0) o -= bs[4 * C + co];
  if (r == 0 && q == 2) o -= bs[5 * C + co];
  if (r == 2 && q == 0) o -= bs[6 * C + co];
  if (r == 2 && q == 2) o -= bs[7 * C + co];
  return (double)db[co] - o;
}

// Grid (c/64, CNNITMO_CONSUMER_ROWS); a block's 4 waves split its slice of the
// K = cout*taps (co, tap) pairs (w/raw rows k*cin_tot, coalesced over ci) and
// reduce in LDS; every grid row writes one partial row (linear in the slices).
__global__ void bn_consumer_sums_kernel(int mode, const float* __restrict__ w, const float* __restrict__ raw,
                                        int cout, int cin_tot, int ci0, int c, const float* __restrict__ db,
                                        const float* __restrict__ vt, const float* __restrict__ mean,
                                        const float* __restrict__ inv, float* __restrict__ part) {
  const int cl = threadIdx.x & 63, sub = threadIdx.x >> 6;
  const int j = blockIdx.x * 64 + cl;
  const int K = cout * (mode == 1 ? 9 : (mode == 2 ? 4 : 1));
  const int slices = gridDim.y * 4, sl = blockIdx.y * 4 + sub;
  const int k0 = (int)((long)K * sl / slices), k1 = (int)((long)K * (sl + 1) / slices);
  double swv = 0.0, swr = 0.0;
  if (j < c) {
    const int ci = ci0 + j;
    for (int k = k0; k < k1; ++k) {
      const double v = mode == 1 ? conv_v(db, vt, cout, k / 9, k % 9) : (mode == 2 ? (double)vt[k] : (double)db[k]);
      const size_t idx = (size_t)k * cin_tot + ci;
      const double wv = w[idx];
      swv += wv * v;
      swr += wv * raw[idx];
    }
  }
  __shared__ double red[2][256];
  red[0][threadIdx.x] = swv;
  red[1][threadIdx.x] = swr;
  __syncthreads();
  if (sub == 0 && j < c) {
    swv = ((red[0][cl] + red[0][cl + 64]) + red[0][cl + 128]) + red[0][cl + 192];
    swr = ((red[1][cl] + red[1][cl + 64]) + red[1][cl + 128]) + red[1][cl + 192];
    float* o = part + (size_t)blockIdx.y * 2 * c;
    o[j] = (float)swv;
    o[c + j] = (float)(inv[j] * (swr - (double)mean[j] * swv));
  }
}

extern "C" int cnnitmo_bn_consumer_sums(int mode, const float* w, const float* raw, int cout, int cin_tot,
                                        int ci0, int c, const float* db, const float* vtab,
                                        const float* mean, const float* invstd, float* part,
                                        void* stream) {
  CNN_REQUIRE(mode >= 1 && mode <= 3 && ci0 >= 0 && ci0 + c <= cin_tot && (mode == 2 || db),
              "bn_consumer_sums: bad arguments");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(bn_consumer_sums_kernel, dim3((c + 63) / 64, CNNITMO_CONSUMER_ROWS), dim3(256), 0, s,
                     mode, w, raw, cout, cin_tot, ci0, c, db, vtab, mean, invstd, part);
  return cnnitmo_check_launch("bn_consumer_sums");
}

