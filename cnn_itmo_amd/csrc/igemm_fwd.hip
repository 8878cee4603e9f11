#include <cstdio>
// Implicit-GEMM convolution on MFMA, "forward family" (K = taps x channels).
//
// One kernel template serves every GEMM of the U-Net whose reduction runs over
// (tap, channel) of an NHWC source:
//   conv3x3 fwd    (Conv2D 'same', model.py:196)      9 taps, scale 1
//   conv3x3 dgrad  (its input gradient)               9 taps on dz, flipped W
//   tconv2x2 fwd   (Conv2DTranspose s2, model.py:200) 1 tap, N = 4*cout, scatter store
//   tconv2x2 dgrad                                    4 taps, scale 2 gather
//   1-tap GEMM over im2col columns (conv2d_1, Cin=3)
//
// GEMM view: C[m][n] = sum_k A[m][k] * B[n][k]; m = output pixel (n,h,w),
// n = output channel, k = (tap, c).  A rows are gathered per tap from the
// source grid (zero outside = 'same' padding); B is the [N][K] weight matrix.
// Both operands are K-contiguous, so every global load is a 16-byte NHWC
// vector.  A K-step is 64 bytes of K per row (32 bf16 / 16 f32).  Tiles are
// staged through LDS (double buffered, one barrier per K-step) and consumed by
// v_mfma_f32_16x16x32_bf16 (bf16) or 4x v_mfma_f32_16x16x4_f32 (f32; lane
// group g owns channels 4g..4g+3 so each lane reads one 16-byte fragment per
// 4 MFMAs).  Epilogue: bias, ReLU, optional inference BN affine, BN partial
// sums (deterministic per-tile slabs), store (plain or tconv pixel-scatter).
#include <cstdlib>
#include <cstring>

#include "igemm_common.h"

// LDS image of a [rows][64 B] tile: 16-byte chunk c of row r stored at slot
// c ^ (((r >> 3) & 1) << 1).  With 16-row MFMA groups read by ds_read_b128
// (lane l: row l&15, chunk l>>4) every 16-lane bank group hits 16 distinct
// 16-byte slots (conflict-free); the staging ds_write_b128 stays conflict-free.
__device__ __forceinline__ int tile_off(int row, int chunk) {
  return (row << 6) + ((chunk ^ (((row >> 3) & 1) << 1)) << 4);
}

template <typename T, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void igemm_fwd_kernel(const FwdArgs p) {
  constexpr int VE = Vec16<T>::N;
  constexpr int KE = 4 * VE;  // K elements per step (64 bytes)
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int A_SEGS = BM * 4, B_SEGS = BN * 4;
  constexpr int SA = (A_SEGS + 255) / 256, SB = (B_SEGS + 255) / 256;
  constexpr int STAGE = (BM + BN) * 64;
  static_assert(WM * WN == 4, "4 waves");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lid = xcd_remap(blockIdx.x, p.mblocks * p.nblocks);
  const int mb = lid / p.nblocks, nb = lid - mb * p.nblocks;
  const long m0 = (long)mb * BM;
  const int n0 = nb * BN;
  const long K = (long)p.ntaps * p.cin;

  const T* __restrict__ A = (const T*)p.a;
  const T* __restrict__ B = (const T*)p.b;

  // Per-thread A rows (fixed over K): image index and base coordinates.
  int a_img[SA], a_h[SA], a_w[SA];
  const long hw = (long)p.ho * p.wo;
#pragma unroll
  for (int j = 0; j < SA; ++j) {
    const int seg = tid + j * 256;
    const long m = m0 + (seg >> 2);
    a_img[j] = -1;
    a_h[j] = 0;
    a_w[j] = 0;
    if (seg < A_SEGS && m < p.M) {
      const int img = (int)(m / hw);
      const int rem = (int)(m - (long)img * hw);
      const int oh = rem / p.wo;
      a_img[j] = img;
      a_h[j] = oh * p.scale;
      a_w[j] = (rem - oh * p.wo) * p.scale;
    }
  }
  const int chunk = tid & 3;

  uint4 ra[SA], rb[SB];
  const int steps_per_tap = p.cin / KE;
  const int nk = p.ntaps * steps_per_tap;

  auto load = [&](int tap, int c0) {
    const int ddy = ((p.dyc >> (2 * tap)) & 3) - 1, ddx = ((p.dxc >> (2 * tap)) & 3) - 1;
#pragma unroll
    for (int j = 0; j < SA; ++j) {
      const int hh = a_h[j] + ddy, ww = a_w[j] + ddx;
      uint4 v = make_uint4(0, 0, 0, 0);
      if (a_img[j] >= 0 && hh >= 0 && hh < p.hs && ww >= 0 && ww < p.ws) {
        const size_t off = ((size_t)((long)a_img[j] * p.hs + hh) * p.ws + ww) * p.a_ld + p.a_off +
                           c0 + chunk * VE;
        v = *reinterpret_cast<const uint4*>(A + off);
      }
      ra[j] = v;
    }
#pragma unroll
    for (int j = 0; j < SB; ++j) {
      const int seg = tid + j * 256;
      if (seg < B_SEGS) {
        const size_t off = (size_t)(n0 + (seg >> 2)) * K + (long)tap * p.cin + c0 + chunk * VE;
        rb[j] = *reinterpret_cast<const uint4*>(B + off);
      }
    }
  };
  auto store = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + BM * 64;
#pragma unroll
    for (int j = 0; j < SA; ++j) {
      const int seg = tid + j * 256;
      if (seg < A_SEGS) *reinterpret_cast<uint4*>(As + tile_off(seg >> 2, chunk)) = ra[j];
    }
#pragma unroll
    for (int j = 0; j < SB; ++j) {
      const int seg = tid + j * 256;
      if (seg < B_SEGS) *reinterpret_cast<uint4*>(Bs + tile_off(seg >> 2, chunk)) = rb[j];
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  int tap = 0, c0 = 0;
  load(0, 0);
  store(0);
  __syncthreads();
  int cur = 0;
  for (int ks = 0; ks < nk; ++ks) {
    const bool more = ks + 1 < nk;
    if (more) {
      c0 += KE;
      if (c0 == p.cin) { c0 = 0; ++tap; }
      load(tap, c0);
    }
    const char* As = smem + cur * STAGE;
    const char* Bs = As + BM * 64;
    uint4 af[FM], bfr[FN];
    const int frow = lane & 15, fch = lane >> 4;
#pragma unroll
    for (int i = 0; i < FM; ++i)
      af[i] = *reinterpret_cast<const uint4*>(As + tile_off(wm * TM + i * 16 + frow, fch));
#pragma unroll
    for (int j = 0; j < FN; ++j)
      bfr[j] = *reinterpret_cast<const uint4*>(Bs + tile_off(wn * TN + j * 16 + frow, fch));
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) Mma<T>::run(acc[i][j], af[i], bfr[j]);
    if (more) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  // ---------------- epilogue ----------------
  const bool relu = p.flags & CNNITMO_RELU, aff = p.flags & CNNITMO_AFFINE,
             stats = p.flags & CNNITMO_STATS;
  T* __restrict__ O = (T*)p.out;
  float bj[FN], sj[FN], hj[FN];
  int coj[FN], tapoff[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * TN + j * 16 + (lane & 15);
    int co = n, tp = 0;
    if (p.scatter) {
      tp = n / p.cout;
      co = n - tp * p.cout;
    }
    coj[j] = co;
    tapoff[j] = (tp >> 1) * 2 * p.wo + (tp & 1);
    bj[j] = p.bias ? p.bias[(p.flags & CNNITMO_BIAS_PER_COL) ? n : co] : 0.f;
    sj[j] = aff ? p.aff_scale[co] : 1.f;
    hj[j] = aff ? p.aff_shift[co] : 0.f;
  }
  float s1[FN], s2[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) s1[j] = s2[j] = 0.f;

#pragma unroll
  for (int i = 0; i < FM; ++i) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long m = m0 + wm * TM + i * 16 + (lane >> 4) * 4 + r;
      if (m >= p.M) continue;
      int boh = 1, bow = 1;
      if (p.border) {
        const int rem = (int)(m % hw);
        boh = rem / p.wo;
        bow = rem - boh * p.wo;
      }
      long pixbase;
      if (p.scatter) {
        const int img = (int)(m / hw);
        const int rem = (int)(m - (long)img * hw);
        const int ii = rem / p.wo, jj = rem - ii * p.wo;
        pixbase = ((long)img * 2 * p.ho + 2 * ii) * 2 * p.wo + 2 * jj;
      } else {
        pixbase = m;
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        float v = acc[i][j][r] + bj[j];
        if (p.border) v -= border_corr(p.border + (size_t)coj[j] * 8, boh, bow, p.ho, p.wo);
        if (relu) v = fmaxf(v, 0.f);
        if (aff) v = v * sj[j] + hj[j];
        s1[j] += v;
        s2[j] += v * v;
        const size_t off = (size_t)(pixbase + (p.scatter ? tapoff[j] : 0)) * p.out_ld + p.out_off + coj[j];
        O[off] = from_f32<T>(v);
      }
    }
  }

  if (stats) {
    // rows beyond M contributed nothing (skipped above)
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      s1[j] += __shfl_xor(s1[j], 16, 64);
      s1[j] += __shfl_xor(s1[j], 32, 64);
      s2[j] += __shfl_xor(s2[j], 16, 64);
      s2[j] += __shfl_xor(s2[j], 32, 64);
    }
    float* red = reinterpret_cast<float*>(smem);  // [WM][BN][2]; main loop ended with a barrier
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * TN + j * 16 + lane;
        red[(wm * BN + col) * 2 + 0] = s1[j];
        red[(wm * BN + col) * 2 + 1] = s2[j];
      }
    }
    __syncthreads();
    if (tid < BN) {
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < WM; ++w) {
        t1 += red[(w * BN + tid) * 2 + 0];
        t2 += red[(w * BN + tid) * 2 + 1];
      }
      float* st = p.stats + (size_t)mb * 2 * p.N;
      st[n0 + tid] = t1;
      st[p.N + n0 + tid] = t2;
    }
  }
}

// ----------------------------------------------------------------------------
// Host dispatch
// ----------------------------------------------------------------------------
namespace {

struct Cfg {
  int bm, bn;
};
Cfg pick_cfg(int N) {
  if (N >= 128 && N % 128 == 0) return {128, 128};
  if (N % 64 == 0) return {256, 64};
  return {256, 32};
}

template <typename T>
int launch_fwd(FwdArgs a, hipStream_t s, const char* what) {
  CNN_REQUIRE(a.N % 32 == 0, "%s: output columns %d not a multiple of 32", what, a.N);
  CNN_REQUIRE(a.cin % (4 * Vec16<T>::N) == 0, "%s: channels per tap %d not a multiple of %d", what,
              a.cin, 4 * Vec16<T>::N);
  CNN_REQUIRE(a.a_ld % Vec16<T>::N == 0 && a.a_off % Vec16<T>::N == 0,
              "%s: source view ld/off must be multiples of %d", what, Vec16<T>::N);
  CNN_REQUIRE(a.M > 0 && a.ntaps >= 1 && a.ntaps <= 9, "%s: bad sizes", what);
  Cfg c = pick_cfg(a.N);
  a.mblocks = (int)((a.M + c.bm - 1) / c.bm);
  a.nblocks = a.N / c.bn;
  const long total = (long)a.mblocks * a.nblocks;
  CNN_REQUIRE(total < (1L << 31), "%s: grid too large", what);
  dim3 grid((unsigned)total), block(256);
  if (c.bm == 128)
    hipLaunchKernelGGL((igemm_fwd_kernel<T, 128, 128, 2, 2>), grid, block, 0, s, a);
  else if (c.bn == 64)
    hipLaunchKernelGGL((igemm_fwd_kernel<T, 256, 64, 4, 1>), grid, block, 0, s, a);
  else
    hipLaunchKernelGGL((igemm_fwd_kernel<T, 256, 32, 4, 1>), grid, block, 0, s, a);
  return cnnitmo_check_launch(what);
}

int dispatch(int dtype, const FwdArgs& a, void* stream, const char* what) {
  hipStream_t s = (hipStream_t)stream;
  if (dtype == CNNITMO_BF16 && halo_handles(a)) return launch_halo(a, s, what);
  if (dtype == CNNITMO_F32 && halo_handles(a, true)) return launch_halo(a, s, what, true);
  if (fwd2_handles(a.N)) {
    if (dtype == CNNITMO_BF16) return launch_fwd2<bf16>(a, s, what);
    if (dtype == CNNITMO_F32) return launch_fwd2<float>(a, s, what);
  }
  if (dtype == CNNITMO_BF16) return launch_fwd<bf16>(a, s, what);
  if (dtype == CNNITMO_F32) return launch_fwd<float>(a, s, what);
  cnnitmo_set_error("%s: unsupported dtype %d", what, dtype);
  return CNNITMO_EUNSUPPORTED;
}

FwdArgs base_args() {
  FwdArgs a;
  memset(&a, 0, sizeof(a));
  a.scale = 1;
  a.ntaps = 1;
  a.dyc = a.dxc = 1;  // single tap at offset (0, 0)
  return a;
}

void set_taps3x3(FwdArgs& a) {
  a.ntaps = 9;
  a.dyc = a.dxc = 0;
  for (int r = 0; r < 3; ++r)
    for (int s = 0; s < 3; ++s) {
      a.dyc |= r << (2 * (r * 3 + s));  // offset r-1 encoded as r
      a.dxc |= s << (2 * (r * 3 + s));
    }
}

}  // namespace

// conv3x3 forward: the halo kernel writes one row per (XCD stream, wave), the
// implicit GEMM one per 256 pixels.
extern "C" long cnnitmo_conv3x3_stat_rows(int dtype, int n, int h, int w, int cin, int cout) {
  FwdArgs a = base_args();
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  set_taps3x3(a);
  a.cin = cin; a.N = cout; a.a_ld = cin; a.out_ld = cout; a.M = (long)n * h * w;
  if (dtype == CNNITMO_BF16 && halo_handles(a)) return halo_stat_rows(a);
  if (dtype == CNNITMO_F32 && halo_handles(a, true)) return halo_stat_rows(a, true);
  return cnnitmo_fwd_stat_rows(dtype, a.M, cout);
}

// FwdArgs of cnnitmo_tconv2x2_fwd (dense in / out views) for the planners
static FwdArgs tconv_fwd_args(int n, int h, int w, int cin, int cout, int flags) {
  FwdArgs a = base_args();
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  a.cin = cin; a.N = 4 * cout; a.a_ld = cin; a.out_ld = cout; a.M = (long)n * h * w;
  a.scatter = 1; a.cout = cout; a.flags = flags;
  return a;
}

extern "C" long cnnitmo_tconv2x2_stat_rows(int dtype, int n, int h, int w, int cin, int cout) {
  if (dtype == CNNITMO_BF16 && tconv_stream_handles(0, h, w, cin, cout, false))
    return tconv_stream_rows(0, n, h, w, cin, cout, false);
  {
    FwdArgs t = tconv_fwd_args(n, h, w, cin, cout, CNNITMO_RELU | CNNITMO_STATS);
    if (dtype == CNNITMO_BF16 && tfwd2p_handles(t, true)) return tfwd2p_stat_rows(t);
  }
  if (dtype == CNNITMO_BF16 && tconv_ws_handles(0, cin, cout)) return tconv_ws_rows(cin, cout);
  if (dtype == CNNITMO_F32 && tconv_ws_handles(0, cin, cout, true)) return tconv_ws_rows(cin, cout, true);
  FwdArgs a = base_args();
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  a.cin = cin; a.N = 4 * cout; a.a_ld = cin; a.out_ld = cout; a.M = (long)n * h * w;
  a.scatter = 1; a.cout = cout;
  if (dtype == CNNITMO_BF16 && halo_handles(a)) return halo_stat_rows(a);
  return cnnitmo_fwd_stat_rows(dtype, a.M, 4 * cout);
}

extern "C" int cnnitmo_fwd_stat_rows(int dtype, long m, int ncols) {
  (void)dtype;
  if (fwd2_handles(ncols)) return fwd2_stat_rows(m);
  Cfg c = pick_cfg(ncols);
  return (int)((m + c.bm - 1) / c.bm);
}

extern "C" int cnnitmo_conv3x3_fwd(int dtype, const void* x, int x_ld, int x_off, int n, int h,
                                   int w, int cin, const void* wt, const float* bias, int cout,
                                   void* out, int out_ld, int out_off, int flags,
                                   const float* aff_scale, const float* aff_shift,
                                   float* stat_part, const float* border, void* stream) {
  FwdArgs a = base_args();
  a.a = x; a.a_ld = x_ld; a.a_off = x_off;
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  set_taps3x3(a);
  a.cin = cin; a.b = wt; a.N = cout; a.M = (long)n * h * w;
  a.bias = bias; a.out = out; a.out_ld = out_ld; a.out_off = out_off;
  a.cout = cout; a.flags = flags; a.aff_scale = aff_scale; a.aff_shift = aff_shift;
  a.stats = stat_part;
  a.border = border;
  CNN_REQUIRE(!(flags & CNNITMO_STATS) || stat_part, "conv3x3_fwd: STATS without buffer");
  CNN_REQUIRE(!(flags & CNNITMO_AFFINE) || (aff_scale && aff_shift), "conv3x3_fwd: AFFINE without coefficients");
  return dispatch(dtype, a, stream, "conv3x3_fwd");
}

extern "C" int cnnitmo_conv3x3_fwd_pool(int dtype, const void* x, int x_ld, int x_off, int n, int h, int w,
                                        int cin, const void* wt, const float* bias, int cout, void* out, int out_ld,
                                        int out_off, int flags, const float* aff_scale, const float* aff_shift,
                                        float* stat_part, const float* border, void* pool_out, int pool_ld,
                                        unsigned char* pool_idx, const float* pool_sign, void* stream) {
  FwdArgs a = base_args();
  a.a = x; a.a_ld = x_ld; a.a_off = x_off;
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  set_taps3x3(a);
  a.cin = cin; a.b = wt; a.N = cout; a.M = (long)n * h * w;
  a.bias = bias; a.out = out; a.out_ld = out_ld; a.out_off = out_off;
  a.cout = cout; a.flags = flags; a.aff_scale = aff_scale; a.aff_shift = aff_shift;
  a.stats = stat_part;
  a.border = border;
  a.pool_out = pool_out; a.pool_ld = pool_ld; a.pool_idx = pool_idx; a.pool_sign = pool_sign;
  CNN_REQUIRE(pool_out && pool_idx, "conv3x3_fwd_pool: missing pool buffers");
  CNN_REQUIRE(!(flags & CNNITMO_STATS) || stat_part, "conv3x3_fwd_pool: STATS without buffer");
  CNN_REQUIRE(!(flags & CNNITMO_AFFINE) || (aff_scale && aff_shift), "conv3x3_fwd_pool: AFFINE without coefficients");
  const bool f32 = dtype == CNNITMO_F32;
  if ((dtype != CNNITMO_BF16 && !f32) || !halo_handles(a, f32)) {
    cnnitmo_set_error("conv3x3_fwd_pool: unsupported (halo kernel with an epilogue, even h/w, pool_ld >= cout)");
    return CNNITMO_EUNSUPPORTED;
  }
  return launch_halo(a, (hipStream_t)stream, "conv3x3_fwd_pool", f32);
}

extern "C" int cnnitmo_conv3x3_pool_supported(int dtype, int n, int h, int w, int cin, int cout) {
  FwdArgs a = base_args();
  a.a = (const void*)16; a.a_ld = cin;
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  set_taps3x3(a);
  a.cin = cin; a.N = cout; a.M = (long)n * h * w; a.out_ld = cout; a.cout = cout;
  a.flags = CNNITMO_RELU;
  a.pool_out = (void*)16; a.pool_ld = cout; a.pool_idx = (unsigned char*)16;
  const bool f32 = dtype == CNNITMO_F32;
  if (dtype != CNNITMO_BF16 && !f32) return 0;
  return halo_handles(a, f32) ? 1 : 0;
}

extern "C" int cnnitmo_conv3x3_fwd_head(int dtype, const void* x, int x_ld, int x_off, int n, int h, int w,
                                        int cin, const void* wt, const float* bias, int cout, int flags,
                                        const float* aff_scale, const float* aff_shift, int h_valid,
                                        const float* head_w, const float* head_b, float* yhat, void* stream) {
  FwdArgs a = base_args();
  a.a = x; a.a_ld = x_ld; a.a_off = x_off;
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  set_taps3x3(a);
  a.cin = cin; a.b = wt; a.N = cout; a.M = (long)n * h * w;
  a.bias = bias; a.out_ld = cout; a.cout = cout;
  a.flags = flags; a.aff_scale = aff_scale; a.aff_shift = aff_shift;
  a.head_w = head_w; a.head_b = head_b; a.yhat = yhat; a.head_hv = h_valid;
  CNN_REQUIRE(head_w && head_b && yhat, "conv3x3_fwd_head: missing head buffers");
  CNN_REQUIRE(h_valid > 0 && h_valid <= h, "conv3x3_fwd_head: bad h_valid");
  CNN_REQUIRE((long)n * h_valid * w * 12 < (1L << 31), "conv3x3_fwd_head: yhat too large for 32-bit offsets");
  CNN_REQUIRE(!(flags & CNNITMO_STATS), "conv3x3_fwd_head: the inference forward has no BN sums");
  CNN_REQUIRE(!(flags & CNNITMO_AFFINE) || (aff_scale && aff_shift), "conv3x3_fwd_head: AFFINE without coefficients");
  const bool f32 = dtype == CNNITMO_F32;
  if ((dtype != CNNITMO_BF16 && !f32) || !halo_handles(a, f32)) {
    cnnitmo_set_error("conv3x3_fwd_head: unsupported (halo kernel, 64 output channels)");
    return CNNITMO_EUNSUPPORTED;
  }
  return launch_halo(a, (hipStream_t)stream, "conv3x3_fwd_head", f32);
}

extern "C" int cnnitmo_conv3x3_head_supported(int dtype, int n, int h, int w, int cin, int cout) {
  FwdArgs a = base_args();
  a.a = (const void*)16; a.a_ld = cin;
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  set_taps3x3(a);
  a.cin = cin; a.N = cout; a.M = (long)n * h * w; a.out_ld = cout; a.cout = cout;
  a.flags = CNNITMO_RELU | CNNITMO_AFFINE;
  a.head_w = a.head_b = (const float*)16; a.yhat = (float*)16; a.head_hv = h;
  const bool f32 = dtype == CNNITMO_F32;
  if (dtype != CNNITMO_BF16 && !f32) return 0;
  return halo_handles(a, f32) ? 1 : 0;
}

extern "C" int cnnitmo_conv3x3_fwd_cat(int dtype, const void* x1, int x1_ld, int x1_off, int c1, const void* x2,
                                       int x2_ld, int x2_off, int n, int h, int w, int cin, const void* wt,
                                       const float* bias, int cout, void* out, int out_ld, int out_off, int flags,
                                       const float* aff_scale, const float* aff_shift, float* stat_part,
                                       const float* border, void* stream) {
  FwdArgs a = base_args();
  a.a = x1; a.a_ld = x1_ld; a.a_off = x1_off;
  a.a2 = x2; a.a2_ld = x2_ld; a.a2_off = x2_off; a.cin1 = c1;
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  set_taps3x3(a);
  a.cin = cin; a.b = wt; a.N = cout; a.M = (long)n * h * w;
  a.bias = bias; a.out = out; a.out_ld = out_ld; a.out_off = out_off;
  a.cout = cout; a.flags = flags; a.aff_scale = aff_scale; a.aff_shift = aff_shift;
  a.stats = stat_part;
  a.border = border;
  CNN_REQUIRE(x1 && x2 && c1 > 0 && c1 < cin, "conv3x3_fwd_cat: needs two sources splitting cin");
  CNN_REQUIRE(!(flags & CNNITMO_STATS) || stat_part, "conv3x3_fwd_cat: STATS without buffer");
  CNN_REQUIRE(!(flags & CNNITMO_AFFINE) || (aff_scale && aff_shift), "conv3x3_fwd_cat: AFFINE without coefficients");
  if (dtype != CNNITMO_BF16 || !halo_handles(a)) {
    cnnitmo_set_error("conv3x3_fwd_cat: unsupported (bf16 halo kernel, 32-channel aligned split, with an epilogue)");
    return CNNITMO_EUNSUPPORTED;
  }
  return launch_halo(a, (hipStream_t)stream, "conv3x3_fwd_cat");
}

extern "C" int cnnitmo_conv3x3_fwd_cat_supported(int dtype, int n, int h, int w, int c1, int cin, int cout) {
  if (dtype != CNNITMO_BF16 || c1 <= 0 || c1 >= cin) return 0;
  FwdArgs a = base_args();
  a.a = (const void*)16; a.a_ld = c1;
  a.a2 = (const void*)16; a.a2_ld = cin - c1; a.cin1 = c1;
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  set_taps3x3(a);
  a.cin = cin; a.N = cout; a.M = (long)n * h * w; a.out_ld = cout; a.cout = cout;
  a.flags = CNNITMO_RELU;  // every U-Net conv has the forward epilogue
  return halo_handles(a) ? 1 : 0;
}

// Name of the kernel cnnitmo_conv3x3_fwd (dgrad = 0) or cnnitmo_conv3x3_dgrad
// (dgrad = 1; cin/cout as in the layer) launches for these sizes (for profiles).
extern "C" const char* cnnitmo_conv3x3_kernel_name(int dtype, int n, int h, int w, int cin, int cout,
                                                   int dgrad) {
  FwdArgs a = base_args();
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  set_taps3x3(a);
  a.cin = dgrad ? cout : cin;
  a.N = dgrad ? cin : cout;
  a.a_ld = a.cin; a.out_ld = a.N;
  a.M = (long)n * h * w;
  if (!dgrad) a.flags = CNNITMO_RELU;  // the forward epilogue variant (every U-Net conv has one)
  static thread_local char buf[96];
  if (dtype == CNNITMO_BF16 && halo_handles(a)) return halo_name(a);
  if (dtype == CNNITMO_F32 && halo_handles(a, true)) return halo_name(a, true);  // (no BN sums: inference)
  const char* t = dtype == CNNITMO_BF16 ? "bf16" : "f32";
  if (fwd2_handles(a.N)) {
    const int bn = a.N % 128 == 0 ? 128 : a.N % 64 == 0 ? 64 : a.N % 96 == 0 ? 96 : 32;
    snprintf(buf, sizeof(buf), "igemm_fwd2_kernel<%s,%dx%d>", t, fwd2_bm(a, dtype == CNNITMO_BF16), bn);
  } else {
    const Cfg c = pick_cfg(a.N);
    snprintf(buf, sizeof(buf), "igemm_fwd_kernel<%s,%dx%d>", t, c.bm, c.bn);
  }
  return buf;
}

extern "C" const char* cnnitmo_tconv2x2_kernel_name(int dtype, int n, int h, int w, int cin, int cout,
                                                    int dgrad) {
  if (dtype == CNNITMO_BF16 && tconv_stream_handles(dgrad ? 1 : 0, h, w, cin, cout, false))
    return tconv_stream_name(dgrad ? 1 : 0, h, w, cin, cout, false);
  if (!dgrad && dtype == CNNITMO_BF16 &&
      tfwd2p_handles(tconv_fwd_args(n, h, w, cin, cout, CNNITMO_RELU | CNNITMO_STATS), true))
    return "tconv_fwd2p_kernel<bf16,256x256>";
  if (dtype == CNNITMO_BF16 && tconv_ws_handles(dgrad ? 1 : 0, cin, cout))
    return tconv_ws_name(dgrad ? 1 : 0, cin, cout);
  if (dtype == CNNITMO_F32 && tconv_ws_handles(dgrad ? 1 : 0, cin, cout, true))
    return tconv_ws_name(dgrad ? 1 : 0, cin, cout, true);
  FwdArgs a = base_args();
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  a.cin = dgrad ? cout : cin;
  a.N = dgrad ? cin : 4 * cout;
  a.a_ld = a.cin; a.out_ld = dgrad ? cin : cout; a.cout = cout;
  a.scatter = dgrad ? 0 : 1;
  if (dgrad) {
    a.ntaps = 4; a.scale = 2; a.hs = 2 * h; a.ws = 2 * w;
    a.dyc = a.dxc = 0;
    for (int t = 0; t < 4; ++t) {  // (as cnnitmo_tconv2x2_dgrad)
      a.dyc |= ((t >> 1) + 1) << (2 * t);
      a.dxc |= ((t & 1) + 1) << (2 * t);
    }
  }
  a.M = (long)n * h * w;
  if (dtype == CNNITMO_BF16 && halo_handles(a)) return halo_name(a);
  static thread_local char buf[96];
  const char* t = dtype == CNNITMO_BF16 ? "bf16" : "f32";
  if (fwd2_handles(a.N)) {
    const bool t256 = fwd2_t256(a, dtype == CNNITMO_BF16);
    const int bn = t256 ? 256 : a.N % 128 == 0 ? 128 : a.N % 64 == 0 ? 64 : a.N % 96 == 0 ? 96 : 32;
    const int bm = t256 ? 256 : fwd2_bm(a, dtype == CNNITMO_BF16);
    if (fwd2_pers(a, dtype == CNNITMO_BF16))
      snprintf(buf, sizeof(buf), "igemm_fwd2p_kernel<%s,%dx%d>", t, bm, bn);
    else
      snprintf(buf, sizeof(buf), "igemm_fwd2_kernel<%s,%dx%d>", t, bm, bn);
  } else {
    const Cfg c = pick_cfg(a.N);
    snprintf(buf, sizeof(buf), "igemm_fwd_kernel<%s,%dx%d>", t, c.bm, c.bn);
  }
  return buf;
}

extern "C" int cnnitmo_conv1tap_fwd(int dtype, const void* cols, int k, long m, const void* wt,
                                    const float* bias, int cout, void* out, int out_ld,
                                    int out_off, int flags, const float* aff_scale,
                                    const float* aff_shift, float* stat_part, void* stream) {
  FwdArgs a = base_args();
  a.a = cols; a.a_ld = k; a.a_off = 0;
  a.nimg = 1; a.hs = 1; a.ws = (int)m; a.ho = 1; a.wo = (int)m;
  a.cin = k; a.b = wt; a.N = cout; a.M = m;
  a.bias = bias; a.out = out; a.out_ld = out_ld; a.out_off = out_off;
  a.cout = cout; a.flags = flags; a.aff_scale = aff_scale; a.aff_shift = aff_shift;
  a.stats = stat_part;
  CNN_REQUIRE(m < (1L << 31), "conv1tap_fwd: too many pixels");
  return dispatch(dtype, a, stream, "conv1tap_fwd");
}

extern "C" int cnnitmo_conv3x3_dgrad(int dtype, const void* dz, int n, int h, int w, int cout,
                                     const void* wt_flip, int cin, void* dx, int dx_ld,
                                     int dx_off, void* stream) {
  FwdArgs a = base_args();
  a.a = dz; a.a_ld = cout; a.a_off = 0;
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  set_taps3x3(a);
  a.cin = cout; a.b = wt_flip; a.N = cin; a.M = (long)n * h * w;
  a.out = dx; a.out_ld = dx_ld; a.out_off = dx_off; a.cout = cin;
  return dispatch(dtype, a, stream, "conv3x3_dgrad");
}

namespace {
FwdArgs dgrad_bn_args(int n, int h, int w, int cout, int cin) {
  FwdArgs a = base_args();
  a.a_ld = cout;
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  set_taps3x3(a);
  a.cin = cout; a.N = cin; a.M = (long)n * h * w; a.out_ld = cin; a.cout = cin;
  return a;
}
}  // namespace

// Partial-sum rows cnnitmo_conv3x3_dgrad_bn writes (0: the fused path is not
// available for these sizes / dtype).
extern "C" long cnnitmo_conv3x3_dgrad_bn_rows(int dtype, int n, int h, int w, int cout, int cin, int c0,
                                              int c1) {
  FwdArgs a = dgrad_bn_args(n, h, w, cout, cin);
  a.bnb_c0 = c0; a.bnb_c1 = c1; a.bnb_out = (void*)1; a.bnb_r_ld = 8;
  const bool f32 = dtype == CNNITMO_F32;
  if ((dtype != CNNITMO_BF16 && !f32) || !halo_handles(a, f32)) return 0;
  return halo_stat_rows(a, f32);
}

// Name of the kernel cnnitmo_conv3x3_dgrad_bn launches for these sizes (for profiles).
extern "C" const char* cnnitmo_conv3x3_dgrad_bn_kernel_name(int dtype, int n, int h, int w, int cout, int cin,
                                                            int c0, int c1) {
  FwdArgs a = dgrad_bn_args(n, h, w, cout, cin);
  a.bnb_c0 = c0; a.bnb_c1 = c1; a.bnb_out = (void*)1; a.bnb_r_ld = 8;
  const bool f32 = dtype == CNNITMO_F32;
  if ((dtype != CNNITMO_BF16 && !f32) || !halo_handles(a, f32)) return "";
  return halo_name(a, f32);
}

extern "C" int cnnitmo_conv3x3_dgrad_bn(int dtype, const void* dz, int n, int h, int w, int cout,
                                        const void* wt_flip, int cin, void* dx, int dx_ld, int dx_off,
                                        int c0, int c1, const float* coef, const void* r, int r_ld,
                                        int r_off, void* dz_out, float* part, int parity, void* stream) {
  FwdArgs a = dgrad_bn_args(n, h, w, cout, cin);
  a.a = dz; a.b = wt_flip;
  a.out = dx; a.out_ld = dx ? dx_ld : cin; a.out_off = dx ? dx_off : 0;
  a.bnb_c0 = c0; a.bnb_c1 = c1; a.bnb_par = parity ? 1 : 0;
  a.bnb_coef = coef; a.bnb_r = r; a.bnb_r_ld = r_ld; a.bnb_r_off = r_off; a.bnb_out = dz_out;
  a.stats = part;
  const bool f32 = dtype == CNNITMO_F32;
  CNN_REQUIRE((dtype == CNNITMO_BF16 || f32) && halo_handles(a, f32), "conv3x3_dgrad_bn: unsupported sizes (halo kernel only)");
  CNN_REQUIRE(coef && r && dz_out && part && (dx || (c0 == 0 && c1 == cin)),
              "conv3x3_dgrad_bn: missing buffers");
  return launch_halo(a, (hipStream_t)stream, "conv3x3_dgrad_bn", f32);
}

namespace {
FwdArgs dgrad_bn_pooled_args(int n, int h, int w, int cout, int cin) {
  FwdArgs a = dgrad_bn_args(n, h, w, cout, cin);
  a.bnb_c0 = 0; a.bnb_c1 = cin; a.bnb_out = (void*)1; a.bnb_r_ld = cin;
  a.pool_out = (void*)1; a.pool_ld = cin; a.pool_idx = (unsigned char*)1;
  return a;
}
}  // namespace

// Partial-sum rows cnnitmo_conv3x3_dgrad_bn_pooled writes (0: not available for these sizes).
extern "C" long cnnitmo_conv3x3_dgrad_bn_pooled_rows(int dtype, int n, int h, int w, int cout, int cin) {
  FwdArgs a = dgrad_bn_pooled_args(n, h, w, cout, cin);
  const bool f32 = dtype == CNNITMO_F32;
  if ((dtype != CNNITMO_BF16 && !f32) || !halo_handles(a, f32)) return 0;
  return halo_stat_rows(a, f32);
}

extern "C" const char* cnnitmo_conv3x3_dgrad_bn_pooled_kernel_name(int dtype, int n, int h, int w, int cout,
                                                                   int cin) {
  FwdArgs a = dgrad_bn_pooled_args(n, h, w, cout, cin);
  const bool f32 = dtype == CNNITMO_F32;
  if ((dtype != CNNITMO_BF16 && !f32) || !halo_handles(a, f32)) return "";
  return halo_name(a, f32);
}

extern "C" int cnnitmo_conv3x3_dgrad_bn_pooled(int dtype, const void* dz, int n, int h, int w, int cout,
                                               const void* wt_flip, int cin, const float* coef, const void* r,
                                               int r_ld, int r_off, const void* dy_pool, const unsigned char* idx,
                                               void* dz_out, float* part, void* stream) {
  FwdArgs a = dgrad_bn_pooled_args(n, h, w, cout, cin);
  a.a = dz; a.b = wt_flip;
  a.out = dz_out; a.out_ld = cin; a.out_off = 0;
  a.bnb_coef = coef; a.bnb_r = r; a.bnb_r_ld = r_ld; a.bnb_r_off = r_off; a.bnb_out = dz_out;
  a.pool_out = const_cast<void*>(dy_pool); a.pool_idx = const_cast<unsigned char*>(idx);
  a.stats = part;
  const bool f32 = dtype == CNNITMO_F32;
  CNN_REQUIRE((dtype == CNNITMO_BF16 || f32) && halo_handles(a, f32),
              "conv3x3_dgrad_bn_pooled: unsupported sizes (halo kernel, even h and w)");
  CNN_REQUIRE(coef && r && dy_pool && idx && dz_out && part, "conv3x3_dgrad_bn_pooled: missing buffers");
  return launch_halo(a, (hipStream_t)stream, "conv3x3_dgrad_bn_pooled", f32);
}

extern "C" int cnnitmo_tconv2x2_fwd(int dtype, const void* x, int n, int h, int w, int cin,
                                    const void* k, const float* bias, int cout, void* out,
                                    int out_ld, int out_off, int flags, const float* aff_scale,
                                    const float* aff_shift, float* stat_part, void* stream) {
  FwdArgs a = base_args();
  a.a = x; a.a_ld = cin; a.a_off = 0;
  a.nimg = n; a.hs = h; a.ws = w; a.ho = h; a.wo = w;
  a.cin = cin; a.b = k; a.N = 4 * cout; a.M = (long)n * h * w;
  a.bias = bias; a.out = out; a.out_ld = out_ld; a.out_off = out_off;
  a.scatter = 1; a.cout = cout; a.flags = flags;
  a.aff_scale = aff_scale; a.aff_shift = aff_shift; a.stats = stat_part;
  CNN_REQUIRE(!(flags & CNNITMO_STATS) || stat_part, "tconv2x2_fwd: STATS without buffer");
  if (dtype == CNNITMO_BF16 && tconv_stream_handles(0, h, w, cin, cout, false))
    return launch_tconv_stream(0, x, cin, 0, k, n, h, w, cin, cout, out, out_ld, out_off, bias, flags, aff_scale,
                               aff_shift, stat_part, nullptr, nullptr, 0, 0, (hipStream_t)stream, "tconv2x2_fwd");
  if (dtype == CNNITMO_BF16 && tfwd2p_handles(a, true)) return launch_tfwd2p(a, (hipStream_t)stream, "tconv2x2_fwd");
  if (dtype == CNNITMO_BF16 && tconv_ws_handles(0, cin, cout))
    return launch_tconv_ws(0, x, cin, 0, k, n, h, w, cin, cout, out, out_ld, out_off, bias, flags, aff_scale,
                           aff_shift, stat_part, (hipStream_t)stream, "tconv2x2_fwd");
  if (dtype == CNNITMO_F32 && tconv_ws_handles(0, cin, cout, true))
    return launch_tconv_ws(0, x, cin, 0, k, n, h, w, cin, cout, out, out_ld, out_off, bias, flags, aff_scale,
                           aff_shift, stat_part, (hipStream_t)stream, "tconv2x2_fwd", true);
  return dispatch(dtype, a, stream, "tconv2x2_fwd");
}

extern "C" int cnnitmo_tconv2x2_dgrad(int dtype, const void* dout, int n, int h, int w, int cout,
                                      const void* kT, int cin, void* dx, void* stream) {
  FwdArgs a = base_args();
  a.a = dout; a.a_ld = cout; a.a_off = 0;
  a.nimg = n; a.hs = 2 * h; a.ws = 2 * w; a.ho = h; a.wo = w; a.scale = 2;
  a.ntaps = 4;
  a.dyc = a.dxc = 0;
  for (int t = 0; t < 4; ++t) {  // tap t = (a, b): offset (a, b) on the 2x grid
    a.dyc |= ((t >> 1) + 1) << (2 * t);
    a.dxc |= ((t & 1) + 1) << (2 * t);
  }
  a.cin = cout; a.b = kT; a.N = cin; a.M = (long)n * h * w;
  a.out = dx; a.out_ld = cin; a.out_off = 0; a.cout = cin;
  if (dtype == CNNITMO_BF16 && tconv_stream_handles(1, h, w, cin, cout, false))
    return launch_tconv_stream(1, dout, cout, 0, kT, n, h, w, cin, cout, dx, cin, 0, nullptr, 0, nullptr, nullptr,
                               nullptr, nullptr, nullptr, 0, 0, (hipStream_t)stream, "tconv2x2_dgrad");
  if (dtype == CNNITMO_BF16 && tconv_ws_handles(1, cin, cout))
    return launch_tconv_ws(1, dout, cout, 0, kT, n, h, w, cin, cout, dx, cin, 0, nullptr, 0, nullptr, nullptr,
                           nullptr, (hipStream_t)stream, "tconv2x2_dgrad");
  if (dtype == CNNITMO_F32 && tconv_ws_handles(1, cin, cout, true))
    return launch_tconv_ws(1, dout, cout, 0, kT, n, h, w, cin, cout, dx, cin, 0, nullptr, 0, nullptr, nullptr,
                           nullptr, (hipStream_t)stream, "tconv2x2_dgrad", true);
  return dispatch(dtype, a, stream, "tconv2x2_dgrad");
}

extern "C" long cnnitmo_tconv2x2_dgrad_bn_rows(int dtype, int n, int h, int w, int cout, int cin) {
  if (dtype != CNNITMO_BF16 || !tconv_stream_handles(1, h, w, cin, cout, true)) return 0;
  return tconv_stream_rows(1, n, h, w, cin, cout, true);
}

// Name of the kernel cnnitmo_tconv2x2_dgrad_bn launches for these sizes (for profiles).
extern "C" const char* cnnitmo_tconv2x2_dgrad_bn_kernel_name(int dtype, int n, int h, int w, int cout, int cin) {
  (void)n;
  if (dtype != CNNITMO_BF16 || !tconv_stream_handles(1, h, w, cin, cout, true)) return "";
  return tconv_stream_name(1, h, w, cin, cout, true);
}

extern "C" int cnnitmo_tconv2x2_dgrad_bn(int dtype, const void* dout, int n, int h, int w, int cout,
                                         const void* kT, int cin, const float* coef, const void* r, int r_ld,
                                         int r_off, void* dz_out, float* part, void* stream) {
  CNN_REQUIRE(dtype == CNNITMO_BF16 && tconv_stream_handles(1, h, w, cin, cout, true),
              "tconv2x2_dgrad_bn: unsupported sizes (bf16 stream kernel only)");
  CNN_REQUIRE(coef && r && dz_out && part, "tconv2x2_dgrad_bn: missing buffers");
  return launch_tconv_stream(1, dout, cout, 0, kT, n, h, w, cin, cout, dz_out, cin, 0, nullptr, 0, nullptr,
                             nullptr, part, coef, r, r_ld, r_off, (hipStream_t)stream, "tconv2x2_dgrad_bn");
}
