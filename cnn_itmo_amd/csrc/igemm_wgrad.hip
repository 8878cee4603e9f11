#include <cstdio>
// Implicit-GEMM weight gradients on MFMA (K = pixels).
//
//   conv3x3 wgrad  (TF Conv2DBackpropFilter for model.py:196):
//       dW[co][t][ci] = sum_p dz[p][co] * x[p + off_t][ci]
//   tconv2x2 wgrad (for model.py:200):
//       dK[t][co][ci] = sum_{(i,j)} dout[(2i+a, 2j+b)][co] * x[(i,j)][ci]
//
// GEMM view per tap: C[m][n] = sum_p A[srcA(p)][m] * B[srcB(p)][n] with
// m = gradient channel, n = input channel, p over an iteration pixel grid.
// The pixel reduction (up to 66.8 M at 1080p batch 32) is split into slabs
// ("split-K"); every block writes its own fp32 slab and cnnitmo's reduce
// kernel sums them in a fixed order, so results are bitwise reproducible.
// NHWC tiles are staged [pixel][channel] in LDS; MFMA operands need K (pixels)
// contiguous per lane, so bf16 fragments are read with ds_read_b64_tr_b16
// (4 pixel rows x 16 channels -> column-major) and f32 fragments with
// ds_read_b32 (v_mfma_f32_16x16x4_f32 takes one element per lane).
#include <algorithm>
#include <cstring>

#include <cstdlib>

#include "igemm_common.h"

struct WgradArgs {
  const void* a;
  long a_ld;
  int a_off, ha, wa, a_scale;
  const void* b;
  long b_ld;
  int b_off, hb, wb, b_scale;
  int nimg, hg, wg;  // iteration grid
  int ntaps;
  int ayc, axc, byc, bxc;  // per-tap offsets, 2-bit fields: ((code >> 2t) & 3) - 1
  int M, N;
  float* out;
  long split_stride, tap_stride;
  int out_ld;
  int mblocks, nblocks, splits;
  long P, pix_per_split;
};

// ---- LDS images ------------------------------------------------------------
// bf16: [BP=32 rows][R cols] with 32-byte column blocks XOR-swizzled by row so
// that the 8 rows a 32-lane half reads in one ds_read_b64_tr_b16 land in 8
// distinct 32-byte bank slots ("wgrad LDS image").
template <int R> __device__ __forceinline__ int trswz(int row) {
  if constexpr (R == 32) return (row >> 3) & 1;
  if constexpr (R == 64) return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  return (row & 3) | (((row >> 3) & 1) << 2);  // R == 128
}
template <int R> __device__ __forceinline__ int bf_off(int row, int col) {
  return row * (R * 2) + ((((col >> 4) ^ trswz<R>(row))) << 5) + ((col & 15) << 1);
}
// f32: [BP=16 rows][R cols] with 64-byte blocks XOR-swizzled by row parity so
// the two rows a 32-lane half reads with ds_read_b32 use disjoint banks.
template <int R> __device__ __forceinline__ int f_off(int row, int col) {
  return row * (R * 4) + ((((col >> 4) ^ (row & 1))) << 6) + ((col & 15) << 2);
}

template <typename T> struct WT;
template <> struct WT<bf16> { static constexpr int BP = 32; };
template <> struct WT<float> { static constexpr int BP = 16; };

template <typename T, int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(256) void igemm_wgrad_kernel(const WgradArgs p) {
  constexpr int BP = WT<T>::BP;
  constexpr int VE = Vec16<T>::N;
  constexpr int TM = BM / WM, TN = BN / WN;
  constexpr int FM = TM / 16, FN = TN / 16;
  constexpr int SEGA = BM / VE, SEGB = BN / VE;  // 16-byte segments per pixel row
  constexpr int A_SEGS = BP * SEGA, B_SEGS = BP * SEGB;
  constexpr int SA = (A_SEGS + 255) / 256, SB = (B_SEGS + 255) / 256;
  constexpr int A_BYTES = BP * BM * (int)sizeof(T), B_BYTES = BP * BN * (int)sizeof(T);
  constexpr int STAGE = A_BYTES + B_BYTES;
  static_assert(WM * WN == 4, "4 waves");
  __shared__ __attribute__((aligned(16))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles = p.mblocks * p.nblocks;
  const int total = tiles * p.ntaps * p.splits;
  int lid = xcd_remap(blockIdx.x, total);
  const int split = lid / (tiles * p.ntaps);
  lid -= split * tiles * p.ntaps;
  const int tap = lid / tiles;
  lid -= tap * tiles;
  const int mb = lid / p.nblocks, nb = lid - mb * p.nblocks;
  const int m0 = mb * BM, n0 = nb * BN;
  const int ady = ((p.ayc >> (2 * tap)) & 3) - 1, adx = ((p.axc >> (2 * tap)) & 3) - 1;
  const int bdy = ((p.byc >> (2 * tap)) & 3) - 1, bdx = ((p.bxc >> (2 * tap)) & 3) - 1;

  const long pbeg = (long)split * p.pix_per_split;
  const long pend = min(p.P, pbeg + p.pix_per_split);
  const int nk = (int)((pend - pbeg + BP - 1) / BP);

  const T* __restrict__ A = (const T*)p.a;
  const T* __restrict__ B = (const T*)p.b;

  // Per-thread staging rows: pixel coordinates advanced incrementally by BP.
  int ai_img[SA], ai_h[SA], ai_w[SA];
  int bi_img[SB], bi_h[SB], bi_w[SB];
  long a_pix[SA], b_pix[SB];
  const long hw = (long)p.hg * p.wg;
  auto decode = [&](long pix, int& img, int& h, int& w) {
    img = (int)(pix / hw);
    const int rem = (int)(pix - (long)img * hw);
    h = rem / p.wg;
    w = rem - h * p.wg;
  };
#pragma unroll
  for (int j = 0; j < SA; ++j) {
    a_pix[j] = pbeg + (tid + j * 256) / SEGA;
    decode(a_pix[j], ai_img[j], ai_h[j], ai_w[j]);
  }
#pragma unroll
  for (int j = 0; j < SB; ++j) {
    b_pix[j] = pbeg + (tid + j * 256) / SEGB;
    decode(b_pix[j], bi_img[j], bi_h[j], bi_w[j]);
  }
  auto advance = [&](int& img, int& h, int& w) {
    w += BP;
    while (w >= p.wg) {
      w -= p.wg;
      if (++h == p.hg) { h = 0; ++img; }
    }
  };

  uint4 ra[SA], rb[SB];
  auto load = [&]() {
#pragma unroll
    for (int j = 0; j < SA; ++j) {
      const int seg = tid + j * 256;
      uint4 v = make_uint4(0, 0, 0, 0);
      const int hh = ai_h[j] * p.a_scale + ady, ww = ai_w[j] * p.a_scale + adx;
      if (seg < A_SEGS && a_pix[j] < pend && hh >= 0 && hh < p.ha && ww >= 0 && ww < p.wa) {
        const size_t off = ((size_t)((long)ai_img[j] * p.ha + hh) * p.wa + ww) * p.a_ld + p.a_off +
                           m0 + (seg % SEGA) * VE;
        v = *reinterpret_cast<const uint4*>(A + off);
      }
      ra[j] = v;
    }
#pragma unroll
    for (int j = 0; j < SB; ++j) {
      const int seg = tid + j * 256;
      uint4 v = make_uint4(0, 0, 0, 0);
      const int hh = bi_h[j] * p.b_scale + bdy, ww = bi_w[j] * p.b_scale + bdx;
      if (seg < B_SEGS && b_pix[j] < pend && hh >= 0 && hh < p.hb && ww >= 0 && ww < p.wb) {
        const size_t off = ((size_t)((long)bi_img[j] * p.hb + hh) * p.wb + ww) * p.b_ld + p.b_off +
                           n0 + (seg % SEGB) * VE;
        v = *reinterpret_cast<const uint4*>(B + off);
      }
      rb[j] = v;
    }
#pragma unroll
    for (int j = 0; j < SA; ++j) {
      a_pix[j] += BP;
      advance(ai_img[j], ai_h[j], ai_w[j]);
    }
#pragma unroll
    for (int j = 0; j < SB; ++j) {
      b_pix[j] += BP;
      advance(bi_img[j], bi_h[j], bi_w[j]);
    }
  };
  auto store = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + A_BYTES;
#pragma unroll
    for (int j = 0; j < SA; ++j) {
      const int seg = tid + j * 256;
      if (seg < A_SEGS) {
        const int row = seg / SEGA, col = (seg % SEGA) * VE;
        const int off = std::is_same<T, bf16>::value ? bf_off<BM>(row, col) : f_off<BM>(row, col);
        *reinterpret_cast<uint4*>(As + off) = ra[j];
      }
    }
#pragma unroll
    for (int j = 0; j < SB; ++j) {
      const int seg = tid + j * 256;
      if (seg < B_SEGS) {
        const int row = seg / SEGB, col = (seg % SEGB) * VE;
        const int off = std::is_same<T, bf16>::value ? bf_off<BN>(row, col) : f_off<BN>(row, col);
        *reinterpret_cast<uint4*>(Bs + off) = rb[j];
      }
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  if (nk > 0) {
    load();
    store(0);
  }
  __syncthreads();
  int cur = 0;
  const int g = lane >> 4, li = lane & 15;
  for (int ks = 0; ks < nk; ++ks) {
    const bool more = ks + 1 < nk;
    if (more) load();
    const char* As = smem + cur * STAGE;
    const char* Bs = As + A_BYTES;
    if constexpr (std::is_same<T, bf16>::value) {
      const int q = li >> 2, pp = li & 3;
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int col = wm * TM + i * 16 + 4 * pp;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4, As + bf_off<BM>(8 * g + q, col)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4, As + bf_off<BM>(8 * g + 4 + q, col)));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * TN + j * 16 + 4 * pp;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4, Bs + bf_off<BN>(8 * g + q, col)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(
            LDS_PTR(s16x4, Bs + bf_off<BN>(8 * g + 4 + q, col)));
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int row = 4 * e + g;
        float af[FM], bfr[FN];
#pragma unroll
        for (int i = 0; i < FM; ++i)
          af[i] = *reinterpret_cast<const float*>(As + f_off<BM>(row, wm * TM + i * 16 + li));
#pragma unroll
        for (int j = 0; j < FN; ++j)
          bfr[j] = *reinterpret_cast<const float*>(Bs + f_off<BN>(row, wn * TN + j * 16 + li));
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    if (more) store(cur ^ 1);
    __syncthreads();
    cur ^= 1;
  }

  float* __restrict__ O = p.out + (size_t)split * p.split_stride + (size_t)tap * p.tap_stride;
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int m = m0 + wm * TM + i * 16 + g * 4 + r;
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int n = n0 + wn * TN + j * 16 + li;
        O[(size_t)m * p.out_ld + n] = acc[i][j][r];
      }
    }
}

// Folded input BN (the GEMM ran on r, the layer's true input is y = r*s + h,
// zero outside the image): dW[row][col] = s[ci]*raw + h[ci]*V(row, col) where
// V is the sum of the output gradient over the pixels whose tap hits the image.
//  conv  (mode 1, row = co, col = t*cin + ci):  V = db[co] - oob(co, t), oob
//        from the border sums bs[8][cout] = {top, bot, left, right, 4 corners}.
//  tconv (mode 2, row = tap*cout + co, col = ci): V = par[row] (parity sums).
struct WFold {
  int mode;  // 0 none, 1 conv3x3, 2 tconv2x2
  int cin, cout;
  const float* s;
  const float* h;
  const float* db;  // mode 1: [cout]
  const float* v;   // mode 1: border sums [8][cout]; mode 2: parity sums [4*cout]
  float* raw;       // optional: the uncorrected sum (gradient w.r.t. the folded weights' r-GEMM)
};

__device__ __forceinline__ float fold_v(const WFold& f, int row, int col) {
  if (f.mode == 2) return f.v[row];
  const int t = col / f.cin, r = t / 3, q = t - 3 * r;
  const float* b = f.v;
  const int C = f.cout, co = row;
  float o = 0.f;
  if (r == 0) o += b[0 * C + co];
  if (r == 2) o += b[1 * C + co];
  if (q == 0) o += b[2 * C + co];
  if (q == 2) o += b[3 * C + co];
  if (r == 0 && q == 0) o -= b[4 * C + co];
  if (r == 0 && q == 2) o -= b[5 * C + co];
  if (r == 2 && q == 0) o -= b[6 * C + co];
  if (r == 2 && q == 2) o -= b[7 * C + co];
  return f.db[co] - o;
}

// Sum the split slabs: out[row*cols_out + c] = sum_s ws[s][row*cols_in + c]
// (then the folded-BN correction when f.mode != 0).  A workgroup owns E consecutive
// outputs; its S wave groups sum contiguous slab ranges (four loads in flight per
// lane), and group 0 adds the S partials in order: the same fixed order on every run.
// (One thread per output summing every slab in sequence was latency-bound: 0.1-0.4 ms
// per launch at 36-500 slabs, 1.5 ms per step.)
template <int E, int S>
__global__ __launch_bounds__(E * S) void slab_reduce_kernel(const float* __restrict__ ws, long slab, int splits,
                                                            int rows, int cols_in, int cols_out,
                                                            float* __restrict__ out, WFold f) {
  __shared__ float part[S][E];
  const int e = threadIdx.x % E, g = threadIdx.x / E;
  const long total = (long)rows * cols_out;
  const long i = (long)blockIdx.x * E + e;
  const bool ok = i < total;
  const int row = ok ? (int)(i / cols_out) : 0, c = ok ? (int)(i - (long)row * cols_out) : 0;
  const long src = (long)row * cols_in + c;
  const int per = (splits + S - 1) / S, k0 = g * per, k1 = min(k0 + per, splits);
  float s = 0.f;
  if (ok) {
    int k = k0;
    for (; k + 4 <= k1; k += 4) {
      const float a0 = ws[(size_t)k * slab + src], a1 = ws[(size_t)(k + 1) * slab + src];
      const float a2 = ws[(size_t)(k + 2) * slab + src], a3 = ws[(size_t)(k + 3) * slab + src];
      s += a0;
      s += a1;
      s += a2;
      s += a3;
    }
    for (; k < k1; ++k) s += ws[(size_t)k * slab + src];
  }
  if constexpr (S > 1) {
    part[g][e] = s;
    __syncthreads();
    if (g == 0) {
#pragma unroll
      for (int q = 1; q < S; ++q) s += part[q][e];
    }
  }
  if (g == 0 && ok) {
    if (f.raw) f.raw[i] = s;
    if (f.mode) {
      const int ci = c % f.cin;
      s = s * f.s[ci] + f.h[ci] * fold_v(f, row, c);
    }
    out[i] = s;
  }
}

// launch of slab_reduce_kernel over rows x cols_out outputs: more slab groups per
// output when there are many slabs and few outputs
static void slab_reduce(const float* ws, long slab, int splits, int rows, int cols_in, int cols_out, float* out,
                        const WFold& f, hipStream_t s) {
  const long total = (long)rows * cols_out;
#define SRL(E, S)                                                                                              \
  hipLaunchKernelGGL((slab_reduce_kernel<E, S>), dim3((unsigned)((total + E - 1) / E)), dim3(E * S), 0, s, ws, \
                     slab, splits, rows, cols_in, cols_out, out, f)
  if (splits >= 64) SRL(64, 16);
  else if (splits >= 8) SRL(64, 4);
  else SRL(256, 1);
#undef SRL
}

// ----------------------------------------------------------------------------
namespace {

int pick_tile(int x) { return x % 128 == 0 ? 128 : (x % 64 == 0 ? 64 : 32); }

struct Plan {
  int bm, bn, mblocks, nblocks, splits;
  long pps;
};

template <typename T>
Plan make_plan(long P, int M, int N, int ntaps) {
  Plan pl;
  pl.bm = pick_tile(M);
  pl.bn = pick_tile(N);
  pl.mblocks = M / pl.bm;
  pl.nblocks = N / pl.bn;
  const long tiles = (long)pl.mblocks * pl.nblocks * ntaps;
  constexpr int BP = WT<T>::BP;
  const long ksteps = (P + BP - 1) / BP;
  long splits = (2048 + tiles - 1) / tiles;
  splits = std::min(splits, std::max(1L, ksteps / 8));  // >= 8 K-steps per slab
  // keep the slab workspace <= 512 MiB
  const long slab_bytes = (long)M * N * ntaps * 4;
  splits = std::max(1L, std::min(splits, (512L << 20) / slab_bytes));
  const long steps_per = (ksteps + splits - 1) / splits;
  pl.pps = steps_per * BP;
  pl.splits = (int)((P + pl.pps - 1) / pl.pps);
  return pl;
}

template <typename T, int BM, int BN>
void launch_cfg(const WgradArgs& a, hipStream_t s, dim3 grid) {
  constexpr int WM = (BM >= BN) ? ((BM == 4 * BN) ? 4 : 2) : ((BN == 4 * BM) ? 1 : 2);
  constexpr int WN = 4 / WM;
  hipLaunchKernelGGL((igemm_wgrad_kernel<T, BM, BN, WM, WN>), grid, dim3(256), 0, s, a);
}

template <typename T>
void launch_any(const WgradArgs& a, int bm, int bn, hipStream_t s, dim3 grid) {
#define CNN_W(BMv, BNv) \
  if (bm == BMv && bn == BNv) return launch_cfg<T, BMv, BNv>(a, s, grid);
  CNN_W(128, 128) CNN_W(128, 64) CNN_W(128, 32)
  CNN_W(64, 128) CNN_W(64, 64) CNN_W(64, 32)
  CNN_W(32, 128) CNN_W(32, 64) CNN_W(32, 32)
#undef CNN_W
}

// bf16: the v2 kernel (igemm_wgrad2.hip); returns splits written, < 0 if not taken.
int try_wgrad2(const WgradArgs& a, int tapdep, void* ws, size_t ws_bytes, hipStream_t s) {
  Wgrad2Args b;
  memset(&b, 0, sizeof(b));
  b.a = (const bf16*)a.a; b.a_ld = a.a_ld; b.a_off = a.a_off; b.ha = a.ha; b.wa = a.wa; b.a_scale = a.a_scale;
  b.b = (const bf16*)a.b; b.b_ld = a.b_ld; b.b_off = a.b_off; b.hb = a.hb; b.wb = a.wb; b.b_scale = a.b_scale;
  b.nimg = a.nimg; b.hg = a.hg; b.wg = a.wg; b.ntaps = a.ntaps;
  b.ayc = a.ayc; b.axc = a.axc; b.byc = a.byc; b.bxc = a.bxc; b.a_tapdep = tapdep;
  b.M = a.M; b.N = a.N; b.tap_stride = a.tap_stride; b.out_ld = a.out_ld;
  return launch_wgrad2(b, ws, ws_bytes, s);
}

template <typename T>
int run_wgrad(WgradArgs a, float* out_final, int rows, int cols_in, int cols_out, void* ws,
              size_t ws_bytes, hipStream_t s, const char* what, const WFold& fold, int tapdep = 0) {
  CNN_REQUIRE(a.M % 32 == 0 && a.N % 32 == 0, "%s: channel counts %d/%d must be multiples of 32",
              what, a.M, a.N);
  CNN_REQUIRE(a.a_ld % Vec16<T>::N == 0 && a.b_ld % Vec16<T>::N == 0 && a.b_off % Vec16<T>::N == 0,
              "%s: views must be 16-byte aligned", what);
  a.P = (long)a.nimg * a.hg * a.wg;
  CNN_REQUIRE(a.P > 0, "%s: empty", what);
  const long slab = (long)a.M * a.N * a.ntaps;
  if constexpr (std::is_same<T, bf16>::value) {
    const int splits = try_wgrad2(a, tapdep, ws, ws_bytes, s);
    if (splits > 0) {
      int rc = cnnitmo_check_launch(what);
      if (rc) return rc;
      slab_reduce((const float*)ws, slab, splits, rows, cols_in, cols_out, out_final, fold, s);
      return cnnitmo_check_launch(what);
    }
  }
  Plan pl = make_plan<T>(a.P, a.M, a.N, a.ntaps);
  CNN_REQUIRE(ws && ws_bytes >= (size_t)pl.splits * slab * 4, "%s: workspace too small (%zu < %zu)",
              what, ws_bytes, (size_t)pl.splits * slab * 4);
  a.out = (float*)ws;
  a.split_stride = slab;
  a.mblocks = pl.mblocks;
  a.nblocks = pl.nblocks;
  a.splits = pl.splits;
  a.pix_per_split = pl.pps;
  const long total = (long)pl.mblocks * pl.nblocks * a.ntaps * pl.splits;
  launch_any<T>(a, pl.bm, pl.bn, s, dim3((unsigned)total));
  int rc = cnnitmo_check_launch(what);
  if (rc) return rc;
  slab_reduce((const float*)ws, slab, pl.splits, rows, cols_in, cols_out, out_final, fold, s);
  return cnnitmo_check_launch(what);
}

template <typename T>
size_t ws_bytes_for(long P, int M, int N, int ntaps) {
  Plan pl = make_plan<T>(P, M, N, ntaps);
  size_t b = (size_t)pl.splits * M * N * ntaps * 4;
  if (std::is_same<T, bf16>::value) b = std::max(b, wgrad2_ws_bytes(P, M, N, ntaps));
  return b;
}

}  // namespace

extern "C" size_t cnnitmo_wgrad_workspace_bytes(int dtype, int n, int h, int w, int cin, int cout,
                                                int ntaps) {
  const long P = (long)n * h * w;
  if (dtype == CNNITMO_BF16) {
    size_t b = ws_bytes_for<bf16>(P, cout, cin, ntaps);
    if (ntaps == 9) b = std::max(b, wgrad_halo_ws_bytes(n, h, w, cin, cout));
    return b;
  }
  size_t b = ws_bytes_for<float>(P, cout, cin, ntaps);
  if (ntaps == 9) b = std::max(b, wgrad_halo_f32_ws_bytes(n, h, w, cin, cout));
  return b;
}

extern "C" size_t cnnitmo_tconv2x2_wgrad_workspace_bytes(int dtype, int n, int h, int w, int cin,
                                                         int cout) {
  const long P = (long)n * h * w;
  return dtype == CNNITMO_BF16 ? std::max(ws_bytes_for<bf16>(P, cout, cin, 4), wgrad_tconv_ws_bytes(n, h, w, cin, cout))
                               : std::max(ws_bytes_for<float>(P, cout, cin, 4), wgrad_tconv_f32_ws_bytes(n, h, w, cin, cout));
}

extern "C" int cnnitmo_conv_wgrad(int dtype, int ntaps, const void* x, int x_ld, int x_off,
                                  const void* dz, int n, int h, int w, int cin, int cout,
                                  float* dw, int dw_cols, const float* fold_scale,
                                  const float* fold_shift, const float* fold_db,
                                  const float* fold_border, float* raw_out, void* workspace,
                                  size_t ws_bytes, void* stream) {
  CNN_REQUIRE(ntaps == 9 || ntaps == 1, "conv_wgrad: ntaps must be 9 or 1");
  WFold f{0, cin, cout, fold_scale, fold_shift, fold_db, fold_border, raw_out};
  if (fold_scale) {
    CNN_REQUIRE(ntaps == 9 && fold_shift && fold_db && fold_border && (dw_cols <= 0 || dw_cols == 9 * cin),
                "conv_wgrad: folded BN needs ntaps 9, shift, db and border sums");
    f.mode = 1;
  }
  WgradArgs a;
  memset(&a, 0, sizeof(a));
  a.a = dz; a.a_ld = cout; a.a_off = 0; a.ha = h; a.wa = w; a.a_scale = 1;
  a.b = x; a.b_ld = x_ld; a.b_off = x_off; a.hb = h; a.wb = w; a.b_scale = 1;
  a.nimg = n; a.hg = h; a.wg = w;
  a.ntaps = ntaps;
  for (int t = 0; t < ntaps; ++t) {
    const int r = ntaps == 9 ? t / 3 : 1, s = ntaps == 9 ? t % 3 : 1;
    a.ayc |= 1 << (2 * t);
    a.axc |= 1 << (2 * t);
    a.byc |= r << (2 * t);
    a.bxc |= s << (2 * t);
  }
  a.M = cout; a.N = cin;
  a.tap_stride = cin; a.out_ld = ntaps * cin;
  const int cols_out = dw_cols > 0 ? dw_cols : ntaps * cin;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == CNNITMO_BF16 && ntaps == 9) {
    const int splits = launch_wgrad_halo((const bf16*)x, x_ld, x_off, (const bf16*)dz, n, h, w, cin, cout,
                                         (float*)workspace, ws_bytes, s);
    if (splits > 0) {
      int rc = cnnitmo_check_launch("conv_wgrad");
      if (rc) return rc;
      const long slab = (long)cout * 9 * cin;
      slab_reduce((const float*)workspace, slab, splits, cout, 9 * cin, cols_out, dw, f, s);
      return cnnitmo_check_launch("conv_wgrad");
    }
  }
  if (dtype == CNNITMO_F32 && ntaps == 9) {
    const int splits = launch_wgrad_halo_f32((const float*)x, x_ld, x_off, (const float*)dz, n, h, w, cin, cout,
                                             (float*)workspace, ws_bytes, s);
    if (splits > 0) {
      int rc = cnnitmo_check_launch("conv_wgrad");
      if (rc) return rc;
      const long slab = (long)cout * 9 * cin;
      slab_reduce((const float*)workspace, slab, splits, cout, 9 * cin, cols_out, dw, f, s);
      return cnnitmo_check_launch("conv_wgrad");
    }
  }
  if (dtype == CNNITMO_BF16)
    return run_wgrad<bf16>(a, dw, cout, ntaps * cin, cols_out, workspace, ws_bytes, s, "conv_wgrad", f);
  if (dtype == CNNITMO_F32)
    return run_wgrad<float>(a, dw, cout, ntaps * cin, cols_out, workspace, ws_bytes, s, "conv_wgrad", f);
  cnnitmo_set_error("conv_wgrad: unsupported dtype %d", dtype);
  return CNNITMO_EUNSUPPORTED;
}

extern "C" size_t cnnitmo_wgrad_cat_workspace_bytes(int n, int h, int w, int c1, int cin, int cout) {
  return c1 == 32 ? wgrad_halo_ws_bytes(n, h, w, cin, cout, true) : 0;
}

extern "C" int cnnitmo_conv_wgrad_cat(int dtype, const void* x1, int x1_ld, int x1_off, int c1, const void* x2,
                                      int x2_ld, int x2_off, const void* dz, int n, int h, int w, int cin, int cout,
                                      float* dw, const float* fold_scale, const float* fold_shift,
                                      const float* fold_db, const float* fold_border, float* raw_out,
                                      void* workspace, size_t ws_bytes, void* stream) {
  CNN_REQUIRE(dtype == CNNITMO_BF16 && c1 == 32 && x1 && x2,
              "conv_wgrad_cat: bf16 with a 32-channel first source only");
  WFold f{0, cin, cout, fold_scale, fold_shift, fold_db, fold_border, raw_out};
  if (fold_scale) {
    CNN_REQUIRE(fold_shift && fold_db && fold_border, "conv_wgrad_cat: folded BN needs shift, db and border sums");
    f.mode = 1;
  }
  hipStream_t s = (hipStream_t)stream;
  const int splits = launch_wgrad_halo((const bf16*)x1, x1_ld, x1_off, (const bf16*)dz, n, h, w, cin, cout,
                                       (float*)workspace, ws_bytes, s, (const bf16*)x2, x2_ld, x2_off);
  CNN_REQUIRE(splits > 0, "conv_wgrad_cat: unsupported sizes (%dx%d, %d+%d -> %d) or workspace too small", h, w,
              c1, cin - c1, cout);
  int rc = cnnitmo_check_launch("conv_wgrad_cat");
  if (rc) return rc;
  const long slab = (long)cout * 9 * cin;
  slab_reduce((const float*)workspace, slab, splits, cout, 9 * cin, 9 * cin, dw, f, s);
  return cnnitmo_check_launch("conv_wgrad_cat");
}

extern "C" int cnnitmo_tconv2x2_wgrad(int dtype, const void* x, const void* dout, int n, int h,
                                      int w, int cin, int cout, float* dk, const float* fold_scale,
                                      const float* fold_shift, const float* fold_par, float* raw_out,
                                      void* workspace, size_t ws_bytes, void* stream) {
  WFold f{0, cin, cout, fold_scale, fold_shift, nullptr, fold_par, raw_out};
  if (fold_scale) {
    CNN_REQUIRE(fold_shift && fold_par, "tconv2x2_wgrad: folded BN needs shift and parity sums");
    f.mode = 2;
  }
  WgradArgs a;
  memset(&a, 0, sizeof(a));
  a.a = dout; a.a_ld = cout; a.a_off = 0; a.ha = 2 * h; a.wa = 2 * w; a.a_scale = 2;
  a.b = x; a.b_ld = cin; a.b_off = 0; a.hb = h; a.wb = w; a.b_scale = 1;
  a.nimg = n; a.hg = h; a.wg = w;
  a.ntaps = 4;
  for (int t = 0; t < 4; ++t) {
    a.ayc |= ((t >> 1) + 1) << (2 * t);
    a.axc |= ((t & 1) + 1) << (2 * t);
    a.byc |= 1 << (2 * t);
    a.bxc |= 1 << (2 * t);
  }
  a.M = cout; a.N = cin;
  a.tap_stride = (long)cout * cin; a.out_ld = cin;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == CNNITMO_BF16) {
    const int splits = launch_wgrad_tconv((const bf16*)x, cin, 0, (const bf16*)dout, n, h, w, cin, cout,
                                          (float*)workspace, ws_bytes, s);
    if (splits > 0) {
      int rc = cnnitmo_check_launch("tconv2x2_wgrad");
      if (rc) return rc;
      const long slab = 4L * cout * cin;
      slab_reduce((const float*)workspace, slab, splits, 4 * cout, cin, cin, dk, f, s);
      return cnnitmo_check_launch("tconv2x2_wgrad");
    }
  }
  if (dtype == CNNITMO_F32) {
    const int splits = launch_wgrad_tconv_f32((const float*)x, cin, 0, (const float*)dout, n, h, w, cin, cout,
                                              (float*)workspace, ws_bytes, s);
    if (splits > 0) {
      int rc = cnnitmo_check_launch("tconv2x2_wgrad");
      if (rc) return rc;
      slab_reduce((const float*)workspace, 4L * cout * cin, splits, 4 * cout, cin, cin, dk, f, s);
      return cnnitmo_check_launch("tconv2x2_wgrad");
    }
  }
  if (dtype == CNNITMO_BF16)
    return run_wgrad<bf16>(a, dk, 4 * cout, cin, cin, workspace, ws_bytes, s, "tconv2x2_wgrad", f, 1);
  if (dtype == CNNITMO_F32)
    return run_wgrad<float>(a, dk, 4 * cout, cin, cin, workspace, ws_bytes, s, "tconv2x2_wgrad", f);
  cnnitmo_set_error("tconv2x2_wgrad: unsupported dtype %d", dtype);
  return CNNITMO_EUNSUPPORTED;
}

// Label of the main kernel cnnitmo_conv_wgrad (ntaps 9 / 1) or
// cnnitmo_tconv2x2_wgrad (ntaps 4) launches for these sizes (for profiles;
// each is followed by slab_reduce_kernel).
extern "C" const char* cnnitmo_wgrad_cat_kernel_name(int n, int h, int w, int c1, int cin, int cout) {
  return c1 == 32 ? wgrad_halo_name(n, h, w, cin, cout, true) : "";
}

extern "C" const char* cnnitmo_wgrad_kernel_name(int dtype, int ntaps, int n, int h, int w, int cin,
                                                 int cout) {
  if (dtype == CNNITMO_BF16 && ntaps == 9) {
    const char* hn = wgrad_halo_name(n, h, w, cin, cout);
    if (hn[0]) return hn;
  }
  if (dtype == CNNITMO_BF16 && ntaps == 4) {
    const char* tn = wgrad_tconv_name(n, h, w, cin, cout);
    if (tn[0]) return tn;
  }
  if (dtype == CNNITMO_F32 && ntaps == 4) {
    const char* tn = wgrad_tconv_f32_name(n, h, w, cin, cout);
    if (tn[0]) return tn;
  }
  if (dtype == CNNITMO_F32 && ntaps == 9) {
    const char* fn = wgrad_halo_f32_name(n, h, w, cin, cout);
    if (fn[0]) return fn;
  }
  const long P = (long)n * h * w;
  static thread_local char buf[80];
  if (dtype == CNNITMO_BF16) {
    const W2Label l = wgrad2_label(P, cout, cin, ntaps);
    if (l.ok) {
      snprintf(buf, sizeof(buf), "igemm_wgrad2_kernel<%d,%d,tpb%d>", l.bm, l.bn, l.tpb);
      return buf;
    }
  }
  const int bm = pick_tile(cout), bn = pick_tile(cin);
  snprintf(buf, sizeof(buf), "igemm_wgrad_kernel<%s,%d,%d>", dtype == CNNITMO_BF16 ? "bf16" : "f32", bm, bn);
  return buf;
}
