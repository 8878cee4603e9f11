// Weight gradients, v2 (bf16): direct-to-LDS pipelined MFMA with multi-tap blocks.
//
//   C_t[m][n] = sum_p A[srcA_t(p)][m] * B[srcB_t(p)][n]   for the taps t of a block
//
// (conv3x3: A = dz unshifted, B = x shifted by tap t; tconv2x2: A = dout at the
// tap's parity, B = x).  One block owns one (m-tile, n-tile) for TPB taps and a
// contiguous pixel range (split-K); the tap-independent operand is loaded once
// per 64-pixel K-step and reused for all TPB taps, the tap-dependent one is
// gathered per tap.  Operands: LDS image [pixel][channel] filled by
// global_load_lds_dwordx4 (inline asm, see igemm_fwd2.hip), read back
// transposed with ds_read_b64_tr_b16 (K = pixels contiguous per lane); 32-byte
// column blocks XOR-swizzled by row exactly as igemm_wgrad.hip, with the
// swizzle moved to the DMA source address.  fp32 slabs per split, reduced by
// slab_reduce_kernel in a fixed order (bitwise reproducible).
#include <algorithm>
#include <cstring>

#include "igemm_common.h"

#pragma clang diagnostic ignored "-Winline-asm"

// per-TU zero page (no -fgpu-rdc): padding / out-of-range rows DMA from here
static __device__ __attribute__((aligned(256))) unsigned char g_zero_page[256] = {0};

namespace {

__device__ __forceinline__ unsigned lds_addr2(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ void glds(const void* gsrc, const char* lds) {
  const unsigned a = __builtin_amdgcn_readfirstlane(lds_addr2(lds));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(a) : "m0");
}
template <int N> __device__ __forceinline__ void waitvm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

template <int R> __device__ __forceinline__ int trswz(int row) {
  if constexpr (R == 32) return (row >> 3) & 1;
  if constexpr (R == 64) return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  return (row & 3) | (((row >> 3) & 1) << 2);  // R == 128
}
template <int R> __device__ __forceinline__ int bfo(int row, int col) {
  return row * (R * 2) + (((col >> 4) ^ trswz<R>(row)) << 5) + ((col & 15) << 1);
}

}  // namespace

template <int BM, int BN, int WM, int WN, int TPB, int ST>
struct W2Cfg {
  static constexpr int NW = WM * WN, NT = 64 * NW;
  static constexpr int BP = 64;  // pixels per K-step (two 16x16x32 substeps)
  static constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  static constexpr int A_BYTES = BP * BM * 2, B_BYTES = BP * BN * 2;
  static constexpr int A_INS = A_BYTES / 1024, B_INS = B_BYTES / 1024;
  static constexpr int ROWS_A = 1024 / (BM * 2), ROWS_B = 1024 / (BN * 2);  // pixel rows per DMA
};

// DEP = which operand is tap-dependent: 0 -> B (conv3x3), 1 -> A (tconv)
template <int BM, int BN, int WM, int WN, int TPB, int ST, int DEP>
__global__ __launch_bounds__(WM * WN * 64) void igemm_wgrad2_kernel(const Wgrad2Args p) {
  using C = W2Cfg<BM, BN, WM, WN, TPB, ST>;
  constexpr int BP = C::BP, FM = C::FM, FN = C::FN, TM = C::TM, TN = C::TN, NW = C::NW;
  constexpr int NA_T = DEP == 1 ? TPB : 1, NB_T = DEP == 0 ? TPB : 1;  // tiles per stage
  constexpr int STAGE = NA_T * C::A_BYTES + NB_T * C::B_BYTES;
  constexpr int INS_A = NA_T * C::A_INS, INS_B = NB_T * C::B_INS;
  static_assert(INS_A % NW == 0 && INS_B % NW == 0, "DMA instructions must split evenly over waves");
  constexpr int LA = INS_A / NW, LB = INS_B / NW;
  constexpr int L = LA + LB;  // DMA per wave per stage
  static_assert(ST * STAGE <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[ST * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int tiles = p.mblocks * p.nblocks;
  int lid = xcd_remap(blockIdx.x, tiles * p.tgroups * p.splits);
  const int split = lid / (tiles * p.tgroups);
  lid -= split * tiles * p.tgroups;
  const int tg = lid / tiles;
  lid -= tg * tiles;
  const int mb = lid / p.nblocks, nb = lid - mb * p.nblocks;
  const int m0 = mb * BM, n0 = nb * BN, t0 = tg * TPB;
  const long pbeg = (long)split * p.pix_per_split;
  const long pend = min(p.P, pbeg + p.pix_per_split);
  const int nk = (int)((pend - pbeg + BP - 1) / BP);
  const long hw = (long)p.hg * p.wg;

  // DMA bookkeeping: wave w issues A instructions w*LA .. w*LA+LA-1 (tile images
  // [tile][1 KB pieces]) and likewise for B.  Per instruction this lane covers one
  // pixel row and one 16-byte channel chunk (source-swizzled for the tr-reads).
  struct Row {
    int tile, col, img, h, w;
    long pix;
  };
  auto make_row = [&](int gi, int per, int rowbytes, int R) {
    Row r;
    r.tile = gi / per;
    const int off = (gi % per) * 1024 + lane * 16;
    const int row = off / rowbytes, pos = off % rowbytes;
    const int pb = pos >> 5, half = (pos >> 4) & 1;
    const int sw = R == 32 ? trswz<32>(row) : (R == 64 ? trswz<64>(row) : trswz<128>(row));
    r.col = (pb ^ sw) * 16 + half * 8;
    r.pix = pbeg + row;
    r.img = (int)(r.pix / hw);
    const int rem = (int)(r.pix - (long)r.img * hw);
    r.h = rem / p.wg;
    r.w = rem - r.h * p.wg;
    return r;
  };
  Row ra[LA], rb[LB];
#pragma unroll
  for (int q = 0; q < LA; ++q) ra[q] = make_row(wave * LA + q, C::A_INS, BM * 2, BM);
#pragma unroll
  for (int q = 0; q < LB; ++q) rb[q] = make_row(wave * LB + q, C::B_INS, BN * 2, BN);

  auto adv = [&](Row& r) {
    r.pix += BP;
    r.w += BP;
    while (r.w >= p.wg) {
      r.w -= p.wg;
      if (++r.h == p.hg) { r.h = 0; ++r.img; }
    }
  };
  auto issue = [&](int buf) {
    char* S = smem + buf * STAGE;
#pragma unroll
    for (int q = 0; q < LA; ++q) {
      const Row& r = ra[q];
      const int tap = t0 + r.tile;
      const void* src = g_zero_page;
      if (r.pix < pend && (DEP == 0 || tap < p.ntaps)) {
        const int dy = DEP == 1 ? ((p.ayc >> (2 * tap)) & 3) - 1 : 0;
        const int dx = DEP == 1 ? ((p.axc >> (2 * tap)) & 3) - 1 : 0;
        const int hh = r.h * p.a_scale + dy, ww = r.w * p.a_scale + dx;
        if ((unsigned)hh < (unsigned)p.ha && (unsigned)ww < (unsigned)p.wa)
          src = p.a + ((size_t)((long)r.img * p.ha + hh) * p.wa + ww) * p.a_ld + p.a_off + m0 + r.col;
      }
      glds(src, S + (wave * LA + q) * 1024);
    }
#pragma unroll
    for (int q = 0; q < LB; ++q) {
      const Row& r = rb[q];
      const int tap = t0 + r.tile;
      const void* src = g_zero_page;
      if (r.pix < pend && (DEP == 1 || tap < p.ntaps)) {
        const int dy = DEP == 0 ? ((p.byc >> (2 * tap)) & 3) - 1 : 0;
        const int dx = DEP == 0 ? ((p.bxc >> (2 * tap)) & 3) - 1 : 0;
        const int hh = r.h * p.b_scale + dy, ww = r.w * p.b_scale + dx;
        if ((unsigned)hh < (unsigned)p.hb && (unsigned)ww < (unsigned)p.wb)
          src = p.b + ((size_t)((long)r.img * p.hb + hh) * p.wb + ww) * p.b_ld + p.b_off + n0 + r.col;
      }
      glds(src, S + INS_A * 1024 + (wave * LB + q) * 1024);
    }
#pragma unroll
    for (int q = 0; q < LA; ++q) adv(ra[q]);
#pragma unroll
    for (int q = 0; q < LB; ++q) adv(rb[q]);
  };

  f32x4 acc[TPB][FM][FN];
#pragma unroll
  for (int t = 0; t < TPB; ++t)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  auto compute = [&](int buf) {
    const char* S = smem + buf * STAGE;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      const int r0 = kk * 32 + 8 * g + qq;
      bf16x8 af[NA_T][FM], bfr[NB_T][FN];
#pragma unroll
      for (int ta = 0; ta < NA_T; ++ta)
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const char* As = S + ta * C::A_BYTES;
          const int col = wm * TM + i * 16 + 4 * pp;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, As + bfo<BM>(r0, col)));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, As + bfo<BM>(r0 + 4, col)));
          af[ta][i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
      for (int tb = 0; tb < NB_T; ++tb)
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const char* Bs = S + NA_T * C::A_BYTES + tb * C::B_BYTES;
          const int col = wn * TN + j * 16 + 4 * pp;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Bs + bfo<BN>(r0, col)));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Bs + bfo<BN>(r0 + 4, col)));
          bfr[tb][j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
      for (int t = 0; t < TPB; ++t)
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[t][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[DEP == 1 ? t : 0][i], bfr[DEP == 0 ? t : 0][j],
                                                                 acc[t][i][j], 0, 0, 0);
    }
  };

  if (nk > 0) issue(0);
#pragma unroll
  for (int s = 1; s < ST - 1; ++s)
    if (s < nk) issue(s);
  for (int t = 0; t < nk; ++t) {
    if constexpr (ST == 3) {
      if (t + 1 < nk) waitvm<L>(); else waitvm<0>();
    } else {
      waitvm<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (t + ST - 1 < nk) issue((t + ST - 1) % ST);
    compute(t % ST);
  }

#pragma unroll
  for (int t = 0; t < TPB; ++t) {
    if (t0 + t >= p.ntaps) continue;
    float* __restrict__ O = p.out + (size_t)split * p.split_stride + (size_t)(t0 + t) * p.tap_stride;
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int m = m0 + wm * TM + i * 16 + g * 4 + r;
#pragma unroll
        for (int j = 0; j < FN; ++j) O[(size_t)m * p.out_ld + n0 + wn * TN + j * 16 + li] = acc[t][i][j][r];
      }
  }
}

// ----------------------------------------------------------------------------
struct W2Plan {
  int bm, bn, tpb, mblocks, nblocks, tgroups, splits;
  long pps;
};

// Tile per (M, N, taps); chosen on tools/bench_layers.py measurements.
static void w2_tiles(int M, int N, int ntaps, int& bm, int& bn, int& tpb) {
  bm = M % 128 == 0 ? 128 : (M % 64 == 0 ? 64 : 32);
  bn = N % 128 == 0 ? 128 : (N % 64 == 0 ? 64 : 32);
  if (bm == 128 && bn == 128) { tpb = 1; return; }
  if (ntaps == 9) tpb = (bm * bn <= 32 * 64) ? 9 : 3;  // small tiles: reuse dz over taps
  else if (ntaps == 4) tpb = (bm * bn <= 64 * 64) ? 4 : 2;
  else tpb = 1;
  if (bm * bn >= 128 * 64 && tpb > 3) tpb = ntaps == 4 ? 2 : 3;
}

static W2Plan w2_plan(long P, int M, int N, int ntaps) {
  W2Plan pl;
  w2_tiles(M, N, ntaps, pl.bm, pl.bn, pl.tpb);
  pl.mblocks = M / pl.bm;
  pl.nblocks = N / pl.bn;
  pl.tgroups = (ntaps + pl.tpb - 1) / pl.tpb;
  const long tiles = (long)pl.mblocks * pl.nblocks * pl.tgroups;
  const long ksteps = (P + 63) / 64;
  long splits = (2048 + tiles - 1) / tiles;
  splits = std::min(splits, std::max(1L, ksteps / 4));
  const long slab_bytes = (long)M * N * ntaps * 4;
  splits = std::max(1L, std::min(splits, (512L << 20) / slab_bytes));
  const long steps_per = (ksteps + splits - 1) / splits;
  pl.pps = steps_per * 64;
  pl.splits = (int)((P + pl.pps - 1) / pl.pps);
  return pl;
}

size_t wgrad2_ws_bytes(long P, int M, int N, int ntaps) {
  const W2Plan pl = w2_plan(P, M, N, ntaps);
  return (size_t)pl.splits * M * N * ntaps * 4;
}

template <int BM, int BN, int WM, int WN, int TPB, int DEP>
static void w2_launch(const Wgrad2Args& a, hipStream_t s, unsigned grid) {
  constexpr int ST = (BM == 128 && BN == 128) ? 3 : 2;
  hipLaunchKernelGGL((igemm_wgrad2_kernel<BM, BN, WM, WN, TPB, ST, DEP>), dim3(grid), dim3(WM * WN * 64), 0, s, a);
}

// conv3x3 (DEP 0): taps per block 1 / 3 / 9; tconv (DEP 1): 1 / 2 / 4.
// dry_run: only report whether the plan is one of the instantiated kernels
static bool w2_dispatch(const Wgrad2Args& a, const W2Plan& pl, hipStream_t s, unsigned grid, int dep,
                        bool dry_run = false) {
#define W2(BMv, BNv, WMv, WNv, TPBv, DEPv)                                     \
  if (pl.bm == BMv && pl.bn == BNv && pl.tpb == TPBv && dep == DEPv) {        \
    if (!dry_run) w2_launch<BMv, BNv, WMv, WNv, TPBv, DEPv>(a, s, grid);      \
    return true;                                                              \
  }
  // reachable (tile, taps-per-block) plans of w2_tiles; anything else falls back to
  // v1 -- including 128x128, where v1's 2-stage register pipeline at 3 waves/SIMD
  // measured 1.7x faster than this kernel (tools/bench_layers.py, dec6/dec7 wgrad)
  W2(128, 64, 2, 2, 3, 0) W2(64, 128, 2, 2, 3, 0) W2(64, 64, 2, 2, 3, 0)
  W2(128, 32, 4, 1, 3, 0) W2(32, 128, 1, 4, 3, 0) W2(64, 32, 2, 2, 9, 0) W2(32, 64, 2, 2, 9, 0)
  W2(32, 32, 2, 2, 9, 0) W2(32, 32, 2, 2, 1, 0)
  W2(128, 64, 2, 2, 2, 1) W2(64, 128, 2, 2, 2, 1) W2(64, 64, 2, 2, 4, 1)
  W2(128, 32, 4, 1, 4, 1) W2(32, 128, 1, 4, 4, 1) W2(64, 32, 2, 2, 4, 1) W2(32, 64, 2, 2, 4, 1)
  W2(32, 32, 2, 2, 4, 1)
#undef W2
  return false;
}

// Returns the number of split slabs written (> 0), or < 0 if this plan is
// unsupported or the workspace is too small (caller falls back to v1).
int launch_wgrad2(Wgrad2Args a, void* ws, size_t ws_bytes, hipStream_t s) {
  a.P = (long)a.nimg * a.hg * a.wg;
  const W2Plan pl = w2_plan(a.P, a.M, a.N, a.ntaps);
  const long slab = (long)a.M * a.N * a.ntaps;
  if (!ws || ws_bytes < (size_t)pl.splits * slab * 4) return -1;
  a.out = (float*)ws;
  a.split_stride = slab;
  a.mblocks = pl.mblocks;
  a.nblocks = pl.nblocks;
  a.tgroups = pl.tgroups;
  a.splits = pl.splits;
  a.pix_per_split = pl.pps;
  const long total = (long)pl.mblocks * pl.nblocks * pl.tgroups * pl.splits;
  return w2_dispatch(a, pl, s, (unsigned)total, a.a_tapdep) ? pl.splits : -2;
}

W2Label wgrad2_label(long P, int M, int N, int ntaps) {
  const W2Plan pl = w2_plan(P, M, N, ntaps);
  W2Label l{false, pl.bm, pl.bn, pl.tpb};
  Wgrad2Args a;
  memset(&a, 0, sizeof(a));
  l.ok = w2_dispatch(a, pl, nullptr, 0, ntaps == 4 ? 1 : 0, true);
  return l;
}
