// Weight gradient of the stride-2 2x2 Conv2DTranspose (bf16; up6..up9 of the
// U-Net, model.py:199-200), row-streaming form:
//
//   dK[t=(a,b)][co][ci] = sum_{(n,y,x)} dy[n][2y+a][2x+b][co] * x[n][y][x][ci]
//
// A workgroup owns a strip of TW low-resolution columns, a contiguous range of
// (image, row) rows and a (BM output x BN input channel) block, and keeps ALL
// FOUR taps of that block in registers.  Per low-resolution row it loads the
// x row segment once (shared by the four taps) and the two output-gradient
// rows 2y and 2y+1 once (each dy pixel belongs to exactly one tap).  The
// generic implicit-GEMM wgrad (igemm_wgrad.hip) instead re-gathers x per tap
// and synchronises every 32 pixels through registers: 373 TFLOP/s on up6-up8.
//
// LDS images are [pixel][channel] rows filled by buffer_load_dwordx4 ... lds.
// The dy rows are DE-INTERLEAVED on the way in (image row b*TW + k holds column
// 2k+b), so each tap reads consecutive rows with ds_read_b64_tr_b16 and the
// row swizzle of wgrad_halo.hip stays conflict-free.  Columns past the image
// edge (the partial last strip) and the pipeline's run-out loads use an
// out-of-range buffer offset, which lands zeros.  Output: one fp32 slab
// [4*cout][cin] (row = t*cout + co) per (strip, row range), summed in a fixed
// order by slab_reduce_kernel (igemm_wgrad.hip), which also applies the
// folded-BN correction.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "dma.h"
#include "igemm_common.h"

#pragma clang diagnostic ignored "-Winline-asm"

namespace {

using dma::i32x4;


template <int R> __device__ __forceinline__ int trswz(int row) {
  if constexpr (R == 64) return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  return (row & 3) | (((row >> 3) & 1) << 2);  // R == 128
}
template <int R> __device__ __forceinline__ int bfo(int row, int col) {
  return row * (R * 2) + (((col >> 4) ^ trswz<R>(row)) << 5) + ((col & 15) << 1);
}

struct WTArgs {
  const bf16* dy;  // [n][2H][2W][cout]
  int cout;
  const bf16* x;  // view [n][H][W][x_ld] at x_off
  long x_ld;
  int x_off;
  int nimg, H, W, cin;
  float* out;  // slabs [units][4*cout][cin]
  long slab;
  int strips, cbm, cbn, units;
  long rows_per;
};

// 2 x WM x 2 waves: a (dy row parity) x cout halves x cin halves; each wave keeps
// taps (a, 0) and (a, 1) of its 64 x 64 tile.
template <int BM, int BN, int TW, int D>
struct WTCfg {
  static constexpr int WM = BM / 64, WN = BN / 64, NW = 2 * WM * WN, NT = NW * 64;
  static constexpr int FM = 4, FN = 4;
  static constexpr int XB = TW * BN * 2 / 1024;      // DMA instructions (1 KB) per x row segment
  static constexpr int DB = 2 * TW * BM * 2 / 1024;  // per dy row segment (2*TW pixels)
  static constexpr int GB = XB + 2 * DB;             // per step
  static constexpr int PER = GB / NW;                // per wave per step
  static constexpr int SLOT = GB * 1024, S = D + 1, SMEM = S * SLOT;
  static_assert(GB % NW == 0 && XB % NW == 0 && DB % NW == 0, "uniform DMA split");
  static_assert(TW % 32 == 0, "K steps of 32 pixels");
  static_assert(SMEM <= 160 * 1024, "LDS");
};

template <int BM, int BN, int TW, int D>
__global__ __launch_bounds__(2 * (BM / 64) * (BN / 64) * 64) void wgrad_tconv_kernel(const WTArgs p) {
  using C = WTCfg<BM, BN, TW, D>;
  constexpr int NW = C::NW, WN = C::WN, FM = C::FM, FN = C::FN, XB = C::XB, DB = C::DB, PER = C::PER;
  extern __shared__ __attribute__((aligned(1024))) char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wa = wave / (NW / 2), wq = wave - wa * (NW / 2);
  const int wm = wq / WN, wn = wq - (wq / WN) * WN;

  // block -> (unit, channel block): the channel blocks of one unit sit on one XCD
  // (they share its dy / x rows through that XCD's L2)
  const int CB = p.cbm * p.cbn;
  const int lid = xcd_remap(blockIdx.x, p.units * CB);
  const int cb = lid % CB, unit = lid / CB;
  const int strip = unit % p.strips, rs = unit / p.strips;
  const int m0 = (cb / p.cbn) * BM, n0 = (cb % p.cbn) * BN;
  const int x0 = strip * TW;
  const long total_rows = (long)p.nimg * p.H;
  const long g0 = (long)rs * p.rows_per;
  const long g1 = g0 + p.rows_per < total_rows ? g0 + p.rows_per : total_rows;
  const int nrows = (int)(g1 - g0);

  // ---- per-lane DMA geometry (fixed for the launch) ------------------------
  // every wave issues PER instructions per step: q < XB/NW -> x, else dy
  constexpr int QX = XB / NW, QD = 2 * DB / NW;
  unsigned xoff[QX], doff[QD];
#pragma unroll
  for (int q = 0; q < QX; ++q) {
    const int off = (wave + q * NW) * 1024 + lane * 16;
    const int row = off / (BN * 2), pos = off - row * (BN * 2);
    const int col = (((pos >> 5) ^ trswz<BN>(row)) << 4) + ((pos >> 4) & 1) * 8;
    xoff[q] = x0 + row < p.W ? (unsigned)((row * p.x_ld + col) * 2) : dma::OOB;
  }
#pragma unroll
  for (int q = 0; q < QD; ++q) {
    const int ins = wave + q * NW;  // 0 .. 2*DB-1: [DB of row 2y][DB of row 2y+1]
    const int a = ins / DB;
    const int off = (ins - a * DB) * 1024 + lane * 16;
    const int row = off / (BM * 2), pos = off - row * (BM * 2);
    const int col = (((pos >> 5) ^ trswz<BM>(row)) << 4) + ((pos >> 4) & 1) * 8;
    const int b = row / TW, k = row - b * TW;  // image row b*TW + k <- column 2k+b
    // a selects the second dy row: one row is 2W pixels further
    doff[q] = x0 + k < p.W ? (unsigned)((((long)a * 2 * p.W + 2 * k + b) * p.cout + col) * 2) : dma::OOB;
  }

  auto issue = [&](long g, int slot) {
    char* S = smem + slot * C::SLOT;
    const bool ok = g < g1;
    const long gg = ok ? g : g0;
    const i32x4 rx = dma::rsrc((uintptr_t)(p.x + ((size_t)gg * p.W + x0) * p.x_ld + p.x_off + n0));
#pragma unroll
    for (int q = 0; q < QX; ++q) dma::lds16(ok ? xoff[q] : dma::OOB, rx, S + (wave + q * NW) * 1024);
    const i32x4 rd = dma::rsrc((uintptr_t)(p.dy + ((size_t)(2 * gg) * 2 * p.W + 2 * x0) * p.cout + m0));
#pragma unroll
    for (int q = 0; q < QD; ++q) dma::lds16(ok ? doff[q] : dma::OOB, rd, S + (XB + wave + q * NW) * 1024);
  };

  f32x4 acc[2][FM][FN];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
#pragma unroll
  for (int k = 0; k < D; ++k) issue(g0 + k, k);
  int slot = 0, nslot = D;
  for (int k = 0; k < nrows; ++k) {
    dma::wait_vm<D * PER - PER>();  // this step's group landed (D-1 younger groups may fly)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    issue(g0 + k + D, nslot);  // into the slot every wave finished reading last step
    const char* Xs = smem + slot * C::SLOT;
    const char* Ds = Xs + XB * 1024 + wa * DB * 1024;
#pragma unroll
    for (int kk = 0; kk < TW / 32; ++kk) {
      const int r0 = kk * 32 + 8 * g + qq;
      bf16x8 bfr[FN];
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * 64 + j * 16 + 4 * pp;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Xs + bfo<BN>(r0, col)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Xs + bfo<BN>(r0 + 4, col)));
        bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        bf16x8 af[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int col = wm * 64 + i * 16 + 4 * pp;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Ds + bfo<BM>(b * TW + r0, col)));
          const s16x4 hi =
              __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Ds + bfo<BM>(b * TW + r0 + 4, col)));
          af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[b][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[b][i][j], 0, 0, 0);
      }
    }
    slot = slot + 1 == C::S ? 0 : slot + 1;
    nslot = nslot + 1 == C::S ? 0 : nslot + 1;
  }
  dma::wait_vm<0>();  // run-out loads (zeros) drain before the workgroup ends

  // ---- this workgroup's slab: [4*cout][cin], row = (2a+b)*cout + co ----------
  float* __restrict__ O = p.out + (size_t)unit * p.slab;
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = m0 + wm * 64 + i * 16 + g * 4 + rr;
        const size_t row = (size_t)(2 * wa + b) * p.cout + co;
#pragma unroll
        for (int j = 0; j < FN; ++j) O[row * p.cin + n0 + wn * 64 + j * 16 + li] = acc[b][i][j][rr];
      }
}

#ifndef WT_D_DEF
#define WT_D_DEF 2
#endif
constexpr int WT_TW = 32, WT_D = WT_D_DEF;

struct WTPlan {
  int bm, bn, strips, cbm, cbn, units, smem;
  long rows_per;
};

bool wt_plan(int n, int h, int w, int cin, int cout, WTPlan& pl) {
  pl.bm = cout % 128 == 0 ? 128 : (cout % 64 == 0 ? 64 : 0);
  pl.bn = cin % 128 == 0 ? 128 : 0;
  if (!pl.bm || !pl.bn) return false;
  pl.strips = (w + WT_TW - 1) / WT_TW;
  pl.cbm = cout / pl.bm;
  pl.cbn = cin / pl.bn;
  const int nw = 2 * (pl.bm / 64) * (pl.bn / 64);
  pl.smem = (WT_D + 1) * (WT_TW * pl.bn * 2 + 2 * 2 * WT_TW * pl.bm * 2);
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      ncu = prop.multiProcessorCount;
    if (ncu <= 0) ncu = 256;
  }
  const int occ = std::max(1, std::min((160 * 1024) / pl.smem, 16 / nw));
  const long slots = (long)ncu * occ;
  const long rows = (long)n * h;
  const long per = (long)pl.strips * pl.cbm * pl.cbn;
  long best = 1;
  double best_eff = -1.0;
  // at most two rounds of resident workgroups: every extra unit is another fp32
  // slab for slab_reduce_kernel to read
  for (long rs = 1; rs <= rows && per * rs <= 2 * slots; ++rs) {
    const long blocks = per * rs;
    const long rounds = (blocks + slots - 1) / slots;
    double eff = (double)blocks / (double)(rounds * slots);
    if (blocks < slots / 2) eff *= 0.5;
    if (eff > best_eff + 1e-3) { best_eff = eff; best = rs; }
  }
  pl.rows_per = (rows + best - 1) / best;
  pl.units = pl.strips * (int)((rows + pl.rows_per - 1) / pl.rows_per);
  return true;
}

template <int BM>
void wt_launch(const WTArgs& a, unsigned grid, int smem, hipStream_t s) {
  auto k = wgrad_tconv_kernel<BM, 128, WT_TW, WT_D>;
  static bool attr = [&] {
    return hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024) ==
           hipSuccess;
  }();
  (void)attr;
  hipLaunchKernelGGL(k, dim3(grid), dim3(WTCfg<BM, 128, WT_TW, WT_D>::NT), smem, s, a);
}

// ---- fp32 (fp32 training, main.py:126-132) -----------------------------------
// The same row walk with fp32 rows and v_mfma_f32_16x16x4_f32, 64 x 64 channel blocks
// (a 128-channel fp32 row segment set would not fit three slots).  No transposed LDS read
// exists for 32-bit elements: a lane builds each fragment (four MFMAs, k = pixel 4e + g)
// from four ds_read_b32 of consecutive pixel rows, whose 64-byte channel blocks are
// XOR-swizzled by row parity (the two rows a 32-lane half reads land on disjoint banks, as
// in wgrad_halo_f32).  8 waves = 2 (dy row parity a) x 2 (cout halves) x 2 (cin halves),
// each keeping taps (a, 0) and (a, 1) of its 32 x 32 tile.
template <int C> __device__ __forceinline__ int wfo(int row, int col) {
  return row * (C * 4) + ((((col >> 4) ^ (row & 1))) << 6) + ((col & 15) << 2);
}
constexpr int WTF_BM = 64, WTF_BN = 64, WTF_TW = 32, WTF_D = 2, WTF_NW = 8;
constexpr int WTF_XB = WTF_TW * WTF_BN * 4 / 1024;      // 8 DMA instructions per x row segment
constexpr int WTF_DB = 2 * WTF_TW * WTF_BM * 4 / 1024;  // 16 per dy row segment
constexpr int WTF_GB = WTF_XB + 2 * WTF_DB, WTF_PER = WTF_GB / WTF_NW;
constexpr int WTF_SLOT = WTF_GB * 1024, WTF_S = WTF_D + 1, WTF_SMEM = WTF_S * WTF_SLOT;
static_assert(WTF_GB % WTF_NW == 0 && WTF_XB % WTF_NW == 0 && WTF_DB % WTF_NW == 0, "uniform DMA split");
static_assert(WTF_SMEM <= 160 * 1024, "LDS");

struct WTFArgs {
  const float* dy;
  int cout;
  const float* x;
  long x_ld;
  int x_off;
  int nimg, H, W, cin;
  float* out;
  long slab;
  int strips, cbm, cbn, units;
  long rows_per;
};

__global__ __launch_bounds__(WTF_NW * 64) void wgrad_tconv_f32_kernel(const WTFArgs p) {
  constexpr int NW = WTF_NW, TW = WTF_TW, XB = WTF_XB, DB = WTF_DB, BM = WTF_BM, BN = WTF_BN, D = WTF_D;
  constexpr int PER = WTF_PER, FM = 2, FN = 2;
  __shared__ __attribute__((aligned(1024))) char smem[WTF_SMEM];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wa = wave >> 2, wm = (wave >> 1) & 1, wn = wave & 1;
  const int CB = p.cbm * p.cbn;
  const int lid = xcd_remap(blockIdx.x, p.units * CB);
  const int cb = lid % CB, unit = lid / CB;
  const int strip = unit % p.strips, rs = unit / p.strips;
  const int m0 = (cb / p.cbn) * BM, n0 = (cb % p.cbn) * BN;
  const int x0 = strip * TW;
  const long total_rows = (long)p.nimg * p.H;
  const long g0 = (long)rs * p.rows_per;
  const long g1 = g0 + p.rows_per < total_rows ? g0 + p.rows_per : total_rows;
  const int nrows = (int)(g1 - g0);

  // LDS slot (row, 64-byte block k) holds logical block k ^ (row & 1)
  constexpr int QX = XB / NW, QD = 2 * DB / NW;
  unsigned xoff[QX], doff[QD];
#pragma unroll
  for (int q = 0; q < QX; ++q) {
    const int off = (wave + q * NW) * 1024 + lane * 16;
    const int row = off / (BN * 4), pos = off - row * (BN * 4);
    const int col = (((pos >> 6) ^ (row & 1)) << 4) + ((pos >> 4) & 3) * 4;
    xoff[q] = x0 + row < p.W ? (unsigned)((row * p.x_ld + col) * 4) : dma::OOB;
  }
#pragma unroll
  for (int q = 0; q < QD; ++q) {
    const int ins = wave + q * NW;  // 0 .. 2*DB-1: [DB of row 2y][DB of row 2y+1]
    const int a = ins / DB;
    const int off = (ins - a * DB) * 1024 + lane * 16;
    const int row = off / (BM * 4), pos = off - row * (BM * 4);
    const int col = (((pos >> 6) ^ (row & 1)) << 4) + ((pos >> 4) & 3) * 4;
    const int b = row / TW, k = row - b * TW;  // image row b*TW + k <- column 2k+b
    doff[q] = x0 + k < p.W ? (unsigned)((((long)a * 2 * p.W + 2 * k + b) * p.cout + col) * 4) : dma::OOB;
  }
  auto issue = [&](long g, int slot) {
    char* S = smem + slot * WTF_SLOT;
    const bool ok = g < g1;
    const long gg = ok ? g : g0;
    const i32x4 rx = dma::rsrc((uintptr_t)(p.x + ((size_t)gg * p.W + x0) * p.x_ld + p.x_off + n0));
#pragma unroll
    for (int q = 0; q < QX; ++q) dma::lds16(ok ? xoff[q] : dma::OOB, rx, S + (wave + q * NW) * 1024);
    const i32x4 rd = dma::rsrc((uintptr_t)(p.dy + ((size_t)(2 * gg) * 2 * p.W + 2 * x0) * p.cout + m0));
#pragma unroll
    for (int q = 0; q < QD; ++q) dma::lds16(ok ? doff[q] : dma::OOB, rd, S + (XB + wave + q * NW) * 1024);
  };

  f32x4 acc[2][FM][FN];
#pragma unroll
  for (int t = 0; t < 2; ++t)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15;
#pragma unroll
  for (int k = 0; k < D; ++k) issue(g0 + k, k);
  int slot = 0, nslot = D;
  for (int k = 0; k < nrows; ++k) {
    dma::wait_vm<D * PER - PER>();  // this step's group landed (D-1 younger groups may fly)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    issue(g0 + k + D, nslot);  // into the slot every wave finished reading last step
    const char* Xs = smem + slot * WTF_SLOT;
    const char* Ds = Xs + XB * 1024 + wa * DB * 1024;
#pragma unroll
    for (int kk = 0; kk < TW / 16; ++kk) {
      float bfr[FN][4];
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e)
          bfr[j][e] = *reinterpret_cast<const float*>(Xs + wfo<BN>(kk * 16 + 4 * e + g, wn * 32 + j * 16 + li));
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        float af[FM][4];
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int e = 0; e < 4; ++e)
            af[i][e] = *reinterpret_cast<const float*>(Ds + wfo<BM>(b * TW + kk * 16 + 4 * e + g, wm * 32 + i * 16 + li));
#pragma unroll
        for (int e = 0; e < 4; ++e)
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j)
              acc[b][i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i][e], bfr[j][e], acc[b][i][j], 0, 0, 0);
      }
    }
    slot = slot + 1 == WTF_S ? 0 : slot + 1;
    nslot = nslot + 1 == WTF_S ? 0 : nslot + 1;
  }
  dma::wait_vm<0>();  // run-out loads (zeros) drain before the workgroup ends

  float* __restrict__ O = p.out + (size_t)unit * p.slab;
#pragma unroll
  for (int b = 0; b < 2; ++b)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = m0 + wm * 32 + i * 16 + g * 4 + rr;
        const size_t row = (size_t)(2 * wa + b) * p.cout + co;
#pragma unroll
        for (int j = 0; j < FN; ++j) O[row * p.cin + n0 + wn * 32 + j * 16 + li] = acc[b][i][j][rr];
      }
}

// row split for the fp32 kernel: the bf16 plan's policy at one 120 KB workgroup per CU
bool wtf_plan(int n, int h, int w, int cin, int cout, WTPlan& pl) {
  if (cout % WTF_BM || cin % WTF_BN) return false;
  pl.bm = WTF_BM;
  pl.bn = WTF_BN;
  pl.strips = (w + WTF_TW - 1) / WTF_TW;
  pl.cbm = cout / WTF_BM;
  pl.cbn = cin / WTF_BN;
  pl.smem = WTF_SMEM;
  int ncu = 0, dev = 0;
  hipDeviceProp_t prop;
  if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess) ncu = prop.multiProcessorCount;
  if (ncu <= 0) ncu = 256;
  const long slots = ncu;
  const long rows = (long)n * h;
  const long per = (long)pl.strips * pl.cbm * pl.cbn;
  long best = 1;
  double best_eff = -1.0;
  for (long rs = 1; rs <= rows && per * rs <= 2 * slots; ++rs) {
    const long blocks = per * rs;
    const long rounds = (blocks + slots - 1) / slots;
    double eff = (double)blocks / (double)(rounds * slots);
    if (blocks < slots / 2) eff *= 0.5;
    if (eff > best_eff + 1e-3) { best_eff = eff; best = rs; }
  }
  pl.rows_per = (rows + best - 1) / best;
  pl.units = pl.strips * (int)((rows + pl.rows_per - 1) / pl.rows_per);
  return true;
}

}  // namespace

size_t wgrad_tconv_f32_ws_bytes(int n, int h, int w, int cin, int cout) {
  WTPlan pl;
  if (!wtf_plan(n, h, w, cin, cout, pl)) return 0;
  return (size_t)pl.units * 4 * cout * cin * 4;
}

// fp32: returns the number of slabs written (>0) or -1 when this path does not apply.
int launch_wgrad_tconv_f32(const float* x, long x_ld, int x_off, const float* dy, int n, int h, int w, int cin,
                           int cout, float* ws, size_t ws_bytes, hipStream_t s) {
  WTPlan pl;
  if (!wtf_plan(n, h, w, cin, cout, pl)) return -1;
  if (x_ld % 4 || x_off % 4) return -1;
  const size_t need = (size_t)pl.units * 4 * cout * cin * 4;
  if (!ws || ws_bytes < need) return -1;
  WTFArgs a;
  memset(&a, 0, sizeof(a));
  a.dy = dy; a.cout = cout; a.x = x; a.x_ld = x_ld; a.x_off = x_off;
  a.nimg = n; a.H = h; a.W = w; a.cin = cin;
  a.out = ws; a.slab = 4L * cout * cin;
  a.strips = pl.strips; a.cbm = pl.cbm; a.cbn = pl.cbn; a.units = pl.units; a.rows_per = pl.rows_per;
  const unsigned grid = (unsigned)(pl.units * pl.cbm * pl.cbn);
  hipLaunchKernelGGL(wgrad_tconv_f32_kernel, dim3(grid), dim3(WTF_NW * 64), 0, s, a);
  return pl.units;
}

const char* wgrad_tconv_f32_name(int n, int h, int w, int cin, int cout) {
  WTPlan pl;
  if (!wtf_plan(n, h, w, cin, cout, pl)) return "";
  return "wgrad_tconv_f32_kernel<64,64,32>";
}

size_t wgrad_tconv_ws_bytes(int n, int h, int w, int cin, int cout) {
  WTPlan pl;
  if (!wt_plan(n, h, w, cin, cout, pl)) return 0;
  return (size_t)pl.units * 4 * cout * cin * 4;
}

// Returns the number of slabs written (>0) or -1 when this path does not apply.
int launch_wgrad_tconv(const bf16* x, long x_ld, int x_off, const bf16* dy, int n, int h, int w, int cin,
                       int cout, float* ws, size_t ws_bytes, hipStream_t s) {
  WTPlan pl;
  if (!wt_plan(n, h, w, cin, cout, pl)) return -1;
  if (x_ld % 8 || x_off % 8) return -1;
  const size_t need = (size_t)pl.units * 4 * cout * cin * 4;
  if (!ws || ws_bytes < need) return -1;
  WTArgs a;
  memset(&a, 0, sizeof(a));
  a.dy = dy; a.cout = cout; a.x = x; a.x_ld = x_ld; a.x_off = x_off;
  a.nimg = n; a.H = h; a.W = w; a.cin = cin;
  a.out = ws; a.slab = 4L * cout * cin;
  a.strips = pl.strips; a.cbm = pl.cbm; a.cbn = pl.cbn; a.units = pl.units; a.rows_per = pl.rows_per;
  const unsigned grid = (unsigned)(pl.units * pl.cbm * pl.cbn);
  if (pl.bm == 128) wt_launch<128>(a, grid, pl.smem, s);
  else wt_launch<64>(a, grid, pl.smem, s);
  return pl.units;
}

const char* wgrad_tconv_name(int n, int h, int w, int cin, int cout) {
  WTPlan pl;
  if (!wt_plan(n, h, w, cin, cout, pl)) return "";
  static thread_local char buf[64];
  snprintf(buf, sizeof(buf), "wgrad_tconv_kernel<%d,%d,%d>", pl.bm, pl.bn, WT_TW);
  return buf;
}
