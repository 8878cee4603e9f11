// Weight gradient of the 3x3 'same' conv (bf16, every U-Net 3x3 layer),
// sliding-window form:
//
//   dW[co][t=(r,s)][ci] = sum_p dz[p][co] * x[p + (r-1, s-1)][ci]
//
// A workgroup owns a vertical strip of TW pixel columns, a contiguous range of
// (image, row) rows, and a (BM output x BN input channel) block; ALL nine taps
// of that block accumulate in registers.  Walking down the strip one row per
// step, it loads each dz row once and each x row once (plus a 1-pixel
// horizontal halo): the three x rows y-1, y, y+1 stay in an LDS ring and the
// nine taps are nine (row, column-shift) windows of it.  The implicit-GEMM
// wgrad (igemm_wgrad2.hip) instead re-gathers x for every tap; with 32..192
// channels per pixel that re-read bounds it (dec9: 265 TFLOP/s).
//
// LDS images are [pixel][channel] rows filled by global_load_lds_dwordx4 and
// read transposed with ds_read_b64_tr_b16 (K = pixels contiguous per lane); the
// 32-byte column blocks are XOR-swizzled by row (trswz), conflict-free for
// windows starting at any row (the column shift s; tools/check_swizzle.py).  Output: one fp32 slab [cout][9][cin] per (strip, row range),
// reduced in a fixed order by slab_reduce_kernel (igemm_wgrad.hip), which also
// applies the folded-BN correction.
#include <algorithm>
#include <cstdio>
#include <cstring>

#include "dma.h"
#include "igemm_common.h"

#pragma clang diagnostic ignored "-Winline-asm"

namespace {

using dma::i32x4;


// row swizzle of the 32-byte column blocks of an R-channel bf16 row
template <int R> __device__ __forceinline__ int trswz(int row) {
  if constexpr (R == 32 || R == 96) return (row >> 3) & 1;
  if constexpr (R == 64) return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  return (row & 3) | (((row >> 3) & 1) << 2);  // R == 128
}
template <int R> __device__ __forceinline__ int bfo(int row, int col) {
  return row * (R * 2) + (((col >> 4) ^ trswz<R>(row)) << 5) + ((col & 15) << 1);
}

struct WHArgs {
  const bf16* dz;  // [P][cout]
  int cout;
  const bf16* x;  // view [P][x_ld] at x_off
  long x_ld;
  int x_off;
  const bf16* x2;  // CAT: input channels [32, cin) from x2 [P][x2_ld] at x2_off (x holds [0, 32))
  long x2_ld;
  int x2_off;
  int nimg, H, W, cin;
  float* out;  // slabs [splits][cout][9*cin]
  long slab;
  int strips, cbm, cbn, rsplits;
  long rows_per;  // row steps per workgroup
  int cbase;      // first input channel of the launch's column blocks (a split 128 + 64 launch)
};

// Waves: three groups (one per kernel row r = 0, 1, 2), each WM x WN over the
// (BM, BN) block, so every wave keeps 3 taps x its tile in accumulators.
// D: groups (dz row + x row) issued ahead; R: rows per barrier step.
// CAT: the input is a concatenate read from its two members (model.py:261,
// [conv1 32 | up9 64]) without a concat buffer; an x row image is then two images,
// [XROWS][32] (KB 0..XBA) and [XROWS][BN-32] (KB XBA..), each swizzled as its own
// width, so that every DMA instruction reads one member.
template <int BM, int BN, int TW, int WM, int WN, int D, int R, bool CAT = false>
struct WHCfg {
  static constexpr int NWG = WM * WN, NW = 3 * NWG, NT = NW * 64;
  static constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16, KS = TW / 32;
  static constexpr int XROWS = TW + 2;
  static constexpr int XBA = CAT ? (XROWS * 32 * 2 + 1023) / 1024 : 0;  // KB of the first member's image
  static constexpr int XB = CAT ? XBA + (XROWS * (BN - 32) * 2 + 1023) / 1024
                                : (XROWS * BN * 2 + 1023) / 1024;  // KB (= DMA instructions) per x row
  static constexpr int DB = TW * BM * 2 / 1024;              // per dz row
  static constexpr int XS = D + R + 2, DS = D + R;           // ring slots
  static constexpr int SMEM = ((XS + 1) * XB + DS * DB) * 1024;  // + one all-zero x row
  static constexpr int LX = (XB + NW - 1) / NW, LD = (DB + NW - 1) / NW;  // max DMA per wave per row
  static_assert(TW * BM * 2 % 1024 == 0, "dz rows must be whole KB");
  static_assert(D >= R, "a step multiplies R rows, so at least R groups must be in flight at its wait");
  static_assert(SMEM <= 160 * 1024, "LDS");
};

template <int BM, int BN, int TW, int WM, int WN, int D, int R, bool CAT = false>
__global__ __launch_bounds__(3 * WM * WN * 64) void wgrad_halo_kernel(const WHArgs p) {
  using C = WHCfg<BM, BN, TW, WM, WN, D, R, CAT>;
  static_assert(!CAT || BN == 96, "CAT: a 32 + 64 channel input in one block");
  constexpr int NW = C::NW, TM = C::TM, TN = C::TN, FM = C::FM, FN = C::FN, KS = C::KS;
  constexpr int XB = C::XB, DB = C::DB, XS = C::XS, DS = C::DS, LX = C::LX, LD = C::LD;
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  char* const xbase = smem;
  char* const zrow = smem + XS * XB * 1024;  // all-zero x row: taps across the image edge
  char* const dbase = zrow + XB * 1024;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR) for the vmcnt switch
  const int wr = wave / C::NWG, wq = wave - wr * C::NWG;  // kernel row of this wave's taps
  const int wm = wq / WN, wn = wq % WN;
  // consecutive logical ids (the cbm x cbn column blocks of one strip and row range,
  // which read the same dz / x rows) run on one XCD: the re-reads are L2 hits
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int cb = bid % (p.cbm * p.cbn);
  bid /= p.cbm * p.cbn;
  const int strip = bid % p.strips;
  const int rs = bid / p.strips;
  const int m0 = (cb / p.cbn) * BM, n0 = p.cbase + (cb % p.cbn) * BN;
  const int x0 = strip * TW;
  const long total_rows = (long)p.nimg * p.H;
  const long g0 = (long)rs * p.rows_per;
  const long g1 = g0 + p.rows_per < total_rows ? g0 + p.rows_per : total_rows;
  const int nrows = (int)(g1 - g0);
  const int split = rs * p.strips + strip;

  // ---- per-lane DMA geometry (fixed for the launch) --------------------------
  // x row image: XROWS pixel rows (columns x0-1 .. x0+TW) of BN channels
  unsigned xoff[LX];  // byte offset from pixel (row g, column x0 - 1), dma::OOB outside the image
  bool xact[LX];      // this wave issues DMA q
#pragma unroll
  for (int q = 0; q < LX; ++q) {
    const int ins = wave + q * NW;
    xact[q] = ins < XB;
    if constexpr (CAT) {
      const bool first = ins < C::XBA;  // an instruction of the first member's image
      const int rw = first ? 64 : (BN - 32) * 2;
      const int off = (first ? ins : ins - C::XBA) * 1024 + lane * 16;
      const int row = off / rw, pos = off - row * rw;
      const int sw = first ? trswz<32>(row) : trswz<BN - 32>(row);
      const int col = (((pos >> 5) ^ sw) << 4) + ((pos >> 4) & 1) * 8;
      const int xx = x0 - 1 + row;
      const long ld = first ? p.x_ld : p.x2_ld;
      xoff[q] = row < C::XROWS && xx >= 0 && xx < p.W ? (unsigned)((row * ld + col) * 2) : dma::OOB;
    } else {
      const int off = ins * 1024 + lane * 16;
      const int row = off / (BN * 2), pos = off - row * (BN * 2);
      const int col = (((pos >> 5) ^ trswz<BN>(row)) << 4) + ((pos >> 4) & 1) * 8;
      const int xx = x0 - 1 + row;
      xoff[q] = row < C::XROWS && xx >= 0 && xx < p.W ? (unsigned)((row * p.x_ld + col) * 2) : dma::OOB;
    }
  }
  unsigned doff[LD];
  bool dact[LD];  // (the last strip may overhang the image: zero columns)
#pragma unroll
  for (int q = 0; q < LD; ++q) {
    const int ins = wave + q * NW;
    dact[q] = ins < DB;
    const int off = ins * 1024 + lane * 16;
    const int row = off / (BM * 2), pos = off - row * (BM * 2);
    const int col = (((pos >> 5) ^ trswz<BM>(row)) << 4) + ((pos >> 4) & 1) * 8;
    doff[q] = x0 + row < p.W ? (unsigned)((row * p.cout + col) * 2) : dma::OOB;
  }
  int nx = 0, nd = 0;  // DMA instructions this wave issues per x / dz row
#pragma unroll
  for (int q = 0; q < LX; ++q) nx += xact[q] ? 1 : 0;
#pragma unroll
  for (int q = 0; q < LD; ++q) nd += dact[q] ? 1 : 0;

  auto issue_x = [&](long g, int slot) {
    char* S = xbase + slot * XB * 1024;
    const bool ok = g >= 0 && g < total_rows;
    const long e0 = ((long)g * p.W + x0 - 1) * p.x_ld + p.x_off + n0;  // may be < 0 (first pixel)
    const i32x4 rs = dma::rsrc((uintptr_t)p.x + (uintptr_t)(e0 * 2));
    i32x4 rs2 = rs;
    if constexpr (CAT) {
      const long e2 = ((long)g * p.W + x0 - 1) * p.x2_ld + p.x2_off;
      rs2 = dma::rsrc((uintptr_t)p.x2 + (uintptr_t)(e2 * 2));
    }
#pragma unroll
    for (int q = 0; q < LX; ++q)
      if (xact[q]) dma::lds16(ok ? xoff[q] : dma::OOB, CAT && wave + q * NW >= C::XBA ? rs2 : rs,
                              S + (wave + q * NW) * 1024);
  };
  auto issue_d = [&](long g, int slot) {
    char* S = dbase + slot * DB * 1024;
    const i32x4 rs = dma::rsrc((uintptr_t)(p.dz + ((size_t)g * p.W + x0) * p.cout + m0));
#pragma unroll
    for (int q = 0; q < LD; ++q)
      if (dact[q]) dma::lds16(doff[q], rs, S + (wave + q * NW) * 1024);
  };

  f32x4 acc[3][FM][FN];  // taps (wr, s), s = 0..2
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  for (int i = tid; i < XB * 1024 / 16; i += C::NT)
    *reinterpret_cast<uint4*>(zrow + i * 16) = uint4{0u, 0u, 0u, 0u};
  // (ordered before the first use by the loop's barrier)

  // ---- pipeline: group k = {dz row g0+k, x row g0+k+1}; x rows g0-1, g0 first --
  // D groups are issued ahead; each step (one vmcnt wait + one barrier) multiplies R
  // rows and then issues the R groups that refill the slots of the previous step
  int issued = 0;
  int gq[D + R];  // gq[j]: value of `issued` once group k + j is issued
  int xslot_next = 0;  // slot for the next x row to issue (rows issued in order from g0-1)
  int dslot_next = 0;
  auto issue_group = [&](int j) {
    issue_d(g0 + j, dslot_next);
    dslot_next = dslot_next + 1 == DS ? 0 : dslot_next + 1;
    issue_x(g0 + j + 1, xslot_next);
    xslot_next = xslot_next + 1 == XS ? 0 : xslot_next + 1;
    issued += nd + nx;
  };
  issue_x(g0 - 1, xslot_next);
  xslot_next = xslot_next + 1 == XS ? 0 : xslot_next + 1;
  issue_x(g0, xslot_next);
  xslot_next = xslot_next + 1 == XS ? 0 : xslot_next + 1;
  issued += 2 * nx;
#pragma unroll
  for (int j = 0; j < D + R; ++j) {
    if (j < D && j < nrows) issue_group(j);
    gq[j] = issued;
  }
  int xs0 = 0;  // slot of x row g0+k-1
  int ds0 = 0;  // slot of dz row g0+k
  int y = (int)(g0 % p.H);
  auto nxt = [](int sl, int n) { return sl + 1 == n ? 0 : sl + 1; };
  // one row: taps r = 0,1,2 read x rows y-1, y, y+1 (zero at the image edge)
  auto row = [&](int dsl, int xa, int yy) {
    const char* Ds = dbase + dsl * DB * 1024;
    const int xb = nxt(xa, XS), xc = nxt(xb, XS);
    // rows outside the image read the zero row (a uniform pointer select, no branch:
    // a skipped tap would make the compiler copy the accumulators around it)
    const int xsr = wr == 0 ? xa : (wr == 1 ? xb : xc);
    const char* Xs = (wr == 0 && yy == 0) || (wr == 2 && yy == p.H - 1) ? zrow : xbase + xsr * XB * 1024;
#pragma unroll
    for (int kk = 0; kk < KS; ++kk) {
      const int r0 = kk * 32 + 8 * g + qq;
      bf16x8 af[FM];
#pragma unroll
      for (int i = 0; i < FM; ++i) {
        const int col = wm * TM + i * 16 + 4 * pp;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Ds + bfo<BM>(r0, col)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Ds + bfo<BM>(r0 + 4, col)));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int s = 0; s < 3; ++s) {
        bf16x8 bfr[FN];
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const int col = wn * TN + j * 16 + 4 * pp;
          int a0, a1;
          if constexpr (CAT) {  // the fragment's 16 channels lie in one member's image (wave-uniform)
            const bool first = wn * TN + j * 16 < 32;
            a0 = first ? bfo<32>(r0 + s, col) : C::XBA * 1024 + bfo<BN - 32>(r0 + s, col - 32);
            a1 = first ? bfo<32>(r0 + s + 4, col) : C::XBA * 1024 + bfo<BN - 32>(r0 + s + 4, col - 32);
          } else {
            a0 = bfo<BN>(r0 + s, col);
            a1 = bfo<BN>(r0 + s + 4, col);
          }
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Xs + a0));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Xs + a1));
          bfr[j] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int i = 0; i < FM; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j)
            acc[s][i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[s][i][j], 0, 0, 0);
      }
    }
  };
  for (int k = 0; k < nrows; k += R) {
    const int last = nrows - k < R ? nrows - k - 1 : R - 1;  // rows k .. k+last this step
    dma::wait_vm_small(issued - gq[last]);  // (0 in steady state when D == R, one group when D == R + 1)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (k + D + r < nrows) issue_group(k + D + r);
      gq[D + r] = issued;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      if (r <= last) {
        row(ds0, xs0, y);
        xs0 = nxt(xs0, XS);
        ds0 = nxt(ds0, DS);
        y = y + 1 == p.H ? 0 : y + 1;
      }
    }
#pragma unroll
    for (int q = 0; q < D; ++q) gq[q] = gq[q + R];
  }

  // ---- this workgroup's slab: [cout][9][cin] (its BM x BN block) ----------------
  float* __restrict__ O = p.out + (size_t)split * p.slab;
#pragma unroll
  for (int s = 0; s < 3; ++s)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = m0 + wm * TM + i * 16 + g * 4 + rr;
        const int t = wr * 3 + s;
#pragma unroll
        for (int j = 0; j < FN; ++j)
          O[(size_t)co * 9 * p.cin + t * p.cin + n0 + wn * TN + j * 16 + li] = acc[s][i][j][rr];
      }
}

// ---- fp32 (the fp32 training path, Keras' own precision; main.py:126-132) ---------
// The same sliding-window walk with fp32 rows and v_mfma_f32_16x16x4_f32.  There is no
// transposed LDS read for 32-bit elements, so a lane builds each 16-byte fragment (four
// 16x16x4 MFMAs, k = pixel 4e + g) from four ds_read_b32 of consecutive pixel rows; the
// 64-byte channel blocks of a row are XOR-swizzled by row parity (igemm_wgrad's f_off), so
// the two rows a 32-lane half reads land on disjoint banks.  fp32 MFMA runs at 1/16 of the
// bf16 rate, so neither the LDS reads nor the row DMA come close to binding; the point is
// reading every x row once instead of once per tap (the implicit GEMM re-gathers x nine
// times).  Blocks of 32 / 64 output x 32 / 64 input channels, 64-pixel strips, one row per
// barrier step, two row groups ahead; 3 x (BM/32) x (BN/32) waves of 32 x 32 tiles.
template <int C> __device__ __forceinline__ int ffo(int row, int col) {
  return row * (C * 4) + ((((col >> 4) ^ (row & 1))) << 6) + ((col & 15) << 2);
}

// row groups issued ahead for the fp32 64 x 32 block (enc2a): with D = 2 its 102 KB ring
// allows one 6-wave workgroup per CU; D = 1 (77 KB) two (dec9 on this block: 18.03 -> 17.45
// ms, profiles/r04z_wf_layers.txt).  The 64 x 96 block (dec9, cin 96: one workgroup reads
// each dz row once for all 96 input channels, 12 waves of 32 x 48 tiles, 144 VGPRs) fits
// only with D = 1 (157 KB): dec9's fp32 weight gradient 17.93 -> 12.58 ms (103 -> 147 TF/s,
// 0.93 of fp32 peak), fp32 training 30.96 -> 31.63 frames/s (profiles/r04z_wf96_*).
#ifndef WF_D6432
#define WF_D6432 1
#endif
#ifndef WF_BN96
#define WF_BN96 1
#endif
constexpr int wf_ahead(int bm, int bn) { return bn == 96 ? 1 : (bm == 64 && bn == 32 ? WF_D6432 : 2); }
constexpr int wf_wn(int bn) { return bn == 96 ? 2 : bn / 32; }  // waves across the BN columns

template <int BM, int BN>
struct WF32Cfg {
  static constexpr int WM = BM / 32, WN = wf_wn(BN), NWG = WM * WN, NW = 3 * NWG, NT = NW * 64;
  static constexpr int TW = 64, XROWS = TW + 2, D = wf_ahead(BM, BN), R = 1;
  static constexpr int XB = (XROWS * BN * 4 + 1023) / 1024, DB = TW * BM * 4 / 1024;
  static constexpr int XS = D + R + 2, DS = D + R;
  static constexpr int SMEM = ((XS + 1) * XB + DS * DB) * 1024;
  static constexpr int LX = (XB + NW - 1) / NW, LD = (DB + NW - 1) / NW;
  static_assert(SMEM <= 160 * 1024, "LDS");
};

template <int BM, int BN>
__global__ __launch_bounds__(3 * (BM / 32) * wf_wn(BN) * 64) void wgrad_halo_f32_kernel(const WHArgs p) {
  using C = WF32Cfg<BM, BN>;
  constexpr int NW = C::NW, TW = C::TW, XB = C::XB, DB = C::DB, XS = C::XS, DS = C::DS, LX = C::LX, LD = C::LD;
  constexpr int D = C::D, WN = C::WN;
  constexpr int FM = 2, FN = BN / (16 * WN);  // 32 x 32 (32 x 48 for BN 96) wave tiles
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  char* const xbase = smem;
  char* const zrow = smem + XS * XB * 1024;
  char* const dbase = zrow + XB * 1024;
  const float* X = reinterpret_cast<const float*>(p.x);
  const float* DZ = reinterpret_cast<const float*>(p.dz);

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wr = wave / C::NWG, wq = wave - wr * C::NWG;
  const int wm = wq / WN, wn = wq % WN;
  int bid = xcd_remap(blockIdx.x, gridDim.x);
  const int cb = bid % (p.cbm * p.cbn);
  bid /= p.cbm * p.cbn;
  const int strip = bid % p.strips;
  const int rs = bid / p.strips;
  const int m0 = (cb / p.cbn) * BM, n0 = p.cbase + (cb % p.cbn) * BN;
  const int x0 = strip * TW;
  const long total_rows = (long)p.nimg * p.H;
  const long g0 = (long)rs * p.rows_per;
  const long g1 = g0 + p.rows_per < total_rows ? g0 + p.rows_per : total_rows;
  const int nrows = (int)(g1 - g0);
  const int split = rs * p.strips + strip;

  // DMA geometry: LDS slot (row, piece pc') holds logical piece pc' ^ 4*(row & 1)
  unsigned xoff[LX];
  bool xact[LX];
#pragma unroll
  for (int q = 0; q < LX; ++q) {
    const int ins = wave + q * NW;
    xact[q] = ins < XB;
    const int off = ins * 1024 + lane * 16;
    const int row = off / (BN * 4), pos = off - row * (BN * 4);
    const int col = ((pos >> 4) ^ ((row & 1) << 2)) * 4;
    const int xx = x0 - 1 + row;
    xoff[q] = row < C::XROWS && xx >= 0 && xx < p.W ? (unsigned)((row * p.x_ld + col) * 4) : dma::OOB;
  }
  unsigned doff[LD];
  bool dact[LD];
#pragma unroll
  for (int q = 0; q < LD; ++q) {
    const int ins = wave + q * NW;
    dact[q] = ins < DB;
    const int off = ins * 1024 + lane * 16;
    const int row = off / (BM * 4), pos = off - row * (BM * 4);
    const int col = ((pos >> 4) ^ ((row & 1) << 2)) * 4;
    doff[q] = x0 + row < p.W ? (unsigned)((row * p.cout + col) * 4) : dma::OOB;
  }
  int nx = 0, nd = 0;
#pragma unroll
  for (int q = 0; q < LX; ++q) nx += xact[q] ? 1 : 0;
#pragma unroll
  for (int q = 0; q < LD; ++q) nd += dact[q] ? 1 : 0;

  auto issue_x = [&](long g, int slot) {
    char* S = xbase + slot * XB * 1024;
    const bool ok = g >= 0 && g < total_rows;
    const long e0 = ((long)g * p.W + x0 - 1) * p.x_ld + p.x_off + n0;
    const i32x4 rsc = dma::rsrc((uintptr_t)X + (uintptr_t)(e0 * 4));
#pragma unroll
    for (int q = 0; q < LX; ++q)
      if (xact[q]) dma::lds16(ok ? xoff[q] : dma::OOB, rsc, S + (wave + q * NW) * 1024);
  };
  auto issue_d = [&](long g, int slot) {
    char* S = dbase + slot * DB * 1024;
    const i32x4 rsc = dma::rsrc((uintptr_t)(DZ + ((size_t)g * p.W + x0) * p.cout + m0));
#pragma unroll
    for (int q = 0; q < LD; ++q)
      if (dact[q]) dma::lds16(doff[q], rsc, S + (wave + q * NW) * 1024);
  };

  f32x4 acc[3][FM][FN];
#pragma unroll
  for (int t = 0; t < 3; ++t)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[t][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, li = lane & 15;
  for (int i = tid; i < XB * 1024 / 16; i += C::NT)
    *reinterpret_cast<uint4*>(zrow + i * 16) = uint4{0u, 0u, 0u, 0u};

  int issued = 0;
  int gq[D + 1];
  int xslot_next = 0, dslot_next = 0;
  auto issue_group = [&](int j) {
    issue_d(g0 + j, dslot_next);
    dslot_next = dslot_next + 1 == DS ? 0 : dslot_next + 1;
    issue_x(g0 + j + 1, xslot_next);
    xslot_next = xslot_next + 1 == XS ? 0 : xslot_next + 1;
    issued += nd + nx;
  };
  issue_x(g0 - 1, xslot_next);
  xslot_next = xslot_next + 1 == XS ? 0 : xslot_next + 1;
  issue_x(g0, xslot_next);
  xslot_next = xslot_next + 1 == XS ? 0 : xslot_next + 1;
  issued += 2 * nx;
#pragma unroll
  for (int j = 0; j < D + 1; ++j) {
    if (j < D && j < nrows) issue_group(j);
    gq[j] = issued;
  }
  int xs0 = 0, ds0 = 0;
  int y = (int)(g0 % p.H);
  auto nxt = [](int sl, int n) { return sl + 1 == n ? 0 : sl + 1; };
  for (int k = 0; k < nrows; ++k) {
    dma::wait_vm_small(issued - gq[0]);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (k + D < nrows) issue_group(k + D);
    gq[D] = issued;
    {
      const char* Ds = dbase + ds0 * DB * 1024;
      const int xb = nxt(xs0, XS), xc = nxt(xb, XS);
      const int xsr = wr == 0 ? xs0 : (wr == 1 ? xb : xc);
      const char* Xs = (wr == 0 && y == 0) || (wr == 2 && y == p.H - 1) ? zrow : xbase + xsr * XB * 1024;
#pragma unroll
      for (int kk = 0; kk < TW / 16; ++kk) {
        uint4 af[FM];
#pragma unroll
        for (int i = 0; i < FM; ++i) {
          const int col = wm * 32 + i * 16 + li;
          f32x4 v;
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = *reinterpret_cast<const float*>(Ds + ffo<BM>(kk * 16 + 4 * e + g, col));
          af[i] = __builtin_bit_cast(uint4, v);
        }
#pragma unroll
        for (int s2 = 0; s2 < 3; ++s2) {
          uint4 bfr[FN];
#pragma unroll
          for (int j = 0; j < FN; ++j) {
            const int col = wn * (FN * 16) + j * 16 + li;
            f32x4 v;
#pragma unroll
            for (int e = 0; e < 4; ++e) v[e] = *reinterpret_cast<const float*>(Xs + ffo<BN>(kk * 16 + 4 * e + g + s2, col));
            bfr[j] = __builtin_bit_cast(uint4, v);
          }
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) Mma<float>::run(acc[s2][i][j], af[i], bfr[j]);
        }
      }
    }
    xs0 = nxt(xs0, XS);
    ds0 = nxt(ds0, DS);
    y = y + 1 == p.H ? 0 : y + 1;
#pragma unroll
    for (int q = 0; q < D; ++q) gq[q] = gq[q + 1];
  }

  float* __restrict__ O = p.out + (size_t)split * p.slab;
#pragma unroll
  for (int s2 = 0; s2 < 3; ++s2)
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int co = m0 + wm * 32 + i * 16 + g * 4 + rr;
        const int t = wr * 3 + s2;
#pragma unroll
        for (int j = 0; j < FN; ++j)
          O[(size_t)co * 9 * p.cin + t * p.cin + n0 + wn * (FN * 16) + j * 16 + li] = acc[s2][i][j][rr];
      }
}

// Rows per barrier step.  Timing-only builds of the 64 x 96 block (dec6-dec9; garbage
// results): no s_barrier -11 %, no vmcnt wait -11 %, no row DMA -15 %, none of the
// three -24 % (1.15 -> 1.5 PF/s: the MFMA + fragment-read loop alone); prefetching 4
// rows ahead instead of 2 changed nothing.  So the 64 x 96 block (one workgroup per CU
// at any ring size) multiplies two rows per wait + barrier with three groups ahead
// (152 KB).  Three rows per step would need three groups ahead (D >= R), 165 KB: over
// the LDS.  (profiles/r03g_ab_wgrad_rows.txt timed R3/D2, which violates D >= R: its
// third row read a slot not yet loaded; the parity tests caught it.)  The smaller
// blocks keep one row per step (two workgroups per CU).
#ifndef WH_ROWS96
#define WH_ROWS96 2
#endif
#ifndef WH_ROWS_SMALL
#define WH_ROWS_SMALL 1
#endif
#ifndef WH_ROWS64
#define WH_ROWS64 2
#endif
constexpr int wh_rows(int bm, int bn) {
  return bm == 64 && bn >= 96 ? WH_ROWS96 : (bm == 64 && bn == 64 ? WH_ROWS64 : WH_ROWS_SMALL);
}
// row groups issued ahead (64 x 128: two, the most that fits beside its 17 KB x rows).  For
// 64 x 96 two ahead is neutral (dec8 + dec9 11.38-11.40 vs 11.44-11.45 ms) and one row per
// step with two ahead 6 % slower (profiles/r04zz_wh96_ring_ab.txt)
#ifndef WH_AHEAD96
#define WH_AHEAD96 3
#endif
// the 32 x 32 block on 64-pixel strips (enc1b, HBM-bound): more row groups in flight
#ifndef WH_AHEAD_SMALL
#define WH_AHEAD_SMALL 2
#endif
constexpr int wh_ahead(int bm, int bn, int tw, int r) {
  return r > 1 ? (bn == 128 ? 2 : WH_AHEAD96) : (bm * bn <= 32 * 32 && tw == 64 ? WH_AHEAD_SMALL : 2);
}

// waves per kernel row (WM x WN over the BM x BN block).  64 x 128: 1 x 4 (each 64 x 32:
// fewer fragment reads per MFMA than 2 x 2, and 2 x 2's 32 x 64 tiles spilled at 168
// VGPRs).  32 x 32 (enc1b): one wave per kernel row over the whole block (1 x 2 read 10
// fragments per 6 MFMAs, 1 x 1 16 per 12): 2.14 -> 1.74 ms (profiles/r03zf_ab_enc1b_wn1.txt).
// 64 x 32 (enc2a): WH_WM6432 waves down the 64 output channels (1: 0.89 -> 0.91 ms,
// r03zg_ab_enc2a_wm1.txt, so 2).  More row groups in flight for the 32 x 32 block
// (WH_AHEAD_SMALL 4 / 6 on 64-pixel strips) measured no faster (r03ze_ab_enc1b_wgrad.txt).
#ifndef WH_WN32
#define WH_WN32 1
#endif
#ifndef WH_WM6432
#define WH_WM6432 2
#endif
constexpr int wh_wm(int bm, int bn) {
  return bn == 128 ? 1 : (bm * bn >= 64 * 64 ? 2 : (bm >= 64 ? (bn == 32 ? WH_WM6432 : 2) : 1));
}
constexpr int wh_wn(int bm, int bn) {
  return bn == 128 ? 4 : (bm * bn >= 64 * 64 ? 2 : (bm >= 64 ? 1 : (bm == 32 && bn == 32 ? WH_WN32 : 2)));
}

template <int BM, int BN, int TW>
int wh_occupancy() {  // resident workgroups per CU (registers AND LDS), from the runtime
  static int occ = [] {
    constexpr int WM = wh_wm(BM, BN), WN = wh_wn(BM, BN);
    constexpr int R = wh_rows(BM, BN), D = wh_ahead(BM, BN, TW, R);
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, (const void*)wgrad_halo_kernel<BM, BN, TW, WM, WN, D, R, false>,
                                                     3 * WM * WN * 64, 0) != hipSuccess || n < 1)
      n = 1;
    return n;
  }();
  return occ;
}

int wh_occupancy(int bm, int bn, int tw) {
#define WO(BMv, BNv, TWv) \
  if (bm == BMv && bn == BNv && tw == TWv) return wh_occupancy<BMv, BNv, TWv>();
  WO(64, 128, 64) WO(64, 96, 64) WO(64, 64, 64) WO(64, 32, 64) WO(32, 96, 64) WO(32, 64, 64) WO(32, 32, 64)
  WO(64, 32, 128) WO(32, 64, 128) WO(32, 32, 128)
#undef WO
  return 1;
}

struct WHPlan {
  int bm, bn, tw, strips, cbm, cbn, rsplits, smem;
  long rows_per;
  bool split;  // cin 192: a 128-column launch and a 64-column launch instead of two 96-column blocks
};

bool wh_plan(int n, int h, int w, int cin, int cout, WHPlan& pl, bool cat = false) {
  pl.bm = cout % 64 == 0 ? 64 : (cout == 32 ? 32 : 0);
  pl.bn = cin % 96 == 0 ? 96 : (cin % 64 == 0 ? 64 : (cin % 32 == 0 ? 32 : 0));
  if (!cat && cout % 64 == 0 && cin % 128 == 0) pl.bn = 128;
  pl.split = !cat && cin == 192 && cout % 64 == 0;
  if (pl.split) pl.bn = 128;  // (the planner below sizes the 128-column launch; the 64 one follows it)
  if (!pl.bm || !pl.bn) return false;
  // 128-column strips also when w % 128 != 0 (a partial last strip): enc2a at 960
  // columns 1.12 -> 0.99 ms
  pl.tw = (pl.bm * pl.bn <= 32 * 64 && w % 64 == 0) ? 128 : 64;
  pl.strips = (w + pl.tw - 1) / pl.tw;  // a partial last strip reads zero columns
  pl.cbm = cout / pl.bm;
  pl.cbn = pl.split ? 1 : cin / pl.bn;
  const long rows = (long)n * h;
  const long per = (long)pl.strips * pl.cbm * pl.cbn;
  // whole rounds of resident workgroups: slots = CUs x workgroups per CU (LDS- or
  // register-limited); pick the row split with the least idle tail (fewest splits on ties)
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      ncu = prop.multiProcessorCount;
    if (ncu <= 0) ncu = 256;
  }
  if (cat && !(pl.bn == 96 && cin == 96 && pl.tw == 64)) return false;  // CAT: the [32 | 64] block only
  const int xb = cat ? ((pl.tw + 2) * 64 + 1023) / 1024 + ((pl.tw + 2) * (pl.bn - 32) * 2 + 1023) / 1024
                     : ((pl.tw + 2) * pl.bn * 2 + 1023) / 1024,
            db = pl.tw * pl.bm * 2 / 1024;
  const int R = wh_rows(pl.bm, pl.bn), D = wh_ahead(pl.bm, pl.bn, pl.tw, R);
  const int smem = ((D + R + 3) * xb + (D + R) * db) * 1024;  // WHCfg::SMEM
#ifndef WH_OCC_API
#define WH_OCC_API 1
#endif
  // workgroups per CU: the runtime's occupancy (the 64 x 64 block fits two by LDS but
  // one by registers: 12 waves at 114 VGPRs)
  const int occ = WH_OCC_API && !cat ? wh_occupancy(pl.bm, pl.bn, pl.tw) : std::max(1, (160 * 1024) / smem);
  const long slots = (long)ncu * occ;
  long best = 1;
  double best_eff = -1.0;
  for (long rs = 1; rs <= 64 && rs <= rows; ++rs) {
    const long blocks = per * rs;
    const long rounds = (blocks + slots - 1) / slots;
    double eff = (double)blocks / (double)(rounds * slots);
    if (blocks < slots / 2) eff *= 0.5;  // too few workgroups to fill the chip
    if (eff > best_eff + 1e-3) { best_eff = eff; best = rs; }
  }
  pl.rows_per = (rows + best - 1) / best;
  pl.rsplits = (int)((rows + pl.rows_per - 1) / pl.rows_per);
  return true;
}

template <int BM, int BN, int TW, bool CAT = false>
void wh_launch(const WHArgs& a, unsigned grid, hipStream_t s) {
  // 12 waves (3 per SIMD) for the big blocks, 6 (or 3) for the small ones
  constexpr int WM = wh_wm(BM, BN), WN = wh_wn(BM, BN);
  constexpr int R = wh_rows(BM, BN), D = wh_ahead(BM, BN, TW, R);
  hipLaunchKernelGGL((wgrad_halo_kernel<BM, BN, TW, WM, WN, D, R, CAT>), dim3(grid), dim3(3 * WM * WN * 64), 0, s,
                     a);
}

// fp32 plan: 32 / 64 x 32 / 64 blocks (64 x 96 for cin 96), 64-pixel strips, the row split of
// wh_plan's policy
bool wh_plan_f32(int n, int h, int w, int cin, int cout, WHPlan& pl) {
  pl.bm = cout % 64 == 0 ? 64 : (cout % 32 == 0 ? 32 : 0);
  pl.bn = cin % 64 == 0 ? 64 : (cin % 32 == 0 ? 32 : 0);
  if (WF_BN96 && pl.bm == 64 && cin % 96 == 0 && cin % 64 != 0) pl.bn = 96;
  if (!pl.bm || !pl.bn) return false;
  pl.tw = 64;
  pl.strips = (w + pl.tw - 1) / pl.tw;
  pl.cbm = cout / pl.bm;
  pl.cbn = cin / pl.bn;
  const long rows = (long)n * h;
  const long per = (long)pl.strips * pl.cbm * pl.cbn;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      ncu = prop.multiProcessorCount;
    if (ncu <= 0) ncu = 256;
  }
  const int xb = (66 * pl.bn * 4 + 1023) / 1024, db = 64 * pl.bm * 4 / 1024;
  const int d = wf_ahead(pl.bm, pl.bn);
  const int smem = ((d + 4) * xb + (d + 1) * db) * 1024;  // WF32Cfg::SMEM (R = 1)
  const long slots = (long)ncu * std::max(1, (160 * 1024) / smem);
  long best = 1;
  double best_eff = -1.0;
  for (long r = 1; r <= 64 && r <= rows; ++r) {
    const long blocks = per * r;
    const long rounds = (blocks + slots - 1) / slots;
    double eff = (double)blocks / (double)(rounds * slots);
    if (blocks < slots / 2) eff *= 0.5;
    if (eff > best_eff + 1e-3) { best_eff = eff; best = r; }
  }
  pl.rows_per = (rows + best - 1) / best;
  pl.rsplits = (int)((rows + pl.rows_per - 1) / pl.rows_per);
  return true;
}

}  // namespace

size_t wgrad_halo_ws_bytes(int n, int h, int w, int cin, int cout, bool cat) {
  WHPlan pl;
  if (!wh_plan(n, h, w, cin, cout, pl, cat)) return 0;
  return (size_t)pl.strips * pl.rsplits * cout * 9 * cin * 4;
}

// Returns the number of slabs written (>0) or -1 when this path does not apply.
// x2 != null: the input channels [32, cin) come from x2 (CAT; see WHCfg).
int launch_wgrad_halo(const bf16* x, long x_ld, int x_off, const bf16* dz, int n, int h, int w, int cin,
                      int cout, float* ws, size_t ws_bytes, hipStream_t s, const bf16* x2, long x2_ld,
                      int x2_off) {
  WHPlan pl;
  const bool cat = x2 != nullptr;
  if (!wh_plan(n, h, w, cin, cout, pl, cat)) return -1;
  if (x_ld % 8 || x_off % 8 || (cat && (x2_ld % 8 || x2_off % 8))) return -1;
  const size_t need = (size_t)pl.strips * pl.rsplits * cout * 9 * cin * 4;
  if (!ws || ws_bytes < need) return -1;
  WHArgs a;
  memset(&a, 0, sizeof(a));
  a.dz = dz; a.cout = cout; a.x = x; a.x_ld = x_ld; a.x_off = x_off;
  a.x2 = x2; a.x2_ld = x2_ld; a.x2_off = x2_off;
  a.nimg = n; a.H = h; a.W = w; a.cin = cin;
  a.out = ws; a.slab = (long)cout * 9 * cin;
  a.strips = pl.strips; a.cbm = pl.cbm; a.cbn = pl.cbn; a.rsplits = pl.rsplits; a.rows_per = pl.rows_per;
  const unsigned grid = (unsigned)(pl.strips * pl.cbm * pl.cbn * pl.rsplits);
  if (pl.split) {  // channels [0, 128) on 64 x 128 blocks, [128, 192) on 64 x 64 blocks; the same slabs
    wh_launch<64, 128, 64>(a, grid, s);
    a.cbase = 128;
    wh_launch<64, 64, 64>(a, grid, s);
    return pl.strips * pl.rsplits;
  }
  if (cat) {
    if (pl.bm == 64) wh_launch<64, 96, 64, true>(a, grid, s);
    else wh_launch<32, 96, 64, true>(a, grid, s);
    return pl.strips * pl.rsplits;
  }
#define WH(BMv, BNv, TWv) \
  if (pl.bm == BMv && pl.bn == BNv && pl.tw == TWv) { wh_launch<BMv, BNv, TWv>(a, grid, s); return pl.strips * pl.rsplits; }
  WH(64, 128, 64) WH(64, 96, 64) WH(64, 64, 64) WH(64, 32, 64) WH(32, 96, 64) WH(32, 64, 64) WH(32, 32, 64)
  WH(64, 32, 128) WH(32, 64, 128) WH(32, 32, 128)
#undef WH
  return -1;
}

// kernel label for profiles ("" when this path does not apply)
const char* wgrad_halo_name(int n, int h, int w, int cin, int cout, bool cat) {
  WHPlan pl;
  if (!wh_plan(n, h, w, cin, cout, pl, cat)) return "";
  static thread_local char buf[64];
  if (pl.split)
    snprintf(buf, sizeof(buf), "wgrad_halo_kernel<%d,128+64,%d>", pl.bm, pl.tw);
  else
    snprintf(buf, sizeof(buf), "wgrad_halo_kernel<%d,%d,%d%s>", pl.bm, pl.bn, pl.tw, cat ? ",cat" : "");
  return buf;
}

// fp32: returns the slabs written (> 0) or -1 when this path does not apply.
int launch_wgrad_halo_f32(const float* x, long x_ld, int x_off, const float* dz, int n, int h, int w, int cin,
                          int cout, float* ws, size_t ws_bytes, hipStream_t s) {
  WHPlan pl;
  if (!wh_plan_f32(n, h, w, cin, cout, pl)) return -1;
  if (x_ld % 4 || x_off % 4) return -1;
  const size_t need = (size_t)pl.strips * pl.rsplits * cout * 9 * cin * 4;
  if (!ws || ws_bytes < need) return -1;
  WHArgs a;
  memset(&a, 0, sizeof(a));
  a.dz = (const bf16*)dz; a.cout = cout; a.x = (const bf16*)x; a.x_ld = x_ld; a.x_off = x_off;
  a.nimg = n; a.H = h; a.W = w; a.cin = cin;
  a.out = ws; a.slab = (long)cout * 9 * cin;
  a.strips = pl.strips; a.cbm = pl.cbm; a.cbn = pl.cbn; a.rsplits = pl.rsplits; a.rows_per = pl.rows_per;
  const unsigned grid = (unsigned)(pl.strips * pl.cbm * pl.cbn * pl.rsplits);
#define WF(BMv, BNv)                                                                                        \
  if (pl.bm == BMv && pl.bn == BNv) {                                                                    \
    hipLaunchKernelGGL((wgrad_halo_f32_kernel<BMv, BNv>), dim3(grid), dim3(WF32Cfg<BMv, BNv>::NT), 0, s, a); \
    return pl.strips * pl.rsplits;                                                                       \
  }
  WF(64, 64) WF(64, 32) WF(32, 64) WF(32, 32)
#if WF_BN96
  WF(64, 96)
#endif
#undef WF
  return -1;
}

size_t wgrad_halo_f32_ws_bytes(int n, int h, int w, int cin, int cout) {
  WHPlan pl;
  if (!wh_plan_f32(n, h, w, cin, cout, pl)) return 0;
  return (size_t)pl.strips * pl.rsplits * cout * 9 * cin * 4;
}

const char* wgrad_halo_f32_name(int n, int h, int w, int cin, int cout) {
  WHPlan pl;
  if (!wh_plan_f32(n, h, w, cin, cout, pl)) return "";
  static thread_local char buf[64];
  snprintf(buf, sizeof(buf), "wgrad_halo_kernel<f32,%d,%d,64>", pl.bm, pl.bn);
  return buf;
}
