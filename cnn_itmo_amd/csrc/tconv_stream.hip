// Conv2DTranspose(2, strides=2) forward and input-gradient (model.py
// ConvBNTranspose: up6..up9) as streamed GEMMs with the weight block RESIDENT in
// LDS.  Both are HBM-bound (K = cin or 4*cout <= 2048, one pass over the
// activations), so the kernel is built to stream:
//   * a persistent workgroup per CU owns ONE column block (nb) of the GEMM for
//     its whole life: its weight block (K x BN bf16 <= 64 KB) is DMA'd once,
//   * the activations stream through an LDS-DMA ring (64-pixel tiles x 128-deep
//     K chunks, 16 KB per stage), each byte read from HBM once per column block,
//   * the MFMA runs with the operands swapped (C^T = W^T A^T), so a lane ends up
//     with output channels of one pixel and stores them straight from registers
//     (the weight rows in pair_perm order: 8 consecutive channels, one 16-byte
//     buffer store; out-of-range pixels dropped by the range check): no LDS
//     staging, no barrier in the epilogue.
// MODE 0 (forward): A = x [P][cin] (a row per input pixel), B = k [4*cout][cin];
//   GEMM column n = tap*cout + co is scattered to output pixel (2y+a, 2x+b).
//   Epilogue: bias (per column), ReLU, inference affine, BN partial sums.
// MODE 1 (input gradient): A row of output pixel (y, x) = the four dout pixels
//   (2y+a, 2x+b) x cout (K = tap*cout + co), B = kT [cin][4*cout].
//   EPI: the producer's BN backward fused into the store (as the conv3x3 dgrad's
//   halo EPI 1): dz = [r>0]*(a*g - b*r + e) of the bf16-rounded g, r DMA'd with
//   the tile's last chunk, plus column sums of dz.
#include <algorithm>
#include <cstdio>

#include "dma.h"
#include "igemm_common.h"

namespace {

#pragma clang diagnostic ignored "-Winline-asm"
using dma::i32x4;
typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4_ __attribute__((ext_vector_type(4)));
using dma::OOB;  // voffset beyond num_records: load zeros / drop store

__device__ __forceinline__ __amdgpu_buffer_rsrc_t srsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, 0x7FFFFFF0, 0x00020000);
}
// sum over the 16 lanes of each DPP row (lanes = pixels of a fragment): xor 1, xor 2
// (quad_perm), then half-row and row mirrors; 4 VALU ops, no LDS crossbar traffic
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}
// 64-byte LDS rows, 16-byte piece c of row q at c ^ (((q >> 2) & 1) << 1): every
// ds_read_b128 fragment window (16 consecutive rows) is conflict-free
// (tools/check_swizzle.py, the halo kernel's image).
__device__ __forceinline__ int rsw(int row, int piece) { return (row << 6) + ((piece ^ (((row >> 2) & 1) << 1)) << 4); }

struct TSArgs {
  const bf16* a;   // MODE 0: x view base (+a_off), row stride a_ld; MODE 1: dout [n][2h][2w][cout]
  long a_ld;
  int a_off;
  const bf16* b;   // [N][K]
  int nimg, h, w;  // the small grid (tconv input / input-gradient)
  int cout;        // layer output channels
  int K, N, nblocks, tiles_x;
  long ntiles;     // nimg * h * tiles_x
  bf16* out;       // MODE 0: [n][2h][2w] x out_ld (+out_off); MODE 1: [P] x out_ld (+out_off)
  long out_ld;
  int out_off;
  const float* bias;  // MODE 0, per GEMM column (CNNITMO_BIAS_PER_COL) or per co
  int flags;
  const float* aff_scale;
  const float* aff_shift;
  float* stats;  // MODE 0: [G*WM][2][N]; MODE 1 EPI: [G*WM][N] sums of dz (G = gridDim / nblocks)
  const float* coef;  // MODE 1 EPI: [3][N]
  const bf16* r;
  long r_ld;
  int r_off;
};

template <int MODE, int BN, int ST, bool EPI>
struct TSCfg {
  static constexpr int NT = 512, BM = 64, KC = 128;
  // 8 waves: WM (pixels) x WN (columns), every wave owning >= 32 columns (a pair of
  // fragments, for the 16-byte stores): BN 256/128: 2 x 4, BN 64: 4 x 2
  static constexpr int WN = BN >= 128 ? 4 : BN / 32, WM = 8 / WN;
  static constexpr int FM = BM / 16 / WM, FN = BN / WN / 16;  // wave tile 16*FM px x 16*FN columns
  static constexpr int STAGE = BM * KC * 2;           // 16 KB
  static constexpr int RSLOT = EPI ? BM * BN * 2 : 0;
  static constexpr int PAR = 3 * BN * 4;
  static constexpr int BRES = 64 * 1024;
  static constexpr int SMEM = BRES + PAR + ST * STAGE + 2 * RSLOT;
  static_assert(SMEM <= 160 * 1024, "LDS");
};

template <int MODE, int BN, int ST, bool EPI>
__global__ __launch_bounds__(512) void tconv_stream_kernel(const TSArgs p) {
  using C = TSCfg<MODE, BN, ST, EPI>;
  constexpr int FM = C::FM, FN = C::FN, STAGE = C::STAGE;
  constexpr int PPR = BN / 8;  // 16-byte pieces per R row
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  char* const Bres = smem;
  float* const par = reinterpret_cast<float*>(smem + C::BRES);
  char* const ring = smem + C::BRES + C::PAR;
  char* const rr = ring + ST * STAGE;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  constexpr int WN = C::WN;
  const int wm = wave / WN, wn = wave % WN;  // (rows of the stats / sums: WM per tile)
  // XCD-aware: workgroups are dealt to the 8 XCDs round-robin (b % 8); the
  // column blocks of one tile range live on the SAME XCD, so the re-reads of an
  // A tile by the other column blocks hit that XCD's L2
  const int G = gridDim.x / p.nblocks;
  const int xcd = blockIdx.x & 7, wi = blockIdx.x >> 3, per_xcd = gridDim.x >> 3;
  const int lid = xcd * per_xcd + wi;  // consecutive lids share an XCD
  const int nb = lid % p.nblocks, g = lid / p.nblocks;
  const long per = (p.ntiles + G - 1) / G;
  const long t0 = (long)g * per, t1 = t0 + per < p.ntiles ? t0 + per : p.ntiles;
  if (t0 >= t1) {  // no tiles: this group's partial-sum rows are zero
    const bool st = MODE == 0 ? (p.flags & CNNITMO_STATS) != 0 : EPI;
    const int wm = wave / C::WN;
    const long row = (long)g * C::WM + wm;
    const int cols = (MODE == 0 ? 2 : 1) * p.N;
    if (st && lid % p.nblocks == 0)  // one workgroup per group: the rows span all N columns
      for (int i = (wave % C::WN) * 64 + lane; i < cols; i += C::WN * 64) p.stats[(size_t)row * cols + i] = 0.f;
    return;
  }
  const int K = p.K, nch = K / C::KC, n0 = nb * BN;

  // ---- resident weight block + per-column parameters (once) -------------------
  {
    const int rows = K / 32 * BN;  // 64-byte rows: row = kstep * BN + n
    const i32x4 rs = dma::rsrc((uintptr_t)(p.b + (size_t)n0 * K));
    for (int q = wave; q < rows / 16; q += 8) {
      const int row = q * 16 + (lane >> 2), piece = (lane & 3) ^ (((row >> 2) & 1) << 1);
      const int ks = row / BN, n = pair_perm(row - ks * BN);  // (16-byte stores: see the epilogue)
      dma::lds16((unsigned)((n * K + ks * 32 + piece * 8) * 2), rs, Bres + q * 1024);
    }
    for (int c = tid; c < BN; c += C::NT) {
      const int n = n0 + c;
      if constexpr (MODE == 0) {
        const int co = n % p.cout;
        par[c] = p.bias ? p.bias[(p.flags & CNNITMO_BIAS_PER_COL) ? n : co] : 0.f;
        par[BN + c] = (p.flags & CNNITMO_AFFINE) ? p.aff_scale[co] : 1.f;
        par[2 * BN + c] = (p.flags & CNNITMO_AFFINE) ? p.aff_shift[co] : 0.f;
      } else if constexpr (EPI) {
        par[c] = p.coef[n];
        par[BN + c] = p.coef[p.N + n];
        par[2 * BN + c] = p.coef[2 * p.N + n];
      }
    }
    dma::wait_vm<0>();
    __syncthreads();
  }

  // ---- per-lane DMA geometry of a 16 KB A stage: 16 instructions, 2 per wave ----
  // stage row = ks * 64 + px (ks = 32-deep K step within the chunk)
  int apx[2], aks[2], apc[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = (wave * 2 + i) * 16 + (lane >> 2);
    aks[i] = row >> 6;
    apx[i] = row & 63;
    apc[i] = (lane & 3) ^ (((row >> 2) & 1) << 1);
  }
  // Item positions advance incrementally (one item = (tile, chunk); tiles are consecutive,
  // image -> row -> 64-pixel strip): the 64-bit divisions of a per-item tile_pos were ~250
  // scalar instructions per item, issued in front of every stage's DMA.
  struct It {
    int kc, tl, tx, y, img;  // chunk, tile (relative to t0), strip, row, image
    int tap[2], co[2];       // MODE 1: the K step of each of the wave's two DMA rows (its tap, channel)
  };
  auto it_init = [&](It& s) {
    const int tx = (int)(t0 % p.tiles_x);
    const long ry = t0 / p.tiles_x;
    s.kc = 0;
    s.tl = 0;
    s.tx = tx;
    s.y = (int)(ry % p.h);
    s.img = (int)(ry / p.h);
#pragma unroll
    for (int i = 0; i < 2; ++i) {  // k = kc * 128 + aks * 32 (wave-uniform: aks is the row's 64-block)
      const int k = __builtin_amdgcn_readfirstlane(aks[i] * 32);
      s.tap[i] = MODE == 1 ? k / p.cout : 0;
      s.co[i] = MODE == 1 ? k - s.tap[i] * p.cout : 0;
    }
  };
  auto it_next = [&](It& s) {
    if (++s.kc < nch) {
      if constexpr (MODE == 1) {
#pragma unroll
        for (int i = 0; i < 2; ++i) {  // k += 128 (cout % 32 == 0)
          s.co[i] += 128;
          while (s.co[i] >= p.cout) {
            s.co[i] -= p.cout;
            ++s.tap[i];
          }
        }
      }
      return;
    }
    s.kc = 0;
    if constexpr (MODE == 1) {
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int k = __builtin_amdgcn_readfirstlane(aks[i] * 32);
        s.tap[i] = k / p.cout;
        s.co[i] = k - s.tap[i] * p.cout;
      }
    }
    ++s.tl;
    if (++s.tx < p.tiles_x) return;
    s.tx = 0;
    if (++s.y < p.h) return;
    s.y = 0;
    ++s.img;
  };
  const int W2 = 2 * p.w;

  // the next item (tile, chunk) of the ring; loads: A chunk (+ R tile with the last chunk, EPI)
  It iss;
  it_init(iss);
  auto issue = [&](int slot) -> int {
    const int kc = iss.kc, img = iss.img, y = iss.y, x0 = iss.tx * 64;
    char* S = ring + slot * STAGE;
    if constexpr (MODE == 0) {
      const i32x4 rs = dma::rsrc((uintptr_t)(p.a + (((size_t)img * p.h + y) * p.w + x0) * p.a_ld + p.a_off + kc * 128));
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const bool ok = x0 + apx[i] < p.w;
        dma::lds16(ok ? (unsigned)((apx[i] * p.a_ld + aks[i] * 32 + apc[i] * 8) * 2) : OOB, rs, S + (wave * 2 + i) * 1024);
      }
    } else {
      const i32x4 rs = dma::rsrc((uintptr_t)(p.a + (((size_t)img * 2 * p.h + 2 * y) * W2 + 2 * x0) * p.cout));
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int tap = iss.tap[i], co = iss.co[i];  // 32 | cout: the step lies in one tap
        const bool ok = x0 + apx[i] < p.w;
        const unsigned off = (unsigned)((((tap >> 1) * W2 + 2 * apx[i] + (tap & 1)) * p.cout + co + apc[i] * 8) * 2);
        dma::lds16(ok ? off : OOB, rs, S + (wave * 2 + i) * 1024);
      }
    }
    int n = 2;
    if constexpr (EPI) {
      if (kc == nch - 1) {  // the producer's r tile [64 px][BN] for the fused BN backward
        char* R = rr + (iss.tl & 1) * C::RSLOT;
        const i32x4 rs = dma::rsrc((uintptr_t)(p.r + (((size_t)img * p.h + y) * p.w + x0) * p.r_ld + p.r_off + n0));
        for (int j = wave; j < 64 * PPR / 64; j += 8) {  // 1 KB instructions
          const int slot16 = j * 64 + lane, px = slot16 / PPR, sl = slot16 - px * PPR;
          const int pc = sl ^ (px & (PPR - 1));  // piece swizzle by pixel
          const bool ok = x0 + px < p.w;
          dma::lds16(ok ? (unsigned)((px * p.r_ld + pc * 8) * 2) : OOB, rs, R + j * 1024);
        }
        n += (64 * PPR / 64 + 7 - wave) / 8;
      }
    }
    it_next(iss);
    return n;
  };

  f32x4 acc[FM][FN];
  auto zero = [&]() {
#pragma unroll
    for (int f = 0; f < FM; ++f)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero();

  auto compute = [&](int slot, int kc) {
    const char* S = ring + slot * STAGE;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      uint4 af[FM], bfr[FN];
#pragma unroll
      for (int f = 0; f < FM; ++f)
        af[f] = *reinterpret_cast<const uint4*>(S + rsw(ks * 64 + wm * (16 * FM) + f * 16 + (lane & 15), lane >> 4));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const uint4*>(
            Bres + rsw((kc * 4 + ks) * BN + wn * (BN / WN) + j * 16 + (lane & 15), lane >> 4));
#pragma unroll
      for (int f = 0; f < FM; ++f)
#pragma unroll
        for (int j = 0; j < FN; ++j) Mma<bf16>::run(acc[f][j], bfr[j], af[f]);  // C^T: lanes = pixels
    }
  };

  const bool relu = p.flags & CNNITMO_RELU, aff = p.flags & CNNITMO_AFFINE, stats = p.flags & CNNITMO_STATS;
  // Epilogue straight from the accumulators.  The resident weight rows are in pair_perm
  // order, so fragments (2jp, 2jp+1) give a lane 8 CONSECUTIVE columns c .. c+7 of its
  // pixel: one 16-byte store per (pixel, pair).
  // stores per tile epilogue (all issued, out-of-range ones dropped): FM*FP outputs
  // + MODE 0 stats 4*FP (lanes 0/16/32/48) + EPI sums 2*FP
  constexpr int FP = FN / 2;
  static_assert(FN % 2 == 0, "column pairs");
  constexpr int SOUT = FM * FP;
  const int S = SOUT;
  typedef float f32x8_ __attribute__((ext_vector_type(8)));
  // BN partial sums of the lane's pixels, kept in registers for the whole launch (the
  // workgroup's columns never change): one row per (workgroup group, wave row) at the
  // end instead of one per tile (up9: 1 GB of fp32 partials per step before)
  float s1[FP][8], s2[FP][8];
#pragma unroll
  for (int j = 0; j < FP; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) s1[j][k] = s2[j][k] = 0.f;
  auto epilogue = [&](const It& e, int rslot) {
    const int img = e.img, y = e.y, x0 = e.tx * 64;
    if constexpr (MODE == 0) {
      const __amdgpu_buffer_rsrc_t os =
          srsrc(p.out + (((size_t)img * 2 * p.h + 2 * y) * W2 + 2 * x0) * p.out_ld + p.out_off);
#pragma unroll
      for (int jp = 0; jp < FP; ++jp) {
        const int c = wn * (BN / WN) + jp * 32 + (lane >> 4) * 8;  // first of this lane's 8 columns
        const int n = n0 + c, tap = n / p.cout, co = n - tap * p.cout;  // (8 | cout: one tap)
        const f32x8_ bj = *reinterpret_cast<const f32x8_*>(par + c);
        const f32x8_ sj = *reinterpret_cast<const f32x8_*>(par + BN + c);
        const f32x8_ hj = *reinterpret_cast<const f32x8_*>(par + 2 * BN + c);
#pragma unroll
        for (int f = 0; f < FM; ++f) {
          const int px = wm * (16 * FM) + f * 16 + (lane & 15);
          const bool ok = x0 + px < p.w;
          bf16x8 o;
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            float v = acc[f][2 * jp + (k >> 2)][k & 3] + bj[k];
            if (relu) v = fmaxf(v, 0.f);
            if (aff) v = fmaf(v, sj[k], hj[k]);
            const float vs = ok ? v : 0.f;
            s1[jp][k] += vs;
            s2[jp][k] += vs * vs;
            o[k] = from_f32<bf16>(v);
          }
          const unsigned off = (unsigned)((((tap >> 1) * W2 + 2 * px + (tap & 1)) * p.out_ld + co) * 2);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, o), os, ok ? off : OOB, 0, 0);
        }
      }
    } else {
      const __amdgpu_buffer_rsrc_t os = srsrc(p.out + (((size_t)img * p.h + y) * p.w + x0) * p.out_ld + p.out_off);
      const char* R = rr + rslot * C::RSLOT;
#pragma unroll
      for (int jp = 0; jp < FP; ++jp) {
        const int c = wn * (BN / WN) + jp * 32 + (lane >> 4) * 8;
        f32x8_ ca = {}, cb = {}, ce = {};
        if constexpr (EPI) {
          ca = *reinterpret_cast<const f32x8_*>(par + c);
          cb = *reinterpret_cast<const f32x8_*>(par + BN + c);
          ce = *reinterpret_cast<const f32x8_*>(par + 2 * BN + c);
        }
#pragma unroll
        for (int f = 0; f < FM; ++f) {
          const int px = wm * (16 * FM) + f * 16 + (lane & 15);
          const bool ok = x0 + px < p.w;
          bf16x8 o;
          if constexpr (EPI) {
            // r[px][c..c+7]: piece c/8 of row px, stored at piece (c/8) ^ (px & (PPR-1))
            const bf16x8 rq = *reinterpret_cast<const bf16x8*>(R + (px * PPR + ((c >> 3) ^ (px & (PPR - 1)))) * 16);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float gg = to_f32(from_f32<bf16>(acc[f][2 * jp + (k >> 2)][k & 3])), rvv = to_f32(rq[k]);
              o[k] = from_f32<bf16>(rvv > 0.f ? ca[k] * gg - cb[k] * rvv + ce[k] : 0.f);
              s1[jp][k] += ok ? to_f32(o[k]) : 0.f;
            }
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] = from_f32<bf16>(acc[f][2 * jp + (k >> 2)][k & 3]);
          }
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, o), os,
                                                 ok ? (unsigned)((px * p.out_ld + n0 + c) * 2) : OOB, 0, 0);
        }
      }
    }
    zero();
  };

  // ---- ST-stage ring over items (tile, chunk); vmcnt counted per wave as in the
  // halo kernel: retire in issue order, stores included
  const long T = (t1 - t0) * nch;
  int issued = 0;
  int mq[ST];
#pragma unroll
  for (int k = 0; k < ST - 1; ++k) {
    if (k < T) issued += issue(k);
    mq[k] = issued;
  }
  mq[ST - 1] = issued;
  int slot = 0;
  It cur;  // the item being computed
  it_init(cur);
  for (long q = 0; q < T; ++q) {
    // younger than this item's pieces: the next ST - 2 items' two pieces each, plus around a
    // tile's end its r pieces and epilogue stores; waiting down to 2 (ST - 2) then also retires
    // those r pieces, issued an item or more ago (a two-way wait instead of the switch)
    dma::wait_vm_ge<2 * (ST - 2)>(issued - mq[0]);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (q + ST - 1 < T) {
      issued += issue(slot == 0 ? ST - 1 : slot - 1);
      mq[ST - 1] = issued;
    }
    const int kc = cur.kc;
    compute(slot, kc);
    if (kc == nch - 1) {
      epilogue(cur, cur.tl & 1);
      issued += S;
    }
    it_next(cur);
#pragma unroll
    for (int k = 0; k < ST - 1; ++k) mq[k] = mq[k + 1];
    slot = slot == ST - 1 ? 0 : slot + 1;
  }
  // the launch's partial sums: row (g, wm), the 16 pixel lanes of each fragment folded
  if ((MODE == 0 && stats) || (MODE == 1 && EPI)) {
    const long row = (long)g * C::WM + wm;
    const __amdgpu_buffer_rsrc_t ss = srsrc(p.stats + (size_t)row * (MODE == 0 ? 2 : 1) * p.N);
#pragma unroll
    for (int jp = 0; jp < FP; ++jp) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s1[jp][k] = row16_sum(s1[jp][k]);
        if (MODE == 0) s2[jp][k] = row16_sum(s2[jp][k]);
      }
      const int n = n0 + wn * (BN / WN) + jp * 32 + (lane >> 4) * 8;
      const bool w0 = (lane & 15) == 0;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4_ a1 = {s1[jp][4 * h], s1[jp][4 * h + 1], s1[jp][4 * h + 2], s1[jp][4 * h + 3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, a1), ss, w0 ? (unsigned)((n + 4 * h) * 4) : OOB,
                                               0, 0);
        if (MODE == 0) {
          const f32x4_ a2 = {s2[jp][4 * h], s2[jp][4 * h + 1], s2[jp][4 * h + 2], s2[jp][4 * h + 3]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i32x4, a2), ss,
                                                 w0 ? (unsigned)((p.N + n + 4 * h) * 4) : OOB, 0, 0);
        }
      }
    }
  }
}

struct TSPlan {
  int bn, st;
  bool epi;
};

bool ts_plan(int mode, int h, int w, int cin, int cout, bool epi, TSPlan& pl) {
  if (w < 1 || h < 1) return false;
  const int K = mode == 0 ? cin : 4 * cout, N = mode == 0 ? 4 * cout : cin;
  if (K % 128 || cout % 32 || N % 64) return false;
  int bn = 64 * 1024 / (K * 2);  // the resident weight block: K x BN bf16 <= 64 KB
  bn = bn >= 256 ? 256 : (bn >= 128 ? 128 : (bn >= 64 ? 64 : 0));
  while (bn > 64 && N % bn) bn /= 2;
  if (!bn || N % bn) return false;
  if (epi && bn > 128) bn = 128;  // LDS: two r slots of 64 x BN
  // one column block only: with several, every block streams all of A again and
  // the per-CU LDS-DMA rate (not HBM) becomes the bound: up6 / up7 / up8 forward
  // 2.51 / 4.93 / 3.03 ms against tconv_ws's 0.83 / 1.72 / 2.40
  // (profiles/r03i_ab_tconv_stream_multiblock.txt)
  if (N != bn) return false;
  pl.bn = bn;
  pl.epi = epi;
  if (epi) {
    if (mode != 1) return false;
    // the R slot of tile t is refilled with tile t+2's last chunk: 2 * chunks >= ST
    const int nch = K / 128;
    pl.st = bn == 64 ? 4 : 3;
    while (pl.st > 2 && 2 * nch < pl.st) --pl.st;
    if (2 * nch < pl.st) return false;
  } else {
    pl.st = 5;
  }
  return true;
}

template <int MODE, int BN, int ST, bool EPI>
void ts_launch(const TSArgs& a, int grid, hipStream_t s) {
  hipLaunchKernelGGL((tconv_stream_kernel<MODE, BN, ST, EPI>), dim3(grid), dim3(512), 0, s, a);
}

int num_cus() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      ncu = prop.multiProcessorCount;
    if (ncu <= 0) ncu = 256;
  }
  return ncu;
}

}  // namespace

bool tconv_stream_handles(int mode, int h, int w, int cin, int cout, bool epi) {
  TSPlan pl;
  return ts_plan(mode, h, w, cin, cout, epi, pl);
}

// launch grid: 8 | grid and nblocks | grid / 8 (XCD-aware mapping in the kernel)
int ts_grid(int nblocks) { return 8 * std::max(nblocks, num_cus() / 8 / nblocks * nblocks); }

long tconv_stream_rows(int mode, int n, int h, int w, int cin, int cout, bool epi) {
  TSPlan pl;
  if (!ts_plan(mode, h, w, cin, cout, epi, pl)) return 0;
  const int wm = pl.bn >= 128 ? 2 : 8 / (pl.bn / 32);  // TSCfg::WM: one row per (workgroup group, wave row)
  const int nblocks = (mode == 0 ? 4 * cout : cin) / pl.bn;
  return (long)ts_grid(nblocks) / nblocks * wm;
}

const char* tconv_stream_name(int mode, int h, int w, int cin, int cout, bool epi) {
  TSPlan pl;
  if (!ts_plan(mode, h, w, cin, cout, epi, pl)) return "";
  static thread_local char buf[64];
  snprintf(buf, sizeof(buf), "tconv_stream_kernel<%d,%d%s>", mode, pl.bn, pl.epi ? ",bnb" : "");
  return buf;
}

// mode 0: x [n][h][w] view (x_ld, x_off) -> out [n][2h][2w] view; mode 1: dout -> dx view.
int launch_tconv_stream(int mode, const void* a, long a_ld, int a_off, const void* b, int n, int h, int w,
                        int cin, int cout, void* out, long out_ld, int out_off, const float* bias, int flags,
                        const float* aff_scale, const float* aff_shift, float* stats, const float* coef,
                        const void* r, long r_ld, int r_off, hipStream_t s, const char* what) {
  TSPlan pl;
  const bool epi = coef != nullptr;
  CNN_REQUIRE(ts_plan(mode, h, w, cin, cout, epi, pl), "%s: no stream plan", what);
  CNN_REQUIRE(a_ld % 8 == 0 && a_off % 8 == 0 && out_ld % 4 == 0 && out_off % 4 == 0 && (!epi || (r_ld % 8 == 0 && r_off % 8 == 0)),
              "%s: misaligned views", what);
  TSArgs t;
  t.a = (const bf16*)a; t.a_ld = a_ld; t.a_off = a_off; t.b = (const bf16*)b;
  t.nimg = n; t.h = h; t.w = w; t.cout = cout;
  t.K = mode == 0 ? cin : 4 * cout;
  t.N = mode == 0 ? 4 * cout : cin;
  t.nblocks = t.N / pl.bn;
  t.tiles_x = (w + 63) / 64;
  t.ntiles = (long)n * h * t.tiles_x;
  t.out = (bf16*)out; t.out_ld = out_ld; t.out_off = out_off;
  t.bias = bias; t.flags = flags; t.aff_scale = aff_scale; t.aff_shift = aff_shift; t.stats = stats;
  t.coef = coef; t.r = (const bf16*)r; t.r_ld = r_ld; t.r_off = r_off;
  CNN_REQUIRE(!(flags & CNNITMO_STATS) || stats, "%s: STATS without buffer", what);
  CNN_REQUIRE(!epi || stats, "%s: fused BN backward without a sums buffer", what);
  const int grid = ts_grid(t.nblocks);
#define L1(M, B, S, E) ts_launch<M, B, S, E>(t, grid, s)
  if (mode == 0) {
    if (pl.bn == 256) L1(0, 256, 5, false);
    else if (pl.bn == 128) L1(0, 128, 5, false);
    else L1(0, 64, 5, false);
  } else if (!epi) {
    if (pl.bn == 256) L1(1, 256, 5, false);
    else if (pl.bn == 128) L1(1, 128, 5, false);
    else L1(1, 64, 5, false);
  } else {
    if (pl.bn == 128) {
      if (pl.st == 3) L1(1, 128, 3, true);
      else L1(1, 128, 2, true);
    } else if (pl.bn == 64) {
      if (pl.st == 4) L1(1, 64, 4, true);
      else if (pl.st == 3) L1(1, 64, 3, true);
      else L1(1, 64, 2, true);
    } else {
      cnnitmo_set_error("%s: fused BN backward needs BN <= 128", what);
      return CNNITMO_EUNSUPPORTED;
    }
  }
#undef L1
  return cnnitmo_check_launch(what);
}
