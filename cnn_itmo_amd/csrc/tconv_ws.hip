// Conv2DTranspose(2, strides=2) forward and input-gradient for up6..up8
// (model.py:199-200, ConvBNTranspose) as WEIGHT-STATIONARY GEMMs whose waves
// never synchronise after the prologue.
//
// A workgroup (8 waves, one per CU) owns one column block of the GEMM: its
// weight block [BN][K] (<= 132 KB, rows padded by 32 B so a B fragment's
// ds_read_b128 lane groups hit distinct banks) is copied into LDS once.  Then every wave walks
// its own 32-pixel tiles: A fragments come straight from HBM/L2 into registers
// (16-byte loads, two K-steps in flight), B fragments from LDS, the MFMA runs
// with the operands swapped (C^T: a lane holds 4 consecutive columns of one
// pixel) and the epilogue stores from registers.  No barrier after the
// prologue: one wave's epilogue overlaps the other waves' MFMAs -- the bubble
// that bounds the tile-synchronous kernels on these short-K GEMMs.
//
// The nblk column blocks of a pixel range run on the workgroups of one XCD, so
// the A tile every block re-reads is an L2 hit (blockIdx % 8 = XCD).
//
// MODE 0 (forward): A = x [P][cin] view, B = k [4*cout][cin] (n = tap*cout + co),
//   out pixel (2y + tap/2, 2x + tap%2); bias (per column or channel), ReLU,
//   inference affine, BN partial sums (per tile, DPP row sums added into the
//   wave's LDS slice; one row per wave at the end: rows = tconv_ws_rows).
// MODE 1 (input gradient): A row of input pixel (y, x) = the four dout pixels
//   (2y+a, 2x+b) x cout (k = tap*cout + co), B = kT [cin][4*cout]; dx [P][cin] (bf16, or
//   fp32 for fp32 training's up8 / up9).
#include <cstdio>

#include "igemm_common.h"

namespace {

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
constexpr int NW = 8;  // waves per workgroup
// weight-block rows are K*2 + WS_PAD bytes: with K*2 a multiple of 256 B the B-fragment
// ds_read_b128 (lane: row l & 15, 16-B piece l >> 4) is conflict-free over the four
// gfx950 lane groups ({0-3,12-15,20-27}, ...; MI355X_MICROARCH.md LDS table) at a
// 32-byte pad; the former 16-byte pad cost 0.5 extra LDS cycles per cycle (PMC)
constexpr int WS_PAD = 32;
#ifndef TWS_LINES
#define TWS_LINES 1
#endif
// fp32 stores as whole lines: measured slower in the fp32 inference step (98.0-98.2 vs
// 98.6-98.7 frames/s, profiles/r04o_ws_ab.txt), off by default
#ifndef TWS_F32_LINES
#define TWS_F32_LINES 0
#endif
#ifndef TWS_PD
#define TWS_PD 4  // A K-steps in flight per wave (3: 9.64, 4: 9.48, 6: 9.56 ms over up6-up8 fwd+dgrad)
#endif

struct WSArgs {
  const void* a;
  long a_ld;
  int a_off;
  const void* b;  // [N][K]
  int nimg, h, w, cout, K, N;
  void* out;
  long out_ld;
  int out_off;
  const float* bias;
  int flags;
  const float* aff_scale;
  const float* aff_shift;
  float* stats;  // [rows][2][N]
  int nblk, gpx;  // column blocks; pixel groups per XCD
  long tiles;     // 32-pixel tiles
};

__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}

// FM: 16-pixel fragment rows per wave tile (tile = 16 * FM pixels).  SQ: distinct BN-stat
// column pairs of the block (BN / 32, or half that when the block spans two taps of the
// same channels: BN = 2 * cout, whose pair q and q + SQ hold one channel's sums).
// TE = float: the fp32 forward (MODE 0; BN sums in fp32 training).  A 16-byte fragment
// piece is KE = 8 bf16 / 4 fp32 channels, so one K-step (four lane groups) is KS = 32 / 16
// channels and 64 bytes in either type; Mma<float> runs a fragment as four 16x16x4 MFMAs.
template <int MODE, int BN, int NKS, int FM = 2, int SQ = BN / 32, typename TE = bf16>
__global__ __launch_bounds__(NW * 64) void tconv_ws_kernel(const WSArgs p) {
  constexpr int FN = BN / 16, TP = 16 * FM;
  constexpr int ES = sizeof(TE), KE = 16 / ES, KS = 64 / ES;
  const TE* __restrict__ PA = (const TE*)p.a;
  const TE* __restrict__ PB = (const TE*)p.b;
  TE* __restrict__ PO = (TE*)p.out;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int K = p.K, ldsrow = K * ES + WS_PAD;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int xcd = blockIdx.x & 7, i = blockIdx.x >> 3;
  const int nb = i % p.nblk, grp = i / p.nblk;
  const int gidx = xcd * p.gpx + grp, ngrp = 8 * p.gpx;
  const long per = (p.tiles + ngrp - 1) / ngrp;
  const long t0 = gidx * per, t1 = t0 + per < p.tiles ? t0 + per : p.tiles;
  // the weight block, once; LDS row nn holds block column pair_perm(nn), so a lane's
  // fragment pair (2q, 2q+1) ends up with 8 consecutive columns (16-byte stores)
  const int pieces = K / KE;
  for (int q = tid; q < BN * pieces; q += NW * 64) {
    const int row = q / pieces, pc = q - row * pieces;
    *reinterpret_cast<uint4*>(smem + row * ldsrow + pc * 16) =
        *reinterpret_cast<const uint4*>(PB + (size_t)(nb * BN + pair_perm(row)) * K + pc * KE);
  }
  // the block's epilogue parameters [3][BN] (bias, affine scale, shift by true column),
  // in LDS: a global load in the epilogue would make its vmcnt wait retire the next
  // tile's A loads too
  float* par = reinterpret_cast<float*>(smem + BN * ldsrow);
  if constexpr (MODE == 0) {
    const bool af = p.flags & CNNITMO_AFFINE;
    for (int c = tid; c < BN; c += NW * 64) {
      const int n = nb * BN + c, co = n % p.cout;
      par[c] = p.bias ? p.bias[(p.flags & CNNITMO_BIAS_PER_COL) ? n : co] : 0.f;
      par[BN + c] = af ? p.aff_scale[co] : 1.f;
      par[2 * BN + c] = af ? p.aff_shift[co] : 0.f;
    }
  }
  __syncthreads();

  const bool relu = p.flags & CNNITMO_RELU, aff = p.flags & CNNITMO_AFFINE, stats = p.flags & CNNITMO_STATS;
  const int hw = p.h * p.w;
  const long P = (long)p.nimg * hw;
  const int frow = lane & 15, kq = lane >> 4;
  const char* Bl = smem + frow * ldsrow + kq * 16;
  constexpr int nks = NKS;  // K / KS, compile-time: the K loop unrolls fully

  // the lane's A row bases for tile t (its two fragment rows; clamped for a tail tile)
  auto bases = [&](long t, const TE** ab) {
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      const long q = t * TP + f * 16 + frow, pc = q < P ? q : P - 1;
      if constexpr (MODE == 0) {
        ab[f] = PA + pc * p.a_ld + p.a_off + kq * KE;
      } else {
        const int pi = (int)pc, img = pi / hw, rem = pi - img * hw, y = rem / p.w, x = rem - y * p.w;
        ab[f] = PA + (((size_t)img * 2 * p.h + 2 * y) * 2 * p.w + 2 * x) * p.cout + kq * KE;
      }
    }
  };
  auto loadA = [&](const TE* const* ab, int ks, uint4* dst) {
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      if constexpr (MODE == 0) {
        dst[f] = *reinterpret_cast<const uint4*>(ab[f] + ks * KS);
      } else {
        const int k0 = ks * KS, tap = k0 / p.cout, co = k0 - tap * p.cout;
        dst[f] = *reinterpret_cast<const uint4*>(ab[f] + ((tap >> 1) * 2 * p.w + (tap & 1)) * p.cout + co);
      }
    }
  };
  // A of TWS_PD K-steps in flight per wave, pipelined ACROSS tiles: the last K-steps of
  // a tile issue the first ones of the wave's next tile, so its epilogue overlaps them.
  // Every load is unconditional (pointer / index selects, no branch), which keeps the
  // compiler's vmcnt counting exact: with conditional loads it waited for all of them
  // at every unrolled group (vmcnt(0)).  nks % TWS_PD == 0 (ws_plan).
  // BN partial sums of the lane's pixels for its 8 columns of each fragment pair, kept
  // in registers for the whole launch (one DPP reduction at the end instead of one per
  // tile: the per-tile reduction was as much VALU issue as the tile's MFMAs)
  constexpr int FP = FN / 2;
  // fp32 output of (fragment base pixel pb, block column pair qq): a pair is 32 channels = one
  // 128-byte line per pixel.  TWS_F32_LINES: one DPP exchange (line_pair) so that store 1
  // writes pixels pb..pb+7 and store 2 pixels pb+8..pb+15 as whole lines (lane (frow, kq):
  // 16 bytes at channel kq*8 + 4*(frow >> 3) of pixel pb + (frow & 7) / + 8); otherwise
  // each lane's two 16-byte pieces of its own pixel (half lines per instruction)
  auto dst32 = [&](long pi, int c) -> float* {  // block column c of pixel pi
    const int n = nb * BN + c;
    if constexpr (MODE == 0) {
      const int tap = n / p.cout, co = n - tap * p.cout;
      const int ip = (int)pi, img = ip / hw, rem = ip - img * hw, y = rem / p.w, x = rem - y * p.w;
      const size_t op = ((size_t)img * 2 * p.h + 2 * y + (tap >> 1)) * 2 * p.w + 2 * x + (tap & 1);
      return (float*)PO + op * p.out_ld + p.out_off + co;
    } else {
      return (float*)PO + (size_t)pi * p.out_ld + p.out_off + n;
    }
  };
  auto st32 = [&](long pb, long pix, bool ok, int qq, const float* vf) {
    const uint4 a = __builtin_bit_cast(uint4, float4{vf[0], vf[1], vf[2], vf[3]});
    const uint4 b = __builtin_bit_cast(uint4, float4{vf[4], vf[5], vf[6], vf[7]});
    if constexpr (TWS_F32_LINES) {
      uint4 v1, v2;
      line_pair(a, b, frow, v1, v2);
      const int c = qq * 32 + kq * 8 + 4 * (frow >> 3);
      const long p1 = pb + (frow & 7), p2 = p1 + 8;
      if (p1 < P) *reinterpret_cast<uint4*>(dst32(p1, c)) = v1;
      if (p2 < P) *reinterpret_cast<uint4*>(dst32(p2, c)) = v2;
    } else if (ok) {
      uint4* d = reinterpret_cast<uint4*>(dst32(pix, qq * 32 + kq * 8));
      d[0] = a;
      d[1] = b;
    }
  };
  float s1[MODE == 0 ? SQ : 1][8], s2[MODE == 0 ? SQ : 1][8];
#pragma unroll
  for (int q = 0; q < (MODE == 0 ? SQ : 1); ++q)
#pragma unroll
    for (int k = 0; k < 8; ++k) s1[q][k] = s2[q][k] = 0.f;
  uint4 Ab[TWS_PD][FM];
  const TE* abc[FM];
  const TE* abn[FM];
  long t = t0 + wave;
  bases(t < t1 ? t : t0, abc);
#pragma unroll
  for (int j = 0; j < TWS_PD - 1; ++j) loadA(abc, j, Ab[j]);
  for (; t < t1; t += NW) {
    bases(t + NW < t1 ? t + NW : t, abn);  // (no next tile: harmless reloads of this one)
    long px[FM];
#pragma unroll
    for (int f = 0; f < FM; ++f) px[f] = t * TP + f * 16 + frow;
    f32x4 acc[FM][FN];
#pragma unroll
    for (int f = 0; f < FM; ++f)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto compute = [&](int ks, const uint4* a) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const uint4 bfr = *reinterpret_cast<const uint4*>(Bl + j * 16 * ldsrow + ks * 64);
#pragma unroll
        for (int f = 0; f < FM; ++f) Mma<TE>::run(acc[f][j], bfr, a[f]);  // C^T: lanes = pixels
      }
    };
#pragma unroll
    for (int ks = 0; ks < nks; ks += TWS_PD) {
#pragma unroll
      for (int j = 0; j < TWS_PD; ++j) {
        const int kn = ks + j + TWS_PD - 1;
        const bool cur = kn < nks;
        const TE* sel[FM];
#pragma unroll
        for (int f = 0; f < FM; ++f) sel[f] = cur ? abc[f] : abn[f];
        loadA(sel, cur ? kn : kn - nks, Ab[(j + TWS_PD - 1) % TWS_PD]);
        __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of this step's MFMAs
        compute(ks + j, Ab[j]);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
#pragma unroll
    for (int f = 0; f < FM; ++f) abc[f] = abn[f];
    // epilogue from registers: fragment pair (2q, 2q+1) gives the lane 8 consecutive
    // columns n .. n+7 of its pixel (pair_perm) -> one 16-byte store per (pixel, pair)
    // (8-byte stores, one per fragment, took 40 % of up8's forward: store-issue-bound).
    // TWS_LINES: the pairs go out in couples (q, q+1) as whole 128-byte lines, 8 pixels
    // per store instruction, after one DPP exchange (line_pair); otherwise every store
    // instruction writes 16 pixels x 64 bytes.
    static_assert(FP % 2 == 0, "pair couples");
#pragma unroll
    for (int q = 0; q < FP; q += 2) {
      uint4 pk[2][FM];
#pragma unroll
      for (int hq = 0; hq < 2; ++hq) {
        const int qq = q + hq;
        if constexpr (MODE == 0) {
          float bj[8], sj[8], hj[8];
          const int cl = qq * 32 + kq * 8;  // the block column of the lane's first channel
          Pack16<float>::load(par + cl, bj);
          Pack16<float>::load(par + cl + 4, bj + 4);
          Pack16<float>::load(par + BN + cl, sj);
          Pack16<float>::load(par + BN + cl + 4, sj + 4);
          Pack16<float>::load(par + 2 * BN + cl, hj);
          Pack16<float>::load(par + 2 * BN + cl + 4, hj + 4);
#pragma unroll
          for (int f = 0; f < FM; ++f) {
            const bool ok = px[f] < P;
            bf16x8 o;
            float vf[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              float v = acc[f][2 * qq + (k >> 2)][k & 3] + bj[k];
              if (relu) v = fmaxf(v, 0.f);
              if (aff) v = fmaf(v, sj[k], hj[k]);
              const float vs = ok ? v : 0.f;
              s1[qq % SQ][k] += vs;
              s2[qq % SQ][k] += vs * vs;
              o[k] = (bf16)v;
              vf[k] = v;
            }
            pk[hq][f] = __builtin_bit_cast(uint4, o);
            if constexpr (ES == 4) st32(t * TP + f * 16, px[f], ok, qq, vf);
          }
        } else if constexpr (ES == 4) {  // fp32 input gradient
#pragma unroll
          for (int f = 0; f < FM; ++f) {
            float vf[8];
#pragma unroll
            for (int k = 0; k < 8; ++k) vf[k] = acc[f][2 * qq + (k >> 2)][k & 3];
            st32(t * TP + f * 16, px[f], px[f] < P, qq, vf);
          }
        } else {
#pragma unroll
          for (int f = 0; f < FM; ++f) {
            bf16x8 o;
#pragma unroll
            for (int k = 0; k < 8; ++k) o[k] = (bf16)acc[f][2 * qq + (k >> 2)][k & 3];
            pk[hq][f] = __builtin_bit_cast(uint4, o);
          }
        }
      }
      // destination of (pixel index pi, block column pair qq, the lane's octet)
      auto dst = [&](long pi, int qq) -> TE* {
        const int n = nb * BN + qq * 32 + kq * 8;
        if constexpr (MODE == 0) {
          const int tap = n / p.cout, co = n - tap * p.cout;
          const int ip = (int)pi, img = ip / hw, rem = ip - img * hw, y = rem / p.w, x = rem - y * p.w;
          const size_t op = ((size_t)img * 2 * p.h + 2 * y + (tap >> 1)) * 2 * p.w + 2 * x + (tap & 1);
          return PO + op * p.out_ld + p.out_off + co;
        } else {
          return PO + (size_t)pi * p.out_ld + p.out_off + n;
        }
      };
      if constexpr (ES == 4) continue;  // (stored above)
#pragma unroll
      for (int f = 0; f < FM; ++f) {
#if TWS_LINES
        uint4 v1, v2;
        line_pair(pk[0][f], pk[1][f], frow, v1, v2);
        const int qq = q + (frow >> 3);
        const long p1 = t * TP + f * 16 + (frow & 7), p2 = p1 + 8;
        if (p1 < P) *reinterpret_cast<uint4*>(dst(p1, qq)) = v1;
        if (p2 < P) *reinterpret_cast<uint4*>(dst(p2, qq)) = v2;
#else
        if (px[f] < P) {
          *reinterpret_cast<uint4*>(dst(px[f], q)) = pk[0][f];
          *reinterpret_cast<uint4*>(dst(px[f], q + 1)) = pk[1][f];
        }
#endif
      }
    }
  }
  if constexpr (MODE == 0) {
    if (stats) {  // one row per wave: row = (group, wave), columns of this block
      // each wave's [BN][2] slice of LDS over the weight block (every wave is past its MFMAs)
      __syncthreads();
      float* sl = reinterpret_cast<float*>(smem) + wave * BN * 2;
#pragma unroll
      for (int q = 0; q < FP; ++q)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          // (BN = 2 cout: the channel's sums go to its first tap's column, zero to the other)
          const float a1 = q < SQ ? row16_sum(s1[q % SQ][k]) : 0.f, a2 = q < SQ ? row16_sum(s2[q % SQ][k]) : 0.f;
          if (frow == 0) {
            const int c = q * 32 + kq * 8 + k;
            sl[c * 2] = a1;
            sl[c * 2 + 1] = a2;
          }
        }
      __syncthreads();
      const long row = (long)gidx * NW + wave;
      for (int q = lane; q < BN; q += 64) {
        p.stats[(size_t)row * 2 * p.N + nb * BN + q] = sl[q * 2];
        p.stats[(size_t)row * 2 * p.N + p.N + nb * BN + q] = sl[q * 2 + 1];
      }
    }
  }
}

struct WSPlan {
  int bn, nblk, gpx;
};

bool ws_plan(int mode, int cin, int cout, WSPlan& pl, bool f32 = false) {
  // (fp32 inference forward, up6-up8: 0.61-0.69 -> 0.79-0.80 of fp32 peak against the
  // implicit GEMM, 1080p b8 fp32 inference 94.3 -> 95.9 frames/s, profiles/r03zp_*)
  if (cout % 32 || cin % 32) return false;
  // the bf16 input gradient (up8, K = 512) runs on igemm_fwd2p_kernel: 1.52 -> 1.31 ms
  // (profiles/r05/r05t2_ab_up8_dgrad_fwd2p.txt)
  if (mode == 1 && !f32) return false;
  const int K = mode == 0 ? cin : 4 * cout, N = mode == 0 ? 4 * cout : cin;
  if (f32) {  // fp32 forward: the widest block whose fp32 rows fit (K 512: 64, 256 / 128: 128)
    // K = 128 is up9 (128 -> 64 channels at full resolution), which ran on igemm_fwd2's
    // 128 x 128 tiles at 0.49 of fp32 peak (a 256-column block spills: 16 fp32 fragments).
    // fp32 input gradient (training): K = 4 * cout = 256 (up9) / 512 (up8)
    if ((K != 128 && K != 256 && K != 512) || (mode == 1 && K == 128)) return false;
    const int bn = K == 512 ? 64 : 128;
    if (N % bn || N / bn > 32 || 32 % (N / bn)) return false;
    pl.bn = bn;
    pl.nblk = N / bn;
    pl.gpx = 32 / pl.nblk;
    return true;
  }
  // K = 256 or 512: the row padding below is conflict-free (K % 128 == 0) and the K loop
  // is compiled for K / 32 = 8 or 16 steps (a multiple of TWS_PD)
  if (K != 256 && K != 512) return false;
  // (a 256-column forward block at K = 256 (up8), 16-pixel wave tiles: 2.33 ms against BN
  // 128's 2.01-2.06 once the stores write whole lines, profiles/r03z_ab_lines_bn256.txt)
  int bn = 128;
  while (bn >= 64 && (long)bn * (K * 2 + WS_PAD) + 3 * bn * 4 > 148 * 1024) bn /= 2;
  if (bn < 64 || N % bn) return false;
  const int nblk = N / bn;
  if (nblk > 32 || 32 % nblk) return false;
  // where it measured faster than the halo / implicit-GEMM paths (tools/ab_env.sh,
  // b32 1080p): every forward at BN 128 (up6 1.50 -> 1.08, up7 2.62 -> 1.98, up8
  // 3.16 -> 2.98 ms).  (The bf16 input gradients moved to igemm_fwd2p_kernel, above.)
  if (bn != 128) return false;
  pl.bn = bn;
  pl.nblk = nblk;
  pl.gpx = 32 / nblk;
  return true;
}

}  // namespace

bool tconv_ws_handles(int mode, int cin, int cout, bool f32) {
  WSPlan pl;
  return ws_plan(mode, cin, cout, pl, f32);
}

// BN partial-sum rows of the forward: one per (pixel group, wave)
long tconv_ws_rows(int cin, int cout, bool f32) {
  WSPlan pl;
  if (!ws_plan(0, cin, cout, pl, f32)) return 0;
  return 8L * pl.gpx * NW;
}

const char* tconv_ws_name(int mode, int cin, int cout, bool f32) {
  WSPlan pl;
  if (!ws_plan(mode, cin, cout, pl, f32)) return "";
  static thread_local char buf[64];
  snprintf(buf, sizeof(buf), "tconv_ws_kernel<%s%d,%d>", f32 ? "f32," : "", mode, pl.bn);
  return buf;
}

int launch_tconv_ws(int mode, const void* a, long a_ld, int a_off, const void* b, int n, int h, int w, int cin,
                    int cout, void* out, long out_ld, int out_off, const float* bias, int flags,
                    const float* aff_scale, const float* aff_shift, float* stats, hipStream_t s, const char* what,
                    bool f32) {
  WSPlan pl;
  CNN_REQUIRE(ws_plan(mode, cin, cout, pl, f32), "%s: no weight-stationary plan", what);
  CNN_REQUIRE(a_ld % 8 == 0 && a_off % 8 == 0 && out_ld % 4 == 0 && out_off % 4 == 0, "%s: misaligned views", what);
  CNN_REQUIRE((long)n * h * w < (1L << 31), "%s: too many pixels", what);
  CNN_REQUIRE(!(flags & CNNITMO_STATS) || (stats && mode == 0), "%s: STATS without buffer", what);
  WSArgs t;
  t.a = a; t.a_ld = a_ld; t.a_off = a_off; t.b = b;
  t.nimg = n; t.h = h; t.w = w; t.cout = cout;
  t.K = mode == 0 ? cin : 4 * cout;
  t.N = mode == 0 ? 4 * cout : cin;
  t.out = out; t.out_ld = out_ld; t.out_off = out_off;
  t.bias = bias; t.flags = flags; t.aff_scale = aff_scale; t.aff_shift = aff_shift; t.stats = stats;
  t.nblk = pl.nblk; t.gpx = pl.gpx;
  const int tp = 32;  // pixels per wave tile
  t.tiles = ((long)n * h * w + tp - 1) / tp;
  const int grid = 8 * pl.gpx * pl.nblk;  // 256: one workgroup per CU
  const size_t lds = (size_t)pl.bn * (t.K * (f32 ? 4 : 2) + WS_PAD) + 3 * pl.bn * sizeof(float);
  static bool attr = [] {  // dynamic LDS beyond 64 KB
    (void)hipFuncSetAttribute((const void*)tconv_ws_kernel<0, 128, 8>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)tconv_ws_kernel<0, 128, 16>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)tconv_ws_kernel<0, 64, 32, 2, 2, float>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)tconv_ws_kernel<0, 128, 16, 2, 4, float>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)tconv_ws_kernel<0, 128, 8, 2, 4, float>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)tconv_ws_kernel<1, 64, 32, 2, 2, float>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    (void)hipFuncSetAttribute((const void*)tconv_ws_kernel<1, 128, 16, 2, 4, float>, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    return true;
  }();
  (void)attr;
#define TWL(M, KS) hipLaunchKernelGGL((tconv_ws_kernel<M, 128, KS>), dim3(grid), dim3(NW * 64), lds, s, t)
  if (f32 && mode == 1) {  // K / 16 steps
    if (t.K == 512) hipLaunchKernelGGL((tconv_ws_kernel<1, 64, 32, 2, 2, float>), dim3(grid), dim3(NW * 64), lds, s, t);
    else hipLaunchKernelGGL((tconv_ws_kernel<1, 128, 16, 2, 4, float>), dim3(grid), dim3(NW * 64), lds, s, t);
  } else if (f32) {  // K / 16 steps
    if (t.K == 512) hipLaunchKernelGGL((tconv_ws_kernel<0, 64, 32, 2, 2, float>), dim3(grid), dim3(NW * 64), lds, s, t);
    else if (t.K == 256) hipLaunchKernelGGL((tconv_ws_kernel<0, 128, 16, 2, 4, float>), dim3(grid), dim3(NW * 64), lds, s, t);
    else hipLaunchKernelGGL((tconv_ws_kernel<0, 128, 8, 2, 4, float>), dim3(grid), dim3(NW * 64), lds, s, t);
  } else {
    if (t.K == 256) TWL(0, 8);
    else TWL(0, 16);
  }
#undef TWL
  return cnnitmo_check_launch(what);
}
