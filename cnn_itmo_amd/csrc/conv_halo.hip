// 3x3 'same' convolution (forward and input-gradient) for the high-resolution,
// few-channel layers of the U-Net (enc1b, enc2a/b, dec8, dec9: 32..192 channels
// at 1920x1088 and 960x544), bf16.
//
// The implicit GEMM of igemm_fwd2.hip gathers A once per tap, so every input
// pixel crosses L2 -> LDS nine times; with few channels per pixel that re-read,
// not the MFMA, bounds those layers.  Here a workgroup owns a 4 x 64 tile of
// output pixels and stages its (4+2) x (64+2) input halo ONCE per 32-channel
// chunk; the nine taps are nine shifted windows of the same LDS image:
//   A fragment (tap r,s; output row y, 16 columns x0..x0+15) =
//       patch rows (y+r)*66 + x0+s .. +15   (consecutive LDS rows, any start)
//   B fragment (tap t; 16 output channels) = wstage rows t*BN + j*16 .. +15
// LDS rows are 64 B (32 bf16); piece c of row q is stored at piece
// c ^ (((q >> 2) & 1) << 1), which keeps every ds_read_b128 lane group
// conflict-free for windows starting at ANY row (exhaustive check:
// tools/check_swizzle.py).  Operands arrive by global_load_lds_dwordx4 (lane-linear LDS
// image, swizzle applied to the source piece).
//
// Persistent grid: one workgroup per CU walks a contiguous range of
// (tile, column-block) items, tiles ordered image -> column strip -> row so the
// next tile's halo rows are the previous tile's last rows (L2 hits).  A 2-stage
// LDS ring overlaps the loads of item t+1 with the MFMAs of item t; the epilogue
// (bias, ReLU, inference BN affine, folded-BN border correction, BN partial
// sums: the same semantics as igemm_fwd2) stages each wave's 64 x BN tile in
// the stage it just consumed and stores 16-byte rows.
#include <cstdio>

#include "igemm_common.h"

// timing-only experiment builds (tools/halo_exp.sh), results are garbage:
// 1 = no DMA wait, 2 = no MFMA, 3 = no epilogue, 4 = no DMA issue/wait,
// 5 = epilogue without its global stores, 6 = epilogue without the C-tile LDS writes,
// 7 = epilogue without C-tile LDS writes and barriers
#ifndef HALO_EXP
#define HALO_EXP 0
#endif
// 1: EPI 0 epilogue straight from the MFMA registers (operands swapped so a lane
// holds 4 consecutive channels of one pixel: 8-byte buffer stores, DPP row sums,
// no C tile in LDS, no barrier unless BN statistics are gathered); 0 (default):
// LDS-staged.  Measured A/B (tools/ab_layers.sh, tools/ab_bench.sh): per layer
// within +-5 % either way without statistics, and the training forward (with
// statistics) 8 % slower (845 vs 917 TF/s): the epilogue's cost is the MFMA pipe
// idling while all eight waves store, which neither variant hides.
// taps over which the next item's LDS-DMA pieces are issued (0 = all KT taps).
// 5 of 9 (tools/ab_libs.sh, b32 1080p): dec6-dec9 + enc2b/enc3b fwd+dgrad
// 64.4 -> 63.7 ms (dec7/dec8 fwd -2..4 %, the last pieces land sooner)
#ifndef HALO_PF_TAPS
#define HALO_PF_TAPS 5
#endif
#ifndef HALO_REGEPI
#define HALO_REGEPI 0
#endif

namespace {

__device__ __attribute__((aligned(256))) unsigned char h_zero_page[256] = {0};
// store sink for the output pieces of a partial tile that fall outside the image
// (the store is still issued: every wave must issue a fixed count of vector-memory
// ops per item for the counted vmcnt waits)
__device__ __attribute__((aligned(256))) uint4 h_sink[64];

#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}
typedef int i32x4 __attribute__((ext_vector_type(4)));
// raw buffer descriptor over [base, base + 2 GB): a load at voffset >= OOB_OFF is
// dropped by the range check and lands zeros (halo padding, pad rows)
constexpr unsigned OOB_OFF = 0x80000000u;
__device__ __forceinline__ i32x4 buf_rsrc(uintptr_t base) {
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)base);
  r.y = __builtin_amdgcn_readfirstlane((int)(unsigned)(base >> 32)) & 0xFFFF;
  r.z = 0x7FFFFFF0;
  r.w = 0x00020000;
  return r;
}
// one 16-byte piece per lane -> the wave's 1 KiB LDS image at `lds` (LDS-DMA)
__device__ __forceinline__ void blds16(unsigned voff, i32x4 rs, const char* lds) {
  const unsigned a = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
               "s"(a) : "memory");
}
template <int N> __device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// s_waitcnt takes an immediate: dispatch a wave-uniform count (0..31)
__device__ __forceinline__ void wait_vm_dyn(int n) {
  switch (n) {
#define W1(k) case k: wait_vm<k>(); break;
    W1(0) W1(1) W1(2) W1(3) W1(4) W1(5) W1(6) W1(7) W1(8) W1(9) W1(10) W1(11) W1(12) W1(13) W1(14) W1(15)
    W1(16) W1(17) W1(18) W1(19) W1(20) W1(21) W1(22) W1(23) W1(24) W1(25) W1(26) W1(27) W1(28) W1(29)
    W1(30) W1(31)
#undef W1
    default: wait_vm<0>(); break;
  }
}

typedef unsigned u32x2 __attribute__((ext_vector_type(2)));
// buffer resource over [p, p + 2 GB) from a wave-uniform pointer
__device__ __forceinline__ __amdgpu_buffer_rsrc_t out_rsrc(const void* p) {
  const uintptr_t a = (uintptr_t)p;
  const uintptr_t u = (uintptr_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a) |
                      ((uintptr_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32)) << 32);
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, (short)0, 0x7FFFFFF0, 0x00020000);
}
// sum over the 16 lanes of each DPP row (quad_perm xor 1, xor 2, then the half-row
// and row mirrors): 4 VALU ops, no LDS crossbar traffic
__device__ __forceinline__ float row16_sum(float v) {
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0xB1, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x4E, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x141, 0xF, 0xF, false));
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x140, 0xF, 0xF, false));
  return v;
}

__device__ __forceinline__ int hswz(int row, int piece) {
  return (row << 6) + ((piece ^ (((row >> 2) & 1) << 1)) << 4);
}

// Tile TH x TW GEMM-row pixels, one wave per tile row (FM = TW/16 fragments),
// BN output columns per item, ST-deep LDS ring.
//   MODE 0: conv3x3 'same' (9 taps, (TH+2) x (TW+2) halo patch)
//   MODE 1: Conv2DTranspose(2, s2) forward: a 1x1 GEMM over the input pixels
//           (TH x TW patch, no halo) whose column n = tap*cout + co is scattered
//           to output pixel (2y + tap/2, 2x + tap%2)
template <int MODE, int TH, int TW, int BN, int ST, int EPI = 0>
struct HaloCfg {
  static constexpr int NWAVE = TH <= 8 ? TH : 8, NT = NWAVE * 64;
  static constexpr int RPW = TH / NWAVE;  // tile rows per wave
  static constexpr int FMR = TW / 16, FM = RPW * FMR, FN = BN / 16;
  static constexpr int KT = MODE == 0 ? 9 : 1;  // taps
  static constexpr int PW = MODE == 0 ? TW + 2 : TW, PROWS = (MODE == 0 ? TH + 2 : TH) * PW;
  static constexpr int P_INSTR = ((PROWS + 15) / 16 + NWAVE - 1) / NWAVE * NWAVE;
  static constexpr int B_ROWS = KT * BN;
  static constexpr int B_INSTR = ((B_ROWS + 15) / 16 + NWAVE - 1) / NWAVE * NWAVE;
  static constexpr int NPI = P_INSTR / NWAVE, NBI = B_INSTR / NWAVE;
  static constexpr int PATCH = P_INSTR * 1024;
  static constexpr int STAGE = PATCH + B_INSTR * 1024;
  static constexpr int CLD = BN + 8;  // C staging row (bf16), per wave TW rows
  static constexpr int C_BYTES = NWAVE * RPW * TW * CLD * 2;
  // cross-wave partial sums: [NWAVE][BN][2] (BN stats) or [NWAVE][BN][4] (EPI 1 parity sums)
  static constexpr int RED_BYTES = NWAVE * BN * (EPI ? 16 : 8);
  // the epilogue stages C in the stage it just consumed when it fits, else in its own region
  static constexpr bool C_IN_STAGE = C_BYTES + RED_BYTES <= STAGE;
  static constexpr int C_OFF = ST * STAGE;
  static constexpr int SMEM = ST * STAGE + (C_IN_STAGE ? 0 : C_BYTES + RED_BYTES);
  static constexpr int SG = TH * TW / 256;  // BN-partial-sum rows per tile (256 pixels each)
  static_assert(TH * TW % 256 == 0 && TW % 16 == 0, "tile");
};

struct HaloArgs {
  FwdArgs f;
  int tiles_x, tiles_y;  // per image
  long npairs;           // tiles * nblocks
  long per_block;        // contiguous items per workgroup
  int nchunks;           // cin / 32
};

// EPI 1 (MODE 0 dgrad only): the producer's BN backward fused into the store, see
// FwdArgs::bnb_* and epilogue_bnb below.
template <int MODE, int TH, int TW, int BN, int ST, int EPI>
__global__ __launch_bounds__((HaloCfg<MODE, TH, TW, BN, ST, EPI>::NT)) void halo_gemm_kernel(const HaloArgs h) {
  using C = HaloCfg<MODE, TH, TW, BN, ST, EPI>;
  constexpr int KT = C::KT;
  static_assert(C::SMEM <= 160 * 1024, "LDS");
  constexpr int NWAVE = C::NWAVE, FM = C::FM, FN = C::FN, STAGE = C::STAGE, PW = C::PW;
  constexpr int RPW = C::RPW, FMR = C::FMR;
  constexpr int NPI = C::NPI, NBI = C::NBI;
  constexpr int CPR = BN / 8;  // 16-byte output pieces per pixel
  constexpr int CPRP = CPR <= 4 ? 4 : (CPR <= 8 ? 8 : 16);  // EPI 1: lanes per pixel (power of 2)
  constexpr bool REG = EPI == 0 && HALO_REGEPI && HALO_EXP == 0;
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];
  const FwdArgs& p = h.f;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR) for the vmcnt switch
  const long q0 = (long)blockIdx.x * h.per_block;
  const long q1 = q0 + h.per_block < h.npairs ? q0 + h.per_block : h.npairs;
  if (q0 >= q1) return;
  const int nch = h.nchunks;
  const long T = (q1 - q0) * nch;
  const bf16* __restrict__ X = (const bf16*)p.a;
  const bf16* __restrict__ Wt = (const bf16*)p.b;
  const int K = KT * p.cin;
  const int tpi = h.tiles_x * h.tiles_y;

  // position of an item: (img, tile row, tile column, column block, chunk);
  // tile rows fastest so consecutive tiles share halo rows
  struct Pos {
    int img, y0, x0, nb, ch;
  };
  Pos ip;
  {
    const int q = (int)q0;  // npairs < 2^31 (checked by the launcher)
    const int tile = q / p.nblocks;
    ip.nb = q - tile * p.nblocks;
    ip.img = tile / tpi;
    const int rem = tile - ip.img * tpi;
    const int txi = rem / h.tiles_y;
    ip.y0 = (rem - txi * h.tiles_y) * TH;
    ip.x0 = txi * TW;
    ip.ch = 0;
  }
  auto step = [&](Pos& s) {
    if (++s.ch < nch) return;
    s.ch = 0;
    if (++s.nb < p.nblocks) return;
    s.nb = 0;
    s.y0 += TH;
    if (s.y0 < p.ho) return;
    s.y0 = 0;
    s.x0 += TW;
    if (s.x0 < p.wo) return;
    s.x0 = 0;
    ++s.img;
  };

  // per-lane load geometry, fixed for the whole launch: one glds instruction =
  // 16 LDS rows x 4 pieces of 16 B; lane -> (row, piece), source piece swizzled
  const int lrow = lane >> 2, lpc = lane & 3;
  constexpr int lo = MODE == 0 ? 1 : 0;  // halo reach above / left of the tile
  int ppy[NPI], ppx[NPI];
  unsigned poff[NPI];  // byte offset of the lane's source piece from the patch origin (tile origin - lo rows/cols)
#pragma unroll
  for (int i = 0; i < NPI; ++i) {
    const int row = (wave * NPI + i) * 16 + lrow;
    const int piece = lpc ^ (((row >> 2) & 1) << 1);
    const int py = row / PW, px = row - (row / PW) * PW;
    ppy[i] = row < C::PROWS ? py - lo : -(1 << 29);  // padded rows: never in bounds, never loaded
    ppx[i] = px - lo;
    poff[i] = (unsigned)((((long)py * p.ws + px) * p.a_ld + piece * 8) * 2);
  }
  unsigned boff[NBI];
#pragma unroll
  for (int i = 0; i < NBI; ++i) {
    const int row = (wave * NBI + i) * 16 + lrow;  // = tap * BN + n
    const int piece = lpc ^ (((row >> 2) & 1) << 1);
    const int tap = row / BN, n = row - (row / BN) * BN;
    boff[i] = row < C::B_ROWS ? (unsigned)((n * K + tap * p.cin + piece * 8) * 2) : OOB_OFF;
  }

  // The loads of an item are prepared once (descriptors, per-piece offsets) and
  // issued piece by piece: the main loop spreads them between the taps of the
  // previous item's MFMAs, so LDS-DMA issue overlaps matrix work instead of
  // stalling every wave at the top of the chunk.
  constexpr int L = NPI + NBI;  // LDS-DMA instructions per wave per item
  uintptr_t pbase = 0, bbase = 0;  // descriptor bases (built into SGPRs at each use)
  char* iPs = smem;
  unsigned pvo[NPI];
  auto issue_prep = [&](int buf) {
    const Pos& s = ip;
    iPs = smem + buf * STAGE;
    const long po = ((long)s.img * p.hs + s.y0 - lo) * p.ws + s.x0 - lo;  // patch origin pixel (may be < 0)
    pbase = (uintptr_t)X + (uintptr_t)((po * p.a_ld + p.a_off + s.ch * 32) * 2);
    bbase = (uintptr_t)(Wt + (size_t)s.nb * BN * K + s.ch * 32);
#pragma unroll
    for (int i = 0; i < NPI; ++i) {
      const int yy = s.y0 + ppy[i], xx = s.x0 + ppx[i];
      const bool ok = (unsigned)yy < (unsigned)p.hs && (unsigned)xx < (unsigned)p.ws;
      pvo[i] = ok ? poff[i] : OOB_OFF;
    }
  };
  auto issue_piece = [&](int k) {  // k: compile-time after unrolling
    if constexpr (HALO_EXP == 4) return;
    if (k < NPI) blds16(pvo[k], buf_rsrc(pbase), iPs + (wave * NPI + k) * 1024);
    else blds16(boff[k - NPI], buf_rsrc(bbase), iPs + C::PATCH + (wave * NBI + k - NPI) * 1024);
  };

  f32x4 acc[FM][FN];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();

  // fragment-read addresses: A window row = rbase + c with c = r*PW + 16i + s
  // compile-time; the swizzle bit of (rbase + c) depends only on (c & 7), so the
  // 8 residues are precomputed and c*64 becomes an immediate offset.
  const int frow = lane & 15, fpc = lane >> 4;
  const int rbase = wave * RPW * PW + frow;
  int apre[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) apre[k] = rbase * 64 + ((fpc ^ ((((rbase + k) >> 2) & 1) << 1)) << 4);
  const int bpre = frow * 64 + ((fpc ^ (((frow >> 2) & 1) << 1)) << 4);
  // Fragments are double-buffered across taps: tap t+1's ds_reads are issued
  // before tap t's MFMAs (pinned by sched barriers), so a whole tap of MFMAs
  // covers their latency instead of the just-in-time reads the scheduler emits.
  // the next item's LDS-DMA pieces are spread over the first PFT taps
  constexpr int PFT = HALO_PF_TAPS > 0 && HALO_PF_TAPS < KT ? HALO_PF_TAPS : KT;
  auto compute = [&](int buf, bool pf) {
    const char* Ps = smem + buf * STAGE;
    const char* Bs = Ps + C::PATCH;
    uint4 af[2][FM], bfr[2][FN];
    auto load = [&](int tap, int sl) {
      const int r = MODE == 0 ? tap / 3 : 0, s = MODE == 0 ? tap - 3 * (tap / 3) : 0;
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int c = (f / FMR + r) * PW + (f % FMR) * 16 + s;  // tile row f/FMR of this wave
        af[sl][f] = *reinterpret_cast<const uint4*>(Ps + apre[c & 7] + c * 64);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[sl][j] = *reinterpret_cast<const uint4*>(Bs + bpre + (tap * BN + j * 16) * 64);
    };
    load(0, 0);
#pragma unroll
    for (int tap = 0; tap < KT; ++tap) {
      const int cur = tap & 1;
      if (tap + 1 < KT) load(tap + 1, cur ^ 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j)
          if constexpr (HALO_EXP == 2) acc[i][j][0] += __builtin_bit_cast(float, af[cur][i].x ^ bfr[cur][j].y);
          else if constexpr (REG) Mma<bf16>::run(acc[i][j], bfr[cur][j], af[cur][i]);  // C^T: lanes = pixels
          else Mma<bf16>::run(acc[i][j], af[cur][i], bfr[cur][j]);
      // the next item's LDS-DMA pieces due after this tap
      if (pf) {
#pragma unroll
        for (int k = 0; k < L; ++k)
          if ((k * PFT) / L == tap) issue_piece(k);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  const bool relu = p.flags & CNNITMO_RELU, aff = p.flags & CNNITMO_AFFINE,
             stats = p.flags & CNNITMO_STATS;
  auto epilogue = [&](const Pos& e, int buf) {
    const int img = e.img, y0 = e.y0, x0 = e.x0;
    const int n0 = e.nb * BN;
    const int oh0 = y0 + wave * RPW;  // first tile row of this wave
    char* cbase = C::C_IN_STAGE ? smem + buf * STAGE : smem + C::C_OFF;
    bf16* Cs = reinterpret_cast<bf16*>(cbase) + wave * RPW * TW * C::CLD;
    float* red = reinterpret_cast<float*>(cbase + C::C_BYTES);  // [NWAVE][BN][2]
    // MODE 1: GEMM column n = tap*cout + co (a block may span several taps when BN > cout)
    float s1[FN], s2[FN];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int n = n0 + j * 16 + (lane & 15);
      const int co = MODE == 1 ? n % p.cout : n;
      const float bj = p.bias ? p.bias[(p.flags & CNNITMO_BIAS_PER_COL) ? n : co] : 0.f;
      const float sj = aff ? p.aff_scale[co] : 1.f, hj = aff ? p.aff_shift[co] : 0.f;
      const float* U = p.border ? p.border + (size_t)n * 8 : nullptr;
      s1[j] = s2[j] = 0.f;
#pragma unroll
      for (int f = 0; f < FM; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = f / FMR, col = (f % FMR) * 16 + (lane >> 4) * 4 + r;  // pixel (row rr, col) of the wave
          const int oh = oh0 + rr;
          float v = acc[f][j][r] + bj;
          if (U) v -= border_corr(U, oh, x0 + col, p.ho, p.wo);
          if (relu) v = fmaxf(v, 0.f);
          if (aff) v = v * sj + hj;
          const float vs = (oh < p.ho && x0 + col < p.wo) ? v : 0.f;  // partial tiles: valid pixels only
          s1[j] += vs;
          s2[j] += vs * vs;
          if constexpr (HALO_EXP != 6 && HALO_EXP != 7) Cs[(rr * TW + col) * C::CLD + j * 16 + (lane & 15)] = from_f32<bf16>(v);
          else if (p.N < 0) Cs[0] = from_f32<bf16>(v);
        }
    }
    if (stats) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        s1[j] += __shfl_xor(s1[j], 16, 64);
        s1[j] += __shfl_xor(s1[j], 32, 64);
        s2[j] += __shfl_xor(s2[j], 16, 64);
        s2[j] += __shfl_xor(s2[j], 32, 64);
      }
      if (lane < 16) {
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          red[(wave * BN + j * 16 + lane) * 2 + 0] = s1[j];
          red[(wave * BN + j * 16 + lane) * 2 + 1] = s2[j];
        }
      }
    }
    if constexpr (HALO_EXP != 7) __syncthreads();
    if (stats && tid < C::SG * BN) {
      // one partial-sum row per 256 pixels: rows = M / 256 (= cnnitmo_fwd_stat_rows)
      const int g = tid / BN, col = tid - g * BN;
      constexpr int WPG = NWAVE / C::SG;  // waves per 256-pixel group
      float t1 = 0.f, t2 = 0.f;
#pragma unroll
      for (int w = 0; w < WPG; ++w) {
        t1 += red[((g * WPG + w) * BN + col) * 2 + 0];
        t2 += red[((g * WPG + w) * BN + col) * 2 + 1];
      }
      const long tile = ((long)img * h.tiles_y + y0 / TH) * h.tiles_x + x0 / TW;
      float* st = p.stats + (size_t)(tile * C::SG + g) * 2 * p.N;
      st[n0 + col] = t1;
      st[p.N + n0 + col] = t2;
    }
    // each wave stores its TW pixels x BN channels as 16-byte row pieces
    bf16* __restrict__ O = (bf16*)p.out;
    // MODE 0: output pixel (oh, x0 + col); MODE 1: (2*oh + tap/2, 2*(x0 + col) + tap%2) of the 2x grid
    constexpr int PSTEP = MODE == 0 ? 1 : 2;  // output pixels per GEMM row step
#pragma unroll
    for (int idx = lane; idx < RPW * TW * CPR; idx += 64) {
      const int px = idx / CPR, cc = idx - px * CPR;
      const int rr = px / TW, col = px - rr * TW, oh = oh0 + rr;
      const int n = n0 + cc * 8;  // first column of this 16-byte piece (8 | cout)
      const int tp = MODE == 1 ? n / p.cout : 0, co = MODE == 1 ? n - tp * p.cout : n;
      const long mrow = MODE == 0 ? ((long)img * p.ho + oh) * p.wo + x0
                                  : ((long)img * 2 * p.ho + 2 * oh + (tp >> 1)) * 2 * p.wo + 2 * x0 + (tp & 1);
      const uint4 v = *reinterpret_cast<const uint4*>(Cs + px * C::CLD + cc * 8);
      uint4* dst = (oh < p.ho && x0 + col < p.wo)
                       ? reinterpret_cast<uint4*>(O + (size_t)(mrow + PSTEP * col) * p.out_ld + p.out_off + co)
                       : h_sink + lane;
      if constexpr (HALO_EXP == 5) {
        if (p.N < 0) *dst = v;
      } else {
        *dst = v;
      }
    }
    zero_acc();
  };

  // REG: the epilogue straight from the (swapped-operand) accumulators: lane = pixel
  // (lane & 15) of fragment f, 4 consecutive columns (lane >> 4) * 4 + r of
  // fragment j.  Bias, border correction, ReLU, inference affine, then one 8-byte
  // buffer store per (f, j) (out-of-image pixels: offset beyond the range, dropped;
  // every lane issues FM*FN stores).  BN sums: DPP row sums over the 16 pixels of
  // each fragment, then across the waves of each 256-pixel group through LDS.
  auto epilogue_reg = [&](const Pos& e, int buf) {
    const int img = e.img, y0 = e.y0, x0 = e.x0;
    const int n0 = e.nb * BN;
    const int oh0 = y0 + wave * RPW;
    const bf16* base = MODE == 0
                           ? (const bf16*)p.out + (((size_t)img * p.ho + oh0) * p.wo + x0) * p.out_ld + p.out_off
                           : (const bf16*)p.out + (((size_t)img * 2 * p.ho + 2 * oh0) * 2 * p.wo + 2 * x0) * p.out_ld +
                                 p.out_off;
    const __amdgpu_buffer_rsrc_t os = out_rsrc(base);
    float s1[FN][4], s2[FN][4];
#pragma unroll
    for (int j = 0; j < FN; ++j) {
      const int c = j * 16 + (lane >> 4) * 4;  // first of this lane's 4 columns in the block
      const int n = n0 + c;
      const int tp = MODE == 1 ? n / p.cout : 0, co = MODE == 1 ? n - tp * p.cout : n;
      // 16-byte loads: 4 | column, parameter slices 16-byte aligned
      const float4 b4 = p.bias ? *reinterpret_cast<const float4*>(p.bias + ((p.flags & CNNITMO_BIAS_PER_COL) ? n : co))
                               : make_float4(0.f, 0.f, 0.f, 0.f);
      const float4 s4 = aff ? *reinterpret_cast<const float4*>(p.aff_scale + co) : make_float4(1.f, 1.f, 1.f, 1.f);
      const float4 h4 = aff ? *reinterpret_cast<const float4*>(p.aff_shift + co) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float bj[4] = {b4.x, b4.y, b4.z, b4.w}, sj[4] = {s4.x, s4.y, s4.z, s4.w}, hj[4] = {h4.x, h4.y, h4.z, h4.w};
#pragma unroll
      for (int r = 0; r < 4; ++r) s1[j][r] = s2[j][r] = 0.f;
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int rr = f / FMR, col = (f % FMR) * 16 + (lane & 15);
        const int oh = oh0 + rr, ow = x0 + col;
        const bool ok = oh < p.ho && ow < p.wo;
        bf16 o[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = acc[f][j][r] + bj[r];
          if (p.border) v -= border_corr(p.border + (size_t)(n + r) * 8, oh, ow, p.ho, p.wo);
          if (relu) v = fmaxf(v, 0.f);
          if (aff) v = v * sj[r] + hj[r];
          const float vs = ok ? v : 0.f;
          s1[j][r] += vs;
          s2[j][r] += vs * vs;
          o[r] = from_f32<bf16>(v);
        }
        u32x2 pk;
        __builtin_memcpy(&pk, o, 8);
        const long el = MODE == 0 ? ((long)rr * p.wo + col) * p.out_ld + co
                                  : ((long)(2 * rr + (tp >> 1)) * 2 * p.wo + 2 * col + (tp & 1)) * p.out_ld + co;
        __builtin_amdgcn_raw_buffer_store_b64(pk, os, ok ? (unsigned)(el * 2) : 0x80000000u, 0, 0);
      }
    }
    if (stats) {
      // every wave has left the stage before the sums reuse it
      __syncthreads();
      float* red = reinterpret_cast<float*>(smem + buf * STAGE);  // [NWAVE][BN][2]
#pragma unroll
      for (int j = 0; j < FN; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const float a1 = row16_sum(s1[j][r]), a2 = row16_sum(s2[j][r]);
          if ((lane & 15) == 0) {
            const int c = j * 16 + (lane >> 4) * 4 + r;
            red[(wave * BN + c) * 2 + 0] = a1;
            red[(wave * BN + c) * 2 + 1] = a2;
          }
        }
      __syncthreads();
      if (tid < C::SG * BN) {
        const int g = tid / BN, col = tid - g * BN;
        constexpr int WPG = NWAVE / C::SG;  // waves per 256-pixel group
        float t1 = 0.f, t2 = 0.f;
#pragma unroll
        for (int w = 0; w < WPG; ++w) {
          t1 += red[((g * WPG + w) * BN + col) * 2 + 0];
          t2 += red[((g * WPG + w) * BN + col) * 2 + 1];
        }
        const long tile = ((long)img * h.tiles_y + y0 / TH) * h.tiles_x + x0 / TW;
        float* st = p.stats + (size_t)(tile * C::SG + g) * 2 * p.N;
        st[n0 + col] = t1;
        st[p.N + n0 + col] = t2;
      }
    }
    zero_acc();
  };

  // EPI 1: dgrad output columns [bnb_c0, bnb_c1) are the gradient g of a folded BN
  // output whose backward coefficients are known (consumer-derived sums): store
  // dz = [r>0]*(a*g - b*r + e) of the bf16-rounded g (as cnnitmo_bn_bwd_apply does)
  // into bnb_out and its column sums (by pixel parity) into stats rows; the other
  // columns are stored as g.  Works in the 16-byte piece layout of the store loop:
  // lane l always owns piece column cc = l % CPRP and pixel-column parity
  // (l / CPRP) & 1 (CPRP = CPR rounded up to a power of 2, x0 even); the pixel-row parity of its i-th piece
  // is compile-time (y0, oh0 even).  The r pieces are loaded first and waited for
  // with vmcnt(0) after the C tile is staged (that also retires the in-flight
  // prefetch of the next item).
  static_assert(EPI == 0 || (MODE == 0 && TH % 2 == 0 && TW % 2 == 0 && RPW % 2 == 0), "EPI 1 layout");
  constexpr int NPC = EPI ? RPW * TW * CPRP / 64 : 1;  // pieces per lane (lanes with cc >= CPR idle)
  constexpr int PXS = 64 / CPRP;                       // pixel step between a lane's pieces
  static_assert(EPI == 0 || TW % PXS == 0, "row parity per piece");
  // r pieces and coefficients of the item being stored
  uint4 rv[NPC];
  float ca[8], cb[8], ce[8];
  auto bnb_prefetch = [&](const Pos& e) {
    const int x0 = e.x0, oh0 = e.y0 + wave * RPW;
    const int cc = lane % CPRP, n = e.nb * BN + cc * 8;
    const int c0 = p.bnb_c0, cbn = p.bnb_c1 - p.bnb_c0;
    const bool fz = cc < CPR && n >= c0 && n < p.bnb_c1;
    const int nz = fz ? n - c0 : 0;
    const bf16* __restrict__ R = (const bf16*)p.bnb_r;
#pragma unroll
    for (int i = 0; i < NPC; ++i) {
      const int px = lane / CPRP + PXS * i;
      const int rr = px / TW, col = px - rr * TW, oh = oh0 + rr;
      const bool ok = fz && oh < p.ho && x0 + col < p.wo;
      const long m = ((long)e.img * p.ho + oh) * p.wo + x0 + col;
      rv[i] = *reinterpret_cast<const uint4*>(ok ? (const void*)(R + (size_t)m * p.bnb_r_ld + p.bnb_r_off + nz)
                                                 : (const void*)h_zero_page);
    }
    const float* cp = p.bnb_coef + nz;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ca[k] = fz ? cp[k] : 0.f;
      cb[k] = fz ? cp[cbn + k] : 0.f;
      ce[k] = fz ? cp[2 * cbn + k] : 0.f;
    }
  };
  auto epilogue_bnb = [&](const Pos& e, int buf) {
    bnb_prefetch(e);  // (issuing these before the item's last compute measured slower)
    const int img = e.img, y0 = e.y0, x0 = e.x0;
    const int n0 = e.nb * BN;
    const int oh0 = y0 + wave * RPW;
    char* cbase = C::C_IN_STAGE ? smem + buf * STAGE : smem + C::C_OFF;
    bf16* Cs = reinterpret_cast<bf16*>(cbase) + wave * RPW * TW * C::CLD;
    float* red = reinterpret_cast<float*>(cbase + C::C_BYTES);  // [NWAVE][BN][4]
    const int cc = lane % CPRP, n = n0 + cc * 8;
    const bool on = cc < CPR;  // BN = 48: 6 of every 8 lanes
    const int c0 = p.bnb_c0, cbn = p.bnb_c1 - p.bnb_c0;
    const bool fz = on && n >= c0 && n < p.bnb_c1;
    const int nz = fz ? n - c0 : 0;
    // g -> LDS (bf16) in the MFMA layout
#pragma unroll
    for (int j = 0; j < FN; ++j)
#pragma unroll
      for (int f = 0; f < FM; ++f)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int rr = f / FMR, col = (f % FMR) * 16 + (lane >> 4) * 4 + r;
          Cs[(rr * TW + col) * C::CLD + j * 16 + (lane & 15)] = from_f32<bf16>(acc[f][j][r]);
        }
    __syncthreads();
    wait_vm<0>();
    float sm[2][8];  // [pixel-row parity][channel] sums of this lane's (column-parity) pixels
#pragma unroll
    for (int k = 0; k < 8; ++k) sm[0][k] = sm[1][k] = 0.f;
    bf16* __restrict__ O = (bf16*)p.out;
    bf16* __restrict__ Z = (bf16*)p.bnb_out;
#pragma unroll
    for (int i = 0; i < NPC; ++i) {
      const int px = lane / CPRP + PXS * i;
      const int rr = px / TW, col = px - rr * TW, oh = oh0 + rr;
      const int rp = ((PXS * i) / TW) & 1;  // compile-time row parity of this piece
      const bool valid = on && oh < p.ho && x0 + col < p.wo;
      const long m = ((long)img * p.ho + oh) * p.wo + x0 + col;
      uint4 v = *reinterpret_cast<const uint4*>(Cs + px * C::CLD + (on ? cc : 0) * 8);
      if (fz) {
        const bf16* gv = reinterpret_cast<const bf16*>(&v);
        const bf16* rq = reinterpret_cast<const bf16*>(&rv[i]);
        uint4 o;
        bf16* ov = reinterpret_cast<bf16*>(&o);
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float g = to_f32(gv[k]), r = to_f32(rq[k]);
          const bf16 d = from_f32<bf16>(r > 0.f ? ca[k] * g - cb[k] * r + ce[k] : 0.f);
          ov[k] = d;
          sm[rp][k] += valid ? to_f32(d) : 0.f;
        }
        v = o;
      }
      uint4* dst = !valid ? h_sink + lane
                   : fz   ? reinterpret_cast<uint4*>(Z + (size_t)m * cbn + nz)
                          : reinterpret_cast<uint4*>(O + (size_t)m * p.out_ld + p.out_off + n);
      *dst = v;
    }
    // lanes sharing (cc, column parity) differ in lane bits >= log2(2*CPRP)
#pragma unroll
    for (int o = 2 * CPRP; o < 64; o <<= 1)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        sm[0][k] += __shfl_xor(sm[0][k], o, 64);
        sm[1][k] += __shfl_xor(sm[1][k], o, 64);
      }
    if (lane < 2 * CPRP && on) {
      const int cp = lane / CPRP;  // pixel-column parity
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        red[(wave * BN + cc * 8 + k) * 4 + 0 * 2 + cp] = sm[0][k];
        red[(wave * BN + cc * 8 + k) * 4 + 1 * 2 + cp] = sm[1][k];
      }
    }
    __syncthreads();
    if (tid < C::SG * BN) {
      const int g = tid / BN, col = tid - g * BN;
      const int nn = n0 + col;
      constexpr int WPG = NWAVE / C::SG;
      if (nn >= c0 && nn < p.bnb_c1) {
        float t[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int w = 0; w < WPG; ++w)
#pragma unroll
          for (int k = 0; k < 4; ++k) t[k] += red[((g * WPG + w) * BN + col) * 4 + k];
        const long tile = ((long)img * h.tiles_y + y0 / TH) * h.tiles_x + x0 / TW;
        const long row = tile * C::SG + g;
        if (p.bnb_par) {
          float* st = p.stats + (size_t)row * 4 * cbn + (nn - c0);
#pragma unroll
          for (int k = 0; k < 4; ++k) st[(size_t)k * cbn] = t[k];
        } else {
          p.stats[(size_t)row * cbn + (nn - c0)] = (t[0] + t[1]) + (t[2] + t[3]);
        }
      }
    }
    zero_acc();
  };

  // ST-stage ring over items.  vmcnt retires in issue order and counts the
  // epilogue's global stores too, so the wave tracks how many vector-memory ops
  // it issued after the loads of the item it is about to consume and waits for
  // exactly the older ones (the younger loads and stores stay in flight).  The
  // count is a lower bound for waves whose stats stores were exec-masked off,
  // which only makes their wait stricter.
  // output store instructions per wave
  constexpr int NST = EPI ? RPW * TW * CPRP / 64 : (REG ? FM * FN : (RPW * TW * CPR + 63) / 64);
  static_assert(RPW * TW * CPR % 64 == 0, "every lane issues the same number of stores");
  // BN partial sums are stored by threads tid < SG*BN: waves 0 .. (SG*BN-1)/64
  // EPI 1: the sums stores are not counted (an undercount only makes a wait stricter)
  const int S = NST + ((!EPI && stats && wave * 64 < C::SG * BN) ? 2 : 0);
  Pos ep = ip;  // position of the item being computed
  int issued = 0;
  int mq[ST];  // mq[k]: value of `issued` right after the loads of item t+k
#pragma unroll
  for (int k = 0; k < ST - 1; ++k) {
    mq[k] = issued;
    if (k < T) {
      issue_prep(k);
#pragma unroll
      for (int q = 0; q < L; ++q) issue_piece(q);
      step(ip);
      issued += L;
      mq[k] = issued;
    }
  }
  mq[ST - 1] = issued;
  int buf = 0;  // stage of item t
  for (long t = 0; t < T; ++t) {
    if constexpr (HALO_EXP != 1 && HALO_EXP != 4) wait_vm_dyn(issued - mq[0]);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    const bool pf = t + ST - 1 < T;
    if (pf) issue_prep(buf == 0 ? ST - 1 : buf - 1);  // stage (t + ST - 1) % ST
    compute(buf, pf);  // issues those loads between its taps
    if (pf) {
      step(ip);
      issued += L;
      mq[ST - 1] = issued;
    }
    if (ep.ch == nch - 1) {
      // every wave is done reading this stage: reuse it for the C tile (REG: no C tile)
      if constexpr (HALO_EXP != 7 && !REG) __syncthreads();
      if constexpr (HALO_EXP == 3) {
        if (p.N < 0) {  // never: keeps the MFMA results alive
          float t = 0.f;
#pragma unroll
          for (int i = 0; i < FM; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) t += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
          ((float*)p.out)[tid] = t;
        }
        zero_acc();
      } else {
        if constexpr (EPI == 1) epilogue_bnb(ep, buf);
        else if constexpr (REG) epilogue_reg(ep, buf);
        else epilogue(ep, buf);
        issued += S;
      }
    }
    step(ep);
#pragma unroll
    for (int k = 0; k < ST - 1; ++k) mq[k] = mq[k + 1];
    buf = buf == ST - 1 ? 0 : buf + 1;
  }
}

template <int MODE, int TH, int TW, int BN, int EPI = 0>
void launch_cfg(const HaloArgs& h, hipStream_t s) {
  // one workgroup per CU (LDS-limited); as many ring stages as fit in 160 KB
  const dim3 grid((unsigned)((h.npairs + h.per_block - 1) / h.per_block));
  const dim3 block((HaloCfg<MODE, TH, TW, BN, 2, EPI>::NT));
  if constexpr (HaloCfg<MODE, TH, TW, BN, 5, EPI>::SMEM <= 160 * 1024)
    hipLaunchKernelGGL((halo_gemm_kernel<MODE, TH, TW, BN, 5, EPI>), grid, block, 0, s, h);
  else if constexpr (HaloCfg<MODE, TH, TW, BN, 3, EPI>::SMEM <= 160 * 1024)
    hipLaunchKernelGGL((halo_gemm_kernel<MODE, TH, TW, BN, 3, EPI>), grid, block, 0, s, h);
  else
    hipLaunchKernelGGL((halo_gemm_kernel<MODE, TH, TW, BN, 2, EPI>), grid, block, 0, s, h);
}

int halo_cfg_env() {
  static const int v = [] {
    const char* e = getenv("CNNITMO_HALO_CFG");
    return e ? atoi(e) : 0;
  }();
  return v;
}

struct HaloPlan {
  int mode, bn, th, tw, epi;
};

// mode 0: conv3x3 stride 1 ('same'); mode 1: tconv2x2 s2 forward (pixel scatter)
bool halo_plan(const FwdArgs& a, HaloPlan& pl) {
  static const int en = [] {
    const char* e = getenv("CNNITMO_HALO");
    return e ? atoi(e) : 1;
  }();
  if (!en) return false;
  if (a.cin % 32 || a.a_ld % 8 || a.a_off % 8 || a.out_ld % 8 || a.out_off % 8) return false;
  pl.epi = 0;
  if (a.bnb_out) {  // fused BN backward: conv3x3 dgrad, 16x32 tiles, BN 64 / 32
    if (a.ntaps != 9 || a.scale != 1 || a.scatter || a.hs != a.ho || a.ws != a.wo) return false;
    if (a.bnb_c0 % 8 || a.bnb_c1 % 8 || a.bnb_c0 < 0 || a.bnb_c1 > a.N || a.bnb_c0 >= a.bnb_c1 ||
        a.bnb_r_ld % 8 || a.bnb_r_off % 8)
      return false;
    pl.mode = 0;
    pl.epi = 1;
    pl.bn = a.N % 64 == 0 ? 64 : (a.N % 48 == 0 ? 48 : (a.N % 32 == 0 ? 32 : 0));
    pl.th = 16;
    pl.tw = 32;
    return pl.bn != 0;
  }
  if (a.ntaps == 9 && a.scale == 1 && !a.scatter && a.hs == a.ho && a.ws == a.wo) {
    pl.mode = 0;
    static const int force = [] {
      const char* e = getenv("CNNITMO_HALO_BN");
      return e ? atoi(e) : 0;
    }();
    if (force == 32 && a.N % 32 == 0) pl.bn = 32;
    else pl.bn = a.N % 64 == 0 ? 64 : (a.N % 48 == 0 ? 48 : (a.N % 32 == 0 ? 32 : 0));
    if (!pl.bn) return false;
    // tile: 0 = 4x64 (4 waves), 1 = 8x32 (8 waves), 2 = 8x64 (8 waves, BN = 32 only),
    //       3 = 16x32 (8 waves x 2 rows: twice the pixels per weight-tile load)
    const int e = halo_cfg_env();
    int shape = 3;  // measured fastest for every BN (tools/bench_layers.py)
    if (e >= 1 && e <= 4 && (e != 3 || pl.bn == 32)) shape = e - 1;
    pl.th = shape == 0 ? 4 : (shape == 3 ? 16 : 8);
    pl.tw = (shape == 1 || shape == 3) ? 32 : 64;
    return true;
  }
  if (a.ntaps == 1 && a.scale == 1 && a.scatter && a.hs == a.ho && a.ws == a.wo && a.cout % 32 == 0 &&
      a.N == 4 * a.cout) {
    pl.mode = 1;
    static const int m1bn = [] {
      const char* e = getenv("CNNITMO_HALO_M1BN");
      return e ? atoi(e) : 128;
    }();
    pl.bn = m1bn == 64 ? 64 : 128;  // a block may span taps: pieces are scattered one by one
    pl.th = 8;
    pl.tw = 32;
    return true;
  }
  return false;
}

}  // namespace

bool halo_handles(const FwdArgs& a) {
  HaloPlan pl;
  return halo_plan(a, pl);
}

int launch_halo(FwdArgs a, hipStream_t s, const char* what) {
  HaloPlan pl;
  CNN_REQUIRE(halo_plan(a, pl), "%s: no halo plan", what);
  HaloArgs h;
  h.f = a;
  h.f.nblocks = a.N / pl.bn;
  h.tiles_x = (a.wo + pl.tw - 1) / pl.tw;  // partial edge tiles are masked
  h.tiles_y = (a.ho + pl.th - 1) / pl.th;
  h.nchunks = a.cin / 32;
  const long tiles = (long)a.nimg * h.tiles_x * h.tiles_y;
  h.npairs = tiles * h.f.nblocks;
  CNN_REQUIRE(h.npairs * h.nchunks < (1L << 31), "%s: too many tiles", what);
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      ncu = prop.multiProcessorCount;
    if (ncu <= 0) ncu = 256;
  }
  h.per_block = (h.npairs + ncu - 1) / ncu;
  CNN_REQUIRE(!(a.flags & CNNITMO_STATS) || a.stats, "%s: STATS without buffer", what);
  if (pl.epi == 1) {
    if (pl.bn == 64) launch_cfg<0, 16, 32, 64, 1>(h, s);
    else if (pl.bn == 48) launch_cfg<0, 16, 32, 48, 1>(h, s);
    else launch_cfg<0, 16, 32, 32, 1>(h, s);
  } else if (pl.mode == 1) {
    if (pl.bn == 128) launch_cfg<1, 8, 32, 128>(h, s);
    else launch_cfg<1, 8, 32, 64>(h, s);
  } else if (pl.th == 4) {
    if (pl.bn == 64) launch_cfg<0, 4, 64, 64>(h, s);
    else if (pl.bn == 48) launch_cfg<0, 4, 64, 48>(h, s);
    else launch_cfg<0, 4, 64, 32>(h, s);
  } else if (pl.th == 16) {
    if (pl.bn == 64) launch_cfg<0, 16, 32, 64>(h, s);
    else if (pl.bn == 48) launch_cfg<0, 16, 32, 48>(h, s);
    else launch_cfg<0, 16, 32, 32>(h, s);
  } else if (pl.tw == 32) {
    if (pl.bn == 64) launch_cfg<0, 8, 32, 64>(h, s);
    else if (pl.bn == 48) launch_cfg<0, 8, 32, 48>(h, s);
    else launch_cfg<0, 8, 32, 32>(h, s);
  } else {
    launch_cfg<0, 8, 64, 32>(h, s);
  }
  return cnnitmo_check_launch(what);
}

const char* halo_name(const FwdArgs& a) {
  HaloPlan pl;
  if (!halo_plan(a, pl)) return "";
  static thread_local char buf[64];
  snprintf(buf, sizeof(buf), "halo_gemm_kernel<%d,%d,%d,%d%s>", pl.mode, pl.th, pl.tw, pl.bn,
           pl.epi ? ",bnb" : "");
  return buf;
}

// BN partial-sum rows written by the halo kernel: one per 256 GEMM rows of each
// (possibly partial) tile.
long halo_stat_rows(const FwdArgs& a) {
  HaloPlan pl;
  if (!halo_plan(a, pl)) return 0;
  const long tiles = (long)a.nimg * ((a.ho + pl.th - 1) / pl.th) * ((a.wo + pl.tw - 1) / pl.tw);
  return tiles * (pl.th * pl.tw / 256);
}
