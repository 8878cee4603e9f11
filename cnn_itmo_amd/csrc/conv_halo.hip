// 3x3 'same' convolution, forward and input-gradient, bf16: every U-Net 3x3
// layer from enc1b on (model.py:196 Conv2D(filters, 3, padding='same') -> ReLU
// -> BatchNormalization, and its input gradient); and the fp32 inference forward
// (predict.py:62 at fp32) with 16-channel chunks.
//
// GEMM view: rows = output pixels, columns = output channels (N), K = 9 taps x
// Cin.  A workgroup owns a 16 x 32 output tile and a block of BN columns.  Per
// 32-channel chunk it stages the (16+2) x (32+2) input halo ONCE in LDS
// (LDS-DMA) together with the chunk's 9 x BN x 32 weights; the nine taps are
// nine shifted windows of the same halo image:
//   pixel fragment (tap r,s; tile row y, 16 columns x..x+15) =
//       patch rows (y + r) * 34 + x + s .. +15   (consecutive LDS rows, any start)
// LDS rows are 64 B (32 bf16); piece c of row q sits at piece c ^ (((q>>2)&1)<<1),
// conflict-free for ds_read_b128 windows starting at ANY row
// (tools/check_swizzle.py).  An ST-stage ring overlaps the DMA of item t+1 with
// the MFMAs of item t; vmcnt is counted per wave (it retires in issue order and
// also counts the epilogue's stores), so a wave waits for exactly the loads of
// the item it is about to consume.
//
// Work distribution (persistent: one 512-thread workgroup per CU, XCD-aware).
// The dispatcher deals blocks b, b+8, b+16, ... to one XCD; xcd_remap numbers
// them so that each XCD holds a contiguous range of logical ids, and consecutive
// ids form `streams` groups of `nblocks` workgroups: a stream walks a contiguous range of tiles
// (image -> column strip -> row, so consecutive tiles share halo rows) and each
// of its nblocks workgroups computes one BN-column block of every tile.  So the
// nblocks workgroups of a stream read the same halo at about the same time
// (one fabric read per XCD, L2 hits for the rest), a workgroup's weights are a
// fixed 1/nblocks slice, and its output columns never change: its epilogue
// parameters sit in LDS and its BN partial sums stay in registers for the whole
// launch (one partial-sum row per (stream, wave), rows = halo_stat_rows).
//
// MFMA 16x16x32 bf16 with the operands swapped (C^T = W^T X^T): a lane ends up
// with one pixel and 4 consecutive channels per fragment.  The weight rows are
// permuted inside each 32-column pair of fragments (pair_perm, igemm_common.h) so that a lane's
// two fragments hold 8 CONSECUTIVE channels: one 16-byte store per (pixel, 8
// channels) straight from registers, no C tile in LDS, no barrier in the
// epilogue.
//
// EPI 0: store g (input gradient).  EPI 1: forward epilogue: bias, folded-BN
// zero-padding border correction, ReLU, inference affine, BN partial sums (by
// flags).  EPI 2: input gradient with the producer's BN backward fused (FwdArgs
// bnb_*): columns [c0, c1) become dz = [r>0]*(a*g - b*r + e) of the bf16-rounded
// g (as cnnitmo_bn_bwd_apply computes it) plus sums of dz by pixel parity; the
// other columns are stored as g.
#include <cstdio>
#include <type_traits>

#include "dma.h"
#include "igemm_common.h"

namespace {

using dma::OOB;

// 8 waves (2 per SIMD, 64 x BN wave tiles).  (Measured and removed: one wave per SIMD with
// 128 x BN wave tiles and AGPR accumulators, 8-10 % slower on every layer; the fused dgrad's
// r loads issued during the last tap with the sums in LDS slots, 15-20 % slower; whole-line
// epilogue stores, neutral; 8-row tiles for dec9's forward with all weights resident, 2 %
// slower)
constexpr int TH = 16, TW = 32, NWAVE = 8, NT = NWAVE * 64;
constexpr int RPW = TH / NWAVE, FMR = TW / 16, FM = RPW * FMR;  // tile rows / fragments per wave
constexpr int KT = 9, PW = TW + 2, PROWS = (TH + 2) * PW;         // halo patch: 18 x 34 rows of 64 B
constexpr int PPC = (PROWS + 15) / 16;                            // patch pieces (1 KiB = 16 rows)
constexpr int NPI = (PPC + NWAVE - 1) / NWAVE;                    // patch pieces per wave
// taps over which the next item's DMA pieces are issued (3 and 8 measured no better,
// profiles/r02l_ab_halo_knobs.txt)
constexpr int PFT = 5;

// RES: the workgroup's weights for the whole K (at most RCH chunks) stay resident in
// LDS, loaded once per launch; a ring stage then holds the halo patch only.  For the
// small-K layers (cin <= 64: level 1 and 2) the per-item weight pieces were half of
// every stage's DMA.
constexpr int RCH = 2;
template <int BN, bool RES, int THT = 16> struct HCfg {
  static constexpr int RCH = ::RCH;
  static constexpr int PPC = ((THT + 2) * PW + 15) / 16, NPI = (PPC + NWAVE - 1) / NWAVE;
  static constexpr int FN = BN / 16, FP = FN / 2;        // fragments / 32-column pairs
  static constexpr int BPC = KT * BN / 16;               // weight pieces
  static constexpr int NBI = (BPC + NWAVE - 1) / NWAVE;  // weight pieces per wave
  static constexpr int L = RES ? NPI : NPI + NBI;        // DMA instructions per wave per item
  static constexpr int PATCH = PPC * 1024;
  static constexpr int STAGE = RES ? PATCH : PATCH + BPC * 1024;
  static constexpr int ST = 2;
  static constexpr int WRES = ST * STAGE;                   // resident weights (RES)
  static constexpr int SCR = WRES + (RES ? RCH * BPC * 1024 : 0);  // 1 KiB sink for the padding pieces
  static constexpr int PAR = SCR + 1024;    // [4][BN] fp32 epilogue parameters (bias, scale, shift, pool mode)
  static constexpr int UTB = PAR + 4 * BN * 4;  // [BN][8] fp32 border table
  static constexpr int SMEM = UTB + BN * 8 * 4;
  static constexpr int NST = (THT / NWAVE) * FMR * FP;  // 16-byte stores per wave per epilogue
  static_assert(SMEM <= 160 * 1024, "LDS");
  static_assert(BN % 32 == 0, "column pairs");
};


// row_ror:N within each 16-lane row (DPP)
template <int N> __device__ __forceinline__ float dpp_ror(float x) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(x), 0x120 + N, 0xF, 0xF, false));
}

// store sink for EPI 2's out-of-image pixels (global stores, fixed count per wave)
__device__ __attribute__((aligned(256))) uint4 h_sink[64];

struct HaloArgs {
  FwdArgs f;
  int tiles_x, tiles_y, nchunks, nblocks, streams;
  long tiles;
};

// TE = bf16 (every launch of the training step) or float (the fp32 inference forward,
// EPI 1 only).  An LDS row is 64 B either way: CC = 32 bf16 or 16 fp32 channels per
// chunk, and one 16-byte piece is PE = 8 or 4 channels; Mma<float> runs a 16-byte
// fragment as four 16x16x4 f32 MFMAs, so the fragment reads, the swizzle and the
// operand-swapped register layout are the same.  fp32 stores take two 16-byte stores per
// (pixel, 8 channels).
// POOL (EPI 1): the 2x2 MaxPooling2D of the stored output rides on the epilogue (SURVEY 7,
// hard part 2): a wave's two tile rows are a row of 2x2 windows and the window's right
// column is the neighbouring lane (DPP quad_perm xor 1), so the even lanes write the
// pooled value and its window index (first maximum, window order (0,0),(0,1),(1,0),(1,1),
// on the values as stored).  Training stores r = relu(conv) with the BN folded into the
// consumers; y = r*s + h is monotone in r with the sign of s = gamma * invstd, i.e. of gamma
// (known before the batch statistics), so the pooled y is s * (max r) + h where gamma > 0
// and s * (min r) + h where gamma < 0: the kernel pools r by the per-channel mode sign(gamma)
// (pool_sign), and the pooled value is itself a folded value.  Inference stores y (AFFINE)
// and pools it by its maximum.
// ALT, EPI 1 (NOSUM): no BN partial sums (the inference forward): the 2 x FP x 8 accumulators live
// across the whole launch otherwise.  ALT, EPI 2 (ALLF): every column is BN-fused (c0 = 0, c1 = N),
// or (bf16, streamed weights) c0 is a multiple of BN and c1 = N, so that a column block is fused or
// plain as a whole (dec6's [skip 256 | up 512]): the epilogue has no per-column branch.  A per-lane
// `fused` test in the value loop compiles to an exec-mask branch per value (about ten scalar
// instructions each, 91 such branches per epilogue); the ALLF epilogue stores through raw-buffer
// offsets from the wave's first pixel.
// POOL (EPI 2): the deferred MaxPooling2D backward of the producer's output rides on the fused BN
// backward (cnnitmo_conv3x3_dgrad_bn_pooled): every column is BN-fused, and the gradient the
// dgrad computes (the concat skip path) is first increased by the pooled gradient routed to this
// pixel by the window indices (pool_out = dy_pool, pool_idx; the pool's [n][ho/2][wo/2][N]).  A
// wave's two tile rows are one row of 2x2 windows, so a lane's window position is
// (tile row, pixel-column parity) and the pooled row it reads is shared by both rows.
template <typename TE, int BN, int EPI, bool RES, bool POOL = false, int THT = 16, bool ALT = false>
__global__ __launch_bounds__(NT) void halo_conv_kernel(const HaloArgs h) {
  constexpr bool NOSUM = EPI == 1 && ALT, ALLF = EPI == 2 && ALT;
  using C = HCfg<BN, RES, THT>;
  constexpr int TH = THT, RPW = TH / NWAVE, FM = RPW * FMR, PROWS = (TH + 2) * PW;  // (shadow the 16-row defaults)
  constexpr int PPC = C::PPC, NPI = C::NPI;
  static_assert(RPW >= 1, "a tile row per wave at least");
  constexpr int FN = C::FN, FP = C::FP, L = C::L, NBI = C::NBI, STAGE = C::STAGE, ST = C::ST;
  constexpr int ES = sizeof(TE), CC = 64 / ES, PE = 16 / ES;
  static_assert(!POOL || ((EPI == 1 || EPI == 2) && RPW == 2), "pooling: whole window rows per wave");
  // stores per wave per epilogue (+ POOL: a value and an index store per window row and column block)
  // (EPI 3: three 4-byte yhat stores per fragment instead of the output rows)
  constexpr int NST = EPI == 3 ? FM * 3
                               : C::NST * (ES == 4 ? 2 : 1) + (POOL && EPI == 1 ? FP * (RPW / 2) * FMR * (ES == 4 ? 3 : 2) : 0);
  constexpr int SMEM = C::SMEM;
  static_assert(SMEM <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[SMEM];
  const FwdArgs& p = h.f;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR) for the vmcnt switch
  // logical id: contiguous per XCD (xcd_remap), so a stream's workgroups share one
  // XCD's L2 except where a stream straddles two XCDs
  const int lid = xcd_remap(blockIdx.x, gridDim.x);
  const int nb = lid % h.nblocks, gs = lid / h.nblocks;
  if (gs >= h.streams) return;  // the leftover workgroups (< nblocks) own nothing
  const long nstr = h.streams;
  const long t0 = h.tiles * gs / nstr, t1 = h.tiles * (gs + 1) / nstr;
  const int nch = h.nchunks;
  const long T = (t1 - t0) * nch;
  const int n0 = nb * BN;
  const int K = KT * p.cin;
  const int tpi = h.tiles_x * h.tiles_y;
  const TE* __restrict__ X = (const TE*)p.a;
  const TE* __restrict__ Wt = (const TE*)p.b;
  float* par = reinterpret_cast<float*>(smem + C::PAR);
  float* utb = reinterpret_cast<float*>(smem + C::UTB);
  // the workgroup's epilogue parameters (ordered before any epilogue by the ring barrier)
  if constexpr (EPI == 1 || EPI == 3) {
    const bool aff = p.flags & CNNITMO_AFFINE;
    for (int i = tid; i < 4 * BN; i += NT) {
      const int k = i / BN, c = n0 + i % BN;
      const float sg = k == 3 && p.pool_sign ? p.pool_sign[c] : 1.f;
      par[i] = k == 0 ? (p.bias ? p.bias[c] : 0.f) : k == 1 ? (aff ? p.aff_scale[c] : 1.f)
             : k == 2 ? (aff ? p.aff_shift[c] : 0.f) : (sg > 0.f ? 1.f : (sg < 0.f ? -1.f : 0.f));
    }
    if constexpr (EPI == 3) {  // the head: weights [3][BN] and bias [3] over the border table
      for (int i = tid; i < 3 * BN + 3; i += NT) utb[i] = i < 3 * BN ? p.head_w[i] : p.head_b[i - 3 * BN];
    } else {
      for (int i = tid; i < 8 * BN; i += NT) utb[i] = p.border ? p.border[(size_t)n0 * 8 + i] : 0.f;
    }
  } else if constexpr (EPI == 2) {
    const int cbn = p.bnb_c1 - p.bnb_c0;
    for (int i = tid; i < 3 * BN; i += NT) {
      const int k = i / BN, c = n0 + i % BN;
      // (ALLF: a plain column gets a = 1, b = e = 0, so the fused expression stores g itself)
      par[i] = (c >= p.bnb_c0 && c < p.bnb_c1) ? p.bnb_coef[k * cbn + c - p.bnb_c0] : (ALLF && k == 0 ? 1.f : 0.f);
    }
  }

  // item position: (image, tile row, tile column, chunk); tile rows fastest
  struct Pos {
    int img, y0, x0, ch;
  };
  Pos ip;
  {
    const long tile = t0;  // < 2^31 (checked by the launcher)
    ip.img = (int)(tile / tpi);
    const int rem = (int)(tile - (long)ip.img * tpi);
    const int txi = rem / h.tiles_y;
    ip.y0 = (rem - txi * h.tiles_y) * TH;
    ip.x0 = txi * TW;
    ip.ch = 0;
  }
  Pos ep = ip;  // position of the item being computed (the ring below advances ip ahead of it)
  auto step = [&](Pos& s) {
    if (++s.ch < nch) return;
    s.ch = 0;
    s.y0 += TH;
    if (s.y0 < p.ho) return;
    s.y0 = 0;
    s.x0 += TW;
    if (s.x0 < p.wo) return;
    s.x0 = 0;
    ++s.img;
  };

  // per-lane DMA geometry, fixed for the launch: one instruction = 16 LDS rows x
  // 4 pieces of 16 B; lane -> (row, piece), source piece swizzled
  const int lrow = lane >> 2, lpc = lane & 3;
  int ppy[NPI], ppx[NPI];
  // EPI 1 (two-source capable): 4 * (source pixel offset from the patch origin) + swizzled
  // piece, the row pitch chosen per chunk; otherwise the byte offset of the lane's piece
  unsigned pkey[NPI];
#pragma unroll
  for (int i = 0; i < NPI; ++i) {
    const int row = (wave * NPI + i) * 16 + lrow;
    const int piece = lpc ^ (((row >> 2) & 1) << 1);
    const int py = row / PW, px = row - (row / PW) * PW;
    ppy[i] = row < PROWS ? py - 1 : -(1 << 29);  // padding rows: never in bounds
    ppx[i] = px - 1;
    pkey[i] = EPI == 1 ? (unsigned)((py * p.ws + px) * 4 + piece)
                       : (unsigned)((((long)py * p.ws + px) * p.a_ld + piece * PE) * ES);
  }
  // the source of a chunk: a (channels < cin1 or a single source) or a2
  const TE* __restrict__ X2 = (const TE*)p.a2;
  const int cin1 = p.a2 ? p.cin1 : p.cin;
  unsigned boff[NBI];
#pragma unroll
  for (int i = 0; i < NBI; ++i) {
    const int row = (wave * NBI + i) * 16 + lrow;  // = tap * BN + nn
    const int piece = lpc ^ (((row >> 2) & 1) << 1);
    const int tap = row / BN, nn = row - (row / BN) * BN;
    boff[i] = row < KT * BN ? (unsigned)((pair_perm(nn) * K + tap * p.cin + piece * PE) * ES) : OOB;
  }
  uintptr_t pbase = 0, bbase = 0;
  char* iPs = smem;
  unsigned pvo[NPI];
  // the tile's patch origin in each source (64-bit products), recomputed at its first chunk only;
  // a chunk then adds its channel offset
  uintptr_t tb1 = 0, tb2 = 0;
  const uintptr_t wb0 = (uintptr_t)(Wt + (size_t)n0 * K);
  auto issue_prep = [&](int buf) {
    const Pos& s = ip;
    iPs = smem + buf * STAGE;
    const int c = s.ch * CC;
    if (s.ch == 0) {
      const long po = ((long)s.img * p.hs + s.y0 - 1) * p.ws + s.x0 - 1;  // patch origin pixel (may be < 0)
      tb1 = (uintptr_t)X + (uintptr_t)((po * p.a_ld + p.a_off) * ES);
      if constexpr (EPI == 1) tb2 = (uintptr_t)X2 + (uintptr_t)((po * p.a2_ld + p.a2_off - cin1) * ES);
    }
    bbase = wb0 + (uintptr_t)(c * ES);
    if constexpr (EPI == 1) {
      const bool second = c >= cin1;
      const long ld = second ? p.a2_ld : p.a_ld;
      pbase = (second ? tb2 : tb1) + (uintptr_t)(c * ES);
#pragma unroll
      for (int i = 0; i < NPI; ++i) {
        const int yy = s.y0 + ppy[i], xx = s.x0 + ppx[i];
        const bool ok = (unsigned)yy < (unsigned)p.hs && (unsigned)xx < (unsigned)p.ws;
        // (any offset with the top bit set is out of range: OR-ing it in keeps this branch-free)
        pvo[i] = ((pkey[i] >> 2) * (unsigned)ld + (pkey[i] & 3) * PE) * ES | (ok ? 0u : OOB);
      }
    } else {
      pbase = tb1 + (uintptr_t)(c * ES);
#pragma unroll
      for (int i = 0; i < NPI; ++i) {
        const int yy = s.y0 + ppy[i], xx = s.x0 + ppx[i];
        const bool ok = (unsigned)yy < (unsigned)p.hs && (unsigned)xx < (unsigned)p.ws;
        pvo[i] = ok ? pkey[i] : OOB;
      }
    }
  };
  auto issue_piece = [&](int k) {  // k: compile-time after unrolling
    if (k < NPI) {
      const int gp = wave * NPI + k;
      dma::lds16(pvo[k], dma::rsrc(pbase), gp < PPC ? iPs + gp * 1024 : smem + C::SCR);
    } else if constexpr (!RES) {
      const int gp = wave * NBI + (k - NPI);
      dma::lds16(boff[k - NPI], dma::rsrc(bbase), gp < C::BPC ? iPs + C::PATCH + gp * 1024 : smem + C::SCR);
    }
  };

  f32x4 acc[FM][FN];
  auto zero_acc = [&]() {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero_acc();

  // fragment-read addresses: window row = rbase + c, c = r*PW + 16i + s compile-time;
  // the swizzle bit of (rbase + c) depends only on c & 7
  const int frow = lane & 15, fpc = lane >> 4;
  const int rbase = wave * RPW * PW + frow;
  int apre[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) apre[k] = rbase * 64 + ((fpc ^ ((((rbase + k) >> 2) & 1) << 1)) << 4);
  const int bpre = frow * 64 + ((fpc ^ (((frow >> 2) & 1) << 1)) << 4);
  // Fragments are double-buffered across taps (tap t+1's ds_reads before tap t's
  // MFMAs, pinned by sched barriers); the next item's DMA pieces go out over the
  // first PFT taps.
  const int g = lane >> 4, pxl = lane & 15;  // channel group (8 channels per pair) / pixel of the fragment

  // EPI 2: r of the wave's pixels (base at its first pixel; byte offset per (fragment,
  // pair), OOB for out-of-image pixels and columns outside [c0, c1))
  auto r_base = [&](const Pos& e) {
    const long m0 = ((long)e.img * p.ho + e.y0 + wave * RPW) * p.wo + e.x0;
    return (const TE*)p.bnb_r + m0 * p.bnb_r_ld + p.bnb_r_off;
  };
  auto r_off = [&](const Pos& e, int f, int q) {
    const int c = n0 + 32 * q + 8 * g;
    const int rr = f / FMR, col = (f % FMR) * 16 + pxl;
    const bool ok = e.y0 + wave * RPW + rr < p.ho && e.x0 + col < p.wo && c >= p.bnb_c0 && c < p.bnb_c1;
    return ok ? (unsigned)((((long)rr * p.wo + col) * p.bnb_r_ld + (c - p.bnb_c0)) * ES) : OOB;
  };
  // EPI 2 + POOL: the pooled gradient and window indices of the lane's windows (both tile rows
  // of a wave share one pooled row): [column block][pair], 8 channels each
  constexpr int PRQ = POOL && EPI == 2 ? FMR : 1, PRP = POOL && EPI == 2 ? FP : 1;
  dma::i32x4 gpv[PRQ][PRP][ES == 4 ? 2 : 1];
  dma::i32x2 ipv[PRQ][PRP];
  auto load_route = [&](const Pos& e) {
    if constexpr (POOL && EPI == 2) {
      const int ho2 = p.ho / 2, wo2 = p.wo / 2;
      const size_t pb = (((size_t)e.img * ho2 + (e.y0 + wave * RPW) / 2) * wo2 + e.x0 / 2) * p.pool_ld + n0;
      const __amdgpu_buffer_rsrc_t gs = dma::brsrc((const TE*)p.pool_out + pb);
      const __amdgpu_buffer_rsrc_t is = dma::brsrc(p.pool_idx + pb);
      const bool rok = e.y0 + wave * RPW < p.ho;
#pragma unroll
      for (int cb = 0; cb < FMR; ++cb)
#pragma unroll
        for (int q = 0; q < FP; ++q) {
          const bool ok = rok && e.x0 + cb * 16 + pxl < p.wo;
          const unsigned o = (unsigned)((cb * 8 + (pxl >> 1)) * p.pool_ld + 32 * q + 8 * g);  // elements
#pragma unroll
          for (int h2 = 0; h2 < (ES == 4 ? 2 : 1); ++h2)
            gpv[cb][q][h2] = __builtin_amdgcn_raw_buffer_load_b128(gs, ok ? o * ES + 16 * h2 : OOB, 0, 0);
          ipv[cb][q] = __builtin_amdgcn_raw_buffer_load_b64(is, ok ? o : OOB, 0, 0);
        }
    }
  };
  // the routed pooled gradient of channels 8g..8g+7 of pair q for fragment f (window position
  // (tile row, pixel-column parity)): added to the dgrad's value
  auto routed = [&](int f, int q, float* gr) {
    if constexpr (POOL && EPI == 2) {
      const int rr = f / FMR, cb = f % FMR;
      const unsigned k = (unsigned)(rr * 2 + (pxl & 1));
      const unsigned i0 = (unsigned)ipv[cb][q][0], i1 = (unsigned)ipv[cb][q][1];
      float gv[8];
      if constexpr (ES == 2) {
        const bf16x8 b8 = __builtin_bit_cast(bf16x8, gpv[cb][q][0]);
#pragma unroll
        for (int j = 0; j < 8; ++j) gv[j] = to_f32(b8[j]);
      } else {
        const f32x4 a = __builtin_bit_cast(f32x4, gpv[cb][q][0]), b = __builtin_bit_cast(f32x4, gpv[cb][q][1]);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          gv[j] = a[j];
          gv[4 + j] = b[j];
        }
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const unsigned ij = ((j < 4 ? i0 : i1) >> (8 * (j & 3))) & 0xFFu;
        gr[j] = ij == k ? gv[j] : 0.f;
      }
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) gr[j] = 0.f;
    }
  };
  // EPI 2 (bf16): r of the tile (and the routed pool gradient) for the fused BN backward.
  // EARLY (32-column blocks, whose registers have room for them): issued at the start of
  // the tile's last item, so that item's MFMAs cover their HBM latency; otherwise after the
  // MFMAs (the BN-64 kernels sit at 256 VGPRs).  Early vs late on the 32-column kernels:
  // 215.4 / 215.4 vs 215.4 / 213.9 frames/s (profiles/r05/r05d_ab_early_r.txt).
  // (r through the free ring stage by LDS-DMA during the tile's last item, the next tile's
  // first item loaded after the MFMAs, the epilogue reading r from LDS: 15-28 % slower on
  // every 64-column fused dgrad with streamed weights, profiles/r05/r05z10_ab_r_via_lds.txt;
  // without any epilogue these launches run 19-57 % faster, r05z8_probe_noepi2.txt.)
  // (An L2 touch of the r lines at the start of the tile's last item, one 4-byte LDS-DMA
  // per lane: 1-11 % slower on every 64-column fused dgrad, profiles/r05/r05z3_ab_r_touch.txt.)
  // (Single-buffered fragments on the 64-column kernels, which frees the registers for early
  // r loads: every 64-column fused dgrad 8-27 % slower, 218.0 -> 212.2 frames/s,
  // profiles/r05/r05q_ab_sb64_early_r.txt.)
  constexpr bool EARLY = EPI == 2 && ES == 2 && FP == 1;
  constexpr int NEARLY = FM * FP + (POOL && EPI == 2 ? 2 * FMR * FP : 0);  // loads per wave
  dma::i32x4 rv[EPI == 2 && ES == 2 ? FM : 1][EPI == 2 && ES == 2 ? FP : 1];
  auto load_r16 = [&](const Pos& e) {
    if constexpr (EPI == 2 && ES == 2) {
      const __amdgpu_buffer_rsrc_t rs = dma::brsrc(r_base(e));
#pragma unroll
      for (int f = 0; f < FM; ++f)
#pragma unroll
        for (int q = 0; q < FP; ++q) rv[f][q] = __builtin_amdgcn_raw_buffer_load_b128(rs, r_off(e, f, q), 0, 0);
      load_route(e);
    }
  };
  auto compute = [&](int buf, bool pf, int ch) {
    const char* Ps = smem + buf * STAGE;
    const char* Bs = RES ? smem + C::WRES + ch * (C::BPC * 1024) : Ps + C::PATCH;
    uint4 af[2][FM], bfr[2][FN];
    auto load = [&](int tap, int sl) {
      const int r = tap / 3, s = tap - 3 * (tap / 3);
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int c = (f / FMR + r) * PW + (f % FMR) * 16 + s;
        af[sl][f] = *reinterpret_cast<const uint4*>(Ps + apre[c & 7] + c * 64);
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) bfr[sl][j] = *reinterpret_cast<const uint4*>(Bs + bpre + (tap * BN + j * 16) * 64);
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
        for (int j = 0; j < FN; ++j) Mma<TE>::run(acc[i][j], bfr[cur][j], af[cur][i]);  // C^T: lanes = pixels
      if (pf) {
#pragma unroll
        for (int k = 0; k < L; ++k)
          if ((k * PFT) / L == tap) issue_piece(k);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // BN partial sums of the lane's pixels for its 8 channels of each pair (EPI 1), or
  // sums of dz by pixel-row parity (EPI 2; the lane's pixel-column parity is lane & 1)
  constexpr int NSUM = EPI == 0 || EPI == 3 || NOSUM ? 1 : FP;
  float sa[NSUM][8], sb[NSUM][8];
#pragma unroll
  for (int q = 0; q < NSUM; ++q)
#pragma unroll
    for (int k = 0; k < 8; ++k) sa[q][k] = sb[q][k] = 0.f;

  auto lds8 = [&](const float* src, float* v) {
    const float4 a = *reinterpret_cast<const float4*>(src), b = *reinterpret_cast<const float4*>(src + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w; v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  };
  auto pack8 = [&](const float* v) {
    bf16x8 o;
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = (bf16)v[k];
    return __builtin_bit_cast(dma::i32x4, o);
  };

  // EPI 0 / 1: stores through a buffer descriptor at the wave's first pixel (whole 128-byte
  // lines per store instruction measured neutral here: profiles/r03z_ab_halo_lines.txt)
  // the pooled training forward stores r with the BN folded into its consumers: no affine
  // epilogue (halo_plan), which keeps the bf16 BN-64 kernel from spilling
  constexpr bool AFFOK = !(POOL && !NOSUM);
  auto epilogue = [&](const Pos& e) {
    const int oh0 = e.y0 + wave * RPW;
    const TE* obase = (const TE*)p.out + (((size_t)e.img * p.ho + oh0) * p.wo + e.x0) * p.out_ld + p.out_off + n0;
    const __amdgpu_buffer_rsrc_t os = dma::brsrc(obase);
    const bool relu = p.flags & CNNITMO_RELU, aff = p.flags & CNNITMO_AFFINE;
    const bool bt = EPI == 1 && p.border && (oh0 == 0 || oh0 + RPW >= p.ho || e.x0 == 0 || e.x0 + TW >= p.wo);
    // POOL: the wave's pooled rows start at (oh0 / 2, x0 / 2) of the [n][ho/2][wo/2] output
    const size_t pofs = (((size_t)e.img * (p.ho / 2) + oh0 / 2) * (p.wo / 2) + e.x0 / 2) * p.pool_ld + n0;
    const __amdgpu_buffer_rsrc_t ps = dma::brsrc(POOL ? (const TE*)p.pool_out + pofs : obase);
    const __amdgpu_buffer_rsrc_t pis = dma::brsrc(POOL ? (const unsigned char*)p.pool_idx + pofs : (const unsigned char*)obase);
    // POOL: the running maximum of the lane's window (value and window index per channel)
    float pb[8];
    unsigned pa[2] = {0u, 0u};
    // EPI 3: the head's three dot products of each fragment's pixels, this lane's 16 channels
    float zf[EPI == 3 ? FM : 1][3];
    if constexpr (EPI == 3) {
#pragma unroll
      for (int f = 0; f < FM; ++f) zf[f][0] = zf[f][1] = zf[f][2] = 0.f;
    }
#pragma unroll
    for (int q = 0; q < FP; ++q) {
      const int cl = 32 * q + 8 * g;  // the lane's first column in the block
      float bj[8], sj[8], hj[8], md[8], hw[EPI == 3 ? 3 : 1][8];
      if constexpr (EPI == 1 || EPI == 3) {
        lds8(par + cl, bj);
        if constexpr (AFFOK) {
          lds8(par + BN + cl, sj);
          lds8(par + 2 * BN + cl, hj);
        }
      }
      if constexpr (EPI == 3) {
#pragma unroll
        for (int j = 0; j < 3; ++j) lds8(utb + j * BN + cl, hw[j]);
      }
      if constexpr (POOL) lds8(par + 3 * BN + cl, md);
#pragma unroll
      for (int fi = 0; fi < FM; ++fi) {
        // POOL: fragments in window order (pooled row rp, column block cb, tile row 2rp+rl)
        const int rp = fi / (2 * FMR), cb = (fi % (2 * FMR)) / 2, rl = fi % 2;
        const int f = POOL ? (2 * rp + rl) * FMR + cb : fi;
        const int rr = f / FMR, col = (f % FMR) * 16 + pxl;
        const int oh = oh0 + rr, ow = e.x0 + col;
        const bool ok = oh < p.ho && ow < p.wo;
        float v[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) v[k] = acc[f][2 * q + (k >> 2)][k & 3];
        if constexpr (EPI == 1 || EPI == 3) {
#pragma unroll
          for (int k = 0; k < 8; ++k) v[k] += bj[k];
          if (bt && (oh == 0 || oh == p.ho - 1 || ow == 0 || ow == p.wo - 1) && POOL && !RES) {
            // (the pooled non-resident kernel keeps the branching form: the branch-free one pushes
            // its fragment-address table into scratch inside the K loop)
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] -= border_corr(utb + (cl + k) * 8, oh, ow, p.ho, p.wo);
          } else if (bt && (oh == 0 || oh == p.ho - 1 || ow == 0 || ow == p.wo - 1)) {
            // border_corr (igemm_common.h) without its per-lane branches (each an exec-mask branch
            // around an LDS load): the same terms in the same order, absent ones as exact zeros
            const float t = oh == 0 ? 1.f : 0.f, b = oh == p.ho - 1 ? 1.f : 0.f;
            const float l = ow == 0 ? 1.f : 0.f, r = ow == p.wo - 1 ? 1.f : 0.f;
            const float tl = t * l, tr = t * r, bl = b * l, br = b * r;
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float4 u0 = *reinterpret_cast<const float4*>(utb + (cl + k) * 8);
              const float4 u1 = *reinterpret_cast<const float4*>(utb + (cl + k) * 8 + 4);
              float c = 0.f;
              c = fmaf(t, u0.x, c);
              c = fmaf(b, u0.y, c);
              c = fmaf(l, u0.z, c);
              c = fmaf(r, u0.w, c);
              c = fmaf(-tl, u1.x, c);
              c = fmaf(-tr, u1.y, c);
              c = fmaf(-bl, u1.z, c);
              c = fmaf(-br, u1.w, c);
              v[k] -= c;
            }
          }
          if (relu) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
          }
          if (AFFOK && aff) {
#pragma unroll
            for (int k = 0; k < 8; ++k) v[k] = fmaf(v[k], sj[k], hj[k]);
          }
          if constexpr (!NOSUM && EPI == 1) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              const float vs = ok ? v[k] : 0.f;
              sa[q][k] += vs;
              sb[q][k] += vs * vs;
            }
          }
        }
        dma::i32x4 pk8{};
        if constexpr (EPI == 3) {
#pragma unroll
          for (int j = 0; j < 3; ++j)
#pragma unroll
            for (int k = 0; k < 8; ++k) zf[f][j] = fmaf(v[k], hw[j][k], zf[f][j]);
        } else if constexpr (ES == 4) {
          const unsigned off = (unsigned)((((long)rr * p.wo + col) * p.out_ld + cl) * 4);
          const float4 lo = {v[0], v[1], v[2], v[3]}, hi = {v[4], v[5], v[6], v[7]};
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dma::i32x4, lo), os, ok ? off : OOB, 0, 0);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dma::i32x4, hi), os, ok ? off + 16 : OOB, 0, 0);
        } else {
          const unsigned off = (unsigned)((((long)rr * p.wo + col) * p.out_ld + cl) * 2);
          pk8 = pack8(v);
          __builtin_amdgcn_raw_buffer_store_b128(pk8, os, ok ? off : OOB, 0, 0);
        }
        if constexpr (POOL && EPI == 1) {
          // this window row as stored: the lane's pixel (tl) and its right neighbour (tr, DPP
          // quad_perm xor 1); a running maximum over the rows in window order (0,0), (0,1),
          // (1,0), (1,1), the first maximum winning (strict compares)
          float tl[8], tr[8];
          if constexpr (ES == 4) {
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              tl[k] = v[k];
              tr[k] = __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v[k]), 0xB1, 0xF, 0xF, false));
            }
          } else {  // bf16: the packed store operand and the neighbour's (4 dwords by DPP), unpacked
            dma::i32x4 nb;
#pragma unroll
            for (int d = 0; d < 4; ++d) nb[d] = __builtin_amdgcn_update_dpp(0, pk8[d], 0xB1, 0xF, 0xF, false);
            const bf16x8 bl = __builtin_bit_cast(bf16x8, pk8), br = __builtin_bit_cast(bf16x8, nb);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              tl[k] = to_f32(bl[k]);
              tr[k] = to_f32(br[k]);
            }
          }
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            const unsigned sh = 8 * (k & 3);
            float best;
            unsigned a;
            if (rl == 0) {
              best = tl[k];
              a = 0;
              if (md[k] * tr[k] > md[k] * best) { best = tr[k]; a = 1; }
            } else {
              best = pb[k];
              a = (pa[k >> 2] >> sh) & 0xFFu;
              if (md[k] * tl[k] > md[k] * best) { best = tl[k]; a = 2; }
              if (md[k] * tr[k] > md[k] * best) { best = tr[k]; a = 3; }
            }
            pb[k] = best;
            pa[k >> 2] = (pa[k >> 2] & ~(0xFFu << sh)) | (a << sh);
          }
          if (rl == 1) {  // window complete
            const float* pv = pb;
            const bool pok = (pxl & 1) == 0 && oh0 + 2 * rp < p.ho && e.x0 + cb * 16 + pxl < p.wo;
            const unsigned pe = (unsigned)((rp * (p.wo / 2) + cb * 8 + (pxl >> 1)) * p.pool_ld + cl);  // elements
            if constexpr (ES == 4) {
              const float4 lo = {pv[0], pv[1], pv[2], pv[3]}, hi = {pv[4], pv[5], pv[6], pv[7]};
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dma::i32x4, lo), ps, pok ? pe * 4 : OOB, 0, 0);
              __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dma::i32x4, hi), ps, pok ? pe * 4 + 16 : OOB, 0, 0);
            } else {
              __builtin_amdgcn_raw_buffer_store_b128(pack8(pv), ps, pok ? pe * 2 : OOB, 0, 0);
            }
            typedef int i32x2_ __attribute__((ext_vector_type(2)));
            __builtin_amdgcn_raw_buffer_store_b64(i32x2_{(int)pa[0], (int)pa[1]}, pis, pok ? pe : OOB, 0, 0);
          }
        }
      }
    }
    if constexpr (EPI == 3) {
      // the 64 channels of a pixel sit on the 4 lane groups (lanes pxl + 16 g): two exchanges
      // complete the dot products, then group 0 writes sigmoid(z + b) as 3 floats
      const __amdgpu_buffer_rsrc_t ys = dma::brsrc(p.yhat);
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int rr = f / FMR, col = (f % FMR) * 16 + pxl;
        const int oh = oh0 + rr, ow = e.x0 + col;
        const bool ok = g == 0 && oh < p.head_hv && ow < p.wo;
        const unsigned yo = (unsigned)((((long)e.img * p.head_hv + oh) * p.wo + ow) * 12);
#pragma unroll
        for (int j = 0; j < 3; ++j) {
          float z = zf[f][j];
          z += __shfl_xor(z, 16, 64);
          z += __shfl_xor(z, 32, 64);
          const float yv = 1.f / (1.f + expf(-(z + utb[3 * BN + j])));
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_int(yv), ys, ok ? yo + 4 * j : OOB, 0, 0);
        }
      }
    }
    zero_acc();
  };

  // EPI 2: r loaded through a buffer descriptor (out-of-range -> zeros), stores to
  // dz or g by column (global stores; out-of-image pixels go to the sink).  bf16: g is
  // rounded to bf16 first (as cnnitmo_bn_bwd_apply reads it from a bf16 buffer); fp32:
  // r of one column pair at a time (two 16-byte pieces per (pixel, 8 channels)).
  auto epilogue_bnb16 = [&](const Pos& e, int npost) {
    const int oh0 = e.y0 + wave * RPW;
    const int c0 = p.bnb_c0, c1 = p.bnb_c1, cbn = c1 - c0;
    const long m0 = ((long)e.img * p.ho + oh0) * p.wo + e.x0;  // the wave's first pixel
    // (late loads: the wait also retires the next item's DMA, issued during this item's
    // first taps.  Pulling these pieces into L2 one item ahead by LDS-DMA into the sink
    // measured 15-25 % slower on every fused dgrad (dec6-dec8), whether issued before or
    // after the ring's pieces.  Non-temporal r loads and epilogue stores (to keep the patch
    // lines in L2 for the next chunk) measured 1-4 % slower on levels 0-2.)
    if constexpr (EARLY) {
      dma::wait_vm_ge<L>(npost);  // the early loads, not the npost (0 or L) younger DMA pieces
    } else {
      load_r16(e);
      dma::wait_vm<0>();
    }
    bf16* __restrict__ O = (bf16*)p.out;
    bf16* __restrict__ Z = (bf16*)p.bnb_out;
#pragma unroll
    for (int q = 0; q < FP; ++q) {
      const int cl = 32 * q + 8 * g, c = n0 + cl;
      const bool fz = ALLF || (c >= c0 && c < c1);
      float ca[8], cb[8], ce[8];
      lds8(par + cl, ca);
      lds8(par + BN + cl, cb);
      lds8(par + 2 * BN + cl, ce);
      // ALLF: the pair's columns at the wave's first pixel, in dz (a fused block) or in the plain
      // gradient's view (a block below c0, whose r reads as 0: the ReLU test then compares with -1)
      // (the resident-weight and routed kernels take c0 = 0 only: launch_cfg)
      const bool bfz = !ALLF || RES || POOL || n0 >= c0;
      const __amdgpu_buffer_rsrc_t zs =
          dma::brsrc(!ALLF ? (const void*)Z
                           : bfz ? (const void*)(Z + m0 * cbn + (n0 - c0) + 32 * q)
                                 : (const void*)(O + m0 * p.out_ld + p.out_off + n0 + 32 * q));
      const long zld = bfz ? (long)cbn : p.out_ld;
      const float rmin = bfz ? 0.f : -1.f;
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int rr = f / FMR, col = (f % FMR) * 16 + pxl;
        const bool ok = oh0 + rr < p.ho && e.x0 + col < p.wo;
        float gr[8];
        routed(f, q, gr);
        const bf16x8 rq = __builtin_bit_cast(bf16x8, rv[f][q]);
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          // (as cnnitmo_bn_bwd_apply_pooled: the bf16 gradient, then the routed pooled one)
          float gk = to_f32(from_f32<bf16>(acc[f][2 * q + (k >> 2)][k & 3]));
          if constexpr (POOL) gk += gr[k];
          const float r = to_f32(rq[k]);
          if (fz) {
            // (an out-of-image pixel reads r = 0, so its dz is 0 and adds nothing to the sums: the
            // sums take no `ok` select.  This holds because rv comes from load_r16's raw-buffer loads
            // at r_off, which is OOB (the load returns 0) for every out-of-image or out-of-range
            // piece; the fp32 twin, epilogue_bnb32, keeps the select.)
            o[k] = from_f32<bf16>(r > rmin ? ca[k] * gk - cb[k] * r + ce[k] : 0.f);
            if (rr == 0) sa[q][k] += to_f32(o[k]);
            else sb[q][k] += to_f32(o[k]);
          } else {
            o[k] = from_f32<bf16>(gk);
          }
        }
        if constexpr (ALLF) {
          const unsigned off = (unsigned)((((long)rr * p.wo + col) * zld + 8 * g) * 2);
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dma::i32x4, o), zs, ok ? off : OOB, 0, 0);
        } else {
          const long m = m0 + (long)rr * p.wo + col;
          uint4* dst = !ok ? h_sink + lane
                       : fz ? reinterpret_cast<uint4*>(Z + (size_t)m * cbn + (c - c0))
                            : reinterpret_cast<uint4*>(O + (size_t)m * p.out_ld + p.out_off + c);
          *dst = __builtin_bit_cast(uint4, o);
        }
      }
    }
    zero_acc();
  };

  auto epilogue_bnb32 = [&](const Pos& e) {
    const int oh0 = e.y0 + wave * RPW;
    const int c0 = p.bnb_c0, c1 = p.bnb_c1, cbn = c1 - c0;
    const long m0 = ((long)e.img * p.ho + oh0) * p.wo + e.x0;  // the wave's first pixel
    const __amdgpu_buffer_rsrc_t rs = dma::brsrc(r_base(e));
    constexpr int RQ = ES == 2 ? FP : 1;  // column pairs whose r is in flight at once
    constexpr int RP = ES == 2 ? 1 : 2;   // 16-byte r pieces per (pixel, 8 channels)
    dma::i32x4 rv[FM][RQ][RP];
    auto load_r = [&](int q0) {
#pragma unroll
      for (int f = 0; f < FM; ++f)
#pragma unroll
        for (int qq = 0; qq < RQ; ++qq) {
          const unsigned o = r_off(e, f, q0 + qq);
#pragma unroll
          for (int h2 = 0; h2 < RP; ++h2) rv[f][qq][h2] = __builtin_amdgcn_raw_buffer_load_b128(rs, o == OOB ? OOB : o + 16 * h2, 0, 0);
        }
      // (also retires the next item's DMA, issued during this item's first taps).  Pulling
      // these pieces into L2 one item ahead by LDS-DMA into the sink measured 15-25 %
      // slower on every fused dgrad (dec6-dec8), whether issued before or after the
      // ring's pieces.  Non-temporal r loads and epilogue stores (to keep the patch
      // lines in L2 for the next chunk) measured 1-4 % slower on levels 0-2.
      dma::wait_vm<0>();
    };
    TE* __restrict__ O = (TE*)p.out;
    TE* __restrict__ Z = (TE*)p.bnb_out;
    load_route(e);  // (retired by load_r's wait)
    if constexpr (ES == 2) load_r(0);
#pragma unroll
    for (int q = 0; q < FP; ++q) {
      if constexpr (ES == 4) load_r(q);
      const int qr = ES == 2 ? q : 0;
      const int cl = 32 * q + 8 * g, c = n0 + cl;
      const bool fz = ALLF || (c >= c0 && c < c1);
      const __amdgpu_buffer_rsrc_t zs = dma::brsrc(ALLF ? (const void*)(Z + m0 * cbn + n0 + 32 * q) : (const void*)Z);
      float ca[8], cb[8], ce[8];
      lds8(par + cl, ca);
      lds8(par + BN + cl, cb);
      lds8(par + 2 * BN + cl, ce);
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        const int rr = f / FMR, col = (f % FMR) * 16 + pxl;
        const bool ok = oh0 + rr < p.ho && e.x0 + col < p.wo;
        const long m = m0 + (long)rr * p.wo + col;
        float v[8], rf[8], gr[8];
        routed(f, q, gr);
        if constexpr (ES == 2) {
          const bf16x8 rq = __builtin_bit_cast(bf16x8, rv[f][qr][0]);
#pragma unroll
          for (int k = 0; k < 8; ++k) rf[k] = to_f32(rq[k]);
        } else {
          const f32x4 r0 = __builtin_bit_cast(f32x4, rv[f][qr][0]), r1 = __builtin_bit_cast(f32x4, rv[f][qr][RP - 1]);
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            rf[k] = r0[k];
            rf[4 + k] = r1[k];
          }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float gk = to_f32(from_f32<TE>(acc[f][2 * q + (k >> 2)][k & 3]));
          if constexpr (POOL) gk += gr[k];
          const float r = rf[k];
          if (fz) {
            v[k] = to_f32(from_f32<TE>(r > 0.f ? ca[k] * gk - cb[k] * r + ce[k] : 0.f));
            sa[q][k] += (ok && rr == 0) ? v[k] : 0.f;
            sb[q][k] += (ok && rr == 1) ? v[k] : 0.f;
          } else {
            v[k] = gk;
          }
        }
        TE* dp = fz ? Z + (size_t)m * cbn + (c - c0) : O + (size_t)m * p.out_ld + p.out_off + c;
        if constexpr (ALLF) {  // as in epilogue_bnb16
          const unsigned off = (unsigned)((((long)rr * p.wo + col) * cbn + 8 * g) * ES);
          if constexpr (ES == 2) {
            __builtin_amdgcn_raw_buffer_store_b128(pack8(v), zs, ok ? off : OOB, 0, 0);
          } else {
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dma::i32x4, f32x4{v[0], v[1], v[2], v[3]}), zs,
                                                   ok ? off : OOB, 0, 0);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dma::i32x4, f32x4{v[4], v[5], v[6], v[7]}), zs,
                                                   ok ? off + 16 : OOB, 0, 0);
          }
        } else if constexpr (ES == 2) {
          uint4* dst = !ok ? h_sink + lane : reinterpret_cast<uint4*>(dp);
          *dst = __builtin_bit_cast(uint4, pack8(v));
        } else {
          uint4* d0 = !ok ? h_sink + lane : reinterpret_cast<uint4*>(dp);
          uint4* d1 = !ok ? h_sink + lane : reinterpret_cast<uint4*>(dp + 4);
          *d0 = __builtin_bit_cast(uint4, f32x4{v[0], v[1], v[2], v[3]});
          *d1 = __builtin_bit_cast(uint4, f32x4{v[4], v[5], v[6], v[7]});
        }
      }
    }
    zero_acc();
  };

  auto epilogue_bnb = [&](const Pos& e, int npost) {
    if constexpr (ES == 2) epilogue_bnb16(e, npost);
    else epilogue_bnb32(e);
  };

  if constexpr (RES) {  // the resident weights: every chunk's pieces, then a full drain
    for (int ch = 0; ch < nch; ++ch) {
      const uintptr_t wb = (uintptr_t)(Wt + (size_t)n0 * K + ch * CC);
      char* dst = smem + C::WRES + ch * (C::BPC * 1024);
#pragma unroll
      for (int i = 0; i < NBI; ++i) {
        const int gp = wave * NBI + i;
        dma::lds16(boff[i], dma::rsrc(wb), gp < C::BPC ? dst + gp * 1024 : smem + C::SCR);
      }
    }
    dma::wait_vm<0>();
    __syncthreads();
  }
  // ST-stage ring over items (see the file comment for the vmcnt accounting)
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
  int buf = 0;
  for (long t = 0; t < T; ++t) {
    // younger than this item's pieces: the previous tile's epilogue stores (NST) or nothing.
    // (The generic fused dgrad, dec6's, keeps the switch: with the two-way wait its register
    // allocation reloads fragment addresses from scratch inside the K loop.)
    if constexpr (EPI == 2 && !ALLF) dma::wait_vm_dyn(issued - mq[0]);
    else dma::wait_vm_ge<NST>(issued - mq[0]);
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
#ifndef HALO_PROBE_NODMA  // timing probes (tools/build_variant.sh): no DMA after the prologue /
#define HALO_PROBE_NODMA 0  // no forward epilogue; results are garbage
#endif
#ifndef HALO_PROBE_NOEPI
#define HALO_PROBE_NOEPI 0
#endif
    const bool pf = t + ST - 1 < T && !HALO_PROBE_NODMA;
    if (pf) issue_prep(buf == 0 ? ST - 1 : buf - 1);  // stage (t + ST - 1) % ST
    if constexpr (EARLY) {
      if (ep.ch == nch - 1) {  // the tile's last item: its epilogue's loads go out now
        load_r16(ep);
        issued += NEARLY;
      }
    }
    const bool act = ep.y0 + wave * RPW < p.ho;
    if (act) {
      compute(buf, pf, ep.ch);  // issues those loads between its taps
    } else if (pf) {     // the wave's rows are all below the frame: no MFMAs, DMA share only
#pragma unroll
      for (int q = 0; q < L; ++q) issue_piece(q);
    }
    if (pf) {
      step(ip);
      issued += L;
      mq[ST - 1] = issued;
    }
#ifndef HALO_PROBE_NOEPI2
#define HALO_PROBE_NOEPI2 0
#endif
    if (ep.ch == nch - 1 && ((HALO_PROBE_NOEPI && EPI == 1) || (HALO_PROBE_NOEPI2 && EPI == 2))) {  // (probe: the accumulators stay live)
      float z = 0.f;
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) z += acc[i][j][0] + acc[i][j][1] + acc[i][j][2] + acc[i][j][3];
      if (p.flags == 0x7fff0000) ((float*)p.out)[lane] = z;
      zero_acc();
    } else if (ep.ch == nch - 1) {
      if constexpr (EPI == 2) epilogue_bnb(ep, pf ? L : 0);
      else epilogue(ep);
      issued += NST;
    }
    step(ep);
#pragma unroll
    for (int k = 0; k < ST - 1; ++k) mq[k] = mq[k + 1];
    buf = buf == ST - 1 ? 0 : buf + 1;
  }

  // partial-sum rows: one per (stream, wave); the 16 pixel lanes are folded here
  const long row = (long)gs * NWAVE + wave;
  if constexpr (EPI == 1 && !NOSUM) {
    if (p.flags & CNNITMO_STATS) {
#pragma unroll
      for (int q = 0; q < FP; ++q)
#pragma unroll
        for (int k = 0; k < 8; ++k)
#pragma unroll
          for (int o = 1; o < 16; o <<= 1) {
            sa[q][k] += __shfl_xor(sa[q][k], o, 64);
            sb[q][k] += __shfl_xor(sb[q][k], o, 64);
          }
      if (pxl == 0) {
        float* st = p.stats + (size_t)row * 2 * p.N + n0;
#pragma unroll
        for (int q = 0; q < FP; ++q)
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            st[32 * q + 8 * g + k] = sa[q][k];
            st[p.N + 32 * q + 8 * g + k] = sb[q][k];
          }
      }
    }
  } else if constexpr (EPI == 2) {
    const int c0 = p.bnb_c0, c1 = p.bnb_c1, cbn = c1 - c0;
    // lanes of equal pixel-column parity (lane & 1) within the 16
#pragma unroll
    for (int q = 0; q < FP; ++q)
#pragma unroll
      for (int k = 0; k < 8; ++k)
#pragma unroll
        for (int o = 2; o < 16; o <<= 1) {
          sa[q][k] += __shfl_xor(sa[q][k], o, 64);
          sb[q][k] += __shfl_xor(sb[q][k], o, 64);
        }
    if (!p.bnb_par) {
#pragma unroll
      for (int q = 0; q < FP; ++q)
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          sa[q][k] += sb[q][k];
          sa[q][k] += __shfl_xor(sa[q][k], 1, 64);
        }
    }
    if (pxl < 2) {
      const int cp = pxl;  // pixel-column parity
#pragma unroll
      for (int q = 0; q < FP; ++q) {
        const int c = n0 + 32 * q + 8 * g;
        if (c >= c0 && c < c1) {
          if (p.bnb_par) {
            float* st = p.stats + (size_t)row * 4 * cbn + (c - c0);
#pragma unroll
            for (int k = 0; k < 8; ++k) {
              st[(size_t)(0 * 2 + cp) * cbn + k] = sa[q][k];
              st[(size_t)(1 * 2 + cp) * cbn + k] = sb[q][k];
            }
          } else if (cp == 0) {
            float* st = p.stats + (size_t)row * cbn + (c - c0);
#pragma unroll
            for (int k = 0; k < 8; ++k) st[k] = sa[q][k];
          }
        }
      }
    }
  }
}

struct HaloPlan {
  int bn, epi, th;
  bool res;
};

int halo_ncu() {
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    hipDeviceProp_t prop;
    if (hipGetDevice(&dev) == hipSuccess && hipGetDeviceProperties(&prop, dev) == hipSuccess)
      ncu = prop.multiProcessorCount;
    if (ncu < 8) ncu = 256;
  }
  return ncu;
}

// conv3x3 stride 1 'same' (forward or input-gradient), 64-byte chunks (32 bf16 / 16 fp32
// channels); fp32: one source (forward with BN sums, plain and fused input gradients)
bool halo_plan(const FwdArgs& a, HaloPlan& pl, bool f32 = false) {
  static const int en = [] {
    const char* e = getenv("CNNITMO_HALO");
    return e ? atoi(e) : 1;
  }();
  // (fp32: 82.9 -> 94.8 frames/s at 1080p b8 inference, the kernel at 0.87 of fp32 peak
  // against the implicit GEMM's 0.75, profiles/r03zl_*)
  if (!en) return false;
  if (f32) {
    if (a.cin % 16 || a.a_ld % 4 || a.a_off % 4 || a.out_ld % 4 || a.out_off % 4) return false;
    if (a.a2) return false;
  } else if (a.cin % 32 || a.a_ld % 8 || a.a_off % 8 || a.out_ld % 8 || a.out_off % 8) {
    return false;
  }
  if (a.a2 && (a.cin1 % 32 || a.cin1 <= 0 || a.cin1 >= a.cin || a.a2_ld % 8 || a.a2_off % 8 || a.bnb_out))
    return false;
  if (a.ntaps != 9 || a.scale != 1 || a.scatter || a.hs != a.ho || a.ws != a.wo) return false;
  if (a.pool_out && (a.a2 || a.ho % 2 || a.wo % 2 || a.pool_ld % 8 || a.pool_ld < a.N || !a.pool_idx))
    return false;
  // the routed pooled gradient (EPI 2): every column BN-fused, pooled [..][N] rows
  if (a.pool_out && a.bnb_out && (a.bnb_c0 != 0 || a.bnb_c1 != a.N || a.pool_ld != a.N || a.bnb_par)) return false;
  // pooled forward: BN sums (training, BN folded: r stored) or the affine (inference), not both
  if (a.pool_out && (a.flags & CNNITMO_STATS) && (a.flags & CNNITMO_AFFINE)) return false;
  pl.bn = a.N % 64 == 0 ? 64 : (a.N % 32 == 0 ? 32 : 0);
  // the routed-pool dgrad (EPI 2 + POOL): 32-column blocks, whose epilogue keeps the pooled
  // gradient and indices in registers without spilling (64-column blocks measured 0.3 %
  // slower on the bench step, profiles/r05/r05c_ab_route_bn64.txt).  The other fused BN-backward
  // dgrads keep 64 columns: 32-column blocks, whose r loads can go out early, measured 3 %
  // slower for all of them and 1 % for those up to 64 columns (r05e_ab_bnb_bn32.txt,
  // r05h_ab_bnb_bn32_64.txt)
  if (a.pool_out && a.bnb_out && a.N % 32 == 0) pl.bn = 32;
  if (!pl.bn || a.N / pl.bn > halo_ncu() / 8) return false;
  if (a.bnb_out) {  // fused BN backward (input gradient)
    if (a.bnb_c0 % 8 || a.bnb_c1 % 8 || a.bnb_c0 < 0 || a.bnb_c1 > a.N || a.bnb_c0 >= a.bnb_c1 ||
        a.bnb_r_ld % 8 || a.bnb_r_off % 8)
      return false;
    pl.epi = 2;
  } else if (a.yhat) {  // the forward with the sigmoid head (one 64-column block: all channels)
    if (a.N != 64 || pl.bn != 64 || a.a2 || a.pool_out || a.stats || a.border || (a.flags & CNNITMO_STATS) ||
        !a.head_w || !a.head_b)
      return false;
    pl.epi = 3;
  } else {
    pl.epi = (a.flags || a.bias || a.border || a.stats) ? 1 : 0;
    if (a.a2 && pl.epi != 1) return false;  // two sources: the forward-epilogue kernels only
  }
  pl.res = a.cin <= (f32 ? 16 : 32) * RCH;
  pl.th = 16;
  return true;
}

template <typename T, int BN, int EPI>
void launch_cfg(const HaloArgs& h, bool res, int grid, hipStream_t s) {
  if constexpr (EPI == 2) {
    if (h.f.pool_out) {  // the routed pooled gradient (cnnitmo_conv3x3_dgrad_bn_pooled; 32-column blocks,
                         // every column fused: halo_plan)
      if constexpr (BN == 32) {
        if (res) hipLaunchKernelGGL((halo_conv_kernel<T, BN, EPI, true, true, 16, true>), dim3(grid), dim3(NT), 0, s, h);
        else hipLaunchKernelGGL((halo_conv_kernel<T, BN, EPI, false, true, 16, true>), dim3(grid), dim3(NT), 0, s, h);
      }
      return;
    }
    // ALLF: every column fused, or (bf16) every block either fused or plain
    const bool allf = h.f.bnb_c1 == h.f.N &&
                      (h.f.bnb_c0 == 0 || (std::is_same<T, bf16>::value && !res && h.f.bnb_c0 % BN == 0));
    if (allf) {
      if (res) hipLaunchKernelGGL((halo_conv_kernel<T, BN, EPI, true, false, 16, true>), dim3(grid), dim3(NT), 0, s, h);
      else hipLaunchKernelGGL((halo_conv_kernel<T, BN, EPI, false, false, 16, true>), dim3(grid), dim3(NT), 0, s, h);
      return;
    }
  }
  if constexpr (EPI == 1) {
    const bool nst = !(h.f.flags & CNNITMO_STATS);  // inference: the kernels without BN sums
    if (h.f.pool_out) {
      if (nst) {
        if (res) hipLaunchKernelGGL((halo_conv_kernel<T, BN, EPI, true, true, 16, true>), dim3(grid), dim3(NT), 0, s, h);
        else hipLaunchKernelGGL((halo_conv_kernel<T, BN, EPI, false, true, 16, true>), dim3(grid), dim3(NT), 0, s, h);
      } else {
        if (res) hipLaunchKernelGGL((halo_conv_kernel<T, BN, EPI, true, true>), dim3(grid), dim3(NT), 0, s, h);
        else hipLaunchKernelGGL((halo_conv_kernel<T, BN, EPI, false, true>), dim3(grid), dim3(NT), 0, s, h);
      }
      return;
    }
    if (nst) {
      if (res) hipLaunchKernelGGL((halo_conv_kernel<T, BN, EPI, true, false, 16, true>), dim3(grid), dim3(NT), 0, s, h);
      else hipLaunchKernelGGL((halo_conv_kernel<T, BN, EPI, false, false, 16, true>), dim3(grid), dim3(NT), 0, s, h);
      return;
    }
  }
  if (res) hipLaunchKernelGGL((halo_conv_kernel<T, BN, EPI, true>), dim3(grid), dim3(NT), 0, s, h);
  else hipLaunchKernelGGL((halo_conv_kernel<T, BN, EPI, false>), dim3(grid), dim3(NT), 0, s, h);
}

int halo_streams(const FwdArgs& a, const HaloPlan& pl) { return halo_ncu() / (a.N / pl.bn); }

}  // namespace

bool halo_handles(const FwdArgs& a, bool f32) {
  HaloPlan pl;
  return halo_plan(a, pl, f32);
}

int launch_halo(FwdArgs a, hipStream_t s, const char* what, bool f32) {
  HaloPlan pl;
  CNN_REQUIRE(halo_plan(a, pl, f32), "%s: no halo plan", what);
  HaloArgs h;
  h.f = a;
  h.tiles_x = (a.wo + TW - 1) / TW;  // partial edge tiles are masked
  h.tiles_y = (a.ho + pl.th - 1) / pl.th;
  h.nchunks = a.cin / (f32 ? 16 : 32);
  h.tiles = (long)a.nimg * h.tiles_x * h.tiles_y;
  h.nblocks = a.N / pl.bn;
  h.streams = halo_streams(a, pl);
  CNN_REQUIRE(h.streams >= 1, "%s: %d column blocks exceed the workgroups", what, h.nblocks);
  CNN_REQUIRE(h.tiles * h.nchunks < (1L << 31), "%s: too many tiles", what);
  CNN_REQUIRE(!(a.flags & CNNITMO_STATS) || a.stats, "%s: STATS without buffer", what);
  const int grid = halo_ncu();
  if (f32 && pl.epi == 3) {
    launch_cfg<float, 64, 3>(h, pl.res, grid, s);
  } else if (f32 && pl.epi == 1) {
    if (pl.bn == 64) launch_cfg<float, 64, 1>(h, pl.res, grid, s);
    else launch_cfg<float, 32, 1>(h, pl.res, grid, s);
  } else if (f32 && pl.epi == 2) {
    if (pl.bn == 64) launch_cfg<float, 64, 2>(h, pl.res, grid, s);
    else launch_cfg<float, 32, 2>(h, pl.res, grid, s);
  } else if (f32) {
    if (pl.bn == 64) launch_cfg<float, 64, 0>(h, pl.res, grid, s);
    else launch_cfg<float, 32, 0>(h, pl.res, grid, s);
  } else if (pl.epi == 2) {
    if (pl.bn == 64) launch_cfg<bf16, 64, 2>(h, pl.res, grid, s);
    else launch_cfg<bf16, 32, 2>(h, pl.res, grid, s);
  } else if (pl.epi == 3) {
    launch_cfg<bf16, 64, 3>(h, pl.res, grid, s);
  } else if (pl.epi == 1) {
    if (pl.bn == 64) launch_cfg<bf16, 64, 1>(h, pl.res, grid, s);
    else launch_cfg<bf16, 32, 1>(h, pl.res, grid, s);
  } else {
    if (pl.bn == 64) launch_cfg<bf16, 64, 0>(h, pl.res, grid, s);
    else launch_cfg<bf16, 32, 0>(h, pl.res, grid, s);
  }
  return cnnitmo_check_launch(what);
}

const char* halo_name(const FwdArgs& a, bool f32) {
  HaloPlan pl;
  if (!halo_plan(a, pl, f32)) return "";
  static thread_local char buf[64];
  snprintf(buf, sizeof(buf), "halo_conv_kernel<%s%d,%d%s%s>", f32 ? "f32," : "", pl.bn, pl.epi, pl.res ? ",wres" : "",
           a.pool_out ? (pl.epi == 2 ? ",route" : ",pool") : "");
  return buf;
}

// BN partial-sum rows written by the halo kernel: one per (stream, wave).
long halo_stat_rows(const FwdArgs& a, bool f32) {
  HaloPlan pl;
  if (!halo_plan(a, pl, f32)) return 0;
  return (long)halo_streams(a, pl) * NWAVE;
}
