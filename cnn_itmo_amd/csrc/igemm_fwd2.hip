// Implicit-GEMM convolution, forward family, v2: direct-to-LDS pipelined MFMA.
//
// Same GEMM as igemm_fwd.hip (C[m][n] = sum_k A[m][k] B[n][k], m = output pixel,
// k = (tap, channel), A gathered per tap from an NHWC source with zero
// padding), restructured for gfx950's memory pipeline:
//   * operands go HBM/L2 -> LDS with global_load_lds_dwordx4 (no VGPR staging):
//     each lane supplies its own gather address (padding rows point at a zero
//     page); the LDS image is lane-linear, so the XOR swizzle is applied to the
//     SOURCE chunk and mirrored on the ds_read (guide rule 21);
//   * K-step = 128 bytes per row (64 bf16 / 32 f32), flat over (tap, channel)
//     so Cin = 32 or 96 and tap-straddling steps need no special case;
//   * ST-stage LDS ring with counted `s_waitcnt vmcnt` and ONE raw s_barrier per
//     K-step: loads for steps t+1..t+ST-1 stay in flight across the barrier
//     while step t is multiplied;
//   * epilogue (bias, ReLU, inference BN affine, BN partial sums) in registers,
//     then the tile is staged through LDS and stored as 16-byte row vectors
//     (plain NHWC view or the Conv2DTranspose pixel scatter).
// LDS image: [rows][128 B], 16-byte chunk c of row r at slot c ^ ((r >> 1) & 7):
// conflict-free for the fragment reads (lane l: row l&15, chunk 4*kk + (l>>4))
// in every ds_read_b128 bank group (derivation in DESIGN.md).
#include <algorithm>
#include <cstdlib>

#include "dma.h"
#include "igemm_common.h"

__device__ __attribute__((aligned(256))) unsigned char g_zero_page[256] = {0};

// One LDS-DMA wave-instruction: lane l copies 16 bytes from its own gsrc to
// LDS[lds + 16*l].  Issued from inline asm on purpose: when hipcc sees the
// builtin it cannot prove later ds_reads of OTHER ring slots don't alias the
// in-flight DMA and inserts s_waitcnt vmcnt(0) before them, serialising the
// pipeline.  Ordering is instead guaranteed by the counted vmcnt + s_barrier
// protocol of the main loop (and the "memory" clobber).
#pragma clang diagnostic ignored "-Winline-asm"
__device__ __forceinline__ unsigned lds_addr(const void* p) {
  return (unsigned)(size_t)(const __attribute__((address_space(3))) char*)p;
}
__device__ __forceinline__ void glds16(const void* gsrc, const char* lds) {
  const unsigned a = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  asm volatile("s_mov_b32 m0, %1\n\tglobal_load_lds_dwordx4 %0, off" ::"v"(gsrc), "s"(a) : "m0");
}

template <int N> __device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ int swz_off(int row, int chunk) {
  return (row << 7) + ((chunk ^ ((row >> 1) & 7)) << 4);
}

template <typename T, int BM, int BN, int WM, int WN, int ST>
struct Fwd2Cfg {
  static constexpr int NW = WM * WN, NT = NW * 64;
  static constexpr int VE = Vec16<T>::N, KE = 8 * VE;
  static constexpr int TM = BM / WM, TN = BN / WN, FM = TM / 16, FN = TN / 16;
  static constexpr int A_INSTR = BM / 8, B_INSTR = BN / 8;
  static constexpr int NA = A_INSTR / NW, NB = B_INSTR / NW;
  static constexpr int L = NA + NB;  // glds per wave per stage
  static constexpr int STAGE = (BM + BN) * 128;
  static constexpr int CLD = BN + 16 / (int)sizeof(T);  // padded C-tile row (elements)
  static constexpr int C_BYTES = BM * CLD * (int)sizeof(T);
  static constexpr int SMEM = (ST * STAGE > C_BYTES + WM * BN * 8) ? ST * STAGE : C_BYTES + WM * BN * 8;
  static_assert(A_INSTR % NW == 0 && B_INSTR % NW == 0, "loads must split evenly over waves");
  static_assert(NA % 2 == 0, "A row-block parity must be compile-time");
  static_assert(SMEM <= 160 * 1024, "LDS");
};

template <typename T, int BM, int BN, int WM, int WN, int ST>
__global__ __launch_bounds__(WM * WN * 64) void igemm_fwd2_kernel(const FwdArgs p) {
  using C = Fwd2Cfg<T, BM, BN, WM, WN, ST>;
  constexpr int VE = C::VE, KE = C::KE, TM = C::TM, TN = C::TN, FM = C::FM, FN = C::FN;
  constexpr int NA = C::NA, NB = C::NB, STAGE = C::STAGE;
  __shared__ __attribute__((aligned(1024))) char smem[C::SMEM];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int lid = xcd_remap(blockIdx.x, p.mblocks * p.nblocks);
  const int mb = lid / p.nblocks, nb = lid - mb * p.nblocks;
  const long m0 = (long)mb * BM;
  const int n0 = nb * BN;
  const int K = p.ntaps * p.cin;
  const int nk = (K + KE - 1) / KE;
  const T* __restrict__ A = (const T*)p.a;
  const T* __restrict__ B = (const T*)p.b;

  // ---- per-lane load bookkeeping -------------------------------------------
  const int sub = lane >> 3, pslot = lane & 7;
  // logical chunk held by this lane's LDS slot: pslot ^ ((row >> 1) & 7), row = blk*8 + sub
  const int cA0 = pslot ^ (sub >> 1), cA1 = cA0 ^ 4;  // row block even / odd
  int a_img[NA], a_h[NA], a_w[NA];
  const long hw = (long)p.ho * p.wo;
#pragma unroll
  for (int i = 0; i < NA; ++i) {
    const long m = m0 + (wave * NA + i) * 8 + sub;
    a_img[i] = -1;
    a_h[i] = a_w[i] = 0;
    if (m < p.M) {
      const int img = (int)(m / hw);
      const int rem = (int)(m - (long)img * hw);
      const int oh = rem / p.wo;
      a_img[i] = img;
      a_h[i] = oh * p.scale;
      a_w[i] = (rem - oh * p.wo) * p.scale;
    }
  }
  // (tap, channel) of the chunk this lane loads, for even/odd row blocks
  int tap0 = (cA0 * VE) / p.cin, ch0 = (cA0 * VE) - tap0 * p.cin;
  int tap1 = (cA1 * VE) / p.cin, ch1 = (cA1 * VE) - tap1 * p.cin;
  int kb0 = cA0 * VE, kb1 = cA1 * VE;  // B-side k of the same chunks

  auto advance = [&]() {
    ch0 += KE;
    while (ch0 >= p.cin) { ch0 -= p.cin; ++tap0; }
    ch1 += KE;
    while (ch1 >= p.cin) { ch1 -= p.cin; ++tap1; }
    kb0 += KE;
    kb1 += KE;
  };

  auto issue = [&](int buf) {
    char* As = smem + buf * STAGE;
    char* Bs = As + BM * 128;
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const int tap = (i & 1) ? tap1 : tap0;
      const int ch = (i & 1) ? ch1 : ch0;
      const void* src = g_zero_page;
      if (a_img[i] >= 0 && tap < p.ntaps) {
        const int hh = a_h[i] + ((p.dyc >> (2 * tap)) & 3) - 1;
        const int ww = a_w[i] + ((p.dxc >> (2 * tap)) & 3) - 1;
        if ((unsigned)hh < (unsigned)p.hs && (unsigned)ww < (unsigned)p.ws)
          src = A + ((size_t)((long)a_img[i] * p.hs + hh) * p.ws + ww) * p.a_ld + p.a_off + ch;
      }
      glds16(src, As + (wave * NA + i) * 1024);
    }
#pragma unroll
    for (int i = 0; i < NB; ++i) {
      const int blk = wave * NB + i;
      const int k = (blk & 1) ? kb1 : kb0;
      const void* src = g_zero_page;
      if (k < K) src = B + (size_t)(n0 + blk * 8 + sub) * K + k;
      glds16(src, Bs + blk * 1024);
    }
  };

  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + BM * 128;
    const int frow = lane & 15, fg = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      uint4 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const uint4*>(As + swz_off(wm * TM + i * 16 + frow, kk * 4 + fg));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const uint4*>(Bs + swz_off(wn * TN + j * 16 + frow, kk * 4 + fg));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) Mma<T>::run(acc[i][j], af[i], bfr[j]);
    }
  };

  // ---- main loop: ST-stage ring, one barrier per K-step ----------------------
  issue(0);
  advance();
#pragma unroll
  for (int s = 1; s < ST - 1; ++s)
    if (s < nk) { issue(s); advance(); }
  for (int t = 0; t < nk; ++t) {
    if constexpr (ST == 3) {
      if (t + 1 < nk) wait_vm<C::L>(); else wait_vm<0>();
    } else {
      wait_vm<0>();
    }
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");  // compiler fence: no LDS read hoisted above the barrier
    __builtin_amdgcn_sched_barrier(0);
    if (t + ST - 1 < nk) {
      issue((t + ST - 1) % ST);
      advance();
    }
    compute(t % ST);
  }
  __syncthreads();

  // ---- epilogue ----------------------------------------------------------------
  const bool relu = p.flags & CNNITMO_RELU, aff = p.flags & CNNITMO_AFFINE,
             stats = p.flags & CNNITMO_STATS;
  float bj[FN], sj[FN], hj[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) {
    const int n = n0 + wn * TN + j * 16 + (lane & 15);
    const int co = p.scatter ? n % p.cout : n;
    bj[j] = p.bias ? p.bias[(p.flags & CNNITMO_BIAS_PER_COL) ? n : co] : 0.f;
    sj[j] = aff ? p.aff_scale[co] : 1.f;
    hj[j] = aff ? p.aff_shift[co] : 0.f;
  }
  float s1[FN], s2[FN];
#pragma unroll
  for (int j = 0; j < FN; ++j) s1[j] = s2[j] = 0.f;
  T* Cs = reinterpret_cast<T*>(smem);
#pragma unroll
  for (int i = 0; i < FM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int row = wm * TM + i * 16 + (lane >> 4) * 4 + r;
      const bool valid = m0 + row < p.M;
      int boh = 1, bow = 1;  // interior unless a border table is given
      if (p.border && valid) {
        const long m = m0 + row;
        const int rem = (int)(m % hw);
        boh = rem / p.wo;
        bow = rem - boh * p.wo;
      }
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        float v = acc[i][j][r] + bj[j];
        if (p.border)
          v -= border_corr(p.border + (size_t)(n0 + wn * TN + j * 16 + (lane & 15)) * 8, boh, bow, p.ho, p.wo);
        if (relu) v = fmaxf(v, 0.f);
        if (aff) v = v * sj[j] + hj[j];
        if (valid) {
          s1[j] += v;
          s2[j] += v * v;
        }
        Cs[row * C::CLD + wn * TN + j * 16 + (lane & 15)] = from_f32<T>(v);
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
    float* red = reinterpret_cast<float*>(smem + C::C_BYTES);  // [WM][BN][2]
    if (lane < 16) {
#pragma unroll
      for (int j = 0; j < FN; ++j) {
        const int col = wn * TN + j * 16 + lane;
        red[(wm * BN + col) * 2 + 0] = s1[j];
        red[(wm * BN + col) * 2 + 1] = s2[j];
      }
    }
  }
  __syncthreads();
  if (stats && tid < BN) {
    const float* red = reinterpret_cast<const float*>(smem + C::C_BYTES);
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
  // coalesced 16-byte row stores
  T* __restrict__ O = (T*)p.out;
  constexpr int CPR = BN / VE;  // chunks per row
  for (int idx = tid; idx < BM * CPR; idx += C::NT) {
    const int row = idx / CPR, cc = idx - row * CPR;
    const long m = m0 + row;
    if (m >= p.M) continue;
    const uint4 v = *reinterpret_cast<const uint4*>(Cs + row * C::CLD + cc * VE);
    const int n = n0 + cc * VE;
    size_t off;
    if (p.scatter) {
      const int tp = n / p.cout, co = n - tp * p.cout;
      const int img = (int)(m / hw);
      const int rem = (int)(m - (long)img * hw);
      const int ii = rem / p.wo, jj = rem - ii * p.wo;
      const long pix = ((long)img * 2 * p.ho + 2 * ii + (tp >> 1)) * 2 * p.wo + 2 * jj + (tp & 1);
      off = (size_t)pix * p.out_ld + p.out_off + co;
    } else {
      off = (size_t)m * p.out_ld + p.out_off + n;
    }
    *reinterpret_cast<uint4*>(O + off) = v;
  }
}

// ----------------------------------------------------------------------------
// Persistent form of the 256 x 256 bf16 launch, for the Conv2DTranspose input gradient
// (up6 / up7, K = 4 taps x Cout; a plain store epilogue: it issues no loads, so it never
// waits on the next tile's ring DMA).  One workgroup per CU walks
// its XCD's contiguous tile range (XCD x owns tiles [T*x/8, T*(x+1)/8); its Gx workgroups
// take every Gx-th tile, so the XCD's resident tiles are consecutive: both column blocks
// of a row block share the A rows in that XCD's L2).  The ring runs across tile
// boundaries: the next tile's first K-step is loaded during the current tile's last one,
// so a tile has no prologue bubble.  The MFMA runs with the operands swapped (C^T) on
// pair_perm'd weight rows, so each lane holds 8 consecutive output channels of one pixel
// and the epilogue is 16-byte buffer stores straight from the accumulators (no LDS C tile,
// no barrier): FM * FN / 2 stores per wave per tile, issued unconditionally (rows past M
// get an out-of-range offset and are dropped) so the next K-step's counted wait is exact.
template <int BM, int BN, int WM, int WN>
__global__ __launch_bounds__(WM * WN * 64) void igemm_fwd2p_kernel(const FwdArgs p) {
  using C = Fwd2Cfg<bf16, BM, BN, WM, WN, 2>;
  constexpr int VE = C::VE, KE = C::KE, TM = C::TM, TN = C::TN, FM = C::FM, FN = C::FN;
  constexpr int NA = C::NA, NB = C::NB, STAGE = C::STAGE;
  constexpr int NS = FM * FN / 2;  // epilogue stores per wave per tile
  static_assert(FN % 2 == 0 && TN % 32 == 0, "column pairs");
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int T = p.mblocks * p.nblocks;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, gx = gridDim.x >> 3;
  const int q8 = T >> 3, r8 = T & 7;
  const int tbeg = xcd * q8 + (xcd < r8 ? xcd : r8), tcnt = q8 + (xcd < r8 ? 1 : 0);
  if (slot >= tcnt) return;  // (whole workgroup: no barrier reached)
  const int nmine = (tcnt - slot + gx - 1) / gx;
  const int K = p.ntaps * p.cin;
  const int nk = (K + KE - 1) / KE;
  const int S = nmine * nk;
  const bf16* __restrict__ A = (const bf16*)p.a;
  const bf16* __restrict__ B = (const bf16*)p.b;
  const long hw = (long)p.ho * p.wo;

  // ---- issue side: the tile whose K-steps are being loaded ----------------------
  // Every K-step lies inside one tap (cin % KE == 0) and every tap is in range (source
  // grid = 2 x the iteration grid), so a piece's address is a per-tile lane offset (its
  // row's source pixel and chunk) plus a wave-uniform per-step offset (tap, channel) in
  // the buffer instruction's SGPR slot: no address arithmetic per load.
  const int sub = lane >> 3, pslot = lane & 7;
  const int cA0 = pslot ^ (sub >> 1), cA1 = cA0 ^ 4;
  unsigned voa[NA], vob[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
    vob[i] = (unsigned)(((long)pair_perm((wave * NB + i) * 8 + sub) * K + ((i & 1) ? cA1 : cA0) * VE) * 2);
  const long pix_ld = p.a_ld * 2;  // bytes per source pixel
  const unsigned hw32 = (unsigned)hw, wo32 = (unsigned)p.wo;
  dma::i32x4 ra, rb;
  int i_k = 0, i_j = 0, i_tap = 0, i_ch = 0;
  auto set_issue = [&](int j) {  // j-th tile of this workgroup
    const int tile = tbeg + slot + j * gx;
    const int mb = tile / p.nblocks;
    const unsigned m0 = (unsigned)mb * BM;
    const unsigned img0 = m0 / hw32, r0 = m0 - img0 * hw32, oh0 = r0 / wo32;
    const long p0 = ((long)img0 * p.hs + 2 * oh0) * p.ws + 2 * (r0 - oh0 * wo32);
    ra = dma::rsrc((uintptr_t)(A + p0 * p.a_ld + p.a_off));
    rb = dma::rsrc((uintptr_t)(B + (size_t)(tile - mb * p.nblocks) * BN * K));
    // source pixel of row m relative to row m0's: 2 x (its iteration-grid offset), each
    // iteration row spanning 2 source rows (image boundaries included: hs = 2 ho)
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const unsigned d = (wave * NA + i) * 8 + sub, m = m0 + d;
      const unsigned rows = (r0 % wo32 + d) / wo32, col = (r0 % wo32 + d) - rows * wo32;
      const unsigned px = rows * 2 * (unsigned)p.ws + 2 * col - 2 * (r0 % wo32);
      voa[i] = m < (unsigned)p.M ? px * (unsigned)pix_ld + ((i & 1) ? cA1 : cA0) * VE * 2 : dma::OOB;
    }
    i_k = i_tap = i_ch = 0;
  };
  auto advance = [&]() {
    if (++i_k == nk) {
      if (++i_j < nmine) set_issue(i_j);
      return;
    }
    i_ch += KE;
    if (i_ch == p.cin) { i_ch = 0; ++i_tap; }
  };
  const unsigned lds0 = dma::lds_addr(smem);
  auto issue = [&](int buf) {
    const unsigned As = lds0 + buf * STAGE, Bs = As + BM * 128;
    const unsigned sa = (unsigned)((((i_tap >> 1) * p.ws + (i_tap & 1)) * pix_ld) + i_ch * 2);
    const unsigned sb = (unsigned)(i_k * KE * 2);
#pragma unroll
    for (int i = 0; i < NA; ++i) dma::lds16s(voa[i], ra, sa, As + (wave * NA + i) * 1024);
#pragma unroll
    for (int i = 0; i < NB; ++i) dma::lds16s(vob[i], rb, sb, Bs + (wave * NB + i) * 1024);
  };

  f32x4 acc[FM][FN];
  auto zero = [&]() {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero();
  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + BM * 128;
    const int frow = lane & 15, fg = lane >> 4;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      uint4 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const uint4*>(As + swz_off(wm * TM + i * 16 + frow, kk * 4 + fg));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const uint4*>(Bs + swz_off(wn * TN + j * 16 + frow, kk * 4 + fg));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) Mma<bf16>::run(acc[i][j], bfr[j], af[i]);  // C^T
    }
  };
  auto epilogue = [&](int j) {
    const int tile = tbeg + slot + j * gx;
    const int mb = tile / p.nblocks;
    const long m0 = (long)mb * BM;
    const int n0 = (tile - mb * p.nblocks) * BN;
    const __amdgpu_buffer_rsrc_t os = dma::brsrc((const bf16*)p.out + m0 * p.out_ld + p.out_off + n0);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const int row = wm * TM + i * 16 + (lane & 15);
      const bool ok = m0 + row < p.M;
#pragma unroll
      for (int q = 0; q < FN / 2; ++q) {
        const int c = wn * TN + 32 * q + 8 * (lane >> 4);
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) o[k] = (bf16)acc[i][2 * q + (k >> 2)][k & 3];
        const unsigned off = (unsigned)(((long)row * p.out_ld + c) * 2);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dma::i32x4, o), os, ok ? off : dma::OOB, 0, 0);
      }
    }
  };

  // ---- main loop: one flat K-step sequence over this workgroup's tiles ---------------
  set_issue(0);
  issue(0);
  advance();
  int ck = 0, cj = 0;  // compute side: K-step within tile, tile
  bool stored = false;
  for (int g = 0; g < S; ++g) {
    if (stored) dma::wait_vm<NS>(); else dma::wait_vm<0>();  // (the stores were issued after the loads)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (g + 1 < S) {
      issue((g + 1) & 1);
      advance();
    }
    compute(g & 1);
    stored = false;
    if (++ck == nk) {
      epilogue(cj);
      zero();
      ck = 0;
      ++cj;
      stored = true;
    }
  }
}

// The same persistent walk for the Conv2DTranspose FORWARD in training (bf16, up6-up8):
// C[m][n] = x[m] . K[n] with n = tap * Cout + co, bias + ReLU in the epilogue, each lane's 8
// consecutive columns (one tap) stored as 16 bytes at output pixel (2i + tap/2, 2j + tap%2),
// and the BN partial sums (sum v, sum v^2 of the stored values' fp32 precursors) kept in
// registers for the whole launch.  For the sums to stay in registers a workgroup keeps ONE
// column block: slot s of an XCD takes column block s % nblocks and every
// (Gx/nblocks)-th row block of the XCD's contiguous row-block range (the nblocks
// workgroups of a row block run side by side and share its x rows in L2).  Stats rows:
// one per (XCD, slot / nblocks, wave row), every (row, column) written exactly once (a
// workgroup without tiles writes zeros).
// TRAIN: the training flags (ReLU + BN sums, no affine) as constants: with runtime flags the
// compiler computes both sides of each flag test per value and selects (two selects and an FMA
// per value that the training step never needs).
template <int BM, int BN, int WM, int WN, bool TRAIN = false>
__global__ __launch_bounds__(WM * WN * 64) void tconv_fwd2p_kernel(const FwdArgs p) {
  using C = Fwd2Cfg<bf16, BM, BN, WM, WN, 2>;
  constexpr int VE = C::VE, KE = C::KE, TM = C::TM, TN = C::TN, FM = C::FM, FN = C::FN;
  constexpr int NA = C::NA, NB = C::NB, STAGE = C::STAGE, FP = FN / 2;
  constexpr int NS = FM * FP;  // epilogue stores per wave per tile
  static_assert(FN % 2 == 0 && TN % 32 == 0, "column pairs");
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE + 3 * BN * 4];
  float* bias_s = reinterpret_cast<float*>(smem + 2 * STAGE);  // [3][BN]: bias, affine scale, shift

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave / WN, wn = wave % WN;
  const int frow = lane & 15, g = lane >> 4;
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3, gx = gridDim.x >> 3;
  const int nb = slot % p.nblocks, s2 = slot / p.nblocks, gs = gx / p.nblocks;
  const int q8 = p.mblocks >> 3, r8 = p.mblocks & 7;
  const int mbeg = xcd * q8 + (xcd < r8 ? xcd : r8), mcnt = q8 + (xcd < r8 ? 1 : 0);
  const int nmine = s2 < mcnt ? (mcnt - s2 + gs - 1) / gs : 0;
  const int K = p.cin;
  const int nk = K / KE;
  const int S = nmine * nk;
  const int n0 = nb * BN;
  const bf16* __restrict__ A = (const bf16*)p.a;
  const bf16* __restrict__ B = (const bf16*)p.b;
  const unsigned hw32 = (unsigned)((long)p.ho * p.wo), wo32 = (unsigned)p.wo;
  const bool relu = TRAIN || (p.flags & CNNITMO_RELU), stats = TRAIN || (p.flags & CNNITMO_STATS);
  const bool aff = !TRAIN && (p.flags & CNNITMO_AFFINE);
  for (int i = tid; i < BN; i += WM * WN * 64) {
    const int n = n0 + i, co = n - (n / p.cout) * p.cout;
    bias_s[i] = !p.bias ? 0.f : p.bias[(p.flags & CNNITMO_BIAS_PER_COL) ? n : co];
    bias_s[BN + i] = aff ? p.aff_scale[co] : 1.f;
    bias_s[2 * BN + i] = aff ? p.aff_shift[co] : 0.f;
  }
  // the lane's two 8-column groups: tap and channel (8 | cout: a group never straddles taps)
  int tq[FP], cq[FP];
#pragma unroll
  for (int q = 0; q < FP; ++q) {
    const int n = n0 + wn * TN + 32 * q + 8 * g;
    tq[q] = n / p.cout;
    cq[q] = n - tq[q] * p.cout;
  }

  const int sub = lane >> 3, pslot = lane & 7;
  const int cA0 = pslot ^ (sub >> 1), cA1 = cA0 ^ 4;
  unsigned voa[NA], vob[NB];
#pragma unroll
  for (int i = 0; i < NB; ++i)
    vob[i] = (unsigned)(((long)pair_perm((wave * NB + i) * 8 + sub) * K + ((i & 1) ? cA1 : cA0) * VE) * 2);
  dma::i32x4 ra, rb;
  int i_k = 0, i_j = 0;
  auto set_issue = [&](int j) {
    const unsigned m0 = (unsigned)(mbeg + s2 + j * gs) * BM;
    ra = dma::rsrc((uintptr_t)(A + (size_t)m0 * p.a_ld + p.a_off));
    rb = dma::rsrc((uintptr_t)(B + (size_t)n0 * K));
#pragma unroll
    for (int i = 0; i < NA; ++i) {
      const unsigned d = (wave * NA + i) * 8 + sub;
      voa[i] = m0 + d < (unsigned)p.M ? (unsigned)((d * p.a_ld + ((i & 1) ? cA1 : cA0) * VE) * 2) : dma::OOB;
    }
    i_k = 0;
  };
  auto advance = [&]() {
    if (++i_k == nk && ++i_j < nmine) set_issue(i_j);
  };
  const unsigned lds0 = dma::lds_addr(smem);
  auto issue = [&](int buf) {
    const unsigned As = lds0 + buf * STAGE, Bs = As + BM * 128;
    const unsigned so = (unsigned)(i_k * KE * 2);
#pragma unroll
    for (int i = 0; i < NA; ++i) dma::lds16s(voa[i], ra, so, As + (wave * NA + i) * 1024);
#pragma unroll
    for (int i = 0; i < NB; ++i) dma::lds16s(vob[i], rb, so, Bs + (wave * NB + i) * 1024);
  };

  f32x4 acc[FM][FN];
  auto zero = [&]() {
#pragma unroll
    for (int i = 0; i < FM; ++i)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  zero();
  float s1[FP][8], s2v[FP][8];
#pragma unroll
  for (int q = 0; q < FP; ++q)
#pragma unroll
    for (int k = 0; k < 8; ++k) s1[q][k] = s2v[q][k] = 0.f;
  auto compute = [&](int buf) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + BM * 128;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      uint4 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; ++i)
        af[i] = *reinterpret_cast<const uint4*>(As + swz_off(wm * TM + i * 16 + frow, kk * 4 + g));
#pragma unroll
      for (int j = 0; j < FN; ++j)
        bfr[j] = *reinterpret_cast<const uint4*>(Bs + swz_off(wn * TN + j * 16 + frow, kk * 4 + g));
#pragma unroll
      for (int i = 0; i < FM; ++i)
#pragma unroll
        for (int j = 0; j < FN; ++j) Mma<bf16>::run(acc[i][j], bfr[j], af[i]);  // C^T
    }
  };
  const float invw = 1.f / (float)p.wo;
  const long out_px = (long)p.out_ld * 2;  // bytes per output pixel
  auto epilogue = [&](int j) {
    const unsigned m0 = (unsigned)(mbeg + s2 + j * gs) * BM;
    const unsigned img0 = m0 / hw32, r0 = m0 - img0 * hw32, i0 = r0 / wo32, j0 = r0 - i0 * wo32;
    // output pixel of input pixel (i, j) and tap (a, b): (2i + a, 2j + b) of a 2h x 2w image;
    // relative to output row 2 i0 of image img0, input row offset R from row i0 (across
    // image boundaries too: 2h output rows per h input rows)
    const long obase = ((long)img0 * 2 * p.ho + 2 * i0) * 2 * p.wo;
    const __amdgpu_buffer_rsrc_t os = dma::brsrc((const bf16*)p.out + obase * p.out_ld + p.out_off);
#pragma unroll
    for (int i = 0; i < FM; ++i) {
      const unsigned d = wm * TM + i * 16 + frow;
      const bool ok = m0 + d < (unsigned)p.M;
      const unsigned pos = j0 + d;
      int R = (int)((float)pos * invw);
      int col = (int)pos - R * (int)wo32;
      if (col >= (int)wo32) { ++R; col -= (int)wo32; }
      if (col < 0) { --R; col += (int)wo32; }
#pragma unroll
      for (int q = 0; q < FP; ++q) {
        const int cl = wn * TN + 32 * q + 8 * g;
        const float4 b0 = *reinterpret_cast<const float4*>(bias_s + cl);
        const float4 b1 = *reinterpret_cast<const float4*>(bias_s + cl + 4);
        const float bj[8] = {b0.x, b0.y, b0.z, b0.w, b1.x, b1.y, b1.z, b1.w};
        float sj[8], hj[8];
        if (aff) {
          const float4 c0 = *reinterpret_cast<const float4*>(bias_s + BN + cl);
          const float4 c1 = *reinterpret_cast<const float4*>(bias_s + BN + cl + 4);
          const float4 d0 = *reinterpret_cast<const float4*>(bias_s + 2 * BN + cl);
          const float4 d1 = *reinterpret_cast<const float4*>(bias_s + 2 * BN + cl + 4);
          sj[0] = c0.x; sj[1] = c0.y; sj[2] = c0.z; sj[3] = c0.w; sj[4] = c1.x; sj[5] = c1.y; sj[6] = c1.z; sj[7] = c1.w;
          hj[0] = d0.x; hj[1] = d0.y; hj[2] = d0.z; hj[3] = d0.w; hj[4] = d1.x; hj[5] = d1.y; hj[6] = d1.z; hj[7] = d1.w;
        }
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float v = acc[i][2 * q + (k >> 2)][k & 3] + bj[k];
          if (relu) v = fmaxf(v, 0.f);
          if (aff) v = fmaf(v, sj[k], hj[k]);
          const float vs = ok ? v : 0.f;
          s1[q][k] += vs;
          s2v[q][k] = fmaf(vs, vs, s2v[q][k]);
          o[k] = (bf16)v;
        }
        const unsigned opx = (unsigned)((2 * R + (tq[q] >> 1)) * 2 * p.wo + 2 * col + (tq[q] & 1));
        const unsigned off = (unsigned)(opx * out_px + cq[q] * 2);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(dma::i32x4, o), os, ok ? off : dma::OOB, 0, 0);
      }
    }
  };

  set_issue(0);  // (a workgroup without tiles computes addresses it never uses)
  if (S > 0) {
    issue(0);
    advance();
  }
  int ck = 0, cj = 0;
  bool stored = false;
  for (int t = 0; t < S; ++t) {
    if (stored) dma::wait_vm<NS>(); else dma::wait_vm<0>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    __builtin_amdgcn_sched_barrier(0);
    if (t + 1 < S) {
      issue((t + 1) & 1);
      advance();
    }
    compute(t & 1);
    stored = false;
    if (++ck == nk) {
      epilogue(cj);
      zero();
      ck = 0;
      ++cj;
      stored = true;
    }
  }
  if (stats) {  // fold the 16 pixel lanes, one row per (XCD, slot / nblocks, wave row)
    const long row = ((long)xcd * gs + s2) * WM + wm;
    float* st = p.stats + row * 2 * p.N;
#pragma unroll
    for (int q = 0; q < FP; ++q)
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        float a1 = s1[q][k], a2 = s2v[q][k];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          a1 += __shfl_xor(a1, o, 64);
          a2 += __shfl_xor(a2, o, 64);
        }
        if (frow == 0) {
          const int n = n0 + wn * TN + 32 * q + 8 * g + k;
          st[n] = a1;
          st[p.N + n] = a2;
        }
      }
  }
}

// ----------------------------------------------------------------------------
namespace {
struct Cfg2 {
  int bn;
};
// Tile choice (measured on MI355X, tools/bench_layers.py): the 8-wave 256x128
// tile with a 3-deep ring for N % 128 == 0; otherwise 4-wave 256-row tiles with a
// 2-deep ring (2 blocks/CU hide the gather latency better than a deeper ring at
// 1 block/CU).  N == 32 stays on v1 (see use_fwd2()).
Cfg2 pick2(int N) {
  if (N % 128 == 0) return {128};
  if (N % 64 == 0) return {64};
  if (N % 96 == 0) return {96};
  return {32};
}

int stages_for(int bn) { return bn == 128 ? 3 : 2; }

template <typename T, int BM, int BN, int WM, int WN>
void launch_st(const FwdArgs& a, hipStream_t s, dim3 grid) {
  if (stages_for(BN) == 2)
    hipLaunchKernelGGL((igemm_fwd2_kernel<T, BM, BN, WM, WN, 2>), grid, dim3(WM * WN * 64), 0, s, a);
  else
    hipLaunchKernelGGL((igemm_fwd2_kernel<T, BM, BN, WM, WN, 3>), grid, dim3(WM * WN * 64), 0, s, a);
}
}  // namespace

int fwd2_stat_rows(long m) { return (int)((m + 255) / 256); }

// Row tile of the v2 launch: 128 x 128 tiles with a 2-deep ring (64-68 KB, two
// workgroups per CU: one workgroup's prologue and LDS-staged epilogue overlap the
// other's MFMAs) for the bf16 Conv2DTranspose input gradient (up6/up7 0.87/1.93 ->
// 0.83/1.81 ms) and for every fp32 launch with N % 128 == 0 (inference dec6-dec8
// 15.4-15.8 -> 15.0-15.3 ms); launches with BN partial sums keep 256-row tiles (the
// sums rows are per 256 rows).
int fwd2_bm(const FwdArgs& a, bool bf16) {
  if (a.N % 128 || a.stats) return 256;
  return (!bf16 || (a.ntaps == 4 && a.scale == 2)) ? 128 : 256;
}
bool fwd2_handles(int N) { return N != 32; }

// bf16 Conv2DTranspose input gradient (K = 1024 / 2048): 256 x 256 tiles (8 waves of
// 128 x 64, 2-deep 128 KB ring, one workgroup per CU) move half the LDS-DMA bytes per
// MFMA of the 128 x 128 tiles: up6 / up7 0.83 / 1.80 -> 0.70 / 1.66 ms
// (profiles/r03z_ab_fwd2_256.txt)
bool fwd2_t256(const FwdArgs& a, bool bf16) {
  return bf16 && a.ntaps == 4 && a.scale == 2 && a.N % 256 == 0 && !a.stats;
}

// ... as the persistent kernel (igemm_fwd2p_kernel) for the input-gradient geometry when
// nothing is asked of the epilogue but the store (others: the one-tile-per-workgroup launch)
bool fwd2_pers(const FwdArgs& a, bool bf16) {
  return fwd2_t256(a, bf16) && !a.scatter && !a.border && !a.bias && !a.flags &&
         a.hs == 2 * a.ho && a.ws == 2 * a.wo && a.cin % 64 == 0 && a.dyc == 0xa5 && a.dxc == 0x99 && !a.cin1 && a.M < (1L << 31) &&
         (2L * (256 / a.wo + 2) + 2) * a.ws * a.a_ld * 2 < (1L << 31);  // (a tile's source span: 32-bit offsets)
}

static int cu_count();
// the bf16 Conv2DTranspose forward (bias or folded per-column bias, ReLU, inference affine,
// BN partial sums) on tconv_fwd2p_kernel (others: tconv_stream / tconv_ws).  The plan
// (tfwd2p_handles) depends on the sizes and flags only, so cnnitmo_tconv2x2_stat_rows (which asks
// it with dense views) always sizes the stats buffer for the kernel the launch will run; the view
// conditions (16-byte alignment, 32-bit buffer offsets of the strides) are not part of the plan
// but requirements of the launch: a view that fails them is an error, never a silent fall-back to
// a kernel with a different stat-row count.
bool tfwd2p_handles(const FwdArgs& a, bool bf16) {
  const int gx = std::max(cu_count() / 8, 1);
  return bf16 && a.scatter && a.ntaps == 1 && a.N % 256 == 0 && a.cin % 64 == 0 && a.cout % 8 == 0 &&
         !a.border && !(a.flags & ~(CNNITMO_RELU | CNNITMO_STATS | CNNITMO_BIAS_PER_COL | CNNITMO_AFFINE)) &&
         a.M < (1L << 31) && gx % (a.N / 256) == 0;
}
long tfwd2p_stat_rows(const FwdArgs& a) { return 8L * (std::max(cu_count() / 8, 1) / (a.N / 256)) * 2; }
int launch_tfwd2p(FwdArgs a, hipStream_t s, const char* what) {
  CNN_REQUIRE(tfwd2p_handles(a, true), "%s: unsupported by tconv_fwd2p", what);
  CNN_REQUIRE(a.a_off % 8 == 0 && a.a_ld % 8 == 0 && a.out_ld % 8 == 0 && a.out_off % 8 == 0,
              "%s: views must be 16-byte aligned", what);
  CNN_REQUIRE((long)256 * a.a_ld * 2 < (1L << 31) && (2L * (256 / a.wo + 3)) * 2 * a.wo * a.out_ld * 2 < (1L << 31),
              "%s: row strides exceed the kernel's 32-bit buffer offsets", what);
  CNN_REQUIRE(!(a.flags & CNNITMO_STATS) || a.stats, "%s: STATS without buffer", what);
  a.mblocks = (int)((a.M + 255) / 256);
  a.nblocks = a.N / 256;
  const int g = 8 * std::max(cu_count() / 8, 1);
  const int fl = a.flags & ~CNNITMO_BIAS_PER_COL;
  if (fl == (CNNITMO_RELU | CNNITMO_STATS))
    hipLaunchKernelGGL((tconv_fwd2p_kernel<256, 256, 2, 4, true>), dim3((unsigned)g), dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((tconv_fwd2p_kernel<256, 256, 2, 4>), dim3((unsigned)g), dim3(512), 0, s, a);
  return cnnitmo_check_launch(what);
}

static int cu_count() {
  static const int n = [] {
    int dev = 0, v = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return v;
  }();
  return n;
}

template <typename T>
int launch_fwd2(FwdArgs a, hipStream_t s, const char* what) {
  constexpr int VE = Vec16<T>::N;
  CNN_REQUIRE(a.N % 32 == 0, "%s: output columns %d not a multiple of 32", what, a.N);
  CNN_REQUIRE(a.cin % VE == 0, "%s: channels per tap %d not a multiple of %d", what, a.cin, VE);
  CNN_REQUIRE(a.a_ld % VE == 0 && a.a_off % VE == 0 && a.out_ld % VE == 0 && a.out_off % VE == 0,
              "%s: views must be 16-byte aligned", what);
  CNN_REQUIRE(!a.scatter || a.cout % VE == 0, "%s: scatter needs cout %% %d == 0", what, VE);
  CNN_REQUIRE(a.M > 0 && a.ntaps >= 1 && a.ntaps <= 9, "%s: bad sizes", what);
  const Cfg2 c = pick2(a.N);
  if constexpr (sizeof(T) == 2) {
    if (fwd2_pers(a, true)) {
      a.mblocks = (int)((a.M + 255) / 256);
      a.nblocks = a.N / 256;
      const long t = (long)a.mblocks * a.nblocks;
      CNN_REQUIRE(t < (1L << 31), "%s: grid too large", what);
      CNN_REQUIRE((long)256 * a.out_ld * 2 + (long)a.N * 2 < (1L << 31), "%s: output row too wide", what);
      const long g = 8 * std::min((long)std::max(cu_count() / 8, 1), (t + 7) / 8);  // one per CU, 8 | grid
      hipLaunchKernelGGL((igemm_fwd2p_kernel<256, 256, 2, 4>), dim3((unsigned)g), dim3(512), 0, s, a);
      return cnnitmo_check_launch(what);
    }
    if (fwd2_t256(a, true)) {
      a.mblocks = (int)((a.M + 255) / 256);
      a.nblocks = a.N / 256;
      CNN_REQUIRE((long)a.mblocks * a.nblocks < (1L << 31), "%s: grid too large", what);
      hipLaunchKernelGGL((igemm_fwd2_kernel<T, 256, 256, 2, 4, 2>), dim3((unsigned)(a.mblocks * a.nblocks)),
                         dim3(512), 0, s, a);
      return cnnitmo_check_launch(what);
    }
  }
  if (fwd2_bm(a, sizeof(T) == 2) == 128) {
    {
      a.mblocks = (int)((a.M + 127) / 128);
      a.nblocks = a.N / 128;
      CNN_REQUIRE((long)a.mblocks * a.nblocks < (1L << 31), "%s: grid too large", what);
      hipLaunchKernelGGL((igemm_fwd2_kernel<T, 128, 128, 2, 4, 2>), dim3((unsigned)(a.mblocks * a.nblocks)),
                         dim3(512), 0, s, a);
      return cnnitmo_check_launch(what);
    }
  }
  a.mblocks = (int)((a.M + 255) / 256);
  a.nblocks = a.N / c.bn;
  const long total = (long)a.mblocks * a.nblocks;
  CNN_REQUIRE(total < (1L << 31), "%s: grid too large", what);
  const dim3 grid((unsigned)total);
  switch (c.bn) {
    case 128: launch_st<T, 256, 128, 4, 2>(a, s, grid); break;
    case 96: launch_st<T, 256, 96, 4, 1>(a, s, grid); break;
    case 64: launch_st<T, 256, 64, 4, 1>(a, s, grid); break;
    default: launch_st<T, 256, 32, 4, 1>(a, s, grid); break;
  }
  return cnnitmo_check_launch(what);
}

template int launch_fwd2<bf16>(FwdArgs, hipStream_t, const char*);
template int launch_fwd2<float>(FwdArgs, hipStream_t, const char*);
