// Conv2DTranspose(2, strides=2) input gradient for the deep up-sampling layers
// (model.py:200, ConvBNTranspose of up6 / up7: K = 4*cout = 2048 / 1024, N = cin = 512)
// as a persistent GEMM with the weights streamed through LDS in K chunks and the
// activation gradient read straight into registers.
//
//   dx[p][ci] = sum_{tap=(a,b), co} dout[(2y+a, 2x+b)][co] * kT[ci][tap*cout + co]
//
// tconv_ws keeps a whole [BN][K] weight block resident, which needs K <= 512; at
// K = 1024 / 2048 the block does not fit, and these two layers ran on the generic
// implicit GEMM (igemm_fwd2, 256 x 256 tiles), whose A and B both go through
// per-lane LDS-DMA and whose tiles are not persistent (ring prologue and LDS-staged
// epilogue per tile).  Here:
//   * a workgroup (8 waves, one per CU) owns a 128-column block for its whole life and
//     walks 256-pixel passes (32 pixels per wave); per pass the K dimension is swept in
//     chunks of 256 (8 K-steps of 32): chunk c+1's weights [128][256] (64 KB) are read
//     into registers during chunk c and written to the other half of a 128 KB LDS double
//     buffer before the chunk's barrier (one barrier per 8 K-steps);
//   * A (the four dout pixels of a dx pixel, each cout contiguous: a K-step of 32 lies in
//     one tap) comes from HBM / L2 straight into registers, KC_PD K-steps in flight,
//     pipelined across chunk and pass boundaries; every load is a plain load the
//     compiler counts (no LDS-DMA whose vmcnt it cannot see);
//   * the MFMA runs with the operands swapped (C^T: a lane holds 4 consecutive channels
//     of one pixel); with pair_perm weight rows a lane's fragment pair holds 8
//     consecutive channels and the epilogue stores whole 128-byte lines from registers
//     (line_pair), no LDS staging;
//   * the 4 column blocks of a pixel range run on one XCD (blockIdx % 8), so 3 of the 4
//     reads of every A line are L2 hits.
#include <cstdio>

#include "igemm_common.h"

namespace {

#ifndef KC_DEFAULT_ON
#define KC_DEFAULT_ON 0
#endif
#ifndef KC_FM_DEF
#define KC_FM_DEF 2
#endif
#ifndef KC_PD_DEF
#define KC_PD_DEF 4
#endif
constexpr int KC_NW = 8, KC_BN = 128, KC_KSC = 8, KC_FM = KC_FM_DEF, KC_PD = KC_PD_DEF;
constexpr int KC_TP = 16 * KC_FM * KC_NW;       // pixels per pass
constexpr int KC_CHUNK = KC_KSC * KC_BN * 64;   // bytes per weight chunk (64 KB)
constexpr int KC_BPT = KC_CHUNK / 16 / (KC_NW * 64);  // 16-byte weight pieces per thread per chunk (8)

struct KCArgs {
  const bf16* dout;  // [n][2h][2w][cout]
  const bf16* kT;    // [cin][4*cout]: row = input channel, k = tap*cout + co
  bf16* dx;          // [n*h*w][cin]
  int nimg, h, w, cin;
  int nblk, gpx;
  long passes;
};

// 64-byte LDS rows, 16-byte piece c of row q at c ^ (((q >> 2) & 1) << 1): the B fragment
// windows (16 consecutive rows) are conflict-free (tools/check_swizzle.py, the halo image)
__device__ __forceinline__ int kc_rsw(int row, int piece) { return (row << 6) + ((piece ^ (((row >> 2) & 1) << 1)) << 4); }

// NKC = K / 256 chunks; COUT = 64 * NKC (cout 256: up7, 512: up6)
template <int NKC>
__global__ __launch_bounds__(KC_NW * 64) void tconv_kc_kernel(const KCArgs p) {
  constexpr int COUT = 64 * NKC, K = 4 * COUT, NKS = NKC * KC_KSC;
  constexpr int FM = KC_FM, FN = KC_BN / 16, FP = FN / 2, PD = KC_PD;
  static_assert(KC_KSC % PD == 0, "ring positions are compile-time within a chunk");
  __shared__ __attribute__((aligned(1024))) char smem[2 * KC_CHUNK];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int xcd = blockIdx.x & 7, bi = blockIdx.x >> 3;
  const int nb = bi % p.nblk, grp = bi / p.nblk;
  const int gidx = xcd * p.gpx + grp, ngrp = 8 * p.gpx;
  const long per = (p.passes + ngrp - 1) / ngrp;
  const long q0 = gidx * per, q1 = q0 + per < p.passes ? q0 + per : p.passes;
  if (q0 >= q1) return;  // (whole workgroup: no barrier is left waiting)
  const int n0 = nb * KC_BN;
  const int hw = p.h * p.w;
  const long P = (long)p.nimg * hw;
  const int W2 = 2 * p.w;
  const int frow = lane & 15, kq = lane >> 4;

  // ---- weight chunk staging: thread pieces u = tid + 512 i; row nn = u >> 5 (16 + i
  // apart), 16-byte piece pi = u & 31 of its 512 contiguous bytes (coalesced reads);
  // LDS row = ksl * 128 + nn holds block column pair_perm(nn) (16-byte stores)
  int boff[KC_BPT];
  const int pi = tid & 31, ksl = pi >> 2, bpc = pi & 3;
#pragma unroll
  for (int i = 0; i < KC_BPT; ++i) {
    const int nn = (tid >> 5) + 16 * i;
    boff[i] = (n0 + pair_perm(nn)) * K + ksl * 32 + bpc * 8;
  }
  const int bdst = kc_rsw(ksl * KC_BN + (tid >> 5), bpc);  // + 1024 * i (row + 16 i: same swizzle bit)
  uint4 breg[KC_BPT];
  auto loadB = [&](int kc) {
#pragma unroll
    for (int i = 0; i < KC_BPT; ++i) breg[i] = *reinterpret_cast<const uint4*>(p.kT + boff[i] + kc * 256);
  };
  auto storeB = [&](int buf) {
#pragma unroll
    for (int i = 0; i < KC_BPT; ++i) *reinterpret_cast<uint4*>(smem + buf * KC_CHUNK + bdst + 1024 * i) = breg[i];
  };

  // ---- A: the lane's two fragment rows of pass q (clamped for a tail pass)
  auto bases = [&](long q, const bf16** ab) {
#pragma unroll
    for (int f = 0; f < FM; ++f) {
      const long pix = q * KC_TP + wave * (16 * FM) + f * 16 + frow, pc = pix < P ? pix : P - 1;
      const int ip = (int)pc, img = ip / hw, rem = ip - img * hw, y = rem / p.w, x = rem - y * p.w;
      ab[f] = p.dout + (((size_t)img * 2 * p.h + 2 * y) * W2 + 2 * x) * COUT + kq * 8;
    }
  };
  // K-step g (32 channels of one tap): element offset inside the pixel's 2x2 dout block
  auto aoff = [&](int g) {
    const int k0 = g * 32, tap = k0 / COUT, co = k0 - tap * COUT;
    return ((tap >> 1) * W2 + (tap & 1)) * COUT + co;
  };
  auto loadA = [&](const bf16* const* ab, int g, uint4* dst) {
    const int o = aoff(g);
#pragma unroll
    for (int f = 0; f < FM; ++f) dst[f] = *reinterpret_cast<const uint4*>(ab[f] + o);
  };

  uint4 Ab[PD][FM];
  const bf16* abc[FM];
  const bf16* abn[FM];
  bases(q0, abc);
  loadB(0);
#pragma unroll
  for (int j = 0; j < PD - 1; ++j) loadA(abc, j, Ab[j]);
  storeB(0);
  __syncthreads();
  int c = 0;  // chunks consumed (LDS buffer c & 1)
  for (long q = q0; q < q1; ++q) {
    const bool more = q + 1 < q1;
    bases(more ? q + 1 : q, abn);  // (no next pass: harmless reloads of this one)
    f32x4 acc[FM][FN];
#pragma unroll
    for (int f = 0; f < FM; ++f)
#pragma unroll
      for (int j = 0; j < FN; ++j) acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int kc = 0; kc < NKC; ++kc) {
      const bool tail = !more && kc == NKC - 1;  // the launch's last chunk: nothing to stage
      if (!tail) loadB(kc + 1 < NKC ? kc + 1 : 0);
      const char* Bs = smem + (c & 1) * KC_CHUNK;
#pragma unroll
      for (int ks = 0; ks < KC_KSC; ++ks) {
        const int g = kc * KC_KSC + ks + PD - 1;  // K-step whose A this step loads
        const bool cur = g < NKS;
        const bf16* sel[FM];
#pragma unroll
        for (int f = 0; f < FM; ++f) sel[f] = cur ? abc[f] : abn[f];
        loadA(sel, cur ? g : g - NKS, Ab[(ks + PD - 1) % PD]);
        __builtin_amdgcn_sched_barrier(0);  // keep the loads ahead of this step's MFMAs
#pragma unroll
        for (int j = 0; j < FN; ++j) {
          const uint4 bfr = *reinterpret_cast<const uint4*>(Bs + kc_rsw(ks * KC_BN + j * 16 + frow, kq));
#pragma unroll
          for (int f = 0; f < FM; ++f) Mma<bf16>::run(acc[f][j], bfr, Ab[ks % PD][f]);  // C^T: lanes = pixels
        }
        __builtin_amdgcn_sched_barrier(0);
      }
      if (!tail) storeB((c + 1) & 1);  // the other buffer: every wave is past chunk c - 1
      __syncthreads();
      ++c;
    }
#pragma unroll
    for (int f = 0; f < FM; ++f) abc[f] = abn[f];
    // epilogue from registers: pairs (2q, 2q+1) hold 8 consecutive channels of a pixel;
    // pair couples go out as whole 128-byte lines, 8 pixels per store instruction
#pragma unroll
    for (int qp = 0; qp < FP; qp += 2) {
      uint4 pk[2][FM];
#pragma unroll
      for (int hq = 0; hq < 2; ++hq)
#pragma unroll
        for (int f = 0; f < FM; ++f) {
          bf16x8 o;
#pragma unroll
          for (int k = 0; k < 8; ++k) o[k] = (bf16)acc[f][2 * (qp + hq) + (k >> 2)][k & 3];
          pk[hq][f] = __builtin_bit_cast(uint4, o);
        }
#pragma unroll
      for (int f = 0; f < FM; ++f) {
        uint4 v1, v2;
        line_pair(pk[0][f], pk[1][f], frow, v1, v2);
        const int n = n0 + (qp + (frow >> 3)) * 32 + kq * 8;
        const long p1 = q * KC_TP + wave * (16 * FM) + f * 16 + (frow & 7), p2 = p1 + 8;
        if (p1 < P) *reinterpret_cast<uint4*>(p.dx + (size_t)p1 * p.cin + n) = v1;
        if (p2 < P) *reinterpret_cast<uint4*>(p.dx + (size_t)p2 * p.cin + n) = v2;
      }
    }
  }
}

// Off by default (CNNITMO_TCONV_KC=1 enables it): parity-green, but 1.38 / 2.87 ms on
// up6 / up7 against igemm_fwd2's 0.69 / 1.65 (profiles/r04b_kc_ab.txt)
bool kc_plan(int cin, int cout, int& nblk, int& gpx) {
  static const int en = [] {
    const char* e = getenv("CNNITMO_TCONV_KC");
    return e ? atoi(e) : KC_DEFAULT_ON;
  }();
  if (!en || (cout != 256 && cout != 512) || cin % KC_BN) return false;
  nblk = cin / KC_BN;
  if (nblk > 32 || 32 % nblk) return false;
  gpx = 32 / nblk;
  return true;
}

}  // namespace

bool tconv_kc_handles(int cin, int cout) {
  int nblk, gpx;
  return kc_plan(cin, cout, nblk, gpx);
}

const char* tconv_kc_name(int cin, int cout) {
  int nblk, gpx;
  if (!kc_plan(cin, cout, nblk, gpx)) return "";
  static thread_local char buf[48];
  snprintf(buf, sizeof(buf), "tconv_kc_kernel<%d>", cout / 64);
  return buf;
}

int launch_tconv_kc(const void* dout, int n, int h, int w, int cout, const void* kT, int cin, void* dx, hipStream_t s,
                    const char* what) {
  int nblk, gpx;
  CNN_REQUIRE(kc_plan(cin, cout, nblk, gpx), "%s: no K-chunked plan", what);
  CNN_REQUIRE((long)n * h * w < (1L << 31) && (long)cin * 4 * cout < (1L << 31), "%s: too large", what);
  KCArgs a;
  a.dout = (const bf16*)dout; a.kT = (const bf16*)kT; a.dx = (bf16*)dx;
  a.nimg = n; a.h = h; a.w = w; a.cin = cin;
  a.nblk = nblk; a.gpx = gpx;
  a.passes = ((long)n * h * w + KC_TP - 1) / KC_TP;
  const dim3 grid(8 * gpx * nblk), block(KC_NW * 64);
  if (cout == 512) hipLaunchKernelGGL((tconv_kc_kernel<8>), grid, block, 0, s, a);
  else hipLaunchKernelGGL((tconv_kc_kernel<4>), grid, block, 0, s, a);
  return cnnitmo_check_launch(what);
}
