// First layer of the U-Net, Conv2D(32, 3, 'same') on the 3-channel SDR input
// (/root/reference/model.py:208), bf16, without an im2col round trip through HBM.
//
// The 3x3x3 patches of an output row segment (256 pixels) are built in LDS from
// the fp32 input rows (fused /255-input cast to bf16 and the zero padding of
// predict.py:59's pad-to-16 rows), so the layer reads 12 B and writes 64 B per
// pixel instead of 12 + 64 (im2col) + 64 + 64 (GEMM):
//
//   conv_c3_fwd_kernel    persistent (3 workgroups per CU); unit = RPB output rows x
//                         256 pixels, its RPB+2 input rows LDS-DMA'd double-buffered
//                         (the next unit's in flight); the MFMA operand is built from
//                         the fp32 LDS image in registers (lane = pixel), 8 MFMAs
//                         16x16x32 per wave and row against the weights held in
//                         registers, epilogue bias + ReLU (+ inference BN affine) +
//                         BN partial sums (one row per workgroup for the launch),
//                         one 16-byte store per (pixel, 8 channels) from registers.
//                         1.82 -> 1.07 ms at 1088x1920 b32 (4.7 TB/s; the earlier
//                         one-shot design staged the rows with scalar loads and
//                         built A and C tiles in LDS behind four barriers per row).
//   conv_c3_wgrad_kernel  dW[co][k] = sum_p dz[p][co] * col[p][k]: per 256-pixel unit
//                         the dz row and the columns go to LDS as [pixel][32] rows
//                         and are read transposed (ds_read_b64_tr_b16: pixels are
//                         the MFMA reduction axis); the next unit's loads are in
//                         flight under the current one; persistent grid, one fp32
//                         slab per workgroup, fixed-order fold.
//
// HBM-bound: fwd 12 B read + 64 B written per pixel (+ stats), wgrad 12 + 64 B read
// (fp32: 128 B written / read per pixel instead of 64).
//
// The forward also runs in fp32 (TO = float, the fp32 inference path of predict.py:62):
// the same per-lane operand (8 k-values gathered from the fp32 image) goes to the MFMA
// as two 16-byte fp32 fragments (Mma<float>: four 16x16x4 f32 MFMAs each) against the
// weights in the same k order, and each (pixel, 8 channels) leaves as two 16-byte
// stores: 12 B read + 128 B written per pixel, replacing im2col (128 B written, 128 B
// read back) + a 1-tap GEMM.
#include "dma.h"
#include "igemm_common.h"

namespace {

constexpr int SEG = 256;  // pixels per row segment (one per thread)
constexpr int RPB = 4;    // output rows per forward workgroup

// Persistent forward: workgroup b takes units b, b + G, ... (unit = RPB output rows x
// 256 pixels).  The unit's RPB+2 input rows (264 pixels from w0-4, so every 16-byte
// piece is aligned to the row's 4-pixel grid) go to LDS by LDS-DMA, double-buffered:
// the next unit's pieces are in flight while the current unit is computed.  Each wave
// owns 64 pixels of a row and builds its MFMA operand straight from the fp32 image
// (lane = pixel, 8 k-values per lane group); the MFMA runs with the operands swapped
// and pair_perm weight rows, so a lane holds 8 consecutive output channels of one
// pixel: one 16-byte store per (pixel, 8 channels) from registers, no barrier in the
// row loop.
constexpr int XPW = SEG + 8;                // staged pixels per row (w0-4 .. w0+SEG+4)
constexpr int XRW = XPW * 3;                // floats per staged row (792)
constexpr int XPC = XRW / 4;                // 16-byte pieces per staged row (198)
constexpr int XNI = ((RPB + 2) * XPC + 63) / 64;  // 64-piece DMA instructions per unit (19)
constexpr int XBUF = XNI * 64 * 4;          // floats per LDS buffer (sink-padded)
#ifndef C3_GRID
#define C3_GRID 768                         // persistent workgroups (3 per CU on 256 CUs)
#endif

struct C3Fwd2 {
  const float* x;
  int n, hv, h, w, segs, rpn;
  long units;
  const void* wt;  // [32 cout][32 k] in TO
  const float* bias;
  void* out;
  long out_ld;
  int out_off;
  int flags;
  const float* aff_scale;
  const float* aff_shift;
  float* stats;  // [gridDim.x][2][32]
};

#ifndef C3_F32_LINES
#define C3_F32_LINES 0                      // fp32 stores as whole 128-byte lines (line_pair): neutral
#endif                                      // in the fp32 inference step and 23 VGPRs of spill
                                            // (profiles/r04o_c3_ab.txt), off by default
#ifndef C3_MINW
#define C3_MINW 3                           // waves per SIMD the register budget is sized for
#endif
template <typename TO, bool AFF>
__global__ __launch_bounds__(256, C3_MINW) void conv_c3_fwd_kernel(const C3Fwd2 a) {
  constexpr bool F32 = sizeof(TO) == 4;
  __shared__ __attribute__((aligned(1024))) float xs[2][XBUF];
  __shared__ float red[4][2][32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, pxl = lane & 15;
  const long G = gridDim.x;
  const int w3 = a.w * 3;
  // K order of this kernel (k' = 8g + e): lane groups 0-2 take kernel row r = g, its 9
  // consecutive (s, c) floats 0..7; group 3 takes float 8 of rows 0-2 and five zeros.
  // So a lane reads its 8 values at base + e * stride (stride 1 or one staged row).
  // (group 3's five zero slots re-read its first value: finite input times a zero weight)
  const int kb = (g < 3 ? g : 0) * XRW + (g < 3 ? 0 : 8);
  int koff[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) koff[e] = g < 3 ? e : (e < 3 ? e * XRW : 0);
  // weights (A operand: row i of block j = output channel pair_perm(16j + i), its
  // k' values gathered from the [32 cout][32 k] (k = tap*3 + c) rows)
  // (fp32: the 8 values as two 16-byte fragments, k order e = 4h + i in both operands)
  uint4 bw[2][F32 ? 2 : 1];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const TO* wr = (const TO*)a.wt + pair_perm(16 * j + pxl) * 32;
    float t[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) t[e] = g < 3 ? to_f32(wr[9 * g + e]) : (e < 3 ? to_f32(wr[9 * e + 8]) : 0.f);
    if constexpr (F32) {
      bw[j][0] = __builtin_bit_cast(uint4, f32x4{t[0], t[1], t[2], t[3]});
      bw[j][1] = __builtin_bit_cast(uint4, f32x4{t[4], t[5], t[6], t[7]});
    } else {
      bf16x8 tb;
#pragma unroll
      for (int e = 0; e < 8; ++e) tb[e] = (bf16)t[e];
      bw[j][0] = __builtin_bit_cast(uint4, tb);
    }
  }
  const bool relu = a.flags & CNNITMO_RELU, stats = a.flags & CNNITMO_STATS;
  float bj[8], sj[AFF ? 8 : 1], hj[AFF ? 8 : 1], s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int co = 8 * g + k;
    bj[k] = a.bias ? a.bias[co] : 0.f;
    if constexpr (AFF) {
      sj[k] = a.aff_scale[co];
      hj[k] = a.aff_shift[co];
    }
    s1[k] = s2[k] = 0.f;
  }
  struct Unit {
    int img, h0, w0;
  };
  auto unit = [&](long u) {
    const int seg = (int)(u % a.segs);
    const long rb = u / a.segs;
    return Unit{(int)(rb / a.rpn), (int)(rb % a.rpn) * RPB, seg * SEG};
  };
  // the unit's pieces: instruction t (pieces 64t .. 64t+63) by wave t % 4
  auto issue = [&](const Unit& un, int buf) {
    const dma::i32x4 rs = dma::rsrc((uintptr_t)(a.x + (size_t)un.img * a.hv * w3));  // per image: 32-bit offsets
    const long f00 = (long)(un.w0 - 4) * 3;
#pragma unroll
    for (int q = 0; q < (XNI + 3) / 4; ++q) {
      const int t = wave + 4 * q;
      if (t < XNI) {
        const int i = t * 64 + lane;
        const int r = i / XPC, pc = i - (i / XPC) * XPC;
        const int hh = un.h0 - 1 + r;
        const long f0 = f00 + pc * 4;
        // whole pieces only: the piece straddling the row end (w % 4 != 0) would read past
        // the tensor at its last row; it lands zeros here and is patched below
        const bool ok = i < (RPB + 2) * XPC && hh >= 0 && hh < a.hv && f0 >= 0 && f0 + 4 <= w3;
        dma::lds16(ok ? (unsigned)(((long)hh * w3 + f0) * 4) : dma::OOB, rs, (const char*)(xs[buf] + t * 256));
      }
    }
  };
  const int nis = (XNI - wave + 3) / 4;  // instructions per unit issued by this wave
  long u = blockIdx.x;
  int buf = 0;
  if (u < a.units) issue(unit(u), 0);
  for (; u < a.units; u += G) {
    const Unit un = unit(u);
    const int npx = min(SEG, a.w - un.w0), nrow = min(RPB, a.h - un.h0);
    __syncthreads();  // the other buffer's previous unit is consumed
    const bool more = u + G < a.units;
    if (more) issue(unit(u + G), buf ^ 1);
    dma::wait_vm_dyn(more ? nis : 0);  // this unit's pieces (and older stores) have landed
    __syncthreads();
    const float* X = xs[buf];
    if (w3 & 3) {  // the piece straddling the right frame edge: its nv valid floats by guarded loads
      const int nv = w3 & 3, e0 = w3 - nv - (int)((long)(un.w0 - 4) * 3);  // its first float in the staged row
      if (e0 < XRW && tid < (RPB + 2) * 4) {
        const int r = tid >> 2, k = tid & 3, hh = un.h0 - 1 + r;
        const bool ok = k < nv && hh >= 0 && hh < a.hv;
        const_cast<float*>(X)[r * XRW + e0 + k] = ok ? a.x[((size_t)un.img * a.hv + hh) * w3 + (w3 - nv) + k] : 0.f;
      }
      __syncthreads();
    }
    const int p0 = wave * 64;  // the wave's first pixel of the segment
    if (p0 < npx) {
#pragma unroll 1
      for (int rr = 0; rr < nrow; ++rr) {
        const long prow = ((long)un.img * a.h + un.h0 + rr) * a.w + un.w0;
        const float* src = X + rr * XRW + kb + (p0 + pxl + 3) * 3;
#pragma unroll
        for (int f = 0; f < 4; ++f) {
          f32x4 acc[2];
          if constexpr (F32) {
            float xv[8];
#pragma unroll
            for (int e = 0; e < 8; ++e) xv[e] = src[f * 48 + koff[e]];
            const uint4 x0 = __builtin_bit_cast(uint4, f32x4{xv[0], xv[1], xv[2], xv[3]});
            const uint4 x1 = __builtin_bit_cast(uint4, f32x4{xv[4], xv[5], xv[6], xv[7]});
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
              Mma<float>::run(acc[j], bw[j][0], x0);  // C^T: lanes = pixels
              Mma<float>::run(acc[j], bw[j][F32 ? 1 : 0], x1);
            }
          } else {
            bf16x8 xb;
#pragma unroll
            for (int e = 0; e < 8; ++e) xb[e] = from_f32<bf16>(src[f * 48 + koff[e]]);
            const uint4 xf = __builtin_bit_cast(uint4, xb);
#pragma unroll
            for (int j = 0; j < 2; ++j) {
              acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
              Mma<bf16>::run(acc[j], bw[j][0], xf);  // C^T: lanes = pixels
            }
          }
          const int px = p0 + f * 16 + pxl;
          const bool ok = px < npx;
          float v[8];
#pragma unroll
          for (int k = 0; k < 8; ++k) {
            float t = acc[k >> 2][k & 3] + bj[k];
            if (relu) t = fmaxf(t, 0.f);
            if constexpr (AFF) t = fmaf(t, sj[k], hj[k]);  // (explicit: the same rounding for every fragment)
            v[k] = t;
            const float vs = ok ? t : 0.f;
            s1[k] += vs;
            s2[k] += vs * vs;
          }
          if constexpr (F32 && C3_F32_LINES) {
            // a pixel's 32 fp32 channels are one 128-byte line: after one DPP exchange
            // (line_pair) store 1 writes pixels 0-7 and store 2 pixels 8-15 of the fragment
            // as whole lines (lane (pxl, g): channels 8g + 4*(pxl >> 3) .. +3)
            const uint4 lo = __builtin_bit_cast(uint4, float4{v[0], v[1], v[2], v[3]});
            const uint4 hi = __builtin_bit_cast(uint4, float4{v[4], v[5], v[6], v[7]});
            uint4 v1, v2;
            line_pair(lo, hi, pxl, v1, v2);
            const int q1 = p0 + f * 16 + (pxl & 7), q2 = q1 + 8, c = 8 * g + 4 * (pxl >> 3);
            if (q1 < npx) *reinterpret_cast<uint4*>((float*)a.out + (prow + q1) * a.out_ld + a.out_off + c) = v1;
            if (q2 < npx) *reinterpret_cast<uint4*>((float*)a.out + (prow + q2) * a.out_ld + a.out_off + c) = v2;
          } else if (ok) {
            TO* o = (TO*)a.out + (prow + px) * a.out_ld + a.out_off + 8 * g;
            Pack16<TO>::store(o, v);
            if constexpr (F32) Pack16<TO>::store(o + 4, v + 4);
          }
        }
      }
    }
    buf ^= 1;
  }
  if (stats) {
#pragma unroll
    for (int k = 0; k < 8; ++k)
#pragma unroll
      for (int o = 1; o < 16; o <<= 1) {
        s1[k] += __shfl_xor(s1[k], o, 64);
        s2[k] += __shfl_xor(s2[k], o, 64);
      }
    if (pxl == 0) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        red[wave][0][8 * g + k] = s1[k];
        red[wave][1][8 * g + k] = s2[k];
      }
    }
    __syncthreads();
    if (tid < 64) {
      const int q = tid >> 5, co = tid & 31;
      a.stats[(size_t)blockIdx.x * 64 + q * 32 + co] =
          (red[0][q][co] + red[1][q][co]) + (red[2][q][co] + red[3][q][co]);
    }
  }
}

// bf16 [pixel][32] LDS row image with the 32-byte column blocks XOR-swizzled by
// (row >> 3) & 1 (wgrad_halo.hip's trswz<32>), read transposed by ds_read_b64_tr_b16
__device__ __forceinline__ int tr32(int row, int col) {
  return row * 64 + ((((col >> 4) ^ (row >> 3)) & 1) << 5) + ((col & 15) << 1);
}

// Persistent weight gradient: unit = one 256-pixel row segment; its dz row (as
// [pixel][32] rows, trswz-swizzled by the DMA's source addressing) and its three
// input rows (the forward's fp32 image) are LDS-DMA'd double-buffered, the next
// unit's in flight under the current one.  Wave w reduces pixels 64w .. 64w+63:
// dz^T fragments by ds_read_b64_tr_b16, column fragments (8 pixels of one k) built
// from the fp32 image in registers; one [32][32] fp32 slab per workgroup.
constexpr int WDP = SEG * 4;                // dz pieces per unit (16 B = 8 channels)
constexpr int WXP = 3 * XPC;                // image pieces per unit (3 rows)
constexpr int WXI = (WXP + 63) / 64;        // image DMA instructions (10)
constexpr int WNI = WDP / 64 + WXI;         // DMA instructions per unit (26)
constexpr int WBUF = WDP * 16 + WXI * 1024; // bytes per LDS buffer
constexpr int WG_GRID = 768;                // persistent workgroups (3 per CU: 2 x 26 KB LDS each)

__global__ __launch_bounds__(256) void conv_c3_wgrad_kernel(const float* __restrict__ x, int n, int hv, int h,
                                                            int w, int segs, const bf16* __restrict__ dz,
                                                            long units, float* __restrict__ slabs) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * WBUF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  const long G = gridDim.x;
  const int w3 = w * 3;
  (void)n;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the lane's column k = 16j + li of the image: (r, s, c) offset (k >= 27: any finite value)
  int kof[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = 16 * j + li;
    kof[j] = k < 27 ? (k / 9) * XRW + ((k % 9) / 3) * 3 + k % 3 : 0;
  }
  struct Unit {
    int img, oh, w0;
  };
  auto unit = [&](long u) {
    const long row = u / segs;
    return Unit{(int)(row / h), (int)(row % h), (int)(u % segs) * SEG};
  };
  auto issue = [&](const Unit& un, int buf) {
    char* B = lds + buf * WBUF;
    const dma::i32x4 zs = dma::rsrc((uintptr_t)(dz + ((size_t)un.img * h + un.oh) * w * 32));
    const dma::i32x4 xr = dma::rsrc((uintptr_t)(x + (size_t)un.img * hv * w3));
    const long f00 = (long)(un.w0 - 4) * 3;
#pragma unroll
    for (int q = 0; q < (WNI + 3) / 4; ++q) {
      const int T = wave + 4 * q;
      if (T < WDP / 64) {  // dz: LDS row = pixel, 16-byte piece pc holds logical piece pc ^ swz
        const int row = T * 16 + (lane >> 2), pc = lane & 3;
        const int lp = pc ^ (((row >> 3) & 1) << 1);
        const bool ok = un.w0 + row < w;
        dma::lds16(ok ? (unsigned)(((un.w0 + row) * 32 + lp * 8) * 2) : dma::OOB, zs, B + T * 1024);
      } else if (T < WNI) {  // image rows oh-1 .. oh+1
        const int t = T - WDP / 64, i = t * 64 + lane;
        const int r = i / XPC, pc = i - (i / XPC) * XPC;
        const int hh = un.oh - 1 + r;
        const long f0 = f00 + pc * 4;
        const bool ok = i < WXP && hh >= 0 && hh < hv && f0 >= 0 && f0 + 4 <= w3;  // (edge piece: patched)
        dma::lds16(ok ? (unsigned)(((long)hh * w3 + f0) * 4) : dma::OOB, xr, B + WDP * 16 + t * 1024);
      }
    }
  };
  const int nis = (WNI - wave + 3) / 4;
  long u = blockIdx.x;
  int buf = 0;
  if (u < units) issue(unit(u), 0);
  for (; u < units; u += G) {
    const Unit un = unit(u);
    const int npx = min(SEG, w - un.w0);
    __syncthreads();
    const bool more = u + G < units;
    if (more) issue(unit(u + G), buf ^ 1);
    dma::wait_vm_dyn(more ? nis : 0);
    __syncthreads();
    const char* Ds = lds + buf * WBUF;
    const float* X = reinterpret_cast<const float*>(Ds + WDP * 16);
    if (w3 & 3) {  // the piece straddling the right frame edge: its nv valid floats by guarded loads
      const int nv = w3 & 3, e0 = w3 - nv - (un.w0 - 4) * 3;
      if (e0 < XRW && tid < 3 * 4) {
        const int r = tid >> 2, k = tid & 3, hh = un.oh - 1 + r;
        const bool ok = k < nv && hh >= 0 && hh < hv;
        const_cast<float*>(X)[r * XRW + e0 + k] = ok ? x[((size_t)un.img * hv + hh) * w3 + (w3 - nv) + k] : 0.f;
      }
      __syncthreads();
    }
    if (wave * 64 < npx) {
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const int r0 = wave * 64 + ks * 32 + 8 * g + qq;
        const int pb = wave * 64 + ks * 32 + 8 * g + 3;  // the lane's first pixel in the image (+3: w0-4 origin, s=0 at -1)
        bf16x8 af[2], bfr[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          const int col = i * 16 + 4 * pp;
          const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Ds + tr32(r0, col)));
          const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Ds + tr32(r0 + 4, col)));
          af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        }
#pragma unroll
        for (int j = 0; j < 2; ++j) {
          const float* src = X + kof[j] + pb * 3;
#pragma unroll
          for (int e = 0; e < 8; ++e) bfr[j][e] = from_f32<bf16>(src[3 * e]);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
      }
    }
    buf ^= 1;
  }
  __syncthreads();  // every DMA has landed (the last unit waited for all) and every read is done
  float* part = reinterpret_cast<float*>(lds);
  const int fk = lane >> 4, frow = lane & 15;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[wave * 1024 + (i * 16 + fk * 4 + r) * 32 + j * 16 + frow] = acc[i][j][r];
  __syncthreads();
  for (int e = tid; e < 1024; e += 256)
    slabs[(size_t)blockIdx.x * 1024 + e] = (part[e] + part[1024 + e]) + (part[2048 + e] + part[3072 + e]);
}

// fp32 weight gradient (fp32 training, main.py:126-132): the same persistent unit walk with
// dz as [pixel][32] fp32 rows (128 B) and 16x16x4 f32 MFMAs.  The reduction axis is the
// pixel: with Mma<float>'s k order a lane group g holds 4 consecutive pixels 4g..4g+3 of a
// 16-pixel fragment, so the dz operand is 4 scalar LDS reads per lane (row = pixel, column =
// channel; no transposed read exists for 32-bit elements) and the image-column operand 4
// scalar reads as in the bf16 kernel.  84 KB of LDS (two 42 KB buffers): one workgroup per CU.
constexpr int FDP = SEG * 8;                // fp32 dz pieces per unit (16 B = 4 channels)
constexpr int FNI = FDP / 64 + WXI;         // DMA instructions per unit (42)
constexpr int FBUF = FDP * 16 + WXI * 1024; // bytes per LDS buffer
constexpr int FG_GRID = 256;                // persistent workgroups (one per CU)

__global__ __launch_bounds__(256) void conv_c3_wgrad_f32_kernel(const float* __restrict__ x, int n, int hv, int h,
                                                                int w, int segs, const float* __restrict__ dz,
                                                                long units, float* __restrict__ slabs) {
  __shared__ __attribute__((aligned(1024))) char lds[2 * FBUF];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15;
  const long G = gridDim.x;
  const int w3 = w * 3;
  (void)n;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int kof[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = 16 * j + li;
    kof[j] = k < 27 ? (k / 9) * XRW + ((k % 9) / 3) * 3 + k % 3 : 0;
  }
  struct Unit {
    int img, oh, w0;
  };
  auto unit = [&](long u) {
    const long row = u / segs;
    return Unit{(int)(row / h), (int)(row % h), (int)(u % segs) * SEG};
  };
  auto issue = [&](const Unit& un, int buf) {
    char* B = lds + buf * FBUF;
    const dma::i32x4 zs = dma::rsrc((uintptr_t)(dz + ((size_t)un.img * h + un.oh) * w * 32));
    const dma::i32x4 xr = dma::rsrc((uintptr_t)(x + (size_t)un.img * hv * w3));
    const long f00 = (long)(un.w0 - 4) * 3;
#pragma unroll
    for (int q = 0; q < (FNI + 3) / 4; ++q) {
      const int T = wave + 4 * q;
      if (T < FDP / 64) {  // dz: LDS row = pixel (8 pieces of 4 channels), natural order
        const int pc = T * 64 + lane, row = pc >> 3;
        const bool ok = un.w0 + row < w;
        dma::lds16(ok ? (unsigned)(((un.w0 + row) * 32 + (pc & 7) * 4) * 4) : dma::OOB, zs, B + T * 1024);
      } else if (T < FNI) {  // image rows oh-1 .. oh+1
        const int t = T - FDP / 64, i = t * 64 + lane;
        const int r = i / XPC, pc = i - (i / XPC) * XPC;
        const int hh = un.oh - 1 + r;
        const long f0 = f00 + pc * 4;
        const bool ok = i < WXP && hh >= 0 && hh < hv && f0 >= 0 && f0 + 4 <= w3;  // (edge piece: patched)
        dma::lds16(ok ? (unsigned)(((long)hh * w3 + f0) * 4) : dma::OOB, xr, B + FDP * 16 + t * 1024);
      }
    }
  };
  const int nis = (FNI - wave + 3) / 4;
  long u = blockIdx.x;
  int buf = 0;
  if (u < units) issue(unit(u), 0);
  for (; u < units; u += G) {
    const Unit un = unit(u);
    const int npx = min(SEG, w - un.w0);
    __syncthreads();
    const bool more = u + G < units;
    if (more) issue(unit(u + G), buf ^ 1);
    dma::wait_vm_dyn(more ? nis : 0);
    __syncthreads();
    const float* D = reinterpret_cast<const float*>(lds + buf * FBUF);
    const float* X = D + FDP * 4;
    if (w3 & 3) {  // the piece straddling the right frame edge: its nv valid floats by guarded loads
      const int nv = w3 & 3, e0 = w3 - nv - (un.w0 - 4) * 3;
      if (e0 < XRW && tid < 3 * 4) {
        const int r = tid >> 2, k = tid & 3, hh = un.oh - 1 + r;
        const bool ok = k < nv && hh >= 0 && hh < hv;
        const_cast<float*>(X)[r * XRW + e0 + k] = ok ? x[((size_t)un.img * hv + hh) * w3 + (w3 - nv) + k] : 0.f;
      }
      __syncthreads();
    }
    if (wave * 64 < npx) {
#pragma unroll
      for (int fr = 0; fr < 4; ++fr) {
        const int p0 = wave * 64 + fr * 16 + 4 * g;  // the lane's first pixel of the fragment
        float a[2][4], b[2][4];
#pragma unroll
        for (int s = 0; s < 4; ++s) {
#pragma unroll
          for (int i = 0; i < 2; ++i) a[i][s] = D[(p0 + s) * 32 + 16 * i + li];
#pragma unroll
          for (int j = 0; j < 2; ++j) b[j][s] = X[kof[j] + (p0 + s + 3) * 3];  // (+3: w0-4 origin, s=0 at -1)
        }
#pragma unroll
        for (int s = 0; s < 4; ++s)
#pragma unroll
          for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i][s], b[j][s], acc[i][j], 0, 0, 0);
      }
    }
    buf ^= 1;
  }
  __syncthreads();
  float* part = reinterpret_cast<float*>(lds);
  const int fk = lane >> 4, frow = lane & 15;
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 4; ++r) part[wave * 1024 + (i * 16 + fk * 4 + r) * 32 + j * 16 + frow] = acc[i][j][r];
  __syncthreads();
  for (int e = tid; e < 1024; e += 256)
    slabs[(size_t)blockIdx.x * 1024 + e] = (part[e] + part[1024 + e]) + (part[2048 + e] + part[3072 + e]);
}

// dw[co][k] (k < 27) = sum over the slabs: one workgroup per output channel, 8
// slab ranges per column summed in order, then folded in a fixed order
__global__ __launch_bounds__(256) void conv_c3_wgrad_fold_kernel(const float* __restrict__ slabs, int nslab,
                                                                 float* __restrict__ dw) {
  __shared__ float red[8][32];
  const int co = blockIdx.x, k = threadIdx.x & 31, part = threadIdx.x >> 5;
  const int per = (nslab + 7) / 8, b0 = part * per, b1 = min(b0 + per, nslab);
  float s = 0.f;
  for (int b = b0; b < b1; ++b) s += slabs[(size_t)b * 1024 + co * 32 + k];
  red[part][k] = s;
  __syncthreads();
  if (threadIdx.x < 27) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 8; ++q) t += red[q][threadIdx.x];
    dw[co * 27 + threadIdx.x] = t;
  }
}


}  // namespace

static long c3_units(int n, int h, int w) { return (long)n * ((h + RPB - 1) / RPB) * ((w + SEG - 1) / SEG); }

extern "C" long cnnitmo_conv_c3_stat_rows(int n, int h, int w) {
  return std::min<long>(c3_units(n, h, w), C3_GRID);
}

extern "C" int cnnitmo_conv_c3_fwd(int dtype, const float* x, int n, int h_valid, int h, int w, const void* wt,
                                   const float* bias, void* out, int out_ld, int out_off, int flags,
                                   const float* aff_scale, const float* aff_shift, float* stat_part, void* stream) {
  CNN_REQUIRE(dtype == CNNITMO_BF16 || dtype == CNNITMO_F32, "conv_c3_fwd: unsupported dtype %d", dtype);
  CNN_REQUIRE(x && wt && out, "conv_c3_fwd: null pointer");
  CNN_REQUIRE(n > 0 && h > 0 && w > 0 && h_valid >= 0 && h_valid <= h, "conv_c3_fwd: bad shape");
  const int al = dtype == CNNITMO_BF16 ? 8 : 4;  // 16-byte aligned pixel rows
  CNN_REQUIRE(out_ld % al == 0 && out_off % al == 0 && out_ld >= out_off + 32, "conv_c3_fwd: output view");
  CNN_REQUIRE(!(flags & CNNITMO_STATS) || stat_part, "conv_c3_fwd: STATS without buffer");
  CNN_REQUIRE(!(flags & CNNITMO_AFFINE) || (aff_scale && aff_shift), "conv_c3_fwd: AFFINE without coefficients");
  C3Fwd2 a;
  a.x = x; a.n = n; a.hv = h_valid; a.h = h; a.w = w;
  a.segs = (w + SEG - 1) / SEG;
  a.rpn = (h + RPB - 1) / RPB;
  a.units = c3_units(n, h, w);
  a.wt = wt; a.bias = bias; a.out = out; a.out_ld = out_ld; a.out_off = out_off;
  a.flags = flags; a.aff_scale = aff_scale; a.aff_shift = aff_shift; a.stats = stat_part;
  CNN_REQUIRE((long)h_valid * w * 3 < (1L << 29), "conv_c3_fwd: frame too large for 32-bit offsets");
  const long blocks = cnnitmo_conv_c3_stat_rows(n, h, w);
  const dim3 grid((unsigned)blocks);
  hipStream_t s = (hipStream_t)stream;
  const bool af = flags & CNNITMO_AFFINE;
  if (dtype == CNNITMO_F32) {
    if (af) hipLaunchKernelGGL((conv_c3_fwd_kernel<float, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_c3_fwd_kernel<float, false>), grid, dim3(256), 0, s, a);
  } else {
    if (af) hipLaunchKernelGGL((conv_c3_fwd_kernel<bf16, true>), grid, dim3(256), 0, s, a);
    else hipLaunchKernelGGL((conv_c3_fwd_kernel<bf16, false>), grid, dim3(256), 0, s, a);
  }
  return cnnitmo_check_launch("conv_c3_fwd");
}

extern "C" size_t cnnitmo_conv_c3_wgrad_workspace_bytes(int n, int h, int w) {
  (void)n; (void)h; (void)w;
  return (size_t)std::max(WG_GRID, FG_GRID) * 1024 * sizeof(float);
}

extern "C" int cnnitmo_conv_c3_wgrad(int dtype, const float* x, int n, int h_valid, int h, int w, const void* dz,
                                     float* dw, void* workspace, size_t ws_bytes, void* stream) {
  CNN_REQUIRE(dtype == CNNITMO_BF16 || dtype == CNNITMO_F32, "conv_c3_wgrad: unsupported dtype %d", dtype);
  CNN_REQUIRE(x && dz && dw && workspace, "conv_c3_wgrad: null pointer");
  CNN_REQUIRE(n > 0 && h > 0 && w > 0 && h_valid >= 0 && h_valid <= h, "conv_c3_wgrad: bad shape");
  CNN_REQUIRE(ws_bytes >= cnnitmo_conv_c3_wgrad_workspace_bytes(n, h, w), "conv_c3_wgrad: workspace too small");
  const int segs = (w + SEG - 1) / SEG;
  const long units = (long)n * h * segs;
  CNN_REQUIRE((long)h_valid * w * 3 < (1L << 29) && (long)w * 64 < (1L << 31), "conv_c3_wgrad: frame too large");
  const int blocks = (int)std::min<long>(units, dtype == CNNITMO_F32 ? FG_GRID : WG_GRID);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == CNNITMO_F32)
    hipLaunchKernelGGL(conv_c3_wgrad_f32_kernel, dim3(blocks), dim3(256), 0, s, x, n, h_valid, h, w, segs,
                       (const float*)dz, units, (float*)workspace);
  else
    hipLaunchKernelGGL(conv_c3_wgrad_kernel, dim3(blocks), dim3(256), 0, s, x, n, h_valid, h, w, segs,
                       (const bf16*)dz, units, (float*)workspace);
  hipLaunchKernelGGL(conv_c3_wgrad_fold_kernel, dim3(32), dim3(256), 0, s, (const float*)workspace, blocks, dw);
  return cnnitmo_check_launch("conv_c3_wgrad");
}
