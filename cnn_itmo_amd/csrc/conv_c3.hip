// First layer of the U-Net, Conv2D(32, 3, 'same') on the 3-channel SDR input
// (/root/reference/model.py:208), bf16, without an im2col round trip through HBM.
//
// The 3x3x3 patches of an output row segment (256 pixels) are built in LDS from
// the fp32 input rows (fused /255-input cast to bf16 and the zero padding of
// predict.py:59's pad-to-16 rows), so the layer reads 12 B and writes 64 B per
// pixel instead of 12 + 64 (im2col) + 64 + 64 (GEMM):
//
//   conv_c3_fwd_kernel    one workgroup = RPB output rows x 256 pixels; the RPB+2
//                         input rows are staged once; per row: A tile [256 px][32 k]
//                         (k = (r*3+s)*3 + c, 27 used), 8 MFMAs 16x16x32 per wave
//                         against the [32 cout][32 k] weights held in registers,
//                         epilogue bias + ReLU (+ inference BN affine) + BN partial
//                         sums (one row per workgroup), 16-byte stores of the bf16 row.
//   conv_c3_wgrad_kernel  dW[co][k] = sum_p dz[p][co] * col[p][k]: per 256-pixel unit
//                         the dz row and the columns go to LDS as [pixel][32] rows
//                         and are read transposed (ds_read_b64_tr_b16: pixels are
//                         the MFMA reduction axis); the next unit's loads are in
//                         flight under the current one; persistent grid, one fp32
//                         slab per workgroup, fixed-order fold.
//
// HBM-bound: fwd 12 B read + 64 B written per pixel (+ stats), wgrad 12 + 64 B read.
#include "igemm_common.h"

namespace {

constexpr int SEG = 256;  // pixels per row segment (one per thread)
constexpr int RPB = 4;    // output rows per forward workgroup
constexpr int ALD = 40;   // A/C tile row stride in bf16 (80 B)

struct C3Fwd {
  const float* x;
  int n, hv, h, w, segs, rpn;
  const bf16* wt;  // [32 cout][32 k]
  const float* bias;
  bf16* out;
  long out_ld;
  int out_off;
  int flags;
  const float* aff_scale;
  const float* aff_shift;
  float* stats;  // [blocks][2][32]
};

__device__ __forceinline__ void stage_rows(const float* __restrict__ x, int n, int hv, int w, int hfirst, int nrows,
                                           int w0, float* xs) {
  constexpr int PWC = (SEG + 2) * 3;
  for (int i = threadIdx.x; i < nrows * PWC; i += 256) {
    const int r = i / PWC, q = i - r * PWC;
    const int hh = hfirst + r, ww = w0 - 1 + q / 3;
    float v = 0.f;
    if (hh >= 0 && hh < hv && ww >= 0 && ww < w) v = x[(((long)n * hv + hh) * w + ww) * 3 + q % 3];
    xs[r * PWC + q] = v;
  }
}

// the 32 column values (27 taps x channels + 5 zeros) of pixel t, input rows xs[r0 .. r0+2]
__device__ __forceinline__ void patch(const float* xs, int r0, int t, float* v) {
  constexpr int PWC = (SEG + 2) * 3;
#pragma unroll
  for (int k = 0; k < 32; ++k) {
    const int tap = k / 3, c = k - tap * 3;
    v[k] = k < 27 ? xs[(r0 + tap / 3) * PWC + (t + tap % 3) * 3 + c] : 0.f;
  }
}

__global__ __launch_bounds__(256) void conv_c3_fwd_kernel(const C3Fwd a) {
  __shared__ float xs[(RPB + 2) * (SEG + 2) * 3];
  __shared__ __attribute__((aligned(16))) bf16 at[SEG * ALD];
  __shared__ float red[4][2][32];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int seg = blockIdx.x % a.segs;
  const long rb = blockIdx.x / a.segs;
  const int n = (int)(rb / a.rpn), h0 = (int)(rb % a.rpn) * RPB;
  const int w0 = seg * SEG, npx = min(SEG, a.w - w0);
  const int nrow = min(RPB, a.h - h0);
  stage_rows(a.x, n, a.hv, a.w, h0 - 1, nrow + 2, w0, xs);
  const int frow = lane & 15, fk = lane >> 4;
  uint4 bw[2];
  float bj[2], sj[2], hj[2];
  const bool relu = a.flags & CNNITMO_RELU, aff = a.flags & CNNITMO_AFFINE, stats = a.flags & CNNITMO_STATS;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int co = j * 16 + frow;
    bw[j] = *reinterpret_cast<const uint4*>(a.wt + co * 32 + fk * 8);
    bj[j] = a.bias ? a.bias[co] : 0.f;
    sj[j] = aff ? a.aff_scale[co] : 1.f;
    hj[j] = aff ? a.aff_shift[co] : 0.f;
  }
  float s1[2] = {0.f, 0.f}, s2[2] = {0.f, 0.f};
  __syncthreads();
  for (int rr = 0; rr < nrow; ++rr) {
    {
      float v[32];
      patch(xs, rr, tid, v);
#pragma unroll
      for (int j = 0; j < 32; j += 8) Pack16<bf16>::store(at + tid * ALD + j, v + j);
    }
    __syncthreads();
    f32x4 acc[4][2];
#pragma unroll
    for (int f = 0; f < 4; ++f) {
      const uint4 af = *reinterpret_cast<const uint4*>(at + (wave * 64 + f * 16 + frow) * ALD + fk * 8);
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        acc[f][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        Mma<bf16>::run(acc[f][j], af, bw[j]);
      }
    }
    __syncthreads();  // the A tile is consumed: it becomes the C tile
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int px = wave * 64 + f * 16 + fk * 4 + r;
          float v = acc[f][j][r] + bj[j];
          if (relu) v = fmaxf(v, 0.f);
          if (aff) v = v * sj[j] + hj[j];
          const float vs = px < npx ? v : 0.f;
          s1[j] += vs;
          s2[j] += vs * vs;
          at[px * ALD + j * 16 + frow] = from_f32<bf16>(v);
        }
    __syncthreads();
    const long prow = ((long)n * a.h + h0 + rr) * a.w + w0;
    for (int i = tid; i < npx * 4; i += 256) {
      const int px = i >> 2, pc = i & 3;
      *reinterpret_cast<uint4*>(a.out + (prow + px) * a.out_ld + a.out_off + pc * 8) =
          *reinterpret_cast<const uint4*>(at + px * ALD + pc * 8);
    }
    __syncthreads();
  }
  if (stats) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      s1[j] += __shfl_xor(s1[j], 16, 64);
      s1[j] += __shfl_xor(s1[j], 32, 64);
      s2[j] += __shfl_xor(s2[j], 16, 64);
      s2[j] += __shfl_xor(s2[j], 32, 64);
      if (lane < 16) {
        red[wave][0][j * 16 + lane] = s1[j];
        red[wave][1][j * 16 + lane] = s2[j];
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

// One unit = one 256-pixel row segment.  The next unit's input rows and dz row are
// loaded into registers while the current one is built and multiplied (the loads
// are the whole cost of this layer; the MFMA work per unit is 16 instructions).
__global__ __launch_bounds__(256) void conv_c3_wgrad_kernel(const float* __restrict__ x, int n, int hv, int h,
                                                            int w, int segs, const bf16* __restrict__ dz,
                                                            long units, long per_block, float* __restrict__ slabs) {
  constexpr int PWC = (SEG + 2) * 3, XN = (3 * PWC + 255) / 256;
  __shared__ float xs[3 * PWC];
  __shared__ __attribute__((aligned(16))) char Ds[SEG * 64];
  __shared__ __attribute__((aligned(16))) char Cs[SEG * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g = lane >> 4, li = lane & 15, qq = li >> 2, pp = li & 3;
  (void)n;
  f32x4 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const long u0 = (long)blockIdx.x * per_block, u1 = min(u0 + per_block, units);
  float xr[XN];
  uint4 dr[4];
  auto load = [&](long u) {
    const int seg = (int)(u % segs);
    const long row = u / segs;  // img * h + oh
    const int img = (int)(row / h), oh = (int)(row % h);
    const int w0 = seg * SEG, npx = min(SEG, w - w0);
#pragma unroll
    for (int q = 0; q < XN; ++q) {
      const int i = tid + q * 256;
      const int r = i / PWC, c = i - r * PWC;
      const int hh = oh - 1 + r, ww = w0 - 1 + c / 3;
      xr[q] = (i < 3 * PWC && hh >= 0 && hh < hv && ww >= 0 && ww < w)
                  ? x[(((long)img * hv + hh) * w + ww) * 3 + c % 3] : 0.f;
    }
    if (tid < npx) {
      const uint4* src = reinterpret_cast<const uint4*>(dz + ((size_t)row * w + w0 + tid) * 32);
#pragma unroll
      for (int q = 0; q < 4; ++q) dr[q] = src[q];
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) dr[q] = uint4{0u, 0u, 0u, 0u};
    }
  };
  if (u0 < u1) load(u0);
  for (long u = u0; u < u1; ++u) {
    const int npx = min(SEG, w - (int)(u % segs) * SEG);
#pragma unroll
    for (int q = 0; q < XN; ++q)
      if (tid + q * 256 < 3 * PWC) xs[tid + q * 256] = xr[q];
#pragma unroll
    for (int q = 0; q < 4; ++q) *reinterpret_cast<uint4*>(Ds + tr32(tid, q * 8)) = dr[q];
    if (u + 1 < u1) load(u + 1);  // in flight under this unit's work
    __syncthreads();
    {
      float v[32];
      patch(xs, 0, tid, v);
      if (tid >= npx) {
#pragma unroll
        for (int k = 0; k < 32; ++k) v[k] = 0.f;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) Pack16<bf16>::store(reinterpret_cast<bf16*>(Cs + tr32(tid, q * 8)), v + q * 8);
    }
    __syncthreads();
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int r0 = wave * 64 + ks * 32 + 8 * g + qq;
      bf16x8 af[2], bfr[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int col = i * 16 + 4 * pp;
        const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Ds + tr32(r0, col)));
        const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Ds + tr32(r0 + 4, col)));
        af[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
        const s16x4 lo2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Cs + tr32(r0, col)));
        const s16x4 hi2 = __builtin_amdgcn_ds_read_tr16_b64_v4i16(LDS_PTR(s16x4, Cs + tr32(r0 + 4, col)));
        bfr[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo2, hi2, 0, 1, 2, 3, 4, 5, 6, 7));
      }
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j)
          acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    __syncthreads();
  }
  // per-wave 32x32 partials -> LDS (reusing Ds/Cs as fp32 [4][32][32]) -> slab
  float* part = reinterpret_cast<float*>(Ds);
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

constexpr int WG_BLOCKS = 1024;

}  // namespace

extern "C" long cnnitmo_conv_c3_stat_rows(int n, int h, int w) {
  return (long)n * ((h + RPB - 1) / RPB) * ((w + SEG - 1) / SEG);
}

extern "C" int cnnitmo_conv_c3_fwd(const float* x, int n, int h_valid, int h, int w, const void* wt,
                                   const float* bias, void* out, int out_ld, int out_off, int flags,
                                   const float* aff_scale, const float* aff_shift, float* stat_part, void* stream) {
  CNN_REQUIRE(x && wt && out, "conv_c3_fwd: null pointer");
  CNN_REQUIRE(n > 0 && h > 0 && w > 0 && h_valid >= 0 && h_valid <= h, "conv_c3_fwd: bad shape");
  CNN_REQUIRE(out_ld % 8 == 0 && out_off % 8 == 0 && out_ld >= out_off + 32, "conv_c3_fwd: output view");
  CNN_REQUIRE(!(flags & CNNITMO_STATS) || stat_part, "conv_c3_fwd: STATS without buffer");
  CNN_REQUIRE(!(flags & CNNITMO_AFFINE) || (aff_scale && aff_shift), "conv_c3_fwd: AFFINE without coefficients");
  C3Fwd a;
  a.x = x; a.n = n; a.hv = h_valid; a.h = h; a.w = w;
  a.segs = (w + SEG - 1) / SEG;
  a.rpn = (h + RPB - 1) / RPB;
  a.wt = (const bf16*)wt; a.bias = bias; a.out = (bf16*)out; a.out_ld = out_ld; a.out_off = out_off;
  a.flags = flags; a.aff_scale = aff_scale; a.aff_shift = aff_shift; a.stats = stat_part;
  const long blocks = cnnitmo_conv_c3_stat_rows(n, h, w);
  CNN_REQUIRE(blocks < (1L << 31), "conv_c3_fwd: too large");
  hipLaunchKernelGGL(conv_c3_fwd_kernel, dim3((unsigned)blocks), dim3(256), 0, (hipStream_t)stream, a);
  return cnnitmo_check_launch("conv_c3_fwd");
}

extern "C" size_t cnnitmo_conv_c3_wgrad_workspace_bytes(int n, int h, int w) {
  (void)n; (void)h; (void)w;
  return (size_t)WG_BLOCKS * 1024 * sizeof(float);
}

extern "C" int cnnitmo_conv_c3_wgrad(const float* x, int n, int h_valid, int h, int w, const void* dz, float* dw,
                                     void* workspace, size_t ws_bytes, void* stream) {
  CNN_REQUIRE(x && dz && dw && workspace, "conv_c3_wgrad: null pointer");
  CNN_REQUIRE(n > 0 && h > 0 && w > 0 && h_valid >= 0 && h_valid <= h, "conv_c3_wgrad: bad shape");
  CNN_REQUIRE(ws_bytes >= cnnitmo_conv_c3_wgrad_workspace_bytes(n, h, w), "conv_c3_wgrad: workspace too small");
  const int segs = (w + SEG - 1) / SEG;
  const long units = (long)n * h * segs;
  const long per = (units + WG_BLOCKS - 1) / WG_BLOCKS;
  const int blocks = (int)((units + per - 1) / per);
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(conv_c3_wgrad_kernel, dim3(blocks), dim3(256), 0, s, x, n, h_valid, h, w, segs,
                     (const bf16*)dz, units, per, (float*)workspace);
  hipLaunchKernelGGL(conv_c3_wgrad_fold_kernel, dim3(32), dim3(256), 0, s, (const float*)workspace, blocks, dw);
  return cnnitmo_check_launch("conv_c3_wgrad");
}
