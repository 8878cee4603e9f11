// Dataset generation and HDR reconstruction maps of the reference's MATLAB
// scripts, in float64 like MATLAB's doubles:
//
//   Reinhard.m:10-24        Y = RGB2Lum(hdr); G = exp(sum(log(max(Y, realmin))) * (1/(H*W)))
//                           X = (0.18/G) * Y; L = X/(1+X); sdr_c = hdr_c * (L / Y)
//   virtual_camera.m:10-31  X = (0.18*2^v/G) * Y; X = min(1, (1+n)*(X^y/(n+X^y)))
//                           sdr_c = hdr_c * (X / Y)
//   inverse_Reinhard.m:1-23 In = (u8/255)^2.2; I = RGB2Lum(In); X = I/(I-1)
//                           G_X = exp(sum(log(max(X, realmin))) * (1/(H*W)))
//                           G_E = exp(P*log(G_X)/PB1 - PB2*log(a)/PB1)  (PB1/PB2: #I==0 / #I~=0)
//                           E = G_E*X/a; E(isnan) = realmin; E(E >= 2^32) = 2^32
//                           hdr_c = In_c * (E / I)
//   (exact inverse)         for a linear SDR image and the HDR log-average g:
//                           X = I/(1-I); E = g*X/a; hdr_c = sdr_c * (E / I)
//
// RGB2Lum is not part of the reference: the luminance weights are an argument
// (Rec. 709 by default on the host).  IEEE double semantics reproduce MATLAB's
// for 0/0, x/0, log(0) and min(1, NaN) = 1 (fmin).  imwrite's double -> uint8
// (uint8(255*x): round half away from zero, saturate, NaN -> 0) is available as
// the u8 output of the forward maps.  Sums are two-level and deterministic
// (fixed block partition, fixed-order final fold); MATLAB's are sequential,
// which differs only in the last bits.
//
// HBM-bound: 12 B read + 12 B (fp32) / 3 B (u8) written per pixel per map; the
// statistics pass reads 12 B (fp32) or 3 B (u8) per pixel.
#include "common.h"

// no FMA contraction: the products and sums round like MATLAB's (and numpy's) doubles
#pragma clang fp contract(off)

namespace {

constexpr int TB = 256;  // threads per block
constexpr int BLK_PER_IMG = 256;  // blocks per image in the statistics pass
constexpr double REALMIN = 2.2250738585072014e-308;

struct Lum {
  double r, g, b;
};

__device__ __forceinline__ double lum(const Lum& c, double R, double G, double B) { return c.r * R + c.g * G + c.b * B; }

__device__ __forceinline__ double decode_sdr(uint8_t v) { return pow((double)v / 255.0, 2.2); }

// mode 0: log(max(Y, realmin)) of an fp32 HDR image (Reinhard / virtual camera)
// mode 1: log(max(X, realmin)), X = I/(I-1) of a uint8 SDR image (inverse_Reinhard.m as written)
// stats per image: [sum of logs, count of zero luminance]
__global__ __launch_bounds__(TB) void stats_partial_kernel(int mode, const void* __restrict__ img, long hw, Lum lc,
                                                           double* __restrict__ part) {
  const int im = blockIdx.y;
  double s = 0.0, z = 0.0;
  for (long p = (long)blockIdx.x * TB + threadIdx.x; p < hw; p += (long)BLK_PER_IMG * TB) {
    double Y;
    if (mode == 0) {
      const float* q = (const float*)img + ((long)im * hw + p) * 3;
      Y = lum(lc, q[0], q[1], q[2]);
      s += log(fmax(Y, REALMIN));
    } else {
      const uint8_t* q = (const uint8_t*)img + ((long)im * hw + p) * 3;
      Y = lum(lc, decode_sdr(q[0]), decode_sdr(q[1]), decode_sdr(q[2]));
      const double X = Y / (Y - 1.0);
      s += log(fmax(X, REALMIN));
    }
    z += Y == 0.0 ? 1.0 : 0.0;
  }
  __shared__ double sh[2][TB];
  sh[0][threadIdx.x] = s;
  sh[1][threadIdx.x] = z;
  __syncthreads();
  for (int o = TB / 2; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      sh[0][threadIdx.x] += sh[0][threadIdx.x + o];
      sh[1][threadIdx.x] += sh[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    double* d = part + ((long)im * BLK_PER_IMG + blockIdx.x) * 2;
    d[0] = sh[0][0];
    d[1] = sh[1][0];
  }
}

__global__ void stats_final_kernel(const double* __restrict__ part, int n, double* __restrict__ stats) {
  const int im = blockIdx.x * blockDim.x + threadIdx.x;
  if (im >= n) return;
  double s = 0.0, z = 0.0;
  for (int b = 0; b < BLK_PER_IMG; ++b) {
    s += part[((long)im * BLK_PER_IMG + b) * 2];
    z += part[((long)im * BLK_PER_IMG + b) * 2 + 1];
  }
  stats[2 * im] = s;
  stats[2 * im + 1] = z;
}

// MATLAB uint8(255*x): round half away from zero, saturate, NaN -> 0
__device__ __forceinline__ uint8_t im2uint8(double x) {
  const double v = 255.0 * x;
  if (!(v > 0.0)) return 0;  // also NaN
  if (v >= 255.0) return 255;
  return (uint8_t)floor(v + 0.5);
}

// curve 0: Reinhard; 1: virtual camera.  params per image: [key*2^v, n, y]
__global__ __launch_bounds__(TB) void tonemap_kernel(int curve, const float* __restrict__ hdr, int n, long hw,
                                                     Lum lc, const double* __restrict__ params,
                                                     const double* __restrict__ stats, int out_u8,
                                                     void* __restrict__ out) {
  const long i = (long)blockIdx.x * TB + threadIdx.x;
  if (i >= (long)n * hw) return;
  const int im = (int)(i / hw);
  const double G = exp(stats[2 * im] * (1.0 / (double)hw));
  const double dt = params[3 * im] / G;
  const float* q = hdr + i * 3;
  const double R = q[0], Gc = q[1], B = q[2];
  const double Y = lum(lc, R, Gc, B);
  double X = dt * Y, L;
  if (curve == 0) {
    L = X / (1.0 + X);
  } else {
    const double cn = params[3 * im + 1], cy = params[3 * im + 2];
    const double Xy = pow(X, cy);
    L = fmin(1.0, (1.0 + cn) * (Xy / (cn + Xy)));
  }
  const double f = L / Y;
  const double o0 = R * f, o1 = Gc * f, o2 = B * f;
  if (out_u8) {
    uint8_t* o = (uint8_t*)out + i * 3;
    o[0] = im2uint8(o0);
    o[1] = im2uint8(o1);
    o[2] = im2uint8(o2);
  } else {
    float* o = (float*)out + i * 3;
    o[0] = (float)o0;
    o[1] = (float)o1;
    o[2] = (float)o2;
  }
}

// mode 1: inverse_Reinhard.m as written (uint8 SDR, 2.2 decode, X = I/(I-1), G_E from the stats)
// mode 2: the exact inverse of Reinhard.m for a known log-average g: linear fp32 SDR,
//         X = I/(1-I), E = g*X/a (same clamps)
__global__ __launch_bounds__(TB) void inverse_kernel(int mode, const void* __restrict__ sdr, int n, long hw,
                                                     Lum lc, const double* __restrict__ stats, double a, double g,
                                                     float* __restrict__ out) {
  const long i = (long)blockIdx.x * TB + threadIdx.x;
  if (i >= (long)n * hw) return;
  const int im = (int)(i / hw);
  double R, Gc, B, GE;
  if (mode == 1) {
    const double GX = exp(stats[2 * im] * (1.0 / (double)hw));
    const double P = (double)hw, PB1 = stats[2 * im + 1], PB2 = P - PB1;
    GE = exp(P * log(GX) / PB1 - PB2 * log(a) / PB1);
    const uint8_t* q = (const uint8_t*)sdr + i * 3;
    R = decode_sdr(q[0]);
    Gc = decode_sdr(q[1]);
    B = decode_sdr(q[2]);
  } else {
    GE = g;
    const float* q = (const float*)sdr + i * 3;
    R = q[0];
    Gc = q[1];
    B = q[2];
  }
  const double I = lum(lc, R, Gc, B);
  const double X = mode == 1 ? I / (I - 1.0) : I / (1.0 - I);
  double E = GE * X / a;
  if (E != E) E = REALMIN;
  if (E >= 4294967296.0) E = 4294967296.0;
  const double f = E / I;
  float* o = out + i * 3;
  o[0] = (float)(R * f);
  o[1] = (float)(Gc * f);
  o[2] = (float)(B * f);
}

Lum lum_of(const double* c) { return c ? Lum{c[0], c[1], c[2]} : Lum{0.2126, 0.7152, 0.0722}; }

}  // namespace

extern "C" size_t cnnitmo_tonemap_workspace_bytes(int n) { return (size_t)n * BLK_PER_IMG * 2 * sizeof(double); }

extern "C" int cnnitmo_tonemap_stats(int mode, const void* img, int n, int h, int w, const double* lum_coef,
                                     double* stats, void* workspace, size_t ws_bytes, void* stream) {
  CNN_REQUIRE(mode == 0 || mode == 1, "tonemap_stats: mode %d", mode);
  CNN_REQUIRE(img && stats && workspace, "tonemap_stats: null pointer");
  CNN_REQUIRE(n > 0 && n <= 65535 && h > 0 && w > 0, "tonemap_stats: bad shape");
  CNN_REQUIRE(ws_bytes >= cnnitmo_tonemap_workspace_bytes(n), "tonemap_stats: workspace too small");
  hipStream_t s = (hipStream_t)stream;
  const long hw = (long)h * w;
  hipLaunchKernelGGL(stats_partial_kernel, dim3(BLK_PER_IMG, n), dim3(TB), 0, s, mode, img, hw, lum_of(lum_coef),
                     (double*)workspace);
  hipLaunchKernelGGL(stats_final_kernel, dim3((n + 63) / 64), dim3(64), 0, s, (const double*)workspace, n, stats);
  return cnnitmo_check_launch("tonemap_stats");
}

extern "C" int cnnitmo_tonemap_apply(int curve, const float* hdr, int n, int h, int w, const double* lum_coef,
                                     const double* params, const double* stats, int out_u8, void* out,
                                     void* stream) {
  CNN_REQUIRE(curve == 0 || curve == 1, "tonemap_apply: curve %d", curve);
  CNN_REQUIRE(hdr && params && stats && out, "tonemap_apply: null pointer");
  CNN_REQUIRE(n > 0 && h > 0 && w > 0, "tonemap_apply: bad shape");
  const long hw = (long)h * w, tot = (long)n * hw;
  hipLaunchKernelGGL(tonemap_kernel, dim3((unsigned)((tot + TB - 1) / TB)), dim3(TB), 0, (hipStream_t)stream, curve,
                     hdr, n, hw, lum_of(lum_coef), params, stats, out_u8, out);
  return cnnitmo_check_launch("tonemap_apply");
}

extern "C" int cnnitmo_inverse_reinhard_apply(int mode, const void* sdr, int n, int h, int w,
                                              const double* lum_coef, const double* stats, double a, double g,
                                              float* out, void* stream) {
  CNN_REQUIRE(mode == 1 || mode == 2, "inverse_reinhard_apply: mode %d", mode);
  CNN_REQUIRE(sdr && out && (mode == 2 || stats), "inverse_reinhard_apply: null pointer");
  CNN_REQUIRE(n > 0 && h > 0 && w > 0, "inverse_reinhard_apply: bad shape");
  const long hw = (long)h * w, tot = (long)n * hw;
  hipLaunchKernelGGL(inverse_kernel, dim3((unsigned)((tot + TB - 1) / TB)), dim3(TB), 0, (hipStream_t)stream, mode,
                     sdr, n, hw, lum_of(lum_coef), stats, a, g, out);
  return cnnitmo_check_launch("inverse_reinhard_apply");
}
