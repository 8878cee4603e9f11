// Training-data augmentation on the GPU: the reference's paired
// ImageDataGenerator (rescale 1/255, rotation_range 90, horizontal/vertical
// flips, zoom_range 0.2; /root/reference/main.py:71-77), i.e. Keras 2.2.4's
// keras_preprocessing apply_transform + standardize per frame:
//
//   out[r][c] = scale * bilinear_nearest(src, A * (r', c') + t)     (scipy.ndimage
//               .affine_transform, order 1, mode 'nearest': clamp-to-edge)
//   (r', c') = (fv ? h-1-r : r, fh ? w-1-c : c)                     (flip_axis after
//                                                                    the affine map)
//
// A (2x2) and t come from the host (transform_matrix_offset_center of
// rotation @ zoom, in float64 as Keras computes them).  Coordinates and the
// interpolation run in float64 like scipy's; the result is rounded to float32,
// then multiplied by `scale` in float32 (standardize's x *= rescale).
// HBM-bound gather: one thread per output pixel, all channels.
#include "common.h"

namespace {

template <typename T, int C>
__global__ __launch_bounds__(256) void augment_affine_kernel(const T* __restrict__ src, int h, int w,
                                                             const double* __restrict__ mats,
                                                             const int* __restrict__ flips, float scale,
                                                             float* __restrict__ dst, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const long hw = (long)h * w;
  const int img = (int)(i / hw);
  const int rem = (int)(i - (long)img * hw);
  int r = rem / w, c = rem - (rem / w) * w;
  const int fl = flips[img];
  if (fl & 2) r = h - 1 - r;  // flip_vertical (row axis)
  if (fl & 1) c = w - 1 - c;  // flip_horizontal (column axis)
  const double* m = mats + 6 * (long)img;
  const double rin = m[0] * r + m[1] * c + m[2];
  const double cin = m[3] * r + m[4] * c + m[5];
  const double rf = floor(rin), cf = floor(cin);
  const double fr = rin - rf, fc = cin - cf;
  // clamp-to-edge neighbours (mode 'nearest'); coordinates beyond +-2^30 saturate
  const long ri = (long)fmin(fmax(rf, -1073741824.0), 1073741824.0);
  const long ci = (long)fmin(fmax(cf, -1073741824.0), 1073741824.0);
  const int r0 = (int)min(max(ri, 0L), (long)h - 1), r1 = (int)min(max(ri + 1, 0L), (long)h - 1);
  const int c0 = (int)min(max(ci, 0L), (long)w - 1), c1 = (int)min(max(ci + 1, 0L), (long)w - 1);
  const T* s = src + (size_t)img * hw * C;
  const T* p00 = s + ((size_t)r0 * w + c0) * C;
  const T* p01 = s + ((size_t)r0 * w + c1) * C;
  const T* p10 = s + ((size_t)r1 * w + c0) * C;
  const T* p11 = s + ((size_t)r1 * w + c1) * C;
  float* o = dst + (size_t)i * C;
#pragma unroll
  for (int k = 0; k < C; ++k) {
    const double top = (1.0 - fc) * (double)p00[k] + fc * (double)p01[k];
    const double bot = (1.0 - fc) * (double)p10[k] + fc * (double)p11[k];
    const float v = (float)((1.0 - fr) * top + fr * bot);
    o[k] = v * scale;
  }
}

template <typename T>
int launch(const void* src, int n, int h, int w, int c, const double* mats, const int* flips, float scale,
           float* dst, hipStream_t s) {
  const long total = (long)n * h * w;
  const dim3 grid((unsigned)((total + 255) / 256)), block(256);
  if (c == 3)
    hipLaunchKernelGGL((augment_affine_kernel<T, 3>), grid, block, 0, s, (const T*)src, h, w, mats, flips, scale,
                       dst, total);
  else
    hipLaunchKernelGGL((augment_affine_kernel<T, 1>), grid, block, 0, s, (const T*)src, h, w, mats, flips, scale,
                       dst, total);
  return cnnitmo_check_launch("augment_affine");
}

}  // namespace

extern "C" int cnnitmo_augment_affine(int src_u8, const void* src, int n, int h, int w, int c, const double* mats,
                                      const int* flips, float scale, float* dst, void* stream) {
  CNN_REQUIRE(src && mats && flips && dst, "augment_affine: null pointer");
  CNN_REQUIRE(n > 0 && h > 0 && w > 0 && (c == 1 || c == 3), "augment_affine: bad shape %d x %d x %d x %d", n, h,
              w, c);
  CNN_REQUIRE((long)n * h * w < (1L << 40), "augment_affine: too large");
  return src_u8 ? launch<uint8_t>(src, n, h, w, c, mats, flips, scale, dst, (hipStream_t)stream)
                : launch<float>(src, n, h, w, c, mats, flips, scale, dst, (hipStream_t)stream);
}
