// HBM streaming ceilings on this box (tools/hbm_probe.py drives it through ctypes):
// what a plain copy, a pure read and the BN-apply access shape (two 16-byte reads and
// one 16-byte write per lane) reach with U independent 16-byte vectors per lane per
// iteration, and with the next iteration's loads issued before this one's stores.
// Not part of the product; built by tools/hbm_probe.py into /tmp.
#include <hip/hip_runtime.h>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// out[i] = in[i], U vectors per lane per iteration, grid-stride over blocks of U*256 vectors
template <int U>
__global__ __launch_bounds__(256) void copy_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, long n) {
  const long step = (long)gridDim.x * 256 * U;
  for (long b = (long)blockIdx.x * 256 * U + threadIdx.x; b < n; b += step) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = b + u * 256 < n ? in[b + u * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + u * 256 < n) out[b + u * 256] = v[u];
  }
}

// copy with cache-policy variants (MODE 0: nt load + nt store, 1: nt store, 2: nt load,
// 3: plain load + sc1 store (write-through, the line is dropped from L2))
template <int U, int MODE>
__global__ __launch_bounds__(256) void copyp_kernel(const u32x4* __restrict__ in, u32x4* __restrict__ out, long n) {
  const long step = (long)gridDim.x * 256 * U;
  for (long b = (long)blockIdx.x * 256 * U + threadIdx.x; b < n; b += step) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = b + u * 256;
      if (MODE == 0 || MODE == 2) v[u] = i < n ? __builtin_nontemporal_load(in + i) : u32x4{0, 0, 0, 0};
      else v[u] = i < n ? in[i] : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = b + u * 256;
      if (i >= n) continue;
      if (MODE == 0 || MODE == 1) __builtin_nontemporal_store(v[u], out + i);
      else if (MODE == 3) asm volatile("global_store_dwordx4 %0, %1, off sc1" ::"v"(out + i), "v"(v[u]) : "memory");
      else out[i] = v[u];
    }
  }
}

// sum of everything (pure read)
template <int U>
__global__ __launch_bounds__(256) void read_kernel(const u32x4* __restrict__ in, long n, unsigned* sink) {
  const long step = (long)gridDim.x * 256 * U;
  unsigned acc = 0;
  for (long b = (long)blockIdx.x * 256 * U + threadIdx.x; b < n; b += step) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = b + u * 256 < n ? in[b + u * 256] : u32x4{0, 0, 0, 0};
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

// partial-line read: 64 useful bytes (4 lanes x 16 B) per "pixel" of PS 16-byte vectors
// (PS = 4: contiguous; 8: half of each 128-B line; 12: the level-1 concat's 64 of 192 B)
template <int U>
__global__ __launch_bounds__(256) void part_kernel(const u32x4* __restrict__ in, long n, int ps, unsigned* sink) {
  const long step = (long)gridDim.x * 256 * U;
  unsigned acc = 0;
  for (long b = (long)blockIdx.x * 256 * U + threadIdx.x; b < n; b += step) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long i = b + u * 256;
      v[u] = i < n ? in[(i >> 2) * ps + (i & 3)] : u32x4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
  }
  if (acc == 0x12345678u) sink[threadIdx.x] = acc;
}

// apply shape: out = f(a, b), U vectors of each per lane per iteration; PF: the next
// iteration's loads are issued before this iteration's stores
template <int U, bool PF>
__global__ __launch_bounds__(256) void apply_kernel(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                                    u32x4* __restrict__ out, long n) {
  const long step = (long)gridDim.x * 256 * U;
  long i = (long)blockIdx.x * 256 * U + threadIdx.x;
  u32x4 va[U], vb[U];
  auto ld = [&](long j) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const bool ok = j + u * 256 < n;
      va[u] = ok ? a[j + u * 256] : u32x4{0, 0, 0, 0};
      vb[u] = ok ? b[j + u * 256] : u32x4{0, 0, 0, 0};
    }
  };
  if (PF) ld(i);
  for (; i < n; i += step) {
    if (!PF) ld(i);
    u32x4 r[U];
#pragma unroll
    for (int u = 0; u < U; ++u) r[u] = va[u] + vb[u];
    if (PF) ld(i + step);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i + u * 256 < n) out[i + u * 256] = r[u];
  }
}

extern "C" int hbm_probe(int kind, int u, int pf, const void* a, const void* b, void* out, long nvec, int grid,
                         void* stream) {
  hipStream_t s = (hipStream_t)stream;
  const u32x4* A = (const u32x4*)a;
  const u32x4* B = (const u32x4*)b;
  u32x4* O = (u32x4*)out;
#define DISP(K, ...)                                                            \
  switch (u) {                                                                  \
    case 1: hipLaunchKernelGGL((K<1 __VA_ARGS__>), dim3(grid), dim3(256), 0, s, ARGS); break; \
    case 2: hipLaunchKernelGGL((K<2 __VA_ARGS__>), dim3(grid), dim3(256), 0, s, ARGS); break; \
    case 4: hipLaunchKernelGGL((K<4 __VA_ARGS__>), dim3(grid), dim3(256), 0, s, ARGS); break; \
    case 8: hipLaunchKernelGGL((K<8 __VA_ARGS__>), dim3(grid), dim3(256), 0, s, ARGS); break; \
    default: return -1;                                                         \
  }
  if (kind == 0) {
#define ARGS A, O, nvec
    DISP(copy_kernel)
#undef ARGS
  } else if (kind >= 16 && kind < 20) {
#define ARGS A, O, nvec
    if (kind == 16) { DISP(copyp_kernel, , 0) }
    else if (kind == 17) { DISP(copyp_kernel, , 1) }
    else if (kind == 18) { DISP(copyp_kernel, , 2) }
    else { DISP(copyp_kernel, , 3) }
#undef ARGS
  } else if (kind == 1) {
#define ARGS A, nvec, (unsigned*)O
    DISP(read_kernel)
#undef ARGS
  } else if (kind >= 4 && kind < 16) {  // part_kernel, ps = kind
#define ARGS A, nvec, kind, (unsigned*)O
    DISP(part_kernel)
#undef ARGS
  } else {
#define ARGS A, B, O, nvec
    if (pf) {
      DISP(apply_kernel, , true)
    } else {
      DISP(apply_kernel, , false)
    }
#undef ARGS
  }
#undef DISP
  return hipGetLastError() == hipSuccess ? 0 : -2;
}
