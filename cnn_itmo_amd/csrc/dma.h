// LDS-DMA and raw-buffer helpers shared by the LDS-ring kernels (conv_halo,
// wgrad_halo, wgrad_tconv, tconv_stream).  gfx950 only.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#pragma clang diagnostic ignored "-Winline-asm"

namespace dma {

typedef int i32x4 __attribute__((ext_vector_type(4)));
typedef int i32x2 __attribute__((ext_vector_type(2)));

// voffset at or beyond num_records: a load lands zeros, a store is dropped
constexpr unsigned OOB = 0x80000000u;

// LDS address of a generic pointer into LDS: the low 32 bits of a flat address in the shared
// aperture are the LDS offset.  (The address-space cast also maps a null pointer, a compare and
// two selects per call: about five scalar instructions per LDS-DMA piece.)
__device__ __forceinline__ unsigned lds_addr(const void* p) { return (unsigned)(uintptr_t)p; }

// raw buffer descriptor over [base, base + 2 GB) from a wave-uniform address
__device__ __forceinline__ i32x4 rsrc(uintptr_t base) {
  i32x4 r;
  r.x = __builtin_amdgcn_readfirstlane((int)(unsigned)base);
  r.y = __builtin_amdgcn_readfirstlane((int)(unsigned)(base >> 32)) & 0xFFFF;
  r.z = 0x7FFFFFF0;
  r.w = 0x00020000;
  return r;
}

// the same as a __amdgpu_buffer_rsrc_t (for the raw_buffer_load/store builtins)
__device__ __forceinline__ __amdgpu_buffer_rsrc_t brsrc(const void* p) {
  const uintptr_t a = (uintptr_t)p;
  const uintptr_t u = (uintptr_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)a) |
                      ((uintptr_t)(unsigned)__builtin_amdgcn_readfirstlane((int)(unsigned)(a >> 32)) << 32);
  return __builtin_amdgcn_make_buffer_rsrc((void*)u, (short)0, 0x7FFFFFF0, 0x00020000);
}

// one 16-byte piece per lane -> the wave's 1 KiB LDS image at `lds` (LDS-DMA,
// lane-linear destination)
__device__ __forceinline__ void lds16(unsigned voff, i32x4 rs, const char* lds) {
  const unsigned a = __builtin_amdgcn_readfirstlane(lds_addr(lds));
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds" ::"v"(voff), "s"(rs),
               "s"(a) : "memory");
}

// the same with a wave-uniform byte offset added in the SGPR slot (not range-checked:
// voff alone decides whether the piece is in range)
// (LDS destination as a 32-bit LDS address: no generic-pointer conversion per piece)
__device__ __forceinline__ void lds16s(unsigned voff, i32x4 rs, unsigned soff, unsigned lds) {
  const unsigned a = __builtin_amdgcn_readfirstlane(lds);
  const unsigned so = __builtin_amdgcn_readfirstlane(soff);
  asm volatile("s_mov_b32 m0, %3\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %2 offen lds" ::"v"(voff), "s"(rs),
               "s"(so), "s"(a) : "memory");
}

template <int N> __device__ __forceinline__ void wait_vm() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}
// Wait until at most n vector-memory operations are outstanding, for a call site whose n is
// A or 0 (anything else waits for A if n >= A, for all otherwise: never less than asked).  Two
// uniform branches instead of wait_vm_dyn's 48-way switch, which the structurizer turns into
// a chain of flag tests (tens of scalar instructions per wait).
template <int A> __device__ __forceinline__ void wait_vm_ge(int n) {
  if (n >= A) wait_vm<A>();
  else wait_vm<0>();
}

// s_waitcnt takes an immediate: dispatch a wave-uniform count (0..47; larger waits for all)
__device__ __forceinline__ void wait_vm_dyn(int n) {
  switch (n) {
#define W1(k) case k: wait_vm<k>(); break;
    W1(0) W1(1) W1(2) W1(3) W1(4) W1(5) W1(6) W1(7) W1(8) W1(9) W1(10) W1(11) W1(12) W1(13) W1(14) W1(15)
    W1(16) W1(17) W1(18) W1(19) W1(20) W1(21) W1(22) W1(23) W1(24) W1(25) W1(26) W1(27) W1(28) W1(29)
    W1(30) W1(31) W1(32) W1(33) W1(34) W1(35) W1(36) W1(37) W1(38) W1(39) W1(40) W1(41) W1(42) W1(43)
    W1(44) W1(45) W1(46) W1(47)
#undef W1
    default: wait_vm<0>(); break;
  }
}

// Exact wait for a count that is usually small: counts 0..3 go through a short chain of uniform
// branches, others through wait_vm_dyn.
__device__ __forceinline__ void wait_vm_small(int n) {
  if (n <= 0) wait_vm<0>();
  else if (n == 1) wait_vm<1>();
  else if (n == 2) wait_vm<2>();
  else if (n == 3) wait_vm<3>();
  else wait_vm_dyn(n);
}

}  // namespace dma
