// Shared declarations of the forward-family implicit-GEMM kernels.
#pragma once
#include "common.h"

struct FwdArgs {
  const void* a;
  long a_ld;
  int a_off;
  int nimg, hs, ws;  // source grid
  int ho, wo;        // iteration grid (GEMM rows are its pixels)
  int scale;         // source pixel = (h*scale + dy[t], w*scale + dx[t])
  int ntaps;
  int dyc, dxc;  // tap t offset = ((code >> 2t) & 3) - 1 (2-bit fields, no dynamic indexing)
  int cin;  // channels per tap
  const void* b;
  int N;
  long M;
  const float* bias;
  void* out;
  long out_ld;
  int out_off;
  int scatter;  // tconv 2x2 s2 scatter: column n = tap*cout + co
  int cout;
  int flags;
  const float* aff_scale;
  const float* aff_shift;
  float* stats;  // [mblocks][2][N]
  int mblocks, nblocks;
  const float* border;  // folded-BN zero-padding correction [cout][8] (conv3x3 fwd), or null
  // conv3x3 dgrad with the producer's BN backward fused (halo kernel only): output
  // columns [bnb_c0, bnb_c1) become dz = [r>0]*(a*g - b*r + e) -> bnb_out [M][c1-c0],
  // with partial sums of dz -> stats [rows][bnb_par ? 4 : 1][c1-c0]
  int bnb_c0, bnb_c1, bnb_par;
  const float* bnb_coef;  // [3][c1-c0]
  const void* bnb_r;
  long bnb_r_ld;
  int bnb_r_off;
  void* bnb_out;
  // two-source input (a concatenate consumed without a concat buffer; halo kernel only):
  // channels [0, cin1) come from a (a_ld, a_off), channels [cin1, cin) from a2 (channel
  // c - cin1 at a2_ld, a2_off).  cin1 = 0: a single source.
  const void* a2;
  long a2_ld;
  int a2_off;
  int cin1;
  // the output's 2x2 MaxPooling2D fused into the forward epilogue (halo kernel, EPI 1):
  // pooled values [n][ho/2][wo/2] x pool_ld, window index bytes (same layout), per-channel
  // mode sign(pool_sign[c]) (null: max)
  void* pool_out;
  long pool_ld;
  unsigned char* pool_idx;
  const float* pool_sign;
  // the sigmoid head fused into the forward epilogue (halo kernel, EPI 3; inference): yhat
  // [n][head_hv][wo][3] fp32 = sigmoid(y . head_w[3][N] + head_b), y (the conv's epilogue
  // output) never stored
  const float* head_w;
  const float* head_b;
  float* yhat;
  int head_hv;
};

// Out-of-bounds-tap correction for a folded BN shift (see cnnitmo_fold_conv3x3):
// pixel (oh, ow) of an ho x wo 'same' conv loses sum_{t OOB} u_t[co].
__device__ __forceinline__ float border_corr(const float* __restrict__ U, int oh, int ow, int ho, int wo) {
  const bool top = oh == 0, bot = oh == ho - 1, lef = ow == 0, rig = ow == wo - 1;
  if (!(top | bot | lef | rig)) return 0.f;
  float c = 0.f;
  if (top) c += U[0];
  if (bot) c += U[1];
  if (lef) c += U[2];
  if (rig) c += U[3];
  if (top & lef) c -= U[4];
  if (top & rig) c -= U[5];
  if (bot & lef) c -= U[6];
  if (bot & rig) c -= U[7];
  return c;
}

// Column permutation inside each 32-column pair of 16x16x32 MFMA fragments: when LDS
// weight row nn holds GEMM column pair_perm(nn) and the MFMA runs with the operands
// swapped (C^T = W^T A^T), lane group g (= lane >> 4) of fragments (2p, 2p+1) holds the
// 8 CONSECUTIVE columns 32p + 8g .. +7 of its pixel (4 per fragment): one 16-byte
// store per (pixel, 8 columns) straight from the accumulators.
__host__ __device__ constexpr int pair_perm(int nn) {
  return 32 * (nn >> 5) + 8 * ((nn & 15) >> 2) + 4 * ((nn >> 4) & 1) + (nn & 3);
}

// Whole 128-byte lines from that layout.  Lane (frow = lane & 15, g = lane >> 4) holds
// octet g of pixel frow for the column pairs q (a) and q + 1 (b): 64 contiguous bytes
// of each pixel per pair, so a plain store instruction writes 16 pixels x 64 B.  After
// one exchange with lane frow ^ 8 (DPP row_ror:8), store 1 writes pixels 0-7 and store 2
// pixels 8-15 of the fragment, each as 8 whole lines: lane (frow, g) stores octet g of
// pair q + (frow >> 3) of pixel (frow & 7) (v1) and of pixel 8 + (frow & 7) (v2).
__device__ __forceinline__ void line_pair(const uint4& a, const uint4& b, int frow, uint4& v1, uint4& v2) {
  const bool lo = frow < 8;
  const uint4 x = lo ? b : a;  // what the partner lane needs from this one
  uint4 y;
  y.x = __builtin_amdgcn_update_dpp(0, (int)x.x, 0x128, 0xF, 0xF, false);
  y.y = __builtin_amdgcn_update_dpp(0, (int)x.y, 0x128, 0xF, 0xF, false);
  y.z = __builtin_amdgcn_update_dpp(0, (int)x.z, 0x128, 0xF, 0xF, false);
  y.w = __builtin_amdgcn_update_dpp(0, (int)x.w, 0x128, 0xF, 0xF, false);
  v1 = lo ? a : y;
  v2 = lo ? y : b;
}

template <typename T> struct Mma;
template <> struct Mma<bf16> {
  static __device__ __forceinline__ void run(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8, a),
                                                 __builtin_bit_cast(bf16x8, b), acc, 0, 0, 0);
  }
};
template <> struct Mma<float> {
  static __device__ __forceinline__ void run(f32x4& acc, const uint4& a, const uint4& b) {
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.x), __uint_as_float(b.x), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.y), __uint_as_float(b.y), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.z), __uint_as_float(b.z), acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a.w), __uint_as_float(b.w), acc, 0, 0, 0);
  }
};


// v2 (direct-to-LDS pipelined) forward family, igemm_fwd2.hip
template <typename T>
int launch_fwd2(FwdArgs a, hipStream_t s, const char* what);
int fwd2_stat_rows(long m);
bool fwd2_handles(int N);  // v2 is the faster kernel for this column count
int fwd2_bm(const FwdArgs& a, bool bf16);  // row tile of the v2 launch (128 or 256)
bool fwd2_t256(const FwdArgs& a, bool bf16);  // 256 x 256 tiles (bf16 tconv input gradient)
bool fwd2_pers(const FwdArgs& a, bool bf16);  // ... in the persistent kernel
// the bf16 Conv2DTranspose forward in training, persistent (igemm_fwd2.hip)
bool tfwd2p_handles(const FwdArgs& a, bool bf16);
long tfwd2p_stat_rows(const FwdArgs& a);
int launch_tfwd2p(FwdArgs a, hipStream_t s, const char* what);

// halo-tiled 3x3 conv (bf16, 4x64 output tiles), conv_halo.hip
bool halo_handles(const FwdArgs& a, bool f32 = false);  // f32: the fp32 forward / plain dgrad
int launch_halo(FwdArgs a, hipStream_t s, const char* what, bool f32 = false);
const char* halo_name(const FwdArgs& a, bool f32 = false);
long halo_stat_rows(const FwdArgs& a, bool f32 = false);

// tconv_stream.hip: Conv2DTranspose fwd (mode 0) / input-gradient (mode 1) as a
// streamed GEMM with the weight block resident in LDS (bf16)
bool tconv_stream_handles(int mode, int h, int w, int cin, int cout, bool epi);
long tconv_stream_rows(int mode, int n, int h, int w, int cin, int cout, bool epi);
const char* tconv_stream_name(int mode, int h, int w, int cin, int cout, bool epi);
int launch_tconv_stream(int mode, const void* a, long a_ld, int a_off, const void* b, int n, int h, int w,
                        int cin, int cout, void* out, long out_ld, int out_off, const float* bias, int flags,
                        const float* aff_scale, const float* aff_shift, float* stats, const float* coef,
                        const void* r, long r_ld, int r_off, hipStream_t s, const char* what);

// tconv_ws.hip: Conv2DTranspose fwd (mode 0) / input-gradient (mode 1) as a
// weight-stationary GEMM, barrier-free after the prologue (bf16; up6..up8)
// (f32: the fp32 inference forward, no BN sums)
bool tconv_ws_handles(int mode, int cin, int cout, bool f32 = false);
long tconv_ws_rows(int cin, int cout, bool f32 = false);
const char* tconv_ws_name(int mode, int cin, int cout, bool f32 = false);
int launch_tconv_ws(int mode, const void* a, long a_ld, int a_off, const void* b, int n, int h, int w, int cin,
                    int cout, void* out, long out_ld, int out_off, const float* bias, int flags,
                    const float* aff_scale, const float* aff_shift, float* stats, hipStream_t s, const char* what,
                    bool f32 = false);

// v2 (direct-to-LDS, multi-tap) bf16 weight gradients, igemm_wgrad2.hip
struct Wgrad2Args {
  const bf16* a;  // A operand source (gradient): channels m
  long a_ld;
  int a_off, ha, wa, a_scale;
  const bf16* b;  // B operand source (activation): channels n
  long b_ld;
  int b_off, hb, wb, b_scale;
  int nimg, hg, wg;
  int ntaps;
  int ayc, axc, byc, bxc;  // per-tap offsets (2-bit fields, value+1)
  int a_tapdep;            // 1: A depends on the tap (tconv), 0: B does (conv)
  int M, N;
  float* out;
  long split_stride, tap_stride;
  int out_ld;
  int mblocks, nblocks, tgroups, splits;
  long P, pix_per_split;
};

int launch_wgrad2(Wgrad2Args a, void* ws, size_t ws_bytes, hipStream_t s);
struct W2Label {
  bool ok;
  int bm, bn, tpb;
};
W2Label wgrad2_label(long P, int M, int N, int ntaps);
size_t wgrad2_ws_bytes(long P, int M, int N, int ntaps);

// row-streaming bf16 tconv2x2 weight gradient (all four taps per block), wgrad_tconv.hip
size_t wgrad_tconv_ws_bytes(int n, int h, int w, int cin, int cout);
const char* wgrad_tconv_name(int n, int h, int w, int cin, int cout);
int launch_wgrad_tconv(const bf16* x, long x_ld, int x_off, const bf16* dy, int n, int h, int w, int cin,
                       int cout, float* ws, size_t ws_bytes, hipStream_t s);
// its fp32 form (64 x 64 channel blocks, scalar-read fragments)
size_t wgrad_tconv_f32_ws_bytes(int n, int h, int w, int cin, int cout);
const char* wgrad_tconv_f32_name(int n, int h, int w, int cin, int cout);
int launch_wgrad_tconv_f32(const float* x, long x_ld, int x_off, const float* dy, int n, int h, int w, int cin,
                           int cout, float* ws, size_t ws_bytes, hipStream_t s);
// sliding-window bf16 3x3 weight gradient for the high-resolution layers, wgrad_halo.hip
// (x2 != null: a concatenate's two members, channels [0, 32) from x and [32, cin) from x2)
size_t wgrad_halo_ws_bytes(int n, int h, int w, int cin, int cout, bool cat = false);
const char* wgrad_halo_name(int n, int h, int w, int cin, int cout, bool cat = false);
int launch_wgrad_halo(const bf16* x, long x_ld, int x_off, const bf16* dz, int n, int h, int w, int cin,
                      int cout, float* ws, size_t ws_bytes, hipStream_t s, const bf16* x2 = nullptr,
                      long x2_ld = 0, int x2_off = 0);
// the same walk in fp32 (v_mfma_f32_16x16x4_f32), for fp32 training
size_t wgrad_halo_f32_ws_bytes(int n, int h, int w, int cin, int cout);
const char* wgrad_halo_f32_name(int n, int h, int w, int cin, int cout);
int launch_wgrad_halo_f32(const float* x, long x_ld, int x_off, const float* dz, int n, int h, int w, int cin,
                          int cout, float* ws, size_t ws_bytes, hipStream_t s);
