// Pyramid-head 3x3 convolution (Cout <= 16, f32 output) with the fused GroupNorm+SiLU prologue:
// the NCSNpp output_skip heads  pyr = conv3x3(SiLU(GN(h)), C -> 4) + up2(pyr)  (ncsnpp.py:348-366,
// layers.py:100-110).  The generic register-staged GEMM (conv_mfma_kernel) re-read every input pixel
// nine times through an im2col tile and synchronised per 64-channel k-step for 4 useful output
// channels; here the (4+2) x (64+2) halo of each 32-channel chunk is staged once (GroupNorm+SiLU
// applied in registers, zero padding kept), all 9 taps read it from LDS, and the next chunk's halo
// is loaded into registers under the current chunk's MFMAs.  The kernel is bound by one HBM pass
// over h and the GroupNorm+SiLU VALU; tile 8 rows x 32 px (halo 10 x 34 = 340 rows: 14 % fewer
// transformed halo vectors per pixel than 4 x 64's 396), each wave owns 2 image rows x 32 px x 16
// channels (4 of them real).
#include "conv_common.h"

namespace snrse_conv {
namespace {

constexpr int KH_TH = 8, KH_TW = 32, KH_HC = KH_TW + 2;
constexpr int KH_RW = KH_TH / 4;                // image rows per wave
constexpr int KH_HROWS = (KH_TH + 2) * KH_HC;  // 340
constexpr int KH_HJ = (KH_HROWS + 63) / 64;    // halo rows per thread: (tid >> 2) + 64 j
constexpr int KH_HALO = KH_HROWS * 64;         // 21760 B
constexpr int KH_WP = 9 * 16 * 4;              // 16-B weight pieces of one chunk: 9 taps x 16 co x 4
constexpr int KH_WJ = (KH_WP + 255) / 256;     // per thread (3)
constexpr int KH_MAXC = 1024;                  // input channels the LDS GroupNorm table holds
constexpr int KH_LDS = KH_HALO + 9 * 1024 + 2 * KH_MAXC * 4;  // + 9 taps x 16 co x 64 B + [2][C] affine

SNRSE_DEV int kh_swz(int row, int chunk) { return (row << 6) + ((chunk ^ ((row >> 1) & 3)) << 4); }

#define KH_LOAD_H(C_, HV)                                                                                      \
  do {                                                                                                         \
    const bool in_ = (C_) < nc;                                                                                \
    const int ch_ = in_ ? (C_) * 32 : 0;                                                                       \
    const bool u1_ = ch_ >= p.C0;                                                                              \
    const __amdgpu_buffer_rsrc_t r_ = u1_ ? make_rsrc(p.src1, p.bytes1) : make_rsrc(p.src0, p.bytes0);         \
    const int cs_ = u1_ ? p.C1 : p.C0, cc_ = (u1_ ? ch_ - p.C0 : ch_) + hcol * 8;                              \
    _Pragma("unroll") for (int j = 0; j < KH_HJ; ++j) {                                                        \
      const int voff_ = (hok[j] && in_) ? (hpix[j] * cs_ + cc_) * 2 : (int)0x80000000;                         \
      HV[j] = __builtin_amdgcn_raw_buffer_load_b128(r_, voff_, 0, 0);                                          \
    }                                                                                                          \
  } while (0)
#define KH_LOAD_W(C_)                                                                                          \
  do {                                                                                                         \
    const bool in_ = (C_) < nc;                                                                                \
    const int ch_ = (C_) * 32;                                                                                 \
    _Pragma("unroll") for (int k = 0; k < KH_WJ; ++k) {                                                        \
      const int pc_ = tid + 256 * k; /* tap (pc >> 6), co ((pc >> 2) & 15), 16-B chunk (pc & 3) */              \
      const int voff_ = (pc_ < KH_WP && in_) ? ((((pc_ >> 2) & 15) * K1 + (pc_ >> 6) * Cin + ch_ + (pc_ & 3) * 8) * 2) \
                                             : (int)0x80000000;                                                \
      wv[k] = __builtin_amdgcn_raw_buffer_load_b128(rw, voff_, 0, 0);                                          \
    }                                                                                                          \
  } while (0)

// grid: B * (H / 8) * (W / 32) workgroups of 256.  GNM: 0 no prologue, 1 GroupNorm affine, 2 + SiLU.
// Round 5: the halo of chunk c + 2 is requested as soon as chunk c's registers are in LDS (two register
// buffers: two chunks of transform + MFMA work of cover instead of one MFMA phase; level 0 in situ 421 -> 390 us,
// profiles/r05m_c2_dispatch_shapes.jsonl), every chunk issues the same loads (out-of-range offsets past the last
// chunk load zeros) so the compiler's vmcnt model stays exact, and the GroupNorm affine of the image is staged
// once in LDS (per-chunk scale / shift registers would have cost the third workgroup per CU).
#ifndef SNRSE_HEAD_MINB
#define SNRSE_HEAD_MINB 1  // workgroups per CU the register allocation is bounded for (A/B builds)
#endif
template <typename T, int GNM>
__global__ __launch_bounds__(256, SNRSE_HEAD_MINB) void conv_head_kernel(ConvParams p) {
  __shared__ __attribute__((aligned(16))) char smem[KH_LDS];
  char* const halo = smem;
  char* const wsl = smem + KH_HALO;
  float* const gtab = (float*)(smem + KH_HALO + 9 * 1024);  // [2][Cin] scale, shift (prescaled for GNM 2)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntw = p.W / KH_TW, nth = p.H / KH_TH;
  int t = blockIdx.x;
  const int w0 = (t % ntw) * KH_TW;
  t /= ntw;
  const int h0 = (t % nth) * KH_TH;
  const int b = t / nth;
  const int Cin = p.C0 + p.C1;
  const int nc = Cin >> 5;
  const int K1 = 9 * Cin;
  const int hcol = tid & 3;
  constexpr bool gn = GNM > 0;
  const int lrow = lane & 15, lg = lane >> 4;
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.wgt, p.wbytes);

  int hpix[KH_HJ];
  bool hok[KH_HJ];
#pragma unroll
  for (int j = 0; j < KH_HJ; ++j) {
    const int hr = (tid >> 2) + 64 * j;
    const int hy = hr / KH_HC, hx = hr - hy * KH_HC;
    const int ih = h0 + hy - 1, iw = w0 + hx - 1;
    hok[j] = hr < KH_HROWS && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
    hpix[j] = (b * p.H + ih) * p.W + iw;
  }
  u32x4 hv[KH_HJ], hw[KH_HJ], wv[KH_WJ];

  // acc[i]: D[co = 4 lg + e][px = w0 + 16 i + lrow]  (A = weights, B = halo pixels)
  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  // the affine table's loads go first: the in-order vmcnt wait before its LDS stores then leaves the halo
  // and weight loads behind it in flight
  float gsc[KH_MAXC / 256], gsh[KH_MAXC / 256];
  if constexpr (gn) {
#pragma unroll
    for (int k = 0; k < KH_MAXC / 256; ++k) {
      const int i = tid + 256 * k;
      if (i < Cin) {
        gsc[k] = p.gn_scale[(size_t)b * Cin + i];
        gsh[k] = p.gn_shift[(size_t)b * Cin + i];
      }
    }
  }
  KH_LOAD_H(0, hv);
  KH_LOAD_W(0);
  KH_LOAD_H(1, hw);
  if constexpr (gn) {
#pragma unroll
    for (int k = 0; k < KH_MAXC / 256; ++k) {
      const int i = tid + 256 * k;
      if (i < Cin) {
        gtab[i] = GNM == 2 ? gsc[k] * kNegLog2e : gsc[k];  // gn_xform8's prescaled SiLU affine
        gtab[Cin + i] = GNM == 2 ? gsh[k] * kNegLog2e : gsh[k];
      }
    }
    __syncthreads();
  }
  auto step = [&](int c, u32x4 (&h)[KH_HJ]) {
    // registers -> LDS: GroupNorm + SiLU on the halo (rows outside the image stay zero), weights
    float sc[8], sh[8];
    if constexpr (gn) {
      const float* gp = gtab + c * 32 + hcol * 8;
      const f32x4 s0 = *(const f32x4*)gp, s1 = *(const f32x4*)(gp + 4);
      const f32x4 t0 = *(const f32x4*)(gp + Cin), t1 = *(const f32x4*)(gp + Cin + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc[e] = s0[e]; sc[4 + e] = s1[e];
        sh[e] = t0[e]; sh[4 + e] = t1[e];
      }
    }
#pragma unroll
    for (int j = 0; j < KH_HJ; ++j) {
      const int hr = (tid >> 2) + 64 * j;
      if (j == KH_HJ - 1 && hr >= KH_HROWS) break;
      u32x4 v = h[j];
      if constexpr (gn) v = gn_xform8<T, GNM>(v, sc, sh, hok[j]);  // rows outside the image: the conv's zero padding
      *(u32x4*)(halo + kh_swz(hr, hcol)) = v;
    }
#pragma unroll
    for (int k = 0; k < KH_WJ; ++k) {
      const int pc = tid + 256 * k;
      if (pc < KH_WP) *(u32x4*)(wsl + (pc >> 6) * 1024 + kh_swz((pc >> 2) & 15, pc & 3)) = wv[k];
    }
    // both register sets are free again: the next chunk's weights first (the in-order vmcnt wait before their
    // LDS store then does not wait on the later halo), then the halo two chunks ahead (past the end: zeros)
    KH_LOAD_W(c + 1);
    KH_LOAD_H(c + 2, h);
    __syncthreads();
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int dy = tp / 3 - 1, dx = tp % 3 - 1;
      const int hbase = (wid * KH_RW + dy + 1) * KH_HC + dx + 1 + lrow;
      const u32x4 a = *(const u32x4*)(wsl + tp * 1024 + kh_swz(lrow, lg));
#pragma unroll
      for (int i = 0; i < 4; ++i) {  // pixels 16 i .. of the wave's 64: row (16 i) / TW, column (16 i) % TW
        const u32x4 bx = *(const u32x4*)(halo + kh_swz(hbase + (16 * i / KH_TW) * KH_HC + (16 * i) % KH_TW, lg));
        acc[i] = mfma_chunk<T>(a, bx, acc[i]);
      }
    }
    __syncthreads();
  };
  for (int c = 0; c < nc; c += 2) {  // nc is even: 16-bit channels come in 64-channel K-tiles (snrse_conv2d)
    step(c, hv);
    step(c + 1, hw);
  }
  // epilogue: lanes with 4 lg < Cout hold channels 4 lg .. 4 lg + 3 of one pixel
  const int co = 4 * lg;
  if (co < p.Cout) {
    f32x4 add = {0.f, 0.f, 0.f, 0.f};
    if (p.bias) add = f32x4{p.bias[co], p.bias[co + 1], p.bias[co + 2], p.bias[co + 3]};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const size_t m = ((size_t)b * p.H + h0 + wid * KH_RW + 16 * i / KH_TW) * p.W + w0 + (16 * i) % KH_TW + lrow;
      f32x4 v = acc[i] + add;
      if (p.res) v += *(const f32x4*)((const float*)p.res + m * p.res_ld + co);
      v *= p.out_scale;
      *(f32x4*)((float*)p.out + m * p.out_ld + co) = v;
    }
  }
}
// Round 5, Cout = 4: the 3 x 3 head as a 1 x 1 GEMM over the halo.  conv_head_kernel reads the halo once per
// tap (9 x 4 pixel fragments + a weight fragment per wave and chunk: ~184 KB of LDS reads per workgroup and
// chunk for 4 useful output channels); here every halo pixel's 36 tap partials  P[px][4 tap + co] =
// sum_ci x[px][ci] w[co][tap][ci]  accumulate over the chunks in registers (A = halo pixels, read once per
// chunk; B = the chunk's 36 (+ 12 zero) weight columns), and only after the last chunk does each output
// pixel sum its 9 shifted partials,  y[px][co] = sum_tap P[px + off(tap)][4 tap + co],  staged through LDS
// one 16-column block at a time.  LDS reads per workgroup and chunk: ~36 KB.
constexpr int KP_PB = (KH_HROWS + 15) / 16;     // 16-pixel blocks covering the halo (22: 352 rows)
constexpr int KP_NB = (KP_PB + 3) / 4;          // per wave (6)
constexpr int KP_PS = 20;                       // partials row stride (floats): conflict-free column writes
constexpr int KP_STAGE = KP_PB * 16 * KP_PS * 4;  // 28160 B: the halo (22528 B) and, at the end, a partials block
constexpr int KP_LDS = KP_STAGE + 3 * 1024 + 2 * KH_MAXC * 4;

SNRSE_DEV int kp_opaque(int v) {  // a copy the compiler cannot see through: values derived from it are recomputed
  int r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}
// the halo pixel offsets are recomputed per chunk from an opaque copy of the thread index (a few VALU ops) instead
// of living in six registers across the loop: at three workgroups per CU (<= 168 registers) the compiler spilled
// one, and the reload's vmcnt(0) waited on every halo load in flight
#define KP_LOAD_H(C_, HV)                                                                                      \
  do {                                                                                                         \
    const bool in_ = (C_) < nc;                                                                                \
    const int ch_ = in_ ? (C_) * 32 : 0;                                                                       \
    const bool u1_ = ch_ >= p.C0;                                                                              \
    const __amdgpu_buffer_rsrc_t r_ = u1_ ? make_rsrc(p.src1, p.bytes1) : make_rsrc(p.src0, p.bytes0);         \
    const int cs_ = u1_ ? p.C1 : p.C0, cc_ = (u1_ ? ch_ - p.C0 : ch_) + hcol * 8;                              \
    const int tq_ = kp_opaque(tid);                                                                            \
    _Pragma("unroll") for (int j = 0; j < KH_HJ; ++j) {                                                        \
      const int hr_ = (tq_ >> 2) + 64 * j;                                                                     \
      const int hy_ = hr_ / KH_HC, hx_ = hr_ - hy_ * KH_HC;                                                    \
      const int pix_ = (b * p.H + h0 + hy_ - 1) * p.W + w0 + hx_ - 1;                                          \
      const int voff_ = (hok[j] && in_) ? (pix_ * cs_ + cc_) * 2 : (int)0x80000000;                            \
      HV[j] = __builtin_amdgcn_raw_buffer_load_b128(r_, voff_, 0, 0);                                          \
    }                                                                                                          \
  } while (0)
#define KP_LOAD_W(C_)                                                                                          \
  do {                                                                                                         \
    const bool in_ = (C_) < nc;                                                                                \
    const int col_ = tid >> 2, tap_ = col_ >> 2, co_ = col_ & 3; /* column 4 tap + co, 16-B chunk tid & 3 */    \
    const int voff_ = (in_ && col_ < 36 && co_ < p.Cout)                                                       \
                          ? ((co_ * K1 + tap_ * Cin + (C_) * 32 + (tid & 3) * 8) * 2)                          \
                          : (int)0x80000000;                                                                   \
    wv = __builtin_amdgcn_raw_buffer_load_b128(rw, voff_, 0, 0);                                               \
  } while (0)

#ifndef SNRSE_HEADP_MINB
#define SNRSE_HEADP_MINB 3  // three workgroups per CU: <= 168 VGPR + AGPR (the 72 partials accumulators are AGPRs)
#endif
template <typename T, int GNM>
__global__ __launch_bounds__(256, SNRSE_HEADP_MINB) void conv_head_part_kernel(ConvParams p) {
  __shared__ __attribute__((aligned(16))) char smem[KP_LDS];
  char* const halo = smem;
  char* const wsl = smem + KP_STAGE;
  float* const gtab = (float*)(smem + KP_STAGE + 3 * 1024);  // [2][Cin] scale, shift (prescaled for GNM 2)
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntw = p.W / KH_TW, nth = p.H / KH_TH;
  int t = blockIdx.x;
  const int w0 = (t % ntw) * KH_TW;
  t /= ntw;
  const int h0 = (t % nth) * KH_TH;
  const int b = t / nth;
  const int Cin = p.C0 + p.C1;
  const int nc = Cin >> 5;
  const int K1 = 9 * Cin;
  const int hcol = tid & 3;
  constexpr bool gn = GNM > 0;
  const int lrow = lane & 15, lg = lane >> 4;
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.wgt, p.wbytes);

  bool hok[KH_HJ];
#pragma unroll
  for (int j = 0; j < KH_HJ; ++j) {
    const int hr = (tid >> 2) + 64 * j;
    const int hy = hr / KH_HC, hx = hr - hy * KH_HC;
    const int ih = h0 + hy - 1, iw = w0 + hx - 1;
    hok[j] = hr < KH_HROWS && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
  }
  u32x4 hv[KH_HJ], hw[KH_HJ], wv;
  // acc[k][cb]: P[px = 16 (wid + 4 k) + 4 lg + e][col = 16 cb + lrow]
  f32x4 acc[KP_NB][3];
#pragma unroll
  for (int k = 0; k < KP_NB; ++k)
#pragma unroll
    for (int cb = 0; cb < 3; ++cb) acc[k][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  float gsc[KH_MAXC / 256], gsh[KH_MAXC / 256];
  if constexpr (gn) {
#pragma unroll
    for (int k = 0; k < KH_MAXC / 256; ++k) {
      const int i = tid + 256 * k;
      if (i < Cin) {
        gsc[k] = p.gn_scale[(size_t)b * Cin + i];
        gsh[k] = p.gn_shift[(size_t)b * Cin + i];
      }
    }
  }
  KP_LOAD_H(0, hv);
  KP_LOAD_W(0);
  KP_LOAD_H(1, hw);
  if (tid < (KP_PB * 16 - KH_HROWS) * 4)  // the padding rows past the halo: zeros (their partials are never read)
    *(u32x4*)(halo + kh_swz(KH_HROWS + (tid >> 2), tid & 3)) = u32x4{0u, 0u, 0u, 0u};
  if constexpr (gn) {
#pragma unroll
    for (int k = 0; k < KH_MAXC / 256; ++k) {
      const int i = tid + 256 * k;
      if (i < Cin) {
        gtab[i] = GNM == 2 ? gsc[k] * kNegLog2e : gsc[k];  // gn_xform8's prescaled SiLU affine
        gtab[Cin + i] = GNM == 2 ? gsh[k] * kNegLog2e : gsh[k];
      }
    }
    __syncthreads();
  }
  auto step = [&](int c, u32x4 (&h)[KH_HJ]) {
    float sc[8], sh[8];
    if constexpr (gn) {
      const float* gp = gtab + c * 32 + hcol * 8;
      const f32x4 s0 = *(const f32x4*)gp, s1 = *(const f32x4*)(gp + 4);
      const f32x4 t0 = *(const f32x4*)(gp + Cin), t1 = *(const f32x4*)(gp + Cin + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        sc[e] = s0[e]; sc[4 + e] = s1[e];
        sh[e] = t0[e]; sh[4 + e] = t1[e];
      }
    }
#pragma unroll
    for (int j = 0; j < KH_HJ; ++j) {
      const int hr = (tid >> 2) + 64 * j;
      if (j == KH_HJ - 1 && hr >= KH_HROWS) break;
      u32x4 v = h[j];
      if constexpr (gn) v = gn_xform8<T, GNM>(v, sc, sh, hok[j]);  // rows outside the image: the conv's zero padding
      *(u32x4*)(halo + kh_swz(hr, hcol)) = v;
    }
    if (tid < 192) *(u32x4*)(wsl + kh_swz(tid >> 2, tid & 3)) = wv;  // 48 columns x 4 16-B chunks
    KP_LOAD_W(c + 1);
    KP_LOAD_H(c + 2, h);
    __syncthreads();
    // (the weight fragments are re-read per pixel block: 8 registers fewer than holding all three, which kept the
    // kernel at three workgroups per CU without a spill -- a spill reload's vmcnt(0) waited on every halo load)
#pragma unroll
    for (int k = 0; k < KP_NB; ++k) {
      const int pb = wid + 4 * k;
      if (pb < KP_PB) {
        const u32x4 a = *(const u32x4*)(halo + kh_swz(pb * 16 + lrow, lg));
#pragma unroll
        for (int cb = 0; cb < 3; ++cb)
          acc[k][cb] = mfma_chunk<T>(a, *(const u32x4*)(wsl + kh_swz(cb * 16 + lrow, lg)), acc[k][cb]);
      }
    }
    __syncthreads();
  };
  for (int c = 0; c < nc; c += 2) {  // nc is even: 16-bit channels come in 64-channel K-tiles (snrse_conv2d)
    step(c, hv);
    step(c + 1, hw);
  }
  // the shifted sum: thread = output pixel (tile row r, column x), one 16-column block (taps 4 cb ..) at a time
  float* const part = (float*)smem;
  const int r = tid >> 5, x = tid & 31;
  f32x4 y = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int cb = 0; cb < 3; ++cb) {
#pragma unroll
    for (int k = 0; k < KP_NB; ++k) {
      const int pb = wid + 4 * k;
      if (pb < KP_PB) {
#pragma unroll
        for (int e = 0; e < 4; ++e) part[(pb * 16 + lg * 4 + e) * KP_PS + lrow] = acc[k][cb][e];
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int tap = 4 * cb + j;
      if (tap < 9) {
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        y += *(const f32x4*)(part + ((r + dy + 1) * KH_HC + x + dx + 1) * KP_PS + 4 * j);
      }
    }
    __syncthreads();
  }
  const size_t m = ((size_t)b * p.H + h0 + r) * p.W + w0 + x;
  if (p.bias) y += f32x4{p.bias[0], p.bias[1], p.bias[2], p.bias[3]};
  if (p.res) y += *(const f32x4*)((const float*)p.res + m * p.res_ld);
  y *= p.out_scale;
  *(f32x4*)((float*)p.out + m * p.out_ld) = y;
}
#undef KP_LOAD_W
#undef KP_LOAD_H
#undef KH_LOAD_H
#undef KH_LOAD_W

// fp32 form for the split-bf16 parity mode (SNRSE_F32X3): fp32 activations, weights pre-split per 32-element
// K-tile into 32 hi then 32 lo bf16 (ops.split_weight).  Each halo vector (8 fp32 channels, 2 x 16 B) gets
// the GroupNorm(+SiLU) in fp32 exactly as conv_x3h_kernel applies it, then is split into hi = bf16(x) and
// lo = bf16(x - hi) halves stored in two LDS halos; every tap accumulates hi.hi + hi.lo + lo.hi.  Replaces
// the fp32 mode's separate gn_act pass and register-staged Cout <= 16 GEMM (the fp32 input is read once).
constexpr int KH3_WP = 2 * KH_WP;                // hi + lo weight pieces of one chunk
constexpr int KH3_WJ = (KH3_WP + 255) / 256;     // per thread (5)
constexpr int KH3_LDS = 2 * KH_HALO + 2 * 9 * 1024;  // 61,952 B

#define KH3_LOAD(C_)                                                                                           \
  do {                                                                                                         \
    const int ch_ = (C_) * 32;                                                                                 \
    const bool u1_ = ch_ >= p.C0;                                                                              \
    const __amdgpu_buffer_rsrc_t r_ = u1_ ? make_rsrc(p.src1, p.bytes1) : make_rsrc(p.src0, p.bytes0);         \
    const int cs_ = u1_ ? p.C1 : p.C0, cc_ = (u1_ ? ch_ - p.C0 : ch_) + hcol * 8;                              \
    _Pragma("unroll") for (int j = 0; j < KH_HJ; ++j) {                                                        \
      const int voff_ = hok[j] ? (hpix[j] * cs_ + cc_) * 4 : (int)0x80000000;                                  \
      hv0[j] = __builtin_amdgcn_raw_buffer_load_b128(r_, voff_, 0, 0);                                         \
      hv1[j] = __builtin_amdgcn_raw_buffer_load_b128(r_, voff_ + 16, 0, 0);                                    \
    }                                                                                                          \
    _Pragma("unroll") for (int k = 0; k < KH3_WJ; ++k) {                                                       \
      const int pc_ = tid + 256 * k, h_ = pc_ >= KH_WP, pp_ = pc_ - h_ * KH_WP;                                \
      /* tap (pp >> 6), co ((pp >> 2) & 15), 16-B chunk (pp & 3) of the hi (h = 0) or lo (h = 1) half */       \
      const int voff_ = pc_ < KH3_WP ? ((((pp_ >> 2) & 15) * 2 * K1 + 2 * ((pp_ >> 6) * Cin + ch_) + h_ * 32 +    \
                                         (pp_ & 3) * 8) * 2)                                                   \
                                      : (int)0x80000000;                                                       \
      wv[k] = __builtin_amdgcn_raw_buffer_load_b128(rw, voff_, 0, 0);                                          \
    }                                                                                                          \
    if (gn) {                                                                                                  \
      const float* sp_ = p.gn_scale + (size_t)b * Cin + ch_ + hcol * 8;                                        \
      const float* hp_ = p.gn_shift + (size_t)b * Cin + ch_ + hcol * 8;                                        \
      gs0 = *(const f32x4*)sp_;                                                                                \
      gs1 = *(const f32x4*)(sp_ + 4);                                                                          \
      gh0 = *(const f32x4*)hp_;                                                                                \
      gh1 = *(const f32x4*)(hp_ + 4);                                                                          \
    }                                                                                                          \
  } while (0)

template <int GNM>
__global__ __launch_bounds__(256) void conv_head_x3_kernel(ConvParams p) {
  __shared__ __attribute__((aligned(16))) char smem[KH3_LDS];
  char* const halo_hi = smem;
  char* const halo_lo = smem + KH_HALO;
  char* const wsl_hi = smem + 2 * KH_HALO;
  char* const wsl_lo = wsl_hi + 9 * 1024;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ntw = p.W / KH_TW, nth = p.H / KH_TH;
  int t = blockIdx.x;
  const int w0 = (t % ntw) * KH_TW;
  t /= ntw;
  const int h0 = (t % nth) * KH_TH;
  const int b = t / nth;
  const int Cin = p.C0 + p.C1;
  const int nc = Cin >> 5;
  const int K1 = 9 * Cin;
  const int hcol = tid & 3;
  constexpr bool gn = GNM > 0;
  const int lrow = lane & 15, lg = lane >> 4;
  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.wgt, p.wbytes);

  int hpix[KH_HJ];
  bool hok[KH_HJ];
#pragma unroll
  for (int j = 0; j < KH_HJ; ++j) {
    const int hr = (tid >> 2) + 64 * j;
    const int hy = hr / KH_HC, hx = hr - hy * KH_HC;
    const int ih = h0 + hy - 1, iw = w0 + hx - 1;
    hok[j] = hr < KH_HROWS && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
    hpix[j] = (b * p.H + ih) * p.W + iw;
  }
  u32x4 hv0[KH_HJ], hv1[KH_HJ], wv[KH3_WJ];
  f32x4 gs0 = {1.f, 1.f, 1.f, 1.f}, gs1 = gs0, gh0 = {0.f, 0.f, 0.f, 0.f}, gh1 = gh0;

  f32x4 acc[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  KH3_LOAD(0);
  for (int c = 0; c < nc; ++c) {
#pragma unroll
    for (int j = 0; j < KH_HJ; ++j) {
      const int hr = (tid >> 2) + 64 * j;
      if (j == KH_HJ - 1 && hr >= KH_HROWS) break;
      float x[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        x[k] = __uint_as_float(hv0[j][k]);
        x[4 + k] = __uint_as_float(hv1[j][k]);
      }
      if constexpr (gn) {
        const float sc[8] = {gs0[0], gs0[1], gs0[2], gs0[3], gs1[0], gs1[1], gs1[2], gs1[3]};
        const float sh[8] = {gh0[0], gh0[1], gh0[2], gh0[3], gh1[0], gh1[1], gh1[2], gh1[3]};
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float y = fmaf(x[k], sc[k], sh[k]);
          x[k] = hok[j] ? (GNM == 2 ? silu(y) : y) : 0.f;  // outside the image: the conv's zero padding
        }
      }
      u32x4 hi, lo;
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        hi[k] = pack_bf16x2(x[2 * k], x[2 * k + 1]);
        lo[k] = pack_bf16x2(x[2 * k] - __uint_as_float(hi[k] << 16), x[2 * k + 1] - __uint_as_float(hi[k] & 0xffff0000u));
      }
      *(u32x4*)(halo_hi + kh_swz(hr, hcol)) = hi;
      *(u32x4*)(halo_lo + kh_swz(hr, hcol)) = lo;
    }
#pragma unroll
    for (int k = 0; k < KH3_WJ; ++k) {
      const int pc = tid + 256 * k, h = pc >= KH_WP, pp = pc - h * KH_WP;
      if (pc < KH3_WP) *(u32x4*)((h ? wsl_lo : wsl_hi) + (pp >> 6) * 1024 + kh_swz((pp >> 2) & 15, pp & 3)) = wv[k];
    }
    __syncthreads();
    if (c + 1 < nc) KH3_LOAD(c + 1);
#pragma unroll
    for (int tp = 0; tp < 9; ++tp) {
      const int dy = tp / 3 - 1, dx = tp % 3 - 1;
      const int hbase = (wid * KH_RW + dy + 1) * KH_HC + dx + 1 + lrow;
      const u32x4 ah = *(const u32x4*)(wsl_hi + tp * 1024 + kh_swz(lrow, lg));
      const u32x4 al = *(const u32x4*)(wsl_lo + tp * 1024 + kh_swz(lrow, lg));
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int ho = kh_swz(hbase + (16 * i / KH_TW) * KH_HC + (16 * i) % KH_TW, lg);
        const u32x4 bh = *(const u32x4*)(halo_hi + ho);
        const u32x4 bl = *(const u32x4*)(halo_lo + ho);
        acc[i] = mfma_chunk<bf16_t>(ah, bh, acc[i]);
        acc[i] = mfma_chunk<bf16_t>(ah, bl, acc[i]);
        acc[i] = mfma_chunk<bf16_t>(al, bh, acc[i]);
      }
    }
    __syncthreads();
  }
  const int co = 4 * lg;
  if (co < p.Cout) {
    f32x4 add = {0.f, 0.f, 0.f, 0.f};
    if (p.bias) add = f32x4{p.bias[co], p.bias[co + 1], p.bias[co + 2], p.bias[co + 3]};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const size_t m = ((size_t)b * p.H + h0 + wid * KH_RW + 16 * i / KH_TW) * p.W + w0 + (16 * i) % KH_TW + lrow;
      f32x4 v = acc[i] + add;
      if (p.res) v += *(const f32x4*)((const float*)p.res + m * p.res_ld + co);
      v *= p.out_scale;
      *(f32x4*)((float*)p.out + m * p.out_ld + co) = v;
    }
  }
}
#undef KH3_LOAD

}  // namespace

// Pyramid heads of the levels the tiled kernel cannot take (H % 8 or W % 32 != 0: the 8 x 16 and 4 x 8 levels
// of the C2 pyramid, ncsnpp.py:348-366).  They ran on the register-staged GEMM (conv_mfma_kernel, 8-32
// workgroups walking 36 K-tiles: ~46 us per launch, profiles/r05a_c2_dispatch_shapes.jsonl) after a separate
// gn_act pass.  Here one wave owns PX = 8 consecutive output pixels of one row; a lane owns 4 input channels of
// every 256-channel pass and keeps their 9 taps x 4 output channels of weights in registers (packed bf16);
// each of the 3 x (PX + 2) input pixels is loaded once (8 B per lane), GroupNorm(+SiLU)-transformed in fp32
// (zero padding stays zero) and accumulated into the up to 3 output pixels it feeds.  The PX x 4 per-lane
// partial sums are reduced across the wave with bfly_sum<32>, which leaves lane l with output (px l / 4,
// co l % 4): the 32 results are one contiguous 128-B f32 store.  Cout == 4, C1 == 0, C0 % 256 == 0.
constexpr int KS_PX = 8;

// SPLIT (the fp32x3 mode): fp32 input (16-B loads of 4 channels) and weights pre-split per 32-element K-tile into
// 32 hi then 32 lo bf16 (ops.split_weight); the lane's weights are hi + lo in fp32, so the head is exact fp32 FMAs.
// T: the 16-bit format of the input and weights (bf16 for SPLIT)
template <typename T, int GNM, bool SPLIT>
__global__ __launch_bounds__(256) void conv_head_small_kernel(ConvParams p) {
  const int lane = threadIdx.x & 63;
  const int wv = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int nxw = (p.W + KS_PX - 1) / KS_PX;
  if (wv >= p.B * p.H * nxw) return;  // wave-uniform: whole waves past the end
  const int xw = wv % nxw;
  const int t = wv / nxw;
  const int y = t % p.H, b = t / p.H;
  const int x0 = xw * KS_PX;
  const int C = p.C0, K1 = 9 * C;
  const bf16_t* wg = (const bf16_t*)p.wgt;
  float acc[KS_PX][4];
#pragma unroll
  for (int i = 0; i < KS_PX; ++i)
#pragma unroll
    for (int co = 0; co < 4; ++co) acc[i][co] = 0.f;
  for (int c0 = 0; c0 < C; c0 += 256) {
    const int c = c0 + 4 * lane;
    f32x4 wq[9][4];
#pragma unroll
    for (int tp = 0; tp < 9; ++tp)
#pragma unroll
      for (int co = 0; co < 4; ++co) {
        const int k = tp * C + c;
        uint2 h;
        f32x4 w;
        if constexpr (SPLIT) {
          const bf16_t* wp = wg + (size_t)co * 2 * K1 + (k >> 5) * 64 + (k & 31);
          h = *(const uint2*)wp;
          const uint2 l = *(const uint2*)(wp + 32);
          w = f32x4{__uint_as_float(h.x << 16) + __uint_as_float(l.x << 16),
                    __uint_as_float(h.x & 0xffff0000u) + __uint_as_float(l.x & 0xffff0000u),
                    __uint_as_float(h.y << 16) + __uint_as_float(l.y << 16),
                    __uint_as_float(h.y & 0xffff0000u) + __uint_as_float(l.y & 0xffff0000u)};
        } else {
          h = *(const uint2*)(wg + (size_t)co * K1 + k);
          w = f32x4{H16<T>::lo(h.x), H16<T>::hi(h.x), H16<T>::lo(h.y), H16<T>::hi(h.y)};
        }
        wq[tp][co] = w;
      }
    f32x4 gs = {1.f, 1.f, 1.f, 1.f}, gh = {0.f, 0.f, 0.f, 0.f};
    if constexpr (GNM > 0) {
      gs = *(const f32x4*)(p.gn_scale + (size_t)b * C + c);
      gh = *(const f32x4*)(p.gn_shift + (size_t)b * C + c);
    }
#pragma unroll
    for (int dy = -1; dy <= 1; ++dy) {
      const int yy = y + dy;
      if (yy < 0 || yy >= p.H) continue;  // wave-uniform
#pragma unroll
      for (int j = 0; j < KS_PX + 2; ++j) {
        const int xx = x0 - 1 + j;
        if (xx < 0 || xx >= p.W) continue;  // wave-uniform
        const size_t pix = ((size_t)b * p.H + yy) * p.W + xx;
        float v[4];
        if constexpr (SPLIT) {
          const f32x4 r = *(const f32x4*)((const float*)p.src0 + pix * C + c);
          v[0] = r[0]; v[1] = r[1]; v[2] = r[2]; v[3] = r[3];
        } else {
          const uint2 raw = *(const uint2*)((const bf16_t*)p.src0 + pix * C + c);
          v[0] = H16<T>::lo(raw.x); v[1] = H16<T>::hi(raw.x);
          v[2] = H16<T>::lo(raw.y); v[3] = H16<T>::hi(raw.y);
        }
        if constexpr (GNM > 0) {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const float a = fmaf(v[e], gs[e], gh[e]);
            v[e] = GNM == 2 ? (SPLIT ? silu_exact(a) : silu(a)) : a;
          }
        }
#pragma unroll
        for (int dx = -1; dx <= 1; ++dx) {
          const int i = j - 1 - dx;  // the output pixel x0 + i reads this column through tap dx
          if (i < 0 || i >= KS_PX) continue;
          const int tp = (dy + 1) * 3 + dx + 1;
#pragma unroll
          for (int co = 0; co < 4; ++co) {
            const f32x4 w = wq[tp][co];
            float a = acc[i][co];
            a = fmaf(v[0], w[0], a);
            a = fmaf(v[1], w[1], a);
            a = fmaf(v[2], w[2], a);
            a = fmaf(v[3], w[3], a);
            acc[i][co] = a;
          }
        }
      }
    }
  }
  float pp[4 * KS_PX];
#pragma unroll
  for (int i = 0; i < KS_PX; ++i)
#pragma unroll
    for (int co = 0; co < 4; ++co) pp[4 * i + co] = acc[i][co];
  const float s = bfly_sum<4 * KS_PX>(pp, lane);
  const int i = (lane & 31) >> 2, co = lane & 3, x = x0 + i;
  if (lane < 32 && x < p.W) {
    const size_t m = ((size_t)b * p.H + y) * p.W + x;
    float o = s + (p.bias ? p.bias[co] : 0.f);
    if (p.res) o += ((const float*)p.res)[m * p.res_ld + co];
    ((float*)p.out)[m * p.out_ld + co] = o * p.out_scale;
  }
}

bool head_small_ok(const ConvParams& p) {
  if (p.ksize != 3 || p.Cout != 4 || p.C1 != 0 || p.C0 <= 0 || p.C0 % 256 || p.B <= 0) return false;
  if (p.sc_src || p.temb || p.comb_src || p.stats) return false;
  return (long long)p.B * p.H * ((p.W + KS_PX - 1) / KS_PX) < 0x7fffffffLL;
}

// split: the fp32x3 form (fp32 input, split weights); f16: fp16 input and weights (else bf16)
int launch_head_small(const ConvParams& p, hipStream_t s, bool split, bool f16) {
  if (!head_small_ok(p)) return SNRSE_EINVAL;
  const long long waves = (long long)p.B * p.H * ((p.W + KS_PX - 1) / KS_PX);
  const unsigned blocks = (unsigned)((waves + 3) / 4);
#define SNRSE_HS(T_, G_, S_) hipLaunchKernelGGL((conv_head_small_kernel<T_, G_, S_>), dim3(blocks), dim3(256), 0, s, p)
  if (split) {
    if (!p.gn_scale) SNRSE_HS(bf16_t, 0, true);
    else if (!p.gn_act) SNRSE_HS(bf16_t, 1, true);
    else SNRSE_HS(bf16_t, 2, true);
  } else if (f16) {
    if (!p.gn_scale) SNRSE_HS(f16_t, 0, false);
    else if (!p.gn_act) SNRSE_HS(f16_t, 1, false);
    else SNRSE_HS(f16_t, 2, false);
  } else {
    if (!p.gn_scale) SNRSE_HS(bf16_t, 0, false);
    else if (!p.gn_act) SNRSE_HS(bf16_t, 1, false);
    else SNRSE_HS(bf16_t, 2, false);
  }
#undef SNRSE_HS
  return (int)hipGetLastError();
}

// x3: the split-bf16 head (conv_head_x3_kernel), which has no LDS GroupNorm table and so no channel cap
bool head_ok(const ConvParams& p, bool x3) {
  if (p.ksize != 3 || p.Cout > 16 || p.Cout % 4 || p.H % KH_TH || p.W % KH_TW || p.B <= 0) return false;
  if (p.C0 % 32 || p.C1 % 32 || p.C0 + p.C1 <= 0 || (!x3 && p.C0 + p.C1 > KH_MAXC)) return false;
  if (p.sc_src || p.temb || p.comb_src || p.stats) return false;
  if (p.out_ld % 4 || (p.res && p.res_ld % 4)) return false;
  const long long lim = 0x7ff00000ll;
  return p.bytes0 < lim && p.bytes1 < lim && p.wbytes < lim;
}

template <typename T>
static int launch_head_t(const ConvParams& p, hipStream_t s, bool part, unsigned tiles) {
  if (part && p.Cout == 4) {
    if (!p.gn_scale) hipLaunchKernelGGL((conv_head_part_kernel<T, 0>), dim3(tiles), dim3(256), 0, s, p);
    else if (!p.gn_act) hipLaunchKernelGGL((conv_head_part_kernel<T, 1>), dim3(tiles), dim3(256), 0, s, p);
    else hipLaunchKernelGGL((conv_head_part_kernel<T, 2>), dim3(tiles), dim3(256), 0, s, p);
    return (int)hipGetLastError();
  }
  if (!p.gn_scale) hipLaunchKernelGGL((conv_head_kernel<T, 0>), dim3(tiles), dim3(256), 0, s, p);
  else if (!p.gn_act) hipLaunchKernelGGL((conv_head_kernel<T, 1>), dim3(tiles), dim3(256), 0, s, p);
  else hipLaunchKernelGGL((conv_head_kernel<T, 2>), dim3(tiles), dim3(256), 0, s, p);
  return (int)hipGetLastError();
}

int launch_head(const ConvParams& p, hipStream_t s, bool part, bool f16) {
  if (!head_ok(p)) return SNRSE_EINVAL;
  const long long tiles = (long long)p.B * (p.H / KH_TH) * (p.W / KH_TW);
  if (tiles <= 0 || tiles > 0x7fffffffLL) return SNRSE_EINVAL;
  return f16 ? launch_head_t<f16_t>(p, s, part, (unsigned)tiles) : launch_head_t<bf16_t>(p, s, part, (unsigned)tiles);
}

// the split-bf16 form: same shape contract, fp32 activations (p.bytes* are fp32 extents)
int launch_head_x3(const ConvParams& p, hipStream_t s) {
  if (!head_ok(p, true)) return SNRSE_EINVAL;
  const long long tiles = (long long)p.B * (p.H / KH_TH) * (p.W / KH_TW);
  if (tiles <= 0 || tiles > 0x7fffffffLL) return SNRSE_EINVAL;
  if (!p.gn_scale) hipLaunchKernelGGL(conv_head_x3_kernel<0>, dim3((unsigned)tiles), dim3(256), 0, s, p);
  else if (!p.gn_act) hipLaunchKernelGGL(conv_head_x3_kernel<1>, dim3((unsigned)tiles), dim3(256), 0, s, p);
  else hipLaunchKernelGGL(conv_head_x3_kernel<2>, dim3((unsigned)tiles), dim3(256), 0, s, p);
  return (int)hipGetLastError();
}

}  // namespace snrse_conv
