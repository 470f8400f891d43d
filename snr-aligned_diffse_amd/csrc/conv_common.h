// Shared parameter block and device helpers of the implicit-GEMM conv kernels
// (conv.hip: v1/v2/v5 kernels + C-ABI; conv_head.hip: pyramid heads).
#pragma once
#include "common.h"

#include <type_traits>
#include <utility>

namespace snrse_conv {

template <typename T> struct ConvTraits;
template <> struct ConvTraits<bf16_t> {
  static constexpr int KT = 64;  // elements per K-tile (128 B)
  static constexpr int EPC = 8;  // elements per 16-B chunk
};
template <> struct ConvTraits<f16_t> {
  static constexpr int KT = 64;
  static constexpr int EPC = 8;
};
template <> struct ConvTraits<float> {
  static constexpr int KT = 32;
  static constexpr int EPC = 4;
};

struct ConvParams {
  const void* src0; int C0;
  const void* src1; int C1;
  int B, H, W;
  int ksize;
  const void* wgt;  // [Npad][ksize*ksize*Cin]
  const void* sc_src; int Csc;    // shortcut source(s): [M][Csc] (+ [M][Csc1])
  const void* sc_src1; int Csc1;
  const void* sc_wgt;  // [Npad][Csc + Csc1]
  const float* bias;   // [Cout]
  const float* temb; int temb_stride;  // [B][temb_stride] (pre-offset to this layer's column 0)
  const void* res; int res_ld;         // residual [M][res_ld] (same dtype as output)
  float out_scale;
  const float* comb_src;  // [M][4] f32 input-skip pyramid (Combine.Conv_0 input)
  const float* comb_w;    // [Cout][4]
  const float* comb_b;    // [Cout]
  void* out; int Cout; int out_ld;
  double* stats;  // optional [B][SLOTS][Cout][2] per-channel (sum, sumsq) of the output (zeroed by launcher)
  int M;
  int ntn;        // N tiles (v2 grid)
  long long bytes0, bytes1, sc_bytes0, sc_bytes1, wbytes, sc_wbytes;  // buffer extents (v2)
  const float* gn_scale;  // optional [B][Cin] GroupNorm scale/shift applied to the main input (halo path)
  const float* gn_shift;
  int gn_act;             // SiLU after the GroupNorm affine
  float* ws;              // split-K partial sums [ksplit][M][Cout] f32 (caller-registered workspace)
  int ksplit;             // K splits of the v2 GEMM (1: the epilogue runs in the GEMM itself)
  unsigned long long* stamps;  // timing-diagnostic build only (-DSNRSE_STAMPS): [blocks][8][32]
  int epi_nt;      // image-tile epilogue: non-temporal output stores
};

#ifdef SNRSE_STAMPS
// Diagnostic build: s_memtime stamps of the halo kernel's segments (LDS, copied out at the
// end).  Read their shares, never the build's run time (the stamp waits forbid overlaps).
inline unsigned long long* g_stamp_buf = nullptr;
#define SNRSE_STAMP(I)                                                                        \
  do {                                                                                      \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    unsigned long long t_;                                                                  \
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");              \
    __builtin_amdgcn_sched_barrier(0);                                                      \
    if (lane == 0) lst[(I)] = t_;                                                           \
  } while (0)
#else
#define SNRSE_STAMP(I) \
  do {                 \
  } while (0)
#endif

template <typename T>
SNRSE_DEV f32x4 mfma_chunk(const u32x4& a, const u32x4& b, f32x4 acc);

template <>
SNRSE_DEV f32x4 mfma_chunk<bf16_t>(const u32x4& a, const u32x4& b, f32x4 acc) {
  return H16<bf16_t>::mfma(a, b, acc);
}
template <>
SNRSE_DEV f32x4 mfma_chunk<f16_t>(const u32x4& a, const u32x4& b, f32x4 acc) {
  return H16<f16_t>::mfma(a, b, acc);
}
template <>
SNRSE_DEV f32x4 mfma_chunk<float>(const u32x4& a, const u32x4& b, f32x4 acc) {
#pragma unroll
  for (int j = 0; j < 4; ++j)
    acc = __builtin_amdgcn_mfma_f32_16x16x4f32(__uint_as_float(a[j]), __uint_as_float(b[j]), acc, 0, 0, 0);
  return acc;
}

SNRSE_DEV int swz(int row, int chunk) { return (row << 7) + ((chunk ^ (row & 7)) << 4); }

// f(integral_constant<int, 0>) ... f(integral_constant<int, N - 1>): compile-time step indices for hand-scheduled loops
template <int N, typename F, int... S>
SNRSE_DEV void static_for_impl(F&& f, std::integer_sequence<int, S...>) {
  (f(std::integral_constant<int, S>{}), ...);
}
template <int N, typename F>
SNRSE_DEV void static_for(F&& f) {
  static_for_impl<N>(f, std::make_integer_sequence<int, N>{});
}

SNRSE_DEV __amdgpu_buffer_rsrc_t make_rsrc(const void* base, long long bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  const int n = __builtin_amdgcn_readfirstlane((int)bytes);
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0, n, 0x00020000);
}

// Pyramid heads (conv_head.hip): 3x3, Cout <= 16, f32 output, optional fused GroupNorm+SiLU.
// f16: the input / weights are IEEE fp16 (else bf16)
int launch_head(const ConvParams& p, hipStream_t s, bool part, bool f16);
int launch_head_x3(const ConvParams& p, hipStream_t s);
bool head_ok(const ConvParams& p, bool x3 = false);
int launch_head_small(const ConvParams& p, hipStream_t s, bool split = false, bool f16 = false);
bool head_small_ok(const ConvParams& p);

// Epilogue flags as a compile-time mask (EF >= 0: the halo GEMMs' common configurations, no per-pass
// branches) or read from the parameters at run time (EF = -1).
enum { EF_TEMB = 1, EF_RES = 2, EF_COMB = 4, EF_STATS = 8, EF_NT = 16, EF_RT = -1 };
inline int epi_flags(const ConvParams& p) {  // host side (launch dispatch)
  return (p.temb ? EF_TEMB : 0) | (p.res ? EF_RES : 0) | (p.comb_src ? EF_COMB : 0) | (p.stats ? EF_STATS : 0) |
         (p.epi_nt ? EF_NT : 0);
}

// Halo image rows of 64 B (32 bf16 channels), 16-B chunk swizzled by (row >> 1) & 3: conflict-free
// ds_read_b128 lane groups for any 16 consecutive rows.
SNRSE_DEV int swz64(int row, int chunk) { return (row << 6) + ((chunk ^ ((row >> 1) & 3)) << 4); }

// GroupNorm prologue of the halo kernels (v5 GEMM, pyramid head) on one 16-B vector (8 channels of the 16-bit format
// T, out in T): GNM 1 = affine,
// 2 = affine + SiLU; `ok` = inside the image (else the conv's zero padding).  Written stage by stage
// over the 8 elements (8 independent exp / rcp chains) so the schedule can hide the transcendental
// latencies; element by element the chain was fully serial with an s_nop after every exp and rcp.
//
// GNM 2 takes the affine PRESCALED by -log2(e) (gn_silu_prescale): with z = -y log2(e),
//   SiLU(y) = y / (1 + 2^-y log2 e) = z * rcp(-(1 + 2^z) / ln 2),
// so the exp argument needs no multiply and 1 + 2^z folds its scale into one fma: 5 VALU per element
// (fma, exp, fma, rcp, mul) instead of 6.  z -> +inf gives -0 (SiLU's limit), z -> -inf gives y.
SNRSE_DEV float gn_silu_prescale(float v) { return v * kNegLog2e; }  // (kNegLog2e: common.h)

template <typename T, int GNM>
SNRSE_DEV u32x4 gn_xform8(const u32x4 v, const float* sc, const float* sh, bool ok) {
  float y[8];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    y[2 * i] = fmaf(H16<T>::lo(v[i]), sc[2 * i], sh[2 * i]);
    y[2 * i + 1] = fmaf(H16<T>::hi(v[i]), sc[2 * i + 1], sh[2 * i + 1]);
  }
  if constexpr (GNM == 2) {
    // y holds z here.  sched_barrier(0) between the stages: without it the scheduler (at the
    // kernel's 256-VGPR limit) re-serialises the 8 chains to save registers
    float e[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = __builtin_amdgcn_exp2f(y[k]);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < 8; ++k) e[k] = __builtin_amdgcn_rcpf(fmaf(e[k], kNegInvLn2, kNegInvLn2));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int k = 0; k < 8; ++k) y[k] *= e[k];
  }
  // zero padding as an AND mask: a select here becomes an exec-masked branch around the whole transform
  const uint32_t okm = 0u - (uint32_t)ok;
  u32x4 o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = H16<T>::pack(y[2 * i], y[2 * i + 1]) & okm;
  return o;
}

}  // namespace snrse_conv
