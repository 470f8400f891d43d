// Shared device helpers for the snrse HIP kernels (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define SNRSE_DEV __device__ __forceinline__

// Element storage types.  bf16 is kept as raw 16-bit patterns so loads/stores stay
// vectorised (Guideline 13) and conversions are explicit.
typedef uint16_t bf16_t;

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8_mfma;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

SNRSE_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }

// round-to-nearest-even f32 -> bf16 (NaN kept a NaN)
SNRSE_DEV bf16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x007fffffu)) return (bf16_t)((u >> 16) | 0x40);
  u += 0x7fffu + ((u >> 16) & 1u);
  return (bf16_t)(u >> 16);
}

// two f32 -> packed bf16x2 with the hardware RNE convert (v_cvt_pk_bf16_f32; NaN stays NaN)
SNRSE_DEV uint32_t pack_bf16x2(float lo, float hi) {
  typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2_t;
  const bf16x2_t v = {(__bf16)lo, (__bf16)hi};
  return __builtin_bit_cast(uint32_t, v);
}

// IEEE binary16 storage: the 16-bit fast path's format since round 6 (8 more significand bits' worth of
// accuracy than bf16 at the same bytes and the same MFMA rate; bf16 missed SURVEY 8(c)'s 1e-2 bound,
// profiles/r06a_bf16_attribution.jsonl).  A distinct type, so a kernel's format template argument picks the
// conversions and the MFMA.
struct f16_t {
  uint16_t bits;
};
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8_mfma;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2_t;

// The two 16-bit formats: the halves of a packed 32-bit word, the packing convert (round to nearest even:
// v_cvt_pk_bf16_f32 / v_cvt_pk_f16_f32) and the 16x16x32 MFMA with fp32 accumulation.
template <typename T> struct H16;
template <> struct H16<bf16_t> {
  SNRSE_DEV static float lo(uint32_t v) { return __uint_as_float(v << 16); }
  SNRSE_DEV static float hi(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }
  SNRSE_DEV static uint32_t pack(float a, float b) { return pack_bf16x2(a, b); }
  SNRSE_DEV static f32x4 mfma(const u32x4& a, const u32x4& b, f32x4 acc) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(bf16x8_mfma, a),
                                                   __builtin_bit_cast(bf16x8_mfma, b), acc, 0, 0, 0);
  }
};
template <> struct H16<f16_t> {
  SNRSE_DEV static float lo(uint32_t v) { return (float)__builtin_bit_cast(f16x2_t, v)[0]; }
  SNRSE_DEV static float hi(uint32_t v) { return (float)__builtin_bit_cast(f16x2_t, v)[1]; }
  SNRSE_DEV static uint32_t pack(float a, float b) {
    const f16x2_t v = {(_Float16)a, (_Float16)b};
    return __builtin_bit_cast(uint32_t, v);
  }
  SNRSE_DEV static f32x4 mfma(const u32x4& a, const u32x4& b, f32x4 acc) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(__builtin_bit_cast(f16x8_mfma, a),
                                                  __builtin_bit_cast(f16x8_mfma, b), acc, 0, 0, 0);
  }
};
// a 16-B vector of 8 16-bit values <-> 8 floats
template <typename T>
SNRSE_DEV void unpack8(const u32x4& r, float* v) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = H16<T>::lo(r[i]);
    v[2 * i + 1] = H16<T>::hi(r[i]);
  }
}
template <typename T>
SNRSE_DEV u32x4 pack8(const float* v) {
  u32x4 r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = H16<T>::pack(v[2 * i], v[2 * i + 1]);
  return r;
}

template <typename T> struct Elem;
template <> struct Elem<float> {
  static constexpr int kBytes = 4;
  SNRSE_DEV static float to_f(float v) { return v; }
  SNRSE_DEV static float from_f(float v) { return v; }
};
template <> struct Elem<bf16_t> {
  static constexpr int kBytes = 2;
  SNRSE_DEV static float to_f(bf16_t v) { return bf2f(v); }
  SNRSE_DEV static bf16_t from_f(float v) { return f2bf(v); }
};
template <> struct Elem<f16_t> {
  static constexpr int kBytes = 2;
  SNRSE_DEV static float to_f(f16_t v) { return (float)__builtin_bit_cast(_Float16, v.bits); }
  SNRSE_DEV static f16_t from_f(float v) { return f16_t{__builtin_bit_cast(uint16_t, (_Float16)v)}; }
};

// bf16-path SiLU: v_exp_f32 + v_rcp_f32 (1 ulp) instead of an IEEE division (~10 VALU ops);
// its error is far below the bf16 rounding of the result.
SNRSE_DEV float silu(float x) { return x * __builtin_amdgcn_rcpf(1.0f + __expf(-x)); }
// SiLU of y from its prescaled form z = -y log2(e) (the GroupNorm affine folded with -log2(e)):
// y / (1 + 2^z) = z * rcp(-(1 + 2^z) / ln 2) -- fma, exp, fma, rcp, mul per element (one multiply fewer
// than silu(fma(x, s, t))); z -> +inf gives -0, z -> -inf gives y.
constexpr float kNegLog2e = -1.44269504088896341f;
constexpr float kNegInvLn2 = -1.44269504088896341f;  // -1 / ln 2 (= -log2 e)
SNRSE_DEV float silu_z(float z) {
  return z * __builtin_amdgcn_rcpf(fmaf(__builtin_amdgcn_exp2f(z), kNegInvLn2, kNegInvLn2));
}

// Accurate SiLU for the fp32 parity mode (matches torch's x * sigmoid(x) to ~1 ulp).
SNRSE_DEV float silu_exact(float x) { return x / (1.0f + expf(-x)); }

SNRSE_DEV float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
SNRSE_DEV float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
// Sum of N per-lane partial vectors over the wave (N a power of two <= 64), transposed: lane l returns the
// full sum of element l % N.  Butterfly: at the stage of lane bit b a lane keeps the half of its elements whose
// index bit b equals its own lane bit and adds the partner's copy of them (N - 1 shuffles for N sums, instead of
// 6 N for N separate wave reductions); the lane bits above log2 N are folded at the end.
template <int N>
SNRSE_DEV float bfly_sum(float (&p)[N], int lane) {
  static_assert(N >= 1 && N <= 64 && (N & (N - 1)) == 0, "N: power of two <= 64");
  int lb = 0;
#pragma unroll
  for (int n = N; n > 1; n >>= 1, ++lb) {
    const bool hi = (lane >> lb) & 1;
#pragma unroll
    for (int i = 0; i < n / 2; ++i) {
      const float keep = hi ? p[2 * i + 1] : p[2 * i];
      const float send = hi ? p[2 * i] : p[2 * i + 1];
      p[i] = keep + __shfl_xor(send, 1 << lb, 64);
    }
  }
  float v = p[0];
#pragma unroll
  for (int b = lb; b < 6; ++b) v += __shfl_xor(v, 1 << b, 64);
  return v;
}

SNRSE_DEV float dot4(const f32x4& a, const f32x4& b) {
  return fmaf(a[0], b[0], fmaf(a[1], b[1], fmaf(a[2], b[2], a[3] * b[3])));
}

SNRSE_DEV double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// dtype codes shared with the C-ABI (include/snrse.h)
// F16 (round 6): the 16-bit fast path's default format, like BF16 on every 16-bit entry; F64: snrse_upfirdn2d
// only; F32X3: snrse_conv2d's split-bf16 fp32 GEMM (pre-split weights)
enum { SNRSE_F32 = 0, SNRSE_BF16 = 1, SNRSE_F16 = 2, SNRSE_F64 = 3, SNRSE_F32X3 = 4 };
inline bool snrse_is16(int dtype) { return dtype == SNRSE_BF16 || dtype == SNRSE_F16; }

// GroupNorm statistics buffers are [B][SNRSE_STAT_SLOTS][C][2] doubles: producers spread
// their atomics over the slots (a few hundred workgroups per image would otherwise queue on
// the same 2*C addresses), consumers sum the slots.
#define SNRSE_STAT_SLOTS 16

// Caller-owned launch context (include/snrse.h `snrse_ctx`): the tuning switches, the split-K
// workspace and the read-backs of the latest launch.  Host memory only.  The entries that take one
// read and write nothing else, so calls with distinct contexts are independent (one context per
// concurrently issuing host thread / stream); a NULL context means the process default one, which
// snrse_set_option / snrse_set_workspace edit (abi.cpp).
struct snrse_ctx {
  // switches (names as in snrse_set_option)
  int conv_variant = 0;        // 0 auto, 1 register-staged v1, 2 LDS-DMA v2, 5 halo v5
  int splitk = 1;              // 0: no K splitting of the small-image GEMMs
  int splitk_target = 256;     // workgroups a split-K launch aims for (C2 sweep: 256 best)
  int epi_nt = 2;              // halo-GEMM non-temporal output stores: 0 off, 1 on, 2 above epi_nt_mb
  int epi_nt_mb = 256;         // MB of output above which epi_nt = 2 streams (the Infinity Cache size)
  int h5_specialise = 1;       // compile-time epilogue flags for the common bf16 (halo GEMM) and fp32x3 (x3h pair
                               // schedule) ResBlock configurations
  int h5_tw = 0;               // halo tile width: 0 auto (32 where H % 8 == 0), 64, 32
  int stats_zeroed = 0;        // statistics buffers arrive zeroed (the caller clears one arena)
  int resample_variant = 0;    // 0 row-strip, 1 LDS-tiled gn_resample
  int resample_nt = 0;         // non-temporal stores in gn_resample
  int resample_down_rows = 4;  // output rows per down-sampling row strip (1, 2, 4; 4 fastest since r03)
  int x3_tile = 0;             // split-bf16 fp32 GEMM tile: 0 auto, 1 128x128, 2 256x128, 3 128x256, 4 halo
  int x3_tw = 0;               // fp32x3 halo GEMM tile: 0 auto (8 x 32 where H % 8 == 0, W % 32 == 0), 64 = 4 x 64
  int x3_nt = 1;               // fp32x3 halo GEMM: non-temporal output stores by the epi_nt rule (+0.3 %, r04r)
  int x3_spread = 2;           // halo split GEMM: 2 the pair schedule (2 taps per phase), 1 one tap per phase with the next
                               // chunk's halo stored one piece per tap, 0 the same stored in one go
  int head_small = 1;          // pyramid heads (Cout 4, bf16): 1 the wave-per-8-pixels kernel where the tiled head cannot
                               // take the image (H % 8 or W % 32), 2 also for <= 16384 output pixels, 0 never
  int head_part = 1;           // tiled pyramid head, Cout 4 (bf16): 1 the halo's 36 tap partials as a 1x1 GEMM + shifted
                               // sum (conv_head_part_kernel), 0 nine tap GEMMs over the halo (conv_head_kernel)
  int gn_slice = 1;            // small-image gn_apply with the statistics fold: 1 blocks own 64-channel slices (each
                               // folds 1/(C/64) of the image's statistics), 0 every block folds all C channels
  int ic_lds = 3;              // bf16 input conv: 1 the workgroup's input rows staged in LDS (W <= 1024), 2 the same
                               // with the channels split over wave pairs (4 waves / SIMD), 3 the output staged
                               // through LDS for 1-KB contiguous stores, 0 streaming loads
  // split-K workspace: [splits][M][Cout] f32 partial sums (NULL: no splitting)
  float* ws = nullptr;
  size_t ws_bytes = 0;
  // read-backs of the latest launch through this context
  int last_kernel = 0, last_ksplit = 1, last_epi_nt = 0, last_chunks = 1, last_tw = 0;
  // diagnostic timing (snrse_ctx_probe_begin): an event pair around each snrse_conv2d call
  hipEvent_t* probe_ev = nullptr;  // [2 * probe_cap]
  int* probe_kernel = nullptr;     // [probe_cap] generation that ran
  int probe_cap = 0, probe_n = 0;
};
// bracket one snrse_conv2d call with the context's next probe event pair (no-op when probing is off)
int snrse_ctx_probe_mark(snrse_ctx& c, hipStream_t s, bool end);
// `c`, or the process default context when c == NULL
snrse_ctx* snrse_ctx_resolve(snrse_ctx* c);
SNRSE_DEV size_t stat_idx(int b, int slot, int c, int C) {
  return (((size_t)b * SNRSE_STAT_SLOTS + slot) * C + c) * 2;
}
// (sum, sumsq) of channel c of image b, folded over the slots
SNRSE_DEV void stat_fold(const double* st, int b, int c, int C, double& s, double& ss) {
#pragma unroll 4
  for (int k = 0; k < SNRSE_STAT_SLOTS; ++k) {
    const double* q = st + stat_idx(b, k, c, C);
    s += q[0];
    ss += q[1];
  }
}

#define SNRSE_RET(expr)                              \
  do {                                               \
    hipError_t _e = (expr);                          \
    if (_e != hipSuccess) return (int)_e;            \
  } while (0)
#define SNRSE_LAUNCH_CHECK() SNRSE_RET(hipGetLastError())
#define SNRSE_EINVAL ((int)hipErrorInvalidValue)
