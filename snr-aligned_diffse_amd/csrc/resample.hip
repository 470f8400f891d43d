// LDS-tiled GroupNorm-apply + SiLU + FIR [1,3,3,1] down/up-sampling, and the elementwise
// GroupNorm-apply (+ SiLU) over a channel concatenation, both from precomputed per-(b, c)
// scale / shift (snrse_gn_scale_shift).  bf16 storage (the row-strip kernel also f32), f32 arithmetic
// (gfx950).
//
// Reference ops replaced (BigGAN ResBlock with up / down, layerspp.py:245-268):
//   h = act(GroupNorm_0(x)); h = upsample_2d / downsample_2d(h, fir_kernel)   (:245-257)
//   x = upsample_2d / downsample_2d(x, fir_kernel)  -- the shortcut input     (:249, :255)
//   up_or_down_sampling.py:195-257 (upfirdn2d with k = outer([1,3,3,1]) / 64, gain 1 (down)
//   or 4 (up), zero padding of the activated tensor).
// One pass reads x once, activates every input pixel once (the per-output gn_apply kernel
// re-activated each input 4x (down) / 16x (up) and folded the statistics in every block), and
// writes both the activated and the raw resampled tensors; the block's input tile is staged in
// LDS (raw bf16; activated bf16 for down, f32 for up; f32 FIR arithmetic).
#include "common.h"

#include <type_traits>

// switches (snrse_ctx, common.h): "resample_variant" 0 auto (row strips where C / 8 divides 64), 1 tiled;
// "resample_down_rows" output rows per down strip (1, 2, 4); "resample_nt" 1 = non-temporal stores in the
// row-strip kernel

namespace {

constexpr int kCB = 16;  // channels per block (two 8 x bf16 vectors per pixel)
constexpr int kNV = kCB / 8;

enum { MODE_DOWN = 1, MODE_UP = 2 };

template <int MODE> struct RTile;
// down x2: out[i] = sum_a k[a] x[2i + a - 1]; out tile 8 x 16 <- in tile 18 x 34
template <> struct RTile<MODE_DOWN> {
  static constexpr int OTY = 8, OTX = 16, ITY = 2 * OTY + 2, ITX = 2 * OTX + 2;
  SNRSE_DEV static int in0(int o0) { return 2 * o0 - 1; }
};
// up x2: out[2q] = (x[q-1] + 3 x[q]) / 4, out[2q+1] = (3 x[q] + x[q+1]) / 4; out tile 16 x 32 <- in 10 x 18
template <> struct RTile<MODE_UP> {
  static constexpr int OTY = 16, OTX = 32, ITY = OTY / 2 + 2, ITX = OTX / 2 + 2;
  SNRSE_DEV static int in0(int o0) { return o0 / 2 - 1; }
};

// Linear block id -> XCD-contiguous logical id: consecutive workgroups are dealt round-robin over
// the 8 XCDs, so without the remap the channel groups of one pixel tile (which share every
// 128-byte line of the input) would be fetched by 8 different L2s.
SNRSE_DEV int xcd_logical(int i, int n) {
  if (n & 7) return i;
  return (i & 7) * (n >> 3) + (i >> 3);
}

// grid: B * tiles_y * tiles_x * (C / 16) blocks of 256.  scale/shift [B][C] f32 or null (identity).
// E: the 16-bit format (bf16_t / f16_t)
template <typename E, int MODE>
__global__ __launch_bounds__(256) void gn_resample_kernel(const E* __restrict__ src, int C, int H, int W,
                                                          int tiles_x, int tiles_y, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, int act,
                                                          E* __restrict__ out_act, E* __restrict__ out_raw) {
  using T = RTile<MODE>;
  constexpr int NPX = T::ITY * T::ITX;
  // down: the activated tile is kept as bf16 (2 x 19.6 KB instead of 39 + 19.6 KB, so 4 blocks
  // share a CU: level-0 759 -> 501 us); up (17 KB tile, 4 taps per output) keeps f32, where the
  // extra unpacking cost more than the occupancy gained
  using ActT = std::conditional_t<MODE == MODE_DOWN, E, float>;
  __shared__ __attribute__((aligned(16))) ActT s_act[NPX * kCB];
  __shared__ __attribute__((aligned(16))) E s_raw[NPX * kCB];
  const int ncg = C / kCB;
  int id = xcd_logical(blockIdx.x, gridDim.x);
  const int cg = id % ncg;
  id /= ncg;
  const int tx = id % tiles_x;
  id /= tiles_x;
  const int ty = id % tiles_y;
  const int b = id / tiles_y;
  const int Ho = MODE == MODE_DOWN ? H / 2 : 2 * H, Wo = MODE == MODE_DOWN ? W / 2 : 2 * W;
  const int oy0 = ty * T::OTY, ox0 = tx * T::OTX;
  const int iy0 = T::in0(oy0), ix0 = T::in0(ox0);
  const int c0 = cg * kCB;
  const int tid = threadIdx.x;

  // stage: raw bf16 + act(x * scale + shift) f32; outside the image both are zero (zero padding).
  // Every thread keeps one 8-channel half of the group (v = tid & 1, since 256 % kNV == 0), so its
  // scale / shift are loaded once, and all of its input vectors are issued before the first use
  // (NIT loads in flight per thread instead of one).
  static_assert(256 % kNV == 0, "channel half per thread");
  constexpr int NIT = (NPX * kNV + 255) / 256;
  const int v = tid % kNV;
  const int c = c0 + 8 * v;
  float sc[8], sh[8];
  if (scale) {
    const float* sp = scale + (size_t)b * C + c;
    const float* hp = shift + (size_t)b * C + c;
    const f32x4 s0 = *(const f32x4*)sp, s1 = *(const f32x4*)(sp + 4);
    const f32x4 h0 = *(const f32x4*)hp, h1 = *(const f32x4*)(hp + 4);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      sc[i] = s0[i]; sc[i + 4] = s1[i];
      sh[i] = h0[i]; sh[i + 4] = h1[i];
    }
  } else {
#pragma unroll
    for (int i = 0; i < 8; ++i) { sc[i] = 1.f; sh[i] = 0.f; }
  }
  u32x4 rv[NIT];
  bool inb[NIT];
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int idx = tid + 256 * k;
    const int p = idx / kNV;
    const int ly = p / T::ITX, lx = p - ly * T::ITX;
    const int iy = iy0 + ly, ix = ix0 + lx;
    inb[k] = idx < NPX * kNV && iy >= 0 && iy < H && ix >= 0 && ix < W;
    rv[k] = inb[k] ? *(const u32x4*)(src + (((size_t)b * H + iy) * W + ix) * C + c) : u32x4{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int k = 0; k < NIT; ++k) {
    const int idx = tid + 256 * k;
    if (idx >= NPX * kNV) break;
    const int p = idx / kNV;
    float x[8], a[8];
    unpack8<E>(rv[k], x);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const float y = fmaf(x[i], sc[i], sh[i]);
      a[i] = inb[k] ? (act ? silu(y) : y) : 0.f;
    }
    *(u32x4*)(s_raw + p * kCB + 8 * v) = rv[k];
    if constexpr (MODE == MODE_DOWN) {
      *(u32x4*)(s_act + p * kCB + 8 * v) = pack8<E>(a);
    } else {
      f32x4* d = (f32x4*)(s_act + p * kCB + 8 * v);
      d[0] = f32x4{a[0], a[1], a[2], a[3]};
      d[1] = f32x4{a[4], a[5], a[6], a[7]};
    }
  }
  __syncthreads();

  constexpr int NOUT = T::OTY * T::OTX * kNV;
  for (int idx = tid; idx < NOUT; idx += 256) {
    const int p = idx / kNV;  // idx % kNV == v: the thread's channel half, as in the staging
    const int ly = p / T::OTX, lx = p - ly * T::OTX;
    const int oy = oy0 + ly, ox = ox0 + lx;
    if (oy >= Ho || ox >= Wo) continue;
    float oa[8], orw[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      oa[i] = 0.f;
      orw[i] = 0.f;
    }
    auto tap = [&](int py, int px, float w) {
      const int q = (py * T::ITX + px) * kCB + 8 * v;
      float x[8], ac[8];
      if constexpr (MODE == MODE_DOWN) {
        unpack8<E>(*(const u32x4*)(s_act + q), ac);
      } else {
        const f32x4 a0 = *(const f32x4*)(s_act + q), a1 = *(const f32x4*)(s_act + q + 4);
#pragma unroll
        for (int i = 0; i < 4; ++i) { ac[i] = a0[i]; ac[i + 4] = a1[i]; }
      }
      unpack8<E>(*(const u32x4*)(s_raw + q), x);
#pragma unroll
      for (int i = 0; i < 8; ++i) oa[i] = fmaf(ac[i], w, oa[i]);
#pragma unroll
      for (int i = 0; i < 8; ++i) orw[i] = fmaf(x[i], w, orw[i]);
    };
    if constexpr (MODE == MODE_DOWN) {
      const float k1[4] = {0.125f, 0.375f, 0.375f, 0.125f};
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) tap(2 * ly + a, 2 * lx + bb, k1[a] * k1[bb]);
    } else {
      // tile origins are even, so the local parity is the global one
      const int y0 = ((ly & 1) ? (ly >> 1) : (ly >> 1) - 1) + 1, x0 = ((lx & 1) ? (lx >> 1) : (lx >> 1) - 1) + 1;
      const float wy0 = (ly & 1) ? 0.75f : 0.25f, wx0 = (lx & 1) ? 0.75f : 0.25f;
      tap(y0, x0, wy0 * wx0);
      tap(y0, x0 + 1, wy0 * (1.f - wx0));
      tap(y0 + 1, x0, (1.f - wy0) * wx0);
      tap(y0 + 1, x0 + 1, (1.f - wy0) * (1.f - wx0));
    }
    const size_t o = (((size_t)b * Ho + oy) * Wo + ox) * C + c0 + 8 * v;
    *(u32x4*)(out_act + o) = pack8<E>(oa);
    if (out_raw) *(u32x4*)(out_raw + o) = pack8<E>(orw);
  }
}

// out [B][HW][C0 + C1] = act(x * scale + shift) of the channel concatenation (src0 | src1).
// grid (nblk, B): each block stages its image's scale / shift in LDS.
// T = bf16 (fast SiLU: v_exp + v_rcp, far below the bf16 rounding of the result) or float (the fp32
// parity mode: x / (1 + exp(-x)) as torch computes it); one 16-B vector per thread (8 bf16 / 4 f32)
template <typename T>
__global__ __launch_bounds__(256) void gn_act_kernel(const T* __restrict__ src0, int C0,
                                                     const T* __restrict__ src1, int C1, int HW,
                                                     int pix_per_blk, const float* __restrict__ scale,
                                                     const float* __restrict__ shift, int act,
                                                     T* __restrict__ out) {
  constexpr int V = 16 / (int)sizeof(T);
  extern __shared__ __attribute__((aligned(16))) float s_ss[];  // scale[C], shift[C]
  const int C = C0 + C1;
  const int b = blockIdx.y;
  for (int c = threadIdx.x; c < C; c += 256) {
    s_ss[c] = scale ? scale[(size_t)b * C + c] : 1.f;
    s_ss[C + c] = scale ? shift[(size_t)b * C + c] : 0.f;
  }
  __syncthreads();
  const int LP = C / V;
  const int p0 = blockIdx.x * pix_per_blk;
  const int p1 = min(HW, p0 + pix_per_blk);
  const int total = (p1 - p0) * LP;
  for (int idx = threadIdx.x; idx < total; idx += 256) {
    const int pix = p0 + idx / LP;
    const int c = (idx % LP) * V;
    const T* s = c < C0 ? src0 + ((size_t)b * HW + pix) * C0 + c : src1 + ((size_t)b * HW + pix) * C1 + (c - C0);
    const u32x4 raw = *(const u32x4*)s;
    u32x4 o;
    if constexpr (sizeof(T) == 2) {
      float x[8];
      unpack8<T>(raw, x);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const float y = fmaf(x[i], s_ss[c + i], s_ss[C + c + i]);
        x[i] = act ? silu(y) : y;
      }
      o = pack8<T>(x);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float y = fmaf(__uint_as_float(raw[i]), s_ss[c + i], s_ss[C + c + i]);
        o[i] = __float_as_uint(act ? silu_exact(y) : y);
      }
    }
    *(u32x4*)(out + ((size_t)b * HW + pix) * C + c) = o;
  }
}

// ---------------------------------------------------------------------------------------------------
// Row-strip variant (default where C / 8 divides 64).  The tiled kernel above gives each block 16
// channels of a pixel tile, so every wave-wide load or store touches 32 B of each 256-B pixel (C = 128)
// and the lines are completed by other blocks; at level 0 that ran at ~3 TB/s.  Here a thread owns one
// 8-channel vector of ONE output row over a segment of L output positions, and the NV = C / 8 lanes of a
// pixel are adjacent, so each wave instruction moves 64 / NV whole pixels (full 128-B lines).  The
// separable FIR [1,3,3,1] runs in registers: the vertical taps per input column (act and raw), then the
// horizontal taps over a sliding window of column values.  The GroupNorm + SiLU of an input vector is
// recomputed by each strip that reads it (down: (2 RD + 2) / RD x for strips of RD output rows, 1.5x at
// the default RD = 2; up: 4x; VALU, not bytes).
//   down: out(oy, ox) = sum_ab k[a] k[b] x(2oy-1+a, 2ox-1+b), k = [1,3,3,1]/8
//   up:   out(2p+i, 2q+j) from input rows {p-1, p} (i = 0) or {p, p+1} (i = 1) with weights (1/4, 3/4) /
//         (3/4, 1/4), and the same in columns: out(.., 2q) = (V(q-1) + 3 V(q)) / 4, out(.., 2q+1) =
//         (3 V(q) + V(q+1)) / 4
// Zero padding applies to the activated tensor and to x (out-of-image vectors are 0 for both).

// CPT channels of one pixel: bf16 16 B (8 ch) or 8 B (4 ch); f32 16 B (4 ch)
template <typename E, int CPT> struct RVec;
template <typename H> struct RVec16_8 {  // 16-bit formats (bf16_t / f16_t), 8 channels
  typedef u32x4 T;
  SNRSE_DEV static T load(__amdgpu_buffer_rsrc_t r, int off) { return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0); }
  SNRSE_DEV static void unpack(const T v, float* x) { unpack8<H>(v, x); }
  SNRSE_DEV static T pack(const float* x) { return pack8<H>(x); }
};
template <typename H> struct RVec16_4 {  // 16-bit formats, 4 channels
  typedef __attribute__((ext_vector_type(2))) unsigned int T;
  SNRSE_DEV static T load(__amdgpu_buffer_rsrc_t r, int off) { return __builtin_amdgcn_raw_buffer_load_b64(r, off, 0, 0); }
  SNRSE_DEV static void unpack(const T v, float* x) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      x[2 * i] = H16<H>::lo(v[i]);
      x[2 * i + 1] = H16<H>::hi(v[i]);
    }
  }
  SNRSE_DEV static T pack(const float* x) { return T{H16<H>::pack(x[0], x[1]), H16<H>::pack(x[2], x[3])}; }
};
template <> struct RVec<bf16_t, 8> : RVec16_8<bf16_t> {};
template <> struct RVec<f16_t, 8> : RVec16_8<f16_t> {};
template <> struct RVec<bf16_t, 4> : RVec16_4<bf16_t> {};
template <> struct RVec<f16_t, 4> : RVec16_4<f16_t> {};
template <> struct RVec<float, 4> {
  typedef u32x4 T;
  SNRSE_DEV static T load(__amdgpu_buffer_rsrc_t r, int off) { return __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0); }
  SNRSE_DEV static void unpack(const T v, float* x) {
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = __uint_as_float(v[i]);
  }
  SNRSE_DEV static T pack(const float* x) {
    return T{__float_as_uint(x[0]), __float_as_uint(x[1]), __float_as_uint(x[2]), __float_as_uint(x[3])};
  }
};

template <int CPT> struct RowVec {  // act and raw values of one CPT-channel vector
  float a[CPT], r[CPT];
};

SNRSE_DEV __amdgpu_buffer_rsrc_t rs_rsrc(const void* base, unsigned bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// Strips are numbered per image up to a multiple of the strips of one wave (64 / NV), so a wave never
// straddles two images: the image base is wave-uniform (one buffer resource, 32-bit offsets, hardware
// zero-fill of out-of-image vectors).  NV lanes (CPT channels each) cover one pixel, C = NV * CPT.
// RD (down only): output rows per strip.  A strip of RD rows reads 2 RD + 2 input rows, so each input
// vector's GroupNorm + SiLU is evaluated (2 RD + 2) / RD times instead of 4 (the kernel's VALU) and each
// input row is fetched by fewer strips (L2 traffic).
template <typename E, int MODE, int NV, int CPT, int RD = 1>
__global__ __launch_bounds__(256) void gn_resample_rows_kernel(const E* __restrict__ src, int H, int W, int L,
                                                               int nseg, int nrows, const float* __restrict__ scale,
                                                               const float* __restrict__ shift, int act,
                                                               E* __restrict__ out_act,
                                                               E* __restrict__ out_raw, int nblk, int B,
                                                               int sp_img, int nt) {
  using V = RVec<E, CPT>;
  constexpr int C = NV * CPT, SPB = 256 / NV;  // strips per block
  // XCD-aware bijective remap: consecutive logical blocks (neighbouring output rows, which share input
  // rows) run on one XCD and its L2
  const int q8 = nblk >> 3, r8 = nblk & 7, xcd = blockIdx.x & 7, pos = blockIdx.x >> 3;
  const int lb = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int v = threadIdx.x % NV;
  const int gs = lb * SPB + threadIdx.x / NV;
  const int b = __builtin_amdgcn_readfirstlane(gs / sp_img);
  const int ls = gs - b * sp_img;  // strip within the image
  if (b >= B || ls >= nrows * nseg) return;  // padding strips
  const int seg = ls % nseg;
  static_assert(MODE == MODE_DOWN || RD == 1, "multi-row strips: down only");
  const int orow = (ls / nseg) * RD;  // (first) output row
  const int Ho = MODE == MODE_DOWN ? H / 2 : 2 * H, Wo = MODE == MODE_DOWN ? W / 2 : 2 * W;
  // with act: the affine prescaled by -log2(e) for silu_z (common.h)
  const float pre = act ? kNegLog2e : 1.f;
  float sc[CPT], sh[CPT];
#pragma unroll
  for (int i = 0; i < CPT; ++i) {
    sc[i] = (scale ? scale[(size_t)b * C + CPT * v + i] : 1.f) * pre;
    sh[i] = (scale ? shift[(size_t)b * C + CPT * v + i] : 0.f) * pre;
  }
  const __amdgpu_buffer_rsrc_t rsrc = rs_rsrc(src + (size_t)b * H * W * C, (unsigned)((size_t)H * W * C * sizeof(E)));
  constexpr int NR = MODE == MODE_DOWN ? 2 * RD + 2 : 2;  // input rows of the strip's RD output rows
  int iy0;
  float wy[NR];
  if constexpr (MODE == MODE_DOWN) {
    iy0 = 2 * orow - 1;
#pragma unroll
    for (int a = 0; a < NR; ++a) wy[a] = 0.f;  // unused in down mode (per-row tap weights below)
  } else {
    const int p = orow >> 1;
    iy0 = (orow & 1) ? p : p - 1;
    wy[0] = (orow & 1) ? 0.75f : 0.25f;
    wy[1] = 1.f - wy[0];
  }
  bool rowok[NR];
#pragma unroll
  for (int a = 0; a < NR; ++a) rowok[a] = iy0 + a >= 0 && iy0 + a < H;

  // vertical taps of input column ix -> column value (act, raw); the loads are issued one step ahead of
  // their use (software pipelining: the next column's vectors are in flight while this one is filtered)
  struct Raw {
    typename V::T x[NR];
  };
  auto load_col = [&](int ix) {
    Raw rw;
    const bool colok = ix >= 0 && ix < W;
#pragma unroll
    for (int a = 0; a < NR; ++a) {
      const bool ok = colok && rowok[a];
      rw.x[a] = V::load(rsrc, ok ? (((iy0 + a) * W + ix) * C + CPT * v) * (int)sizeof(E) : (int)0x80000000);  // outside: 0
    }
    return rw;
  };
  // down: column values of the RD output rows (row rr takes input rows 2 rr .. 2 rr + 3 of the strip
  // with the vertical taps [1,3,3,1]/8); each input vector is transformed once.  Zero padding: rows
  // outside the image are skipped (their raw loads are 0 too) and an outside column's activated values
  // are cleared once per column, not per element.
  auto eval_cols = [&](const Raw& rw, int ix, RowVec<CPT> (&cv)[RD]) {
    const bool colok = ix >= 0 && ix < W;
    constexpr float kv[4] = {0.125f, 0.375f, 0.375f, 0.125f};
#pragma unroll
    for (int rr = 0; rr < RD; ++rr)
#pragma unroll
      for (int i = 0; i < CPT; ++i) { cv[rr].a[i] = 0.f; cv[rr].r[i] = 0.f; }
#pragma unroll
    for (int a = 0; a < NR; ++a) {
      if (!rowok[a]) continue;
      float x[CPT];
      V::unpack(rw.x[a], x);
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const float z = fmaf(x[i], sc[i], sh[i]);
        const float t = act ? silu_z(z) : z;
#pragma unroll
        for (int rr = 0; rr < RD; ++rr) {
          const int k = a - 2 * rr;
          if (k >= 0 && k < 4) {
            cv[rr].a[i] = fmaf(t, kv[k], cv[rr].a[i]);
            cv[rr].r[i] = fmaf(x[i], kv[k], cv[rr].r[i]);
          }
        }
      }
    }
    if (!colok) {
#pragma unroll
      for (int rr = 0; rr < RD; ++rr)
#pragma unroll
        for (int i = 0; i < CPT; ++i) cv[rr].a[i] = 0.f;
    }
  };
  auto eval_col = [&](const Raw& rw, int ix) {
    const bool colok = ix >= 0 && ix < W;
    RowVec<CPT> cv;
#pragma unroll
    for (int i = 0; i < CPT; ++i) { cv.a[i] = 0.f; cv.r[i] = 0.f; }
#pragma unroll
    for (int a = 0; a < NR; ++a) {
      if (!rowok[a]) continue;
      float x[CPT];
      V::unpack(rw.x[a], x);
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        const float z = fmaf(x[i], sc[i], sh[i]);
        const float t = act ? silu_z(z) : z;
        cv.a[i] = fmaf(t, wy[a], cv.a[i]);
        cv.r[i] = fmaf(x[i], wy[a], cv.r[i]);
      }
    }
    if (!colok) {
#pragma unroll
      for (int i = 0; i < CPT; ++i) cv.a[i] = 0.f;
    }
    return cv;
  };
  auto column = [&](int ix) { return eval_col(load_col(ix), ix); };
  auto store = [&](int ox, const float* a, const float* r, int rr = 0) {
    const size_t o = (((size_t)b * Ho + orow + rr) * Wo + ox) * C + CPT * v;
    if (nt) {
      __builtin_nontemporal_store(V::pack(a), (typename V::T*)(out_act + o));
      if (out_raw) __builtin_nontemporal_store(V::pack(r), (typename V::T*)(out_raw + o));
    } else {
      *(typename V::T*)(out_act + o) = V::pack(a);
      if (out_raw) *(typename V::T*)(out_raw + o) = V::pack(r);
    }
  };

  if constexpr (MODE == MODE_DOWN) {
    // out(ox) = k0 V(2ox-1) + k1 V(2ox) + k1 V(2ox+1) + k0 V(2ox+2): carry only the partial sum of the
    // two columns shared with the previous output
    const int ox0 = seg * L, ox1 = min(Wo, ox0 + L);
    float pa[RD][CPT], pr[RD][CPT];
    {
      RowVec<CPT> c0[RD], c1[RD];
      eval_cols(load_col(2 * ox0 - 1), 2 * ox0 - 1, c0);
      eval_cols(load_col(2 * ox0), 2 * ox0, c1);
#pragma unroll
      for (int rr = 0; rr < RD; ++rr)
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
          // explicit fmaf: the same rounding sequence in every RD instantiation (no contraction choice)
          pa[rr][i] = fmaf(0.375f, c1[rr].a[i], 0.125f * c0[rr].a[i]);
          pr[rr][i] = fmaf(0.375f, c1[rr].r[i], 0.125f * c0[rr].r[i]);
        }
    }
    Raw n2 = load_col(2 * ox0 + 1), n3 = load_col(2 * ox0 + 2);
    for (int ox = ox0; ox < ox1; ++ox) {
      const Raw r2 = n2, r3 = n3;
      if (ox + 1 < ox1) {
        n2 = load_col(2 * ox + 3);
        n3 = load_col(2 * ox + 4);
      }
      RowVec<CPT> c2[RD], c3[RD];
      eval_cols(r2, 2 * ox + 1, c2);
      eval_cols(r3, 2 * ox + 2, c3);
#pragma unroll
      for (int rr = 0; rr < RD; ++rr) {
        float oa[CPT], orw[CPT];
#pragma unroll
        for (int i = 0; i < CPT; ++i) {
          oa[i] = fmaf(0.125f, c3[rr].a[i], fmaf(0.375f, c2[rr].a[i], pa[rr][i]));
          orw[i] = fmaf(0.125f, c3[rr].r[i], fmaf(0.375f, c2[rr].r[i], pr[rr][i]));
          pa[rr][i] = fmaf(0.375f, c3[rr].a[i], 0.125f * c2[rr].a[i]);
          pr[rr][i] = fmaf(0.375f, c3[rr].r[i], 0.125f * c2[rr].r[i]);
        }
        store(ox, oa, orw, rr);
      }
    }
  } else {
    // output columns 2q, 2q+1 for input columns q in [q0, q1)
    const int q0 = seg * L, q1 = min(W, q0 + L);
    RowVec<CPT> cm = column(q0 - 1), cc = column(q0);
    Raw np = load_col(q0 + 1);
    for (int q = q0; q < q1; ++q) {
      const Raw rp = np;
      if (q + 1 < q1) np = load_col(q + 2);
      const RowVec<CPT> cp = eval_col(rp, q + 1);
      float ea[CPT], er[CPT], oa[CPT], orw[CPT];
#pragma unroll
      for (int i = 0; i < CPT; ++i) {
        ea[i] = 0.25f * cm.a[i] + 0.75f * cc.a[i];
        er[i] = 0.25f * cm.r[i] + 0.75f * cc.r[i];
        oa[i] = 0.75f * cc.a[i] + 0.25f * cp.a[i];
        orw[i] = 0.75f * cc.r[i] + 0.25f * cp.r[i];
      }
      store(2 * q, ea, er);
      store(2 * q + 1, oa, orw);
      cm = cc;
      cc = cp;
    }
  }
}

template <typename E, int MODE, int NV, int CPT, int RD = 1>
int launch_rows(const void* src, int B, int H, int W, const float* scale, const float* shift, int act, void* out_act,
                void* out_raw, hipStream_t stream, int nt) {
  const int nrows = MODE == MODE_DOWN ? H / 2 / RD : 2 * H;  // strips per column segment
  const int span = MODE == MODE_DOWN ? W / 2 : W;  // positions a strip walks (output cols / input cols)
  // strip length: 16 positions, shortened on small images until the grid has >= 2^17 threads (8 waves
  // per CU)
  int L = span >= 16 ? 16 : span;
  while (L > 1 && (long long)B * nrows * ((span + L - 1) / L) * NV < (1 << 17)) L >>= 1;
  const int nseg = (span + L - 1) / L;
  constexpr int SPB = 256 / NV, SPW = 64 / NV;
  const long long sp_img = ((long long)nrows * nseg + SPW - 1) / SPW * SPW;  // strips per image, padded
  const long long nblk = (sp_img * B + SPB - 1) / SPB;
  if (nblk > 0x7fffffffLL || sp_img * B > 0x7fffffffLL ||
      (long long)H * W * NV * CPT * (long long)sizeof(E) >= 0x7fffffffLL)
    return SNRSE_EINVAL;
  hipLaunchKernelGGL((gn_resample_rows_kernel<E, MODE, NV, CPT, RD>), dim3((unsigned)nblk), dim3(256), 0, stream,
                     (const E*)src, H, W, L, nseg, nrows, scale, shift, act, (E*)out_act, (E*)out_raw, (int)nblk, B,
                     (int)sp_img, nt);
  return (int)hipGetLastError();
}

// bf16 down: 4 channels per lane (8 input vectors per output column pair stay within 4 waves per SIMD);
// bf16 up: 8 channels per lane (16-B stores); f32: 4 channels per lane (16 B) both ways
template <typename E, int MODE, int RD>
int dispatch_rows_rd(const void* src, int C, int B, int H, int W, const float* scale, const float* shift, int act,
                     void* out_act, void* out_raw, hipStream_t stream, int nt) {
  constexpr int CPT = sizeof(E) == 4 ? 4 : (MODE == MODE_DOWN ? 4 : 8);
  if (C % CPT) return -1;
  switch (C / CPT) {
#define SNRSE_RS_NV(N) \
  case N: return launch_rows<E, MODE, N, CPT, RD>(src, B, H, W, scale, shift, act, out_act, out_raw, stream, nt);
    SNRSE_RS_NV(1)
    SNRSE_RS_NV(2)
    SNRSE_RS_NV(4)
    SNRSE_RS_NV(8)
    SNRSE_RS_NV(16)
    SNRSE_RS_NV(32)
    SNRSE_RS_NV(64)
#undef SNRSE_RS_NV
    default: return -1;  // not handled here
  }
}
// down strips of 4 output rows (bf16 default) hold 10 input vectors per column in flight; f32 vectors
// are twice the registers, so f32 strips stop at 2 rows
template <typename E, int MODE>
int dispatch_rows(const void* src, int C, int B, int H, int W, const float* scale, const float* shift, int act,
                  void* out_act, void* out_raw, hipStream_t stream, const snrse_ctx& cx) {
  if constexpr (MODE == MODE_DOWN) {
    const int Ho = H / 2;
    if constexpr (sizeof(E) == 2)
      if (cx.resample_down_rows >= 4 && Ho % 4 == 0)
        return dispatch_rows_rd<E, MODE, 4>(src, C, B, H, W, scale, shift, act, out_act, out_raw, stream,
                                            cx.resample_nt);
    if (cx.resample_down_rows >= 2 && Ho % 2 == 0)
      return dispatch_rows_rd<E, MODE, 2>(src, C, B, H, W, scale, shift, act, out_act, out_raw, stream, cx.resample_nt);
  }
  return dispatch_rows_rd<E, MODE, 1>(src, C, B, H, W, scale, shift, act, out_act, out_raw, stream, cx.resample_nt);
}

template <int MODE>
int launch_resample(const void* src, int C, int B, int H, int W, const float* scale, const float* shift, int act,
                    void* out_act, void* out_raw, int dtype, hipStream_t stream, const snrse_ctx& cx) {
  if (dtype == SNRSE_F32) {  // the row-strip kernel only (C / 4 dividing 256)
    const int r = dispatch_rows<float, MODE>(src, C, B, H, W, scale, shift, act, out_act, out_raw, stream, cx);
    return r >= 0 ? r : SNRSE_EINVAL;
  }
  const bool f16 = dtype == SNRSE_F16;
  if (cx.resample_variant == 0) {
    const int r = f16 ? dispatch_rows<f16_t, MODE>(src, C, B, H, W, scale, shift, act, out_act, out_raw, stream, cx)
                      : dispatch_rows<bf16_t, MODE>(src, C, B, H, W, scale, shift, act, out_act, out_raw, stream, cx);
    if (r >= 0) return r;
  }
  if (C % kCB) return SNRSE_EINVAL;
  using T = RTile<MODE>;
  const int Ho = MODE == MODE_DOWN ? H / 2 : 2 * H, Wo = MODE == MODE_DOWN ? W / 2 : 2 * W;
  const int tiles_y = (Ho + T::OTY - 1) / T::OTY, tiles_x = (Wo + T::OTX - 1) / T::OTX;
  const long long n = (long long)B * tiles_y * tiles_x * (C / kCB);
  if (n <= 0 || n > 0x7fffffffLL) return SNRSE_EINVAL;
  if (f16)
    hipLaunchKernelGGL((gn_resample_kernel<f16_t, MODE>), dim3((unsigned)n), dim3(256), 0, stream, (const f16_t*)src, C,
                       H, W, tiles_x, tiles_y, scale, shift, act, (f16_t*)out_act, (f16_t*)out_raw);
  else
    hipLaunchKernelGGL((gn_resample_kernel<bf16_t, MODE>), dim3((unsigned)n), dim3(256), 0, stream, (const bf16_t*)src,
                       C, H, W, tiles_x, tiles_y, scale, shift, act, (bf16_t*)out_act, (bf16_t*)out_raw);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" int snrse_gn_resample(snrse_ctx* ctx, const void* src, int C, int B, int H, int W, const float* scale,
                                 const float* shift, int act, int mode, void* out_act, void* out_raw, int dtype,
                                 hipStream_t stream) {
  if (!src || !out_act || C <= 0 || C % (dtype == SNRSE_F32 ? 4 : 8) || B <= 0 || H <= 0 || W <= 0 ||
      (!scale) != (!shift) || (!snrse_is16(dtype) && dtype != SNRSE_F32))
    return SNRSE_EINVAL;
  const snrse_ctx& cx = *snrse_ctx_resolve(ctx);
  if (mode == MODE_DOWN) {
    if ((H & 1) || (W & 1)) return SNRSE_EINVAL;
    return launch_resample<MODE_DOWN>(src, C, B, H, W, scale, shift, act, out_act, out_raw, dtype, stream, cx);
  }
  if (mode == MODE_UP)
    return launch_resample<MODE_UP>(src, C, B, H, W, scale, shift, act, out_act, out_raw, dtype, stream, cx);
  return SNRSE_EINVAL;
}

extern "C" int snrse_gn_act(const void* src0, int C0, const void* src1, int C1, int B, int HW, const float* scale,
                            const float* shift, int act, void* out, int dtype, hipStream_t stream) {
  const int C = C0 + C1;
  if (!snrse_is16(dtype) && dtype != SNRSE_F32) return SNRSE_EINVAL;
  const int V = snrse_is16(dtype) ? 8 : 4;
  if (!src0 || !out || C0 <= 0 || C0 % V || C1 < 0 || C1 % V || (C1 > 0 && !src1) || B <= 0 || HW <= 0 ||
      (!scale) != (!shift) || C > 4096)
    return SNRSE_EINVAL;
  const int LP = C / V;
  int ppb = (8 * 256) / LP;  // ~8 vectors per thread
  if (ppb < 1) ppb = 1;
  dim3 grid((HW + ppb - 1) / ppb, B);
  if (dtype == SNRSE_F16)
    hipLaunchKernelGGL(gn_act_kernel<f16_t>, grid, dim3(256), sizeof(float) * 2 * C, stream, (const f16_t*)src0, C0,
                       (const f16_t*)src1, C1, HW, ppb, scale, shift, act, (f16_t*)out);
  else if (dtype == SNRSE_BF16)
    hipLaunchKernelGGL(gn_act_kernel<bf16_t>, grid, dim3(256), sizeof(float) * 2 * C, stream, (const bf16_t*)src0, C0,
                       (const bf16_t*)src1, C1, HW, ppb, scale, shift, act, (bf16_t*)out);
  else
    hipLaunchKernelGGL(gn_act_kernel<float>, grid, dim3(256), sizeof(float) * 2 * C, stream, (const float*)src0, C0,
                       (const float*)src1, C1, HW, ppb, scale, shift, act, (float*)out);
  return (int)hipGetLastError();
}
