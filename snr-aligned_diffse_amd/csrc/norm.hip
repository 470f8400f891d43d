// GroupNorm statistics, fused GroupNorm-apply + SiLU + FIR up/down-sampling, and the
// generic upfirdn2d entry (gfx950).
//
// Reference ops replaced:
//   nn.GroupNorm(min(C//4,32), C, eps=1e-6)   layerspp.py:221,233,69; ncsnpp.py:210-211,222-223
//   act = nn.SiLU                             layers.py:38-39
//   upsample_2d / downsample_2d (FIR [1,3,3,1]) up_or_down_sampling.py:195-257
//   upfirdn2d (CUDA kernel + pybind)          op/upfirdn2d.py:145-156, upfirdn2d_kernel.cu:107-369
// In a BigGAN ResBlock the order is SiLU(GN(x)) then FIR, with zero padding of the
// activated tensor (layerspp.py:245-257), so the fused kernel activates every tap first.
//
// Statistics: per-channel (sum, sum of squares) accumulated in double by global atomics
// from per-block LDS partials; the apply kernel folds them into per-group mean / rstd and
// per-(b, c) scale / shift.
#include "common.h"

#include <algorithm>

namespace {

template <typename T> struct VecT;
template <> struct VecT<bf16_t> { static constexpr int N = 8; };
template <> struct VecT<f16_t> { static constexpr int N = 8; };
template <> struct VecT<float> { static constexpr int N = 4; };

template <typename T>
SNRSE_DEV void load_vec(const T* p, float* v) {
  const u32x4 r = *(const u32x4*)p;
  if constexpr (sizeof(T) == 2) {
    unpack8<T>(r, v);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = __uint_as_float(r[i]);
  }
}

template <typename T>
SNRSE_DEV void store_vec(T* p, const float* v) {
  u32x4 r;
  if constexpr (sizeof(T) == 2) {
    r = pack8<T>(v);
  } else {
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = __float_as_uint(v[i]);
  }
  *(u32x4*)p = r;
}

// grid (nblk, B), block 256.  sums0 [B][SLOTS][C0][2], sums1 [B][SLOTS][C1][2] double, zeroed by the launcher.
template <typename T>
__global__ __launch_bounds__(256) void gn_stats_kernel(const T* src0, int C0, const T* src1, int C1,
                                                       int HW, int pix_per_blk, double* sums0, double* sums1) {
  constexpr int V = VecT<T>::N;
  const int C = C0 + C1;
  const int LP = C / V;        // vectors per pixel
  const int PY = 256 / LP;     // pixel rows per pass (LP <= 256)
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  extern __shared__ __attribute__((aligned(16))) float red[];  // [C][2]
  for (int i = tid; i < 2 * C; i += 256) red[i] = 0.f;
  __syncthreads();
  const int v = tid % LP, py = tid / LP;
  if (py < PY) {
    const int c = v * V;
    const T* src;
    int cs, cc;
    if (c < C0) { src = src0; cs = C0; cc = c; } else { src = src1; cs = C1; cc = c - C0; }
    float s[V], ss[V];
#pragma unroll
    for (int i = 0; i < V; ++i) { s[i] = 0.f; ss[i] = 0.f; }
    const int p0 = blockIdx.x * pix_per_blk;
    const int p1 = min(HW, p0 + pix_per_blk);
    for (int pix = p0 + py; pix < p1; pix += PY) {
      float x[V];
      load_vec<T>(src + ((size_t)b * HW + pix) * cs + cc, x);
#pragma unroll
      for (int i = 0; i < V; ++i) { s[i] += x[i]; ss[i] = fmaf(x[i], x[i], ss[i]); }
    }
#pragma unroll
    for (int i = 0; i < V; ++i) {
      atomicAdd(&red[2 * (c + i)], s[i]);
      atomicAdd(&red[2 * (c + i) + 1], ss[i]);
    }
  }
  __syncthreads();
  for (int i = tid; i < 2 * C; i += 256) {
    const int c = i >> 1;
    const int slot = blockIdx.x & (SNRSE_STAT_SLOTS - 1);
    if (c < C0) unsafeAtomicAdd(&sums0[stat_idx(b, slot, c, C0) + (i & 1)], (double)red[i]);
    else unsafeAtomicAdd(&sums1[stat_idx(b, slot, c - C0, C1) + (i & 1)], (double)red[i]);
  }
}

enum { MODE_NONE = 0, MODE_DOWN = 1, MODE_UP = 2 };

// Output pixel grid (Ho, Wo); block (256) covers `opix_per_blk` output pixels of batch b.
// scale/shift per channel computed in the prologue (gn) or identity (!gn).
template <typename Tin, typename Tout, int MODE>
__global__ __launch_bounds__(256) void gn_apply_kernel(const Tin* src0, int C0, const Tin* src1, int C1,
                                                       int H, int W, const double* sums,
                                                       const double* sums1, const float* gamma,
                                                       const float* beta, int groups,
                                                       float eps, int act, Tout* out, int opix_per_blk, int csl) {
  constexpr int V = VecT<Tin>::N;
  static_assert(VecT<Tin>::N == VecT<Tout>::N || sizeof(Tout) == 4, "vec");
  const int C = C0 + C1;
  const int b = blockIdx.y;
  const int tid = threadIdx.x;
  // csl > 0 (MODE_NONE, same-size output): this block owns channels [cs0, cs0 + csl) -- whole GroupNorm groups
  // inside one source -- of its pixel range, so it folds only their statistics (blockIdx.x = range * nsl + slice)
  const int nsl = csl > 0 ? C / csl : 1;
  const int cs0 = csl > 0 ? (blockIdx.x % nsl) * csl : 0, cs1 = csl > 0 ? cs0 + csl : C;
  const int bx = csl > 0 ? blockIdx.x / nsl : blockIdx.x;
  extern __shared__ __attribute__((aligned(16))) double gap_red[];  // [C][2] folded channel sums, then scale / shift
  double* const red = gap_red;
  float* const sc = (float*)(red + 2 * C);                         // scale[C], shift[C]
  if (sums) {
    // per channel: the SNRSE_STAT_SLOTS partial sums (independent 16-B loads), then per group from LDS
    for (int c = cs0 + tid; c < cs1; c += 256) {
      const double* st = c < C0 ? sums + stat_idx(b, 0, c, C0) : sums1 + stat_idx(b, 0, c - C0, C1);
      const size_t sstride = 2 * (size_t)(c < C0 ? C0 : C1);
      double s = 0.0, ss = 0.0;
#pragma unroll
      for (int k = 0; k < SNRSE_STAT_SLOTS; ++k) {
        s += st[k * sstride];
        ss += st[k * sstride + 1];
      }
      red[2 * c] = s;
      red[2 * c + 1] = ss;
    }
    __syncthreads();
    const int cg = C / groups;
    const double cnt = (double)cg * H * W;
    for (int c = cs0 + tid; c < cs1; c += 256) {
      const int g = c / cg;
      double s = 0.0, ss = 0.0;
      for (int k = g * cg; k < (g + 1) * cg; ++k) {
        s += red[2 * k];
        ss += red[2 * k + 1];
      }
      const double mean = s / cnt;
      double var = ss / cnt - mean * mean;
      if (var < 0.0) var = 0.0;
      const float rstd = (float)(1.0 / sqrt(var + (double)eps));
      const float scl = rstd * gamma[c];
      sc[c] = scl;
      sc[C + c] = beta[c] - (float)mean * scl;
    }
  } else {
    for (int c = tid; c < C; c += 256) { sc[c] = 1.f; sc[C + c] = 0.f; }
  }
  __syncthreads();
  const int Ho = MODE == MODE_DOWN ? H / 2 : (MODE == MODE_UP ? 2 * H : H);
  const int Wo = MODE == MODE_DOWN ? W / 2 : (MODE == MODE_UP ? 2 * W : W);
  const int LP = C / V;
  const int total = opix_per_blk * LP;
  const int op0 = bx * opix_per_blk;
  if constexpr (MODE == MODE_NONE && sizeof(Tout) == sizeof(Tin)) {
    // elementwise: UNR vectors' loads in flight before any is transformed (a load-use chain per vector held
    // the small-level GroupNorm launches at ~13 us); 16-bit takes the fast SiLU as gn_act does, fp32 the exact one
    constexpr int UNR = 4;
    const int HWo = Ho * Wo;
    const int LS = (cs1 - cs0) / V;  // vectors per pixel in this block's slice
    const int tot = min(opix_per_blk, HWo - op0) * LS;
    for (int base = tid; base < tot; base += 256 * UNR) {
      u32x4 raw[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int idx = base + 256 * u;
        if (idx < tot) {
          const int op = op0 + idx / LS, c = cs0 + (idx % LS) * V;
          raw[u] = *(const u32x4*)(c < C0 ? src0 + ((size_t)b * HWo + op) * C0 + c
                                          : src1 + ((size_t)b * HWo + op) * C1 + (c - C0));
        }
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int idx = base + 256 * u;
        if (idx < tot) {
          const int op = op0 + idx / LS, c = cs0 + (idx % LS) * V;
          float x[V];
          if constexpr (sizeof(Tin) == 2) {
            unpack8<Tin>(raw[u], x);
          } else {
#pragma unroll
            for (int i = 0; i < 4; ++i) x[i] = __uint_as_float(raw[u][i]);
          }
#pragma unroll
          for (int i = 0; i < V; ++i) {
            const float y = fmaf(x[i], sc[c + i], sc[C + c + i]);
            x[i] = act ? (sizeof(Tin) == 2 ? silu(y) : silu_exact(y)) : y;
          }
          store_vec<Tout>(out + ((size_t)b * HWo + op) * C + c, x);
        }
      }
    }
    return;
  }
  for (int idx = tid; idx < total; idx += 256) {
    const int op = op0 + idx / LP;
    if (op >= Ho * Wo) break;
    const int v = idx % LP;
    const int c = v * V;
    const Tin* src;
    int cs, cc;
    if (c < C0) { src = src0; cs = C0; cc = c; } else { src = src1; cs = C1; cc = c - C0; }
    float scl[V], sh[V];
#pragma unroll
    for (int i = 0; i < V; ++i) { scl[i] = sc[c + i]; sh[i] = sc[C + c + i]; }
    const int oy = op / Wo, ox = op - (op / Wo) * Wo;
    float o[V];
#pragma unroll
    for (int i = 0; i < V; ++i) o[i] = 0.f;
    auto tap = [&](int iy, int ix, float wgt) {
      if (iy < 0 || iy >= H || ix < 0 || ix >= W) return;
      float x[V];
      load_vec<Tin>(src + ((size_t)(b * H + iy) * W + ix) * cs + cc, x);
#pragma unroll
      for (int i = 0; i < V; ++i) {
        float y = fmaf(x[i], scl[i], sh[i]);
        if (act) y = silu_exact(y);
        o[i] = fmaf(y, wgt, o[i]);
      }
    };
    if (MODE == MODE_NONE) {
      tap(oy, ox, 1.f);
    } else if (MODE == MODE_DOWN) {
      // out[i] = sum_a k[a] x[2i + a - 1], k = [1,3,3,1]/8 per axis
      const float k1[4] = {0.125f, 0.375f, 0.375f, 0.125f};
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int bb = 0; bb < 4; ++bb) tap(2 * oy + a - 1, 2 * ox + bb - 1, k1[a] * k1[bb]);
    } else {
      // out[2q] = (x[q-1] + 3 x[q]) / 4, out[2q+1] = (3 x[q] + x[q+1]) / 4 per axis
      const int qy = oy >> 1, qx = ox >> 1;
      const int y0 = (oy & 1) ? qy : qy - 1, x0 = (ox & 1) ? qx : qx - 1;
      const float wy0 = (oy & 1) ? 0.75f : 0.25f, wx0 = (ox & 1) ? 0.75f : 0.25f;
      tap(y0, x0, wy0 * wx0);
      tap(y0, x0 + 1, wy0 * (1.f - wx0));
      tap(y0 + 1, x0, (1.f - wy0) * wx0);
      tap(y0 + 1, x0 + 1, (1.f - wy0) * (1.f - wx0));
    }
    Tout* dst = out + ((size_t)b * Ho * Wo + op) * C + c;
    if constexpr (sizeof(Tout) == sizeof(Tin)) {
      store_vec<Tout>(dst, o);
    } else {
#pragma unroll
      for (int i = 0; i < V; ++i) dst[i] = Elem<Tout>::from_f(o[i]);
    }
  }
}

// Generic upfirdn2d on [major, in_h, in_w, minor] (the reference op's layout):
// out[y, x] = sum_{i,j} k[kh-1-i][kw-1-j] * up_pad(in)[y*dy + i][x*dx + j]
// Element types of the reference binding (AT_DISPATCH_FLOATING_TYPES_AND_HALF, upfirdn2d_kernel.cu:311)
// plus bf16: f32 / bf16 / f16 accumulate in f32, f64 in f64.
SNRSE_DEV float ufd_ld(float v) { return v; }
SNRSE_DEV float ufd_ld(bf16_t v) { return bf2f(v); }
SNRSE_DEV float ufd_ld(_Float16 v) { return (float)v; }
SNRSE_DEV double ufd_ld(double v) { return v; }
template <typename T> SNRSE_DEV T ufd_st(float v) { return (T)v; }
template <> SNRSE_DEV bf16_t ufd_st<bf16_t>(float v) { return f2bf(v); }
template <typename T> SNRSE_DEV T ufd_st(double v) { return (T)v; }

template <typename T, typename A>
__global__ void upfirdn2d_kernel(const T* in, T* out, const float* kern, int major, int in_h, int in_w,
                                 int minor, int kh, int kw, int up_x, int up_y, int down_x, int down_y,
                                 int pad_x0, int pad_y0, int out_h, int out_w) {
  const size_t total = (size_t)major * out_h * out_w * minor;
  for (size_t idx = blockIdx.x * (size_t)blockDim.x + threadIdx.x; idx < total;
       idx += (size_t)gridDim.x * blockDim.x) {
    const int mi = idx % minor;
    size_t r = idx / minor;
    const int ox = r % out_w; r /= out_w;
    const int oy = r % out_h;
    const int mj = (int)(r / out_h);
    A acc = 0;
    for (int i = 0; i < kh; ++i) {
      const int uy = oy * down_y + i - pad_y0;  // coordinate in the upsampled grid
      if (uy < 0 || uy % up_y) continue;
      const int iy = uy / up_y;
      if (iy >= in_h) continue;
      for (int j = 0; j < kw; ++j) {
        const int ux = ox * down_x + j - pad_x0;
        if (ux < 0 || ux % up_x) continue;
        const int ix = ux / up_x;
        if (ix >= in_w) continue;
        acc += (A)kern[(kh - 1 - i) * kw + (kw - 1 - j)] * (A)ufd_ld(in[(((size_t)mj * in_h + iy) * in_w + ix) * minor + mi]);
      }
    }
    out[idx] = ufd_st<T>(acc);
  }
}

// scale[b][c] = gamma[c] * rstd(b, g(c)), shift[b][c] = beta[c] - mean(b, g(c)) * scale[b][c].
// One wave per (b, group): the group's cg channels x SNRSE_STAT_SLOTS slotted partial sums are
// folded across the lanes (a per-channel sequential fold took ~10 us per launch at ~100 launches
// per network evaluation).
__global__ __launch_bounds__(64) void gn_scale_shift_kernel(const double* sums0, int C0, const double* sums1, int C1,
                                                            int HW, const float* gamma, const float* beta,
                                                            int groups, float eps, float* scale, float* shift) {
  const int b = blockIdx.x, g = blockIdx.y, lane = threadIdx.x;
  const int C = C0 + C1, cg = C / groups;
  const int n = cg * SNRSE_STAT_SLOTS;
  double s = 0.0, ss = 0.0;
  for (int i = lane; i < n; i += 64) {
    const int k = g * cg + i / SNRSE_STAT_SLOTS, slot = i % SNRSE_STAT_SLOTS;
    const double* q = k < C0 ? sums0 + stat_idx(b, slot, k, C0) : sums1 + stat_idx(b, slot, k - C0, C1);
    s += q[0];
    ss += q[1];
  }
  s = wave_sum_d(s);
  ss = wave_sum_d(ss);
  const double cnt = (double)cg * HW;
  const double mean = s / cnt;
  double var = ss / cnt - mean * mean;
  if (var < 0.0) var = 0.0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  for (int j = lane; j < cg; j += 64) {
    const int c = g * cg + j;
    const float scl = rstd * gamma[c];
    scale[(size_t)b * C + c] = scl;
    shift[(size_t)b * C + c] = beta[c] - (float)mean * scl;
  }
}

}  // namespace

extern "C" int snrse_gn_scale_shift(const double* sums0, int C0, const double* sums1, int C1, int B, int HW,
                                    const float* gamma, const float* beta, int groups, float eps, float* scale,
                                    float* shift, hipStream_t stream) {
  if (!sums0 || (C1 > 0 && !sums1) || groups <= 0 || (C0 + C1) % groups || B <= 0) return SNRSE_EINVAL;
  hipLaunchKernelGGL(gn_scale_shift_kernel, dim3(B, groups), dim3(64), 0, stream, sums0, C0, sums1, C1, HW, gamma,
                     beta, groups, eps, scale, shift);
  return (int)hipGetLastError();
}

extern "C" int snrse_gn_stats(snrse_ctx* ctx, const void* src0, int C0, const void* src1, int C1, int B, int HW,
                              double* sums, double* sums1, int dtype, hipStream_t stream) {
  const int V = snrse_is16(dtype) ? 8 : 4;
  const int C = C0 + C1;
  if (C % V || C0 % V || C / V > 256 || !sums || (C1 > 0 && !sums1)) return SNRSE_EINVAL;
  const bool zeroed = snrse_ctx_resolve(ctx)->stats_zeroed != 0;
  if (!zeroed) SNRSE_RET(hipMemsetAsync(sums, 0, sizeof(double) * 2 * SNRSE_STAT_SLOTS * C0 * B, stream));
  if (C1 > 0 && !zeroed) SNRSE_RET(hipMemsetAsync(sums1, 0, sizeof(double) * 2 * SNRSE_STAT_SLOTS * C1 * B, stream));
  int nblk = (HW + 1023) / 1024;
  if (nblk > 256) nblk = 256;
  const int ppb = (HW + nblk - 1) / nblk;
  dim3 grid(nblk, B);
  const size_t lds = sizeof(float) * 2 * C;
  if (dtype == SNRSE_F16)
    hipLaunchKernelGGL(gn_stats_kernel<f16_t>, grid, dim3(256), lds, stream, (const f16_t*)src0, C0,
                       (const f16_t*)src1, C1, HW, ppb, sums, sums1);
  else if (dtype == SNRSE_BF16)
    hipLaunchKernelGGL(gn_stats_kernel<bf16_t>, grid, dim3(256), lds, stream, (const bf16_t*)src0, C0,
                       (const bf16_t*)src1, C1, HW, ppb, sums, sums1);
  else if (dtype == SNRSE_F32)
    hipLaunchKernelGGL(gn_stats_kernel<float>, grid, dim3(256), lds, stream, (const float*)src0, C0,
                       (const float*)src1, C1, HW, ppb, sums, sums1);
  else
    return SNRSE_EINVAL;
  return (int)hipGetLastError();
}

template <typename Tin, typename Tout>
static int launch_apply(const void* src0, int C0, const void* src1, int C1, int B, int H, int W,
                        const double* sums, const double* sums1, const float* gamma, const float* beta, int groups, float eps,
                        int act, int mode, void* out, hipStream_t stream) {
  const bool slice = snrse_ctx_resolve(nullptr)->gn_slice != 0;  // (the process default context's switch)
  const int C = C0 + C1;
  const int Ho = mode == MODE_DOWN ? H / 2 : (mode == MODE_UP ? 2 * H : H);
  const int Wo = mode == MODE_DOWN ? W / 2 : (mode == MODE_UP ? 2 * W : W);
  const int V = VecT<Tin>::N;
  const int LP = C / V;
  // one 16-B output vector per thread: the 4-channel pyramid FIRs (ncsnpp.py:318, 359) ran 4 pixels x 16 taps
  // per thread at 1024 px per block (up to 35 us per launch at 0.3 of HBM, profiles/r05a_c2_dispatch_shapes.jsonl).
  // With a GroupNorm every block folds its image's statistics first: at most 16 blocks per image then (the small
  // levels, where one launch replaces gn_scale_shift + gn_act; snrse/ops.py gn_apply)
  int opb = 256 / LP;
  if (opb < 1) opb = 1;
  if (sums) opb = std::max(opb, std::min((Ho * Wo + 15) / 16, 16 * 256 / LP));  // <= 16 folds per image, 16 vectors per thread
  int nblk = (Ho * Wo + opb - 1) / opb, csl = 0;
  // the same blocks as 64-channel slices x pixel ranges where a slice holds whole groups of one source: each
  // block folds C / 64 times fewer statistics (16 slots x 16 B per channel, 64 KB per block at C = 256 -- the
  // fold, not the image, was the small-level launch's traffic)
  constexpr int kSl = 64;
  if (slice && sums && mode == MODE_NONE && C > kSl && C % kSl == 0 && C0 % kSl == 0 && (C / groups) <= kSl &&
      kSl % (C / groups) == 0) {
    const int nsl = C / kSl;
    const int npr = std::max(1, nblk / nsl);
    opb = (Ho * Wo + npr - 1) / npr;
    nblk = ((Ho * Wo + opb - 1) / opb) * nsl;
    csl = kSl;
  }
  dim3 grid(nblk, B);
  const size_t lds = sizeof(double) * 2 * C + sizeof(float) * 2 * C;
#define SNRSE_APPLY(MODE_)                                                                          \
  hipLaunchKernelGGL((gn_apply_kernel<Tin, Tout, MODE_>), grid, dim3(256), lds, stream, (const Tin*)src0, \
                     C0, (const Tin*)src1, C1, H, W, sums, sums1, gamma, beta, groups, eps, act, (Tout*)out, opb, csl)
  if (mode == MODE_NONE) SNRSE_APPLY(MODE_NONE);
  else if (mode == MODE_DOWN) SNRSE_APPLY(MODE_DOWN);
  else if (mode == MODE_UP) SNRSE_APPLY(MODE_UP);
  else return SNRSE_EINVAL;
#undef SNRSE_APPLY
  return (int)hipGetLastError();
}

extern "C" int snrse_gn_apply(const void* src0, int C0, const void* src1, int C1, int B, int H, int W,
                              const double* sums, const double* sums1, const float* gamma, const float* beta,
                              int groups,
                              float eps, int act, int mode, void* out, int dtype, hipStream_t stream) {
  const int V = snrse_is16(dtype) ? 8 : 4;
  if ((C0 + C1) % V || C0 % V) return SNRSE_EINVAL;
  if (sums && (!gamma || !beta || groups <= 0 || (C0 + C1) % groups || (C1 > 0 && !sums1))) return SNRSE_EINVAL;
  if (mode == MODE_DOWN && ((H & 1) || (W & 1))) return SNRSE_EINVAL;
  if (dtype == SNRSE_F16)
    return launch_apply<f16_t, f16_t>(src0, C0, src1, C1, B, H, W, sums, sums1, gamma, beta, groups, eps, act,
                                      mode, out, stream);
  if (dtype == SNRSE_BF16)
    return launch_apply<bf16_t, bf16_t>(src0, C0, src1, C1, B, H, W, sums, sums1, gamma, beta, groups, eps, act,
                                        mode, out, stream);
  if (dtype == SNRSE_F32)
    return launch_apply<float, float>(src0, C0, src1, C1, B, H, W, sums, sums1, gamma, beta, groups, eps, act,
                                      mode, out, stream);
  return SNRSE_EINVAL;
}

extern "C" int snrse_upfirdn2d(const void* in, void* out, const float* kernel, int major, int in_h,
                               int in_w, int minor, int kh, int kw, int up_x, int up_y, int down_x,
                               int down_y, int pad_x0, int pad_x1, int pad_y0, int pad_y1, int dtype,
                               hipStream_t stream) {
  if (up_x < 1 || up_y < 1 || down_x < 1 || down_y < 1 || kh < 1 || kw < 1) return SNRSE_EINVAL;
  const int out_h = (in_h * up_y + pad_y0 + pad_y1 - kh) / down_y + 1;
  const int out_w = (in_w * up_x + pad_x0 + pad_x1 - kw) / down_x + 1;
  if (out_h <= 0 || out_w <= 0) return SNRSE_EINVAL;
  const size_t total = (size_t)major * out_h * out_w * minor;
  int blocks = (int)((total + 255) / 256);
  if (blocks > 65536) blocks = 65536;
#define SNRSE_UFD(T, A)                                                                                      \
  hipLaunchKernelGGL((upfirdn2d_kernel<T, A>), dim3(blocks), dim3(256), 0, stream, (const T*)in, (T*)out, kernel, \
                     major, in_h, in_w, minor, kh, kw, up_x, up_y, down_x, down_y, pad_x0, pad_y0, out_h, out_w)
  if (dtype == SNRSE_F32) SNRSE_UFD(float, float);
  else if (dtype == SNRSE_BF16) SNRSE_UFD(bf16_t, float);
  else if (dtype == SNRSE_F16) SNRSE_UFD(_Float16, float);
  else if (dtype == SNRSE_F64) SNRSE_UFD(double, double);
  else return SNRSE_EINVAL;
#undef SNRSE_UFD
  return (int)hipGetLastError();
}
