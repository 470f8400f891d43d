// v8 halo GEMM: 8-wave ping-pong, fully LDS-DMA-fed 3x3 convolution with the fused GroupNorm(+SiLU)
// prologue, bias / temb / residual epilogue and GroupNorm statistics, for the NCSN++ ResBlock convs
// without a fused 1x1 shortcut or Combine term (reference: layerspp.py:244-276 -> layers.py:100-124).
//
// Structure (the "256^2 8-phase template" of cdna_hip_programming.md, adapted to the implicit GEMM):
//   tile    = 8 image rows x 64 px x 128 couts; wave w (0..7) owns image row h0 + w: 64 px x 128 co
//             = acc[2][4][4] of 16x16x32 MFMAs with A = weights, B = halo pixels (D[co][px])
//   phase   = one tap of one 32-channel K chunk: an L section (12 fragment ds_reads, one 1-KB weight
//             LDS-DMA piece for three phases ahead, at taps 0..2 two pieces of the next chunk's halo,
//             at taps 5..8 the in-place GroupNorm(+SiLU) of that halo), a barrier, an M section
//             (32 MFMAs), a barrier.  Waves 4..7 run one barrier behind waves 0..3, so on every SIMD
//             one wave's L section runs beside the other wave's MFMAs.
//   halo    = two buffers of (8+2) x (64+2) rows x 64 B (32 channels); row image hy * 66 + hx, 16-B
//             chunk swizzled by (hx >> 1) & 3: conflict-free for the ds_read_b128 lane groups of any
//             16 consecutive hx, and a tap's row shift is an immediate offset
//   weights = 4-slot ring of one-tap slices (128 co x 32 ch = 8 KB = one piece per wave)
//   persistent over contiguous tile ranges; the next tile's first chunk and first weight slices are
//             prefetched during the current tile's last chunk.
// Every wave issues the same vector-memory operations in every phase (one weight piece; + two halo
// / GroupNorm-affine pieces at taps 0..2 -- re-fetches where nothing is left to prefetch), so each
// in-loop wait is an exact counted vmcnt (k8_wait_vm).  Epilogue: the accumulators of channel
// blocks (2jp, 2jp+1) are exchanged between DPP rows (v_permlane16_swap), so every lane holds 8
// consecutive channels of one pixel: 16-B residual loads and 16-B stores.
#include <stdlib.h>

#include "conv_common.h"

namespace snrse_conv {
namespace {

constexpr int K8_TH = 8, K8_TW = 64, K8_HC = K8_TW + 2;
constexpr int K8_HROWS = (K8_TH + 2) * K8_HC;              // 660
constexpr int K8_NPIECE = 42;                              // 1-KB pieces per halo buffer (rows 660..671 pad)
constexpr int K8_HBUF = K8_NPIECE * 1024;                  // 43008
constexpr int K8_HROWB = K8_HC * 64;                       // 4224 bytes per halo image row
constexpr int K8_TAPB = 128 * 64;                          // one tap: 128 co x 32 ch bf16
constexpr int K8_NSLOT = 4;
constexpr int K8_MAXN = 4;                                 // Cout <= 512
constexpr int K8_OFF_W = 2 * K8_HBUF;                      // 86016
constexpr int K8_OFF_GN = K8_OFF_W + K8_NSLOT * K8_TAPB;   // [2 buffers][scale 32 | shift 32] f32
constexpr int K8_OFF_RED = K8_OFF_GN + 2 * 256;            // [K8_MAXN x 128 co][2] f32
constexpr int K8_LDS = K8_OFF_RED + K8_MAXN * 128 * 2 * 4;  // 123392 B: one workgroup per CU

SNRSE_DEV int k8_hswz(int hy, int hx, int chunk) { return hy * K8_HROWB + hx * 64 + ((chunk ^ ((hx >> 1) & 3)) << 4); }
SNRSE_DEV int k8_wswz(int co, int chunk) { return co * 64 + ((chunk ^ ((co >> 1) & 3)) << 4); }
SNRSE_DEV void k8_glds16(__amdgpu_buffer_rsrc_t r, char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}
SNRSE_DEV void k8_glds4(__amdgpu_buffer_rsrc_t r, char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 4, voff, 0, 0, 0);
}
// a value the compiler cannot see through: per-lane address math derived from it is redone where
// it is used instead of being hoisted into loop-invariant VGPRs
SNRSE_DEV int k8_opaque(int v) {
  int r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}
template <int CTRL>
SNRSE_DEV float k8_dpp(float v) {
  return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), CTRL, 0xf, 0xf, false));
}
// sum over the 16 lanes of a DPP row; every lane of the row receives it
SNRSE_DEV float k8_row_sum16(float v) {
  v += k8_dpp<0xB1>(v);   // quad_perm [1,0,3,2]
  v += k8_dpp<0x4E>(v);   // quad_perm [2,3,0,1]
  v += k8_dpp<0x141>(v);  // row_half_mirror
  v += k8_dpp<0x140>(v);  // row_mirror
  return v;
}
// the L section's closing wait: retire the weight slice the next phase reads (issued two phases
// before), and at tap 4 the halo pieces issued at taps 0..2 (the GroupNorm pass reads them from tap 5:
// an HBM-missing halo piece takes several phases to land)
template <int TP>
SNRSE_DEV void k8_wait_vm() {
  if constexpr (TP == 0) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else if constexpr (TP == 1 || TP == 3) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
  else if constexpr (TP == 2) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
}

struct Tile8 {
  int b, h0, w0, n0;
};

__global__ __launch_bounds__(512, 1) void conv_halo8_kernel(ConvParams p, int T, int stagger) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int grp = wid >> 2;
#ifdef SNRSE_STAMPS
  unsigned long long* const lst = (unsigned long long*)(smem + K8_LDS) + wid * 32;
#endif
  SNRSE_STAMP(0);
  const int G = gridDim.x, g = blockIdx.x;
  const int t_begin = (int)(((long long)g * T) / G);
  const int ntile = (int)(((long long)(g + 1) * T) / G) - t_begin;
  if (ntile <= 0) return;
  // odd workgroups start about half a tile late, so the CUs' epilogue store bursts do not coincide
  if (g & 1) {
    for (int i = 0; i < stagger; ++i) __builtin_amdgcn_s_sleep(127);
  }
  const int Cin = p.C0 + p.C1, ncm = Cin >> 5, K1 = 9 * Cin;
  const int ntw = p.W / K8_TW, nth = p.H / K8_TH;
  const bool has_gn = p.gn_scale != nullptr;
  const int lrow = lane & 15, lg = lane >> 4;
  float* const red = (float*)(smem + K8_OFF_RED);

  // tile order: N tile fastest (the Cout blocks of one pixel tile share its halo in L2), then
  // frames, rows, image
  auto tile_of = [&](int lt) {
    int t = t_begin + lt;
    Tile8 r;
    r.n0 = (t % p.ntn) * 128;
    t /= p.ntn;
    r.w0 = (t % ntw) * K8_TW;
    t /= ntw;
    r.h0 = (t % nth) * K8_TH;
    r.b = t / nth;
    return r;
  };

  // ---- part `part` (0..2) of the raw halo of chunk c of tile tl -> buffer hb: pieces wid + 8 m,
  // m = 2 part, 2 part + 1; m = 5 beyond the 42 pieces fetches the chunk's GroupNorm affine
  // (32 scales | 32 shifts; waves 2..7 fetch the same 256 bytes) -- two operations per wave
  auto halo_issue = [&](const Tile8 tl, int c, int hb, int part) {
    const int ln = k8_opaque(tid) & 63;
    const int ch = c * 32;
    const bool u1 = ch >= p.C0;
    const __amdgpu_buffer_rsrc_t r = u1 ? make_rsrc(p.src1, p.bytes1) : make_rsrc(p.src0, p.bytes0);
    const int cs = u1 ? p.C1 : p.C0, cc = u1 ? ch - p.C0 : ch;
    char* const dst = smem + hb * K8_HBUF;
#pragma unroll
    for (int mm = 0; mm < 2; ++mm) {
      const int m = 2 * part + mm;
      const int k = wid + 8 * m;
      if (k < K8_NPIECE) {
        const int row = k * 16 + (ln >> 2);
        const int hy = row / K8_HC, hx = row - hy * K8_HC;
        const int dc = (ln & 3) ^ ((hx >> 1) & 3);
        const unsigned ih = (unsigned)(tl.h0 + hy - 1), iw = (unsigned)(tl.w0 + hx - 1);
        const bool ok = row < K8_HROWS && ih < (unsigned)p.H && iw < (unsigned)p.W;
        const int voff = ok ? ((((tl.b * p.H + (int)ih) * p.W + (int)iw) * cs + cc + dc * 8) * 2) : (int)0x80000000;
        k8_glds16(r, dst + k * 1024, voff);
      } else {
        const __amdgpu_buffer_rsrc_t rg = has_gn ? make_rsrc(p.gn_scale, 8LL * p.B * Cin) : make_rsrc(p.out, 0);
        const int voff = has_gn ? (((ln < 32 ? tl.b : p.B + tl.b) * Cin + ch + (ln & 31)) * 4) : 0;
        k8_glds4(rg, smem + K8_OFF_GN + hb * 256, voff);
      }
    }
  };
  // ---- one tap's weights (128 co x 32 ch): this wave's 16 rows -> ring slot s
  auto w_issue = [&](const Tile8 tl, int c, int tp, int s) {
    const int ln = k8_opaque(tid) & 63;
    const int co = wid * 16 + (ln >> 2);
    const int dc = (ln & 3) ^ ((co >> 1) & 3);
    const __amdgpu_buffer_rsrc_t r = make_rsrc(p.wgt, p.wbytes);
    k8_glds16(r, smem + K8_OFF_W + s * K8_TAPB + wid * 1024, ((tl.n0 + co) * K1 + tp * Cin + c * 32 + dc * 8) * 2);
  };
  // ---- in-place GroupNorm(+SiLU) of halo row (tid >> 2) + 128 m (logical chunk tid & 3) of buffer hb;
  // rows outside the image stay zero (the zero padding of the activated tensor)
  auto trans_row = [&](const Tile8 tl, int hb, int m) {
    const int tq = k8_opaque(tid);
    const int row = (tq >> 2) + 128 * m;
    if (row < K8_HROWS) {
      const int hy = row / K8_HC, hx = row - hy * K8_HC;
      const int a = hb * K8_HBUF + k8_hswz(hy, hx, tq & 3);
      const unsigned ih = (unsigned)(tl.h0 + hy - 1), iw = (unsigned)(tl.w0 + hx - 1);
      const bool ok = ih < (unsigned)p.H && iw < (unsigned)p.W;
      const float* gt = (const float*)(smem + K8_OFF_GN + hb * 256) + (tq & 3) * 8;
      const f32x4 s0 = *(const f32x4*)gt, s1 = *(const f32x4*)(gt + 4);
      const f32x4 h0 = *(const f32x4*)(gt + 32), h1 = *(const f32x4*)(gt + 36);
      u32x4 v = *(const u32x4*)(smem + a);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float sl = i < 2 ? s0[2 * i] : s1[2 * i - 4], sh = i < 2 ? s0[2 * i + 1] : s1[2 * i - 3];
        const float hl = i < 2 ? h0[2 * i] : h1[2 * i - 4], hh = i < 2 ? h0[2 * i + 1] : h1[2 * i - 3];
        float lo = fmaf(__uint_as_float(v[i] << 16), sl, hl);
        float hi = fmaf(__uint_as_float(v[i] & 0xffff0000u), sh, hh);
        if (p.gn_act) {
          lo = silu(lo);
          hi = silu(hi);
        }
        v[i] = ok ? pack_bf16x2(lo, hi) : 0u;
      }
      *(u32x4*)(smem + a) = v;
    }
  };

  // per-lane fragment offsets: halo (buffer 0, top tap row, column dx; pixel block i adds i * 1024:
  // the swizzle of hx + 16 i equals that of hx) and weights (+ slot * K8_TAPB + j * 1024)
  int hoff[3];
#pragma unroll
  for (int dx = 0; dx < 3; ++dx) hoff[dx] = k8_hswz(wid, lrow + dx, lg);
  const int woff = K8_OFF_W + k8_wswz(lrow, lg);

  f32x4 acc[2][4][4];
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int i = tid; i < K8_MAXN * 256; i += 512) red[i] = 0.f;

  // ---- prologue: chunk 0 of the first tile (+ GroupNorm), weights of phases 0..2
  Tile8 tc = tile_of(0);
  halo_issue(tc, 0, 0, 0);
  halo_issue(tc, 0, 0, 1);
  halo_issue(tc, 0, 0, 2);
  w_issue(tc, 0, 0, 0);
  w_issue(tc, 0, 1, 1);
  w_issue(tc, 0, 2, 2);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  if (has_gn) {
#pragma unroll 1
    for (int m = 0; m < 6; ++m) trans_row(tc, 0, m);
  }
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  SNRSE_STAMP(1);
  if (grp == 1) __builtin_amdgcn_s_setprio(1);  // the second-dispatched half wins VALU arbitration

  int hb = 0, slot = 0;
  const int sslot = blockIdx.x & (SNRSE_STAT_SLOTS - 1);
  // true for the first two phases after the prologue / an epilogue: the weights they wait for were
  // drained before it, so they skip their vmcnt and do not wait on the epilogue's stores
  bool fresh = true;
#pragma unroll 1
  for (int lt = 0; lt < ntile; ++lt) {
    const bool has_nt = lt + 1 < ntile;
    const Tile8 tn = has_nt ? tile_of(lt + 1) : tc;
    if (grp == 1) __builtin_amdgcn_s_barrier();  // waves 4..7 run one barrier behind
#pragma unroll 1
    for (int c = 0; c < ncm; ++c) {
      const bool last_c = c + 1 == ncm;
      const bool has_next = !last_c || has_nt;
      const Tile8 tx = has_next ? (last_c ? tn : tc) : tc;  // owner of the prefetched chunk
      const int cx = has_next ? (last_c ? 0 : c + 1) : c;     // (re-fetch of this one past the end)
      const bool next_gn = has_gn && has_next;
      const int hbo = hb * K8_HBUF, hbn = hb ^ 1;
#if defined(SNRSE_STAMPS) && defined(SNRSE_STAMPS_PHASE)
#define K8_PSTAMP(I)                            \
  do {                                          \
    if (lt == 0 && c == 1 && tp_ < 6) SNRSE_STAMP(I); \
  } while (0)
#else
#define K8_PSTAMP(I) \
  do {               \
  } while (0)
#endif
#define K8_PHASE(TP)                                                                                         \
  do {                                                                                                       \
    constexpr int tp_ = (TP);                                                                                \
    K8_PSTAMP(2 + 4 * tp_);                                                                                  \
    u32x4 bh[4], aw[8];                                                                                      \
    _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                            \
      bh[i] = *(const u32x4*)(smem + hoff[tp_ % 3] + hbo + (tp_ / 3) * K8_HROWB + i * 1024);                         \
    const int wso = woff + slot * K8_TAPB;                                                                   \
    _Pragma("unroll") for (int j = 0; j < 8; ++j) aw[j] = *(const u32x4*)(smem + wso + j * 1024);             \
    if constexpr (tp_ + 3 < 9) w_issue(tc, c, tp_ + 3, (slot + 3) & 3);                                      \
    else if (has_next) w_issue(tx, cx, tp_ - 6, (slot + 3) & 3);                                             \
    else w_issue(tc, c, tp_, (slot + 3) & 3);                                                                \
    if constexpr (tp_ < 3) halo_issue(tx, cx, hbn, tp_);                                                     \
    if constexpr (tp_ >= 5) {                                                                                \
      if (next_gn) {                                                                                         \
        trans_row(tx, hbn, tp_ == 5 ? 0 : (tp_ == 6 ? 1 : 2 * tp_ - 12));                                     \
        if constexpr (tp_ >= 7) trans_row(tx, hbn, 2 * tp_ - 11);                                            \
      }                                                                                                      \
    }                                                                                                        \
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");                                                       \
    if (tp_ > 1 || !fresh) k8_wait_vm<tp_>();                                                                \
    K8_PSTAMP(3 + 4 * tp_);                                                                                  \
    __builtin_amdgcn_s_barrier();                                                                            \
    K8_PSTAMP(4 + 4 * tp_);                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                                       \
    _Pragma("unroll") for (int h = 0; h < 2; ++h)                                                            \
      _Pragma("unroll") for (int i = 0; i < 4; ++i)                                                          \
        _Pragma("unroll") for (int j = 0; j < 4; ++j)                                                        \
          acc[h][i][j] = mfma_chunk<bf16_t>(aw[h * 4 + j], bh[i], acc[h][i][j]);                              \
    __builtin_amdgcn_sched_barrier(0);                                                                       \
    K8_PSTAMP(5 + 4 * tp_);                                                                                  \
    __builtin_amdgcn_s_barrier();                                                                            \
    slot = (slot + 1) & 3;                                                                                   \
  } while (0)
      K8_PHASE(0);
      K8_PHASE(1);
      fresh = false;
      K8_PHASE(2);
      K8_PHASE(3);
      K8_PHASE(4);
      K8_PHASE(5);
      K8_PHASE(6);
      K8_PHASE(7);
      K8_PHASE(8);
#undef K8_PHASE
#undef K8_PSTAMP
      hb = hbn;
    }
    if (grp == 0) __builtin_amdgcn_s_barrier();  // re-align the two wave groups
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    fresh = true;
#if defined(SNRSE_STAMPS) && !defined(SNRSE_STAMPS_PHASE)
    if (lt < 13) SNRSE_STAMP(2 + 2 * lt);
#endif

    // ---- epilogue: exchange channel blocks (2jp, 2jp+1) between DPP rows (lg even <-> lg odd), so
    // lane (lrow, lg) holds channels cl .. cl+7, cl = 64 h + 16 (2 jp + (lg & 1)) + 8 (lg >> 1), of
    // pixel w0 + 16 i + lrow in image row h0 + wid
    {
      const size_t mrow = ((size_t)tc.b * p.H + tc.h0 + wid) * p.W + tc.w0 + lrow;
      const int nn = tc.n0 >> 7;
      // absent operands read through zero-size buffer resources (loads return 0): no branch around
      // a load, so hipcc batches them instead of waiting vmcnt(0) after each
      const __amdgpu_buffer_rsrc_t rbias = make_rsrc(p.bias ? (const void*)p.bias : p.out, p.bias ? 4LL * p.Cout : 0);
      const __amdgpu_buffer_rsrc_t rtemb =
          make_rsrc(p.temb ? (const void*)(p.temb + (size_t)tc.b * p.temb_stride) : p.out, p.temb ? 4LL * p.Cout : 0);
      const __amdgpu_buffer_rsrc_t rres =
          make_rsrc(p.res ? p.res : p.out, p.res ? 2LL * p.M * p.res_ld : 0);
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x4 add[2][2], s1[2][2], s2[2][2];
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const int cl = h * 64 + 16 * (2 * jp + (lg & 1)) + 8 * (lg >> 1);
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const int bo = (tc.n0 + cl + 4 * q) * 4;
            add[jp][q] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rbias, bo, 0, 0)) +
                         __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rtemb, bo, 0, 0));
            s1[jp][q] = f32x4{0.f, 0.f, 0.f, 0.f};
            s2[jp][q] = s1[jp][q];
          }
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const size_t m = mrow + 16 * i;
#pragma unroll
          for (int jp = 0; jp < 2; ++jp) {
            const int n = tc.n0 + h * 64 + 16 * (2 * jp + (lg & 1)) + 8 * (lg >> 1);
            f32x4 a = acc[h][i][2 * jp], bq = acc[h][i][2 * jp + 1];
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a[e]), __float_as_uint(bq[e]), false, false);
              a[e] = __uint_as_float(r[0]);
              bq[e] = __uint_as_float(r[1]);
            }
            f32x4 v0 = a + add[jp][0], v1 = bq + add[jp][1];
            {
              const u32x4 rv = __builtin_amdgcn_raw_buffer_load_b128(rres, (int)((m * p.res_ld + n) * 2), 0, 0);
              v0[0] += __uint_as_float(rv[0] << 16);
              v0[1] += __uint_as_float(rv[0] & 0xffff0000u);
              v0[2] += __uint_as_float(rv[1] << 16);
              v0[3] += __uint_as_float(rv[1] & 0xffff0000u);
              v1[0] += __uint_as_float(rv[2] << 16);
              v1[1] += __uint_as_float(rv[2] & 0xffff0000u);
              v1[2] += __uint_as_float(rv[3] << 16);
              v1[3] += __uint_as_float(rv[3] & 0xffff0000u);
            }
            v0 *= p.out_scale;
            v1 *= p.out_scale;
            const u32x4 o = {pack_bf16x2(v0[0], v0[1]), pack_bf16x2(v0[2], v0[3]), pack_bf16x2(v1[0], v1[1]),
                             pack_bf16x2(v1[2], v1[3])};
            *(u32x4*)((bf16_t*)p.out + m * p.out_ld + n) = o;
            s1[jp][0] += v0;
            s1[jp][1] += v1;
            s2[jp][0] += v0 * v0;
            s2[jp][1] += v1 * v1;
          }
        }
        if (p.stats) {
#pragma unroll
          for (int jp = 0; jp < 2; ++jp) {
            const int cl = h * 64 + 16 * (2 * jp + (lg & 1)) + 8 * (lg >> 1);
#pragma unroll
            for (int q = 0; q < 2; ++q)
#pragma unroll
              for (int e = 0; e < 4; ++e) {
                const float a = k8_row_sum16(s1[jp][q][e]), a2 = k8_row_sum16(s2[jp][q][e]);
                if (lrow == 0) {
                  atomicAdd(&red[(nn * 128 + cl + 4 * q + e) * 2], a);
                  atomicAdd(&red[(nn * 128 + cl + 4 * q + e) * 2 + 1], a2);
                }
              }
          }
        }
      }
    }
    // GroupNorm statistics of an image leave once, when the workgroup moves past it
    if (p.stats && (!has_nt || tn.b != tc.b)) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      for (int i = tid; i < p.ntn * 256; i += 512) {
        const float a = red[i];
        red[i] = 0.f;
        unsafeAtomicAdd(&p.stats[stat_idx(tc.b, sslot, i >> 1, p.Cout) + (i & 1)], (double)a);
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
    }
#if defined(SNRSE_STAMPS) && !defined(SNRSE_STAMPS_PHASE)
    if (lt < 13) SNRSE_STAMP(3 + 2 * lt);
#endif
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    tc = tn;
  }
  SNRSE_STAMP(28);
#ifdef SNRSE_STAMPS
  {
    unsigned long long st_[29];
    if (lane == 0)
      for (int i = 0; i < 29; ++i) st_[i] = lst[i];
    unsigned long long t_end;
    asm volatile("s_waitcnt vmcnt(0)\n\ts_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_end)::"memory");
    unsigned hw, xcc;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    if (lane == 0 && p.stamps) {
      unsigned long long* gs = p.stamps + ((size_t)blockIdx.x * 8 + wid) * 32;
      for (int i = 0; i < 29; ++i) gs[i] = st_[i];
      gs[29] = t_end;
      gs[30] = hw;
      gs[31] = xcc;
    }
  }
#endif
}

}  // namespace

bool halo8_ok(const ConvParams& p) {
  const int Cin = p.C0 + p.C1;
  if (p.ksize != 3 || p.H % K8_TH || p.W % K8_TW || p.Cout % 128 || p.Cout > 128 * K8_MAXN || p.B <= 0) return false;
  if (p.C0 % 32 || p.C1 % 32 || Cin <= 0) return false;
  if (p.sc_src || p.comb_src) return false;  // shortcut / Combine convs stay on v5
  if (p.out_ld % 8 || (p.res && p.res_ld % 8)) return false;
  if (p.bias && ((uintptr_t)p.bias & 15)) return false;
  if (p.temb && (((uintptr_t)p.temb & 15) || p.temb_stride % 4)) return false;
  if (p.gn_scale && p.gn_shift != p.gn_scale + (size_t)p.B * Cin) return false;  // one resource for both
  const long long lim = 0x7ff00000ll;
  if (p.bytes0 >= lim || p.bytes1 >= lim || p.wbytes >= lim || 8LL * p.B * Cin >= lim) return false;
  return true;
}

int launch_halo8(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  if (!halo8_ok(p)) return SNRSE_EINVAL;
  p.ntn = p.Cout / 128;
  const int T = p.B * (p.H / K8_TH) * (p.W / K8_TW) * p.ntn;
#ifdef SNRSE_STAMPS
  constexpr size_t lds = K8_LDS + 8 * 32 * 8;
#else
  constexpr size_t lds = K8_LDS;
#endif
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    SNRSE_RET(hipGetDevice(&dev));
    SNRSE_RET(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    SNRSE_RET(hipFuncSetAttribute((const void*)conv_halo8_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
  }
  const int G = T < ncu ? T : ncu;
  // half a tile (~1.3k cycles per phase, 9 phases per 32-channel chunk, ~17k epilogue; s_sleep 127
  // ~8k cycles) when every workgroup runs enough tiles to amortise it; SNRSE_K8_STAGGER=0 disables
  static const int stagger_on = getenv("SNRSE_K8_STAGGER") ? atoi(getenv("SNRSE_K8_STAGGER")) : 1;
  const int ncm = (p.C0 + p.C1) / 32;
  const int stagger = (stagger_on && T >= 8 * G) ? (ncm * 9 * 1300 + 17000) / 2 / 8128 : 0;
  hipLaunchKernelGGL(conv_halo8_kernel, dim3(G), dim3(512), lds, s, p, T, stagger);
  return (int)hipGetLastError();
}

}  // namespace snrse_conv
