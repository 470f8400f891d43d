// v7 halo GEMM: the 3x3 convolutions of the NCSN++ ResBlocks (layerspp.py:244-276 Conv_0 / Conv_1
// [+ Conv_2 shortcut], ddpm_conv3x3 layers.py:100-124) with the GroupNorm(+SiLU) prologue fused,
// bf16 operands, f32 accumulation, bf16 output (gfx950).
//
// Same work decomposition as v5 (conv.hip): two 256-thread workgroups per CU, tile = 4 image rows x
// 64 px x 128 output channels, wave w computes image row h0 + w (64 px x 128 co, 128 accumulator
// VGPRs), K in 32-channel chunks, weights streamed by LDS-DMA as 3-tap phases into a 2-slot ring.
// What changes is the per-MFMA issue overhead, which PMC showed to be the limiter of v5 (3.9 VALU +
// 2.1 SALU per MFMA, half the MFMA pipe idle; profiles/r02b_*):
//   * halo image chunk-planar, [chunk][400 rows][16 B]: a fragment read (16 consecutive rows of one
//     chunk per lane group) is bank-conflict-free for ANY starting row, so every tap's A-fragment
//     address is the lane's base + a compile-time offset (no per-tap swizzle arithmetic);
//   * GroupNorm(+SiLU) transform on packed f32 pairs (v_pk_fma / v_pk_mul / v_pk_add), the 8
//     v_exp / v_rcp of a vector issued back to back (no transcendental-use s_nop padding), zero
//     padding applied only on tiles that touch the image border;
//   * MFMA operands swapped (D = [co][px]) so each lane's 4 accumulator values are 4 consecutive
//     channels: the epilogue stages the tile in LDS with ds_write_b128 (16 per half instead of 64
//     ds_write_b32) and stores / loads residuals through a wave-uniform buffer resource with the pass
//     offset in an SGPR (no per-pass 64-bit address arithmetic).
#include "conv_common.h"

namespace snrse_conv {
namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int H7_TH = 4, H7_TW = 64, H7_HC = H7_TW + 2;
constexpr int H7_HROWS = (H7_TH + 2) * H7_HC;  // 396 halo pixels
constexpr int H7_PLANE = 400;                  // rows per chunk plane (multiple of 16: conflict-free)
constexpr int H7_HALO_BYTES = 4 * H7_PLANE * 16;  // 25600
constexpr int H7_TAPB = 128 * 64;               // one tap's 128 couts x 32 ch bf16
constexpr int H7_SLOT = 3 * H7_TAPB;            // 24576
constexpr int H7_LDS = H7_HALO_BYTES + 2 * H7_SLOT;  // 74752: two workgroups per CU
constexpr int H7_HJ = 7;                        // halo rows per thread (16 per wave, 64 per pass)
constexpr int H7_LDR = 68;                      // epilogue staging row (floats)

SNRSE_DEV int h7_swz(int row, int chunk) { return (row << 6) + ((chunk ^ ((row >> 1) & 3)) << 4); }

// GroupNorm (+SiLU) of one 16-B vector (8 bf16 channels): y = s x + h [; y = y sigmoid(y)]
template <int GNM>
SNRSE_DEV u32x4 h7_xform(u32x4 v, const f32x2 (&s)[4], const f32x2 (&h)[4]) {
  f32x2 a[4];
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const f32x2 x = {__uint_as_float(v[k] << 16), __uint_as_float(v[k] & 0xffff0000u)};
    a[k] = x * s[k] + h[k];
  }
  if constexpr (GNM == 2) {
    f32x2 e[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = a[k] * -1.44269504088896341f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e[k].x = __builtin_amdgcn_exp2f(e[k].x);
      e[k].y = __builtin_amdgcn_exp2f(e[k].y);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) e[k] = e[k] + 1.0f;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      e[k].x = __builtin_amdgcn_rcpf(e[k].x);
      e[k].y = __builtin_amdgcn_rcpf(e[k].y);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) a[k] = a[k] * e[k];
  }
  u32x4 o;
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = pack_bf16x2(a[k].x, a[k].y);
  return o;
}

template <int S>
SNRSE_DEV float h7_sum_lanes(float v) {  // sum over the lanes sharing lane % S (S = 8), all receive it
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
}

SNRSE_DEV int h7_opaque(int v) {
  int r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

SNRSE_DEV __amdgpu_buffer_rsrc_t h7_rsrc(const void* base, unsigned bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

template <int GNM>
__global__ __launch_bounds__(256, 2) void conv_halo7_kernel(ConvParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const halo = smem;
  char* const ring = smem + H7_HALO_BYTES;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lrow = lane & 15, lg = lane >> 4;

  // XCD-aware bijective remap: consecutive logical tiles (neighbouring image rows) share an XCD
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7, pos = bid >> 3;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int n0 = (wg % p.ntn) * 128;
  int tile = wg / p.ntn;
  const int ntw = p.W / H7_TW, nth = p.H / H7_TH;
  const int w0 = (tile % ntw) * H7_TW;
  tile /= ntw;
  const int h0 = (tile % nth) * H7_TH;
  const int bb = tile / nth;
  const bool edge = h0 == 0 || h0 + H7_TH == p.H || w0 == 0 || w0 + H7_TW == p.W;  // uniform

  const int Cin = p.C0 + p.C1;
  const int cbm = Cin / 32;
  const int Csc_all = p.Csc + p.Csc1;
  const int cbs = p.sc_src ? Csc_all / 32 : 0;
  const int ncb = cbm + cbs;
  const int K1 = 9 * Cin;

  // this thread's halo rows (pixel hr of the (4+2) x (64+2) halo) and 16-B channel chunk.  Lane-derived
  // values are re-derived at each use from an opaque copy of the thread index, so they are not hoisted
  // into VGPRs that stay live across the MFMA phases (256-VGPR budget at two waves per SIMD).
  auto hrow = [&](int t, int j) { return (t & 15) + 16 * (t >> 6) + 64 * j; };
  auto hvalid = [&](int hr, int& pix) {
    const int hy = hr / H7_HC, hx = hr - hy * H7_HC;
    const int ih = h0 + hy - 1, iw = w0 + hx - 1;
    pix = (bb * p.H + ih) * p.W + iw;
    return hr < H7_HROWS && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
  };

  u32x4 hv[H7_HJ];
  f32x2 gs[4], gh[4];
  auto halo_load = [&](int c) {
    const void* base;
    long long bytes;
    int cs, cc;
    if (c < cbm) {
      const int ch = c * 32;
      if (ch < p.C0) { base = p.src0; bytes = p.bytes0; cs = p.C0; cc = ch; }
      else { base = p.src1; bytes = p.bytes1; cs = p.C1; cc = ch - p.C0; }
    } else {
      const int ch = (c - cbm) * 32;
      if (ch < p.Csc) { base = p.sc_src; bytes = p.sc_bytes0; cs = p.Csc; cc = ch; }
      else { base = p.sc_src1; bytes = p.sc_bytes1; cs = p.Csc1; cc = ch - p.Csc; }
    }
    const __amdgpu_buffer_rsrc_t r = make_rsrc(base, bytes);
    const int t = h7_opaque((int)threadIdx.x);
    const int c8 = cc + ((t >> 4) & 3) * 8;
#pragma unroll
    for (int j = 0; j < H7_HJ; ++j) {
      int pix;
      const bool ok = hvalid(hrow(t, j), pix);
      hv[j] = __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (pix * cs + c8) * 2 : (int)0x80000000, 0, 0);
    }
  };
  // GroupNorm affine of chunk c's 8 channels of this thread: loaded during the chunk's LAST phase only,
  // so the 16 registers are not live across the other phases' MFMAs
  auto gn_load = [&](int c) {
    if constexpr (GNM > 0) {
      if (c < cbm) {
        const int hc = (h7_opaque((int)threadIdx.x) >> 4) & 3;
        const float* sp = p.gn_scale + (size_t)bb * Cin + c * 32 + hc * 8;
        const float* hp = p.gn_shift + (size_t)bb * Cin + c * 32 + hc * 8;
        const f32x4 s0 = *(const f32x4*)sp, s1 = *(const f32x4*)(sp + 4);
        const f32x4 t0 = *(const f32x4*)hp, t1 = *(const f32x4*)(hp + 4);
        gs[0] = {s0[0], s0[1]}; gs[1] = {s0[2], s0[3]}; gs[2] = {s1[0], s1[1]}; gs[3] = {s1[2], s1[3]};
        gh[0] = {t0[0], t0[1]}; gh[1] = {t0[2], t0[3]}; gh[2] = {t1[0], t1[1]}; gh[3] = {t1[2], t1[3]};
      }
    }
  };
  auto halo_store = [&](int c) {
    const bool tr = GNM > 0 && c < cbm;
    const int t = h7_opaque((int)threadIdx.x);
    const int hst = ((t >> 4) & 3) * (H7_PLANE * 16) + hrow(t, 0) * 16;  // LDS byte offset of row j = 0
#pragma unroll
    for (int j = 0; j < H7_HJ; ++j) {
      const int hr = hrow(t, j);
      u32x4 v = hv[j];
      if constexpr (GNM > 0) {
        if (tr) {
          v = h7_xform<GNM>(v, gs, gh);
          if (edge) {
            int pix;
            if (!hvalid(hr, pix)) v = u32x4{0u, 0u, 0u, 0u};  // the conv's zero padding
          }
        }
      }
      if (j < H7_HJ - 1 || hr < H7_HROWS) *(u32x4*)(halo + hst + j * 64 * 16) = v;
    }
  };
  // weights of phase q (3 taps of main chunk c, or the shortcut chunk) -> ring slot `slot`:
  // 8 pieces of 1 KB (16 rows x 64 B) per tap, lane-linear LDS destination, swizzle on the source
  auto wload = [&](int c, int t0, int nt, int slot) {
    const bool mainw = c < cbm;
    const int wld = mainw ? K1 : Csc_all;
    const int kb = mainw ? c * 32 : (c - cbm) * 32;
    const __amdgpu_buffer_rsrc_t r = mainw ? make_rsrc(p.wgt, p.wbytes) : make_rsrc(p.sc_wgt, p.sc_wbytes);
    char* dst = ring + slot * H7_SLOT;
    const int ln = h7_opaque((int)threadIdx.x) & 63;
    const int rl = ln >> 2, sl = ln & 3;
    for (int ii = wid; ii < nt * 8; ii += 4) {
      const int jt = ii >> 3, pc = ii & 7;
      const int koff = mainw ? (t0 + jt) * Cin + kb : kb;
      const int row = pc * 16 + rl;
      const unsigned voff = (unsigned)(((n0 + row) * wld + koff + (sl ^ ((row >> 1) & 3)) * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          r, (__attribute__((address_space(3))) void*)(dst + jt * H7_TAPB + pc * 1024), 16, voff, 0, 0, 0);
    }
  };

  f32x4 acc[2][4][4];  // [co half][px group][co group]: D = [co][px]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // lane constants of the fragment reads: A = weights (co rows), B = halo pixels
  const int bofs = h7_swz(lrow, lg);                                          // + jt*TAPB + j*1024
  const int aofs = lg * (H7_PLANE * 16) + ((wid + 0) * H7_HC + lrow) * 16;   // + (ky*66 + kx)*16 + i*256

  auto mma_tap = [&](const char* sb, int ha) {
    u32x4 af[4], bfr[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *(const u32x4*)(halo + ha + i * 256);
#pragma unroll
    for (int j = 0; j < 8; ++j) bfr[j] = *(const u32x4*)(sb + bofs + j * 1024);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h][i][j] = mfma_chunk<bf16_t>(bfr[h * 4 + j], af[i], acc[h][i][j]);
  };

  halo_load(0);
  wload(0, 0, cbm > 0 ? 3 : 1, 0);
  gn_load(0);
  halo_store(0);
  // flat phase loop (as v5): phase q = (chunk c, tap row ky); main chunks have 3 phases of 3 taps,
  // shortcut chunks one centre-tap phase; c / ky advance by counters, the ring slot alternates
  const int nq = 3 * cbm + cbs;
  int c = 0, ky = 0;
  for (int q = 0; q < nq; ++q) {
    const bool mainc = c < cbm;
    const bool lastph = !mainc || ky == 2;
    const bool more = c + 1 < ncb;
    // the halo prefetch issued after this phase's weights (first phase of the chunk) may stay in flight
#ifndef SNRSE_H7_ABL_NOSYNC
    if (ky > 0 && more) asm volatile("s_waitcnt vmcnt(7) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
#endif
    if (!lastph) wload(c, (ky + 1) * 3, 3, (q + 1) & 1);
    else if (more) wload(c + 1, 0, c + 1 < cbm ? 3 : 1, (q + 1) & 1);
#ifndef SNRSE_H7_ABL_NOHALO
    if (ky == 0 && more) halo_load(c + 1);
    if (lastph && more) gn_load(c + 1);
#endif
    const char* sb = ring + (q & 1) * H7_SLOT;
    // one MFMA site for both kinds of phase (two sites make the accumulators phi-copied across them):
    // main phases run taps (ky, 0..2), shortcut phases the centre tap of the 1x1 shortcut
    const int ntap = mainc ? 3 : 1;
    const int hb = mainc ? aofs + ky * (H7_HC * 16) : aofs + H7_HC * 16 + 16;
#pragma unroll 1
    for (int kx = 0; kx < ntap; ++kx) mma_tap(sb + kx * H7_TAPB, hb + kx * 16);
#ifndef SNRSE_H7_ABL_NOHALO
    if (lastph && more) {
#ifndef SNRSE_H7_ABL_NOSYNC
      asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave is done reading halo(c)
#endif
      halo_store(c + 1);
    }
#endif
    if (lastph) { ++c; ky = 0; } else { ++ky; }
  }

  // ---------------------------------------------------------------- epilogue
#ifdef SNRSE_H7_ABL_NOEPI
  {
    float t = 0.f;
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) t += acc[h][i][j][0] + acc[h][i][j][1] + acc[h][i][j][2] + acc[h][i][j][3];
    ((float*)p.out)[(size_t)blockIdx.x * 256 + threadIdx.x] = t;  // keeps the accumulators live (diagnostic build)
    return;
  }
#endif
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // LDS is reused as the staging area
  float* const stage = (float*)(smem + wid * (64 * H7_LDR * 4));
  float* const red = (float*)(smem + 4 * (64 * H7_LDR * 4));  // [4 waves][128 co][2]
  const size_t mrow = ((size_t)bb * p.H + h0 + wid) * p.W + w0;  // first pixel of this wave's row
  constexpr int EPC = 8, NCH = 8, RPP = 8, NPASS = 8;          // bf16: 8 channels per lane, 8 rows per pass
  const int cc = lane % NCH, r0 = lane / NCH;
  const unsigned row_bytes = (unsigned)p.out_ld * 2, res_row_bytes = (unsigned)p.res_ld * 2;
  const __amdgpu_buffer_rsrc_t ro = h7_rsrc((const char*)p.out + mrow * row_bytes, 64 * row_bytes);
  __amdgpu_buffer_rsrc_t rr = ro, rc = ro;
  if (p.res) rr = h7_rsrc((const char*)p.res + mrow * res_row_bytes, 64 * res_row_bytes);
  if (p.comb_src) rc = h7_rsrc(p.comb_src + mrow * 4, 64 * 16);
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    if (h) {
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
    }
    // stage this half: lane holds co 16j + 4lg + e of px 16i + lrow -> one 16-B write per (i, j)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) *(f32x4*)(stage + (16 * i + lrow) * H7_LDR + 16 * j + 4 * lg) = acc[h][i][j];
    const int n = n0 + 64 * h + cc * EPC;
    f32x2 add[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) add[k] = f32x2{0.f, 0.f};
    if (p.bias) {
      const f32x4 b0 = *(const f32x4*)(p.bias + n), b1 = *(const f32x4*)(p.bias + n + 4);
      add[0] = {b0[0], b0[1]}; add[1] = {b0[2], b0[3]}; add[2] = {b1[0], b1[1]}; add[3] = {b1[2], b1[3]};
    }
    if (p.temb) {
      const f32x4 t0 = *(const f32x4*)(p.temb + (size_t)bb * p.temb_stride + n);
      const f32x4 t1 = *(const f32x4*)(p.temb + (size_t)bb * p.temb_stride + n + 4);
      add[0] += f32x2{t0[0], t0[1]}; add[1] += f32x2{t0[2], t0[3]};
      add[2] += f32x2{t1[0], t1[1]}; add[3] += f32x2{t1[2], t1[3]};
    }
    f32x4 cw[EPC];
    float cb[EPC];
    if (p.comb_src) {
#pragma unroll
      for (int k = 0; k < EPC; ++k) {
        cw[k] = *(const f32x4*)(p.comb_w + (size_t)(n + k) * 4);
        cb[k] = p.comb_b[n + k];
      }
    }
    u32x4 rpre[NPASS];
    f32x4 qpre[NPASS];
    const unsigned vo = r0 * row_bytes + (unsigned)n * 2;  // this lane's 16-B chunk in its first row
    if (p.res) {
      const unsigned vr = r0 * res_row_bytes + (unsigned)n * 2;
#pragma unroll
      for (int ps = 0; ps < NPASS; ++ps) rpre[ps] = __builtin_amdgcn_raw_buffer_load_b128(rr, vr, ps * RPP * res_row_bytes, 0);
    }
    if (p.comb_src) {
#pragma unroll
      for (int ps = 0; ps < NPASS; ++ps)
        qpre[ps] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rc, r0 * 16, ps * RPP * 16, 0));
    }
    __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the staged tile
    __builtin_amdgcn_wave_barrier();
    f32x2 s1[4], s2[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) { s1[k] = f32x2{0.f, 0.f}; s2[k] = f32x2{0.f, 0.f}; }
#pragma unroll
    for (int ps = 0; ps < NPASS; ++ps) {
      const float* sr = stage + (r0 + ps * RPP) * H7_LDR + cc * EPC;
      const f32x4 a0 = *(const f32x4*)sr, a1 = *(const f32x4*)(sr + 4);
      f32x2 v[4] = {f32x2{a0[0], a0[1]} + add[0], f32x2{a0[2], a0[3]} + add[1], f32x2{a1[0], a1[1]} + add[2],
                    f32x2{a1[2], a1[3]} + add[3]};
      if (p.res) {
#pragma unroll
        for (int k = 0; k < 4; ++k)
          v[k] += f32x2{__uint_as_float(rpre[ps][k] << 16), __uint_as_float(rpre[ps][k] & 0xffff0000u)};
      }
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] *= p.out_scale;
      if (p.comb_src) {
        const f32x4 q = qpre[ps];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k].x += q[0] * cw[2 * k][0] + q[1] * cw[2 * k][1] + q[2] * cw[2 * k][2] + q[3] * cw[2 * k][3] + cb[2 * k];
          v[k].y += q[0] * cw[2 * k + 1][0] + q[1] * cw[2 * k + 1][1] + q[2] * cw[2 * k + 1][2] +
                    q[3] * cw[2 * k + 1][3] + cb[2 * k + 1];
        }
      }
      const u32x4 o = {pack_bf16x2(v[0].x, v[0].y), pack_bf16x2(v[1].x, v[1].y), pack_bf16x2(v[2].x, v[2].y),
                       pack_bf16x2(v[3].x, v[3].y)};
      if (p.epi_nt) __builtin_amdgcn_raw_buffer_store_b128(o, ro, vo, ps * RPP * row_bytes, 2);
      else __builtin_amdgcn_raw_buffer_store_b128(o, ro, vo, ps * RPP * row_bytes, 0);
      if (p.stats) {
#pragma unroll
        for (int k = 0; k < 4; ++k) { s1[k] += v[k]; s2[k] += v[k] * v[k]; }
      }
    }
    if (p.stats) {
      float t1[8], t2[8];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        t1[2 * k] = h7_sum_lanes<NCH>(s1[k].x); t1[2 * k + 1] = h7_sum_lanes<NCH>(s1[k].y);
        t2[2 * k] = h7_sum_lanes<NCH>(s2[k].x); t2[2 * k + 1] = h7_sum_lanes<NCH>(s2[k].y);
      }
      if (r0 == 0) {
#pragma unroll
        for (int k = 0; k < EPC; ++k) {
          red[(wid * 128 + 64 * h + cc * EPC + k) * 2] = t1[k];
          red[(wid * 128 + 64 * h + cc * EPC + k) * 2 + 1] = t2[k];
        }
      }
    }
  }
  if (p.stats) {  // one (sum, sumsq) atomic pair per channel per workgroup
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const int sslot = blockIdx.x & (SNRSE_STAT_SLOTS - 1);
    for (int t = tid; t < 256; t += 256) {
      const float a = red[t] + red[256 + t] + red[512 + t] + red[768 + t];
      unsafeAtomicAdd(&p.stats[stat_idx(bb, sslot, n0 + (t >> 1), p.Cout) + (t & 1)], (double)a);
    }
  }
}

}  // namespace

bool halo7_ok(const ConvParams& p) {
  return p.ksize == 3 && p.H % H7_TH == 0 && p.W % H7_TW == 0 && p.Cout % 128 == 0 && p.C0 % 32 == 0 &&
         p.C1 % 32 == 0 && (p.C0 + p.C1) > 0 && (!p.sc_src || (p.Csc + p.Csc1) % 32 == 0) &&
         p.out_ld % 8 == 0 && (!p.res || p.res_ld % 8 == 0) &&
         (long long)64 * p.out_ld * 2 < 0x7fffffffll && p.bytes0 < 0x7ff00000ll && p.bytes1 < 0x7ff00000ll &&
         p.sc_bytes0 < 0x7ff00000ll && p.sc_bytes1 < 0x7ff00000ll;
}

int launch_halo7(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  if (!halo7_ok(p)) return SNRSE_EINVAL;
  p.ntn = p.Cout / 128;
  const int tiles = p.B * (p.H / H7_TH) * (p.W / H7_TW) * p.ntn;
  const void* fn;
  if (!p.gn_scale) fn = (const void*)conv_halo7_kernel<0>;
  else if (!p.gn_act) fn = (const void*)conv_halo7_kernel<1>;
  else fn = (const void*)conv_halo7_kernel<2>;
  static bool attr[3] = {false, false, false};
  const int gi = !p.gn_scale ? 0 : (!p.gn_act ? 1 : 2);
  if (!attr[gi]) {
    SNRSE_RET(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, H7_LDS));
    attr[gi] = true;
  }
  if (gi == 0) hipLaunchKernelGGL((conv_halo7_kernel<0>), dim3(tiles), dim3(256), H7_LDS, s, p);
  else if (gi == 1) hipLaunchKernelGGL((conv_halo7_kernel<1>), dim3(tiles), dim3(256), H7_LDS, s, p);
  else hipLaunchKernelGGL((conv_halo7_kernel<2>), dim3(tiles), dim3(256), H7_LDS, s, p);
  return (int)hipGetLastError();
}

}  // namespace snrse_conv
