// v9 halo GEMM: the 3x3 convolutions of the NCSN++ ResBlocks (layerspp.py:244-276 Conv_0 / Conv_1
// [+ Conv_2 shortcut], ddpm_conv3x3 layers.py:100-124) with the GroupNorm(+SiLU) prologue fused,
// bf16 operands, f32 accumulation, bf16 output (gfx950).
//
// Same tile and fragment layout as v7 (conv_halo7.hip: two 256-thread workgroups per CU, tile = 4
// image rows x 64 px x 128 output channels, wave w computes image row h0 + w, chunk-planar halo,
// swapped MFMA operands, LDS-staged buffer epilogue).  The v7 ablations (profiles/r02d_h7_ablations.json)
// showed the halo transform and its barrier-separated store costing ~15 % of the kernel, none of it
// under MFMAs.  v9 removes that serialisation:
//   * the halo image is DOUBLE-buffered (2 x 25 KB): chunk c+1's halo is loaded at the first tap of
//     chunk c and transformed + stored one 16-row vector per tap during taps 2..8 of chunk c, so the
//     GroupNorm/SiLU VALU work and the ds_writes run between the MFMA bursts of every tap, and no
//     extra barrier is needed (the tap barrier at the start of chunk c+1 publishes the halo);
//   * to fit the second halo buffer at two workgroups per CU the weight ring holds single taps:
//     3 slots x 8 KB, each tap's weights DMA'd two taps ahead (one barrier per tap; the v7 NOSYNC
//     ablation measured the barriers themselves as free);
//   * the GroupNorm affine of all input channels is staged in LDS once per workgroup (<= 4 KB), so the
//     per-vector transform reads it there instead of holding 16 VGPRs across the MFMA phases.
// LDS: 2 x 25600 (halo) + 3 x 8192 (weights) + 4096 (affine) = 79872 B -> two workgroups per CU.
#include "conv_common.h"

namespace snrse_conv {
namespace {

typedef float f32x2 __attribute__((ext_vector_type(2)));

constexpr int H9_TH = 4, H9_TW = 64, H9_HC = H9_TW + 2;
constexpr int H9_HROWS = (H9_TH + 2) * H9_HC;        // 396 halo pixels
constexpr int H9_PLANE = 400;                        // rows per chunk plane (multiple of 16: conflict-free)
constexpr int H9_HALO = 4 * H9_PLANE * 16;           // 25600 per buffer
constexpr int H9_TAPB = 128 * 64;                    // one tap's 128 couts x 32 ch bf16
constexpr int H9_RING = 2 * H9_HALO;                 // ring offset
constexpr int H9_AFF = H9_RING + 3 * H9_TAPB;        // GroupNorm affine offset (75776)
constexpr int H9_CMAX = 512;                         // input channels the affine area holds
constexpr int H9_LDS = H9_AFF + 2 * H9_CMAX * 4;     // 79872: two workgroups per CU
constexpr int H9_HJ = 7;                             // halo rows per thread (16 per wave, 64 per pass)
constexpr int H9_LDR = 68;                           // epilogue staging row (floats)

SNRSE_DEV int h9_swz(int row, int chunk) { return (row << 6) + ((chunk ^ ((row >> 1) & 3)) << 4); }

SNRSE_DEV int h9_opaque(int v) {
  int r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

// GroupNorm (+SiLU) of one 16-B vector (8 bf16 channels): y = s x + h [; y = y sigmoid(y)]
template <int GNM>
SNRSE_DEV u32x4 h9_xform(u32x4 v, const f32x4& s0, const f32x4& s1, const f32x4& t0, const f32x4& t1) {
  const f32x2 s[4] = {{s0[0], s0[1]}, {s0[2], s0[3]}, {s1[0], s1[1]}, {s1[2], s1[3]}};
  const f32x2 h[4] = {{t0[0], t0[1]}, {t0[2], t0[3]}, {t1[0], t1[1]}, {t1[2], t1[3]}};
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
SNRSE_DEV float h9_sum_lanes(float v) {  // sum over the lanes sharing lane % S (S = 8), all receive it
  v += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x128, 0xf, 0xf, false));
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  v = __uint_as_float(r[0]) + __uint_as_float(r[1]);
  const auto r2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
  return __uint_as_float(r2[0]) + __uint_as_float(r2[1]);
}

SNRSE_DEV __amdgpu_buffer_rsrc_t h9_rsrc(const void* base, unsigned bytes) {
  const uint64_t a = (uint64_t)base;
  const uint32_t lo = __builtin_amdgcn_readfirstlane((uint32_t)a);
  const uint32_t hi = __builtin_amdgcn_readfirstlane((uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc((void*)(((uint64_t)hi << 32) | lo), 0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

#define H9_FENCE() asm volatile("" ::: "memory")  // keeps the VMEM issue order the wait counts assume

template <int GNM>
__global__ __launch_bounds__(256, 2) void conv_halo9_kernel(ConvParams p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* const ring = smem + H9_RING;
  float* const aff = (float*)(smem + H9_AFF);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lrow = lane & 15, lg = lane >> 4;

  // XCD-aware bijective remap: consecutive logical tiles (neighbouring image rows) share an XCD
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7, pos = bid >> 3;
  const int wg = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int n0 = (wg % p.ntn) * 128;
  int tile = wg / p.ntn;
  const int ntw = p.W / H9_TW, nth = p.H / H9_TH;
  const int w0 = (tile % ntw) * H9_TW;
  tile /= ntw;
  const int h0 = (tile % nth) * H9_TH;
  const int bb = tile / nth;
  const bool edge = h0 == 0 || h0 + H9_TH == p.H || w0 == 0 || w0 + H9_TW == p.W;  // uniform

  const int Cin = p.C0 + p.C1;
  const int cbm = Cin / 32;
  const int Csc_all = p.Csc + p.Csc1;
  const int cbs = p.sc_src ? Csc_all / 32 : 0;
  const int ncb = cbm + cbs;
  const int K1 = 9 * Cin;
  const int nq = 9 * cbm + cbs;  // phases: one per tap (main chunks 9, shortcut chunks 1)

  // this thread's halo rows (pixel hr of the (4+2) x (64+2) halo) and 16-B channel chunk; lane-derived
  // values are re-derived at each use from an opaque copy of the thread index (not hoisted into VGPRs
  // that stay live across the MFMA bursts)
  auto hrow = [&](int t, int j) { return (t & 15) + 16 * (t >> 6) + 64 * j; };
  auto hvalid = [&](int hr, int& pix) {
    const int hy = hr / H9_HC, hx = hr - hy * H9_HC;
    const int ih = h0 + hy - 1, iw = w0 + hx - 1;
    pix = (bb * p.H + ih) * p.W + iw;
    return hr < H9_HROWS && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
  };

  u32x4 hv[H9_HJ];
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
    const int t = h9_opaque((int)threadIdx.x);
    const int c8 = cc + ((t >> 4) & 3) * 8;
#pragma unroll
    for (int j = 0; j < H9_HJ; ++j) {
      int pix;
      const bool ok = hvalid(hrow(t, j), pix);
      hv[j] = __builtin_amdgcn_raw_buffer_load_b128(r, ok ? (pix * cs + c8) * 2 : (int)0x80000000, 0, 0);
    }
  };
  // border validity of this thread's 7 halo rows (bit j), for re-applying the zero padding after the
  // GroupNorm affine on border tiles
  int vmask = 0;
#pragma unroll
  for (int j = 0; j < H9_HJ; ++j) {
    int pix;
    vmask |= hvalid(hrow(tid, j), pix) ? (1 << j) : 0;
  }
  // vector j of chunk c's halo -> halo buffer at byte offset hbuf: GroupNorm(+SiLU) on main chunks, a
  // plain copy on shortcut chunks.  Branch-free (selects, and the 4 lanes past the 396 halo rows write
  // the never-read pad rows 396..399), so the scheduler can interleave it with the tap's MFMAs.
  auto halo_store_vec = [&](int c, int j, int hbuf) {
    const int t = h9_opaque((int)threadIdx.x);
    const int hc = (t >> 4) & 3;
    const int hr = hrow(t, j);
    const int hw = (j < H9_HJ - 1 || hr < H9_HROWS) ? hr : H9_HROWS + (hr & 3);
    u32x4 v = hv[j];
    if constexpr (GNM > 0) {
      const float* sp = aff + min(c, cbm - 1) * 32 + hc * 8;
      const f32x4 s0 = *(const f32x4*)sp, s1 = *(const f32x4*)(sp + 4);
      const f32x4 t0 = *(const f32x4*)(sp + Cin), t1 = *(const f32x4*)(sp + Cin + 4);
      u32x4 x = h9_xform<GNM>(v, s0, s1, t0, t1);
      const bool pad = edge && !((vmask >> j) & 1);  // the conv's zero padding
      const bool tr = c < cbm;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = tr ? (pad ? 0u : x[e]) : v[e];
    }
    *(u32x4*)(smem + hbuf + hc * (H9_PLANE * 16) + hw * 16) = v;
  };
  // weights of one tap -> ring slot: main chunk cw tap `tap`, or shortcut chunk cw (>= cbm).  8 pieces
  // of 1 KB (16 rows x 64 B), two per wave, lane-linear LDS destination, swizzle on the source
  auto wload = [&](int cw, int tap, int slot) {
    const bool mainw = cw < cbm;
    const int wld = mainw ? K1 : Csc_all;
    const int koff = mainw ? tap * Cin + cw * 32 : (cw - cbm) * 32;
    const __amdgpu_buffer_rsrc_t r = mainw ? make_rsrc(p.wgt, p.wbytes) : make_rsrc(p.sc_wgt, p.sc_wbytes);
    char* dst = ring + slot * H9_TAPB;
    const int ln = h9_opaque((int)threadIdx.x) & 63;
    const int rl = ln >> 2, sl = ln & 3;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int pc = wid + 4 * u;
      const int row = pc * 16 + rl;
      const unsigned voff = (unsigned)(((n0 + row) * wld + koff + (sl ^ ((row >> 1) & 3)) * 8) * 2);
      __builtin_amdgcn_raw_ptr_buffer_load_lds(
          r, (__attribute__((address_space(3))) void*)(dst + pc * 1024), 16, voff, 0, 0, 0);
    }
  };

  f32x4 acc[2][4][4];  // [co half][px group][co group]: D = [co][px]
#pragma unroll
  for (int h = 0; h < 2; ++h)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[h][i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int bofs = h9_swz(lrow, lg);                                    // + j*1024 within a tap slot
  const int aofs = lg * (H9_PLANE * 16) + (wid * H9_HC + lrow) * 16;   // + hbuf + (ky*66 + kx)*16 + i*256

  auto mma_tap = [&](const char* sb, int ha) {
    u32x4 af[4], bfr[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *(const u32x4*)(smem + ha + i * 256);
#pragma unroll
    for (int j = 0; j < 8; ++j) bfr[j] = *(const u32x4*)(sb + bofs + j * 1024);
#pragma unroll
    for (int h = 0; h < 2; ++h)
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[h][i][j] = mfma_chunk<bf16_t>(bfr[h * 4 + j], af[i], acc[h][i][j]);
  };

  // ------------------------------------------------------------------ prologue
  if constexpr (GNM > 0) {  // GroupNorm affine of every input channel of this image -> LDS
    const int t4 = tid * 4;
    if (t4 < 2 * Cin) {
      const float* src = t4 < Cin ? p.gn_scale + (size_t)bb * Cin + t4 : p.gn_shift + (size_t)bb * Cin + (t4 - Cin);
      *(f32x4*)(aff + t4) = *(const f32x4*)src;
    }
  }
  H9_FENCE();
  halo_load(0);
  H9_FENCE();
  wload(0, 0, 0);
  wload(0, 1, 1);  // phase 1 = tap 1 of chunk 0 (every kernel has >= 1 main chunk)
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // the affine is visible
#pragma unroll
  for (int j = 0; j < H9_HJ; ++j) halo_store_vec(0, j, 0);

  // Every phase issues exactly two DMA loads per wave (past the last phase a dummy reload of chunk 0's
  // tap 0 into the free slot) and every main chunk's first tap seven halo loads (the last chunk reloads
  // itself), so the VMEM queue is the same on every path: the compiler's own waits for the halo
  // registers are exact, and the tap wait below leaves the newer loads in flight:
  //   tap 0: DMA(q+1) -> vmcnt(2);  taps 1, 2: + the 7 halo loads -> vmcnt(9);  taps 3..8: vmcnt(2).
  // ------------------------------------------------------------------ main chunks: 9 taps each
  for (int c = 0; c < cbm; ++c) {
    const bool more = c + 1 < ncb;
    const int hbuf = (c & 1) * H9_HALO, nbuf = H9_HALO - hbuf;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
#ifndef SNRSE_H9_ABL_NOSYNC
      if (k == 1 || k == 2) asm volatile("s_waitcnt vmcnt(9) lgkmcnt(0)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
#endif
      {  // the tap two phases ahead -> slot (k + 2) % 3
        int cw = c, tap = k + 2;
        if (k >= 7) {
          const int pn = 9 * c + k + 2;
          cw = pn >= nq ? 0 : (c + 1 < cbm ? c + 1 : cbm + k - 7);
          tap = (pn >= nq || c + 1 >= cbm) ? 0 : k - 7;
        }
        wload(cw, tap, (k + 2) % 3);
      }
      H9_FENCE();
      if (k == 0) halo_load(more ? c + 1 : c);
      mma_tap(ring + (k % 3) * H9_TAPB, aofs + hbuf + (k / 3) * (H9_HC * 16) + (k % 3) * 16);
#ifndef SNRSE_H9_ABL_NOHALO
      // the last main chunk with no shortcut after it transforms its own reload into the idle buffer
      if (k >= 2) halo_store_vec(more ? c + 1 : c, k - 2, nbuf);
#endif
    }
  }
  // ------------------------------------------------------------------ shortcut chunks: centre tap only
  // halo loads first, then the DMA, so the in-phase halo store waits only for the halo loads; the tap
  // wait counts the previous phase's halo loads + its DMA (9) or the DMA alone (2)
  for (int c = cbm; c < ncb; ++c) {
    const int q = 9 * cbm + (c - cbm);
    const bool more = c + 1 < ncb;
    const int hbuf = (c & 1) * H9_HALO, nbuf = H9_HALO - hbuf;
    if (c > cbm) asm volatile("s_waitcnt vmcnt(9) lgkmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    halo_load(more ? c + 1 : c);
    H9_FENCE();
    wload(q + 2 < nq ? c + 2 : 0, 0, (q + 2) % 3);
    mma_tap(ring + (q % 3) * H9_TAPB, aofs + hbuf + H9_HC * 16 + 16);
    if (more) {
#pragma unroll
      for (int j = 0; j < H9_HJ; ++j) halo_store_vec(c + 1, j, nbuf);
    }
  }

  // ---------------------------------------------------------------- epilogue (as v7)
  asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();  // LDS is reused as the staging area
  float* const stage = (float*)(smem + wid * (64 * H9_LDR * 4));
  float* const red = (float*)(smem + 4 * (64 * H9_LDR * 4));  // [4 waves][128 co][2]
  const size_t mrow = ((size_t)bb * p.H + h0 + wid) * p.W + w0;  // first pixel of this wave's row
  constexpr int EPC = 8, NCH = 8, RPP = 8, NPASS = 8;          // bf16: 8 channels per lane, 8 rows per pass
  const int cc = lane % NCH, r0 = lane / NCH;
  const unsigned row_bytes = (unsigned)p.out_ld * 2, res_row_bytes = (unsigned)p.res_ld * 2;
  const __amdgpu_buffer_rsrc_t ro = h9_rsrc((const char*)p.out + mrow * row_bytes, 64 * row_bytes);
  __amdgpu_buffer_rsrc_t rr = ro, rc = ro;
  if (p.res) rr = h9_rsrc((const char*)p.res + mrow * res_row_bytes, 64 * res_row_bytes);
  if (p.comb_src) rc = h9_rsrc(p.comb_src + mrow * 4, 64 * 16);
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
      for (int j = 0; j < 4; ++j) *(f32x4*)(stage + (16 * i + lrow) * H9_LDR + 16 * j + 4 * lg) = acc[h][i][j];
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
      const float* sr = stage + (r0 + ps * RPP) * H9_LDR + cc * EPC;
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
        const f32x4 qv = qpre[ps];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          v[k].x += qv[0] * cw[2 * k][0] + qv[1] * cw[2 * k][1] + qv[2] * cw[2 * k][2] + qv[3] * cw[2 * k][3] + cb[2 * k];
          v[k].y += qv[0] * cw[2 * k + 1][0] + qv[1] * cw[2 * k + 1][1] + qv[2] * cw[2 * k + 1][2] +
                    qv[3] * cw[2 * k + 1][3] + cb[2 * k + 1];
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
        t1[2 * k] = h9_sum_lanes<NCH>(s1[k].x); t1[2 * k + 1] = h9_sum_lanes<NCH>(s1[k].y);
        t2[2 * k] = h9_sum_lanes<NCH>(s2[k].x); t2[2 * k + 1] = h9_sum_lanes<NCH>(s2[k].y);
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
    const float a = red[tid] + red[256 + tid] + red[512 + tid] + red[768 + tid];
    unsafeAtomicAdd(&p.stats[stat_idx(bb, sslot, n0 + (tid >> 1), p.Cout) + (tid & 1)], (double)a);
  }
}

}  // namespace

bool halo9_ok(const ConvParams& p) {
  return p.ksize == 3 && p.H % H9_TH == 0 && p.W % H9_TW == 0 && p.Cout % 128 == 0 && p.C0 % 32 == 0 &&
         p.C1 % 32 == 0 && (p.C0 + p.C1) > 0 && (p.C0 + p.C1) <= H9_CMAX &&
         (!p.sc_src || (p.Csc + p.Csc1) % 32 == 0) && p.out_ld % 8 == 0 && (!p.res || p.res_ld % 8 == 0) &&
         (long long)64 * p.out_ld * 2 < 0x7fffffffll && p.bytes0 < 0x7ff00000ll && p.bytes1 < 0x7ff00000ll &&
         p.sc_bytes0 < 0x7ff00000ll && p.sc_bytes1 < 0x7ff00000ll;
}

int launch_halo9(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  if (!halo9_ok(p)) return SNRSE_EINVAL;
  p.ntn = p.Cout / 128;
  const int tiles = p.B * (p.H / H9_TH) * (p.W / H9_TW) * p.ntn;
  const int gi = !p.gn_scale ? 0 : (!p.gn_act ? 1 : 2);
  const void* fn = gi == 0 ? (const void*)conv_halo9_kernel<0>
                           : (gi == 1 ? (const void*)conv_halo9_kernel<1> : (const void*)conv_halo9_kernel<2>);
  static bool attr[3] = {false, false, false};
  if (!attr[gi]) {
    SNRSE_RET(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, H9_LDS));
    attr[gi] = true;
  }
  if (gi == 0) hipLaunchKernelGGL((conv_halo9_kernel<0>), dim3(tiles), dim3(256), H9_LDS, s, p);
  else if (gi == 1) hipLaunchKernelGGL((conv_halo9_kernel<1>), dim3(tiles), dim3(256), H9_LDS, s, p);
  else hipLaunchKernelGGL((conv_halo9_kernel<2>), dim3(tiles), dim3(256), H9_LDS, s, p);
  return (int)hipGetLastError();
}

}  // namespace snrse_conv
