// v6 halo GEMM: persistent, fully LDS-DMA-fed 3x3 convolution (+ fused GroupNorm/SiLU prologue,
// fused 1x1 shortcut, bias/temb/residual epilogue and GroupNorm statistics) for the NCSN++
// ResnetBlockBigGANpp convolutions (reference: layerspp.py:244-276 -> layers.py:100-124).
//
// Structure (why: profiles/r01_pmc_sq_conv_v5_v6.json -- the halo kernels are ISSUE-bound, ~20
// non-MFMA instructions per MFMA in a first persistent version; this one is laid out so that the
// per-phase instruction stream is little more than the fragment reads and the MFMAs):
//
//   tile      = 8 image rows x 32 px x 128 output channels; wave w owns rows h0+2w, h0+2w+1
//               (64 px x 128 co = acc[2][4] of v_mfma_f32_32x32x16_bf16, 128 VGPRs; the 32x32
//               shape holds the issue port 8 of its 32 cycles, 16x16x32 8 of 16)
//   chunk     = 32 input channels; a main chunk is 9 tap phases (fully unrolled: tap offsets are
//               ds_read immediates), a shortcut (Conv_2) chunk 1
//   phase     = one tap: 16 MFMAs per wave, one barrier
//   weights   = 4-slot ring of one-tap slices (128 co x 32 ch, 8 KB), LDS-DMA three phases ahead
//   halo      = 2 buffers of (8+2) x (32+2) rows x 64 B; the raw halo of chunk c+1 is LDS-DMA'd at
//               the first phase of chunk c (zero padding from the buffer range check) and the
//               GroupNorm+SiLU transform runs IN PLACE one halo row per thread per phase over
//               phases 3..8, interleaved with the MFMA phases instead of behind a barrier
//   GN affine = per-chunk 32 x (scale, shift) LDS-DMA'd beside the halo; bias / temb slices of
//               the tile LDS-DMA'd at its first phase (no VGPR loads in the pipelined loop)
//   epilogue  = per wave through its slice of the just-finished halo buffer: stage 32 co x 32 px,
//               finish one pixel x 16 channels per lane (16-B residual loads / stores), GroupNorm
//               statistics reduced in LDS over the workgroup's consecutive tiles of one image and
//               flushed as one f64 atomic pair per channel
//
// Every wave issues the same number of LDS-DMA operations per phase (halo pieces + GroupNorm
// affine = 6 per wave at a chunk start, 1 bias/temb piece at a tile start, 2 weight pieces per
// phase), so each in-loop wait is a counted `s_waitcnt vmcnt(N)` for exactly the data the next
// phase reads (raw s_barrier; vmcnt(0) only at the tile boundary, before the epilogue).
// Two 256-thread workgroups per CU (K6_LDS each): one's epilogue runs under the other's MFMAs.
#include "conv_common.h"

#include <type_traits>

namespace snrse_conv {
namespace {

constexpr int K6_TH = 8, K6_TW = 32, K6_HC = K6_TW + 2;
constexpr int K6_HROWS = (K6_TH + 2) * K6_HC;  // 340 halo rows (hy * 34 + hx)
constexpr int K6_NPIECE = 22;                  // 1-KB LDS-DMA pieces per halo (rows 340..351 = pad)
constexpr int K6_HBUF = K6_NPIECE * 1024;      // 22528
constexpr int K6_HROWB = K6_HC * 64;           // bytes per halo image row (2176)
constexpr int K6_TROWS = 6;                    // halo rows transformed per thread: 64 x 6 >= 340
constexpr int K6_TAPB = 128 * 64;              // one tap: 128 co x 32 ch bf16
constexpr int K6_NSLOT = 4;
constexpr int K6_GNB = 256;  // [scale 32][shift 32] f32 of one chunk (4-byte LDS-DMA, 64 lanes)
constexpr int K6_OFF_W = 2 * K6_HBUF;
constexpr int K6_OFF_GN = K6_OFF_W + K6_NSLOT * K6_TAPB;
constexpr int K6_OFF_ST = K6_OFF_GN + 2 * K6_GNB;   // [128 co][2] GroupNorm partial sums
constexpr int K6_OFF_EP = K6_OFF_ST + 128 * 2 * 4;  // [bias 128][temb 128] of the current tile
constexpr int K6_LDS = K6_OFF_EP + 2 * 128 * 4;     // 80384 B
constexpr int K6_LDR = 36;                          // staged epilogue row: 32 px + 4 pad floats
constexpr int K6_STAGE = 32 * K6_LDR * 4;           // per-wave staging bytes (4608)
constexpr int K6_SKIP = 64;                         // wait_vm(): nothing to wait for
constexpr int K6_HOPS = 6;                          // DMA ops per wave at a chunk start
static_assert(64 * K6_TROWS >= K6_HROWS && 16 * K6_NPIECE >= K6_HROWS, "halo rows");
static_assert(4 * K6_HOPS == K6_NPIECE + 2, "halo pieces + 2 GroupNorm-affine ops per chunk");
static_assert(4 * K6_STAGE <= K6_HBUF, "epilogue staging fits one halo buffer");
static_assert(2 * (K6_LDS + 4 * 32 * 8) <= 163840, "two workgroups per CU (stamp builds included)");

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((ext_vector_type(16))) float f32x16;

// Halo LDS image: row = hy * 34 + hx, 64 B (32 bf16 channels); its 16-B chunk is swizzled by
// (hx >> 2) & 3.  A 32x32x16 fragment read takes 32 consecutive hx of one hy (lane -> hx0 + (lane
// & 31), chunk 2 ks + (lane >> 5)); for ANY hx0 the 4 rows of one residue class mod 4 inside a
// ds_read_b128 lane group are hx, hx+12, hx+20, hx+24 (or hx+4, hx+8, hx+16, hx+28), whose
// (hx >> 2) & 3 all differ: conflict-free (SQ_LDS_BANK_CONFLICT = 0).  Because the swizzle does
// not depend on hy, a tap's row shift (dy) is a plain immediate offset of K6_HROWB bytes.
SNRSE_DEV int hswz(int hy, int hx, int chunk) { return hy * K6_HROWB + hx * 64 + ((chunk ^ ((hx >> 2) & 3)) << 4); }
// Weight slot image: row = output channel, same swizzle by (co >> 2) & 3.
SNRSE_DEV int wswz(int co, int chunk) { return co * 64 + ((chunk ^ ((co >> 2) & 3)) << 4); }

SNRSE_DEV void glds16(rsrc_t r, char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}
SNRSE_DEV void glds4(rsrc_t r, char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 4, voff, 0, 0, 0);
}

// s_waitcnt needs an immediate: the (wave-uniform) counts the pipeline produces, the steady one
// first; any other count waits for everything, which is always safe
#define K6_W(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")
SNRSE_DEV void wait_vm(int n) {
  if (n == 4) K6_W(4);
  else if (n >= K6_SKIP) {}
  else if (n == 10) K6_W(10);
  else if (n == 11) K6_W(11);
  else if (n == 2) K6_W(2);
  else if (n == 8) K6_W(8);
  else if (n == 16) K6_W(16);
  else K6_W(0);
}
#undef K6_W

// A copy of v the compiler cannot see through: per-lane address math derived from it is redone
// where it is used instead of being hoisted into dozens of loop-invariant VGPRs (which would leave
// too few registers to keep both k-steps' fragments of a tap in flight).
SNRSE_DEV int opaque(int v) {
  int r;
  asm volatile("v_mov_b32 %0, %1" : "=v"(r) : "v"(v));
  return r;
}

SNRSE_DEV void sync_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
}

SNRSE_DEV f32x16 mfma32(const u32x4& a, const u32x4& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf16x8_mfma, a), __builtin_bit_cast(bf16x8_mfma, b),
                                                  c, 0, 0, 0);
}

struct Tile6 {
  int b, h0, w0, n0;
};

// phase cursor: local tile, chunk, phase-in-chunk
struct Cur6 {
  int lt, c, pi;
};

__global__ __launch_bounds__(256, 2) void conv_halo6_kernel(ConvParams p, int T) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int fr = lane & 31, fh = lane >> 5;
#ifdef SNRSE_STAMPS
  unsigned long long* const lst = (unsigned long long*)(smem + K6_LDS) + wid * 32;
#endif
  SNRSE_STAMP(0);
  const int G = gridDim.x, g = blockIdx.x;
  const int t_begin = (int)(((long long)g * T) / G);
  const int ntile = (int)(((long long)(g + 1) * T) / G) - t_begin;
  if (ntile <= 0) return;

  const int Cin = p.C0 + p.C1;
  const int ncm = Cin >> 5;
  const int Csc_all = p.Csc + p.Csc1;
  const int ncs = p.sc_src ? (Csc_all >> 5) : 0;
  const int nchunk = ncm + ncs;
  const int ntw = p.W / K6_TW, nth = p.H / K6_TH;
  const bool has_gn = p.gn_scale != nullptr;
  const int K1 = 9 * Cin;

  // ---- per-lane address bases (loop invariant)
  // A fragment of (ks, tap column dx) for the wave's first output row: + (mi + dy) * K6_HROWB + halo
  // buffer (recomputed per chunk, see a_bases)
  auto a_bases = [&](int (&ab)[3][2], int hb) {
#pragma unroll
    for (int dx = 0; dx < 3; ++dx)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) ab[dx][ks] = hb * K6_HBUF + hswz(2 * wid, fr + dx, 2 * ks + fh);
  };
  // B fragment of (ks): + slot * K6_TAPB + nj * 2048 (rows 32 nj + fr share the swizzle of fr)
  int bbase[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) bbase[ks] = K6_OFF_W + wswz(fr, 2 * ks + fh);
  // weight LDS-DMA source offsets of this lane's two 1-KB pieces (main / shortcut row strides)
  const int wrow = wid * 16 + (lane >> 2);  // piece 0 row; piece 1 is row + 64 (same swizzle)
  const int wdc8 = (((lane & 3) ^ ((wrow >> 2) & 3)) * 8) * 2;
  const int wl_m0 = wrow * K1 * 2 + wdc8, wl_m1 = wl_m0 + 64 * K1 * 2;
  const int wl_s0 = wrow * Csc_all * 2 + wdc8, wl_s1 = wl_s0 + 64 * Csc_all * 2;

  auto tile_of = [&](int lt) {
    int t = t_begin + lt;
    Tile6 r;
    r.w0 = (t % ntw) * K6_TW;
    t /= ntw;
    r.h0 = (t % nth) * K6_TH;
    t /= nth;
    r.n0 = (t % p.ntn) * 128;
    r.b = t / p.ntn;
    return r;
  };
  auto advance = [&](Cur6 q) {
    const int np = q.c < ncm ? 9 : 1;
    if (++q.pi == np) {
      q.pi = 0;
      if (++q.c == nchunk) {
        q.c = 0;
        ++q.lt;
      }
    }
    return q;
  };

  // ---- raw halo of chunk c of tile tl -> halo buffer hb, + its GroupNorm affine (waves 2, 3 --
  // the same 256 bytes twice, so that every wave issues exactly K6_HOPS operations)
  auto halo_issue = [&](const Tile6& tl, int c, int hb) {
    const int lane = opaque(tid) & 63;
    const void* base;
    long long bytes;
    int cs, ch;
    if (c < ncm) {
      ch = c * 32;
      if (ch < p.C0) { base = p.src0; bytes = p.bytes0; cs = p.C0; }
      else { base = p.src1; bytes = p.bytes1; cs = p.C1; ch -= p.C0; }
    } else {
      ch = (c - ncm) * 32;
      if (ch < p.Csc) { base = p.sc_src; bytes = p.sc_bytes0; cs = p.Csc; }
      else { base = p.sc_src1; bytes = p.sc_bytes1; cs = p.Csc1; ch -= p.Csc; }
    }
    const rsrc_t r = make_rsrc(base, bytes);
    char* dst = smem + hb * K6_HBUF;
    const int pix0 = (tl.b * p.H + tl.h0 - 1) * p.W + tl.w0 - 1;  // halo (0, 0)
#pragma unroll
    for (int j = 0; j < 5; ++j) {
      const int k = wid + 4 * j;
      const int row = k * 16 + (lane >> 2);
      const int hy = row / K6_HC, hx = row - hy * K6_HC;
      const int dc = (lane & 3) ^ ((hx >> 2) & 3);
      const unsigned ih = (unsigned)(tl.h0 + hy - 1), iw = (unsigned)(tl.w0 + hx - 1);
      const bool ok = ih < (unsigned)p.H && iw < (unsigned)p.W;
      const int voff = ok ? (((pix0 + hy * p.W + hx) * cs + ch + dc * 8) * 2) : (int)0x80000000;
      glds16(r, dst + k * 1024, voff);
    }
    if (wid < 2) {  // pieces 20, 21
      const int k = 20 + wid;
      const int row = k * 16 + (lane >> 2);
      const int hy = row / K6_HC, hx = row - hy * K6_HC;
      const int dc = (lane & 3) ^ ((hx >> 2) & 3);
      const unsigned ih = (unsigned)(tl.h0 + hy - 1), iw = (unsigned)(tl.w0 + hx - 1);
      const bool ok = row < K6_HROWS && ih < (unsigned)p.H && iw < (unsigned)p.W;
      const int voff = ok ? (((pix0 + hy * p.W + hx) * cs + ch + dc * 8) * 2) : (int)0x80000000;
      glds16(r, dst + k * 1024, voff);
    } else {
      // gn_shift == gn_scale + B*Cin (checked by the launcher): one resource covers both;
      // lanes 0..31 fetch the 32 scales, lanes 32..63 the 32 shifts (zeros when no GroupNorm)
      const bool gnc = has_gn && c < ncm;
      const rsrc_t rg = gnc ? make_rsrc(p.gn_scale, 8LL * p.B * Cin) : make_rsrc(p.out, 0);
      const int voff = gnc ? (((lane < 32 ? tl.b : p.B + tl.b) * Cin + c * 32 + (lane & 31)) * 4) : 0;
      glds4(rg, smem + K6_OFF_GN + hb * K6_GNB, voff);
    }
  };
  // ---- bias (waves 0, 1) and temb (waves 2, 3) slices of tile tl -> EP: one op per wave
  auto ep_issue = [&](const Tile6& tl) {
    const int lane = opaque(tid) & 63;
    const bool bw = wid < 2;
    const bool have = bw ? p.bias != nullptr : p.temb != nullptr;
    const rsrc_t r = !have ? make_rsrc(p.out, 0)
                     : bw  ? make_rsrc(p.bias + tl.n0, 512)
                           : make_rsrc(p.temb + (size_t)tl.b * p.temb_stride + tl.n0, 512);
    glds4(r, smem + K6_OFF_EP + wid * 256, ((wid & 1) * 64 + lane) * 4);
  };
  // ---- one tap's weights (128 co x 32 ch) of phase (tl, c, pi) -> ring slot s
  auto w_issue = [&, wl_m0, wl_m1, wl_s0, wl_s1](const Tile6& tl, int c, int pi, int s) {
    char* dst = smem + K6_OFF_W + s * K6_TAPB + wid * 1024;
    const bool mainw = c < ncm;
    const rsrc_t r = mainw ? make_rsrc(p.wgt, p.wbytes) : make_rsrc(p.sc_wgt, p.sc_wbytes);
    const int so = mainw ? (tl.n0 * K1 + pi * Cin + c * 32) * 2 : (tl.n0 * Csc_all + (c - ncm) * 32) * 2;
    const int o0 = mainw ? wl_m0 : wl_s0, o1 = mainw ? wl_m1 : wl_s1;
    glds16(r, dst, o0 + so);
    glds16(r, dst + 4096, o1 + so);
  };

  // ---- in-place GroupNorm(+SiLU) of halo row (tid >> 2) + 64 ri, channels 8 (tid & 3) .. +8.
  // Branch-free (so the compiler can interleave it with the tap's MFMAs): rows past the halo
  // (ri = 5, rows 340..383) are clamped onto pad row 351, which no fragment reads; rows outside
  // the image keep their zero padding through the select.
  struct TRow {
    int a;  // LDS byte offset (a pointer here would lose its address space and go through flat ops)
    bool ok;
    u32x4 v;
    f32x4 s0, s1, t0, t1;
  };
  auto trow_load = [&](const Tile6& tl, int hb, int ri) {
    TRow t;
    const int tq = opaque(tid), tdc = tq & 3;
    const int r0 = (tq >> 2) + 64 * ri;
    const int r = r0 < K6_NPIECE * 16 ? r0 : K6_NPIECE * 16 - 1;
    const int hy = r / K6_HC, hx = r - hy * K6_HC;
    const unsigned ih = (unsigned)(tl.h0 + hy - 1), iw = (unsigned)(tl.w0 + hx - 1);
    t.ok = r < K6_HROWS && ih < (unsigned)p.H && iw < (unsigned)p.W;
    t.a = hb * K6_HBUF + hswz(hy, hx, tdc);
    const float* gp = (const float*)(smem + K6_OFF_GN + hb * K6_GNB) + tdc * 8;
    t.s0 = *(const f32x4*)gp;
    t.s1 = *(const f32x4*)(gp + 4);
    t.t0 = *(const f32x4*)(gp + 32);
    t.t1 = *(const f32x4*)(gp + 36);
    t.v = *(const u32x4*)(smem + t.a);
    return t;
  };
  auto trow_store = [&](TRow& t, bool do_tr) {  // gn_act required (halo6_ok)
    const float gsc[8] = {t.s0[0], t.s0[1], t.s0[2], t.s0[3], t.s1[0], t.s1[1], t.s1[2], t.s1[3]};
    const float gsh[8] = {t.t0[0], t.t0[1], t.t0[2], t.t0[3], t.t1[0], t.t1[1], t.t1[2], t.t1[3]};
    u32x4 v = t.v;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const float lo = fmaf(__uint_as_float(v[i] << 16), gsc[2 * i], gsh[2 * i]);
      const float hi = fmaf(__uint_as_float(v[i] & 0xffff0000u), gsc[2 * i + 1], gsh[2 * i + 1]);
      v[i] = !do_tr ? v[i] : t.ok ? pack_bf16x2(silu(lo), silu(hi)) : 0u;
    }
    *(u32x4*)(smem + t.a) = v;
  };
  auto transform_row = [&](const Tile6& tl, int hb, int ri) {
    TRow t = trow_load(tl, hb, ri);
    trow_store(t, true);
  };

  float* const stl = (float*)(smem + K6_OFF_ST);  // [128 co][2] GroupNorm partial sums
  f32x16 acc[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};

  // ---- epilogue of tile tl; acc staged through this wave's slice of halo buffer hb.
  // acc[mi][nj] register e: co = 32 nj + (lane & 31), px = 8 (e >> 2) + 4 (lane >> 5) + (e & 3) of
  // image row h0 + 2 wid + mi.  Pass (mi, nj) stages 32 co x 32 px; lane = (px, 16-channel half).
  auto epilogue = [&](const Tile6& tl, int hb) {
    const int l31 = fr, lh = fh;
    float* const stg = (float*)(smem + hb * K6_HBUF + wid * K6_STAGE);
    const float* const ep = (const float*)(smem + K6_OFF_EP);
#pragma unroll
    for (int mi = 0; mi < 2; ++mi) {
      const size_t m = (size_t)(tl.b * p.H + tl.h0 + 2 * wid + mi) * p.W + tl.w0 + l31;  // this lane's pixel
#pragma unroll
      for (int nj = 0; nj < 4; ++nj) {
        const int nl = nj * 32 + lh * 16;  // tile-local first channel of this lane
        const int n = tl.n0 + nl;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const f32x4 q = {acc[mi][nj][4 * i], acc[mi][nj][4 * i + 1], acc[mi][nj][4 * i + 2], acc[mi][nj][4 * i + 3]};
          *(f32x4*)(stg + l31 * K6_LDR + 8 * i + 4 * lh) = q;
        }
        u32x4 r0 = {0u, 0u, 0u, 0u}, r1 = {0u, 0u, 0u, 0u};
        if (p.res) {
          const bf16_t* rp = (const bf16_t*)p.res + m * p.res_ld + n;
          r0 = *(const u32x4*)rp;
          r1 = *(const u32x4*)(rp + 8);
        }
        float v[16];
#pragma unroll
        for (int k4 = 0; k4 < 4; ++k4) {
          const f32x4 bv = *(const f32x4*)(ep + nl + 4 * k4);
          const f32x4 tv = *(const f32x4*)(ep + 128 + nl + 4 * k4);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[4 * k4 + e] = stg[(lh * 16 + 4 * k4 + e) * K6_LDR + l31] + (bv[e] + tv[e]);
        }
        if (p.res) {
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            v[2 * k] += __uint_as_float(r0[k] << 16);
            v[2 * k + 1] += __uint_as_float(r0[k] & 0xffff0000u);
            v[8 + 2 * k] += __uint_as_float(r1[k] << 16);
            v[8 + 2 * k + 1] += __uint_as_float(r1[k] & 0xffff0000u);
          }
        }
#pragma unroll
        for (int k = 0; k < 16; ++k) v[k] *= p.out_scale;
        u32x4 o0, o1;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          o0[k] = pack_bf16x2(v[2 * k], v[2 * k + 1]);
          o1[k] = pack_bf16x2(v[8 + 2 * k], v[8 + 2 * k + 1]);
        }
        bf16_t* op = (bf16_t*)p.out + m * p.out_ld + n;
        *(u32x4*)op = o0;
        *(u32x4*)(op + 8) = o1;
        if (p.stats) {
#pragma unroll
          for (int k = 0; k < 16; ++k) stg[(lh * 16 + k) * K6_LDR + l31] = v[k];
          const float* sp = stg + l31 * K6_LDR + lh * 16;  // channel l31, pixels 16 lh .. +16
          float s1 = 0.f, s2 = 0.f;
#pragma unroll
          for (int k = 0; k < 4; ++k) {
            const f32x4 a = *(const f32x4*)(sp + 4 * k);
#pragma unroll
            for (int e = 0; e < 4; ++e) { s1 += a[e]; s2 = fmaf(a[e], a[e], s2); }
          }
          s1 += __shfl_xor(s1, 32, 64);
          s2 += __shfl_xor(s2, 32, 64);
          if (lane < 32) {
            atomicAdd(stl + (nj * 32 + lane) * 2, s1);
            atomicAdd(stl + (nj * 32 + lane) * 2 + 1, s2);
          }
        }
      }
    }
  };

  // ---- one tap of the current chunk: 2 k-steps x 2 pixel blocks x 4 channel blocks = 16 MFMAs.
  // A fragments (halo) of tap t+1 are read during tap t (the halo is complete for the whole chunk);
  // B fragments (this tap's weight slot) right after the barrier that publishes them.
  auto load_a = [&](u32x4 (&af)[2][2], const int (&ab)[3][2], int dy, int dx) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi) af[ks][mi] = *(const u32x4*)(smem + ab[dx][ks] + (mi + dy) * K6_HROWB);
  };
  auto load_b = [&](u32x4 (&bfr)[2][4], int woff) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int nj = 0; nj < 4; ++nj) bfr[ks][nj] = *(const u32x4*)(smem + bbase[ks] + woff + nj * 2048);
  };
  auto mfma_tap = [&](const u32x4 (&af)[2][2], const u32x4 (&bfr)[2][4]) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int mi = 0; mi < 2; ++mi)
#pragma unroll
        for (int nj = 0; nj < 4; ++nj) acc[mi][nj] = mfma32(af[ks][mi], bfr[ks][nj], acc[mi][nj]);
  };
  // scheduler hint: one MFMA, then up to four VALU (the GroupNorm transform fills the MFMA gaps)
  auto interleave_hint = [&]() {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x002, 4, 0);  // VALU
    }
  };

  // ---- prologue: chunk 0 of the first tile, weights of phases 0, 1, 2
  stl[tid] = 0.f;
  Cur6 ahead = {0, 0, 0};
  Tile6 tcur = tile_of(0);
  halo_issue(tcur, 0, 0);
#pragma unroll 1
  for (int s = 0; s < K6_NSLOT - 1; ++s) {
    if (ahead.lt < ntile) w_issue(ahead.lt == 0 ? tcur : tile_of(ahead.lt), ahead.c, ahead.pi, s);
    ahead = advance(ahead);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  sync_lds();
  if (has_gn) {
#pragma unroll 1
    for (int ri = 0; ri < K6_TROWS; ++ri) transform_row(tcur, 0, ri);
  }
  sync_lds();
  SNRSE_STAMP(1);

  // ahead = phase Q+3 (the slice the current phase prefetches into slot (slot + 3) & 3)
  int gch = 0;       // chunks completed by this workgroup: halo buffer = gch & 1
  int slot = 0;      // weight ring slot of the current phase
  int prev_ops = 0;  // vector-memory ops the previous phase issued (K6_SKIP: all waited already)

#pragma unroll 1
  for (int lt = 0; lt < ntile; ++lt) {
    const bool has_nt = lt + 1 < ntile;
    const Tile6 tnt = has_nt ? tile_of(lt + 1) : tcur;
    Cur6 wdef = ahead;  // weight prefetch the tile's last phase defers past the epilogue
    int sdef = 0;

    // Phase prologue / epilogue shared by the main and the shortcut chunks.  `ops` counts this
    // wave's vector-memory operations of the current phase in issue order.
    auto w_step = [&](bool tile_last, int& ops) {
      const int s3 = (slot + 3) & 3;
      if (tile_last) {
        wdef = ahead;
        sdef = s3;
      } else if (ahead.lt < ntile) {
        w_issue(ahead.lt == lt ? tcur : tnt, ahead.c, ahead.pi, s3);
        ops += 2;
      }
    };
    auto end_phase = [&](bool tile_last, int n) {
      if (!tile_last) {
        wait_vm(n);
        sync_lds();
      }
      slot = (slot + 1) & 3;
      ahead = advance(ahead);
    };

#pragma unroll 1
    for (int c = 0; c < ncm; ++c) {  // ---- main chunks: 9 taps, unrolled
      const bool last_c = c + 1 == nchunk;
      const bool has_next = !last_c || has_nt;
      const int nc = last_c ? 0 : c + 1;
      const Tile6 tnext = last_c ? tnt : tcur;
      const bool next_gn = has_next && has_gn && nc < ncm;
      const int hb = gch & 1, hnext = hb ^ 1;
      int ab[3][2];
      a_bases(ab, hb);
      // Phases 3..8 each transform one halo row of the next chunk, straight-line: when the next
      // chunk takes no GroupNorm (shortcut source, no next chunk, or a conv without GN) the row
      // is written back unchanged, so the tap's MFMAs stay one block the compiler can interleave
      // the transform into (a branch around either would split the accumulator live ranges).
#pragma unroll
      for (int pi = 0; pi < 9; ++pi) {
        const bool tile_last = last_c && pi == 8;
        int ops = 0;
        if (pi == 0) {
          if (has_next) {
            halo_issue(tnext, nc, hnext);
            ops += K6_HOPS;
          }
          if (c == 0) {
            ep_issue(tcur);
            ops += 1;
          }
        }
        w_step(tile_last, ops);
        u32x4 af[2][2], bfr[2][4];
        load_b(bfr, slot * K6_TAPB);
        load_a(af, ab, pi / 3, pi % 3);
        if (pi >= 3) {
          // the halo issued at phase 0 has landed once phase 2's wait retired W(3), issued after it
          TRow t = trow_load(tnext, hnext, pi - 3);
          mfma_tap(af, bfr);
          trow_store(t, next_gn);
        } else {
          mfma_tap(af, bfr);
        }
        // W(Q+1) was the last op of phase Q-2: everything of phases Q-1 and Q may stay in flight
        const int n = prev_ops >= K6_SKIP ? K6_SKIP : prev_ops + ops;
        prev_ops = ops;
        end_phase(tile_last, n);
      }
      if (!last_c) ++gch;
    }
#pragma unroll 1
    for (int c = ncm; c < nchunk; ++c) {  // ---- shortcut chunks: centre tap only
      const bool last_c = c + 1 == nchunk;
      const bool has_next = !last_c || has_nt;
      const int nc = last_c ? 0 : c + 1;
      const Tile6 tnext = last_c ? tnt : tcur;
      const int hb = gch & 1;
      int ab[3][2];
      a_bases(ab, hb);
      int ops = 0;
      if (has_next) {
        halo_issue(tnext, nc, hb ^ 1);
        ops += K6_HOPS;
      }
      const int hops = ops;
      w_step(last_c, ops);
      {
        u32x4 af[2][2], bfr[2][4];
        load_b(bfr, slot * K6_TAPB);
        load_a(af, ab, 1, 1);
        mfma_tap(af, bfr);
      }
      // the next chunk reads the halo issued here: only this phase's weight slice may remain
      prev_ops = ops;
      end_phase(last_c, ops - hops);
      if (!last_c) ++gch;
    }

    // ---- end of the tile's last phase: everything issued so far (W(Q+1), W(Q+2), the next
    // tile's first halo) lands before the epilogue, so nothing issued ahead of the epilogue's
    // stores is waited for after them
    const bool deferred = has_nt && has_gn && ncs > 0;  // shortcut chunk last: transform the next halo now
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    sync_lds();  // every wave is done reading halo buffer gch & 1 (reused as staging)
#ifdef SNRSE_STAMPS
    if (lt < 13) SNRSE_STAMP(2 + 2 * lt);
#endif
    if (deferred) {
#pragma unroll 1
      for (int ri = 0; ri < K6_TROWS; ++ri) transform_row(tnt, (gch + 1) & 1, ri);
    }
    epilogue(tcur, gch & 1);
    if (p.stats && (!has_nt || tnt.b != tcur.b || tnt.n0 != tcur.n0)) {
      sync_lds();
      const int sl = blockIdx.x & (SNRSE_STAT_SLOTS - 1);
      const float a = stl[tid];
      stl[tid] = 0.f;
      unsafeAtomicAdd(&p.stats[stat_idx(tcur.b, sl, tcur.n0 + (tid >> 1), p.Cout) + (tid & 1)], (double)a);
    }
#ifdef SNRSE_STAMPS
    if (lt < 13) SNRSE_STAMP(3 + 2 * lt);
#endif
    // the deferred slice belongs to the next tile (every tile has >= 9 phases)
    if (wdef.lt < ntile) w_issue(tnt, wdef.c, wdef.pi, sdef);
    sync_lds();
    prev_ops = K6_SKIP;  // the next phase's W(Q+1) landed before the epilogue
    ++gch;
    tcur = tnt;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x16{};
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

bool halo6_ok(const ConvParams& p) {
  const int Cin = p.C0 + p.C1;
  if (p.ksize != 3 || p.H % K6_TH || p.W % K6_TW || p.Cout % 128 || p.B <= 0) return false;
  if (p.C0 % 32 || p.C1 % 32 || Cin <= 0) return false;
  if (p.sc_src && ((p.Csc + p.Csc1) % 32 || p.Csc % 32 || p.Csc1 % 32)) return false;
  if (p.comb_src) return false;  // Combine epilogues stay on the v4/v5 kernels
  if (p.out_ld % 8 || (p.res && p.res_ld % 8)) return false;
  if (p.gn_scale && (p.gn_shift != p.gn_scale + (size_t)p.B * Cin || !p.gn_act)) return false;
  const long long lim = 0x7ff00000ll;
  if (p.bytes0 >= lim || p.bytes1 >= lim || p.sc_bytes0 >= lim || p.sc_bytes1 >= lim || p.wbytes >= lim ||
      p.sc_wbytes >= lim || 8LL * p.B * Cin >= lim)
    return false;
  return true;
}

int launch_halo6(const ConvParams& p0, hipStream_t s) {
  ConvParams p = p0;
  if (!halo6_ok(p)) return SNRSE_EINVAL;
  p.ntn = p.Cout / 128;
  const int T = p.B * (p.H / K6_TH) * (p.W / K6_TW) * p.ntn;
#ifdef SNRSE_STAMPS
  constexpr size_t lds = K6_LDS + 4 * 32 * 8;
#else
  constexpr size_t lds = K6_LDS;
#endif
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    SNRSE_RET(hipGetDevice(&dev));
    SNRSE_RET(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    SNRSE_RET(hipFuncSetAttribute((const void*)conv_halo6_kernel, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
  }
  const int G = T < 2 * ncu ? T : 2 * ncu;
  hipLaunchKernelGGL(conv_halo6_kernel, dim3(G), dim3(256), lds, s, p, T);
  return (int)hipGetLastError();
}

}  // namespace snrse_conv
