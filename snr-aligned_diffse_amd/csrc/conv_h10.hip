// v10 halo GEMM for the bf16 3x3 ResBlock convolutions (reference: ResnetBlockBigGANpp.Conv_0 / Conv_1,
// sgmse/backbones/ncsnpp_utils/layerspp.py:244-276, ddpm_conv3x3 layers.py:100-124; GroupNorm+SiLU prologue
// layerspp.py:258-266).
//
// Structure (one workgroup of 4 waves per CU, one wave per SIMD, up to 512 registers per wave, persistent):
//   * workgroup tile 16 image rows x 32 px = 512 px x 128 couts; wave w computes px half (w & 1) = 8 rows x 32 px
//     and cout half (w >> 1) = 64 couts: 16 x 4 blocks of v_mfma_f32_16x16x32_bf16 = 256 accumulators, computed
//     as D'[cout][px] (weights are the A operand) so that a lane ends with 4 consecutive couts of one pixel and the
//     epilogue stores 8-byte vectors straight from registers (no LDS staging);
//   * K runs in 32-channel chunks x 9 taps; the chunk's halo (18 x 34 rows x 64 B = 39 KB, swizzled 16-B chunks)
//     sits in one of two LDS buffers while the NEXT chunk's halo (of this tile, or of the workgroup's next tile) is
//     loaded, GroupNorm+SiLU-transformed and stored into the other one, a few vectors per tap between the MFMAs of
//     the current chunk -- the transform uses the issue slots the matrix pipe leaves free instead of a VALU-only
//     stretch at the chunk boundary (v5);
//   * weight fragments come straight from global memory (L2-resident, 295 KB per 128->128 layer) into registers,
//     one tap ahead; halo fragments are read from LDS four 16-px blocks ahead, across tap boundaries;
//   * one barrier per chunk (the halo buffers swap); the 512-px tile has 612 halo rows (1.20 x the tile, against
//     1.33 x for v5's 256-px tiles), so there is 10 % less GroupNorm+SiLU work per output.
//   * a fused 1x1 shortcut (Conv_2 as extra K, layerspp.py:268-274) runs as one-tap chunks over an unpadded pixel
//     tile (512 rows x 64 B) in two more LDS buffers: up to two such chunks right before each main chunk, their tiles
//     loaded during the previous main chunk (so at most 2 shortcut chunks per main chunk: nsc <= 2 ncb).
// Shapes: H % 16 == 0, W % 32 == 0, Cout % 128 == 0, shortcut channels <= 2 x main channels.
#include "conv_common.h"

#include <utility>

using namespace snrse_conv;

namespace {
namespace h10 {
constexpr int TH = 16, TW = kH10TileW, HC = TW + 2;
constexpr int HROWS = (TH + 2) * HC;     // 612
constexpr int HBYTES = HROWS * 64;       // 39168
constexpr int VPT = (HROWS * 4 + 255) / 256;  // 10 halo vectors (16 B) per thread: vector tid + 256 k
constexpr int SCBYTES = TH * TW * 64;  // a shortcut chunk's pixel tile (no halo): 512 rows x 64 B
constexpr int SCOFF = 2 * HBYTES;       // two halo buffers, then two shortcut tiles
constexpr int SCV = TH * TW * 4 / 256;  // 8 shortcut vectors per thread per chunk
constexpr int LDS = 2 * HBYTES + 2 * SCBYTES;  // 143,872 B
constexpr int KT = 32;
// the next chunk's halo, vector k (k = 0 .. VPT-1): loaded at 16-px step LOAD0 + STRIDE k (a step = 4 MFMAs),
// transformed over NSLOT consecutive steps from XF0 + STRIDE k (one slice of VALU work beside each MFMA), stored at
// the end of its last slot; 9 taps x 16 steps = 144 steps per chunk
constexpr int STRIDE = 10, XF0 = 40, LOAD0 = XF0 - 32;
static_assert(XF0 + STRIDE * (VPT - 1) + 9 <= 144, "transform schedule fits one chunk");
// up to two shortcut chunks' tiles (2 x 8 vectors per thread) loaded every SCSTRIDE steps from SCL0, stored SCLAG later
constexpr int SCSTRIDE = 6, SCL0 = 4, SCLAG = 30;
static_assert(SCL0 + SCSTRIDE * 15 + SCLAG < 144, "shortcut schedule fits one chunk");

// single VALU instructions as asm statements: with the MFMAs also in asm (program order of volatile asm is kept),
// the interleave below is the issue order -- the compiler neither hoists the transform into a VALU-only block nor
// moves it across the MFMAs (operands are registers only; no wait states needed between these and the MFMAs)
SNRSE_DEV float a_lshl16(uint32_t s) { float d; asm volatile("v_lshlrev_b32 %0, 16, %1" : "=v"(d) : "v"(s)); return d; }
SNRSE_DEV float a_andhi(uint32_t s) { float d; asm volatile("v_and_b32 %0, 0xffff0000, %1" : "=v"(d) : "v"(s)); return d; }
SNRSE_DEV void a_fma(float& d, float b, float c) { asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(d) : "v"(b), "v"(c)); }
SNRSE_DEV float a_exp(float s) { float d; asm volatile("v_exp_f32 %0, %1" : "=v"(d) : "v"(s)); return d; }
// e * (-1/ln2) + (-1/ln2): 0xbfb8aa3b = -log2(e) = -1/ln(2) (kNegInvLn2), k holds the same value
SNRSE_DEV void a_fmamk(float& d, float k) { asm volatile("v_fmamk_f32 %0, %0, 0xbfb8aa3b, %1" : "+v"(d) : "v"(k)); }
SNRSE_DEV void a_rcp(float& d) { asm volatile("v_rcp_f32 %0, %0" : "+v"(d)); }
SNRSE_DEV void a_mul(float& d, float s) { asm volatile("v_mul_f32 %0, %0, %1" : "+v"(d) : "v"(s)); }
SNRSE_DEV uint32_t a_cvtpk(float a, float b) {
  uint32_t d;
  asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(d) : "v"(a), "v"(b));
  return d;
}
SNRSE_DEV void a_and(uint32_t& d, uint32_t m) { asm volatile("v_and_b32 %0, %0, %1" : "+v"(d) : "v"(m)); }
SNRSE_DEV void a_mfma(f32x4& acc, const u32x4& w, const u32x4& h) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(w), "v"(h));
}
}  // namespace h10

// SC: the launch has shortcut chunks (without: no shortcut registers or loads at all)
template <int GNM, int EF, bool SC>
__global__ __launch_bounds__(256, 1) void conv_halo10_kernel(ConvParams p, int ntiles) {
  using namespace h10;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int ph = wid & 1, chh = wid >> 1;
  const int lrow = lane & 15, lg = lane >> 4;

  // contiguous tile range per workgroup; workgroups that share an XCD (blockIdx % 8) take neighbouring ranges
  const int nb = gridDim.x, bid = blockIdx.x;
  const int q8 = nb >> 3, r8 = nb & 7, xcd = bid & 7, pos = bid >> 3;
  const int g = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + pos;
  const int t_begin = (int)((long long)g * ntiles / nb), t_end = (int)((long long)(g + 1) * ntiles / nb);
  if (t_begin >= t_end) return;

  const int H = p.H, W = p.W;
  const int ntw = W / TW, nth = H / TH;
  const int Cin = p.C0 + p.C1, ncb = Cin / KT, K1 = 9 * Cin;
  // fused 1x1 shortcut (Conv_2 as extra K): nsc chunks of 32 channels, the ones of group m (sb(m) .. sb(m + 1) - 1,
  // at most 2) run right before main chunk m, their pixel tiles prepared during main chunk m - 1
  const int Csc_all = SC && p.sc_src ? p.Csc + p.Csc1 : 0, nsc = Csc_all / KT;
  auto sb = [&](int m) { return m * nsc / ncb; };
  const bool f_temb = EF < 0 ? p.temb != nullptr : (EF & EF_TEMB) != 0;
  const bool f_res = EF < 0 ? p.res != nullptr : (EF & EF_RES) != 0;
  const bool f_comb = EF < 0 ? p.comb_src != nullptr : (EF & EF_COMB) != 0;
  const bool f_stats = EF < 0 ? p.stats != nullptr : (EF & EF_STATS) != 0;
  const bool f_nt = EF < 0 ? p.epi_nt != 0 : (EF & EF_NT) != 0;

  const __amdgpu_buffer_rsrc_t rw = make_rsrc(p.wgt, p.wbytes);
  const __amdgpu_buffer_rsrc_t rws = make_rsrc(nsc ? p.sc_wgt : p.wgt, nsc ? p.sc_wbytes : p.wbytes);
  const __amdgpu_buffer_rsrc_t rs0 = make_rsrc(p.src0, p.bytes0);
  const __amdgpu_buffer_rsrc_t rs1 = make_rsrc(p.C1 ? p.src1 : p.src0, p.C1 ? p.bytes1 : p.bytes0);
  const __amdgpu_buffer_rsrc_t rc0 = make_rsrc(nsc ? p.sc_src : p.src0, nsc ? p.sc_bytes0 : p.bytes0);
  const __amdgpu_buffer_rsrc_t rc1 = make_rsrc(p.Csc1 && nsc ? p.sc_src1 : p.src0, p.Csc1 && nsc ? p.sc_bytes1 : p.bytes0);

  // ---- halo fragment addresses: row hr of a buffer at hr * 64 + ((lg ^ ((hr >> 1) & 3)) << 4).  Fragment i of tap
  // (dy, dx) reads row R0 + k with R0 = ph * 8 * HC + lrow and k = ((i >> 1) + dy + 1) * HC + (i & 1) * 16 + dx + 1;
  // the swizzle term depends on (R0 + k) mod 8 = (lrow + k) mod 8 only (8 * HC = 272 = 0 mod 8), so 8 per-lane bases
  // (k mod 8) plus the immediate (k / 8) * 512 address every fragment
  int hb[8];
#pragma unroll
  for (int m = 0; m < 8; ++m) {
    const int r = ph * 8 * HC + lrow + m;
    hb[m] = r * 64 + ((lg ^ ((r >> 1) & 3)) << 4);
  }
  // shortcut tile rows: pixel block i of the wave = rows ph * 256 + 16 i + lrow, swizzle (lrow >> 1) & 3
  const int scb = SCOFF + (ph * 256 + lrow) * 64 + ((lg ^ ((lrow >> 1) & 3)) << 4);

  // ---- per-thread halo vectors of a tile: row (tid >> 2) + 64 k, 16-B chunk tid & 3 (8 channels)
  const int hcol = tid & 3;
  // pixel index of each vector; outside the image (the conv's zero padding) or past the halo: -1.  Branch-free
  // (unsigned range tests, no short-circuit): per-vector exec masks would pin 20 SGPRs across the main loop.  A
  // vector past the halo (only k = VPT - 1 can be) gets a column beyond any image (hx = 1 << 20), so it takes the
  // out-of-range path (its buffer load reads zeros without touching memory, its store is skipped)
  int hyx[VPT];  // halo row / column of vector k: hy * 64 + hx
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int hr = (tid >> 2) + 64 * k;
    const int hy = hr / HC;
    hyx[k] = hr < HROWS ? hy * 64 + (hr - hy * HC) : 1 << 26;
  }
  int hpix[VPT];
  int spix = 0;  // shortcut tile: pixel of this thread's vector r = 0 (vector r: + 2 r W)
  auto halo_geom = [&](int b, int h0, int w0) {
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int ih = h0 + (hyx[k] >> 6) - 1, iw = w0 + (hyx[k] & 63) - 1;  // (past the halo: ih >= 2^20 > H)
      const bool ok = ((unsigned)ih < (unsigned)H) & ((unsigned)iw < (unsigned)W);
      hpix[k] = ok ? (b * H + ih) * W + iw : -1;
    }
    spix = (b * H + h0 + (tid >> 7)) * W + w0 + ((tid >> 2) & 31);
  };
  auto tile_coords = [&](int t, int& n0, int& b, int& h0, int& w0) {
    n0 = (t % p.ntn) * 128;
    t /= p.ntn;
    w0 = (t % ntw) * TW;
    t /= ntw;
    h0 = (t % nth) * TH;
    b = t / nth;
  };

  int gc = -1;  // main chunks done by this workgroup (halo buffer parity); -1 in the prologue
  // ---- state of the group being prepared: its shortcut chunks (first pu0, count pn) and its main chunk pc
  u32x4 hv[VPT];
  u32x4 sv[SC ? 2 * SCV : 1];
  float gsc[8], gsh[8];
  int pc_ch = 0;       // first channel of the main chunk
  bool pc_src1 = false;
  int pc_buf = 0;      // halo buffer it goes to
  int pu0 = 0, pn = 0;
  auto prep_begin = [&](int c, int b) {  // main chunk c of the tile whose geometry is in hpix / spix
    pc_ch = c * KT;
    pc_src1 = pc_ch >= p.C0;
    pu0 = sb(c);
    pn = sb(c + 1) - pu0;
    if constexpr (GNM > 0) {
      const float* s = p.gn_scale + (size_t)b * Cin + pc_ch + hcol * 8;
      const float* t = p.gn_shift + (size_t)b * Cin + pc_ch + hcol * 8;
      const f32x4 s0 = *(const f32x4*)s, s1 = *(const f32x4*)(s + 4);
      const f32x4 t0 = *(const f32x4*)t, t1 = *(const f32x4*)(t + 4);
      const float pre = GNM == 2 ? kNegLog2e : 1.f;  // gn_xform8<2> takes the -log2(e)-prescaled affine
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        gsc[i] = s0[i] * pre; gsc[4 + i] = s1[i] * pre;
        gsh[i] = t0[i] * pre; gsh[4 + i] = t1[i] * pre;
      }
    }
  };
  auto prep_load = [&](int k) {
    const int cs = pc_src1 ? p.C1 : p.C0;
    const int cc = (pc_src1 ? pc_ch - p.C0 : pc_ch) + hcol * 8;
    const int voff = hpix[k] >= 0 ? (hpix[k] * cs + cc) * 2 : (int)0x80000000;
#ifdef H10_EXP_NOHALOLOAD  // timing diagnostics only (results wrong): no halo loads after the prologue
    if (gc >= 0) { hv[k] = u32x4{(uint32_t)voff, 0u, 0u, 0u}; return; }
#endif
    hv[k] = __builtin_amdgcn_raw_buffer_load_b128(pc_src1 ? rs1 : rs0, voff, 0, 0);
  };
  auto prep_store = [&](int k) {  // (prologue: the whole transform at once)
    const int hr = (tid >> 2) + 64 * k;
    if (k == VPT - 1 && hr >= HROWS) return;
    u32x4 v = hv[k];
    if constexpr (GNM > 0) v = gn_xform8<GNM>(v, gsc, gsh, hpix[k] >= 0);
    *(u32x4*)(smem + pc_buf * HBYTES + swz64(hr, hcol)) = v;
  };
  // shortcut vector q of the group: chunk pu0 + q / SCV, tile row (tid >> 2) + 64 (q % SCV); no transform (raw x)
  auto sc_load = [&](int q) {
    if constexpr (!SC) return;
    // (always issued -- past the group's last shortcut chunk it re-reads its first one, a valid address -- so sv[q] is
    // defined on every path and no shortcut vector stays live across the loops)
    const int ch = (q / SCV < pn ? pu0 + q / SCV : pu0) * KT;
    const bool one = ch >= p.Csc;
    const int cs = one ? p.Csc1 : p.Csc;
    const int pix = spix + 2 * (q % SCV) * W;
#ifdef H10_EXP_NOSCLOAD
    if (gc >= 0) { sv[q] = u32x4{(uint32_t)pix, (uint32_t)ch, 0u, 0u}; return; }
#endif
    sv[q] = __builtin_amdgcn_raw_buffer_load_b128(one ? rc1 : rc0, (pix * cs + (one ? ch - p.Csc : ch) + hcol * 8) * 2, 0, 0);
  };
  auto sc_store = [&](int q) {
    if constexpr (!SC) return;
    if (q / SCV >= pn) return;
    *(u32x4*)(smem + SCOFF + (q / SCV) * SCBYTES + swz64((tid >> 2) + 64 * (q % SCV), hcol)) = sv[q];
  };
  // the transform in slots beside the MFMAs of one 16-px step each (xf_slice(step, mfma j) emits the VALU that
  // follows MFMA j): GNM 2: unpack, affine, exp x2, fma, rcp x2, mul, pack + mask (9 slots); GNM 1: unpack, affine,
  // pack + mask; GNM 0: the raw vector is stored (its padding is zero already: out-of-range buffer loads read 0)
  constexpr int NSLOT = GNM == 2 ? 9 : GNM == 1 ? 3 : 1;
  float xy[8], xe[8];
  uint32_t xo[4];
  const float knl2 = kNegInvLn2;
  // slice (ST, J): the VALU issued after MFMA J of step ST (compile-time: every index is a constant)
  auto xf_slice = [&](auto ST, auto J) {
    constexpr int st = decltype(ST)::value, j = decltype(J)::value;
#ifdef H10_EXP_NOXF
    if constexpr (false)
#else
    if constexpr (GNM > 0 && st >= XF0 && (st - XF0) % STRIDE < NSLOT && (st - XF0) / STRIDE < VPT)
#endif
    {
      constexpr int k = (st - XF0) / STRIDE, sl = (st - XF0) % STRIDE;
      constexpr int slot = GNM == 2 ? sl : (sl == 2 ? 8 : sl);  // GNM 1: unpack, affine, pack
      constexpr int e0 = 2 * j, e1 = 2 * j + 1;
      if constexpr (slot == 0) { xy[e0] = a_lshl16(hv[k][j]); xy[e1] = a_andhi(hv[k][j]); }
      if constexpr (slot == 1) { a_fma(xy[e0], gsc[e0], gsh[e0]); a_fma(xy[e1], gsc[e1], gsh[e1]); }
#ifdef H10_EXP_XF_CHEAP  // timing diagnostics only: full-rate multiplies in place of the transcendentals
      if constexpr (slot == 2) { xe[j] = xy[j]; a_mul(xe[j], xy[j]); }
      if constexpr (slot == 3) { xe[4 + j] = xy[4 + j]; a_mul(xe[4 + j], xy[4 + j]); }
      if constexpr (slot == 5) a_mul(xe[j], xy[j]);
      if constexpr (slot == 6) a_mul(xe[4 + j], xy[4 + j]);
#else
      if constexpr (slot == 2) xe[j] = a_exp(xy[j]);
      if constexpr (slot == 3) xe[4 + j] = a_exp(xy[4 + j]);
      if constexpr (slot == 4) { a_fmamk(xe[e0], knl2); a_fmamk(xe[e1], knl2); }
      if constexpr (slot == 5) a_rcp(xe[j]);
      if constexpr (slot == 6) a_rcp(xe[4 + j]);
#endif
      if constexpr (slot == 7) { a_mul(xy[e0], xe[e0]); a_mul(xy[e1], xe[e1]); }
      if constexpr (slot == 8) {
        xo[j] = a_cvtpk(xy[e0], xy[e1]);
        a_and(xo[j], hpix[k] >= 0 ? 0xffffffffu : 0u);  // the conv's zero padding
      }
    }
  };
  auto xf_store = [&](int k) {
    const int hr = (tid >> 2) + 64 * k;
    u32x4 v;
    if constexpr (GNM > 0) v = u32x4{xo[0], xo[1], xo[2], xo[3]};
    else v = hv[k];
    if (k < VPT - 1 || hr < HROWS) *(u32x4*)(smem + pc_buf * HBYTES + swz64(hr, hcol)) = v;
  };

  // ---- weight fragments (A operand): cout row n0 + chh * 64 + 16 j + lrow, 8 channels at lg * 8 of K offset koff;
  // main chunk c, tap t: [Cout][9 Cin] at t Cin + 32 c; shortcut chunk u: [Cout][Csc_all] at 32 u
  auto wload = [&](u32x4 (&wf)[4], int n0, bool sc, int tap, int c) {
    const int ld = sc ? Csc_all : K1;
    const int vb = ((n0 + chh * 64 + lrow) * ld + lg * 8) * 2;
    const int koff = ((sc ? 0 : tap * Cin) + c * KT) * 2;
#ifdef H10_EXP_NOWLOAD
    if (gc >= 0) return;
#endif
#pragma unroll
    for (int j = 0; j < 4; ++j)
      wf[j] = __builtin_amdgcn_raw_buffer_load_b128(sc ? rws : rw, vb, j * 16 * ld * 2 + koff, 0);
  };

  f32x4 acc[16][4];
  u32x4 wcur[4], wnext[4];

  // ---- prologue: the first tile's group 0 (shortcut chunks + main chunk 0), synchronously
  int n0, bb, h0, w0;
  tile_coords(t_begin, n0, bb, h0, w0);
  halo_geom(bb, h0, w0);
  prep_begin(0, bb);
  pc_buf = 0;
#pragma unroll
  for (int k = 0; k < VPT; ++k) prep_load(k);
#pragma unroll
  for (int q = 0; q < (SC ? 2 * SCV : 0); ++q) sc_load(q);
#pragma unroll
  for (int k = 0; k < VPT; ++k) prep_store(k);
#pragma unroll
  for (int q = 0; q < (SC ? 2 * SCV : 0); ++q) sc_store(q);
  wload(wnext, n0, pn > 0, 0, pn > 0 ? pu0 : 0);
  gc = 0;

  for (int t = t_begin; t < t_end; ++t) {
    tile_coords(t, n0, bb, h0, w0);
#pragma unroll
    for (int i = 0; i < 16; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    int nn0 = n0;  // cout tile of the weights loaded for the next tap
    for (int c = 0; c < ncb; ++c) {
      // ---- the shortcut chunks of group c (their tiles in the two shortcut buffers), one tap each
      const int u_end = sb(c + 1);
      for (int u = sb(c); u < u_end; ++u) {
        const int sbuf = u - sb(c);
        const bool nxt_sc = u + 1 < u_end;  // the next chunk: shortcut u + 1, else main chunk c (tap 0)
        if (sbuf == 0) {  // both shortcut tiles of the group were stored during the previous main chunk: one barrier
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __builtin_amdgcn_s_barrier();
        }
        u32x4 sf[16];
        auto sread = [&](int i) { sf[i] = *(const u32x4*)(smem + scb + sbuf * SCBYTES + i * 1024); };
#pragma unroll
        for (int i = 0; i < 4; ++i) sread(i);
#pragma unroll
        for (int j = 0; j < 4; ++j) wcur[j] = wnext[j];
        wload(wnext, n0, nxt_sc, 0, nxt_sc ? u + 1 : c);
        static_for<16>([&](auto I) {
          constexpr int i = decltype(I)::value;
          if constexpr (i + 4 < 16) sread(i + 4);
          static_for<4>([&](auto J) {
            constexpr int j = decltype(J)::value;
            if constexpr (i == 0 && j == 0) asm volatile("s_nop 1" ::: "memory");
            a_mfma(acc[i][j], wcur[j], sf[i]);
          });
          __builtin_amdgcn_sched_barrier(0);
        });
      }
      // ---- main chunk c; prepared meanwhile: group c + 1 of this tile, or group 0 of the next tile; after the
      // workgroup's last chunk, a dummy one (every vector out of range: zeros into free buffers, read by nobody), so
      // the step sequence below has no branches
      const bool last_c = c + 1 == ncb;
      int pb = bb;
      if (last_c) {
        if (t + 1 < t_end) {
          int h0n, w0n;
          tile_coords(t + 1, nn0, pb, h0n, w0n);
          halo_geom(pb, h0n, w0n);  // (this chunk's halo is already in LDS)
        } else {
#pragma unroll
          for (int k = 0; k < VPT; ++k) hpix[k] = -1;
        }
      }
      prep_begin(last_c ? 0 : c + 1, pb);
      pc_buf = (gc + 1) & 1;
      const bool nsc_next = pn > 0;  // the chunk after this one: the next group's first shortcut chunk, or its main chunk
      const int nc = nsc_next ? pu0 : (last_c ? 0 : c + 1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // halo(c) complete in buffer gc & 1; the other buffer and the shortcut tiles free
      const int boff = (gc & 1) * HBYTES;
      int hbc[8];
#pragma unroll
      for (int m = 0; m < 8; ++m) hbc[m] = hb[m] + boff;
      u32x4 hf[9][16];
      auto hread = [&](int tap, int i) {
        const int dy = tap / 3 - 1, dx = tap % 3 - 1;
        const int k = ((i >> 1) + dy + 1) * HC + (i & 1) * 16 + dx + 1;
        hf[tap][i] = *(const u32x4*)(smem + hbc[k & 7] + (k >> 3) * 512);
      };
#pragma unroll
      for (int i = 0; i < 4; ++i) hread(0, i);
      // 9 taps x 16 steps; step (tap, i): the halo fragment 4 steps ahead, then 4 MFMAs (pixel block i x the 4
      // cout blocks), each followed by its slice of the next chunk's halo work
      static_for<144>([&](auto ST) {
        constexpr int st = decltype(ST)::value, tap = st / 16, i = st % 16;
        if constexpr (i == 0) {
#pragma unroll
          for (int j = 0; j < 4; ++j) wcur[j] = wnext[j];
          if constexpr (tap < 8) wload(wnext, n0, false, tap + 1, c);
          else wload(wnext, nn0, nsc_next, 0, nc);
        }
        if constexpr (i + 4 < 16) hread(tap, i + 4);
        else if constexpr (tap < 8) hread(tap + 1, i - 12);
        if constexpr (st >= LOAD0 && (st - LOAD0) % STRIDE == 0 && (st - LOAD0) / STRIDE < VPT) {
          prep_load((st - LOAD0) / STRIDE);
        }
        if constexpr (SC && st >= SCL0 && (st - SCL0) % SCSTRIDE == 0 && (st - SCL0) / SCSTRIDE < 2 * SCV) {
          sc_load((st - SCL0) / SCSTRIDE);
        }
        static_for<4>([&](auto J) {
          constexpr int j = decltype(J)::value;
          if constexpr (i == 0 && j == 0)  // 2 wait states after any compiler VALU write of an operand (a copy)
            asm volatile("s_nop 1" ::: "memory");
          a_mfma(acc[i][j], wcur[j], hf[tap][i]);
          xf_slice(ST, J);
        });
        if constexpr (st >= XF0 + NSLOT - 1 && (st - XF0 - NSLOT + 1) % STRIDE == 0 &&
                      (st - XF0 - NSLOT + 1) / STRIDE < VPT) {
          xf_store((st - XF0 - NSLOT + 1) / STRIDE);
        }
        if constexpr (SC && st >= SCL0 + SCLAG && (st - SCL0 - SCLAG) % SCSTRIDE == 0 &&
                      (st - SCL0 - SCLAG) / SCSTRIDE < 2 * SCV) {
          sc_store((st - SCL0 - SCLAG) / SCSTRIDE);
        }
        // program order at step granularity: the prefetch distances above are the schedule (the scheduler would
        // otherwise hoist the fragment reads of the whole chunk and spill)
        __builtin_amdgcn_sched_barrier(0);
      });
      ++gc;
    }
    // the asm MFMAs' results are read by the epilogue's v_accvgpr_read: wait states hipcc does not insert
    asm volatile("s_nop 15\n\ts_nop 15" ::: "memory");

#ifdef H10_EXP_NOEPI2  // timing diagnostics: the epilogue exists but is skipped at run time (out_scale never equals this)
    if (p.out_scale != 12345.f) continue;
#endif
#ifdef H10_EXP_NOEPI
    {
      float* o = (float*)p.out + (size_t)t * 256 * 64 + lane * 4;
      for (int i = 0; i < 16; ++i)
        for (int j = 0; j < 4; ++j) *(f32x4*)(o + (i * 4 + j) * 256) = acc[i][j];
      continue;
    }
#endif
    // ---- epilogue from registers: acc[i][j][e] = out[pixel(i, lrow)][co0 + 16 j + e]
    const int co0 = n0 + chh * 64 + 4 * lg;
    float add[4][4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const f32x4 bv = *(const f32x4*)(p.bias + co0 + 16 * j);
      f32x4 tv = f32x4{0.f, 0.f, 0.f, 0.f};
      if (f_temb) tv = *(const f32x4*)(p.temb + (size_t)bb * p.temb_stride + co0 + 16 * j);
#pragma unroll
      for (int e = 0; e < 4; ++e) add[j][e] = bv[e] + tv[e];
    }
    // element pairs (e, e + 1) as float2: v_pk_add / v_pk_mul / v_pk_fma_f32 (two elements per VALU instruction; no
    // MFMA runs beside the epilogue, where packed f32 would cost issue slots)
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    f32x2 s1[4][2], s2[4][2];
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int e = 0; e < 2; ++e) { s1[j][e] = f32x2{0.f, 0.f}; s2[j][e] = f32x2{0.f, 0.f}; }
    const int pix0 = (bb * H + h0 + ph * 8) * W + w0 + lrow;
    const float osc = p.out_scale;
    // 16-B stores: cout blocks (2 jp, 2 jp + 1) are exchanged between DPP row pairs (v_permlane16_swap), so lane
    // (lrow, lg) stores the 8 consecutive couts n0 + chh 64 + 16 (2 jp + (lg & 1)) + 8 (lg >> 1) of its pixel -- half
    // the store instructions of 8-B stores (the epilogue is store-issue-bound at one wave per SIMD)
    const int cst = n0 + chh * 64 + 16 * (lg & 1) + 8 * (lg >> 1);
    auto epi = [&](auto SC_) {  // SC_: multiply by out_scale (a uniform branch outside the element loop)
      constexpr bool scale = decltype(SC_)::value;
      const f32x2 osc2 = f32x2{osc, osc};
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int pix = pix0 + (i >> 1) * W + (i & 1) * 16;
        f32x4 q = f32x4{0.f, 0.f, 0.f, 0.f};
        if (f_comb) q = *(const f32x4*)(p.comb_src + (size_t)pix * 4);
        uint32_t pk[4][2];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int co = co0 + 16 * j;
          f32x2 v[2];
#pragma unroll
          for (int e = 0; e < 2; ++e)
            v[e] = f32x2{acc[i][j][2 * e], acc[i][j][2 * e + 1]} + f32x2{add[j][2 * e], add[j][2 * e + 1]};
          if (f_res) {
            const uint2 rv = *(const uint2*)((const bf16_t*)p.res + (size_t)pix * p.res_ld + co);
            v[0] += f32x2{__uint_as_float(rv.x << 16), __uint_as_float(rv.x & 0xffff0000u)};
            v[1] += f32x2{__uint_as_float(rv.y << 16), __uint_as_float(rv.y & 0xffff0000u)};
          }
          if constexpr (scale) {
            v[0] *= osc2;
            v[1] *= osc2;
          }
          if (f_comb) {
#pragma unroll
            for (int e = 0; e < 4; ++e) {
              const f32x4 cw = *(const f32x4*)(p.comb_w + (size_t)(co + e) * 4);
              v[e >> 1][e & 1] += q[0] * cw[0] + q[1] * cw[1] + q[2] * cw[2] + q[3] * cw[3] + p.comb_b[co + e];
            }
          }
          pk[j][0] = pack_bf16x2(v[0][0], v[0][1]);
          pk[j][1] = pack_bf16x2(v[1][0], v[1][1]);
          if (f_stats) {
#pragma unroll
            for (int e = 0; e < 2; ++e) {
              s1[j][e] += v[e];
              s2[j][e] = v[e] * v[e] + s2[j][e];
            }
          }
        }
        bf16_t* orow = (bf16_t*)p.out + (size_t)pix * p.out_ld + cst;
#pragma unroll
        for (int jp = 0; jp < 2; ++jp) {
          const auto r0 = __builtin_amdgcn_permlane16_swap(pk[2 * jp][0], pk[2 * jp + 1][0], false, false);
          const auto r1 = __builtin_amdgcn_permlane16_swap(pk[2 * jp][1], pk[2 * jp + 1][1], false, false);
          const u32x4 o = {r0[0], r1[0], r0[1], r1[1]};
          if (f_nt) __builtin_nontemporal_store(o, (u32x4*)(orow + 32 * jp));
          else *(u32x4*)(orow + 32 * jp) = o;
        }
        __builtin_amdgcn_sched_barrier(0);  // one 16-px block at a time (the 256 accumulator reads are not hoisted)
      }
    };
    if (osc != 1.f) epi(std::integral_constant<bool, true>{});
    else epi(std::integral_constant<bool, false>{});
    if (f_stats) {
      // sum over the 16 pixels of a lane row (lanes with equal lg): DPP row rotations
#pragma unroll
      for (int j = 0; j < 4; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float a = s1[j][e >> 1][e & 1], q2 = s2[j][e >> 1][e & 1];
          a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x128, 0xf, 0xf, false));
          q2 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q2), 0x128, 0xf, 0xf, false));
          a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x124, 0xf, 0xf, false));
          q2 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q2), 0x124, 0xf, 0xf, false));
          a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x122, 0xf, 0xf, false));
          q2 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q2), 0x122, 0xf, 0xf, false));
          a += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(a), 0x121, 0xf, 0xf, false));
          q2 += __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(q2), 0x121, 0xf, 0xf, false));
          s1[j][e >> 1][e & 1] = a;
          s2[j][e >> 1][e & 1] = q2;
        }
      if (lrow == 0) {
        const int slot = blockIdx.x & (SNRSE_STAT_SLOTS - 1);
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            const size_t o = stat_idx(bb, slot, co0 + 16 * j + e, p.Cout);
            unsafeAtomicAdd(&p.stats[o], (double)s1[j][e >> 1][e & 1]);
            unsafeAtomicAdd(&p.stats[o + 1], (double)s2[j][e >> 1][e & 1]);
          }
      }
    }
  }
}

template <int GNM, int EF, bool SC>
int launch_h10_ef(const ConvParams& p, int ntiles, int grid, hipStream_t s) {
  static const hipError_t attr = hipFuncSetAttribute((const void*)conv_halo10_kernel<GNM, EF, SC>,
                                                     hipFuncAttributeMaxDynamicSharedMemorySize, h10::LDS);
  SNRSE_RET(attr);
  hipLaunchKernelGGL((conv_halo10_kernel<GNM, EF, SC>), dim3(grid), dim3(256), h10::LDS, s, p, ntiles);
  return (int)hipGetLastError();
}

#define SNRSE_H10_EF(F, SC) \
  case F: return launch_h10_ef<GNM, F, SC>(p, ntiles, grid, s);
template <int GNM>
int launch_h10_gn(const ConvParams& p, int ntiles, int grid, hipStream_t s, bool specialise) {
  const bool sc = p.sc_src != nullptr;
  if (specialise && p.bias) {
    // the NCSN++ ResBlock configurations: Conv_0 (temb), Conv_1 (residual, or the fused shortcut), non-temporal stores
    // for outputs beyond the L2 / MALL (p.epi_nt)
    if (!sc) {
      switch (epi_flags(p)) {
        SNRSE_H10_EF(EF_TEMB | EF_STATS, false)
        SNRSE_H10_EF(EF_TEMB | EF_STATS | EF_NT, false)
        SNRSE_H10_EF(EF_RES | EF_STATS, false)
        SNRSE_H10_EF(EF_RES | EF_STATS | EF_NT, false)
        default: break;
      }
    } else {
      switch (epi_flags(p)) {
        SNRSE_H10_EF(EF_STATS, true)
        SNRSE_H10_EF(EF_STATS | EF_NT, true)
        default: break;
      }
    }
  }
  return sc ? launch_h10_ef<GNM, EF_RT, true>(p, ntiles, grid, s) : launch_h10_ef<GNM, EF_RT, false>(p, ntiles, grid, s);
}
#undef SNRSE_H10_EF

}  // namespace

namespace snrse_conv {

bool h10_ok(const ConvParams& p) {
  const int ncb = (p.C0 + p.C1) / h10::KT, nsc = p.sc_src ? (p.Csc + p.Csc1) / h10::KT : 0;
  return p.ksize == 3 && p.H % h10::TH == 0 && p.W % h10::TW == 0 && p.Cout % 128 == 0 && nsc <= 2 * ncb && p.bias &&
         (p.C0 + p.C1) % h10::KT == 0 && p.C0 % h10::KT == 0;
}

int launch_h10(ConvParams p, hipStream_t s, int num_cu, bool specialise) {
  p.ntn = p.Cout / 128;
  const int ntiles = p.B * (p.H / h10::TH) * (p.W / h10::TW) * p.ntn;
  const int grid = ntiles < num_cu ? ntiles : num_cu;
  if (!p.gn_scale) return launch_h10_gn<0>(p, ntiles, grid, s, specialise);
  if (!p.gn_act) return launch_h10_gn<1>(p, ntiles, grid, s, specialise);
  return launch_h10_gn<2>(p, ntiles, grid, s, specialise);
}

}  // namespace snrse_conv
