// v6 halo GEMM: persistent, fully LDS-DMA-fed 3x3 convolution (+ fused GroupNorm/SiLU prologue,
// fused 1x1 shortcut, bias/temb/residual epilogue and GroupNorm statistics) for the NCSN++
// ResnetBlockBigGANpp convolutions (reference: layerspp.py:244-276 -> layers.py:100-124).
//
// Why this structure (profiles/r01_*): the v4/v5 halo kernels spend ~18 % of every block in the
// prologue (first halo + weight fetch under an all-CU burst) and ~15 % in a register-staged
// GroupNorm pass behind a barrier.  Here every workgroup is persistent over a contiguous range
// of output tiles and runs ONE software pipeline across chunk and tile boundaries:
//
//   tile      = 8 image rows x 32 px x 128 output channels; wave w owns rows h0+2w, h0+2w+1
//               (64 px x 128 co = acc[2][4] of v_mfma_f32_32x32x16_bf16, 128 VGPRs).  The 32x32
//               shape holds the SIMD's issue port 8 of its 32 cycles (16x16x32: 8 of 16), which
//               leaves room for the in-loop GroupNorm VALU work of the partner wave
//   chunk     = 32 input channels; a main chunk is 9 tap phases, a shortcut (Conv_2) chunk 1
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
// Two 256-thread workgroups per CU (K6_LDS each): one's epilogue / barrier waits run under the
// other's MFMAs.  Every wave counts its own LDS-DMA operations, so each in-loop wait is a counted
// `s_waitcnt vmcnt(N)` for exactly the data the next phase reads (raw s_barrier; vmcnt(0) only
// at the tile boundary, before the epilogue).
#include "conv_common.h"

namespace snrse_conv {
namespace {

constexpr int K6_TH = 8, K6_TW = 32, K6_HC = K6_TW + 2;
constexpr int K6_HROWS = (K6_TH + 2) * K6_HC;  // 340 halo rows
constexpr int K6_NPIECE = 22;                  // 1-KB LDS-DMA pieces per halo (rows 340..351 = pad)
constexpr int K6_HBUF = K6_NPIECE * 1024;      // 22528
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
static_assert(64 * K6_TROWS >= K6_HROWS && 16 * K6_NPIECE >= K6_HROWS, "halo rows");
static_assert(4 * K6_STAGE <= K6_HBUF, "epilogue staging fits one halo buffer");
static_assert(2 * (K6_LDS + 4 * 32 * 8) <= 163840, "two workgroups per CU (stamp builds included)");

typedef __amdgpu_buffer_rsrc_t rsrc_t;
typedef __attribute__((ext_vector_type(16))) float f32x16;

// 64-byte LDS rows (32 bf16 channels), 16-B chunk swizzled by (row >> 2) & 3: for the 32x32x16
// fragment reads (lane -> row r0 + (lane & 31), chunk 2s + (lane >> 5)) every ds_read_b128 lane
// group of 16 hits 16 distinct bank slots for ANY row offset r0 (tap-shifted A fragments): the 4
// rows of one row-residue class in a group are r, r+12, r+20, r+24 (or r+4, r+8, r+16, r+28),
// whose (row >> 2) & 3 are all different.
SNRSE_DEV int swz(int row, int chunk) { return (row << 6) + ((chunk ^ ((row >> 2) & 3)) << 4); }

SNRSE_DEV void glds16(rsrc_t r, char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
}
SNRSE_DEV void glds4(rsrc_t r, char* lds, int voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 4, voff, 0, 0, 0);
}

// s_waitcnt needs an immediate: the (wave-uniform) counts the pipeline produces, most frequent
// first (steady phase: 2 + 2; around a chunk start: 4 + halo ops of this wave); any other count
// waits for everything, which is always safe
#define K6_W(N) asm volatile("s_waitcnt vmcnt(" #N ")" ::: "memory")
SNRSE_DEV void wait_vm(int n) {
  if (n == 4) K6_W(4);
  else if (n >= K6_SKIP) {}
  else if (n == 10) K6_W(10);
  else if (n == 9) K6_W(9);
  else if (n == 2) K6_W(2);
  else if (n == 11) K6_W(11);
  else if (n == 13) K6_W(13);
  else K6_W(0);
}
#undef K6_W

// A copy of v the compiler cannot see through: per-lane address math derived from it is redone
// inside the pipelined loop instead of being hoisted into ~60 loop-invariant VGPRs.
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
  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
#ifdef SNRSE_STAMPS
  const int lane = tid & 63;
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

  // ---- raw halo of chunk c of tile tl -> halo buffer hb (+ its GroupNorm affine, wave 2)
  auto halo_issue = [&](const Tile6& tl, int c, int hb, int tq) {
    const int lane = tq & 63;
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
    for (int k = wid; k < K6_NPIECE; k += 4) {
      const int row = k * 16 + (lane >> 2);
      const int hy = row / K6_HC, hx = row - hy * K6_HC;
      const int ih = tl.h0 + hy - 1, iw = tl.w0 + hx - 1;
      const int dc = (lane & 3) ^ ((row >> 2) & 3);
      const bool ok = row < K6_HROWS && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W;
      const int voff = ok ? ((((tl.b * p.H + ih) * p.W + iw) * cs + ch + dc * 8) * 2) : (int)0x80000000;
      glds16(r, dst + k * 1024, voff);
    }
    if (has_gn && c < ncm && wid == 2) {
      // gn_shift == gn_scale + B*Cin (checked by the launcher): one resource covers both;
      // lanes 0..31 fetch the 32 scales, lanes 32..63 the 32 shifts
      const rsrc_t rg = make_rsrc(p.gn_scale, 8LL * p.B * Cin);
      const int voff = ((lane < 32 ? tl.b : p.B + tl.b) * Cin + c * 32 + (lane & 31)) * 4;
      glds4(rg, smem + K6_OFF_GN + hb * K6_GNB, voff);
    }
  };
  auto halo_ops = [&](int c) { return (wid < 2 ? 6 : 5) + ((has_gn && c < ncm && wid == 2) ? 1 : 0); };
  // ---- bias and temb slices of tile tl -> EP (wave 3), issued at the tile's first phase
  auto ep_issue = [&](const Tile6& tl, int tq) {
    const int lane = tq & 63;
    if (wid == 3) {
      const rsrc_t r = p.bias ? make_rsrc(p.bias, 4LL * p.Cout) : make_rsrc(p.out, 0);  // no bias: zeros
      glds4(r, smem + K6_OFF_EP, (tl.n0 + lane) * 4);
      glds4(r, smem + K6_OFF_EP + 256, (tl.n0 + 64 + lane) * 4);
      if (p.temb) {
        const rsrc_t rt = make_rsrc(p.temb + (size_t)tl.b * p.temb_stride + tl.n0, 512);
        glds4(rt, smem + K6_OFF_EP + 512, lane * 4);
        glds4(rt, smem + K6_OFF_EP + 768, (64 + lane) * 4);
      }
    }
  };
  const int ep_ops = wid == 3 ? (p.temb ? 4 : 2) : 0;

  // ---- one tap's weights (128 co x 32 ch) of phase (tl, c, pi) -> ring slot s
  auto w_issue = [&](const Tile6& tl, int c, int pi, int s, int tq) {
    const int lane = tq & 63;
    const bool mainw = c < ncm;
    const int ldw = mainw ? K1 : Csc_all;
    const int koff = mainw ? pi * Cin + c * 32 : (c - ncm) * 32;
    const rsrc_t r = mainw ? make_rsrc(p.wgt, p.wbytes) : make_rsrc(p.sc_wgt, p.sc_wbytes);
    char* dst = smem + K6_OFF_W + s * K6_TAPB;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int pc = wid + 4 * i;
      const int row = pc * 16 + (lane >> 2);
      const int dc = (lane & 3) ^ ((row >> 2) & 3);
      glds16(r, dst + pc * 1024, ((tl.n0 + row) * ldw + koff + dc * 8) * 2);
    }
  };

  // ---- in-place GroupNorm(+SiLU) of halo row (tq >> 2) + 64 ri, channels 8 (tq & 3) .. +8
  auto transform_row = [&](const Tile6& tl, int hb, int ri, int tq) {
    const int r = (tq >> 2) + 64 * ri;
    const int hy = r / K6_HC, hx = r - hy * K6_HC;
    const int ih = tl.h0 + hy - 1, iw = tl.w0 + hx - 1;
    if (r < K6_HROWS && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W) {  // padding stays zero
      const int dc = tq & 3;
      char* a = smem + hb * K6_HBUF + swz(r, dc);
      const float* gp = (const float*)(smem + K6_OFF_GN + hb * K6_GNB) + dc * 8;
      const f32x4 s0 = *(const f32x4*)gp, s1 = *(const f32x4*)(gp + 4);
      const f32x4 t0 = *(const f32x4*)(gp + 32), t1 = *(const f32x4*)(gp + 36);
      const float gsc[8] = {s0[0], s0[1], s0[2], s0[3], s1[0], s1[1], s1[2], s1[3]};
      const float gsh[8] = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
      u32x4 v = *(const u32x4*)a;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float lo = __uint_as_float(v[i] << 16), hi = __uint_as_float(v[i] & 0xffff0000u);
        lo = fmaf(lo, gsc[2 * i], gsh[2 * i]);
        hi = fmaf(hi, gsc[2 * i + 1], gsh[2 * i + 1]);
        if (p.gn_act) { lo = silu(lo); hi = silu(hi); }
        v[i] = pack_bf16x2(lo, hi);
      }
      *(u32x4*)a = v;
    }
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
  auto epilogue = [&](const Tile6& tl, int hb, int tq) {
    const int lane = tq & 63, l31 = lane & 31, lh = lane >> 5;
    float* const stg = (float*)(smem + hb * K6_HBUF + wid * K6_STAGE);
    const float* const ep = (const float*)(smem + K6_OFF_EP);
    const bool has_t = p.temb != nullptr;
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
          f32x4 add = *(const f32x4*)(ep + nl + 4 * k4);
          if (has_t) {
            const f32x4 tv = *(const f32x4*)(ep + 128 + nl + 4 * k4);
            add[0] += tv[0]; add[1] += tv[1]; add[2] += tv[2]; add[3] += tv[3];
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) v[4 * k4 + e] = stg[(lh * 16 + 4 * k4 + e) * K6_LDR + l31] + add[e];
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

  // ---- prologue: chunk 0 of the first tile, weights of phases 0, 1, 2
  stl[tid] = 0.f;
  Cur6 ahead = {0, 0, 0};
  Tile6 tcur = tile_of(0);
  halo_issue(tcur, 0, 0, tid);
#pragma unroll 1
  for (int s = 0; s < K6_NSLOT - 1; ++s) {
    if (ahead.lt < ntile) w_issue(ahead.lt == 0 ? tcur : tile_of(ahead.lt), ahead.c, ahead.pi, s, tid);
    ahead = advance(ahead);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  sync_lds();
  if (has_gn) {
#pragma unroll 1
    for (int ri = 0; ri < K6_TROWS; ++ri) transform_row(tcur, 0, ri, tid);
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
#pragma unroll 1
    for (int c = 0; c < nchunk; ++c) {
      const bool mainc = c < ncm;
      const int np = mainc ? 9 : 1;
      const bool last_c = c + 1 == nchunk;
      const bool has_next = !last_c || has_nt;
      const int nc = last_c ? 0 : c + 1;
      const Tile6& tnext = last_c ? tnt : tcur;
      const bool next_gn = has_next && has_gn && nc < ncm;
      const int hnext = (gch + 1) & 1;
      int ops = 0;  // vector-memory ops of the current phase, in issue order
      {
        const int tq = opaque(tid);
        if (has_next) {
          halo_issue(tnext, nc, hnext, tq);
          ops += halo_ops(nc);
        }
        if (c == 0) {
          ep_issue(tcur, tq);
          ops += ep_ops;
        }
      }
      const int hops = ops;
      const char* const hbuf = smem + (gch & 1) * K6_HBUF;
#pragma unroll 1
      for (int pi = 0; pi < np; ++pi) {
        const int tq = opaque(tid);
        const bool tile_last = last_c && pi + 1 == np;
        const int s3 = (slot + 3) & 3;
        if (tile_last) {
          wdef = ahead;
          sdef = s3;
        } else if (ahead.lt < ntile) {
          w_issue(ahead.lt == lt ? tcur : tnt, ahead.c, ahead.pi, s3, tq);
          ops += 2;
        }
        // the halo issued at this chunk's phase 0 has landed once phase 2's wait retired it
        if (next_gn && np == 9 && pi >= 3) transform_row(tnext, hnext, pi - 3, tq);

        // one tap: 2 k-steps x 2 pixel blocks x 4 channel blocks = 16 MFMAs per wave
        const int ln = tq & 63, fr = ln & 31, fh = ln >> 5;
        const char* wsl = smem + K6_OFF_W + slot * K6_TAPB;
        const int tap = mainc ? pi : 4;
        const int dy = tap / 3 - 1, dx = tap - (tap / 3) * 3 - 1;
        const int hbase = (2 * wid + dy + 1) * K6_HC + dx + 1 + fr;
#pragma unroll
        for (int ks = 0; ks < 2; ++ks) {
          u32x4 af[2], bfr[4];
#pragma unroll
          for (int mi = 0; mi < 2; ++mi) af[mi] = *(const u32x4*)(hbuf + swz(hbase + mi * K6_HC, 2 * ks + fh));
#pragma unroll
          for (int nj = 0; nj < 4; ++nj) bfr[nj] = *(const u32x4*)(wsl + swz(nj * 32 + fr, 2 * ks + fh));
#pragma unroll
          for (int mi = 0; mi < 2; ++mi)
#pragma unroll
            for (int nj = 0; nj < 4; ++nj) acc[mi][nj] = mfma32(af[mi], bfr[nj], acc[mi][nj]);
        }
        if (!tile_last) {
          // W(Q+1) (issued two phases ago, as that phase's last op) has landed; after a one-phase
          // (shortcut) chunk also the halo issued at its start, which the next chunk reads
          const int n = np == 1 ? ops - hops : (prev_ops >= K6_SKIP ? K6_SKIP : prev_ops + ops);
          wait_vm(n);
          sync_lds();
          prev_ops = ops;
          ops = 0;
        }
        slot = (slot + 1) & 3;
        ahead = advance(ahead);
      }
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
    const int tq = opaque(tid);
    if (deferred) {
#pragma unroll 1
      for (int ri = 0; ri < K6_TROWS; ++ri) transform_row(tnt, (gch + 1) & 1, ri, tq);
    }
    epilogue(tcur, gch & 1, tq);
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
    // the deferred slice is phase 2 of the next tile (every tile has >= 9 phases)
    if (wdef.lt < ntile) w_issue(tnt, wdef.c, wdef.pi, sdef, tq);
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
  if (p.comb_src) return false;  // Combine epilogues stay on the v4 kernel
  if (p.out_ld % 8 || (p.res && p.res_ld % 8)) return false;
  if (p.gn_scale && p.gn_shift != p.gn_scale + (size_t)p.B * Cin) return false;
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
