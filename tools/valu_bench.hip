// Issue-cost micro-benchmark of the VALU instruction mixes a GroupNorm+SiLU transform can use on
// gfx950: cycles per wave-instruction for streams of independent instructions (8 chains), alone and
// interleaved, at 1 and 2 waves per SIMD.  Standalone: hipcc --offload-arch=gfx950 -O3 -o valu_bench
// tools/valu_bench.hip && ./valu_bench.  Prints one JSON line per mix.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define REP8(X) X X X X X X X X

// Each mix: one loop iteration issues the listed instructions on 8 independent registers.
#define MIX_BODY(INSTRS)                                                                   \
  for (int it = 0; it < iters; ++it) {                                                     \
    asm volatile(INSTRS                                                                    \
                 : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), \
                   "+v"(a7)                                                                \
                 : "v"(k)                                                                  \
                 :);                                                                       \
  }

#define ADD8 \
  "v_add_f32 %0, %0, %8\n v_add_f32 %1, %1, %8\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n" \
  "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8\n"
#define EXP8 \
  "v_exp_f32 %0, %0\n v_exp_f32 %1, %1\n v_exp_f32 %2, %2\n v_exp_f32 %3, %3\n" \
  "v_exp_f32 %4, %4\n v_exp_f32 %5, %5\n v_exp_f32 %6, %6\n v_exp_f32 %7, %7\n"
#define RCP8 \
  "v_rcp_f32 %0, %0\n v_rcp_f32 %1, %1\n v_rcp_f32 %2, %2\n v_rcp_f32 %3, %3\n" \
  "v_rcp_f32 %4, %4\n v_rcp_f32 %5, %5\n v_rcp_f32 %6, %6\n v_rcp_f32 %7, %7\n"
#define EXPH8 \
  "v_exp_f16 %0, %0\n v_exp_f16 %1, %1\n v_exp_f16 %2, %2\n v_exp_f16 %3, %3\n" \
  "v_exp_f16 %4, %4\n v_exp_f16 %5, %5\n v_exp_f16 %6, %6\n v_exp_f16 %7, %7\n"
#define EXPADD8 \
  "v_exp_f32 %0, %0\n v_add_f32 %4, %4, %8\n v_exp_f32 %1, %1\n v_add_f32 %5, %5, %8\n" \
  "v_exp_f32 %2, %2\n v_add_f32 %6, %6, %8\n v_exp_f32 %3, %3\n v_add_f32 %7, %7, %8\n"
#define EXPADD2_8 \
  "v_exp_f32 %0, %0\n v_add_f32 %2, %2, %8\n v_add_f32 %3, %3, %8\n v_exp_f32 %1, %1\n" \
  "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8\n"
#define PKFMA8 \
  "v_pk_fma_f32 %0, %0, %8, %0\n v_pk_fma_f32 %1, %1, %8, %1\n v_pk_fma_f32 %2, %2, %8, %2\n v_pk_fma_f32 %3, %3, %8, %3\n" \
  "v_pk_fma_f32 %4, %4, %8, %4\n v_pk_fma_f32 %5, %5, %8, %5\n v_pk_fma_f32 %6, %6, %8, %6\n v_pk_fma_f32 %7, %7, %8, %7\n"
#define PKFMAH8 \
  "v_pk_fma_f16 %0, %0, %8, %0\n v_pk_fma_f16 %1, %1, %8, %1\n v_pk_fma_f16 %2, %2, %8, %2\n v_pk_fma_f16 %3, %3, %8, %3\n" \
  "v_pk_fma_f16 %4, %4, %8, %4\n v_pk_fma_f16 %5, %5, %8, %5\n v_pk_fma_f16 %6, %6, %8, %6\n v_pk_fma_f16 %7, %7, %8, %7\n"
#define DOT2BF8 \
  "v_dot2_f32_bf16 %0, %0, %8, %0\n v_dot2_f32_bf16 %1, %1, %8, %1\n v_dot2_f32_bf16 %2, %2, %8, %2\n v_dot2_f32_bf16 %3, %3, %8, %3\n" \
  "v_dot2_f32_bf16 %4, %4, %8, %4\n v_dot2_f32_bf16 %5, %5, %8, %5\n v_dot2_f32_bf16 %6, %6, %8, %6\n v_dot2_f32_bf16 %7, %7, %8, %7\n"
#define CVTPK8 \
  "v_cvt_pk_bf16_f32 %0, %0, %8\n v_cvt_pk_bf16_f32 %1, %1, %8\n v_cvt_pk_bf16_f32 %2, %2, %8\n v_cvt_pk_bf16_f32 %3, %3, %8\n" \
  "v_cvt_pk_bf16_f32 %4, %4, %8\n v_cvt_pk_bf16_f32 %5, %5, %8\n v_cvt_pk_bf16_f32 %6, %6, %8\n v_cvt_pk_bf16_f32 %7, %7, %8\n"
#define MED3_8 \
  "v_med3_f32 %0, %0, %8, %8\n v_med3_f32 %1, %1, %8, %8\n v_med3_f32 %2, %2, %8, %8\n v_med3_f32 %3, %3, %8, %8\n" \
  "v_med3_f32 %4, %4, %8, %8\n v_med3_f32 %5, %5, %8, %8\n v_med3_f32 %6, %6, %8, %8\n v_med3_f32 %7, %7, %8, %8\n"

template <int MIX>
__global__ void mix_kernel(float* out, unsigned long long* cyc, int iters, float kf) {
  float a0 = threadIdx.x * 1e-3f, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6,
        a7 = a0 + 7;
  float k = kf;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if constexpr (MIX == 0) { MIX_BODY(ADD8) }
  if constexpr (MIX == 1) { MIX_BODY(EXP8) }
  if constexpr (MIX == 2) { MIX_BODY(RCP8) }
  if constexpr (MIX == 3) { MIX_BODY(EXPH8) }
  if constexpr (MIX == 4) { MIX_BODY(EXPADD8) }
  if constexpr (MIX == 5) { MIX_BODY(EXPADD2_8) }
  if constexpr (MIX == 6) { MIX_BODY(PKFMAH8) }
  if constexpr (MIX == 7) { MIX_BODY(DOT2BF8) }
  if constexpr (MIX == 8) { MIX_BODY(CVTPK8) }
  if constexpr (MIX == 9) { MIX_BODY(MED3_8) }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

// v_pk_fma_f32 needs 64-bit operands: separate kernel
__global__ void pkfma32_kernel(double* out, unsigned long long* cyc, int iters, double kf) {
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a[8];
  for (int i = 0; i < 8; ++i) a[i] = f2{threadIdx.x * 1e-3f + i, 1.f};
  f2 k = f2{(float)kf, (float)kf};
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    asm volatile(PKFMA8 : "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]),
                 "+v"(a[7]) : "v"(k) :);
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  float s = 0;
  for (int i = 0; i < 8; ++i) s += a[i][0] + a[i][1];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x % 64 == 0) cyc[blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64] = t1 - t0;
}

static const char* kNames[] = {"8 v_add_f32", "8 v_exp_f32", "8 v_rcp_f32", "8 v_exp_f16",
                               "4 v_exp_f32 + 4 v_add_f32 interleaved", "2 v_exp_f32 + 6 v_add_f32",
                               "8 v_pk_fma_f16", "8 v_dot2_f32_bf16", "8 v_cvt_pk_bf16_f32", "8 v_med3_f32",
                               "8 v_pk_fma_f32"};

template <int MIX>
void run(int wps, int iters) {
  const int threads = 64 * 4 * wps, blocks = 256;  // one workgroup per CU: wps waves per SIMD
  float* out;
  unsigned long long* cyc;
  hipMalloc(&out, sizeof(double) * blocks * threads);
  hipMalloc(&cyc, sizeof(unsigned long long) * blocks * threads / 64);
  for (int rep = 0; rep < 2; ++rep) {
    if constexpr (MIX == 10)
      hipLaunchKernelGGL(pkfma32_kernel, dim3(blocks), dim3(threads), 0, 0, (double*)out, cyc, iters, 1.0000001);
    else
      hipLaunchKernelGGL(mix_kernel<MIX>, dim3(blocks), dim3(threads), 0, 0, out, cyc, iters, 1.0000001f);
  }
  hipDeviceSynchronize();
  const int nw = blocks * threads / 64;
  unsigned long long* h = new unsigned long long[nw];
  hipMemcpy(h, cyc, sizeof(unsigned long long) * nw, hipMemcpyDeviceToHost);
  double s = 0;
  for (int i = 0; i < nw; ++i) s += (double)h[i];
  const double per_iter = s / nw / iters;
  printf("{\"mix\": \"%s\", \"waves_per_simd\": %d, \"cycles_per_iter\": %.2f, \"cycles_per_instr\": %.2f}\n",
         kNames[MIX], wps, per_iter, per_iter / 8.0);
  delete[] h;
  hipFree(out);
  hipFree(cyc);
}

template <int MIX>
void run_all() {
  run<MIX>(1, 4096);
  run<MIX>(2, 4096);
}

int main() {
  run_all<0>(); run_all<1>(); run_all<2>(); run_all<3>(); run_all<4>(); run_all<5>();
  run_all<6>(); run_all<7>(); run_all<8>(); run_all<9>(); run_all<10>();
  return 0;
}
