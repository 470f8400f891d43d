// Same-box HBM calibration for the roofline fractions of the HBM-bound kernels: streaming kernels
// with the read:write byte mixes of the NCSN++ passes, 16-B accesses per lane, grid-stride over
// 1-2 GiB buffers (far beyond the 256 MB Infinity Cache), HIP events over `reps` launches.
//   read        sum of a 2 GiB buffer (read-only ceiling; conv_head<2>'s mix is 95 % read)
//   write       fill of 1 GiB (write-only ceiling; input_conv's mix is 89 % write)
//   copy        1 GiB -> 1 GiB (1:1)
//   read2write1 2 x 1 GiB -> 1 GiB (elementwise a + b), the 2:1 mix of gn_resample down (1.07 GB in,
//               0.54 GB out) and of a GEMM's input:output at level 0
//   read1write2 1 GiB -> 2 x 1 GiB, the 1:2 mix of gn_resample up (0.32 GB in, 2.15 GB out)
// Each mode runs plain and non-temporal stores.  Build: hipcc --offload-arch=gfx950 -O3 -o tools/bin/hbm_calib
// tools/hbm_calib.hip.  Output: one JSON line per (mode, store flavour).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                        \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

template <bool NT>
__device__ inline void st(u32x4* p, u32x4 v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

__global__ __launch_bounds__(256) void k_read(const u32x4* __restrict__ a, size_t n, unsigned* __restrict__ sink) {
  unsigned acc = 0;
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const u32x4 v = a[i];
    acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (acc == 0x9e3779b9u) sink[threadIdx.x] = acc;  // keeps the loads; never true for the fill pattern
}

template <bool NT>
__global__ __launch_bounds__(256) void k_write(u32x4* __restrict__ o, size_t n, unsigned s) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256)
    st<NT>(o + i, u32x4{s, (unsigned)i, s, (unsigned)i});
}

template <bool NT>
__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ o, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) st<NT>(o + i, a[i]);
}

template <bool NT>
__global__ __launch_bounds__(256) void k_r2w1(const u32x4* __restrict__ a, const u32x4* __restrict__ b,
                                              u32x4* __restrict__ o, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) st<NT>(o + i, a[i] + b[i]);
}

template <bool NT>
__global__ __launch_bounds__(256) void k_r1w2(const u32x4* __restrict__ a, u32x4* __restrict__ o1,
                                              u32x4* __restrict__ o2, size_t n) {
  for (size_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const u32x4 v = a[i];
    st<NT>(o1 + i, v);
    st<NT>(o2 + i, v + 1u);
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 20;
  const size_t GB = 1ull << 30, n = GB / 16;
  u32x4 *a, *b, *o1, *o2;
  unsigned* sink;
  CHECK(hipMalloc(&a, 2 * GB));
  CHECK(hipMalloc(&b, GB));
  CHECK(hipMalloc(&o1, GB));
  CHECK(hipMalloc(&o2, GB));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemset(a, 1, 2 * GB));
  CHECK(hipMemset(b, 2, GB));
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grids[] = {cus * 8, cus * 32};  // 8 / 32 resident-size waves of 256 threads per CU
  auto run = [&](const char* mode, bool nt, double bytes, auto launch) {
    double best = 1e30;
    for (int g : grids) {
      launch(g);  // warm-up
      CHECK(hipDeviceSynchronize());
      std::vector<float> ts;
      for (int r = 0; r < reps; ++r) {
        CHECK(hipEventRecord(e0, 0));
        launch(g);
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms = 0.f;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        ts.push_back(ms);
      }
      std::sort(ts.begin(), ts.end());
      const double med = ts[ts.size() / 2];
      printf("{\"mode\": \"%s\", \"nt\": %d, \"grid\": %d, \"bytes\": %.0f, \"ms\": %.4f, \"TBps\": %.3f, "
             "\"frac_of_8TBps\": %.3f}\n",
             mode, (int)nt, g, bytes, med, bytes / med / 1e9, bytes / med / 1e9 / 8.0);
      fflush(stdout);
      best = std::min(best, med);
    }
    return best;
  };
  run("read", false, 2.0 * GB, [&](int g) { hipLaunchKernelGGL(k_read, dim3(g), dim3(256), 0, 0, a, 2 * n, sink); });
  for (int nt = 0; nt < 2; ++nt) {
    run("write", nt, 1.0 * GB, [&](int g) {
      if (nt) hipLaunchKernelGGL(k_write<true>, dim3(g), dim3(256), 0, 0, o1, n, 7u);
      else hipLaunchKernelGGL(k_write<false>, dim3(g), dim3(256), 0, 0, o1, n, 7u);
    });
    run("copy", nt, 2.0 * GB, [&](int g) {
      if (nt) hipLaunchKernelGGL(k_copy<true>, dim3(g), dim3(256), 0, 0, a, o1, n);
      else hipLaunchKernelGGL(k_copy<false>, dim3(g), dim3(256), 0, 0, a, o1, n);
    });
    run("read2write1", nt, 3.0 * GB, [&](int g) {
      if (nt) hipLaunchKernelGGL(k_r2w1<true>, dim3(g), dim3(256), 0, 0, a, b, o1, n);
      else hipLaunchKernelGGL(k_r2w1<false>, dim3(g), dim3(256), 0, 0, a, b, o1, n);
    });
    run("read1write2", nt, 3.0 * GB, [&](int g) {
      if (nt) hipLaunchKernelGGL(k_r1w2<true>, dim3(g), dim3(256), 0, 0, b, o1, o2, n);
      else hipLaunchKernelGGL(k_r1w2<false>, dim3(g), dim3(256), 0, 0, b, o1, o2, n);
    });
  }
  CHECK(hipGetLastError());
  CHECK(hipDeviceSynchronize());
  return 0;
}
