// WRITE_SIZE calibration (measurement only, not part of the library): known
// byte counts written with the store shapes of the library's kernels, run
// under `rocprofv3 --pmc WRITE_SIZE`, so that the PMC write bytes of those
// kernels can be corrected (MI355X_MICROARCH.md: WRITE_SIZE is exact only for
// 16-B-per-lane streaming stores).
//   st16  16 B per lane, 1 KB contiguous per wave instruction, nontemporal
//         (k_decode's maps since round 5)
//   st12  12 B per lane, 768 B contiguous per wave instruction, nontemporal
//         (k_cloud's xyz, global_store_dwordx3 nt)
//   st3   3 B per lane (one short + one byte store), 192 B contiguous (k_cloud's BGR)
//   pts   st12 + st3 interleaved per lane, as k_cloud issues them
// Each kernel writes kBytes[k] bytes once per launch; 5 launches each.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

constexpr int64_t kPts = 6548659;  // config 2's points

struct __attribute__((packed)) F3 { float x, y, z; };
typedef unsigned v4u __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void st16(v4u* o, int64_t n) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const unsigned u = static_cast<unsigned>(i);
    __builtin_nontemporal_store(v4u{u, u + 1, u + 2, u + 3}, o + i);
  }
}
__global__ __launch_bounds__(256) void st12(F3* o, int64_t n) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const float f = static_cast<float>(i);
    float* p = &o[i].x;
    __builtin_nontemporal_store(f, p);
    __builtin_nontemporal_store(f + 1.0f, p + 1);
    __builtin_nontemporal_store(f + 2.0f, p + 2);
  }
}
__global__ __launch_bounds__(256) void st3(uint8_t* o, int64_t n) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    o[3 * i] = static_cast<uint8_t>(i);
    o[3 * i + 1] = static_cast<uint8_t>(i >> 8);
    o[3 * i + 2] = static_cast<uint8_t>(i >> 16);
  }
}
__global__ __launch_bounds__(256) void pts(F3* xyz, uint8_t* bgr, int64_t n) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256) {
    const float f = static_cast<float>(i);
    float* p = &xyz[i].x;
    __builtin_nontemporal_store(f, p);
    __builtin_nontemporal_store(f + 1.0f, p + 1);
    __builtin_nontemporal_store(f + 2.0f, p + 2);
    bgr[3 * i] = static_cast<uint8_t>(i);
    bgr[3 * i + 1] = static_cast<uint8_t>(i >> 8);
    bgr[3 * i + 2] = static_cast<uint8_t>(i >> 16);
  }
}

// FETCH_SIZE of k_cloud's read widths: 8 B per lane (its 12-bit records, 24 B
// per lane as three 8-B loads) and 16 B per lane (the texture), streaming
__global__ __launch_bounds__(256) void ld8(const unsigned long long* in, int64_t n, unsigned long long* sink) {
  unsigned long long acc = 0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256)
    acc ^= in[i];
  if (acc == 0x123456789ull) sink[0] = acc;
}
__global__ __launch_bounds__(256) void ld16(const v4u* in, int64_t n, v4u* sink) {
  v4u acc = {0, 0, 0, 0};
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256)
    acc ^= in[i];
  if (acc.x == 0x1234567u) sink[0] = acc;
}

int main() {
  void *a, *b;
  if (hipMalloc(&a, 16 * kPts + 256) != hipSuccess || hipMalloc(&b, 3 * kPts + 256) != hipSuccess) return 1;
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  const dim3 g(4 * n_cu), t(256);
  for (int r = 0; r < 5; ++r) {
    hipLaunchKernelGGL(st16, g, t, 0, 0, static_cast<v4u*>(a), kPts);  // 16 * kPts bytes
    hipLaunchKernelGGL(st12, g, t, 0, 0, static_cast<F3*>(a), kPts);   // 12 * kPts
    hipLaunchKernelGGL(st3, g, t, 0, 0, static_cast<uint8_t*>(b), kPts);  // 3 * kPts
    hipLaunchKernelGGL(pts, g, t, 0, 0, static_cast<F3*>(a), static_cast<uint8_t*>(b), kPts);  // 15 * kPts
    hipLaunchKernelGGL(ld8, g, t, 0, 0, static_cast<const unsigned long long*>(a), 2 * kPts,
                       static_cast<unsigned long long*>(b));  // reads 16 * kPts
    hipLaunchKernelGGL(ld16, g, t, 0, 0, static_cast<const v4u*>(a), kPts, static_cast<v4u*>(b));  // 16 * kPts
  }
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("{\"points\": %lld, \"bytes\": {\"st16\": %lld, \"st12\": %lld, \"st3\": %lld, \"pts\": %lld, "
         "\"ld8\": %lld, \"ld16\": %lld}}\n",
         static_cast<long long>(kPts), static_cast<long long>(16 * kPts), static_cast<long long>(12 * kPts),
         static_cast<long long>(3 * kPts), static_cast<long long>(15 * kPts), static_cast<long long>(16 * kPts),
         static_cast<long long>(16 * kPts));
  return 0;
}
