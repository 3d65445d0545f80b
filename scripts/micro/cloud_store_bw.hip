// Microbenchmark (measurement only, not part of the library): the write
// pattern of k_cloud at config 2 -- 6.55 M points, f32 xyz (one 12-B store
// per lane, 768 B contiguous per wave instruction) + BGR (3 B per lane) --
// with and without k_cloud's reads (2-B records + 3-B texture per pixel of
// an 8.3 Mpx view), against 16-B-per-lane stores of the same bytes.
// Prints one JSON line per pattern and workgroups per CU.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
constexpr int64_t kHW = 3840LL * 2160;
constexpr int64_t kPts = 6548659;

struct __attribute__((packed)) F3 { float x, y, z; };

// one lane per point: xyz (12 B) + colour (3 B); optional reads of 5 B per
// pixel (a 16-B record load + 3 x 16-B texture loads per 16 pixels)
__global__ __launch_bounds__(256) void pts(F3* xyz, uint8_t* bgr, const v4u* rec, const v4u* tex, int reads, int64_t npts,
                                           unsigned* sink) {
  const int64_t nthreads = static_cast<int64_t>(gridDim.x) * 256;
  unsigned acc = 0;
  if (reads) {
    // the read share of one lane: kHW / 16 record+texture groups over the grid
    for (int64_t g = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; g < kHW / 16; g += nthreads) {
      const v4u r0 = rec[2 * g], r1 = rec[2 * g + 1];
      const v4u t0 = tex[3 * g], t1 = tex[3 * g + 1], t2 = tex[3 * g + 2];
      acc ^= r0[0] ^ r1[1] ^ t0[2] ^ t1[3] ^ t2[0];
    }
  }
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < npts; i += nthreads) {
    const float f = static_cast<float>(i);
    F3 v = {f, f + 1.0f, f + (acc == 7u ? 2.0f : 3.0f)};
    xyz[i] = v;
    bgr[3 * i] = static_cast<uint8_t>(i);
    bgr[3 * i + 1] = static_cast<uint8_t>(i >> 8);
    bgr[3 * i + 2] = static_cast<uint8_t>(i >> 16);
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

// the same bytes as 16-B stores (xyz and colour as flat byte arrays)
__global__ __launch_bounds__(256) void flat16(v4u* xyz, v4u* bgr, const v4u* rec, const v4u* tex, int reads, int64_t npts,
                                              unsigned* sink) {
  const int64_t nthreads = static_cast<int64_t>(gridDim.x) * 256;
  unsigned acc = 0;
  if (reads) {
    for (int64_t g = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; g < kHW / 16; g += nthreads) {
      const v4u r0 = rec[2 * g], r1 = rec[2 * g + 1];
      const v4u t0 = tex[3 * g], t1 = tex[3 * g + 1], t2 = tex[3 * g + 2];
      acc ^= r0[0] ^ r1[1] ^ t0[2] ^ t1[3] ^ t2[0];
    }
  }
  const int64_t nx = npts * 12 / 16, nc = npts * 3 / 16;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < nx; i += nthreads) {
    const unsigned u = static_cast<unsigned>(i);
    xyz[i] = v4u{u, u + 1, u + 2, u + (acc == 7u ? 1u : 3u)};
    if (i < nc) bgr[i] = v4u{u, u, u, u};
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

template <typename L>
static float time_it(L launch, hipEvent_t a, hipEvent_t b) {
  float best = 1e30f;
  for (int r = 0; r < 20; ++r) {
    (void)hipEventRecord(a, 0);
    launch();
    (void)hipEventRecord(b, 0);
    (void)hipEventSynchronize(b);
    float ms = 0.f;
    (void)hipEventElapsedTime(&ms, a, b);
    if (r > 2 && ms < best) best = ms;
  }
  return best;
}

int main() {
  F3* xyz;
  uint8_t* bgr;
  v4u *rec, *tex;
  unsigned* sink;
  if (hipMalloc(&xyz, 12 * kPts + 64) != hipSuccess || hipMalloc(&bgr, 3 * kPts + 64) != hipSuccess ||
      hipMalloc(&rec, 2 * kHW) != hipSuccess || hipMalloc(&tex, 3 * kHW) != hipSuccess || hipMalloc(&sink, 4) != hipSuccess)
    return 1;
  (void)hipMemset(rec, 1, 2 * kHW);
  (void)hipMemset(tex, 2, 3 * kHW);
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int per_cu : {2, 4, 8}) {
    const int grid = per_cu * n_cu;
    for (int reads = 0; reads < 2; ++reads) {
      const float t0 = time_it([&] { hipLaunchKernelGGL(pts, dim3(grid), dim3(256), 0, 0, xyz, bgr, rec, tex, reads, kPts, sink); }, a, b);
      const float t1 = time_it([&] {
        hipLaunchKernelGGL(flat16, dim3(grid), dim3(256), 0, 0, reinterpret_cast<v4u*>(xyz), reinterpret_cast<v4u*>(bgr), rec, tex,
                           reads, kPts, sink);
      }, a, b);
      const double bytes = 15.0 * kPts + (reads ? 5.0 * kHW : 0.0);
      printf("{\"wg_per_cu\": %d, \"reads\": %d, \"points_us\": %.2f, \"flat16_us\": %.2f, \"points_GBps\": %.0f, \"flat16_GBps\": %.0f}\n",
             per_cu, reads, t0 * 1e3, t1 * 1e3, bytes / (t0 * 1e-3) / 1e9, bytes / (t1 * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
  return 0;
}
