// Microbenchmark (measurement only, not part of the library): the cloud-only
// k_decode access pattern -- NPL planes of a view read once (16 B per lane,
// lane = 16 contiguous pixels, wave = 1024-pixel chunk), a synthetic VALU
// load of C dependent-free instructions per chunk, and the 2-B record stores
// (2 x 16 B per lane) -- with and without software pipelining across the
// chunk loop (the next chunk's planes loaded before this chunk's compute).
// Prints one JSON line per (pattern, planes, compute, workgroups per CU).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
constexpr int kChunk = 1024;

// C rounds of 16 independent integer ops per lane over the loaded words (the
// compiler cannot drop them: the result is stored with the records)
template <int C>
__device__ __forceinline__ v4u churn(v4u a, v4u b) {
#pragma unroll
  for (int i = 0; i < C; ++i) {
    a = (a ^ (b >> 3)) + (b << 1);
    b = (b ^ (a >> 5)) + (a | 0x01010101u);
    a = a * 3u + b;
    b = b * 5u ^ a;
  }
  return a ^ b;
}

template <int NPL, int C>
__global__ __launch_bounds__(256, 3) void plain(const uint8_t* st, int64_t HW, int ngroups, v4u* rec, int store) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int cg = blockIdx.x; cg < ngroups; cg += gridDim.x) {
    const int64_t chunk = static_cast<int64_t>(cg) * 4 + wid;
    const int64_t px = chunk * kChunk + lane * 16;
    if (px >= HW) continue;
    v4u v[NPL];
#pragma unroll
    for (int p = 0; p < NPL; ++p) v[p] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(st + p * HW + px));
    v4u a = v[0], b = v[1];
#pragma unroll
    for (int p = 2; p < NPL; p += 2) {
      a ^= v[p];
      b += v[p + 1];
    }
    const v4u r = churn<C>(a, b);
    if (store) {
      rec[chunk * kChunk / 8 + lane] = r;
      rec[chunk * kChunk / 8 + 64 + lane] = r + 1u;
    } else if (r[0] == 0x12345678u && r[1] == 7u) {
      rec[0] = r;
    }
  }
}

// the same, with the next chunk's planes in flight during this chunk's compute
// and stores (two register sets)
template <int NPL, int C>
__global__ __launch_bounds__(256, 2) void piped(const uint8_t* st, int64_t HW, int ngroups, v4u* rec, int store) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  int cg = blockIdx.x;
  if (cg >= ngroups) return;
  auto px_of = [&](int g) -> int64_t {
    const int64_t px = (static_cast<int64_t>(g) * 4 + wid) * kChunk + lane * 16;
    return px < HW ? px : 0;
  };
  v4u v[NPL];
  int64_t px = px_of(cg);
#pragma unroll
  for (int p = 0; p < NPL; ++p) v[p] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(st + p * HW + px));
  for (; cg < ngroups; cg += gridDim.x) {
    const int64_t chunk = static_cast<int64_t>(cg) * 4 + wid;
    v4u a = v[0], b = v[1];
#pragma unroll
    for (int p = 2; p < NPL; p += 2) {
      a ^= v[p];
      b += v[p + 1];
    }
    const int nx = cg + gridDim.x;
    if (nx < ngroups) {
      const int64_t pn = px_of(nx);
#pragma unroll
      for (int p = 0; p < NPL; ++p) v[p] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(st + p * HW + pn));
    }
    const v4u r = churn<C>(a, b);
    if (chunk * kChunk >= HW) continue;
    if (store) {
      rec[chunk * kChunk / 8 + lane] = r;
      rec[chunk * kChunk / 8 + 64 + lane] = r + 1u;
    } else if (r[0] == 0x12345678u && r[1] == 7u) {
      rec[0] = r;
    }
  }
}

template <typename K>
static float time_it(K launch, hipEvent_t a, hipEvent_t b) {
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

template <int NPL, int C>
static void run(const uint8_t* st, int64_t HW, v4u* rec, int n_cu, hipEvent_t a, hipEvent_t b) {
  const int ngroups = static_cast<int>((HW / kChunk + 3) / 4);
  for (int per_cu : {2, 3, 6}) {
    const int grid = per_cu * n_cu;
    for (int store = 0; store < 2; ++store) {
      const float t0 = time_it([&] { hipLaunchKernelGGL((plain<NPL, C>), dim3(grid), dim3(256), 0, 0, st, HW, ngroups, rec, store); }, a, b);
      const float t1 = time_it([&] { hipLaunchKernelGGL((piped<NPL, C>), dim3(grid), dim3(256), 0, 0, st, HW, ngroups, rec, store); }, a, b);
      const double bytes = NPL * static_cast<double>(HW) + (store ? 2.0 * HW : 0.0);
      printf("{\"planes\": %d, \"churn\": %d, \"wg_per_cu\": %d, \"records\": %d, \"plain_us\": %.2f, \"piped_us\": %.2f, "
             "\"plain_GBps\": %.0f, \"piped_GBps\": %.0f}\n",
             NPL, C, per_cu, store, t0 * 1e3, t1 * 1e3, bytes / (t0 * 1e-3) / 1e9, bytes / (t1 * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
}

int main() {
  const int64_t HW = 3840LL * 2160;
  const int64_t bytes = 46 * HW;
  uint8_t* st;
  v4u* rec;
  if (hipMalloc(&st, bytes) != hipSuccess || hipMalloc(&rec, 2 * HW) != hipSuccess) return 1;
  (void)hipMemset(st, 7, bytes);
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  run<24, 0>(st, HW, rec, n_cu, a, b);
  run<24, 12>(st, HW, rec, n_cu, a, b);
  run<24, 48>(st, HW, rec, n_cu, a, b);
  run<16, 12>(st, HW, rec, n_cu, a, b);
  return 0;
}
