// Microbenchmark (measurement only, not part of the library): the HBM floor of
// the cloud-only k_decode access pattern at the multi-view configs' scale --
// V views of 3840x2160, 46-plane stacks ([V][46][H*W]), of which the first 24
// planes are read once (16 B per lane, lane = 16 contiguous pixels, wave =
// 1024-pixel chunk, non-temporal), and the 12-bit records written (24 B per
// lane as two 12-B stores: 1.5 B/px), on k_decode's grid: (workgroups per
// view, V), each workgroup striding over its view's 4-chunk groups.
// Unlike decode_pipeline_bw (one view: its 199 MB of planes fit the 256 MB
// Infinity Cache, so repeated launches are partly served on-die), V = 5 reads
// 995 MB per launch: the re-runs stream from HBM as k_decode's do.
// Prints one JSON line per (views, workgroups per CU, stores).
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v3u __attribute__((ext_vector_type(3)));
constexpr int kChunk = 1024;
constexpr int kPlanesStack = 46;

template <int NPL>
__global__ __launch_bounds__(256, 3) void floor_k(const uint8_t* st, int64_t HW, int64_t vs, int ngroups, uint8_t* rec,
                                                  int store) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int view = blockIdx.y;
  const uint8_t* vb = st + view * vs;
  uint8_t* rb = rec + view * (HW * 3 / 2);
  for (int cg = blockIdx.x; cg < ngroups; cg += gridDim.x) {
    const int64_t chunk = static_cast<int64_t>(cg) * 4 + wid;
    const int64_t px = chunk * kChunk + lane * 16;
    if (px >= HW) continue;
    v4u v[NPL];
#pragma unroll
    for (int p = 0; p < NPL; ++p) v[p] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(vb + p * HW + px));
    v4u a = v[0], b = v[1];
#pragma unroll
    for (int p = 2; p < NPL; p += 2) {
      a ^= v[p];
      b += v[p + 1];
    }
    // the chunk's 1536 record bytes, 24 per lane, in the store shape `store`
    uint8_t* cb = rb + chunk * (kChunk * 3 / 2);
    const uint32_t w[6] = {a.x, a.y, a.z, b.x, b.y, b.w ^ a.w};
    if (store == 1) {  // k_decode's: lane l's 24 B at 24 l, two 12-B stores (stride 24 B per instruction)
      uint32_t* ro = reinterpret_cast<uint32_t*>(cb + 24 * lane);
      *reinterpret_cast<v3u*>(ro) = v3u{w[0], w[1], w[2]};
      *reinterpret_cast<v3u*>(ro + 3) = v3u{w[3], w[4], w[5]};
    } else if (store == 2) {  // halves: 12 B at 12 l, then at 768 + 12 l (768 B contiguous per instruction)
      *reinterpret_cast<v3u*>(cb + 12 * lane) = v3u{w[0], w[1], w[2]};
      *reinterpret_cast<v3u*>(cb + 768 + 12 * lane) = v3u{w[3], w[4], w[5]};
    } else if (store == 3) {  // 16 B at 16 l, 8 B at 1024 + 8 l (1 KB, then 512 B contiguous)
      *reinterpret_cast<v4u*>(cb + 16 * lane) = v4u{w[0], w[1], w[2], w[3]};
      *reinterpret_cast<uint2*>(cb + 1024 + 8 * lane) = make_uint2(w[4], w[5]);
    } else if (store == 4) {  // three 8-B stores, 512 B contiguous each
      for (int k = 0; k < 3; ++k) *reinterpret_cast<uint2*>(cb + 512 * k + 8 * lane) = make_uint2(w[2 * k], w[2 * k + 1]);
    } else if (store == 5) {  // store 3 non-temporal
      __builtin_nontemporal_store(v4u{w[0], w[1], w[2], w[3]}, reinterpret_cast<v4u*>(cb + 16 * lane));
      typedef unsigned v2u __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(v2u{w[4], w[5]}, reinterpret_cast<v2u*>(cb + 1024 + 8 * lane));
    } else if (a.x == 0x12345678u && b.y == 7u) {
      rb[0] = 1;
    }
  }
}

int main(int argc, char** argv) {
  // cloud_decode_floor [views [H W [quick]]]: 5 views of 3840x2160 by default
  const int V = argc > 1 ? atoi(argv[1]) : 5;
  const int64_t HW = argc > 3 ? static_cast<int64_t>(atoi(argv[2])) * atoi(argv[3]) : 3840LL * 2160;
  const int64_t vs = kPlanesStack * HW;
  uint8_t *st, *rec;
  if (hipMalloc(&st, vs * V) != hipSuccess || hipMalloc(&rec, HW * 3 / 2 * V + 64) != hipSuccess) return 1;
  (void)hipMemset(st, 7, vs * V);
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int ngroups = static_cast<int>((HW / kChunk + 3) / 4);
  const bool quick = argc > 4;  // cloud_decode_floor V H W quick: 3 per CU, no records / k_decode's stores only
  for (int per_cu : {3, 4}) {
    if (quick && per_cu != 3) continue;
    const int gx = (per_cu * n_cu + V - 1) / V;
    for (int store = 0; store < (quick ? 2 : 6); ++store) {
      float best = 1e30f, sum = 0.f;
      for (int r = 0; r < 23; ++r) {
        (void)hipEventRecord(a, 0);
        hipLaunchKernelGGL(floor_k<24>, dim3(gx, V), dim3(256), 0, 0, st, HW, vs, ngroups, rec, store);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r >= 3) {
          sum += ms;
          if (ms < best) best = ms;
        }
      }
      const double bytes = (24.0 * HW + (store ? 1.5 * HW : 0.0)) * V;  // (the same 1.5 B/px in every shape)
      const double avg = sum / 20.0;
      printf("{\"views\": %d, \"px_per_view\": %lld, \"wg_per_cu\": %d, \"store_shape\": %d, \"best_us\": %.2f, \"avg_us\": %.2f, "
             "\"GBps_avg\": %.0f, \"frac_avg\": %.3f}\n",
             V, static_cast<long long>(HW), per_cu, store, best * 1e3, avg * 1e3, bytes / (avg * 1e-3) / 1e9, bytes / (avg * 1e-3) / 8e12);
      fflush(stdout);
    }
  }
  return 0;
}
