// Microbenchmark (measurement only, not part of the library): the store floor
// of k_cloud at the multi-view scale.  cloud_store_bw writes one 4K view's
// 98 MB of points, which the 256 MB Infinity Cache can absorb; here V views'
// points (V x 6.55 M by default: 8 views = 786 MB of xyz + BGR) leave for HBM.
// Patterns (one lane per point, grid-stride over the points):
//   0 k_cloud's: xyz as one 12-B store, BGR as a 2-B + a 1-B store
//   1 xyz only (12-B stores)
//   2 BGR only (2-B + 1-B stores)
//   3 the same bytes as 16-B stores (15 B per point: the ideal shape)
//   4 pattern 0 plus k_cloud's reads (12-bit records 1.5 B/px + texture 3 B/px
//     of the views' pixels, 16-B loads)
//   5 pattern 0 with the xyz stores nontemporal (k_cloud since round 5)
//   6 pattern 3 with nontemporal 16-B stores
//   7 pattern 0 with the xyz and BGR stores nontemporal
//   8 pattern 4 with the xyz stores nontemporal (k_cloud's traffic since round 5)
// One JSON line per pattern: avg / best over 20 timed launches.
//   cloud_store_floor [views [points_per_view [pixels_per_view]]]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v3u __attribute__((ext_vector_type(3)));

template <int PAT>
__global__ __launch_bounds__(256) void pts_k(uint8_t* xyz, uint8_t* bgr, const v4u* side, int64_t npts, int64_t nside,
                                             unsigned* sink) {
  const int64_t nthreads = static_cast<int64_t>(gridDim.x) * 256;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  unsigned acc = 0;
  if (PAT == 4 || PAT == 8) {  // the read share: nside 16-B words over the grid
    for (int64_t g = t0; g < nside; g += nthreads) {
      const v4u r = side[g];
      acc ^= r[0] ^ r[3];
    }
  }
  if (PAT == 3 || PAT == 6) {  // 15 B per point as 16-B stores
    const int64_t nw = (15 * npts) / 16;
    for (int64_t i = t0; i < nw; i += nthreads) {
      const unsigned f = static_cast<unsigned>(i);
      if (PAT == 6) __builtin_nontemporal_store(v4u{f, f + 1u, f + 2u, f + 3u}, reinterpret_cast<v4u*>(xyz + 16 * i));
      else *reinterpret_cast<v4u*>(xyz + 16 * i) = v4u{f, f + 1u, f + 2u, f + 3u};
    }
  } else {
    constexpr bool kNtXyz = PAT >= 5, kNtBgr = PAT == 7;
    for (int64_t i = t0; i < npts; i += nthreads) {
      const unsigned f = static_cast<unsigned>(i) ^ acc;
      if (PAT != 2) {
        unsigned* x = reinterpret_cast<unsigned*>(xyz + 12 * i);
        if (kNtXyz) {
          __builtin_nontemporal_store(f, x);
          __builtin_nontemporal_store(f + 1u, x + 1);
          __builtin_nontemporal_store(f + 2u, x + 2);
        } else {
          *reinterpret_cast<v3u*>(x) = v3u{f, f + 1u, f + 2u};
        }
      }
      if (PAT != 1) {
        if (kNtBgr) {
          __builtin_nontemporal_store(static_cast<uint16_t>(f), reinterpret_cast<uint16_t*>(bgr + 3 * i));
          __builtin_nontemporal_store(static_cast<uint8_t>(f >> 16), bgr + 3 * i + 2);
        } else {
          *reinterpret_cast<uint16_t*>(bgr + 3 * i) = static_cast<uint16_t>(f);
          bgr[3 * i + 2] = static_cast<uint8_t>(f >> 16);
        }
      }
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main(int argc, char** argv) {
  const int V = argc > 1 ? atoi(argv[1]) : 8;
  const int64_t ppv = argc > 2 ? atoll(argv[2]) : 6548659;
  const int64_t hw = argc > 3 ? atoll(argv[3]) : 3840LL * 2160;
  const int64_t npts = ppv * V;
  const int64_t nside = (hw * V * 9 / 2) / 16;  // 4.5 B/px: records 1.5 + texture 3
  uint8_t *xyz, *bgr;
  v4u* side;
  unsigned* sink;
  // xyz: 12 B per point (patterns 0, 1, 4) or 16 (15 * npts / 16) B (pattern 3)
  const int64_t xyz_bytes = 15 * npts + 64, bgr_bytes = 3 * npts + 64;
  if (16 * ((15 * npts) / 16) > xyz_bytes || 12 * npts > xyz_bytes || 3 * npts > bgr_bytes) return 4;
  if (hipMalloc(&xyz, xyz_bytes) != hipSuccess || hipMalloc(&bgr, bgr_bytes) != hipSuccess ||
      hipMalloc(&side, 16 * nside + 64) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess)
    return 1;
  (void)hipMemset(side, 1, 16 * nside);
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  for (int per_cu : {4, 8}) {
    const int gx = per_cu * n_cu;
    for (int pat = 0; pat <= 8; ++pat) {
      float best = 1e30f, sum = 0.f;
      for (int r = 0; r < 23; ++r) {
        (void)hipEventRecord(a, 0);
        switch (pat) {
          case 0: hipLaunchKernelGGL(pts_k<0>, dim3(gx), dim3(256), 0, 0, xyz, bgr, side, npts, nside, sink); break;
          case 1: hipLaunchKernelGGL(pts_k<1>, dim3(gx), dim3(256), 0, 0, xyz, bgr, side, npts, nside, sink); break;
          case 2: hipLaunchKernelGGL(pts_k<2>, dim3(gx), dim3(256), 0, 0, xyz, bgr, side, npts, nside, sink); break;
          case 3: hipLaunchKernelGGL(pts_k<3>, dim3(gx), dim3(256), 0, 0, xyz, bgr, side, npts, nside, sink); break;
          case 4: hipLaunchKernelGGL(pts_k<4>, dim3(gx), dim3(256), 0, 0, xyz, bgr, side, npts, nside, sink); break;
          case 5: hipLaunchKernelGGL(pts_k<5>, dim3(gx), dim3(256), 0, 0, xyz, bgr, side, npts, nside, sink); break;
          case 6: hipLaunchKernelGGL(pts_k<6>, dim3(gx), dim3(256), 0, 0, xyz, bgr, side, npts, nside, sink); break;
          case 7: hipLaunchKernelGGL(pts_k<7>, dim3(gx), dim3(256), 0, 0, xyz, bgr, side, npts, nside, sink); break;
          default: hipLaunchKernelGGL(pts_k<8>, dim3(gx), dim3(256), 0, 0, xyz, bgr, side, npts, nside, sink);
        }
        (void)hipEventRecord(b, 0);
        if (hipEventSynchronize(b) != hipSuccess) return 3;
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r >= 3) {
          sum += ms;
          if (ms < best) best = ms;
        }
      }
      const double wbytes = pat == 1 ? 12.0 * npts : pat == 2 ? 3.0 * npts : 15.0 * npts;
      const double rbytes = pat == 4 || pat == 8 ? 16.0 * nside : 0.0;
      const double avg = sum / 20.0;
      printf("{\"views\": %d, \"points\": %lld, \"wg_per_cu\": %d, \"pattern\": %d, \"best_us\": %.2f, \"avg_us\": %.2f, "
             "\"write_GBps\": %.0f, \"total_GBps\": %.0f}\n",
             V, static_cast<long long>(npts), per_cu, pat, best * 1e3, avg * 1e3, wbytes / (avg * 1e-3) / 1e9,
             (wbytes + rbytes) / (avg * 1e-3) / 1e9);
      fflush(stdout);
    }
  }
  return 0;
}
