// libslgpu.so, part 2 -- the merge stage after the per-view clouds (SURVEY.md
// §8(f)-3, server/processing.py:116-182): voxel downsample and statistical
// outlier removal of the merged cloud, as Open3D's PointCloud::VoxelDownSample
// and PointCloud::RemoveStatisticalOutliers compute them (Open3D is not in
// this image: the algorithms are restated from its published source, and
// parity is unpinned -- oracle/merge_oracle.py is the CPU restatement the
// tests check against).
//
//   voxel downsample: min bound (exact reduction) -> linear voxel key of every
//     point, (p - (min - vs/2)) / vs floored per axis -> stable LSD radix sort
//     of (key, index) -> per voxel, the sums of its points and colours in
//     ascending point index (Open3D's AddPoint order, so the f64 sums are
//     bit-identical) / count.  Output in ascending voxel key (Open3D: hash
//     order).
//   statistical outliers: exact k nearest neighbours (the point itself
//     included, nanoflann's ((dx^2 + dy^2) + dz^2) in f64) on a uniform grid of
//     sorted cells, searched ring by ring until the k-th distance is inside the
//     searched cube; mean of the k square roots in ascending order; the cloud
//     mean / std (Bessel) of those means are sequential sums on the host, as
//     std::accumulate / std::inner_product do them; keep 0 < mean < cloud_mean
//     + std_ratio * std.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <limits>
#include <map>
#include <mutex>
#include <vector>

#include "slgpu.h"

#pragma clang fp contract(off)

// from slgpu.hip
int slgpu_fail(sl_ctx* c, int code, const char* msg);
int slgpu_device(const sl_ctx* c);

namespace {

constexpr int kT = 256;
constexpr int kRsItems = 16;                // keys per thread in a radix-sort tile
constexpr int kRsTile = kT * kRsItems;      // 4096
constexpr int kRsBits = 4;                  // digit width
constexpr int kRsBins = 1 << kRsBits;
constexpr int kMaxK = 32;                   // largest nb_neighbors

#define MTRY(ctx, expr)                                                  \
  do {                                                                   \
    hipError_t e_ = (expr);                                              \
    if (e_ != hipSuccess) return slgpu_fail((ctx), SL_EHIP, hipGetErrorString(e_)); \
  } while (0)

// ------------------------------------------------------------------ bounds ----
__global__ __launch_bounds__(kT) void k_bounds(const double* xyz, int64_t n, double* part) {
  __shared__ double s[6][kT];
  double v[6] = {INFINITY, INFINITY, INFINITY, -INFINITY, -INFINITY, -INFINITY};
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * kT) {
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      const double x = xyz[3 * i + k];
      v[k] = fmin(v[k], x);
      v[3 + k] = fmax(v[3 + k], x);
    }
  }
#pragma unroll
  for (int k = 0; k < 6; ++k) s[k][threadIdx.x] = v[k];
  __syncthreads();
  for (int w = kT / 2; w > 0; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) {
#pragma unroll
      for (int k = 0; k < 3; ++k) {
        s[k][threadIdx.x] = fmin(s[k][threadIdx.x], s[k][threadIdx.x + w]);
        s[3 + k][threadIdx.x] = fmax(s[3 + k][threadIdx.x], s[3 + k][threadIdx.x + w]);
      }
    }
    __syncthreads();
  }
  if (threadIdx.x < 6) part[6 * blockIdx.x + threadIdx.x] = s[threadIdx.x][0];
}

// ------------------------------------------------------- grid cell keys ----
// key = (ix * ny + iy) * nz + iz with i_a = floor((p_a - lo_a) / h); index = i.
__global__ __launch_bounds__(kT) void k_cell_keys(const double* xyz, int64_t n, double lo0, double lo1, double lo2,
                                                  double h, int64_t ny, int64_t nz, uint64_t* keys, uint32_t* vals) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i >= n) return;
  const int64_t ix = static_cast<int64_t>(floor((xyz[3 * i] - lo0) / h));
  const int64_t iy = static_cast<int64_t>(floor((xyz[3 * i + 1] - lo1) / h));
  const int64_t iz = static_cast<int64_t>(floor((xyz[3 * i + 2] - lo2) / h));
  keys[i] = static_cast<uint64_t>((ix * ny + iy) * nz + iz);
  vals[i] = static_cast<uint32_t>(i);
}

// ---------------------------------------------------------- radix sort ----
// Stable LSD sort of (uint64 key, uint32 value), kRsBits per pass.  A pass:
// per-tile digit counts (digit-major), one exclusive scan over them, and a
// scatter in which every key's rank inside its tile is the count of equal
// digits before it (thread-contiguous items, so the order is stable).
__device__ __forceinline__ unsigned digit_of(uint64_t k, int shift) {
  return static_cast<unsigned>(k >> shift) & (kRsBins - 1);
}

__global__ __launch_bounds__(kT) void k_rs_count(const uint64_t* keys, int64_t n, int shift, uint32_t* counts,
                                                 int tiles) {
  __shared__ uint32_t s_c[kRsBins];
  if (threadIdx.x < kRsBins) s_c[threadIdx.x] = 0u;
  __syncthreads();
  // the tile's items in any order: lane-interleaved (coalesced) loads
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kRsTile + threadIdx.x;
  uint32_t c[kRsBins];
#pragma unroll
  for (int d = 0; d < kRsBins; ++d) c[d] = 0u;
#pragma unroll
  for (int j = 0; j < kRsItems; ++j) {
    if (base + j * kT < n) {
      const unsigned d = digit_of(keys[base + j * kT], shift);
#pragma unroll
      for (int e = 0; e < kRsBins; ++e) c[e] += (d == static_cast<unsigned>(e)) ? 1u : 0u;
    }
  }
#pragma unroll
  for (int d = 0; d < kRsBins; ++d)
    if (c[d]) atomicAdd(&s_c[d], c[d]);
  __syncthreads();
  if (threadIdx.x < kRsBins) counts[static_cast<int64_t>(threadIdx.x) * tiles + blockIdx.x] = s_c[threadIdx.x];
}

// Exclusive scan of a uint32 array by one workgroup (thread t owns a
// contiguous stretch); the total goes to *total when non-null.
__global__ __launch_bounds__(kT) void k_scan1(uint32_t* a, int64_t n, uint32_t* total) {
  __shared__ uint32_t s[kT];
  const int64_t per = (n + kT - 1) / kT;
  const int64_t lo = min<int64_t>(n, threadIdx.x * per), hi = min<int64_t>(n, lo + per);
  uint32_t sum = 0u;
  for (int64_t i = lo; i < hi; ++i) sum += a[i];
  s[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0u;
    for (int t = 0; t < kT; ++t) {
      const uint32_t v = s[t];
      s[t] = run;
      run += v;
    }
    if (total) *total = run;
  }
  __syncthreads();
  uint32_t run = s[threadIdx.x];
  for (int64_t i = lo; i < hi; ++i) {
    const uint32_t v = a[i];
    a[i] = run;
    run += v;
  }
}

__global__ __launch_bounds__(kT) void k_rs_scatter(const uint64_t* kin, const uint32_t* vin, uint64_t* kout,
                                                   uint32_t* vout, int64_t n, int shift, const uint32_t* offs,
                                                   int tiles) {
  __shared__ uint32_t s[kRsBins * kT];  // [digit][thread] counts, then their exclusive scan
  __shared__ uint32_t s_part[kT];
  __shared__ uint32_t s_start[kRsBins];  // tile-local start of every digit's run
  __shared__ uint64_t s_k[kRsTile];      // the tile in stable digit order
  __shared__ uint32_t s_v[kRsTile];
  const int t = threadIdx.x;
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kRsTile + static_cast<int64_t>(t) * kRsItems;
  uint64_t k[kRsItems];
  uint32_t v[kRsItems];
  unsigned dg[kRsItems];
  uint32_t c[kRsBins];
#pragma unroll
  for (int d = 0; d < kRsBins; ++d) c[d] = 0u;
#pragma unroll
  for (int j = 0; j < kRsItems; ++j) {
    const bool ok = base + j < n;
    k[j] = ok ? kin[base + j] : 0ull;
    v[j] = ok ? vin[base + j] : 0u;
    dg[j] = ok ? digit_of(k[j], shift) : kRsBins;  // kRsBins: no item
#pragma unroll
    for (int e = 0; e < kRsBins; ++e) c[e] += (dg[j] == static_cast<unsigned>(e)) ? 1u : 0u;
  }
#pragma unroll
  for (int d = 0; d < kRsBins; ++d) s[d * kT + t] = c[d];
  __syncthreads();
  // exclusive scan of s[] (digit-major): thread t owns entries [16 t, 16 t + 16)
  uint32_t loc[kRsBins];
  uint32_t sum = 0u;
#pragma unroll
  for (int j = 0; j < kRsBins; ++j) {
    loc[j] = sum;
    sum += s[kRsBins * t + j];
  }
  s_part[t] = sum;
  __syncthreads();
  if (t < 64) {  // scan of the 256 partial sums by one wave (4 per lane)
    uint32_t a0 = s_part[4 * t], a1 = s_part[4 * t + 1], a2 = s_part[4 * t + 2], a3 = s_part[4 * t + 3];
    const uint32_t tot = a0 + a1 + a2 + a3;
    uint32_t inc = tot;
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(inc, d, 64);
      if (t >= d) inc += y;
    }
    uint32_t ex = inc - tot;
    s_part[4 * t] = ex;
    ex += a0;
    s_part[4 * t + 1] = ex;
    ex += a1;
    s_part[4 * t + 2] = ex;
    ex += a2;
    s_part[4 * t + 3] = ex;
  }
  __syncthreads();
  const uint32_t pre = s_part[t];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kRsBins; ++j) s[kRsBins * t + j] = pre + loc[j];
  __syncthreads();
  // item j of thread t with digit d goes to its tile-local rank: (items with
  // a smaller digit) + (d's items in earlier threads) + (d's items earlier in
  // this thread) -- the stable order; the tile is reordered in LDS, then
  // written out run by run (consecutive threads -> consecutive addresses)
  if (t < kRsBins) s_start[t] = s[t * kT];
  uint32_t run[kRsBins];
#pragma unroll
  for (int d = 0; d < kRsBins; ++d) run[d] = 0u;
#pragma unroll
  for (int j = 0; j < kRsItems; ++j) {
    if (dg[j] < static_cast<unsigned>(kRsBins)) {
      const unsigned d = dg[j];
      uint32_t r = 0u;
#pragma unroll
      for (int e = 0; e < kRsBins; ++e)
        if (d == static_cast<unsigned>(e)) {
          r = run[e];
          ++run[e];
        }
      const uint32_t rank = s[d * kT + t] + r;
      s_k[rank] = k[j];
      s_v[rank] = v[j];
    }
  }
  __syncthreads();
  const int64_t tile0 = static_cast<int64_t>(blockIdx.x) * kRsTile;
  const int tn = static_cast<int>(min<int64_t>(kRsTile, n - tile0));
  for (int i = t; i < tn; i += kT) {
    const uint64_t key = s_k[i];
    const unsigned d = digit_of(key, shift);
    const uint32_t pos = offs[static_cast<int64_t>(d) * tiles + blockIdx.x] + (static_cast<uint32_t>(i) - s_start[d]);
    kout[pos] = key;
    vout[pos] = s_v[i];
  }
}

// ------------------------------------------------------------- segments ----
__global__ __launch_bounds__(kT) void k_heads(const uint64_t* keys, int64_t n, uint32_t* flag) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i < n) flag[i] = (i == 0 || keys[i] != keys[i - 1]) ? 1u : 0u;
}

// Exclusive scan of flag[] (multi-workgroup: per-workgroup sums, one
// workgroup scanning them, then the local scans); total -> *total.
__global__ __launch_bounds__(kT) void k_tile_sums(const uint32_t* a, int64_t n, uint32_t* sums) {
  __shared__ uint32_t s[kT];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kRsTile + static_cast<int64_t>(threadIdx.x) * kRsItems;
  uint32_t sum = 0u;
#pragma unroll
  for (int j = 0; j < kRsItems; ++j)
    if (base + j < n) sum += a[base + j];
  s[threadIdx.x] = sum;
  __syncthreads();
  for (int w = kT / 2; w > 0; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) s[threadIdx.x] += s[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) sums[blockIdx.x] = s[0];
}

__global__ __launch_bounds__(kT) void k_tile_scan(const uint32_t* a, int64_t n, const uint32_t* sums, uint32_t* out) {
  __shared__ uint32_t s[kT];
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kRsTile + static_cast<int64_t>(threadIdx.x) * kRsItems;
  uint32_t v[kRsItems];
  uint32_t sum = 0u;
#pragma unroll
  for (int j = 0; j < kRsItems; ++j) {
    v[j] = base + j < n ? a[base + j] : 0u;
    sum += v[j];
  }
  s[threadIdx.x] = sum;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = sums[blockIdx.x];
    for (int t = 0; t < kT; ++t) {
      const uint32_t x = s[t];
      s[t] = run;
      run += x;
    }
  }
  __syncthreads();
  uint32_t run = s[threadIdx.x];
#pragma unroll
  for (int j = 0; j < kRsItems; ++j) {
    if (base + j < n) out[base + j] = run;
    run += v[j];
  }
}

__global__ __launch_bounds__(kT) void k_seg_starts(const uint32_t* flag, const uint32_t* seg, const uint64_t* keys,
                                                   int64_t n, uint32_t* starts, uint64_t* ukeys) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i < n && flag[i]) {
    starts[seg[i]] = static_cast<uint32_t>(i);
    ukeys[seg[i]] = keys[i];
  }
}

// One voxel per thread: its points in ascending index, summed in that order
// (AccumulatedPoint::AddPoint), averaged (GetAveragePoint / GetAverageColor);
// colours as Open3D holds them (c / 255.0) and writes them (round(clamp * 255)).
__global__ __launch_bounds__(kT) void k_voxel_avg(const uint32_t* starts, int64_t n_vox, int64_t n,
                                                  const uint32_t* idx, const double* xyz, const uint8_t* bgr,
                                                  double* oxyz, uint8_t* obgr) {
  const int64_t s = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (s >= n_vox) return;
  const int64_t a = starts[s], b = s + 1 < n_vox ? static_cast<int64_t>(starts[s + 1]) : n;
  double p0 = 0.0, p1 = 0.0, p2 = 0.0, c0 = 0.0, c1 = 0.0, c2 = 0.0;
  for (int64_t j = a; j < b; ++j) {
    const int64_t i = idx[j];
    p0 += xyz[3 * i];
    p1 += xyz[3 * i + 1];
    p2 += xyz[3 * i + 2];
    if (bgr) {
      c0 += static_cast<double>(bgr[3 * i]) / 255.0;
      c1 += static_cast<double>(bgr[3 * i + 1]) / 255.0;
      c2 += static_cast<double>(bgr[3 * i + 2]) / 255.0;
    }
  }
  const double m = static_cast<double>(b - a);
  oxyz[3 * s] = p0 / m;
  oxyz[3 * s + 1] = p1 / m;
  oxyz[3 * s + 2] = p2 / m;
  if (bgr && obgr) {
    const double cc[3] = {c0 / m, c1 / m, c2 / m};
#pragma unroll
    for (int k = 0; k < 3; ++k) obgr[3 * s + k] = static_cast<uint8_t>(round(fmin(1.0, fmax(0.0, cc[k])) * 255.0));
  }
}

// ------------------------------------------------------------------ kNN ----
struct Grid {
  double lo0, lo1, lo2, h;
  int64_t nx, ny, nz;
};

__device__ __forceinline__ int64_t find_cell(const uint64_t* ukeys, int64_t m, uint64_t key) {
  int64_t a = 0, b = m;  // first >= key
  while (a < b) {
    const int64_t c = (a + b) >> 1;
    if (ukeys[c] < key) a = c + 1;
    else b = c;
  }
  return (a < m && ukeys[a] == key) ? a : -1;
}

// 21-bit Morton interleave: bit i of x -> bit 3 i (y: 3 i + 1, z: 3 i + 2).
__host__ __device__ __forceinline__ uint64_t spread3(uint64_t x) {
  x &= 0x1fffffull;
  x = (x | (x << 32)) & 0x1f00000000ffffull;
  x = (x | (x << 16)) & 0x1f0000ff0000ffull;
  x = (x | (x << 8)) & 0x100f00f00f00f00full;
  x = (x | (x << 4)) & 0x10c30c30c30c30c3ull;
  x = (x | (x << 2)) & 0x1249249249249249ull;
  return x;
}

__host__ __device__ __forceinline__ uint64_t morton3(uint64_t x, uint64_t y, uint64_t z) {
  return spread3(x) | (spread3(y) << 1) | (spread3(z) << 2);
}

// Morton key of every point's finest cell (h0, origin lo); index = i.
__global__ __launch_bounds__(kT) void k_morton_keys(const double* xyz, int64_t n, double lo0, double lo1, double lo2,
                                                    double h, uint64_t* keys, uint32_t* vals) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i >= n) return;
  const uint64_t ix = static_cast<uint64_t>(floor((xyz[3 * i] - lo0) / h));
  const uint64_t iy = static_cast<uint64_t>(floor((xyz[3 * i + 1] - lo1) / h));
  const uint64_t iz = static_cast<uint64_t>(floor((xyz[3 * i + 2] - lo2) / h));
  keys[i] = morton3(ix, iy, iz);
  vals[i] = static_cast<uint32_t>(i);
}

// Level l of the cell pyramid: cells of edge h0 * 2^l = Morton key >> 3 l, each
// a contiguous run of the Morton-sorted points.
__global__ __launch_bounds__(kT) void k_heads_shift(const uint64_t* keys, int64_t n, int sh, uint32_t* flag) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i < n) flag[i] = (i == 0 || (keys[i] >> sh) != (keys[i - 1] >> sh)) ? 1u : 0u;
}

__global__ __launch_bounds__(kT) void k_level_cells(const uint32_t* flag, const uint32_t* seg, const uint64_t* keys,
                                                    int64_t n, int sh, uint32_t* starts, uint64_t* ukeys) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i < n && flag[i]) {
    starts[seg[i]] = static_cast<uint32_t>(i);
    ukeys[seg[i]] = keys[i] >> sh;
  }
}

// Cell of every sorted point: (exclusive scan of the cell heads) + head - 1.
__global__ __launch_bounds__(kT) void k_cell_of(const uint32_t* flag, const uint32_t* seg, int64_t n, uint32_t* out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i < n) out[i] = seg[i] + flag[i] - 1u;
}

// Coordinates in Morton order (contiguous candidate runs for the kNN).
__global__ __launch_bounds__(kT) void k_gather_sorted(const double* xyz, const uint32_t* sidx, int64_t n, double* sxyz) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (t >= n) return;
  const int64_t i = sidx[t];
#pragma unroll
  for (int k = 0; k < 3; ++k) sxyz[3 * t + k] = xyz[3 * i + k];
}

// The 27 neighbour cells (-1: empty or outside) of every occupied cell of a
// level, (dx, dy, dz) in -1..1 nesting order.
__global__ __launch_bounds__(kT) void k_cell_neighbours(const uint64_t* ukeys, int64_t m, int64_t nx, int64_t ny,
                                                        int64_t nz, int32_t* nbr);

__device__ __forceinline__ uint64_t compact3(uint64_t x) {
  x &= 0x1249249249249249ull;
  x = (x | (x >> 2)) & 0x10c30c30c30c30c3ull;
  x = (x | (x >> 4)) & 0x100f00f00f00f00full;
  x = (x | (x >> 8)) & 0x1f0000ff0000ffull;
  x = (x | (x >> 16)) & 0x1f00000000ffffull;
  x = (x | (x >> 32)) & 0x1fffffull;
  return x;
}

__global__ __launch_bounds__(kT) void k_cell_neighbours(const uint64_t* ukeys, int64_t m, int64_t nx, int64_t ny,
                                                        int64_t nz, int32_t* nbr) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (c >= m) return;
  const uint64_t key = ukeys[c];
  const int64_t x = static_cast<int64_t>(compact3(key)), y = static_cast<int64_t>(compact3(key >> 1)),
                z = static_cast<int64_t>(compact3(key >> 2));
  int e = 0;
  for (int dx = -1; dx <= 1; ++dx)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dz = -1; dz <= 1; ++dz, ++e) {
        const int64_t a = x + dx, b = y + dy, d = z + dz;
        int64_t f = -1;
        if (a >= 0 && a < nx && b >= 0 && b < ny && d >= 0 && d < nz) f = find_cell(ukeys, m, morton3(a, b, d));
        nbr[27 * c + e] = static_cast<int32_t>(f);
      }
}

// One candidate squared distance into the sorted k-best list bd (ascending;
// bd[kk - 1] is the k-th, kept in kth).
template <int KM>
__device__ __forceinline__ void knn_take(double (&bd)[KM], double& kth, int64_t& found, int64_t kk, int k, double dd) {
  ++found;
  if (dd < kth || found <= kk) {
    double v = dd;
#pragma unroll
    for (int e = 0; e < KM; ++e) {
      const double lo = fmin(bd[e], v), hi = fmax(bd[e], v);
      bd[e] = lo;
      v = hi;
    }
    double t2 = bd[KM - 1];
    if (KM != k || kk != k) {
      t2 = bd[0];
#pragma unroll
      for (int e = 1; e < KM; ++e)
        if (e == kk - 1) t2 = bd[e];
    }
    kth = t2;
  }
}

constexpr int kMaxLevels = 22;

struct Pyramid {
  const uint64_t* ukeys[kMaxLevels];
  const uint32_t* ustart[kMaxLevels];
  int64_t m[kMaxLevels];
  int64_t dim[kMaxLevels][3];  // cells per axis
  double lo0, lo1, lo2, h0;
  int l0, levels;
  unsigned* stats;        // optional: queries finished per level (measurement only)
  uint32_t* slow_q;       // queries not settled at l0 (sorted positions)
  unsigned* slow_n;
  const double* sxyz;     // coordinates in Morton order
  const uint32_t* cell0;  // level-l0 cell of every sorted point
  const int32_t* nbr0;    // level-l0 27-neighbour table
  const uint32_t* fchild[kMaxLevels];  // levels > l0: first child of every cell (+ sentinel)
};

// Mean distance to the k nearest points (the point itself included) of every
// point; queries in Morton order (one per thread).  From level l0 up: the
// 3x3x3 cells around the query's cell at level l (every ring at the top
// level); done once k points are found and the k-th is closer than the
// searched cube's boundary, else the next coarser level starts over.  KM: the
// register list length (k itself for the common k = 20, else kMaxK).
template <int KM>
__global__ __launch_bounds__(kT) void k_knn_mean(const double* xyz, int64_t n, const uint32_t* sidx, Pyramid py,
                                                 int k, double* avg) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (j >= n) return;
  const int64_t qi = sidx[j];
  const double q0 = xyz[3 * qi], q1 = xyz[3 * qi + 1], q2 = xyz[3 * qi + 2];
  const int64_t fx = static_cast<int64_t>(floor((q0 - py.lo0) / py.h0));
  const int64_t fy = static_cast<int64_t>(floor((q1 - py.lo1) / py.h0));
  const int64_t fz = static_cast<int64_t>(floor((q2 - py.lo2) / py.h0));
  const int64_t kk = min<int64_t>(k, n);
  const double margin = 1e-12 * (fabs(q0) + fabs(q1) + fabs(q2) + fabs(py.lo0) + fabs(py.lo1) + fabs(py.lo2));
  double bd[KM];
  // ---- level l0: the 27 cells of the query's cell from its neighbour table,
  // candidates read from the Morton-ordered copy, four loads in flight ----
  {
#pragma unroll
    for (int e = 0; e < KM; ++e) bd[e] = INFINITY;
    double kth = INFINITY;
    int64_t found = 0;
    const int l = py.l0;
    const uint32_t* us = py.ustart[l];
    const int64_t m = py.m[l];
    const int32_t* nb = py.nbr0 + 27 * static_cast<int64_t>(py.cell0[j]);
    for (int e = 0; e < 27; ++e) {
      const int64_t c = nb[e];
      if (c < 0) continue;
      const int64_t a = us[c], b = c + 1 < m ? static_cast<int64_t>(us[c + 1]) : n;
      int64_t t = a;
      for (; t + 4 <= b; t += 4) {
        double p[12];
#pragma unroll
        for (int u = 0; u < 12; ++u) p[u] = py.sxyz[3 * t + u];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const double d0 = q0 - p[3 * u], d1 = q1 - p[3 * u + 1], d2 = q2 - p[3 * u + 2];
          knn_take<KM>(bd, kth, found, kk, k, ((d0 * d0) + d1 * d1) + d2 * d2);  // nanoflann L2_Adaptor order
        }
      }
      for (; t < b; ++t) {
        const double d0 = q0 - py.sxyz[3 * t], d1 = q1 - py.sxyz[3 * t + 1], d2 = q2 - py.sxyz[3 * t + 2];
        knn_take<KM>(bd, kth, found, kk, k, ((d0 * d0) + d1 * d1) + d2 * d2);
      }
    }
    const double h = ldexp(py.h0, l);
    const int64_t cx = fx >> l, cy = fy >> l, cz = fz >> l;
    const int64_t nx = py.dim[l][0], ny = py.dim[l][1], nz = py.dim[l][2];
    const double lo0 = py.lo0 + static_cast<double>(cx - 1) * h, hi0 = py.lo0 + static_cast<double>(cx + 2) * h;
    const double lo1 = py.lo1 + static_cast<double>(cy - 1) * h, hi1 = py.lo1 + static_cast<double>(cy + 2) * h;
    const double lo2 = py.lo2 + static_cast<double>(cz - 1) * h, hi2 = py.lo2 + static_cast<double>(cz + 2) * h;
    double bound = fmin(fmin(q0 - lo0, hi0 - q0), fmin(fmin(q1 - lo1, hi1 - q1), fmin(q2 - lo2, hi2 - q2)));
    bound = fmax(bound - margin - 1e-12 * h, 0.0);
    const bool all = cx - 1 <= 0 && cy - 1 <= 0 && cz - 1 <= 0 && cx + 1 >= nx - 1 && cy + 1 >= ny - 1 &&
                     cz + 1 >= nz - 1;
    if (all || (found >= kk && kth < bound * bound)) {
      if (py.stats) atomicAdd(py.stats + l, 1u);
      double s = 0.0;
#pragma unroll
      for (int e = 0; e < KM; ++e)
        if (e < kk) s += sqrt(bd[e]);
      avg[qi] = kk > 0 ? s / static_cast<double>(kk) : -1.0;
      return;
    }
  }
  // not settled at l0 (an isolated point): to the cooperative kernel
  py.slow_q[atomicAdd(py.slow_n, 1u)] = static_cast<uint32_t>(j);
}

// The queries k_knn_mean left, one wave each, from level l0 + 1 up (the top
// level again, with every ring, when l0 is the top): the lanes split every
// cell's run of Morton-ordered points, each keeping its own k best; after
// every ring the 64 lists are merged by k rounds of wave-min selection, which
// yields the k smallest in ascending order (summed in that order).
template <int KM>
__global__ __launch_bounds__(64) void k_knn_slow(const uint32_t* sidx, int64_t n, Pyramid py, int k, double* avg) {
  const int lane = threadIdx.x;
  const int64_t j = py.slow_q[blockIdx.x];
  const int64_t qi = sidx[j];
  const double q0 = py.sxyz[3 * j], q1 = py.sxyz[3 * j + 1], q2 = py.sxyz[3 * j + 2];
  const int64_t fx = static_cast<int64_t>(floor((q0 - py.lo0) / py.h0));
  const int64_t fy = static_cast<int64_t>(floor((q1 - py.lo1) / py.h0));
  const int64_t fz = static_cast<int64_t>(floor((q2 - py.lo2) / py.h0));
  const int64_t kk = min<int64_t>(k, n);
  const double margin = 1e-12 * (fabs(q0) + fabs(q1) + fabs(q2) + fabs(py.lo0) + fabs(py.lo1) + fabs(py.lo2));
  double bd[KM];
  for (int l = min(py.l0 + 1, py.levels - 1); l < py.levels; ++l) {
#pragma unroll
    for (int e = 0; e < KM; ++e) bd[e] = INFINITY;
    double kth = INFINITY;
    int64_t found = 0;
    const int64_t cx = fx >> l, cy = fy >> l, cz = fz >> l;
    const int64_t nx = py.dim[l][0], ny = py.dim[l][1], nz = py.dim[l][2];
    const uint64_t* uk = py.ukeys[l];
    const uint32_t* us = py.ustart[l];
    const int64_t m = py.m[l];
    const bool top = l == py.levels - 1;
    const double h = ldexp(py.h0, l);
    for (int64_t r = 0; r <= (top ? (int64_t)1 << 40 : 1); ++r) {
      for (int64_t dx = -r; dx <= r; ++dx) {
        const int64_t x = cx + dx;
        if (x < 0 || x >= nx) continue;
        for (int64_t dy = -r; dy <= r; ++dy) {
          const int64_t y = cy + dy;
          if (y < 0 || y >= ny) continue;
          const bool edge = (dx == -r || dx == r || dy == -r || dy == r);
          for (int64_t dz = -r; dz <= r; dz += (edge || r == 0) ? 1 : 2 * r) {
            const int64_t z = cz + dz;
            if (z < 0 || z >= nz) continue;
            const int64_t c = find_cell(uk, m, morton3(x, y, z));
            if (c < 0) continue;
            const int64_t a = us[c], b = c + 1 < m ? static_cast<int64_t>(us[c + 1]) : n;
            for (int64_t t = a + lane; t < b; t += 64) {
              const double d0 = q0 - py.sxyz[3 * t], d1 = q1 - py.sxyz[3 * t + 1], d2 = q2 - py.sxyz[3 * t + 2];
              knn_take<KM>(bd, kth, found, kk, k, ((d0 * d0) + d1 * d1) + d2 * d2);  // nanoflann order
            }
          }
        }
      }
      // the wave's k smallest: k rounds of (value, lane) wave-min on the list heads
      long long fw = found;
#pragma unroll
      for (int d = 32; d > 0; d >>= 1) fw += __shfl_xor(fw, d, 64);
      double tmp[KM];
#pragma unroll
      for (int e = 0; e < KM; ++e) tmp[e] = bd[e];
      double kthw = INFINITY, ssum = 0.0;
      for (int64_t i = 0; i < kk; ++i) {
        double mv = tmp[0];
        int ml = lane;
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) {
          const double ov = __shfl_xor(mv, d, 64);
          const int ol = __shfl_xor(ml, d, 64);
          if (ov < mv || (ov == mv && ol < ml)) {
            mv = ov;
            ml = ol;
          }
        }
        if (lane == ml) {
#pragma unroll
          for (int e = 0; e + 1 < KM; ++e) tmp[e] = tmp[e + 1];
          tmp[KM - 1] = INFINITY;
        }
        kthw = mv;
        ssum += sqrt(mv);
      }
      const double lo0 = py.lo0 + static_cast<double>(cx - r) * h, hi0 = py.lo0 + static_cast<double>(cx + r + 1) * h;
      const double lo1 = py.lo1 + static_cast<double>(cy - r) * h, hi1 = py.lo1 + static_cast<double>(cy + r + 1) * h;
      const double lo2 = py.lo2 + static_cast<double>(cz - r) * h, hi2 = py.lo2 + static_cast<double>(cz + r + 1) * h;
      double bound = fmin(fmin(q0 - lo0, hi0 - q0), fmin(fmin(q1 - lo1, hi1 - q1), fmin(q2 - lo2, hi2 - q2)));
      bound = fmax(bound - margin - 1e-12 * h, 0.0);
      const bool all = cx - r <= 0 && cy - r <= 0 && cz - r <= 0 && cx + r >= nx - 1 && cy + r >= ny - 1 &&
                       cz + r >= nz - 1;
      if (all || (fw >= kk && kthw < bound * bound)) {
        if (lane == 0) {
          avg[qi] = kk > 0 ? ssum / static_cast<double>(kk) : -1.0;
          if (py.stats) atomicAdd(py.stats + kMaxLevels + l, 1u);
        }
        return;
      }
    }
  }
}

// First child (at level l - 1) of every cell of level l >= 1, plus a sentinel
// fc[m_l] = m_{l-1}: the children of cell c are fc[c] .. fc[c + 1] - 1 (a
// parent's children are the consecutive cells whose key >> 3 is its key).
__global__ __launch_bounds__(kT) void k_first_child(const uint64_t* ukeys, int64_t m, const uint64_t* ckeys,
                                                    int64_t mc, uint32_t* fc) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (c > m) return;
  if (c == m) {
    fc[m] = static_cast<uint32_t>(mc);
    return;
  }
  const uint64_t key = ukeys[c] << 3;
  int64_t a = 0, b = mc;  // first child key >= key
  while (a < b) {
    const int64_t h = (a + b) >> 1;
    if (ckeys[h] < key) a = h + 1;
    else b = h;
  }
  fc[c] = static_cast<uint32_t>(a);
}

constexpr int kBestCap = 4096;  // frontier cells per query (LDS)

// Squared distance from q to the box of cell (x, y, z) of edge h, lowered by a
// relative margin far above the rounding of point -> cell assignment and of
// the squared sums: a lower bound of every member point's computed distance.
__device__ __forceinline__ double cell_mind2(const Pyramid& py, uint64_t key, double h, double q0, double q1,
                                             double q2) {
  const double x = static_cast<double>(compact3(key)), y = static_cast<double>(compact3(key >> 1)),
               z = static_cast<double>(compact3(key >> 2));
  auto gap = [&](double lo, double c, double q) {
    const double a = lo + c * h, b = lo + (c + 1.0) * h;
    const double marg = 1e-12 * (fabs(a) + fabs(b) + fabs(q) + fabs(lo)) + 1e-12 * h;
    return fmax(fmax(a - q, q - b) - marg, 0.0);
  };
  const double g0 = gap(py.lo0, x, q0), g1 = gap(py.lo1, y, q1), g2 = gap(py.lo2, z, q2);
  return ((g0 * g0 + g1 * g1) + g2 * g2) * (1.0 - 1e-12);
}

// The queries k_knn_mean left (isolated points), one wave each: best-first
// search of the cell pyramid.  The frontier (cells with a lower bound of their
// points' distances) lives in LDS; each step pops the nearest cell -- its
// children are pushed, or, at the start level, its points are scanned -- until
// the nearest frontier cell is no closer than the k-th best distance.  The k
// best squared distances are one sorted list across the wave (lane i holds the
// i-th smallest): a candidate below the k-th is inserted by one shift.  The
// result is the same multiset of k smallest distances as the exhaustive
// search, so the mean (ascending square roots) is bit-identical.  Frontier
// overflow (more than kBestCap cells) hands the query to k_knn_slow.
template <int KM>
__global__ __launch_bounds__(64) void k_knn_best(const uint32_t* sidx, int64_t n, Pyramid py, int k, double* avg,
                                                 uint32_t* over_q, unsigned* over_n) {
  __shared__ double f_key[kBestCap];
  __shared__ uint32_t f_cell[kBestCap];
  __shared__ uint8_t f_lev[kBestCap];
  __shared__ int f_n;
  const int lane = threadIdx.x;
  const int64_t j = py.slow_q[blockIdx.x];
  const int64_t qi = sidx[j];
  const double q0 = py.sxyz[3 * j], q1 = py.sxyz[3 * j + 1], q2 = py.sxyz[3 * j + 2];
  const int kk = static_cast<int>(min<int64_t>(k, n));
  const int top = py.levels - 1;
  // frontier: every cell of the top level (at most 4 x 4 x 4)
  if (lane == 0) f_n = 0;
  __syncthreads();
  {
    const double h = ldexp(py.h0, top);
    for (int64_t c = lane; c < py.m[top]; c += 64) {
      const int at = atomicAdd(&f_n, 1);
      f_key[at] = cell_mind2(py, py.ukeys[top][c], h, q0, q1, q2);
      f_cell[at] = static_cast<uint32_t>(c);
      f_lev[at] = static_cast<uint8_t>(top);
    }
  }
  __syncthreads();
  double lv = INFINITY;  // the wave's sorted k-best list, entry `lane`
  bool overflow = false;
  for (;;) {
    const int fn = f_n;
    if (fn == 0) break;
    // nearest frontier cell (lowest index on ties)
    double mk = INFINITY;
    int mi = 0x7fffffff;
    for (int e = lane; e < fn; e += 64)
      if (f_key[e] < mk) {
        mk = f_key[e];
        mi = e;
      }
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) {
      const double ok_ = __shfl_xor(mk, d, 64);
      const int oi = __shfl_xor(mi, d, 64);
      if (ok_ < mk || (ok_ == mk && oi < mi)) {
        mk = ok_;
        mi = oi;
      }
    }
    const double kth = __shfl(lv, kk - 1, 64);
    if (mk >= kth) break;  // no frontier cell can hold a point closer than the k-th
    const int64_t cell = f_cell[mi];
    const int l = f_lev[mi];
    __syncthreads();
    if (lane == 0) {  // remove mi: the last entry takes its place
      f_key[mi] = f_key[fn - 1];
      f_cell[mi] = f_cell[fn - 1];
      f_lev[mi] = f_lev[fn - 1];
      f_n = fn - 1;
    }
    __syncthreads();
    if (l <= py.l0) {
      // leaf: the cell's Morton-ordered points, 64 per batch
      const int64_t m = py.m[l];
      const int64_t a = py.ustart[l][cell], b = cell + 1 < m ? static_cast<int64_t>(py.ustart[l][cell + 1]) : n;
      for (int64_t t0 = a; t0 < b; t0 += 64) {
        const int64_t t = t0 + lane;
        double dd = INFINITY;
        if (t < b) {
          const double d0 = q0 - py.sxyz[3 * t], d1 = q1 - py.sxyz[3 * t + 1], d2 = q2 - py.sxyz[3 * t + 2];
          dd = ((d0 * d0) + d1 * d1) + d2 * d2;  // nanoflann L2_Adaptor order
        }
        double kcur = __shfl(lv, kk - 1, 64);
        uint64_t want = __ballot(t < b && dd < kcur);
        while (want) {
          const int src = __builtin_ctzll(want);
          want &= want - 1;
          const double v = __shfl(dd, src, 64);
          if (!(v < kcur)) continue;
          const double up = __shfl_up(lv, 1, 64);
          if (lane < kk && !(lv <= v)) lv = (lane == 0 || up <= v) ? v : up;
          kcur = __shfl(lv, kk - 1, 64);
        }
      }
    } else {
      // inner cell: push the children whose bound is below the k-th
      const uint32_t* fcl = py.fchild[l];
      const int64_t c0 = fcl[cell], c1 = fcl[cell + 1];
      const double h = ldexp(py.h0, l - 1);
      const double kcur = __shfl(lv, kk - 1, 64);
      bool push = false;
      double key2 = 0.0;
      if (lane < c1 - c0) {
        key2 = cell_mind2(py, py.ukeys[l - 1][c0 + lane], h, q0, q1, q2);
        push = key2 < kcur;
      }
      const uint64_t pm = __ballot(push);
      const int np = __popcll(pm);
      if (fn - 1 + np > kBestCap) {
        overflow = true;
        break;
      }
      if (push) {
        const int at = fn - 1 + __popcll(pm & ((1ull << lane) - 1ull));
        f_key[at] = key2;
        f_cell[at] = static_cast<uint32_t>(c0 + lane);
        f_lev[at] = static_cast<uint8_t>(l - 1);
      }
      __syncthreads();
      if (lane == 0) f_n = fn - 1 + np;
      __syncthreads();
    }
  }
  if (overflow) {
    if (lane == 0) over_q[atomicAdd(over_n, 1u)] = static_cast<uint32_t>(j);
    return;
  }
  // mean of the k square roots, ascending (the list order)
  double s = 0.0;
  for (int e = 0; e < kk; ++e) s += sqrt(__shfl(lv, e, 64));
  if (lane == 0) avg[qi] = kk > 0 ? s / static_cast<double>(kk) : -1.0;
}

__global__ __launch_bounds__(kT) void k_keep_flags(const double* avg, int64_t n, double thr, uint32_t* flag) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i < n) flag[i] = (avg[i] > 0.0 && avg[i] < thr) ? 1u : 0u;
}

__global__ __launch_bounds__(kT) void k_compact_index(const uint32_t* flag, const uint32_t* pos, int64_t n,
                                                      int64_t* out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i < n && flag[i]) out[pos[i]] = i;
}

__global__ __launch_bounds__(kT) void k_gather(const double* xyz, const uint8_t* bgr, const int64_t* idx, int64_t m,
                                               double* oxyz, uint8_t* obgr) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (j >= m) return;
  const int64_t i = idx[j];
#pragma unroll
  for (int k = 0; k < 3; ++k) oxyz[3 * j + k] = xyz[3 * i + k];
  if (bgr && obgr)
#pragma unroll
    for (int k = 0; k < 3; ++k) obgr[3 * j + k] = bgr[3 * i + k];
}

// p' = M p for a 4x4 row-major pose: row r = ((m_r0 x + m_r1 y) + m_r2 z) + m_r3
// (Eigen's (M * (x, y, z, 1)).head<3>() in PointCloud::Transform), in place.
__global__ __launch_bounds__(kT) void k_transform(double* xyz, int64_t n, const double* m) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i >= n) return;
  const double x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
#pragma unroll
  for (int r = 0; r < 3; ++r) xyz[3 * i + r] = ((m[4 * r] * x + m[4 * r + 1] * y) + m[4 * r + 2] * z) + m[4 * r + 3];
}

// -------------------------------------------------------------- normals ----
// PointCloud::EstimateNormals(KDTreeSearchParamHybrid(radius, max_nn)) --
// processing.py:178 on the merged cloud (radius 2 voxel, max_nn 30):
// neighbours = the points with ((dx^2 + dy^2) + dz^2) < radius^2 (itself
// included), ascending (distance, index), the first max_nn; fewer than 3 ->
// identity covariance, else cumulants in neighbour order / count ->
// E[ab] - E[a]E[b]; normal = FastEigen3x3 (Geometric Tools' robust symmetric
// 3x3 solver, Open3D utility/Eigen.cpp); a zero result -> (0, 0, 1).
// FastEigen3x3's acos / cos are the fdlibm algorithms (only IEEE basic ops,
// so the same bits as oracle/merge_oracle.py on any host; <= 1 ulp from the
// exact value on the ranges used).
namespace nrm {

constexpr double kPio2Hi = 1.57079632679489655800e+00, kPio2Lo = 6.12323399573676603587e-17;
constexpr double kPi = 3.14159265358979311600e+00;
constexpr double kInvPio2 = 6.36619772367581382433e-01, kPio2_1 = 1.57079632673412561417e+00,
                 kPio2_1t = 6.07710050650619224932e-11;

__device__ __forceinline__ double acos_rational(double z) {
  const double p = z * (1.66666666666666657415e-01 +
                        z * (-3.25565818622400915405e-01 +
                             z * (2.01212532134862925881e-01 +
                                  z * (-4.00555345006794114027e-02 +
                                       z * (7.91534994289814532176e-04 + z * 3.47933107596021167570e-05)))));
  const double q = 1.0 + z * (-2.40339491173441421878e+00 +
                              z * (2.02094576023350569471e+00 +
                                   z * (-6.88283971605453293030e-01 + z * 7.70381505559019352791e-02)));
  return p / q;
}

__device__ double acos_det(double x) {
  const double ax = fabs(x);
  if (ax >= 1.0) return x == 1.0 ? 0.0 : (x == -1.0 ? kPi : __builtin_nan(""));
  if (ax < 0.5) {
    if (ax <= 6.938893903907228e-18) return kPio2Hi + kPio2Lo;  // 2^-57
    const double r = acos_rational(x * x);
    return kPio2Hi - (x - (kPio2Lo - x * r));
  }
  if (x < 0.0) {
    const double z = (1.0 + x) * 0.5;
    const double s = sqrt(z);
    const double r = acos_rational(z);
    const double w = r * s - kPio2Lo;
    return kPi - 2.0 * (s + w);
  }
  const double z = (1.0 - x) * 0.5;
  const double s = sqrt(z);
  const double df = __longlong_as_double(__double_as_longlong(s) & static_cast<long long>(0xFFFFFFFF00000000ull));
  const double c = (z - df * df) / (s + df);
  const double r = acos_rational(z);
  const double w = r * s + c;
  return 2.0 * (df + w);
}

__device__ __forceinline__ double kcos(double x, double y) {
  const double z = x * x;
  double w = z * z;
  const double r = z * (4.16666666666666019037e-02 + z * (-1.38888888888741095749e-03 + z * 2.48015872894767294178e-05)) +
                   w * w * (-2.75573143513906633035e-07 + z * (2.08757232129817482790e-09 + z * -1.13596475577881948265e-11));
  const double hz = 0.5 * z;
  w = 1.0 - hz;
  return w + (((1.0 - w) - hz) + (z * r - x * y));
}

__device__ __forceinline__ double ksin(double x, double y) {
  const double z = x * x;
  const double w = z * z;
  const double r = 8.33333333332248946124e-03 + z * (-1.98412698298579493134e-04 + z * 2.75573137070700676789e-06) +
                   z * w * (-2.50507602534068634195e-08 + z * 1.58969099521155010221e-10);
  const double v = z * x;
  return x - ((z * (0.5 * y - v * r) - y) - v * -1.66666666666666324348e-01);
}

// x in [0, 4]
__device__ double cos_det(double x) {
  if (x <= 0.7853981633974483) return kcos(x, 0.0);
  const double fn = floor(x * kInvPio2 + 0.5);
  const int n = static_cast<int>(fn);
  const double r = x - fn * kPio2_1;
  const double w = fn * kPio2_1t;
  const double y0 = r - w;
  const double y1 = (r - y0) - w;
  switch (n & 3) {
    case 0: return kcos(y0, y1);
    case 1: return -ksin(y0, y1);
    case 2: return -kcos(y0, y1);
    default: return ksin(y0, y1);
  }
}

struct V3 {
  double x, y, z;
};

__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

// A: symmetric, entries a00 a01 a02 a11 a12 a22
struct S3 {
  double a00, a01, a02, a11, a12, a22;
};

__device__ V3 evec0(const S3& A, double e) {
  const V3 r0{A.a00 - e, A.a01, A.a02}, r1{A.a01, A.a11 - e, A.a12}, r2{A.a02, A.a12, A.a22 - e};
  const V3 c01 = cross(r0, r1), c02 = cross(r0, r2), c12 = cross(r1, r2);
  const double d0 = dot(c01, c01), d1 = dot(c02, c02), d2 = dot(c12, c12);
  double dmax = d0;
  int imax = 0;
  if (d1 > dmax) {
    dmax = d1;
    imax = 1;
  }
  if (d2 > dmax) imax = 2;
  const V3 v = imax == 0 ? c01 : (imax == 1 ? c02 : c12);
  const double sq = sqrt(imax == 0 ? d0 : (imax == 1 ? d1 : d2));
  return {v.x / sq, v.y / sq, v.z / sq};
}

__device__ V3 evec1(const S3& A, V3 e0, double e1) {
  V3 U;
  if (fabs(e0.x) > fabs(e0.y)) {
    const double inv = 1.0 / sqrt(e0.x * e0.x + e0.z * e0.z);
    U = {-e0.z * inv, 0.0, e0.x * inv};
  } else {
    const double inv = 1.0 / sqrt(e0.y * e0.y + e0.z * e0.z);
    U = {0.0, e0.z * inv, -e0.y * inv};
  }
  const V3 V = cross(e0, U);
  const V3 AU{A.a00 * U.x + A.a01 * U.y + A.a02 * U.z, A.a01 * U.x + A.a11 * U.y + A.a12 * U.z,
              A.a02 * U.x + A.a12 * U.y + A.a22 * U.z};
  const V3 AV{A.a00 * V.x + A.a01 * V.y + A.a02 * V.z, A.a01 * V.x + A.a11 * V.y + A.a12 * V.z,
              A.a02 * V.x + A.a12 * V.y + A.a22 * V.z};
  double m00 = U.x * AU.x + U.y * AU.y + U.z * AU.z - e1;
  double m01 = U.x * AV.x + U.y * AV.y + U.z * AV.z;
  double m11 = V.x * AV.x + V.y * AV.y + V.z * AV.z - e1;
  const double a00 = fabs(m00), a01 = fabs(m01), a11 = fabs(m11);
  if (a00 >= a11) {
    if (fmax(a00, a01) > 0.0) {
      if (a00 >= a01) {
        m01 /= m00;
        m00 = 1.0 / sqrt(1.0 + m01 * m01);
        m01 *= m00;
      } else {
        m00 /= m01;
        m01 = 1.0 / sqrt(1.0 + m00 * m00);
        m00 *= m01;
      }
      return {m01 * U.x - m00 * V.x, m01 * U.y - m00 * V.y, m01 * U.z - m00 * V.z};
    }
    return U;
  }
  if (fmax(a11, a01) > 0.0) {
    if (a11 >= a01) {
      m01 /= m11;
      m11 = 1.0 / sqrt(1.0 + m01 * m01);
      m01 *= m11;
    } else {
      m11 /= m01;
      m01 = 1.0 / sqrt(1.0 + m11 * m11);
      m11 *= m01;
    }
    return {m11 * U.x - m01 * V.x, m11 * U.y - m01 * V.y, m11 * U.z - m01 * V.z};
  }
  return U;
}

// FastEigen3x3: unit eigenvector of the smallest eigenvalue; 0 for C == 0.
// (max over the 9 entries as Eigen's maxCoeff sees them: the symmetric pairs
// are equal, so the 6 distinct ones.)
__device__ V3 fast_eigen3x3(const S3& C) {
  const double mx = fmax(fmax(fmax(C.a00, C.a01), fmax(C.a02, C.a11)), fmax(C.a12, C.a22));
  if (mx == 0.0) return {0.0, 0.0, 0.0};
  const S3 A{C.a00 / mx, C.a01 / mx, C.a02 / mx, C.a11 / mx, C.a12 / mx, C.a22 / mx};
  const double norm = A.a01 * A.a01 + A.a02 * A.a02 + A.a12 * A.a12;
  if (norm > 0.0) {
    const double q = (A.a00 + A.a11 + A.a22) / 3.0;
    const double b00 = A.a00 - q, b11 = A.a11 - q, b22 = A.a22 - q;
    const double p = sqrt((b00 * b00 + b11 * b11 + b22 * b22 + norm * 2.0) / 6.0);
    const double c00 = b11 * b22 - A.a12 * A.a12;
    const double c01 = A.a01 * b22 - A.a12 * A.a02;
    const double c02 = A.a01 * A.a12 - b11 * A.a02;
    const double det = (b00 * c00 - A.a01 * c01 + A.a02 * c02) / (p * p * p);
    const double half_det = fmin(fmax(det * 0.5, -1.0), 1.0);
    const double angle = acos_det(half_det) / 3.0;
    const double beta2 = cos_det(angle) * 2.0;
    const double beta0 = cos_det(angle + 2.09439510239319549) * 2.0;
    const double beta1 = -(beta0 + beta2);
    const double ev0 = q + p * beta0, ev1 = q + p * beta1, ev2 = q + p * beta2;
    if (half_det >= 0.0) {
      const V3 e2 = evec0(A, ev2);
      if (ev2 < ev0 && ev2 < ev1) return e2;
      const V3 e1 = evec1(A, e2, ev1);
      if (ev1 < ev0 && ev1 < ev2) return e1;
      return cross(e1, e2);
    }
    const V3 e0 = evec0(A, ev0);
    if (ev0 < ev1 && ev0 < ev2) return e0;
    const V3 e1 = evec1(A, e0, ev1);
    if (ev1 < ev0 && ev1 < ev2) return e1;
    return cross(e0, e1);
  }
  if (C.a00 < C.a11 && C.a00 < C.a22) return {1.0, 0.0, 0.0};
  if (C.a11 < C.a00 && C.a11 < C.a22) return {0.0, 1.0, 0.0};
  return {0.0, 0.0, 1.0};
}

}  // namespace nrm

constexpr int kNrmK = 32;  // largest max_nn

// The 27 neighbour cells (-1: empty or outside) of every occupied cell of a
// linear-key grid (key = (ix * ny + iy) * nz + iz), (dx, dy, dz) nesting order.
__global__ __launch_bounds__(kT) void k_cell_neighbours_lin(const uint64_t* ukeys, int64_t m, int64_t nx, int64_t ny,
                                                            int64_t nz, int32_t* nbr) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (c >= m) return;
  const int64_t key = static_cast<int64_t>(ukeys[c]);
  const int64_t x = key / (ny * nz), y = (key / nz) % ny, z = key % nz;
  int e = 0;
  for (int dx = -1; dx <= 1; ++dx)
    for (int dy = -1; dy <= 1; ++dy)
      for (int dz = -1; dz <= 1; ++dz, ++e) {
        const int64_t a = x + dx, b = y + dy, d = z + dz;
        int64_t f = -1;
        if (a >= 0 && a < nx && b >= 0 && b < ny && d >= 0 && d < nz)
          f = find_cell(ukeys, m, static_cast<uint64_t>((a * ny + b) * nz + d));
        nbr[27 * c + e] = static_cast<int32_t>(f);
      }
}

// One query per thread, in cell-sorted order (neighbouring threads share
// cells).  Candidates from the 27 cells of edge >= radius around the query's
// cell; the max_nn best by (d2, index) in a sorted register list.
__global__ __launch_bounds__(kT) void k_normals(const double* xyz, const double* sxyz, const uint32_t* sidx,
                                                const uint64_t* skeys, int64_t n, const uint64_t* ukeys,
                                                const uint32_t* ustart, int64_t m, const int32_t* nbr, double r2,
                                                int max_nn, double* out) {
  const int64_t j = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (j >= n) return;
  const double q0 = sxyz[3 * j], q1 = sxyz[3 * j + 1], q2 = sxyz[3 * j + 2];
  const int64_t cell = find_cell(ukeys, m, skeys[j]);
  double bd[kNrmK];
  uint32_t bi[kNrmK];
#pragma unroll
  for (int e = 0; e < kNrmK; ++e) {
    bd[e] = INFINITY;
    bi[e] = 0xffffffffu;
  }
  int found = 0;
  for (int e = 0; e < 27; ++e) {
    const int32_t cc = nbr[27 * cell + e];
    if (cc < 0) continue;
    const int64_t t1 = cc + 1 < m ? static_cast<int64_t>(ustart[cc + 1]) : n;
    for (int64_t t = ustart[cc]; t < t1; ++t) {
      const double d0 = q0 - sxyz[3 * t], d1 = q1 - sxyz[3 * t + 1], d2 = q2 - sxyz[3 * t + 2];
      const double dd = (d0 * d0 + d1 * d1) + d2 * d2;
      if (!(dd < r2)) continue;
      ++found;
      const uint32_t id = sidx[t];
      if (dd < bd[kNrmK - 1] || (dd == bd[kNrmK - 1] && id < bi[kNrmK - 1])) {
        double v = dd;
        uint32_t vi = id;
#pragma unroll
        for (int k = 0; k < kNrmK; ++k) {
          const bool lt = v < bd[k] || (v == bd[k] && vi < bi[k]);
          const double od = bd[k];
          const uint32_t oi = bi[k];
          bd[k] = lt ? v : od;
          bi[k] = lt ? vi : oi;
          v = lt ? od : v;
          vi = lt ? oi : vi;
        }
      }
    }
  }
  const int cnt = found < max_nn ? found : max_nn;
  nrm::S3 C{1.0, 0.0, 0.0, 1.0, 0.0, 1.0};
  if (cnt >= 3) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0, s4 = 0.0, s5 = 0.0, s6 = 0.0, s7 = 0.0, s8 = 0.0;
#pragma unroll
    for (int k = 0; k < kNrmK; ++k) {
      if (k < cnt) {
        const int64_t i = bi[k];
        const double x = xyz[3 * i], y = xyz[3 * i + 1], z = xyz[3 * i + 2];
        s0 += x;
        s1 += y;
        s2 += z;
        s3 += x * x;
        s4 += x * y;
        s5 += x * z;
        s6 += y * y;
        s7 += y * z;
        s8 += z * z;
      }
    }
    const double k = static_cast<double>(cnt);
    s0 /= k;
    s1 /= k;
    s2 /= k;
    s3 /= k;
    s4 /= k;
    s5 /= k;
    s6 /= k;
    s7 /= k;
    s8 /= k;
    C = {s3 - s0 * s0, s4 - s0 * s1, s5 - s0 * s2, s6 - s1 * s1, s7 - s1 * s2, s8 - s2 * s2};
  }
  nrm::V3 v = nrm::fast_eigen3x3(C);
  if (sqrt(v.x * v.x + v.y * v.y + v.z * v.z) == 0.0) v = {0.0, 0.0, 1.0};
  const int64_t i = sidx[j];
  out[3 * i] = v.x;
  out[3 * i + 1] = v.y;
  out[3 * i + 2] = v.z;
}

__global__ __launch_bounds__(kT) void k_fill_up(double* out, int64_t n) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i >= n) return;
  out[3 * i] = 0.0;
  out[3 * i + 1] = 0.0;
  out[3 * i + 2] = 1.0;
}

// ------------------------------------------------------------------- ICP ----
// registration_icp(source_down, target_down, voxel_size, init,
// TransformationEstimationPointToPlane()) of merge_pro_360
// (processing.py:154-156), Open3D's loop (Registration.cpp RegistrationICP):
// correspondences = each (moved) source point's nearest target point within
// max_distance; the point-to-plane Gauss-Newton step from them; repeated
// until fitness and inlier RMSE both change by less than their relative
// criteria (or max_iteration).  Open3D is not in this image: parity is
// unpinned; oracle/merge_oracle.py restates this exact arithmetic.
constexpr int kIcpBlock = 64;  // source points per fold thread
constexpr int kIcpSums = 29;   // JTJ upper triangle (21), JTr (6), sum of d^2, correspondences

// dense cell table: dense[key] = occupied-cell index (pre-filled with -1)
__global__ __launch_bounds__(kT) void k_icp_dense(const uint64_t* ukeys, int64_t m, int32_t* dense) {
  const int64_t c = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (c < m) dense[ukeys[c]] = static_cast<int32_t>(c);
}

// Nearest target point of every source point q within max_distance:
// ((dx^2 + dy^2) + dz^2) < r2 (nanoflann's strict radius test), the least
// (d2, target index); candidates from the 27 cells (edge >= max_distance)
// around q's cell.  -> corr[i] (target index or -1), dist2[i].
__global__ __launch_bounds__(kT) void k_icp_corr(const double* cur, int64_t n, Grid g, const int32_t* dense,
                                                 const uint64_t* ukeys, int64_t m, const uint32_t* ustart,
                                                 int64_t nt, const double* sxyz, const uint32_t* sidx, double r2,
                                                 int32_t* corr, double* dist2) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i >= n) return;
  const double q0 = cur[3 * i], q1 = cur[3 * i + 1], q2 = cur[3 * i + 2];
  double bd = INFINITY;
  int64_t bi = -1;
  const double f0 = floor((q0 - g.lo0) / g.h), f1 = floor((q1 - g.lo1) / g.h), f2 = floor((q2 - g.lo2) / g.h);
  // a query more than a cell outside the grid (or not finite) has no candidate cell
  if (f0 >= -1.0 && f0 <= static_cast<double>(g.nx) && f1 >= -1.0 && f1 <= static_cast<double>(g.ny) &&
      f2 >= -1.0 && f2 <= static_cast<double>(g.nz)) {
    const int64_t ix = static_cast<int64_t>(f0), iy = static_cast<int64_t>(f1), iz = static_cast<int64_t>(f2);
    for (int dx = -1; dx <= 1; ++dx)
      for (int dy = -1; dy <= 1; ++dy)
        for (int dz = -1; dz <= 1; ++dz) {
          const int64_t a = ix + dx, b = iy + dy, d = iz + dz;
          if (a < 0 || a >= g.nx || b < 0 || b >= g.ny || d < 0 || d >= g.nz) continue;
          const uint64_t key = static_cast<uint64_t>((a * g.ny + b) * g.nz + d);
          const int64_t cc = dense ? static_cast<int64_t>(dense[key]) : find_cell(ukeys, m, key);
          if (cc < 0) continue;
          const int64_t t1 = cc + 1 < m ? static_cast<int64_t>(ustart[cc + 1]) : nt;
          for (int64_t t = ustart[cc]; t < t1; ++t) {
            const double d0 = q0 - sxyz[3 * t], d1 = q1 - sxyz[3 * t + 1], d2 = q2 - sxyz[3 * t + 2];
            const double dd = (d0 * d0 + d1 * d1) + d2 * d2;
            if (!(dd < r2)) continue;
            const int64_t id = sidx[t];
            if (dd < bd || (dd == bd && id < bi)) {
              bd = dd;
              bi = id;
            }
          }
        }
  }
  corr[i] = static_cast<int32_t>(bi);
  dist2[i] = bi >= 0 ? bd : 0.0;
}

// One thread per kIcpBlock source points, in index order: the point-to-plane
// residual r = (vs - vt) . nt and Jacobian J = (vs x nt, nt) of every
// correspondence, folded left to right into JTJ (upper triangle, row-major),
// JTr, the sum of d^2 and the count -> part[b][29].  (TransformationEstimation-
// PointToPlane::ComputeTransformation with the L2 loss: weight 1.)
__global__ __launch_bounds__(kT) void k_icp_fold(const double* cur, int64_t n, const double* tgt, const double* tn,
                                                 const int32_t* corr, const double* dist2, double* part) {
  const int64_t b = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  const int64_t i0 = b * kIcpBlock;
  if (i0 >= n) return;
  const int64_t i1 = i0 + kIcpBlock < n ? i0 + kIcpBlock : n;
  double acc[kIcpSums];
#pragma unroll
  for (int k = 0; k < kIcpSums; ++k) acc[k] = 0.0;
  for (int64_t i = i0; i < i1; ++i) {
    const int64_t j = corr[i];
    if (j < 0) continue;
    const double s0 = cur[3 * i], s1 = cur[3 * i + 1], s2 = cur[3 * i + 2];
    const double n0 = tn[3 * j], n1 = tn[3 * j + 1], n2 = tn[3 * j + 2];
    const double e0 = s0 - tgt[3 * j], e1 = s1 - tgt[3 * j + 1], e2 = s2 - tgt[3 * j + 2];
    const double r = (e0 * n0 + e1 * n1) + e2 * n2;
    const double J[6] = {s1 * n2 - s2 * n1, s2 * n0 - s0 * n2, s0 * n1 - s1 * n0, n0, n1, n2};
    int k = 0;
#pragma unroll
    for (int a = 0; a < 6; ++a)
#pragma unroll
      for (int c = a; c < 6; ++c) acc[k++] += J[a] * J[c];
#pragma unroll
    for (int a = 0; a < 6; ++a) acc[21 + a] += J[a] * r;
    acc[27] += dist2[i];
    acc[28] += 1.0;
  }
#pragma unroll
  for (int k = 0; k < kIcpSums; ++k) part[kIcpSums * b + k] = acc[k];
}

// ------------------------------------------------------------------ host ----
unsigned blocks(int64_t n) { return static_cast<unsigned>((n + kT - 1) / kT); }

struct PinBuf {
  double* p = nullptr;
  ~PinBuf() {
    if (p) (void)hipHostFree(p);
  }
};

// Scratch pool: the merge entry points allocate several buffers of the
// cloud's size per call, and hipFree costs ~44 us each (it waits for the
// device); freed buffers are kept per device (up to kPoolMax bytes per device)
// and a request takes the smallest kept buffer of that device of at least its
// size and at most twice it.  A buffer goes back to the pool only once the
// stream it was used on is idle: DBuf remembers the stream of its entry point
// (PoolStream) and synchronises it when the scope ends, on the error returns
// too, so a reused buffer is never still in use by a queued kernel (on the
// normal path the stream is already synchronised and the extra wait is free).
// sl_merge_pool_trim releases a device's kept buffers.
constexpr size_t kPoolMax = size_t{16} << 30;  // per device

struct Pool {
  std::mutex mu;
  std::multimap<size_t, std::pair<int, void*>> free;  // bytes -> (device, ptr)
  std::map<int, size_t> cached;                       // device -> kept bytes
};

Pool& pool() {
  static Pool* p = new Pool();  // never destroyed: device memory is released with the process
  return *p;
}

thread_local hipStream_t tls_stream = nullptr;  // the running entry point's stream

struct PoolStream {  // RAII: the stream the entry point's scratch is used on
  hipStream_t prev;
  explicit PoolStream(hipStream_t s) : prev(tls_stream) { tls_stream = s; }
  ~PoolStream() { tls_stream = prev; }
};

hipError_t pool_alloc(void** out, size_t bytes) {
  int dev = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e != hipSuccess) return e;
  {
    Pool& P = pool();
    std::lock_guard<std::mutex> lk(P.mu);
    for (auto it = P.free.lower_bound(bytes); it != P.free.end() && it->first <= 2 * bytes; ++it) {
      if (it->second.first != dev) continue;
      *out = it->second.second;
      P.cached[dev] -= it->first;
      P.free.erase(it);
      return hipSuccess;
    }
  }
  return hipMalloc(out, bytes);
}

// ptr must be idle (its stream synchronised)
void pool_free(void* ptr, size_t bytes) {
  int dev = 0;
  if (hipGetDevice(&dev) == hipSuccess) {
    Pool& P = pool();
    std::lock_guard<std::mutex> lk(P.mu);
    if (P.cached[dev] + bytes <= kPoolMax) {
      P.free.emplace(bytes, std::make_pair(dev, ptr));
      P.cached[dev] += bytes;
      return;
    }
  }
  (void)hipFree(ptr);
}

size_t pool_trim(int dev) {
  std::vector<void*> drop;
  size_t bytes = 0;
  {
    Pool& P = pool();
    std::lock_guard<std::mutex> lk(P.mu);
    for (auto it = P.free.begin(); it != P.free.end();) {
      if (it->second.first == dev) {
        drop.push_back(it->second.second);
        bytes += it->first;
        it = P.free.erase(it);
      } else {
        ++it;
      }
    }
    P.cached[dev] = 0;
  }
  for (void* p : drop) (void)hipFree(p);
  return bytes;
}

template <typename T>
struct DBuf {
  T* p = nullptr;
  size_t bytes = 0;
  hipStream_t s = nullptr;
  ~DBuf() {
    if (!p) return;
    (void)hipStreamSynchronize(s);  // idle before reuse (an early error return may leave work queued)
    pool_free(p, bytes);
  }
  hipError_t alloc(int64_t n) {
    bytes = sizeof(T) * static_cast<size_t>(std::max<int64_t>(n, 1));
    s = tls_stream;
    return pool_alloc(reinterpret_cast<void**>(&p), bytes);
  }
};

// min / max bound of n points (device) -> host b[6]
int bounds(sl_ctx* c, const double* xyz, int64_t n, double* b, hipStream_t s) {
  const int nb = static_cast<int>(std::min<int64_t>(1024, (n + kT - 1) / kT));
  DBuf<double> part;
  MTRY(c, part.alloc(6 * nb));
  hipLaunchKernelGGL(k_bounds, dim3(nb), dim3(kT), 0, s, xyz, n, part.p);
  MTRY(c, hipGetLastError());
  std::vector<double> h(6 * static_cast<size_t>(nb));
  MTRY(c, hipMemcpyAsync(h.data(), part.p, sizeof(double) * h.size(), hipMemcpyDeviceToHost, s));
  MTRY(c, hipStreamSynchronize(s));
  for (int k = 0; k < 3; ++k) {
    b[k] = INFINITY;
    b[3 + k] = -INFINITY;
  }
  for (int i = 0; i < nb; ++i)
    for (int k = 0; k < 3; ++k) {
      b[k] = std::min(b[k], h[6 * i + k]);
      b[3 + k] = std::max(b[3 + k], h[6 * i + 3 + k]);
    }
  return SL_OK;
}

// Stable sort of (keys, vals) in place (device), over the low `bits` bits.
int radix_sort(sl_ctx* c, uint64_t* keys, uint32_t* vals, int64_t n, int bits, hipStream_t s) {
  const int tiles = static_cast<int>((n + kRsTile - 1) / kRsTile);
  DBuf<uint64_t> k2;
  DBuf<uint32_t> v2, cnt;
  MTRY(c, k2.alloc(n));
  MTRY(c, v2.alloc(n));
  MTRY(c, cnt.alloc(static_cast<int64_t>(kRsBins) * tiles));
  // exclusive scan of the digit-major counts: tile sums, one workgroup over
  // them, local scans (in place)
  const int64_t n_cnt = static_cast<int64_t>(kRsBins) * tiles;
  const int ctiles = static_cast<int>((n_cnt + kRsTile - 1) / kRsTile);
  DBuf<uint32_t> csum;
  MTRY(c, csum.alloc(ctiles));
  uint64_t *ka = keys, *kb = k2.p;
  uint32_t *va = vals, *vb = v2.p;
  int passes = 0;
  for (int shift = 0; shift < bits; shift += kRsBits, ++passes) {
    hipLaunchKernelGGL(k_rs_count, dim3(tiles), dim3(kT), 0, s, ka, n, shift, cnt.p, tiles);
    hipLaunchKernelGGL(k_tile_sums, dim3(ctiles), dim3(kT), 0, s, cnt.p, n_cnt, csum.p);
    hipLaunchKernelGGL(k_scan1, dim3(1), dim3(kT), 0, s, csum.p, static_cast<int64_t>(ctiles),
                       static_cast<uint32_t*>(nullptr));
    hipLaunchKernelGGL(k_tile_scan, dim3(ctiles), dim3(kT), 0, s, cnt.p, n_cnt, csum.p, cnt.p);
    hipLaunchKernelGGL(k_rs_scatter, dim3(tiles), dim3(kT), 0, s, ka, va, kb, vb, n, shift, cnt.p, tiles);
    MTRY(c, hipGetLastError());
    std::swap(ka, kb);
    std::swap(va, vb);
  }
  if (passes & 1) {  // result is in the scratch pair
    MTRY(c, hipMemcpyAsync(keys, ka, sizeof(uint64_t) * n, hipMemcpyDeviceToDevice, s));
    MTRY(c, hipMemcpyAsync(vals, va, sizeof(uint32_t) * n, hipMemcpyDeviceToDevice, s));
  }
  MTRY(c, hipStreamSynchronize(s));  // scratch is freed on return
  return SL_OK;
}

// Exclusive scan of flag[0..n) -> pos; returns the total on the host.
int scan_flags(sl_ctx* c, const uint32_t* flag, int64_t n, uint32_t* pos, int64_t* total, hipStream_t s) {
  const int tiles = static_cast<int>((n + kRsTile - 1) / kRsTile);
  DBuf<uint32_t> sums, tot;
  MTRY(c, sums.alloc(tiles));
  MTRY(c, tot.alloc(1));
  hipLaunchKernelGGL(k_tile_sums, dim3(tiles), dim3(kT), 0, s, flag, n, sums.p);
  hipLaunchKernelGGL(k_scan1, dim3(1), dim3(kT), 0, s, sums.p, static_cast<int64_t>(tiles), tot.p);
  hipLaunchKernelGGL(k_tile_scan, dim3(tiles), dim3(kT), 0, s, flag, n, sums.p, pos);
  MTRY(c, hipGetLastError());
  uint32_t t = 0;
  MTRY(c, hipMemcpyAsync(&t, tot.p, sizeof(t), hipMemcpyDeviceToHost, s));
  MTRY(c, hipStreamSynchronize(s));
  *total = t;
  return SL_OK;
}

int key_bits(uint64_t max_key) {
  int b = 0;
  while (b < 64 && (max_key >> b) != 0) ++b;
  return std::max(b, 1);
}

// Grid over [lo, hi] with cell h: dims, checked so that linear keys fit 63 bits.
bool make_grid(const double* lo, const double* hi, double h, Grid* g) {
  int64_t d[3];
  for (int k = 0; k < 3; ++k) {
    const double e = floor((hi[k] - lo[k]) / h);
    if (!(e >= 0.0) || e > 2.0e6) return false;
    d[k] = static_cast<int64_t>(e) + 1;
  }
  if (static_cast<double>(d[0]) * static_cast<double>(d[1]) * static_cast<double>(d[2]) > 9.0e18) return false;
  g->lo0 = lo[0];
  g->lo1 = lo[1];
  g->lo2 = lo[2];
  g->h = h;
  g->nx = d[0];
  g->ny = d[1];
  g->nz = d[2];
  return true;
}

// Sort the points into grid cells: sorted keys + point indices, and the
// unique cells with their first position.  Returns the cell count in *m.
int cells(sl_ctx* c, const double* xyz, int64_t n, const Grid& g, DBuf<uint64_t>& keys, DBuf<uint32_t>& idx,
          DBuf<uint64_t>& ukeys, DBuf<uint32_t>& ustart, int64_t* m, hipStream_t s) {
  MTRY(c, keys.alloc(n));
  MTRY(c, idx.alloc(n));
  hipLaunchKernelGGL(k_cell_keys, dim3(blocks(n)), dim3(kT), 0, s, xyz, n, g.lo0, g.lo1, g.lo2, g.h, g.ny, g.nz,
                     keys.p, idx.p);
  MTRY(c, hipGetLastError());
  const uint64_t max_key = static_cast<uint64_t>((g.nx * g.ny) * g.nz - 1);
  int r = radix_sort(c, keys.p, idx.p, n, key_bits(max_key), s);
  if (r) return r;
  DBuf<uint32_t> flag, seg;
  MTRY(c, flag.alloc(n));
  MTRY(c, seg.alloc(n));
  hipLaunchKernelGGL(k_heads, dim3(blocks(n)), dim3(kT), 0, s, keys.p, n, flag.p);
  r = scan_flags(c, flag.p, n, seg.p, m, s);
  if (r) return r;
  MTRY(c, ustart.alloc(*m));
  MTRY(c, ukeys.alloc(*m));
  hipLaunchKernelGGL(k_seg_starts, dim3(blocks(n)), dim3(kT), 0, s, flag.p, seg.p, keys.p, n, ustart.p, ukeys.p);
  MTRY(c, hipGetLastError());
  MTRY(c, hipStreamSynchronize(s));
  return SL_OK;
}

}  // namespace

extern "C" {

int sl_voxel_downsample(sl_ctx* c, const double* xyz, const uint8_t* bgr, int64_t n, double voxel_size,
                        double* out_xyz, uint8_t* out_bgr, int64_t* out_n, void* stream) {
  if (!c || !out_n || n < 0 || (n && (!xyz || !out_xyz))) return SL_EINVAL;
  if (!(voxel_size > 0.0)) return slgpu_fail(c, SL_EINVAL, "voxel_size <= 0.");
  if (n >= (1ll << 31)) return slgpu_fail(c, SL_EINVAL, "at most 2^31 - 1 points");
  *out_n = 0;
  if (n == 0) return SL_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  PoolStream pool_stream(s);
  MTRY(c, hipSetDevice(slgpu_device(c)));
  double b[6];
  int r = bounds(c, xyz, n, b, s);
  if (r) return r;
  // voxel_min_bound = min - vs/2, voxel_max_bound = max + vs/2 (VoxelDownSample)
  double lo[3], hi[3];
  for (int k = 0; k < 3; ++k) {
    lo[k] = b[k] - voxel_size * 0.5;
    hi[k] = b[3 + k] + voxel_size * 0.5;
  }
  double ext = 0.0;
  for (int k = 0; k < 3; ++k) ext = std::max(ext, hi[k] - lo[k]);
  if (voxel_size * std::numeric_limits<int>::max() < ext) return slgpu_fail(c, SL_EINVAL, "voxel_size is too small.");
  Grid g;
  if (!make_grid(lo, b + 3, voxel_size, &g))
    return slgpu_fail(c, SL_EINVAL, "voxel grid exceeds 2e6 voxels per axis / 2^63 voxels");
  DBuf<uint64_t> keys, ukeys;
  DBuf<uint32_t> idx, ustart;
  int64_t m = 0;
  r = cells(c, xyz, n, g, keys, idx, ukeys, ustart, &m, s);
  if (r) return r;
  hipLaunchKernelGGL(k_voxel_avg, dim3(blocks(m)), dim3(kT), 0, s, ustart.p, m, n, idx.p, xyz, bgr, out_xyz,
                     out_bgr);
  MTRY(c, hipGetLastError());
  MTRY(c, hipStreamSynchronize(s));
  *out_n = m;
  return SL_OK;
}

int sl_statistical_outliers(sl_ctx* c, const double* xyz, int64_t n, int nb_neighbors, double std_ratio,
                            double* avg_dist, int64_t* out_index, int64_t* out_n, void* stream) {
  if (!c || !out_n || n < 0 || (n && (!xyz || !avg_dist || !out_index))) return SL_EINVAL;
  if (nb_neighbors < 1 || !(std_ratio > 0.0))
    return slgpu_fail(c, SL_EINVAL, "Illegal input parameters, number of neighbors and standard deviation ratio "
                                    "must be positive");
  if (nb_neighbors > kMaxK) return slgpu_fail(c, SL_EINVAL, "nb_neighbors > 32 is not supported");
  if (n >= (1ll << 31)) return slgpu_fail(c, SL_EINVAL, "at most 2^31 - 1 points");
  *out_n = 0;
  if (n == 0) return SL_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  PoolStream pool_stream(s);
  MTRY(c, hipSetDevice(slgpu_device(c)));
  double b[6];
  int r = bounds(c, xyz, n, b, s);
  if (r) return r;
  // finest cell: 1/8 of the volume-filling size for ~k points per cell, at
  // most 2^20 cells per axis; the pyramid doubles it per level
  double ext[3], vol = 1.0, emax = 0.0;
  for (int k = 0; k < 3; ++k) {
    ext[k] = b[3 + k] - b[k];
    emax = std::max(emax, ext[k]);
  }
  for (int k = 0; k < 3; ++k) vol *= std::max(ext[k], emax * 1e-3);
  double h0 = cbrt(vol * nb_neighbors / static_cast<double>(n)) / 8.0;
  h0 = std::max(h0, emax / 1048575.0);
  if (!(h0 > 0.0) || !std::isfinite(h0)) h0 = 1.0;  // all points coincide (or non-finite input)
  Pyramid py;
  memset(&py, 0, sizeof(py));
  py.lo0 = b[0];
  py.lo1 = b[1];
  py.lo2 = b[2];
  py.h0 = h0;
  int64_t d0[3];
  for (int k = 0; k < 3; ++k) {
    const double e = floor(ext[k] / h0);
    if (!(e >= 0.0) || e >= 2097151.0) return slgpu_fail(c, SL_EINVAL, "non-finite or degenerate point cloud");
    d0[k] = static_cast<int64_t>(e) + 1;
  }
  DBuf<uint64_t> keys;
  DBuf<uint32_t> idx, flag, seg;
  MTRY(c, keys.alloc(n));
  MTRY(c, idx.alloc(n));
  MTRY(c, flag.alloc(n));
  MTRY(c, seg.alloc(n));
  hipLaunchKernelGGL(k_morton_keys, dim3(blocks(n)), dim3(kT), 0, s, xyz, n, py.lo0, py.lo1, py.lo2, h0, keys.p,
                     idx.p);
  MTRY(c, hipGetLastError());
  int bits_axis = 1;
  while ((int64_t{1} << bits_axis) < std::max(d0[0], std::max(d0[1], d0[2]))) ++bits_axis;
  r = radix_sort(c, keys.p, idx.p, n, 3 * bits_axis, s);
  if (r) return r;
  std::vector<DBuf<uint64_t>> lk(kMaxLevels);
  std::vector<DBuf<uint32_t>> ls(kMaxLevels);
  DBuf<uint32_t> cell0;
  DBuf<int32_t> nbr0;
  DBuf<double> sxyz;
  int levels = 0, l0 = -1;
  for (int l = 0; l < kMaxLevels; ++l) {
    int64_t ml = 0;
    hipLaunchKernelGGL(k_heads_shift, dim3(blocks(n)), dim3(kT), 0, s, keys.p, n, 3 * l, flag.p);
    r = scan_flags(c, flag.p, n, seg.p, &ml, s);
    if (r) return r;
    MTRY(c, lk[l].alloc(ml));
    MTRY(c, ls[l].alloc(ml));
    hipLaunchKernelGGL(k_level_cells, dim3(blocks(n)), dim3(kT), 0, s, flag.p, seg.p, keys.p, n, 3 * l, ls[l].p,
                       lk[l].p);
    MTRY(c, hipGetLastError());
    py.ukeys[l] = lk[l].p;
    py.ustart[l] = ls[l].p;
    py.m[l] = ml;
    int64_t dmax = 0;
    for (int k = 0; k < 3; ++k) {
      py.dim[l][k] = ((d0[k] - 1) >> l) + 1;
      dmax = std::max(dmax, py.dim[l][k]);
    }
    levels = l + 1;
    // start level: ~k/2 points per occupied cell (or the top)
    const bool top = dmax <= 4;
    if (l0 < 0 && (top || 2.0 * static_cast<double>(n) >= static_cast<double>(nb_neighbors) * static_cast<double>(ml))) {
      l0 = l;
      MTRY(c, cell0.alloc(n));
      hipLaunchKernelGGL(k_cell_of, dim3(blocks(n)), dim3(kT), 0, s, flag.p, seg.p, n, cell0.p);
      MTRY(c, nbr0.alloc(27 * ml));
      hipLaunchKernelGGL(k_cell_neighbours, dim3(blocks(ml)), dim3(kT), 0, s, lk[l].p, ml, py.dim[l][0],
                         py.dim[l][1], py.dim[l][2], nbr0.p);
      MTRY(c, hipGetLastError());
    }
    if (top) break;  // a few cells per axis
  }
  py.levels = levels;
  py.l0 = l0;
  // first-child tables of the levels above l0 (best-first search of isolated queries)
  std::vector<DBuf<uint32_t>> lfc(kMaxLevels);
  for (int l = l0 + 1; l < levels; ++l) {
    MTRY(c, lfc[l].alloc(py.m[l] + 1));
    hipLaunchKernelGGL(k_first_child, dim3(blocks(py.m[l] + 1)), dim3(kT), 0, s, lk[l].p, py.m[l], lk[l - 1].p,
                       py.m[l - 1], lfc[l].p);
    MTRY(c, hipGetLastError());
    py.fchild[l] = lfc[l].p;
  }
  MTRY(c, sxyz.alloc(3 * n));
  hipLaunchKernelGGL(k_gather_sorted, dim3(blocks(n)), dim3(kT), 0, s, xyz, idx.p, n, sxyz.p);
  MTRY(c, hipGetLastError());
  py.sxyz = sxyz.p;
  py.cell0 = cell0.p;
  py.nbr0 = nbr0.p;
  MTRY(c, hipStreamSynchronize(s));
  DBuf<unsigned> st;
  const bool want_stats = getenv("SLGPU_MERGE_STATS") != nullptr;
  if (want_stats) {
    MTRY(c, st.alloc(2 * kMaxLevels));
    MTRY(c, hipMemsetAsync(st.p, 0, sizeof(unsigned) * 2 * kMaxLevels, s));
    py.stats = st.p;
  }
  DBuf<uint32_t> slow_q;
  DBuf<unsigned> slow_n;
  MTRY(c, slow_q.alloc(n));
  MTRY(c, slow_n.alloc(1));
  MTRY(c, hipMemsetAsync(slow_n.p, 0, sizeof(unsigned), s));
  py.slow_q = slow_q.p;
  py.slow_n = slow_n.p;
  if (nb_neighbors == 20)
    hipLaunchKernelGGL(k_knn_mean<20>, dim3(blocks(n)), dim3(kT), 0, s, xyz, n, idx.p, py, nb_neighbors, avg_dist);
  else
    hipLaunchKernelGGL(k_knn_mean<kMaxK>, dim3(blocks(n)), dim3(kT), 0, s, xyz, n, idx.p, py, nb_neighbors,
                       avg_dist);
  MTRY(c, hipGetLastError());
  unsigned n_slow = 0;
  MTRY(c, hipMemcpyAsync(&n_slow, slow_n.p, sizeof(unsigned), hipMemcpyDeviceToHost, s));
  MTRY(c, hipStreamSynchronize(s));
  DBuf<uint32_t> over_q;  // (function scope: freed after the final synchronisation)
  DBuf<unsigned> over_n;
  if (n_slow) {
    // best-first search; the rare frontier overflow climbs the pyramid (k_knn_slow)
    const bool climb_only = getenv("SLGPU_MERGE_CLIMB") != nullptr;  // measurement only: the old path
    unsigned n_over = n_slow;
    if (!climb_only) {
      MTRY(c, over_q.alloc(n_slow));
      MTRY(c, over_n.alloc(1));
      MTRY(c, hipMemsetAsync(over_n.p, 0, sizeof(unsigned), s));
      if (nb_neighbors == 20)
        hipLaunchKernelGGL(k_knn_best<20>, dim3(n_slow), dim3(64), 0, s, idx.p, n, py, nb_neighbors, avg_dist,
                           over_q.p, over_n.p);
      else
        hipLaunchKernelGGL(k_knn_best<kMaxK>, dim3(n_slow), dim3(64), 0, s, idx.p, n, py, nb_neighbors, avg_dist,
                           over_q.p, over_n.p);
      MTRY(c, hipGetLastError());
      MTRY(c, hipMemcpyAsync(&n_over, over_n.p, sizeof(unsigned), hipMemcpyDeviceToHost, s));
      MTRY(c, hipStreamSynchronize(s));
    }
    if (n_over) {
      Pyramid pq = py;
      if (!climb_only) pq.slow_q = over_q.p;
      if (nb_neighbors == 20)
        hipLaunchKernelGGL(k_knn_slow<20>, dim3(n_over), dim3(64), 0, s, idx.p, n, pq, nb_neighbors, avg_dist);
      else
        hipLaunchKernelGGL(k_knn_slow<kMaxK>, dim3(n_over), dim3(64), 0, s, idx.p, n, pq, nb_neighbors, avg_dist);
      MTRY(c, hipGetLastError());
    }
    if (getenv("SLGPU_MERGE_STATS")) fprintf(stderr, "[slmerge] slow=%u overflow=%u\n", n_slow, climb_only ? 0u : n_over);
  }
  if (want_stats) {
    unsigned h[2 * kMaxLevels];
    MTRY(c, hipMemcpyAsync(h, st.p, sizeof(h), hipMemcpyDeviceToHost, s));
    MTRY(c, hipStreamSynchronize(s));
    fprintf(stderr, "[slmerge] n=%lld h0=%g l0=%d levels=%d m(l0)=%lld fast-done=%u slow-done:", (long long)n, h0,
            py.l0, py.levels, (long long)py.m[py.l0], h[py.l0]);
    for (int l = 0; l < py.levels; ++l) fprintf(stderr, " %u", h[kMaxLevels + l]);
    fprintf(stderr, "\n");
  }
  // cloud mean / std of the positive means: sequential, as std::accumulate /
  // std::inner_product in RemoveStatisticalOutliers.  The means stream to the
  // host through two pinned 1 MB buffers, the copy of one chunk overlapping
  // the (latency-bound) accumulation of the other; the conditional terms are
  // selects, m + (v > 0 ? v : +0.0) -- bit-identical to skipping, m >= +0.
  int64_t valid = 0;
  double mean = 0.0, sq = 0.0;
  {
    constexpr int64_t kCh = int64_t{1} << 17;  // doubles per chunk
    PinBuf pin;
    MTRY(c, hipHostMalloc(reinterpret_cast<void**>(&pin.p), sizeof(double) * 2 * kCh, hipHostMallocDefault));
    hipEvent_t ev[2] = {nullptr, nullptr};
    struct EvGuard {
      hipEvent_t* e;
      ~EvGuard() {
        for (int i = 0; i < 2; ++i)
          if (e[i]) (void)hipEventDestroy(e[i]);
      }
    } evg{ev};
    for (int i = 0; i < 2; ++i) MTRY(c, hipEventCreateWithFlags(&ev[i], hipEventDisableTiming));
    const int64_t nch = (n + kCh - 1) / kCh;
    auto enqueue = [&](int64_t ch) -> hipError_t {
      const int64_t lo = ch * kCh, cnt = std::min(kCh, n - lo);
      hipError_t e = hipMemcpyAsync(pin.p + (ch & 1) * kCh, avg_dist + lo, sizeof(double) * cnt,
                                    hipMemcpyDeviceToHost, s);
      return e == hipSuccess ? hipEventRecord(ev[ch & 1], s) : e;
    };
    for (int pass = 0; pass < 2; ++pass) {
      MTRY(c, enqueue(0));
      if (nch > 1) MTRY(c, enqueue(1));
      for (int64_t ch = 0; ch < nch; ++ch) {
        MTRY(c, hipEventSynchronize(ev[ch & 1]));
        const double* v = pin.p + (ch & 1) * kCh;
        const int64_t cnt = std::min(kCh, n - ch * kCh);
        if (pass == 0) {
          double m = mean;
          int64_t va = valid;
          for (int64_t i = 0; i < cnt; ++i) {
            m = m + (v[i] > 0 ? v[i] : 0.0);
            va += v[i] >= 0.0 ? 1 : 0;  // every point has >= 1 neighbour (itself)
          }
          mean = m;
          valid = va;
        } else {
          double q = sq;
          for (int64_t i = 0; i < cnt; ++i) q = q + (v[i] > 0 ? (v[i] - mean) * (v[i] - mean) : 0);
          sq = q;
        }
        if (ch + 2 < nch) MTRY(c, enqueue(ch + 2));
      }
      if (pass == 0) {
        if (valid == 0) return SL_OK;
        mean /= static_cast<double>(valid);
      }
    }
  }
  const double sd = sqrt(sq / static_cast<double>(valid - 1));
  const double thr = mean + std_ratio * sd;
  hipLaunchKernelGGL(k_keep_flags, dim3(blocks(n)), dim3(kT), 0, s, avg_dist, n, thr, flag.p);
  int64_t kept = 0;
  r = scan_flags(c, flag.p, n, seg.p, &kept, s);
  if (r) return r;
  hipLaunchKernelGGL(k_compact_index, dim3(blocks(n)), dim3(kT), 0, s, flag.p, seg.p, n, out_index);
  MTRY(c, hipGetLastError());
  MTRY(c, hipStreamSynchronize(s));
  *out_n = kept;
  return SL_OK;
}

int sl_select_by_index(sl_ctx* c, const double* xyz, const uint8_t* bgr, const int64_t* index, int64_t m,
                       double* out_xyz, uint8_t* out_bgr, void* stream) {
  if (!c || m < 0 || (m && (!xyz || !index || !out_xyz))) return SL_EINVAL;
  if (m == 0) return SL_OK;
  MTRY(c, hipSetDevice(slgpu_device(c)));
  hipLaunchKernelGGL(k_gather, dim3(blocks(m)), dim3(kT), 0, static_cast<hipStream_t>(stream), xyz, bgr, index, m,
                     out_xyz, out_bgr);
  MTRY(c, hipGetLastError());
  return SL_OK;
}

int sl_transform_points(sl_ctx* c, double* xyz, int64_t n, const double* pose, void* stream) {
  if (!c || n < 0 || (n && (!xyz || !pose))) return SL_EINVAL;
  if (n == 0) return SL_OK;
  MTRY(c, hipSetDevice(slgpu_device(c)));
  hipLaunchKernelGGL(k_transform, dim3(blocks(n)), dim3(kT), 0, static_cast<hipStream_t>(stream), xyz, n, pose);
  MTRY(c, hipGetLastError());
  return SL_OK;
}

// PointCloud::EstimateNormals(KDTreeSearchParamHybrid(radius, max_nn)) of a
// cloud without normals (processing.py:178) -> normals [n, 3] f64.
int sl_estimate_normals(sl_ctx* c, const double* xyz, int64_t n, double radius, int max_nn, double* normals,
                        void* stream) {
  if (!c || n < 0 || (n && (!xyz || !normals))) return SL_EINVAL;
  if (max_nn > kNrmK) return slgpu_fail(c, SL_EINVAL, "max_nn > 32 is not supported");
  if (std::isnan(radius)) return slgpu_fail(c, SL_EINVAL, "radius is NaN");
  if (n >= (1ll << 31)) return slgpu_fail(c, SL_EINVAL, "at most 2^31 - 1 points");
  if (n == 0) return SL_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  PoolStream pool_stream(s);
  MTRY(c, hipSetDevice(slgpu_device(c)));
  // nanoflann searches radius * radius, so a negative radius acts as |radius|
  const double r2 = radius * radius;
  radius = fabs(radius);
  if (!(r2 > 0.0) || max_nn < 3) {  // no point has 3 neighbours: identity covariance -> (0, 0, 1)
    hipLaunchKernelGGL(k_fill_up, dim3(blocks(n)), dim3(kT), 0, s, normals, n);
    MTRY(c, hipGetLastError());
    return SL_OK;
  }
  double b[6];
  int r = bounds(c, xyz, n, b, s);
  if (r) return r;
  double emax = 0.0;
  for (int k = 0; k < 3; ++k) emax = std::max(emax, b[3 + k] - b[k]);
  if (!std::isfinite(emax)) return slgpu_fail(c, SL_EINVAL, "non-finite point coordinates");
  // cells of edge >= radius, so the 27 around a query's cell hold its ball;
  // at most ~1e6 per axis
  const double h = std::max(radius, emax / 1.0e6);
  Grid g;
  if (!make_grid(b, b + 3, h, &g)) return slgpu_fail(c, SL_EINVAL, "normal-search grid is too large");
  DBuf<uint64_t> keys, ukeys;
  DBuf<uint32_t> idx, ustart;
  int64_t m = 0;
  r = cells(c, xyz, n, g, keys, idx, ukeys, ustart, &m, s);
  if (r) return r;
  DBuf<double> sxyz;
  DBuf<int32_t> nbr;
  MTRY(c, sxyz.alloc(3 * n));
  MTRY(c, nbr.alloc(27 * m));
  hipLaunchKernelGGL(k_gather_sorted, dim3(blocks(n)), dim3(kT), 0, s, xyz, idx.p, n, sxyz.p);
  hipLaunchKernelGGL(k_cell_neighbours_lin, dim3(blocks(m)), dim3(kT), 0, s, ukeys.p, m, g.nx, g.ny, g.nz, nbr.p);
  hipLaunchKernelGGL(k_normals, dim3(blocks(n)), dim3(kT), 0, s, xyz, sxyz.p, idx.p, keys.p, n, ukeys.p, ustart.p, m,
                     nbr.p, r2, max_nn, normals);
  MTRY(c, hipGetLastError());
  MTRY(c, hipStreamSynchronize(s));
  return SL_OK;
}

// registration_icp with TransformationEstimationPointToPlane (processing.py:
// 154-156).  Host side of each iteration: the block partials folded left to
// right, the 6x6 normal equations JTJ x = -JTr by a pivoted LDLT (Open3D:
// Eigen's LDLT, icp_update), x = (alpha, beta, gamma, t) ->
// update = [Rz(gamma) Ry(beta) Rx(alpha) | t] (TransformVector6dToMatrix4d),
// transformation = update * transformation, source moved by update.
namespace {

void icp_mat3(const double a[3][3], const double b[3][3], double o[3][3]) {
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) o[i][j] = (a[i][0] * b[0][j] + a[i][1] * b[1][j]) + a[i][2] * b[2][j];
}

void icp_mat4(const double* a, const double* b, double* o) {  // row-major 4x4: o = a b
  double t[16];
  for (int i = 0; i < 4; ++i)
    for (int j = 0; j < 4; ++j)
      t[4 * i + j] = ((a[4 * i] * b[j] + a[4 * i + 1] * b[4 + j]) + a[4 * i + 2] * b[8 + j]) + a[4 * i + 3] * b[12 + j];
  memcpy(o, t, sizeof(t));
}

// 6x6 JTJ x = -JTr (sums: JTJ upper triangle row-major, then JTr) -> update
// (row-major 4x4), as Open3D's SolveLinearSystemPSD (utility/Eigen.cpp: no
// PSD / determinant checks, x = A.ldlt().solve(b)) -- Eigen's LDLT: the
// unblocked left-looking factorisation with diagonal pivoting (the largest
// |a_ii| of the not yet factored diagonal, first on ties), pivots of 0 left
// unscaled, and a solve that zeroes the components of |d_i| <= DBL_MIN (its
// pseudo-inverse of D), so a rank-deficient system still moves along the
// directions it constrains.  Sums of products run left to right (Eigen's
// vectorised order may differ in the last bits; parity with Open3D unpinned).
// false (identity update) only when the solution is not finite.
bool icp_update(const double* sums, double* update) {
  double F[6][6], b[6], x[6], tmp[6];
  int tr[6];
  int k = 0;
  for (int a = 0; a < 6; ++a)
    for (int c = a; c < 6; ++c, ++k) F[a][c] = F[c][a] = sums[k];
  for (int a = 0; a < 6; ++a) b[a] = -sums[21 + a];
  for (int i = 0; i < 16; ++i) update[i] = (i % 5 == 0) ? 1.0 : 0.0;
  bool zero_all = false;
  for (int j = 0; j < 6; ++j) {
    int p = j;
    for (int i = j + 1; i < 6; ++i)
      if (std::fabs(F[i][i]) > std::fabs(F[p][p])) p = i;
    tr[j] = p;
    if (p != j) {  // symmetric swap of rows / columns j and p (full storage)
      for (int q = 0; q < 6; ++q) std::swap(F[j][q], F[p][q]);
      for (int q = 0; q < 6; ++q) std::swap(F[q][j], F[q][p]);
    }
    if (j > 0) {
      for (int q = 0; q < j; ++q) tmp[q] = F[q][q] * F[j][q];
      double d = 0.0;
      for (int q = 0; q < j; ++q) d = d + F[j][q] * tmp[q];
      F[j][j] = F[j][j] - d;
      for (int i = j + 1; i < 6; ++i) {
        double v = 0.0;
        for (int q = 0; q < j; ++q) v = v + F[i][q] * tmp[q];
        F[i][j] = F[i][j] - v;
      }
    }
    const double piv = F[j][j];
    if (j == 0 && !(std::fabs(piv) > 0.0)) {  // the whole diagonal is 0: A = 0, x = 0
      zero_all = true;
      break;
    }
    if (std::fabs(piv) > 0.0)
      for (int i = j + 1; i < 6; ++i) F[i][j] = F[i][j] / piv;
  }
  if (zero_all) {
    for (int i = 0; i < 6; ++i) x[i] = 0.0;
  } else {
    for (int j = 0; j < 6; ++j) std::swap(b[j], b[tr[j]]);  // P b
    for (int i = 0; i < 6; ++i) {                            // L^-1 (unit lower)
      double v = 0.0;
      for (int q = 0; q < i; ++q) v = v + F[i][q] * b[q];
      b[i] = b[i] - v;
    }
    for (int i = 0; i < 6; ++i)  // D^+
      b[i] = std::fabs(F[i][i]) > std::numeric_limits<double>::min() ? b[i] / F[i][i] : 0.0;
    for (int i = 5; i >= 0; --i) {  // L^-T
      double v = 0.0;
      for (int q = i + 1; q < 6; ++q) v = v + F[q][i] * b[q];
      b[i] = b[i] - v;
    }
    for (int j = 5; j >= 0; --j) std::swap(b[j], b[tr[j]]);  // P^T
    for (int i = 0; i < 6; ++i) x[i] = b[i];
  }
  for (int i = 0; i < 6; ++i)
    if (!std::isfinite(x[i])) return false;
  const double ca = std::cos(x[0]), sa = std::sin(x[0]), cb = std::cos(x[1]), sb = std::sin(x[1]);
  const double cg = std::cos(x[2]), sg = std::sin(x[2]);
  const double Rx[3][3] = {{1.0, 0.0, 0.0}, {0.0, ca, -sa}, {0.0, sa, ca}};
  const double Ry[3][3] = {{cb, 0.0, sb}, {0.0, 1.0, 0.0}, {-sb, 0.0, cb}};
  const double Rz[3][3] = {{cg, -sg, 0.0}, {sg, cg, 0.0}, {0.0, 0.0, 1.0}};
  double M[3][3], R[3][3];
  icp_mat3(Ry, Rx, M);
  icp_mat3(Rz, M, R);
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j) update[4 * i + j] = R[i][j];
    update[4 * i + 3] = x[3 + i];
  }
  return true;
}

}  // namespace

int sl_icp_point_to_plane(sl_ctx* c, const double* source, int64_t n_src, const double* target,
                          const double* target_normals, int64_t n_tgt, double max_distance, const double* init,
                          int max_iteration, double relative_fitness, double relative_rmse, double* transformation,
                          double* fitness, double* inlier_rmse, int* iterations, void* stream) {
  if (!c) return SL_EINVAL;
  if (n_src < 0 || n_tgt < 0 || !init || !transformation || max_iteration < 0 || (n_src && !source) ||
      (n_tgt && (!target || !target_normals)))
    return slgpu_fail(c, SL_EINVAL, "sl_icp_point_to_plane: bad sizes or NULL arguments");
  if (n_src >= (1ll << 31) || n_tgt >= (1ll << 31)) return slgpu_fail(c, SL_EINVAL, "at most 2^31 - 1 points");
  if (!(max_distance > 0.0)) return slgpu_fail(c, SL_EINVAL, "max_correspondence_distance must be > 0");
  double T[16];
  memcpy(T, init, sizeof(T));
  double fit = 0.0, rmse = 0.0;
  int iters = 0;
  auto finish = [&]() {
    memcpy(transformation, T, sizeof(T));
    if (fitness) *fitness = fit;
    if (inlier_rmse) *inlier_rmse = rmse;
    if (iterations) *iterations = iters;
    return SL_OK;
  };
  if (n_src == 0 || n_tgt == 0) return finish();
  hipStream_t s = static_cast<hipStream_t>(stream);
  PoolStream pool_stream(s);
  MTRY(c, hipSetDevice(slgpu_device(c)));
  // the target's cell grid (cells of edge >= max_distance: the 27 around a
  // query's cell hold its ball)
  double bnd[6];
  int r = bounds(c, target, n_tgt, bnd, s);
  if (r) return r;
  double emax = 0.0;
  for (int k = 0; k < 3; ++k) emax = std::max(emax, bnd[3 + k] - bnd[k]);
  if (!std::isfinite(emax)) return slgpu_fail(c, SL_EINVAL, "non-finite target coordinates");
  Grid g;
  if (!make_grid(bnd, bnd + 3, std::max(max_distance, emax / 1.0e6), &g))
    return slgpu_fail(c, SL_EINVAL, "correspondence grid is too large");
  DBuf<uint64_t> keys, ukeys;
  DBuf<uint32_t> idx, ustart;
  int64_t m = 0;
  r = cells(c, target, n_tgt, g, keys, idx, ukeys, ustart, &m, s);
  if (r) return r;
  DBuf<double> sxyz, cur, d2, part, dmat;
  DBuf<int32_t> corr, dense;
  MTRY(c, sxyz.alloc(3 * n_tgt));
  hipLaunchKernelGGL(k_gather_sorted, dim3(blocks(n_tgt)), dim3(kT), 0, s, target, idx.p, n_tgt, sxyz.p);
  MTRY(c, hipGetLastError());
  const int64_t ncell = (g.nx * g.ny) * g.nz;
  if (ncell <= (int64_t{1} << 26)) {  // a dense cell table (<= 256 MB), else binary search
    MTRY(c, dense.alloc(ncell));
    MTRY(c, hipMemsetAsync(dense.p, 0xff, sizeof(int32_t) * ncell, s));
    hipLaunchKernelGGL(k_icp_dense, dim3(blocks(m)), dim3(kT), 0, s, ukeys.p, m, dense.p);
    MTRY(c, hipGetLastError());
  }
  const int64_t nb = (n_src + kIcpBlock - 1) / kIcpBlock;
  MTRY(c, cur.alloc(3 * n_src));
  MTRY(c, d2.alloc(n_src));
  MTRY(c, corr.alloc(n_src));
  MTRY(c, part.alloc(kIcpSums * nb));
  MTRY(c, dmat.alloc(16));
  MTRY(c, hipMemcpyAsync(cur.p, source, sizeof(double) * 3 * n_src, hipMemcpyDeviceToDevice, s));
  std::vector<double> hpart(static_cast<size_t>(kIcpSums * nb));
  double sums[kIcpSums];
  // pcd.Transform(init) unless init is the identity (exactly)
  bool ident = true;
  for (int i = 0; i < 16; ++i) ident = ident && T[i] == ((i % 5 == 0) ? 1.0 : 0.0);
  auto move = [&](const double* M) -> int {
    MTRY(c, hipMemcpyAsync(dmat.p, M, sizeof(double) * 16, hipMemcpyHostToDevice, s));
    hipLaunchKernelGGL(k_transform, dim3(blocks(n_src)), dim3(kT), 0, s, cur.p, n_src, dmat.p);
    MTRY(c, hipGetLastError());
    MTRY(c, hipStreamSynchronize(s));  // dmat (device) and M (host) are reused
    return SL_OK;
  };
  if (!ident && (r = move(T))) return r;
  const double r2 = max_distance * max_distance;
  auto evaluate = [&]() -> int {
    hipLaunchKernelGGL(k_icp_corr, dim3(blocks(n_src)), dim3(kT), 0, s, cur.p, n_src, g, dense.p, ukeys.p, m,
                       ustart.p, n_tgt, sxyz.p, idx.p, r2, corr.p, d2.p);
    hipLaunchKernelGGL(k_icp_fold, dim3(blocks(nb)), dim3(kT), 0, s, cur.p, n_src, target, target_normals, corr.p,
                       d2.p, part.p);
    MTRY(c, hipGetLastError());
    MTRY(c, hipMemcpyAsync(hpart.data(), part.p, sizeof(double) * hpart.size(), hipMemcpyDeviceToHost, s));
    MTRY(c, hipStreamSynchronize(s));
    for (int k = 0; k < kIcpSums; ++k) sums[k] = 0.0;
    for (int64_t b = 0; b < nb; ++b)
      for (int k = 0; k < kIcpSums; ++k) sums[k] = sums[k] + hpart[static_cast<size_t>(kIcpSums * b + k)];
    const double cnt = sums[28];
    fit = cnt / static_cast<double>(n_src);
    rmse = cnt > 0.0 ? std::sqrt(sums[27] / cnt) : 0.0;
    return SL_OK;
  };
  if ((r = evaluate())) return r;
  for (int it = 0; it < max_iteration; ++it) {
    double U[16];
    icp_update(sums, U);  // (identity only for a non-finite solution)
    icp_mat4(U, T, T);
    if ((r = move(U))) return r;
    const double f0 = fit, r0 = rmse;
    if ((r = evaluate())) return r;
    iters = it + 1;
    if (std::fabs(f0 - fit) < relative_fitness && std::fabs(r0 - rmse) < relative_rmse) break;
  }
  return finish();
}

// Release the scratch buffers the merge pool keeps for `device` (they are
// otherwise kept for the process's lifetime, up to 16 GiB per device).
int sl_merge_pool_trim(int device, int64_t* released_bytes) {
  int prev = 0;
  if (hipGetDevice(&prev) != hipSuccess || hipSetDevice(device) != hipSuccess) return SL_EHIP;
  const size_t b = pool_trim(device);
  (void)hipSetDevice(prev);
  if (released_bytes) *released_bytes = static_cast<int64_t>(b);
  return SL_OK;
}

}  // extern "C"

// global registration (FPFH, feature matching, RANSAC): the same translation unit
#include "slreg.inl"
