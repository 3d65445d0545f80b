// Read-bandwidth microbenchmark for the stack access pattern of k_decode
// (measurement only, not part of the library): 46 planes of a 3840x2160 view,
// every lane reads 16 bytes of each plane at its pixel offset -- in the
// planar layout the API takes ([plane][H][W]), and in a chunk-tiled layout
// ([chunk of 1024 px][plane][1024 px]) -- against a plain linear float4 read
// of the same bytes.  Prints GB/s per pattern.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
constexpr int kPlanes = 46;
constexpr int64_t kHW = 3840LL * 2160;
constexpr int kChunk = 1024;

__global__ __launch_bounds__(256) void planar(const uint8_t* st, int64_t HW, unsigned* out, int ngroups) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned acc = 0;
  for (int cg = blockIdx.x; cg < ngroups; cg += gridDim.x) {
    const int64_t px = (static_cast<int64_t>(cg) * 4 + wid) * kChunk + lane * 16;
    if (px >= HW) continue;
    v4u v[kPlanes];
#pragma unroll
    for (int p = 0; p < kPlanes; ++p) v[p] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(st + p * HW + px));
#pragma unroll
    for (int p = 0; p < kPlanes; ++p) acc ^= v[p][0] ^ v[p][1] ^ v[p][2] ^ v[p][3];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

// planar reads + k_decode's writes per lane: col, row (64 B each), records
// (32 B), mask (16 B) -- 9 B/px + the 2-B records
__global__ __launch_bounds__(256) void planar_rw(const uint8_t* st, int64_t HW, unsigned* out, int ngroups,
                                                 v4u* col, v4u* row, v4u* rec, v4u* msk) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int cg = blockIdx.x; cg < ngroups; cg += gridDim.x) {
    const int64_t px = (static_cast<int64_t>(cg) * 4 + wid) * kChunk + lane * 16;
    if (px >= HW) continue;
    v4u v[kPlanes];
#pragma unroll
    for (int p = 0; p < kPlanes; ++p) v[p] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(st + p * HW + px));
    v4u a = v[0], b = v[1];
#pragma unroll
    for (int p = 2; p < kPlanes; p += 2) { a ^= v[p]; b += v[p + 1]; }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      col[px / 4 + i] = a + i;
      row[px / 4 + i] = b + i;
    }
    rec[px / 8] = a ^ b;
    rec[px / 8 + 1] = a - b;
    msk[px / 16] = a & b;
  }
}

// the same traffic with each store instruction writing 1 KB contiguous per
// wave (lane l -> bytes 16 l of the instruction's 1 KB), as an LDS transpose
// of the maps would; NT: the maps with nontemporal stores (the library since
// round 5), the records write-through (sc1), as k_decode issues them
template <bool NT>
__device__ inline void st_map(v4u* p, v4u v) {
  if (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}
template <bool NT>
__global__ __launch_bounds__(256) void planar_rw_contig(const uint8_t* st, int64_t HW, unsigned* out, int ngroups,
                                                        v4u* col, v4u* row, v4u* rec, v4u* msk) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int cg = blockIdx.x; cg < ngroups; cg += gridDim.x) {
    const int64_t chunk = static_cast<int64_t>(cg) * 4 + wid;
    const int64_t px = chunk * kChunk + lane * 16;
    if (px >= HW) continue;
    v4u v[kPlanes];
#pragma unroll
    for (int p = 0; p < kPlanes; ++p) v[p] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(st + p * HW + px));
    v4u a = v[0], b = v[1];
#pragma unroll
    for (int p = 2; p < kPlanes; p += 2) { a ^= v[p]; b += v[p + 1]; }
    const int64_t c4 = chunk * kChunk / 4;  // the chunk's first v4u of a 4 B/px map
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      st_map<NT>(col + c4 + 64 * i + lane, a + i);
      st_map<NT>(row + c4 + 64 * i + lane, b + i);
    }
    const int64_t c8 = chunk * kChunk / 8;
    if (NT) {
      const auto rr = __builtin_amdgcn_make_buffer_rsrc(rec + c8, 0, 2048, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(a ^ b, rr, 16 * lane, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(a - b, rr, 1024 + 16 * lane, 0, 16);
    } else {
      rec[c8 + lane] = a ^ b;
      rec[c8 + 64 + lane] = a - b;
    }
    st_map<NT>(msk + chunk * kChunk / 16 + lane, a & b);
  }
}

// quad layout: lane l owns pixels 256 i + 4 l + e (i, e < 4): dword loads
// (256 B contiguous per wave instruction, 4 per plane), contiguous stores
__global__ __launch_bounds__(256) void quad_rw(const uint8_t* st, int64_t HW, unsigned* out, int ngroups,
                                               v4u* col, v4u* row, v4u* rec, v4u* msk) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  for (int cg = blockIdx.x; cg < ngroups; cg += gridDim.x) {
    const int64_t chunk = static_cast<int64_t>(cg) * 4 + wid;
    if (chunk * kChunk >= HW) continue;
    const uint8_t* base = st + chunk * kChunk + 4 * lane;
    unsigned v[kPlanes][4];
#pragma unroll
    for (int p = 0; p < kPlanes; ++p)
#pragma unroll
      for (int i = 0; i < 4; ++i)
        v[p][i] = __builtin_nontemporal_load(reinterpret_cast<const unsigned*>(base + p * HW + 256 * i));
    v4u a, b;
#pragma unroll
    for (int i = 0; i < 4; ++i) { a[i] = v[0][i]; b[i] = v[1][i]; }
#pragma unroll
    for (int p = 2; p < kPlanes; p += 2)
#pragma unroll
      for (int i = 0; i < 4; ++i) { a[i] ^= v[p][i]; b[i] += v[p + 1][i]; }
    const int64_t c4 = chunk * kChunk / 4;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      col[c4 + 64 * i + lane] = a + i;
      row[c4 + 64 * i + lane] = b + i;
    }
    const int64_t c8 = chunk * kChunk / 8;
    rec[c8 + lane] = a ^ b;
    rec[c8 + 64 + lane] = a - b;
    msk[chunk * kChunk / 16 + lane] = a & b;
  }
}

__global__ __launch_bounds__(256) void tiled(const uint8_t* st, int64_t HW, unsigned* out, int ngroups) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  unsigned acc = 0;
  for (int cg = blockIdx.x; cg < ngroups; cg += gridDim.x) {
    const int64_t chunk = static_cast<int64_t>(cg) * 4 + wid;
    if (chunk * kChunk >= HW) continue;
    const uint8_t* t = st + chunk * kChunk * kPlanes + lane * 16;
    v4u v[kPlanes];
#pragma unroll
    for (int p = 0; p < kPlanes; ++p) v[p] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(t + p * kChunk));
#pragma unroll
    for (int p = 0; p < kPlanes; ++p) acc ^= v[p][0] ^ v[p][1] ^ v[p][2] ^ v[p][3];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

__global__ __launch_bounds__(256) void linear(const v4u* st, int64_t n16, unsigned* out) {
  unsigned acc = 0;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n16; i += static_cast<int64_t>(gridDim.x) * 256) {
    const v4u v = __builtin_nontemporal_load(st + i);
    acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  if (acc == 0x12345678u) out[0] = acc;
}

int main() {
  const int64_t bytes = kPlanes * kHW;
  uint8_t* st;
  unsigned* out;
  if (hipMalloc(&st, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  (void)hipMemset(st, 7, bytes);
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  const int ngroups = static_cast<int>((kHW / kChunk + 3) / 4);
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  v4u *col, *row, *rec, *msk;
  if (hipMalloc(&col, 4 * kHW) != hipSuccess || hipMalloc(&row, 4 * kHW) != hipSuccess ||
      hipMalloc(&rec, 2 * kHW) != hipSuccess || hipMalloc(&msk, kHW) != hipSuccess) return 1;
  for (int per_cu : {2, 3, 4, 8}) {
    const int grid = per_cu * n_cu;
    for (int k = 0; k < 7; ++k) {
      float best = 1e30f;
      for (int r = 0; r < 20; ++r) {
        (void)hipEventRecord(a, 0);
        if (k == 0) hipLaunchKernelGGL(planar, dim3(grid), dim3(256), 0, 0, st, kHW, out, ngroups);
        if (k == 1) hipLaunchKernelGGL(tiled, dim3(grid), dim3(256), 0, 0, st, kHW, out, ngroups);
        if (k == 2) hipLaunchKernelGGL(linear, dim3(grid), dim3(256), 0, 0, reinterpret_cast<const v4u*>(st), bytes / 16, out);
        if (k == 3) hipLaunchKernelGGL(planar_rw, dim3(grid), dim3(256), 0, 0, st, kHW, out, ngroups, col, row, rec, msk);
        if (k == 5) hipLaunchKernelGGL(quad_rw, dim3(grid), dim3(256), 0, 0, st, kHW, out, ngroups, col, row, rec, msk);
        if (k == 4) hipLaunchKernelGGL(planar_rw_contig<false>, dim3(grid), dim3(256), 0, 0, st, kHW, out, ngroups, col, row, rec, msk);
        if (k == 6) hipLaunchKernelGGL(planar_rw_contig<true>, dim3(grid), dim3(256), 0, 0, st, kHW, out, ngroups, col, row, rec, msk);
        (void)hipEventRecord(b, 0);
        (void)hipEventSynchronize(b);
        float ms = 0.f;
        (void)hipEventElapsedTime(&ms, a, b);
        if (r > 2 && ms < best) best = ms;
      }
      const double moved = k >= 3 ? bytes + 11.0 * kHW : bytes;
      printf("{\"pattern\": \"%s\", \"wg_per_cu\": %d, \"us\": %.2f, \"GBps\": %.0f}\n",
             k == 0 ? "planar" : k == 1 ? "tiled" : k == 2 ? "linear" : k == 3 ? "planar+kdecode_writes" : k == 4 ? "planar+contiguous_writes" : k == 5 ? "quad+contiguous_writes" : "planar+contiguous_writes_nt", per_cu, best * 1e3,
             moved / (best * 1e-3) / 1e9);
    }
  }
  return 0;
}
