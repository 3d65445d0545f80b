// Microbenchmark (measurement only, not part of the library): why 6 % of
// writes cost the cloud-only k_decode pattern ~28 % of its time.
// cloud_decode_floor's kernel (V views of 3840x2160, 46-plane stacks, the first
// 24 planes read once, 16 B per lane, non-temporal; 1.5 B/px of 12-bit records
// per view) in variants that separate where the cost of the record stores
// arises:
//   0 reads only
//   1 records, k_decode's shape (two 12-B stores per lane, 24 B at 24 lane)
//   2 the same stores into a per-workgroup 6-KB slot rewritten every chunk
//     group (L2-resident: the records never reach HBM)
//   3 records as one 16-B + one 8-B buffer store per lane, default policy
//   4 shape 3 with sc1 (write-through) stores
//   5 shape 1, software-pipelined: a chunk's stores issue after the next
//     chunk's loads (a wait for those loads no longer waits for the stores)
//   6 shape 1 followed by a vmcnt(0) wait (the stores' latency exposed)
//   7 1.5 B/px of extra reads (24 B per lane) instead of the stores
//   8 a plain 16-B copy (read a byte range, write it elsewhere) for reference
//   9 shape 1 as two 12-B buffer stores with sc1, software-pipelined as 5
//  10 shape 1 as two 12-B buffer stores with sc1
//  11 the same with sc1 nt
//  12 the same with sc0 sc1
//  13 16-B stores only, sc1: 16 B at 16 lane, then the even lanes 16 B at
//     1024 + 8 lane (words 4-5 of the lane and of the next one, by DPP)
//  14 13 with default-policy stores
//  15 4's stores, the records of the launch's views interleaved by chunk
//     group (offset of (group, view): (group V + view) 6 KB), so that the
//     workgroups of every view write one contiguous window at a time
//  16 1's stores with 15's layout
//  17-20 15 with the plane loads as buffer loads of cache policy 0 (default),
//     2 (nt, as k_decode), 16 (sc1), 1 (sc0)
//  21-22 reads only, buffer loads of policy 0 / 2
// One JSON line per variant: avg / best over 20 timed launches.
//   write_mix [views [H W]]
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v3u __attribute__((ext_vector_type(3)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
constexpr int kChunk = 1024;
constexpr int kPlanesStack = 46;
constexpr int kNpl = 24;

__device__ __forceinline__ void load_chunk(v4u (&v)[kNpl], const uint8_t* vb, int64_t HW, int64_t px) {
#pragma unroll
  for (int p = 0; p < kNpl; ++p) v[p] = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(vb + p * HW + px));
}

__device__ __forceinline__ void words_of(const v4u (&v)[kNpl], uint32_t (&w)[6]) {
  v4u a = v[0], b = v[1];
#pragma unroll
  for (int p = 2; p < kNpl; p += 2) {
    a ^= v[p];
    b += v[p + 1];
  }
  w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = b.x; w[4] = b.y; w[5] = b.w ^ a.w;
}

template <int AUX>
__device__ __forceinline__ void load_chunk_buf(v4u (&v)[kNpl], const uint8_t* vb, int64_t HW, int64_t px) {
  // (a view's 24 planes span < 2 GiB: one descriptor, plane offsets in soffset)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(vb), 0, static_cast<int>(kNpl * HW), 0x00020000);
#pragma unroll
  for (int p = 0; p < kNpl; ++p) v[p] = __builtin_amdgcn_raw_buffer_load_b128(rs, static_cast<int>(px), p * static_cast<int>(HW), AUX);
}

template <int MODE>
__global__ __launch_bounds__(256, 3) void mix_k(const uint8_t* st, int64_t HW, int64_t vs, int ngroups, uint8_t* rec,
                                                uint8_t* hot) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int view = blockIdx.y;
  const uint8_t* vb = st + view * vs;
  uint8_t* rb = rec + view * (HW * 3 / 2);
  if (MODE == 5) {  // (HW a multiple of 4 chunks: checked on the host)
    int cg = blockIdx.x;
    if (cg >= ngroups) return;
    v4u v[kNpl];
    load_chunk(v, vb, HW, (static_cast<int64_t>(cg) * 4 + wid) * kChunk + lane * 16);
    for (;;) {
      uint32_t w[6];
      words_of(v, w);
      uint32_t* ro = reinterpret_cast<uint32_t*>(rb + (static_cast<int64_t>(cg) * 4 + wid) * (kChunk * 3 / 2) + 24 * lane);
      const int nx = cg + gridDim.x;
      if (nx < ngroups) load_chunk(v, vb, HW, (static_cast<int64_t>(nx) * 4 + wid) * kChunk + lane * 16);
      *reinterpret_cast<v3u*>(ro) = v3u{w[0], w[1], w[2]};
      *reinterpret_cast<v3u*>(ro + 3) = v3u{w[3], w[4], w[5]};
      if (nx >= ngroups) break;
      cg = nx;
    }
    return;
  }
  if (MODE == 9) {  // 5 with sc1 buffer stores
    int cg = blockIdx.x;
    if (cg >= ngroups) return;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(rb, 0, static_cast<int>(HW * 3 / 2), 0x00020000);
    v4u v[kNpl];
    load_chunk(v, vb, HW, (static_cast<int64_t>(cg) * 4 + wid) * kChunk + lane * 16);
    for (;;) {
      uint32_t w[6];
      words_of(v, w);
      const int ro = (cg * 4 + wid) * (kChunk * 3 / 2) + 24 * lane;
      const int nx = cg + gridDim.x;
      if (nx < ngroups) load_chunk(v, vb, HW, (static_cast<int64_t>(nx) * 4 + wid) * kChunk + lane * 16);
      __builtin_amdgcn_raw_buffer_store_b96(v3u{w[0], w[1], w[2]}, rs, ro, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b96(v3u{w[3], w[4], w[5]}, rs, ro + 12, 0, 16);
      if (nx >= ngroups) break;
      cg = nx;
    }
    return;
  }
  for (int cg = blockIdx.x; cg < ngroups; cg += gridDim.x) {
    const int64_t chunk = static_cast<int64_t>(cg) * 4 + wid;
    const int64_t px = chunk * kChunk + lane * 16;
    if (px >= HW) continue;
    v4u v[kNpl];
    if (MODE == 17 || MODE == 21) load_chunk_buf<0>(v, vb, HW, px);
    else if (MODE == 18 || MODE == 22) load_chunk_buf<2>(v, vb, HW, px);
    else if (MODE == 19) load_chunk_buf<16>(v, vb, HW, px);
    else if (MODE == 20) load_chunk_buf<1>(v, vb, HW, px);
    else load_chunk(v, vb, HW, px);
    uint32_t w[6];
    words_of(v, w);
    uint8_t* cb = (MODE == 15 || MODE == 16 || (MODE >= 17 && MODE <= 20))
                      ? rec + ((static_cast<int64_t>(cg) * gridDim.y + view) * 4 + wid) * (kChunk * 3 / 2)
                      : rb + chunk * (kChunk * 3 / 2);
    if (MODE == 1 || MODE == 6 || MODE == 16) {
      uint32_t* ro = reinterpret_cast<uint32_t*>(cb + 24 * lane);
      *reinterpret_cast<v3u*>(ro) = v3u{w[0], w[1], w[2]};
      *reinterpret_cast<v3u*>(ro + 3) = v3u{w[3], w[4], w[5]};
      if (MODE == 6) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    } else if (MODE == 2) {
      uint32_t* ro = reinterpret_cast<uint32_t*>(hot + (static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x) * 6144 +
                                                 wid * 1536 + 24 * lane);
      *reinterpret_cast<v3u*>(ro) = v3u{w[0], w[1], w[2]};
      *reinterpret_cast<v3u*>(ro + 3) = v3u{w[3], w[4], w[5]};
    } else if (MODE == 3 || MODE == 4 || MODE == 15 || (MODE >= 17 && MODE <= 20)) {
      constexpr int aux = MODE != 3 ? 16 : 0;  // 16: sc1
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(cb, 0, kChunk * 3 / 2, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(v4u{w[0], w[1], w[2], w[3]}, rs, 16 * lane, 0, aux);
      __builtin_amdgcn_raw_buffer_store_b64(v2u{w[4], w[5]}, rs, 1024 + 8 * lane, 0, aux);
    } else if (MODE >= 10 && MODE <= 12) {
      constexpr int aux = MODE == 10 ? 16 : MODE == 11 ? 18 : 17;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(cb, 0, kChunk * 3 / 2, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b96(v3u{w[0], w[1], w[2]}, rs, 24 * lane, 0, aux);
      __builtin_amdgcn_raw_buffer_store_b96(v3u{w[3], w[4], w[5]}, rs, 24 * lane + 12, 0, aux);
    } else if (MODE == 13 || MODE == 14) {
      constexpr int aux = MODE == 13 ? 16 : 0;
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(cb, 0, kChunk * 3 / 2, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(v4u{w[0], w[1], w[2], w[3]}, rs, 16 * lane, 0, aux);
      // row_shl:1 -- lane l reads lane l + 1 (even lanes: always within the row)
      const uint32_t n4 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(w[4]), 0x101, 0xf, 0xf, false));
      const uint32_t n5 = static_cast<uint32_t>(__builtin_amdgcn_mov_dpp(static_cast<int>(w[5]), 0x101, 0xf, 0xf, false));
      if (!(lane & 1)) __builtin_amdgcn_raw_buffer_store_b128(v4u{w[4], w[5], n4, n5}, rs, 1024 + 8 * lane, 0, aux);
    } else if (MODE == 7) {
      const v4u x = *reinterpret_cast<const v4u*>(cb + 16 * lane);
      const v2u y = *reinterpret_cast<const v2u*>(cb + 1024 + 8 * lane);
      if ((w[0] ^ x.x ^ y.y) == 0x12345678u && (w[3] + x.w + y.x) == 7u) rb[0] = 1;
    } else if (w[0] == 0x12345678u && w[3] == 7u) {
      rb[0] = 1;
    }
  }
}

__global__ __launch_bounds__(256) void copy_k(const v4u* src, v4u* dst, int64_t n) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(gridDim.x) * 256)
    dst[i] = __builtin_nontemporal_load(src + i);
}

int main(int argc, char** argv) {
  const int V = argc > 1 ? atoi(argv[1]) : 5;
  const int64_t HW = argc > 3 ? static_cast<int64_t>(atoi(argv[2])) * atoi(argv[3]) : 3840LL * 2160;
  if (HW % (4 * kChunk) != 0 || HW * 3 / 2 >= (1LL << 31)) {
    fprintf(stderr, "H*W must be a multiple of %d\n", 4 * kChunk);
    return 2;
  }
  const int64_t vs = kPlanesStack * HW;
  uint8_t *st, *rec, *hot, *dst;
  const int64_t copy_bytes = kNpl * HW * V / 2;  // read + write = the pattern's 24 planes of bytes
  if (hipMalloc(&st, vs * V) != hipSuccess || hipMalloc(&rec, HW * 3 / 2 * V + 64) != hipSuccess ||
      hipMalloc(&dst, copy_bytes) != hipSuccess)
    return 1;
  (void)hipMemset(st, 7, vs * V);
  (void)hipMemset(rec, 3, HW * 3 / 2 * V + 64);
  int n_cu = 256;
  (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
  const int gx = (3 * n_cu + V - 1) / V;
  if (hipMalloc(&hot, static_cast<int64_t>(gx) * V * 6144) != hipSuccess) return 1;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  const int ngroups = static_cast<int>(HW / (4 * kChunk));
  for (int mode = 0; mode <= 22; ++mode) {
    float best = 1e30f, sum = 0.f;
    for (int r = 0; r < 23; ++r) {
      (void)hipEventRecord(a, 0);
      const dim3 g(gx, V), blk(256);
      switch (mode) {
        case 0: hipLaunchKernelGGL(mix_k<0>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 1: hipLaunchKernelGGL(mix_k<1>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 2: hipLaunchKernelGGL(mix_k<2>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 3: hipLaunchKernelGGL(mix_k<3>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 4: hipLaunchKernelGGL(mix_k<4>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 5: hipLaunchKernelGGL(mix_k<5>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 6: hipLaunchKernelGGL(mix_k<6>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 7: hipLaunchKernelGGL(mix_k<7>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 9: hipLaunchKernelGGL(mix_k<9>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 10: hipLaunchKernelGGL(mix_k<10>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 11: hipLaunchKernelGGL(mix_k<11>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 12: hipLaunchKernelGGL(mix_k<12>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 13: hipLaunchKernelGGL(mix_k<13>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 14: hipLaunchKernelGGL(mix_k<14>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 15: hipLaunchKernelGGL(mix_k<15>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 16: hipLaunchKernelGGL(mix_k<16>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 17: hipLaunchKernelGGL(mix_k<17>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 18: hipLaunchKernelGGL(mix_k<18>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 19: hipLaunchKernelGGL(mix_k<19>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 20: hipLaunchKernelGGL(mix_k<20>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 21: hipLaunchKernelGGL(mix_k<21>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        case 22: hipLaunchKernelGGL(mix_k<22>, g, blk, 0, 0, st, HW, vs, ngroups, rec, hot); break;
        default:
          hipLaunchKernelGGL(copy_k, dim3(4 * n_cu), blk, 0, 0, reinterpret_cast<const v4u*>(st), reinterpret_cast<v4u*>(dst),
                             copy_bytes / 16);
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
    const bool extra = mode != 0 && mode != 2 && mode != 8 && mode != 21 && mode != 22;
    const double bytes = mode == 8 ? 2.0 * copy_bytes : (kNpl * static_cast<double>(HW) + (extra ? 1.5 * HW : 0.0)) * V;
    const double avg = sum / 20.0;
    printf("{\"views\": %d, \"px_per_view\": %lld, \"mode\": %d, \"best_us\": %.2f, \"avg_us\": %.2f, \"GBps_avg\": %.0f}\n", V,
           static_cast<long long>(HW), mode, best * 1e3, avg * 1e3, bytes / (avg * 1e-3) / 1e9);
    fflush(stdout);
  }
  return 0;
}
