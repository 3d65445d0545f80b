// libslgpu.so -- MI355X (gfx950, CDNA4) kernels + C ABI for the structured-light
// reconstruction hot path (include/slgpu.h documents the ABI).
//
// Reference behaviour (Nuttoty/Structured_Light_for_3D_Model_Replication):
//   mask           server/sl_system.py:519-535  (fixed variant: multi_point_cloud_process.py:36-38)
//   Gray decode    server/sl_system.py:544-577  (bit b of the sequence -> code bit n-1-b,
//                  strict p > i, shared running file index, prefix-xor Gray -> binary)
//   triangulation  server/sl_system.py:584-653  (np.where order, clip to Wp-1,
//                  |n.r| > 1e-6, t = -(n.Oc + d)/(n.r), P = Oc + r t, BGR colour)
//
// Kernels (one HIP stream, no host synchronisation between them):
//   k_stats  : (adaptive mask) 256-bin histogram of the black plane + max(white -
//              black) per view; the last block of each view turns them into the
//              float32 np.percentile(black, 95) recipe and integer thresholds.
//   k_decode : one 4096-pixel tile per workgroup.  Streams the uint8 stack once
//              with 16-byte buffer loads, forms the Gray bits with a byte-SWAR
//              compare, Gray->binary in registers, applies the mask, writes the
//              maps, and decides point/no-point per pixel (f32 with an exact
//              error bound, f64 when undecided); per-pixel 2-byte records and a
//              point count per tile.
//   k_scan   : exclusive scan of the tile counts -> tile and view offsets.
//   k_cloud  : ray/plane intersection in f64 (reference operation order, no
//              contraction) for the marked pixels, written at tile offset +
//              wave-ballot rank: the reference's np.where order, coalesced.
//
// Everything in this file is compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <initializer_list>
#include <string>
#include <vector>

#include "slgpu.h"

#pragma clang fp contract(off)

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kPx = 16;                  // pixels per lane
constexpr int kTile = kThreads * kPx;    // pixels per workgroup tile
#ifndef SLGPU_RING
#define SLGPU_RING 16
#endif
constexpr int kRing = SLGPU_RING;        // pattern planes in flight per lane

// k_decode mode bits
constexpr int M_MAPS = 1;      // k_decode: write col/row/mask maps
constexpr int M_CODES = 2;     // k_decode: point decision, records + tile counts for k_cloud
constexpr int M_XYZ64 = 4;     // f64 xyz output (else f32)
constexpr int M_FROMMAPS = 8;  // k_decode: input is a caller's (col_map, mask) instead of the stack
constexpr int M_NC = 16;       // rays from a device Nc table instead of pinhole K
constexpr int M_ROWS = 32;     // decode the row sequence

constexpr int kStatBlocks = 256;  // k_stats blocks per view (max)
constexpr int kReps = 16;         // histogram replicas per view
constexpr int kSlot = 272;        // u32 per replica: 256 bins + max + pad (1088 B)

struct ViewStats {
  unsigned done;        // k_stats blocks finished for this view
  int thr_white;        // mask: white > thr_white
  int thr_contrast;     //       white - black > thr_contrast
  float noise_floor;    // np.percentile(black, 95) (float32)
  float dynamic_range;  // max(white - black) (float32)
  unsigned pad[11];
};
static_assert(sizeof(ViewStats) % 64 == 0, "ViewStats keeps 64-B alignment");

struct Header {
  unsigned error;  // sticky device-side failure (reported by sl_sync as SL_ETIMEOUT)
  unsigned pad[15];
};

struct Params {
  const uint8_t* stack;
  int64_t stack_vs;
  int view_bytes;  // n_img * H * W (< 2^31): buffer-descriptor range of one view's stack
  const uint8_t* tex;
  int64_t tex_vs;
  const int32_t* in_col;
  const uint8_t* in_mask;
  int64_t HW;
  int H, W;
  int n_views, tiles_per_view;
  int nc, nr, kc, kr;  // code bits and available bit planes (pairs)
  int mask_mode;
  int mode;
  int dbg;  // measurement-only ablations (SLGPU_DEBUG): 1 = tile from blockIdx, 2 = no look-back,
            // 4 = no k_cloud work after the ranks, 8 = no point/no-point
            // decision, 16 = k_cloud stores without point math, 32 = f32 stand-in
  int Wp;
  const double4* planes;
  const float4* planes32;  // f32 copies for the point/no-point pre-decision
  const double* xn;
  const double* yn;
  const float* xn32;
  const float* yn32;
  const double* nc_rays;
  double o0, o1, o2;
  const double* poses;
  uint16_t* codes;  // [view][HW] packed records (ctx scratch)
  int32_t* col_out;
  int32_t* row_out;
  uint8_t* mask_out;
  void* xyz;
  uint8_t* bgr;
  int64_t* view_offsets;
  ViewStats* stats;
  unsigned* part;  // k_stats histogram replicas [view][kReps][kSlot]
  int* tile_counts;          // k_decode -> k_scan
  long long* tile_offsets;   // k_scan -> k_cloud
  Header* hdr;
};

// ---------------------------------------------------------------- helpers ----

__device__ __forceinline__ uint4 ld16(const uint8_t* p, int n, bool vec) {
  if (vec) return *reinterpret_cast<const uint4*>(p);
  uint32_t w[4] = {0u, 0u, 0u, 0u};
#pragma unroll
  for (int i = 0; i < 16; ++i)
    if (i < n) w[i >> 2] |= static_cast<uint32_t>(p[i]) << (8 * (i & 3));
  return make_uint4(w[0], w[1], w[2], w[3]);
}

__device__ __forceinline__ uint32_t word(const uint4& q, int i) {
  return i == 0 ? q.x : i == 1 ? q.y : i == 2 ? q.z : q.w;
}

__device__ __forceinline__ uint32_t byte_of(const uint4& q, int i) {
  return (word(q, i >> 2) >> (8 * (i & 3))) & 0xffu;
}

// Per-byte unsigned (a > b) for 4 packed pixels: result bit 8k+7 set iff byte k
// of a is greater.  No carries cross bytes: (a|0x80) - ((b&0x7f)+1) stays in
// [0, 254] per byte and its bit 7 is (a&0x7f) > (b&0x7f).  Ties give 0, as the
// reference's strict `img_p > img_i` (sl_system.py:561).
__device__ __forceinline__ uint32_t gt_msb(uint32_t a, uint32_t b) {
  const uint32_t H = 0x80808080u;
  const uint32_t low = (a | H) - ((b & ~H) + 0x01010101u);
  return ((a & ~b) | (~(a ^ b) & low)) & H;
}

// Gray -> binary, the prefix xor that sl_system.py:567-570 iterates to a fixed
// point (codes are < 2^16).
__device__ __forceinline__ uint32_t gray_to_binary(uint32_t g) {
  g ^= g >> 1;
  g ^= g >> 2;
  g ^= g >> 4;
  g ^= g >> 8;
  return g;
}

// --------------------------------------------------------------- k_stats ----
// grid (bx <= kStatBlocks, n_views).  Builds, per view, the 256-bin histogram
// of the black plane and max(white - black):
//   * per-wave LDS histograms, then no-return device atomics into one of
//     kReps replicas of the view's histogram (blockIdx % kReps), so no more
//     than bx/kReps blocks ever add to one address;
//   * every wave drains its atomics (vmcnt(0)), then one lane adds to the
//     view's arrival counter; the block whose add is last reads (and zeroes)
//     the replicas with returning atomics and evaluates numpy's float32
//     percentile recipe.  The replicas are left zeroed for the next call.
__global__ __launch_bounds__(kThreads) void k_stats(Params p, int vec) {
  const int tid = threadIdx.x;
  const int view = blockIdx.y;

  __shared__ unsigned sh[kWaves][256];
  __shared__ unsigned cdf[256];
  __shared__ int s_max[kWaves];
  __shared__ long long s_k[2];
  __shared__ int s_v[2];
  __shared__ float s_gamma;
  __shared__ int s_last;
  const int wid = tid >> 6;
  for (int i = tid; i < kWaves * 256; i += kThreads) (&sh[0][0])[i] = 0u;
  __syncthreads();

  const uint8_t* vb = p.stack + view * p.stack_vs;
  int mx = -1024;
  // kBatch chunks per iteration: all their loads are issued before any is used
  constexpr int kBatch = 4;
  for (int64_t c0 = blockIdx.x; c0 < p.tiles_per_view; c0 += kBatch * gridDim.x) {
    uint4 w[kBatch], b[kBatch];
    int n[kBatch];
#pragma unroll
    for (int i = 0; i < kBatch; ++i) {
      const int64_t px0 = (c0 + static_cast<int64_t>(i) * gridDim.x) * kTile + static_cast<int64_t>(tid) * kPx;
      n[i] = static_cast<int>(min<int64_t>(max<int64_t>(p.HW - px0, 0), kPx));
      const int64_t pl = n[i] > 0 ? px0 : 0;
      w[i] = ld16(vb + pl, n[i], vec);
      b[i] = ld16(vb + p.HW + pl, n[i], vec);
    }
#pragma unroll
    for (int i = 0; i < kBatch; ++i) {
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        if (k < n[i]) {
          const int bk = static_cast<int>(byte_of(b[i], k));
          const int wk = static_cast<int>(byte_of(w[i], k));
          atomicAdd(&sh[wid][bk], 1u);
          mx = max(mx, wk - bk);
        }
      }
    }
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) mx = max(mx, __shfl_xor(mx, d, 64));
  if ((tid & 63) == 0) s_max[wid] = mx;
  __syncthreads();
  unsigned* rep = p.part + (static_cast<int64_t>(view) * kReps + blockIdx.x % kReps) * kSlot;
  {
    const unsigned cnt = sh[0][tid] + sh[1][tid] + sh[2][tid] + sh[3][tid];
    if (cnt) atomicAdd(rep + tid, cnt);
  }
  if (tid == 0) {
    int m = s_max[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) m = max(m, s_max[w]);
    if (m > -1024) atomicMax(rep + 256, static_cast<unsigned>(m + 1024));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (tid == 0) {
    const unsigned prev = __hip_atomic_fetch_add(&p.stats[view].done, 1u, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT);
    s_last = (prev == gridDim.x - 1);
  }
  __syncthreads();
  if (!s_last) return;

  // ---- last block of this view: read + zero the replicas, thresholds ----
  unsigned* reps = p.part + static_cast<int64_t>(view) * kReps * kSlot;
  unsigned h = 0u;
  {
    unsigned v[kReps];
#pragma unroll
    for (int r = 0; r < kReps; ++r) v[r] = atomicExch(reps + r * kSlot + tid, 0u);
#pragma unroll
    for (int r = 0; r < kReps; ++r) h += v[r];
  }
  int m = -1024;
  if (tid < kReps) {
    const unsigned mv = atomicExch(reps + tid * kSlot + 256, 0u);
    if (mv) m = static_cast<int>(mv) - 1024;
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) m = max(m, __shfl_xor(m, d, 64));
  cdf[tid] = h;
  if ((tid & 63) == 0) s_max[wid] = m;
  if (tid == 0) __hip_atomic_store(&p.stats[view].done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __syncthreads();
  for (int d = 1; d < 256; d <<= 1) {  // inclusive scan -> cdf
    const unsigned t = tid >= d ? cdf[tid - d] : 0u;
    __syncthreads();
    cdf[tid] += t;
    __syncthreads();
  }
  if (tid == 0) {
    // np.percentile(black_f32, 95): q = f32(95)/f32(100); virtual index
    // (n-1)*q in float32; neighbours floor / floor+1, both clamped to n-1 when
    // the index is >= n-1 (numpy/lib/_function_base_impl.py _get_indexes);
    // gamma = index - floor (exact in float32).
    const long long n = p.HW;
    const float q = 95.0f / 100.0f;
    const float fn1 = static_cast<float>(n - 1);
    const float vi = fn1 * q;
    long long kp, kn;
    float gamma;
    if (vi >= fn1) {
      kp = kn = n - 1;
      gamma = 0.0f;
    } else {
      const float pf = floorf(vi);
      kp = static_cast<long long>(pf);
      kn = static_cast<long long>(pf + 1.0f);
      gamma = vi - pf;
    }
    s_k[0] = kp;
    s_k[1] = kn;
    s_gamma = gamma;
  }
  __syncthreads();
  {
    const unsigned lo = tid ? cdf[tid - 1] : 0u;
    const unsigned hi = cdf[tid];
    if (static_cast<long long>(lo) <= s_k[0] && s_k[0] < static_cast<long long>(hi)) s_v[0] = tid;
    if (static_cast<long long>(lo) <= s_k[1] && s_k[1] < static_cast<long long>(hi)) s_v[1] = tid;
  }
  __syncthreads();
  if (tid == 0) {
    const float gamma = s_gamma;
    const float a = static_cast<float>(s_v[0]);
    const float b = static_cast<float>(s_v[1]);
    // numpy _lerp: a + (b-a)*t, replaced by b - (b-a)*(1-t) where t >= 0.5
    const float diff = b - a;
    float nf = a + diff * gamma;
    if (gamma >= 0.5f) nf = b - diff * (1.0f - gamma);
    int mc = s_max[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) mc = max(mc, s_max[w]);
    const float dr = static_cast<float>(mc);
    // white and contrast are integers: x > t  <=>  x > floor(t)
    const float tw = nf * 1.5f;
    const float tc = dr * 0.05f;
    p.stats[view].noise_floor = nf;
    p.stats[view].dynamic_range = dr;
    p.stats[view].thr_white = static_cast<int>(floorf(tw));
    p.stats[view].thr_contrast = static_cast<int>(floorf(tc));
  }
}

// -------------------------------------------------------------- k_decode ----

// Advance pixel coordinates (u, v) by 64 pixels.  On the vector path W >= 64,
// so at most one row wrap: branch-free selects.  Otherwise loop.
__device__ __forceinline__ void step64(int& u, int& v, int W, int H, bool vec) {
  u += 64;
  if (vec) {
    const bool wrap = u >= W;
    u -= wrap ? W : 0;
    v = min(v + (wrap ? 1 : 0), H - 1);
  } else {
    while (u >= W) {
      u -= W;
      v = min(v + 1, H - 1);
    }
  }
}

// ------------------------------------------------------------------ layout ----
// A workgroup (4 waves) owns a tile of kTile = 4096 pixels; wave w owns the
// tile's pixels [w*1024, (w+1)*1024).
//   streaming layout  : lane l holds 16 contiguous pixels -> 16-byte loads and
//                       stores, fully coalesced;
//   interleaved layout: in step k lane l holds pixel k*64 + l -> coalesced
//                       table/plane gathers and per-pixel stores.
// Per-wave LDS rows transpose one layout into the other.
//
// Pipeline (one stream): k_stats -> k_decode -> k_scan -> k_cloud.
//   k_decode : Gray decode + mask + point/no-point decision; per-pixel 2-byte
//              records and one point count per tile;
//   k_scan   : exclusive scan of the tile counts (tile and view offsets);
//   k_cloud  : exact f64 points written at their final, np.where-ordered
//              positions.  No inter-workgroup waits anywhere.
constexpr int kWavePx = 64 * kPx;

// Is |n.r| > 1e-6 (sl_system.py:642) for the pixel at (u, v) / ray index q
// whose clipped column code is c?  Decided in f32 with a rigorous error bound
// B: the f32 rounding of the inputs, of the ray and of the dot product stay
// below 2^-21 of S = sum|n_i r_i|, and B uses 2^-18.  Pixels within B of the
// threshold are decided by the exact f64 reference arithmetic.
__device__ __forceinline__ bool has_point(const Params& p, int mode, int c, int u, int v, int64_t q) {
  const float4 pf = p.planes32[c];
  float x, y, z, inv;
  if (mode & M_NC) {
    x = static_cast<float>(p.nc_rays[q]);
    y = static_cast<float>(p.nc_rays[p.HW + q]);
    z = static_cast<float>(p.nc_rays[2 * p.HW + q]);
    inv = 1.0f;
  } else {
    x = p.xn32[u];
    y = p.yn32[v];
    z = 1.0f;
    inv = __frsqrt_rn(x * x + y * y + 1.0f);
  }
  const float a = fabsf((pf.x * x + pf.y * y + pf.z * z) * inv);
  const float S = (fabsf(pf.x * x) + fabsf(pf.y * y) + fabsf(pf.z * z)) * inv;
  const float B = S * 3.814697265625e-06f;  // 2^-18
  if (a > 1e-6f + B) return true;
  if (a < 1e-6f - B) return false;
  double r0, r1, r2;
  if (mode & M_NC) {
    r0 = p.nc_rays[q];
    r1 = p.nc_rays[p.HW + q];
    r2 = p.nc_rays[2 * p.HW + q];
  } else {
    const double xd = p.xn[u], yd = p.yn[v];
    const double nrm = sqrt((xd * xd + yd * yd) + 1.0);
    r0 = xd / nrm;
    r1 = yd / nrm;
    r2 = 1.0 / nrm;
  }
  const double4 pl = p.planes[c];
  return fabs((pl.x * r0 + pl.y * r1) + pl.z * r2) > 1e-6;
}

// ================================================================ k_decode ====
// gray_decode (sl_system.py:519-577): mask, column and row code of every
// pixel, streaming the uint8 stack once (M_FROMMAPS: a caller's col_map + mask
// instead).  Outputs by mode bit:
//   M_MAPS  col/row int32 + mask u8 maps, full frame (what gray_decode returns);
//   M_CODES record16 = min(col, Wp-1) | point << 15 per pixel (np.clip,
//           sl_system.py:626; point = mask & |n.r| > 1e-6) and the tile's
//           point count, for k_scan / k_cloud.
template <int KC, int KR, int MODE, int VEC>
__global__ __launch_bounds__(kThreads, 2) void k_decode(Params p) {
  constexpr bool kStatic = KC >= 0;
  const int mode = MODE >= 0 ? MODE : p.mode;
  const int kc = KC >= 0 ? KC : p.kc;
  const int kr = KR >= 0 ? KR : p.kr;
  const int nc = p.nc, nr = p.nr;
  const bool vload = VEC > 0;

  __shared__ uint32_t s_code[kWaves][kWavePx];  // col | row << 16
  __shared__ uint8_t s_mask[kWaves][kWavePx];
  __shared__ int s_wsum[kWaves];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int64_t HW = p.HW;
  const int view = static_cast<int>(blockIdx.x / p.tiles_per_view);
  const int64_t lt = blockIdx.x - static_cast<int64_t>(view) * p.tiles_per_view;

  // ======================= A) streaming layout =======================
  {
    const int64_t px0 = lt * kTile + static_cast<int64_t>(tid) * kPx;
    const int n_px = static_cast<int>(min<int64_t>(max<int64_t>(HW - px0, 0), kPx));
    const int64_t px_ld = n_px > 0 ? px0 : 0;  // keep loads unconditional and in bounds
    uint32_t* lc = &s_code[wid][lane * kPx];
    uint8_t* lm = &s_mask[wid][lane * kPx];
    if (mode & M_FROMMAPS) {
      // reconstruct_point_cloud's inputs: col_map (clipped, sl_system.py:626) and mask
      const int64_t o = view * HW + px_ld;
      uint32_t col[kPx];
      uint32_t mw[4] = {0u, 0u, 0u, 0u};
      if (vload) {
        const int4* cm = reinterpret_cast<const int4*>(p.in_col + o);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const int4 v = cm[i];
          col[4 * i] = v.x;
          col[4 * i + 1] = v.y;
          col[4 * i + 2] = v.z;
          col[4 * i + 3] = v.w;
        }
        const uint4 mq = *reinterpret_cast<const uint4*>(p.in_mask + o);
#pragma unroll
        for (int k = 0; k < kPx; ++k) mw[k >> 2] |= (byte_of(mq, k) != 0u && k < n_px) ? (1u << (8 * (k & 3))) : 0u;
      } else {
#pragma unroll
        for (int k = 0; k < kPx; ++k) {
          col[k] = k < n_px ? static_cast<uint32_t>(p.in_col[o + k]) : 0u;
          mw[k >> 2] |= (k < n_px && p.in_mask[o + k] != 0) ? (1u << (8 * (k & 3))) : 0u;
        }
      }
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        uint32_t cw[4];
#pragma unroll
        for (int e = 0; e < 4; ++e)
          cw[e] = static_cast<uint32_t>(min(max(static_cast<int>(col[4 * w + e]), 0), p.Wp - 1));
        *reinterpret_cast<uint4*>(lc + 4 * w) = make_uint4(cw[0], cw[1], cw[2], cw[3]);
        *reinterpret_cast<uint32_t*>(lm + 4 * w) = mw[w];
      }
    } else {
      // Plane loads: on the vector path a buffer descriptor of the view's
      // stack (SGPRs) + the lane's 32-bit pixel offset + the plane offset in an SGPR.
      const uint8_t* vbase = p.stack + view * p.stack_vs;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(vbase), 0, p.view_bytes, 0x00020000);
      const int voff = static_cast<int>(px_ld);
      auto ldp = [&](int plane) -> uint4 {
        if (vload) {
          const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, plane * static_cast<int>(HW), 0);
          return make_uint4(v[0], v[1], v[2], v[3]);
        }
        return ld16(vbase + px_ld + static_cast<int64_t>(plane) * HW, n_px, false);
      };
      const uint4 wq = ldp(0);
      const uint4 bq = ldp(1);
      // ---- Gray bit planes: (pattern, inverse) pairs, columns then rows ----
      const int krr = (mode & M_ROWS) ? kr : 0;
      const int npl = 2 * (kc + krr);
      uint32_t cA[4] = {0, 0, 0, 0}, cB[4] = {0, 0, 0, 0};
      uint32_t rA[4] = {0, 0, 0, 0}, rB[4] = {0, 0, 0, 0};
      // Fold one (pattern, inverse) pair into per-byte-lane accumulators:
      // acc = (acc << 1) | bit holds at most 8 bits per byte lane, so no carry
      // crosses into the neighbouring pixel; codes of up to 16 bits use A then B.
      auto consume = [&](const uint4& P, const uint4& I, int pair) {
        uint32_t m[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) m[w] = gt_msb(word(P, w), word(I, w)) >> 7;
        if (pair < kc) {
          if (pair < 8) {
#pragma unroll
            for (int w = 0; w < 4; ++w) cA[w] = (cA[w] << 1) | m[w];
          } else {
#pragma unroll
            for (int w = 0; w < 4; ++w) cB[w] = (cB[w] << 1) | m[w];
          }
        } else if (pair - kc < 8) {
#pragma unroll
          for (int w = 0; w < 4; ++w) rA[w] = (rA[w] << 1) | m[w];
        } else {
#pragma unroll
          for (int w = 0; w < 4; ++w) rB[w] = (rB[w] << 1) | m[w];
        }
      };
      if (kStatic) {
        // fully unrolled: every plane load issues up front (the widest
        // memory-level parallelism a wave can have)
#pragma unroll
        for (int pr = 0; pr < KC + KR; ++pr)
          if (pr < kc + krr) consume(ldp(2 + 2 * pr), ldp(3 + 2 * pr), pr);
      } else {
        uint4 ring[kRing];
#pragma unroll
        for (int j = 0; j < kRing; ++j)
          if (j < npl) ring[j] = ldp(2 + j);
        for (int base = 0; base < npl; base += kRing) {
#pragma unroll
          for (int j = 0; j < kRing; j += 2) {
            const int pl = base + j;
            if (pl < npl) {
              const uint4 P = ring[j];
              const uint4 I = ring[j + 1];
              if (pl + kRing < npl) {
                ring[j] = ldp(2 + pl + kRing);
                ring[j + 1] = ldp(3 + pl + kRing);
              }
              consume(P, I, pl >> 1);
            }
          }
        }
      }
      // ---- mask + Gray -> binary ----
      int thr_w, thr_c;
      if (p.mask_mode == SL_MASK_FIXED) {
        thr_w = 40;
        thr_c = 10;
      } else {
        thr_w = p.stats[view].thr_white;
        thr_c = p.stats[view].thr_contrast;
      }
      const int cBn = kc > 8 ? kc - 8 : 0;
      const int rBn = krr > 8 ? krr - 8 : 0;
      const int cSh = nc - kc;
      const int rSh = nr - krr;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        uint32_t cw[4];
        uint32_t mw = 0u;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int k = 4 * w + e, sft = 8 * e;
          const uint32_t gc = (((cA[w] >> sft) & 0xffu) << cBn) | ((cB[w] >> sft) & 0xffu);
          const uint32_t gr = (((rA[w] >> sft) & 0xffu) << rBn) | ((rB[w] >> sft) & 0xffu);
          const uint32_t col = gray_to_binary(gc << cSh);
          const uint32_t row = (mode & M_ROWS) ? gray_to_binary(gr << rSh) : 0u;
          const int wv = static_cast<int>(byte_of(wq, k));
          const int bv = static_cast<int>(byte_of(bq, k));
          const uint32_t ok = ((k < n_px) && (wv > thr_w) && (wv - bv > thr_c)) ? 1u : 0u;
          cw[e] = col | (row << 16);
          mw |= ok << sft;
        }
        *reinterpret_cast<uint4*>(lc + 4 * w) = make_uint4(cw[0], cw[1], cw[2], cw[3]);
        *reinterpret_cast<uint32_t*>(lm + 4 * w) = mw;
      }
    }
  }
  __syncthreads();

  // ======================= B) interleaved layout =======================
  // Program order: every gather of the point decision, then the map stores,
  // then the decisions and record stores -- vmcnt counts loads and stores in
  // one in-order queue, so no load may wait behind a store.
  const int64_t wpx = lt * kTile + static_cast<int64_t>(wid) * kWavePx + lane;  // step-0 pixel
  const int64_t o = view * HW;
  const bool codes = (mode & M_CODES) != 0;
  const int W = p.W;
  float4 pf[kPx];
  float xs[kPx], ys[kPx];
  uint32_t cc[kPx];
  if (codes) {
    int v = static_cast<int>(min<int64_t>(wpx, HW - 1) / W);
    int u = static_cast<int>(min<int64_t>(wpx, HW - 1) - static_cast<int64_t>(v) * W);
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      cc[k] = min(s_code[wid][64 * k + lane] & 0xffffu, static_cast<uint32_t>(p.Wp - 1)) | (u << 16);
      pf[k] = p.planes32[cc[k] & 0xffffu];
      if (mode & M_NC) {
        const int64_t q = min<int64_t>(wpx + 64 * k, HW - 1);
        xs[k] = static_cast<float>(p.nc_rays[q]);
        ys[k] = static_cast<float>(p.nc_rays[HW + q]);
      } else {
        xs[k] = p.xn32[u];
        ys[k] = p.yn32[v];
      }
      step64(u, v, W, p.H, vload);
    }
  }
  if (mode & M_MAPS) {
#pragma unroll 4
    for (int k = 0; k < kPx; ++k) {
      const int64_t q = wpx + 64 * k;
      if (q < HW) {
        const uint32_t cw = s_code[wid][64 * k + lane];
        p.col_out[o + q] = static_cast<int32_t>(cw & 0xffffu);
        p.row_out[o + q] = static_cast<int32_t>(cw >> 16);
        p.mask_out[o + q] = s_mask[wid][64 * k + lane];
      }
    }
  }
  if (!codes) return;
  int total_w = 0;
#pragma unroll
  for (int k = 0; k < kPx; ++k) {
    const int64_t q = wpx + 64 * k;
    const int c = static_cast<int>(cc[k] & 0xffffu);
    bool pt = false;
    if (s_mask[wid][64 * k + lane]) {
      if (p.dbg & 8) {
        pt = true;
      } else {
        // |n.r| > 1e-6 (sl_system.py:642) decided in f32 with a rigorous
        // error bound B: the f32 rounding of the inputs, of the ray and of the
        // dot product stay below 2^-21 of S = sum|n_i r_i|, and B uses 2^-18.
        // Pixels within B of the threshold take the exact f64 arithmetic.
        const float4 f = pf[k];
        float zf, inv;
        if (mode & M_NC) {
          zf = static_cast<float>(p.nc_rays[2 * HW + min<int64_t>(q, HW - 1)]);
          inv = 1.0f;
        } else {
          zf = 1.0f;
          inv = __frsqrt_rn(xs[k] * xs[k] + ys[k] * ys[k] + 1.0f);
        }
        const float a = fabsf((f.x * xs[k] + f.y * ys[k] + f.z * zf) * inv);
        const float S = (fabsf(f.x * xs[k]) + fabsf(f.y * ys[k]) + fabsf(f.z * zf)) * inv;
        const float B = S * 3.814697265625e-06f;  // 2^-18
        if (a > 1e-6f + B) {
          pt = true;
        } else if (a >= 1e-6f - B) {
          const int u = static_cast<int>(cc[k] >> 16);
          const int v = static_cast<int>(min<int64_t>(q, HW - 1) / W);
          pt = has_point(p, mode, c, u, v, min<int64_t>(q, HW - 1));
        }
      }
    }
    total_w += __popcll(__ballot(pt));
    if (q < HW) p.codes[o + q] = static_cast<uint16_t>(c | (pt ? 0x8000 : 0));
  }
  if (lane == 0) s_wsum[wid] = total_w;
  __syncthreads();
  if (tid == 0) {
    int t = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) t += s_wsum[w];
    p.tile_counts[blockIdx.x] = t;
  }
}

// ================================================================== k_scan ====
// Exclusive scan of the per-tile point counts (tiles of all views in order):
// tile_offsets[t] = points before tile t; view_offsets[v] = points before view
// v, view_offsets[V] = total.  One workgroup of 1024 threads.
__global__ __launch_bounds__(1024) void k_scan(Params p) {
  __shared__ long long s_part[1024];
  const int tid = threadIdx.x;
  const int64_t n = static_cast<int64_t>(p.n_views) * p.tiles_per_view;
  const int64_t per = (n + 1023) / 1024;
  const int64_t lo = min<int64_t>(tid * per, n), hi = min<int64_t>(lo + per, n);
  long long s = 0;
  for (int64_t i = lo; i < hi; ++i) s += p.tile_counts[i];
  s_part[tid] = s;
  __syncthreads();
  for (int d = 1; d < 1024; d <<= 1) {  // inclusive scan of the chunk sums
    const long long t = tid >= d ? s_part[tid - d] : 0ll;
    __syncthreads();
    s_part[tid] += t;
    __syncthreads();
  }
  long long run = tid ? s_part[tid - 1] : 0ll;
  for (int64_t i = lo; i < hi; ++i) {
    if (p.view_offsets && i % p.tiles_per_view == 0) p.view_offsets[i / p.tiles_per_view] = run;
    p.tile_offsets[i] = run;
    run += p.tile_counts[i];
  }
  if (tid == 1023 && p.view_offsets) p.view_offsets[p.n_views] = s_part[1023];
}

// ================================================================= k_cloud ====
// reconstruct_point_cloud's arithmetic (sl_system.py:584-653) for the pixels
// k_decode marked: exact f64 in the reference's operation order, stored at
// tile offset + rank, i.e. in np.where order across tiles and views
// (sl_system.py:601).
template <int MODE, int VEC>
__global__ __launch_bounds__(kThreads, 2) void k_cloud(Params p) {
  const int mode = MODE >= 0 ? MODE : p.mode;
  const bool vload = VEC > 0;

  __shared__ uint16_t s_code[kWaves][kWavePx];  // record16
  __shared__ uint32_t s_aux[kWaves][kWavePx];   // B | G << 8 | R << 16
  __shared__ int s_wsum[kWaves];

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int64_t HW = p.HW;
  const int view = static_cast<int>(blockIdx.x / p.tiles_per_view);
  const int64_t lt = blockIdx.x - static_cast<int64_t>(view) * p.tiles_per_view;
  const long long tile_base = p.tile_offsets[blockIdx.x];  // issued early, used after the scan

  // ============ A) streaming layout: records + colour -> LDS rows ============
  {
    const int64_t px0 = lt * kTile + static_cast<int64_t>(tid) * kPx;
    const int n_px = static_cast<int>(min<int64_t>(max<int64_t>(HW - px0, 0), kPx));
    const int64_t px_ld = n_px > 0 ? px0 : 0;
    const uint16_t* src = p.codes + view * HW + px_ld;
    uint32_t d[kPx / 2];
    if (vload) {
      const uint4 a = reinterpret_cast<const uint4*>(src)[0];
      const uint4 b = reinterpret_cast<const uint4*>(src)[1];
      d[0] = a.x; d[1] = a.y; d[2] = a.z; d[3] = a.w;
      d[4] = b.x; d[5] = b.y; d[6] = b.z; d[7] = b.w;
    } else {
#pragma unroll
      for (int i = 0; i < kPx / 2; ++i) {
        const uint32_t lo = (2 * i < n_px) ? src[2 * i] : 0u;
        const uint32_t hi = (2 * i + 1 < n_px) ? src[2 * i + 1] : 0u;
        d[i] = lo | (hi << 16);
      }
    }
    // colour: BGR texture, or the white plane replicated (the colour imread of
    // a single-channel file 0, sl_system.py:580)
    uint4 tq[3];
    if (p.tex != nullptr) {
      const uint8_t* t = p.tex + view * p.tex_vs + 3 * px_ld;
      tq[0] = ld16(t, 3 * n_px, vload);
      tq[1] = ld16(t + 16, 3 * n_px - 16, vload);
      tq[2] = ld16(t + 32, 3 * n_px - 32, vload);
    } else {
      const uint4 wq = ld16(p.stack + view * p.stack_vs + px_ld, n_px, vload);
      uint32_t t[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) t[i] = 0u;
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        const uint32_t wv = byte_of(wq, k);
#pragma unroll
        for (int c = 0; c < 3; ++c) t[(3 * k + c) >> 2] |= wv << (8 * ((3 * k + c) & 3));
      }
      tq[0] = make_uint4(t[0], t[1], t[2], t[3]);
      tq[1] = make_uint4(t[4], t[5], t[6], t[7]);
      tq[2] = make_uint4(t[8], t[9], t[10], t[11]);
    }
    uint16_t* lc = &s_code[wid][lane * kPx];
    uint32_t* la = &s_aux[wid][lane * kPx];
    if (n_px < kPx) {  // tail pixels are not points
#pragma unroll
      for (int k = 0; k < kPx; ++k)
        if (k >= n_px) d[k >> 1] &= ~(0xffffu << (16 * (k & 1)));
    }
    *reinterpret_cast<uint4*>(lc) = make_uint4(d[0], d[1], d[2], d[3]);
    *reinterpret_cast<uint4*>(lc + 8) = make_uint4(d[4], d[5], d[6], d[7]);
#pragma unroll
    for (int w = 0; w < 4; ++w) {
      uint32_t aw[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = 4 * w + e, b = 3 * k;
        aw[e] = byte_of(tq[b >> 4], b & 15) | (byte_of(tq[(b + 1) >> 4], (b + 1) & 15) << 8) |
                (byte_of(tq[(b + 2) >> 4], (b + 2) & 15) << 16);
      }
      *reinterpret_cast<uint4*>(la + 4 * w) = make_uint4(aw[0], aw[1], aw[2], aw[3]);
    }
  }
  __syncthreads();

  // ============ B) interleaved layout: pixel k*64 + lane of the wave ============
  // ranks: bit k of `mine` = this lane's pixel is a point; rel[k] = its rank
  // among the wave's points of steps <= k; bit k of `steps` = step k has one.
  unsigned mine = 0u, steps = 0u;
  uint32_t rel[kPx];
  int total_w = 0;
#pragma unroll
  for (int k = 0; k < kPx; ++k) {
    const bool pt = (s_code[wid][64 * k + lane] >> 15) & 1u;
    const unsigned long long m = __ballot(pt);
    rel[k] = static_cast<uint32_t>(total_w) +
             __builtin_amdgcn_mbcnt_hi(static_cast<uint32_t>(m >> 32),
                                       __builtin_amdgcn_mbcnt_lo(static_cast<uint32_t>(m), 0u));
    mine |= pt ? (1u << k) : 0u;
    steps |= m ? (1u << k) : 0u;
    total_w += __popcll(m);
  }
  if (lane == 0) s_wsum[wid] = total_w;
  __syncthreads();
  long long base = tile_base;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) base += (w < wid) ? s_wsum[w] : 0;

  // r = (x, y, 1) / sqrt((x*x + y*y) + 1) (sl_system.py:614-621), plane of the
  // clipped code (:624-633), den = (n0 r0 + n1 r1) + n2 r2 (:638),
  // t = -(n.Oc + d) / den (:639, :643), P = Oc + r t (:648); optional pose.
  // Groups of four steps are computed branch-free so their chains interleave,
  // and software-pipelined: the operands of group g+1 are loaded before the
  // points of group g are stored, because vmcnt counts loads and stores in
  // one in-order queue -- a load issued after a store makes its wait also
  // wait for that store.
  const int64_t wpx = lt * kTile + static_cast<int64_t>(wid) * kWavePx + lane;
  const int W = p.W;
  const double* pose = p.poses ? p.poses + 16 * view : nullptr;
  struct Ops {
    double r0[4], r1[4], r2[4];  // rays (Nc) or x, y, - (pinhole)
    double4 pl[4];
  };
  int u = static_cast<int>(min<int64_t>(wpx, HW - 1) % W);
  int v = static_cast<int>(min<int64_t>(wpx, HW - 1) / W);
  auto fetch = [&](int g, Ops& op) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const int k = g + e;
      if (mode & M_NC) {
        const int64_t q = min<int64_t>(wpx + 64 * k, HW - 1);
        op.r0[e] = p.nc_rays[q];
        op.r1[e] = p.nc_rays[HW + q];
        op.r2[e] = p.nc_rays[2 * HW + q];
      } else {
        op.r0[e] = p.xn[u];
        op.r1[e] = p.yn[v];
      }
      op.pl[e] = p.planes[s_code[wid][64 * k + lane] & 0x7fffu];
      step64(u, v, W, p.H, vload);
    }
  };
  Ops cur, nxt;
  fetch(0, cur);
#pragma unroll
  for (int g = 0; g < kPx; g += 4) {
    if (g + 4 < kPx) fetch(g + 4, nxt);
    if (((steps >> g) & 0xfu) != 0u && !(p.dbg & 4)) {
      double X[4], Y[4], Z[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (p.dbg & 16) {  // measurement only: stores without any point math
          X[e] = cur.r0[e];
          Y[e] = cur.r1[e];
          Z[e] = cur.pl[e].w;
          continue;
        }
        if (p.dbg & 32) {  // measurement only: f32 stand-in for the f64 math
          const float x = static_cast<float>(cur.r0[e]), y = static_cast<float>(cur.r1[e]);
          const float in = __frsqrt_rn(x * x + y * y + 1.0f);
          const float4 pf = make_float4(cur.pl[e].x, cur.pl[e].y, cur.pl[e].z, cur.pl[e].w);
          const float tt = -pf.w / ((pf.x * x + pf.y * y + pf.z) * in);
          X[e] = x * in * tt;
          Y[e] = y * in * tt;
          Z[e] = in * tt;
          continue;
        }
        double r0, r1, r2;
        if (mode & M_NC) {
          r0 = cur.r0[e];
          r1 = cur.r1[e];
          r2 = cur.r2[e];
        } else {
          const double x = cur.r0[e], y = cur.r1[e];
          const double nrm = sqrt((x * x + y * y) + 1.0);
          r0 = x / nrm;
          r1 = y / nrm;
          r2 = 1.0 / nrm;
        }
        const double4 pl = cur.pl[e];
        const double den = (pl.x * r0 + pl.y * r1) + pl.z * r2;
        const double num = ((pl.x * p.o0 + pl.y * p.o1) + pl.z * p.o2) + pl.w;
        const double t = -num / den;
        X[e] = p.o0 + r0 * t;
        Y[e] = p.o1 + r1 * t;
        Z[e] = p.o2 + r2 * t;
        if (pose) {
          const double X2 = ((pose[0] * X[e] + pose[1] * Y[e]) + pose[2] * Z[e]) + pose[3];
          const double Y2 = ((pose[4] * X[e] + pose[5] * Y[e]) + pose[6] * Z[e]) + pose[7];
          const double Z2 = ((pose[8] * X[e] + pose[9] * Y[e]) + pose[10] * Z[e]) + pose[11];
          X[e] = X2;
          Y[e] = Y2;
          Z[e] = Z2;
        }
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = g + e;
        if ((mine >> k) & 1u) {
          const long long o = base + rel[k];
          if (mode & M_XYZ64) {
            double* xyz = static_cast<double*>(p.xyz) + 3 * o;
            xyz[0] = X[e];
            xyz[1] = Y[e];
            xyz[2] = Z[e];
          } else {
            float* xyz = static_cast<float*>(p.xyz) + 3 * o;
            xyz[0] = static_cast<float>(X[e]);
            xyz[1] = static_cast<float>(Y[e]);
            xyz[2] = static_cast<float>(Z[e]);
          }
          const uint32_t aux = s_aux[wid][64 * k + lane];
          uint8_t* cc = p.bgr + 3 * o;
          cc[0] = static_cast<uint8_t>(aux);
          cc[1] = static_cast<uint8_t>(aux >> 8);
          cc[2] = static_cast<uint8_t>(aux >> 16);
        }
      }
    }
    cur = nxt;
  }
}

}  // namespace

// ------------------------------------------------------------------ host ----

struct sl_ctx {
  int device = 0;
  std::string err;
  // calibration
  bool has_calib = false;
  int H = 0, W = 0, Wp = 0;
  double Oc[3] = {0, 0, 0};
  double* d_planes = nullptr;
  double* d_xn = nullptr;
  double* d_yn = nullptr;
  float* d_f32 = nullptr;  // planes32 [Wp][4] | xn32 [W] | yn32 [H]
  double* d_nc = nullptr;
  // scratch
  Header* d_hdr = nullptr;
  ViewStats* d_stats = nullptr;
  int64_t cap_views = 0;
  unsigned* d_part = nullptr;
  int64_t cap_part = 0;
  int* d_tile_counts = nullptr;
  int64_t cap_tc = 0;
  long long* d_tile_offsets = nullptr;
  int64_t cap_to = 0;
  uint16_t* d_codes = nullptr;  // k_decode -> k_cloud records
  int64_t cap_codes = 0;
  int last_views = 0;
  int dbg = 0;
  // optional per-launch HIP-event timing of k_stats / k_decode / k_cloud
  std::vector<hipEvent_t> prof_ev;  // kProfEv events per launch slot
  int prof_n = 0;
};

namespace {

int fail(sl_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

#define HIP_TRY(ctx, expr)                                                          \
  do {                                                                              \
    hipError_t e_ = (expr);                                                         \
    if (e_ != hipSuccess)                                                           \
      return fail((ctx), SL_EHIP, std::string(#expr) + ": " + hipGetErrorString(e_)); \
  } while (0)

int bit_count(int n) {  // int(np.ceil(np.log2(n))) for n >= 1
  int b = 0;
  while ((1ll << b) < n) ++b;
  return b;
}

template <typename T>
int grow(sl_ctx* c, T** ptr, int64_t* cap, int64_t need) {
  if (need <= *cap) return SL_OK;
  if (*ptr) HIP_TRY(c, hipFree(*ptr));
  *ptr = nullptr;
  const int64_t n = std::max<int64_t>(need, *cap * 2);
  HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(ptr), sizeof(T) * n));
  HIP_TRY(c, hipMemset(*ptr, 0, sizeof(T) * n));
  *cap = n;
  return SL_OK;
}

int ensure_scratch(sl_ctx* c, int64_t views, int64_t tiles) {
  int r = grow(c, &c->d_stats, &c->cap_views, views);
  if (r) return r;
  r = grow(c, &c->d_part, &c->cap_part, views * kReps * kSlot);
  if (r) return r;
  r = grow(c, &c->d_tile_counts, &c->cap_tc, tiles);
  if (r) return r;
  return grow(c, &c->d_tile_offsets, &c->cap_to, tiles);
}

using KernelFn = void (*)(Params);
constexpr int kProfEv = 4;  // events per launch: before k_stats, k_decode, k_cloud, after

// k_decode specialisations for the benchmark configurations; everything else
// (other bit counts, unaligned frames) runs the generic instantiation.
KernelFn pick_decode(int kc, int kr, int mode, bool vec) {
  if (vec && !(mode & (M_NC | M_FROMMAPS))) {
    const int mr = M_MAPS | M_ROWS, mrc = M_MAPS | M_ROWS | M_CODES;
    if (mode == mrc && kc == 11 && kr == 11) return k_decode<11, 11, mrc, 1>;
    if (mode == mrc && kc == 10 && kr == 10) return k_decode<10, 10, mrc, 1>;
    if (mode == mrc && kc == 10 && kr == 0) return k_decode<10, 0, mrc, 1>;
    if (mode == mr && kc == 11 && kr == 11) return k_decode<11, 11, mr, 1>;
    if (mode == M_CODES && kc == 11) return k_decode<11, 0, M_CODES, 1>;
    if (mode == M_CODES && kc == 10) return k_decode<10, 0, M_CODES, 1>;
  }
  return vec ? k_decode<-1, -1, -1, 1> : k_decode<-1, -1, -1, 0>;
}

KernelFn pick_cloud(int mode, bool vec) {
  if (vec && mode == 0) return k_cloud<0, 1>;  // f32 xyz, pinhole rays
  return vec ? k_cloud<-1, 1> : k_cloud<-1, 0>;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Enqueue [k_stats] -> k_decode -> [k_scan -> k_cloud] on stream s.
// cloud_mode < 0: no cloud.
int launch(sl_ctx* c, Params& p, bool vec, bool do_stats, int decode_mode, int cloud_mode, hipStream_t s) {
  const int64_t tiles = static_cast<int64_t>(p.n_views) * p.tiles_per_view;
  if (tiles >= (1ll << 31)) return fail(c, SL_EINVAL, "too many pixels in one call");
  int r = ensure_scratch(c, p.n_views, tiles);
  if (r) return r;
  if (decode_mode & M_CODES) {
    r = grow(c, &c->d_codes, &c->cap_codes, static_cast<int64_t>(p.n_views) * p.HW + 16);
    if (r) return r;
  }
  p.stats = c->d_stats;
  p.part = c->d_part;
  p.tile_counts = c->d_tile_counts;
  p.tile_offsets = c->d_tile_offsets;
  p.hdr = c->d_hdr;
  p.codes = c->d_codes;
  c->last_views = p.n_views;
  hipEvent_t* ev = nullptr;
  if (!c->prof_ev.empty() && kProfEv * (c->prof_n + 1) <= static_cast<int>(c->prof_ev.size()))
    ev = &c->prof_ev[kProfEv * c->prof_n++];
  if (ev) HIP_TRY(c, hipEventRecord(ev[0], s));
  if (do_stats) {
    const int bx = static_cast<int>(std::max<int64_t>(
        1, std::min<int64_t>({static_cast<int64_t>(p.tiles_per_view), int64_t{kStatBlocks},
                              std::max<int64_t>(1, 2048 / p.n_views)})));
    int vec_flag = vec ? 1 : 0;
    void* args[] = {&p, &vec_flag};
    HIP_TRY(c, hipLaunchKernel(reinterpret_cast<const void*>(k_stats), dim3(bx, p.n_views), dim3(kThreads), args,
                               0, s));
  }
  if (ev) HIP_TRY(c, hipEventRecord(ev[1], s));
  {
    Params q = p;
    q.mode = decode_mode;
    void* args[] = {&q};
    KernelFn fn = pick_decode(q.kc, (decode_mode & M_ROWS) ? q.kr : 0, decode_mode, vec);
    HIP_TRY(c, hipLaunchKernel(reinterpret_cast<const void*>(fn), dim3(static_cast<unsigned>(tiles)),
                               dim3(kThreads), args, 0, s));
  }
  if (ev) HIP_TRY(c, hipEventRecord(ev[2], s));
  if (cloud_mode >= 0) {
    void* sargs[] = {&p};
    HIP_TRY(c, hipLaunchKernel(reinterpret_cast<const void*>(k_scan), dim3(1), dim3(1024), sargs, 0, s));
    Params q = p;
    q.mode = cloud_mode;
    void* args[] = {&q};
    KernelFn fn = pick_cloud(cloud_mode, vec);
    HIP_TRY(c, hipLaunchKernel(reinterpret_cast<const void*>(fn), dim3(static_cast<unsigned>(tiles)),
                               dim3(kThreads), args, 0, s));
  }
  if (ev) HIP_TRY(c, hipEventRecord(ev[3], s));
  return SL_OK;
}

}  // namespace

extern "C" {

int sl_abi_version(void) { return SL_ABI_VERSION; }

int sl_ctx_create(int device, sl_ctx** out) {
  if (!out) return SL_EINVAL;
  *out = nullptr;
  sl_ctx* c = new sl_ctx();
  c->device = device;
  if (const char* d = getenv("SLGPU_DEBUG")) c->dbg = atoi(d);
  hipError_t e = hipSetDevice(device);
  if (e == hipSuccess) e = hipMalloc(reinterpret_cast<void**>(&c->d_hdr), sizeof(Header));
  if (e == hipSuccess) e = hipMemset(c->d_hdr, 0, sizeof(Header));
  if (e != hipSuccess) {
    delete c;
    return SL_EHIP;
  }
  *out = c;
  return SL_OK;
}

void sl_ctx_destroy(sl_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
  for (void* ptr : {static_cast<void*>(c->d_planes), static_cast<void*>(c->d_xn), static_cast<void*>(c->d_yn),
                    static_cast<void*>(c->d_nc), static_cast<void*>(c->d_hdr), static_cast<void*>(c->d_stats),
                    static_cast<void*>(c->d_f32), static_cast<void*>(c->d_codes),
                    static_cast<void*>(c->d_part),
                    static_cast<void*>(c->d_tile_counts), static_cast<void*>(c->d_tile_offsets)})
    if (ptr) (void)hipFree(ptr);
  delete c;
}

const char* sl_ctx_last_error(const sl_ctx* c) { return c ? c->err.c_str() : "null context"; }

int sl_ctx_reserve(sl_ctx* c, int64_t max_views, int64_t max_px) {
  if (!c || max_views < 1 || max_px < 1) return fail(c, SL_EINVAL, "sl_ctx_reserve: bad sizes");
  HIP_TRY(c, hipSetDevice(c->device));
  return ensure_scratch(c, max_views, max_views * ((max_px + kTile - 1) / kTile));
}

int sl_set_calib(sl_ctx* c, int H, int W, const double* K, const double* Oc, const double* planes,
                 int Wp, const double* Nc) {
  if (!c) return SL_EINVAL;
  if (H < 1 || W < 1 || Wp < 1 || !K || !Oc || !planes)
    return fail(c, SL_EINVAL, "sl_set_calib: bad arguments");
  if (Wp > 32768) return fail(c, SL_EINVAL, "sl_set_calib: at most 32768 projector columns");
  HIP_TRY(c, hipSetDevice(c->device));
  const double fx = K[0], fy = K[4], cx = K[2], cy = K[5];
  // (x_v - cx) / fx and (y_v - cy) / fy with integer pixel coordinates
  // (sl_system.py:614-616, calibrate_final :353-358)
  std::vector<double> xn(W), yn(H);
  for (int u = 0; u < W; ++u) xn[u] = (static_cast<double>(u) - cx) / fx;
  for (int v = 0; v < H; ++v) yn[v] = (static_cast<double>(v) - cy) / fy;
  bool use_nc = false;
  const int64_t HW = static_cast<int64_t>(H) * W;
  if (Nc) {
    for (int64_t q = 0; q < HW && !use_nc; ++q) {
      const double x = xn[q % W], y = yn[q / W];
      const double nrm = sqrt((x * x + y * y) + 1.0);
      const double r[3] = {x / nrm, y / nrm, 1.0 / nrm};
      for (int k = 0; k < 3; ++k)
        if (memcmp(&r[k], &Nc[k * HW + q], sizeof(double)) != 0) use_nc = true;
    }
  }
  for (double* ptr : {c->d_planes, c->d_xn, c->d_yn, c->d_nc})
    if (ptr) HIP_TRY(c, hipFree(ptr));
  if (c->d_f32) HIP_TRY(c, hipFree(c->d_f32));
  c->d_planes = c->d_xn = c->d_yn = c->d_nc = nullptr;
  c->d_f32 = nullptr;
  HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_planes), sizeof(double) * 4 * Wp));
  HIP_TRY(c, hipMemcpy(c->d_planes, planes, sizeof(double) * 4 * Wp, hipMemcpyHostToDevice));
  HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_xn), sizeof(double) * W));
  HIP_TRY(c, hipMemcpy(c->d_xn, xn.data(), sizeof(double) * W, hipMemcpyHostToDevice));
  HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_yn), sizeof(double) * H));
  HIP_TRY(c, hipMemcpy(c->d_yn, yn.data(), sizeof(double) * H, hipMemcpyHostToDevice));
  {
    std::vector<float> f(4 * static_cast<size_t>(Wp) + W + H);
    for (int i = 0; i < 4 * Wp; ++i) f[i] = static_cast<float>(planes[i]);
    for (int u = 0; u < W; ++u) f[4 * Wp + u] = static_cast<float>(xn[u]);
    for (int v = 0; v < H; ++v) f[4 * Wp + W + v] = static_cast<float>(yn[v]);
    HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_f32), sizeof(float) * f.size()));
    HIP_TRY(c, hipMemcpy(c->d_f32, f.data(), sizeof(float) * f.size(), hipMemcpyHostToDevice));
  }
  if (use_nc) {
    HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_nc), sizeof(double) * 3 * HW));
    HIP_TRY(c, hipMemcpy(c->d_nc, Nc, sizeof(double) * 3 * HW, hipMemcpyHostToDevice));
  }
  c->Oc[0] = Oc[0];
  c->Oc[1] = Oc[1];
  c->Oc[2] = Oc[2];
  c->H = H;
  c->W = W;
  c->Wp = Wp;
  c->has_calib = true;
  return SL_OK;
}

static int common_out_checks(sl_ctx* c, int n_views, int H, int W, void* xyz, int xyz_dtype,
                             uint8_t* bgr, int64_t cap, int64_t* view_offsets) {
  if (n_views < 1 || H < 1 || W < 1) return fail(c, SL_EINVAL, "bad view count or frame size");
  if (!c->has_calib && xyz) return fail(c, SL_ENOCALIB, "sl_set_calib has not been called");
  if (xyz && (H != c->H || W != c->W))
    return fail(c, SL_ENOCALIB, "frame size differs from the calibrated camera");
  if (xyz && (!bgr || !view_offsets)) return fail(c, SL_EINVAL, "xyz_out needs bgr_out and view_offsets");
  if (xyz && (xyz_dtype != SL_XYZ_F32 && xyz_dtype != SL_XYZ_F64)) return fail(c, SL_EINVAL, "bad xyz_dtype");
  if (xyz && (!aligned16(xyz) || !aligned16(bgr))) return fail(c, SL_EINVAL, "xyz/bgr must be 16-byte aligned");
  if (xyz && cap < static_cast<int64_t>(n_views) * H * W)
    return fail(c, SL_ECAPACITY, "out_capacity < n_views*H*W");
  return SL_OK;
}

static void fill_common(sl_ctx* c, Params& p, int n_views, int H, int W) {
  memset(&p, 0, sizeof(p));
  p.HW = static_cast<int64_t>(H) * W;
  p.H = H;
  p.W = W;
  p.n_views = n_views;
  p.tiles_per_view = static_cast<int>((p.HW + kTile - 1) / kTile);
  p.Wp = c->Wp;
  p.planes = reinterpret_cast<const double4*>(c->d_planes);
  p.xn = c->d_xn;
  p.yn = c->d_yn;
  p.planes32 = reinterpret_cast<const float4*>(c->d_f32);
  p.xn32 = c->d_f32 ? c->d_f32 + 4 * c->Wp : nullptr;
  p.yn32 = c->d_f32 ? c->d_f32 + 4 * c->Wp + c->W : nullptr;
  p.nc_rays = c->d_nc;
  p.o0 = c->Oc[0];
  p.o1 = c->Oc[1];
  p.o2 = c->Oc[2];
  p.dbg = c->dbg;
}

int sl_decode_triangulate(sl_ctx* c, const uint8_t* stack, int64_t stack_vs, int n_views, int n_img,
                          int H, int W, int n_cols, int n_rows, const uint8_t* tex, int64_t tex_vs,
                          int mask_mode, const double* poses, int32_t* col_out, int32_t* row_out,
                          uint8_t* mask_out, void* xyz, int xyz_dtype, uint8_t* bgr, int64_t cap,
                          int64_t* view_offsets, void* stream) {
  if (!c) return SL_EINVAL;
  int r = common_out_checks(c, n_views, H, W, xyz, xyz_dtype, bgr, cap, view_offsets);
  if (r) return r;
  if (!stack) return fail(c, SL_EINVAL, "stack is NULL");
  if (n_cols < 1 || n_rows < 1 || n_cols > 65536 || n_rows > 65536)
    return fail(c, SL_EINVAL, "n_cols / n_rows must be in [1, 65536]");
  if (mask_mode != SL_MASK_ADAPTIVE && mask_mode != SL_MASK_FIXED) return fail(c, SL_EINVAL, "bad mask_mode");
  const bool maps = col_out || row_out || mask_out;
  if (maps && !(col_out && row_out && mask_out)) return fail(c, SL_EINVAL, "maps need col, row and mask outputs");
  if (!maps && !xyz) return fail(c, SL_EINVAL, "nothing to compute: no maps and no cloud requested");
  const int64_t HW = static_cast<int64_t>(H) * W;
  if (stack_vs < static_cast<int64_t>(n_img) * HW) return fail(c, SL_EINVAL, "stack_view_stride too small");
  if (tex && tex_vs < 3 * HW) return fail(c, SL_EINVAL, "tex_view_stride too small");
  // stack length rules of gray_decode (sl_system.py:515-516, 549-554)
  if (n_img < 4) return fail(c, SL_EINVAL, "Not enough images in folder to decode.");
  const int nc = bit_count(n_cols), nr = bit_count(n_rows);
  int idx = 2, pairs = 0;
  for (int b = 0; b < nc + nr; ++b) {
    if (idx >= n_img) break;
    if (idx + 1 >= n_img) return fail(c, SL_EINDEX, "list index out of range");
    idx += 2;
    ++pairs;
  }
  if (static_cast<int64_t>(n_img) * HW >= (1ll << 31) || 3 * HW >= (1ll << 31))
    return fail(c, SL_EINVAL, "one view's stack must be < 2 GiB");
  Params p;
  fill_common(c, p, n_views, H, W);
  p.stack = stack;
  p.stack_vs = stack_vs;
  p.view_bytes = static_cast<int>(static_cast<int64_t>(n_img) * HW);
  p.tex = tex;
  p.tex_vs = tex_vs;
  p.nc = nc;
  p.nr = nr;
  p.kc = std::min(nc, pairs);
  p.kr = pairs - p.kc;
  p.mask_mode = mask_mode;
  p.poses = poses;
  p.col_out = col_out;
  p.row_out = row_out;
  p.mask_out = mask_out;
  p.xyz = xyz;
  p.bgr = bgr;
  p.view_offsets = view_offsets;
  const int nc_bit = (xyz && c->d_nc) ? M_NC : 0;
  const int decode_mode = (maps ? (M_MAPS | M_ROWS) : 0) | (xyz ? M_CODES : 0) | nc_bit;
  const int cloud_mode = xyz ? ((xyz_dtype == SL_XYZ_F64 ? M_XYZ64 : 0) | nc_bit) : -1;
  const bool vec = (W % 16 == 0) && W >= 64 && aligned16(stack) && (stack_vs % 16 == 0) &&
                   (!tex || (aligned16(tex) && tex_vs % 16 == 0)) &&
                   (!maps || (aligned16(col_out) && aligned16(row_out) && aligned16(mask_out)));
  HIP_TRY(c, hipSetDevice(c->device));
  return launch(c, p, vec, mask_mode == SL_MASK_ADAPTIVE, decode_mode, cloud_mode, static_cast<hipStream_t>(stream));
}

int sl_triangulate_maps(sl_ctx* c, const int32_t* col_map, const uint8_t* mask, const uint8_t* tex,
                        int n_views, int H, int W, const double* poses, void* xyz, int xyz_dtype,
                        uint8_t* bgr, int64_t cap, int64_t* view_offsets, void* stream) {
  if (!c) return SL_EINVAL;
  if (!xyz) return fail(c, SL_EINVAL, "xyz_out is NULL");
  int r = common_out_checks(c, n_views, H, W, xyz, xyz_dtype, bgr, cap, view_offsets);
  if (r) return r;
  if (!col_map || !mask || !tex) return fail(c, SL_EINVAL, "col_map, mask and texture are required");
  const int64_t HW = static_cast<int64_t>(H) * W;
  Params p;
  fill_common(c, p, n_views, H, W);
  p.in_col = col_map;
  p.in_mask = mask;
  p.tex = tex;
  p.tex_vs = 3 * HW;
  p.mask_mode = SL_MASK_FIXED;  // unused on this path
  p.poses = poses;
  p.xyz = xyz;
  p.bgr = bgr;
  p.view_offsets = view_offsets;
  const int nc_bit = c->d_nc ? M_NC : 0;
  const int decode_mode = M_FROMMAPS | M_CODES | nc_bit;
  const int cloud_mode = (xyz_dtype == SL_XYZ_F64 ? M_XYZ64 : 0) | nc_bit;
  const bool vec = (W % 16 == 0) && W >= 64 && aligned16(col_map) && aligned16(mask) && aligned16(tex);
  HIP_TRY(c, hipSetDevice(c->device));
  return launch(c, p, vec, false, decode_mode, cloud_mode, static_cast<hipStream_t>(stream));
}

int sl_sync(sl_ctx* c, void* stream) {
  if (!c) return SL_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  Header h;
  HIP_TRY(c, hipMemcpy(&h, c->d_hdr, sizeof(Header), hipMemcpyDeviceToHost));
  if (h.error) {
    HIP_TRY(c, hipMemset(&c->d_hdr->error, 0, sizeof(unsigned)));
    return fail(c, SL_ETIMEOUT, "device-side look-back wait expired");
  }
  return SL_OK;
}

int sl_profile_enable(sl_ctx* c, int max_launches) {
  if (!c || max_launches < 0) return SL_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  for (hipEvent_t e : c->prof_ev) HIP_TRY(c, hipEventDestroy(e));
  c->prof_ev.clear();
  c->prof_n = 0;
  for (int i = 0; i < kProfEv * max_launches; ++i) {
    hipEvent_t e;
    HIP_TRY(c, hipEventCreate(&e));
    c->prof_ev.push_back(e);
  }
  return SL_OK;
}

int sl_profile_read(sl_ctx* c, double* stats_ms, double* decode_ms, double* cloud_ms, int* launches) {
  if (!c) return SL_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  double t[3] = {0.0, 0.0, 0.0};
  for (int i = 0; i < c->prof_n; ++i) {
    hipEvent_t* ev = &c->prof_ev[kProfEv * i];
    HIP_TRY(c, hipEventSynchronize(ev[kProfEv - 1]));
    for (int k = 0; k < 3; ++k) {
      float ms = 0.f;
      HIP_TRY(c, hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
      t[k] += ms;
    }
  }
  if (stats_ms) *stats_ms = t[0];
  if (decode_ms) *decode_ms = t[1];
  if (cloud_ms) *cloud_ms = t[2];
  if (launches) *launches = c->prof_n;
  c->prof_n = 0;
  return SL_OK;
}

int sl_last_thresholds(sl_ctx* c, int view, float* nf, float* dr, int* thr_w, int* thr_c) {
  if (!c) return SL_EINVAL;
  if (view < 0 || view >= c->last_views || !c->d_stats) return fail(c, SL_EINVAL, "no such view");
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipDeviceSynchronize());
  ViewStats s;
  HIP_TRY(c, hipMemcpy(&s, c->d_stats + view, sizeof(ViewStats), hipMemcpyDeviceToHost));
  if (nf) *nf = s.noise_floor;
  if (dr) *dr = s.dynamic_range;
  if (thr_w) *thr_w = s.thr_white;
  if (thr_c) *thr_c = s.thr_contrast;
  return SL_OK;
}

}  // extern "C"
