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
//   k_stats   : 256-bin histogram of the black plane + max(white - black) per view,
//               merged with device atomics; the last block of each view turns them
//               into the float32 np.percentile(black, 95) recipe and integer
//               thresholds.  Also clears the look-back state of k_decode.
//   k_decode  : one 4096-pixel tile per workgroup, 16 pixels per lane.  Streams the
//               uint8 stack once with 16-byte loads, forms the Gray bits with a
//               byte-SWAR compare, Gray->binary in registers, masks, intersects the
//               camera ray with the projector column plane in f64 (reference
//               operation order, no contraction), and compacts points in pixel
//               order: workgroup scan + decoupled look-back across tiles taken in
//               ticket order, staged through LDS so the global stores are 16-byte
//               coalesced.
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
constexpr int kRing = 16;                // pattern planes in flight per lane

// k_decode mode bits
constexpr int M_MAPS = 1;      // write col/row/mask maps
constexpr int M_CLOUD = 2;     // triangulate + compact
constexpr int M_XYZ64 = 4;     // f64 xyz output (else f32)
constexpr int M_FROMMAPS = 8;  // input is (col_map, mask) instead of the stack
constexpr int M_NC = 16;       // rays from a device Nc table instead of pinhole K
constexpr int M_ROWS = 32;     // decode the row sequence

// look-back status word: [63:62] flag, [61:0] value
constexpr unsigned long long kFlagAgg = 1ull << 62;
constexpr unsigned long long kFlagPre = 2ull << 62;
constexpr unsigned long long kValMask = (1ull << 62) - 1;
constexpr unsigned kSpinLimit = 1u << 22;

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
  unsigned ticket;  // k_decode tile ticket
  unsigned error;   // sticky device-side failure (SL_ETIMEOUT)
  unsigned pad[14];
};

struct Params {
  const uint8_t* stack;
  int64_t stack_vs;
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
  int dbg;  // measurement-only ablations (SLGPU_DEBUG): 1 = tile from blockIdx, 2 = no look-back
  int Wp;
  const double4* planes;
  const double* xn;
  const double* yn;
  const double* nc_rays;
  double o0, o1, o2;
  const double* poses;
  int32_t* col_out;
  int32_t* row_out;
  uint8_t* mask_out;
  void* xyz;
  uint8_t* bgr;
  int64_t* view_offsets;
  ViewStats* stats;
  unsigned* part;  // k_stats histogram replicas [view][kReps][kSlot]
  unsigned long long* status;
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

__device__ __forceinline__ unsigned long long ld_status(const unsigned long long* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ void st_status(unsigned long long* p, unsigned long long v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

__device__ __forceinline__ int wave_incl_scan(int v, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(v, d, 64);
    if (lane >= d) v += t;
  }
  return v;
}

// --------------------------------------------------------------- k_stats ----
// grid (bx <= kStatBlocks, n_views).  Clears k_decode's look-back words and
// ticket; with the adaptive mask also builds, per view, the 256-bin histogram
// of the black plane and max(white - black):
//   * per-wave LDS histograms, then no-return device atomics into one of
//     kReps replicas of the view's histogram (blockIdx % kReps), so no more
//     than bx/kReps blocks ever add to one address;
//   * every wave drains its atomics (vmcnt(0)), then one lane adds to the
//     view's arrival counter; the block whose add is last reads (and zeroes)
//     the replicas with returning atomics and evaluates numpy's float32
//     percentile recipe.  The replicas are left zeroed for the next call.
__global__ __launch_bounds__(kThreads) void k_stats(Params p, int64_t n_status, int do_stats,
                                                    int vec) {
  const int tid = threadIdx.x;
  const int view = blockIdx.y;
  const int64_t lin = static_cast<int64_t>(blockIdx.y) * gridDim.x + blockIdx.x;
  const int64_t nblk = static_cast<int64_t>(gridDim.x) * gridDim.y;
  for (int64_t i = lin * kThreads + tid; i < n_status; i += nblk * kThreads) p.status[i] = 0ull;
  if (lin == 0 && tid == 0) p.hdr->ticket = 0u;
  if (!do_stats) return;

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
  for (int64_t c = blockIdx.x; c < p.tiles_per_view; c += gridDim.x) {
    const int64_t px0 = c * kTile + static_cast<int64_t>(tid) * kPx;
    const int n = static_cast<int>(min<int64_t>(max<int64_t>(p.HW - px0, 0), kPx));
    if (n == 0) continue;
    const uint4 w = ld16(vb + px0, n, vec);
    const uint4 b = ld16(vb + p.HW + px0, n, vec);
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      if (k < n) {
        const int bk = static_cast<int>(byte_of(b, k));
        const int wk = static_cast<int>(byte_of(w, k));
        atomicAdd(&sh[wid][bk], 1u);
        mx = max(mx, wk - bk);
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

template <int KC, int KR, int MODE, int VEC>
__global__ __launch_bounds__(kThreads, 2) void k_decode(Params p) {
  constexpr bool kStatic = KC >= 0;
  const int mode = MODE >= 0 ? MODE : p.mode;
  const int kc = KC >= 0 ? KC : p.kc;
  const int kr = KR >= 0 ? KR : p.kr;
  const int nc = p.nc, nr = p.nr;

  __shared__ float s_xyz[3 * kTile + 8];
  __shared__ uint32_t s_bgr[(3 * kTile + 8) / 4 + 2];
  __shared__ int s_wsum[kWaves];
  __shared__ unsigned s_tile;
  __shared__ long long s_excl;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  if (tid == 0) s_tile = (p.dbg & 1) ? blockIdx.x : atomicAdd(&p.hdr->ticket, 1u);
  __syncthreads();
  const unsigned tile = s_tile;
  const int view = static_cast<int>(tile / p.tiles_per_view);
  const int64_t lt = tile - static_cast<int64_t>(view) * p.tiles_per_view;
  const int64_t px0 = lt * kTile + static_cast<int64_t>(tid) * kPx;
  const int n_px = static_cast<int>(min<int64_t>(max<int64_t>(p.HW - px0, 0), kPx));
  const int64_t px_ld = n_px > 0 ? px0 : 0;  // keep loads unconditional and in bounds
  const bool vload = VEC > 0;

  uint32_t codec[kPx], coder[kPx];
  unsigned valid = 0u;  // bit k: pixel k passes the shadow/contrast mask
  uint4 tq0 = make_uint4(0, 0, 0, 0), tq1 = tq0, tq2 = tq0;

  if (!(mode & M_FROMMAPS)) {
    const uint8_t* src = p.stack + view * p.stack_vs + px_ld;
    const int64_t HW = p.HW;
    const uint4 wq = ld16(src, n_px, vload);
    const uint4 bq = ld16(src + HW, n_px, vload);
    if ((mode & M_CLOUD) && p.tex != nullptr) {
      const uint8_t* t = p.tex + view * p.tex_vs + 3 * px_ld;
      if (vload) {
        tq0 = reinterpret_cast<const uint4*>(t)[0];
        tq1 = reinterpret_cast<const uint4*>(t)[1];
        tq2 = reinterpret_cast<const uint4*>(t)[2];
      } else {
        tq0 = ld16(t, 3 * n_px, false);
        tq1 = ld16(t + 16, 3 * n_px - 16, false);
        tq2 = ld16(t + 32, 3 * n_px - 32, false);
      }
    }
    // ---- Gray bit planes: (pattern, inverse) pairs, columns then rows ----
    const int krr = (mode & M_ROWS) ? kr : 0;
    const int npl = 2 * (kc + krr);
    uint32_t cA[4] = {0, 0, 0, 0}, cB[4] = {0, 0, 0, 0};
    uint32_t rA[4] = {0, 0, 0, 0}, rB[4] = {0, 0, 0, 0};
    uint4 ring[kRing];
    const uint8_t* pat = src + 2 * HW;
#pragma unroll
    for (int j = 0; j < kRing; ++j)
      if (j < npl) ring[j] = ld16(pat + j * HW, n_px, vload);
#pragma unroll
    for (int base = 0; base < (kStatic ? 2 * (KC + KR) : npl); base += kRing) {
#pragma unroll
      for (int j = 0; j < kRing; j += 2) {
        const int pl = base + j;
        if (pl < npl) {
          const uint4 P = ring[j];
          const uint4 I = ring[j + 1];
          if (pl + kRing < npl) {
            ring[j] = ld16(pat + (pl + kRing) * HW, n_px, vload);
            ring[j + 1] = ld16(pat + (pl + kRing + 1) * HW, n_px, vload);
          }
          const int pair = pl >> 1;
          uint32_t m[4];
#pragma unroll
          for (int w = 0; w < 4; ++w) m[w] = gt_msb(word(P, w), word(I, w)) >> 7;
          // acc = (acc << 1) | bit: at most 8 bits per byte lane, so no carry
          // crosses into the neighbouring pixel.
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
    for (int k = 0; k < kPx; ++k) {
      const int w = k >> 2, s = 8 * (k & 3);
      const uint32_t gc = (((cA[w] >> s) & 0xffu) << cBn) | ((cB[w] >> s) & 0xffu);
      const uint32_t gr = (((rA[w] >> s) & 0xffu) << rBn) | ((rB[w] >> s) & 0xffu);
      codec[k] = gray_to_binary(gc << cSh);
      coder[k] = (mode & M_ROWS) ? gray_to_binary(gr << rSh) : 0u;
      const int wv = static_cast<int>(byte_of(wq, k));
      const int bv = static_cast<int>(byte_of(bq, k));
      const bool ok = (k < n_px) && (wv > thr_w) && (wv - bv > thr_c);
      valid |= ok ? (1u << k) : 0u;
    }
    if ((mode & M_CLOUD) && p.tex == nullptr) {
      // BGR of 16 pixels = white bytes x3, packed like a [16][3] texture row
      uint32_t t[12];
#pragma unroll
      for (int i = 0; i < 12; ++i) t[i] = 0u;
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        const uint32_t wv = byte_of(wq, k);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const int b = 3 * k + c;
          t[b >> 2] |= wv << (8 * (b & 3));
        }
      }
      tq0 = make_uint4(t[0], t[1], t[2], t[3]);
      tq1 = make_uint4(t[4], t[5], t[6], t[7]);
      tq2 = make_uint4(t[8], t[9], t[10], t[11]);
    }
    // ---- maps ----
    if (mode & M_MAPS) {
      const int64_t o = view * p.HW + px0;
      if (vload && n_px == kPx) {
        int4* cm = reinterpret_cast<int4*>(p.col_out + o);
        int4* rm = reinterpret_cast<int4*>(p.row_out + o);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          cm[i] = make_int4(codec[4 * i], codec[4 * i + 1], codec[4 * i + 2], codec[4 * i + 3]);
          rm[i] = make_int4(coder[4 * i], coder[4 * i + 1], coder[4 * i + 2], coder[4 * i + 3]);
        }
        uint32_t mw[4] = {0, 0, 0, 0};
#pragma unroll
        for (int k = 0; k < kPx; ++k) mw[k >> 2] |= ((valid >> k) & 1u) << (8 * (k & 3));
        *reinterpret_cast<uint4*>(p.mask_out + o) = make_uint4(mw[0], mw[1], mw[2], mw[3]);
      } else {
#pragma unroll
        for (int k = 0; k < kPx; ++k) {
          if (k < n_px) {
            p.col_out[o + k] = static_cast<int32_t>(codec[k]);
            p.row_out[o + k] = static_cast<int32_t>(coder[k]);
            p.mask_out[o + k] = static_cast<uint8_t>((valid >> k) & 1u);
          }
        }
      }
    }
  } else {
    // ---- reconstruct_point_cloud on given maps ----
    const int64_t o = view * p.HW + px_ld;
    const uint8_t* t = p.tex + view * p.tex_vs + 3 * px_ld;
    if (vload) {
      const int4* cm = reinterpret_cast<const int4*>(p.in_col + o);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int4 v = cm[i];
        codec[4 * i] = v.x;
        codec[4 * i + 1] = v.y;
        codec[4 * i + 2] = v.z;
        codec[4 * i + 3] = v.w;
      }
      const uint4 mq = *reinterpret_cast<const uint4*>(p.in_mask + o);
#pragma unroll
      for (int k = 0; k < kPx; ++k) valid |= (byte_of(mq, k) != 0u && k < n_px) ? (1u << k) : 0u;
      tq0 = reinterpret_cast<const uint4*>(t)[0];
      tq1 = reinterpret_cast<const uint4*>(t)[1];
      tq2 = reinterpret_cast<const uint4*>(t)[2];
    } else {
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        codec[k] = k < n_px ? static_cast<uint32_t>(p.in_col[o + k]) : 0u;
        valid |= (k < n_px && p.in_mask[o + k] != 0) ? (1u << k) : 0u;
      }
      tq0 = ld16(t, 3 * n_px, false);
      tq1 = ld16(t + 16, 3 * n_px - 16, false);
      tq2 = ld16(t + 32, 3 * n_px - 32, false);
    }
#pragma unroll
    for (int k = 0; k < kPx; ++k) coder[k] = 0u;
  }

  if (!(mode & M_CLOUD)) return;

  // ---- ray / plane intersection, f64 in the reference's operation order ----
  float fx_[kPx], fy_[kPx], fz_[kPx];
  double dx_[kPx], dy_[kPx], dz_[kPx];
  unsigned pts = 0u;
  {
    int v = static_cast<int>(px0 / p.W);
    int u = static_cast<int>(px0 - static_cast<int64_t>(v) * p.W);
    const double* pose = p.poses ? p.poses + 16 * view : nullptr;
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      dx_[k] = dy_[k] = dz_[k] = 0.0;
      fx_[k] = fy_[k] = fz_[k] = 0.0f;
      if (valid & (1u << k)) {
        double r0, r1, r2;
        if (mode & M_NC) {
          const int64_t q = px0 + k;
          r0 = p.nc_rays[q];
          r1 = p.nc_rays[p.HW + q];
          r2 = p.nc_rays[2 * p.HW + q];
        } else {
          const double x = p.xn[u];
          const double y = p.yn[v];
          // np.linalg.norm(rays, axis=0): sqrt((x*x + y*y) + 1*1)
          const double nrm = sqrt((x * x + y * y) + 1.0);
          r0 = x / nrm;
          r1 = y / nrm;
          r2 = 1.0 / nrm;
        }
        // np.clip(c, 0, Wp-1) (sl_system.py:626)
        const int c = min(max(static_cast<int>(codec[k]), 0), p.Wp - 1);
        const double4 pl = p.planes[c];
        const double den = (pl.x * r0 + pl.y * r1) + pl.z * r2;
        if (fabs(den) > 1e-6) {
          const double num = ((pl.x * p.o0 + pl.y * p.o1) + pl.z * p.o2) + pl.w;
          const double t = -num / den;
          double X = p.o0 + r0 * t;
          double Y = p.o1 + r1 * t;
          double Z = p.o2 + r2 * t;
          if (pose) {
            const double X2 = ((pose[0] * X + pose[1] * Y) + pose[2] * Z) + pose[3];
            const double Y2 = ((pose[4] * X + pose[5] * Y) + pose[6] * Z) + pose[7];
            const double Z2 = ((pose[8] * X + pose[9] * Y) + pose[10] * Z) + pose[11];
            X = X2;
            Y = Y2;
            Z = Z2;
          }
          if (mode & M_XYZ64) {
            dx_[k] = X;
            dy_[k] = Y;
            dz_[k] = Z;
          } else {
            fx_[k] = static_cast<float>(X);
            fy_[k] = static_cast<float>(Y);
            fz_[k] = static_cast<float>(Z);
          }
          pts |= 1u << k;
        }
      }
      if (++u == p.W) {
        u = 0;
        ++v;
      }
    }
  }

  // ---- workgroup scan of point counts ----
  const int cnt = __popc(pts);
  const int incl = wave_incl_scan(cnt, lane);
  if (lane == 63) s_wsum[wid] = incl;
  __syncthreads();
  int woff = 0, total = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) {
    const int s = s_wsum[w];
    woff += (w < wid) ? s : 0;
    total += s;
  }
  const int off = woff + incl - cnt;

  // ---- stage f32 points + colours in LDS (pixel order) ----
  uint8_t* sb = reinterpret_cast<uint8_t*>(s_bgr);
  {
    int o = off;
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      if (pts & (1u << k)) {
        if (!(mode & M_XYZ64)) {
          s_xyz[3 * o + 0] = fx_[k];
          s_xyz[3 * o + 1] = fy_[k];
          s_xyz[3 * o + 2] = fz_[k];
        }
        const int b = 3 * k;
        sb[3 * o + 0] = static_cast<uint8_t>(byte_of(b < 16 ? tq0 : b < 32 ? tq1 : tq2, b & 15));
        sb[3 * o + 1] = static_cast<uint8_t>(
            byte_of((b + 1) < 16 ? tq0 : (b + 1) < 32 ? tq1 : tq2, (b + 1) & 15));
        sb[3 * o + 2] = static_cast<uint8_t>(
            byte_of((b + 2) < 16 ? tq0 : (b + 2) < 32 ? tq1 : tq2, (b + 2) & 15));
        ++o;
      }
    }
  }

  // ---- decoupled look-back over tiles in ticket order (wave 0) ----
  if (wid == 0) {
    unsigned long long* st = p.status;
    if (lane == 0) st_status(st + tile, (tile == 0 ? kFlagPre : kFlagAgg) | static_cast<unsigned long long>(total));
    long long excl = (p.dbg & 2) ? static_cast<long long>(tile) * kTile : 0;
    if (tile > 0 && !(p.dbg & 2)) {
      long long j = static_cast<long long>(tile) - 1;
      unsigned spins = 0;
      for (;;) {
        const long long idx = j - lane;
        const unsigned long long s = idx >= 0 ? ld_status(st + idx) : kFlagPre;
        const unsigned long long flag = s & ~kValMask;
        const unsigned long long pre = __ballot(flag == kFlagPre);
        const unsigned long long zero = __ballot(flag == 0ull);
        const int lp = pre ? __ffsll(static_cast<long long>(pre)) - 1 : 64;
        const unsigned long long before = lp >= 64 ? ~0ull : ((1ull << lp) - 1ull) | (1ull << lp);
        if (zero & before) {
          if (++spins > kSpinLimit) {
            if (lane == 0) atomicOr(&p.hdr->error, 1u);
            break;
          }
          __builtin_amdgcn_s_sleep(1);
          continue;
        }
        long long v = (lane <= lp) ? static_cast<long long>(s & kValMask) : 0ll;
#pragma unroll
        for (int d = 32; d > 0; d >>= 1) v += __shfl_xor(v, d, 64);
        excl += v;
        if (lp < 64) break;
        j -= 64;
      }
      if (lane == 0) st_status(st + tile, kFlagPre | static_cast<unsigned long long>(excl + total));
    }
    if (lane == 0) {
      s_excl = excl;
      if (p.view_offsets) {
        if (lt == 0) p.view_offsets[view] = excl;
        if (tile + 1u == static_cast<unsigned>(p.n_views) * p.tiles_per_view)
          p.view_offsets[p.n_views] = excl + total;
      }
    }
  }
  __syncthreads();
  const long long E = s_excl;

  if (mode & M_XYZ64) {
    double* xyz = static_cast<double*>(p.xyz);
    int o = off;
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      if (pts & (1u << k)) {
        const long long g = 3 * (E + o);
        xyz[g] = dx_[k];
        xyz[g + 1] = dy_[k];
        xyz[g + 2] = dz_[k];
        ++o;
      }
    }
  } else {
    // floats [3E, 3E + 3T) from s_xyz[0 ..): aligned 16-B chunks of the
    // destination, element stores at the ragged ends.
    float* xyz = static_cast<float*>(p.xyz);
    const long long g_lo = 3 * E, g_hi = 3 * (E + total);
    const long long gbase = g_lo & ~3ll;
    const int nchunk = static_cast<int>((g_hi - gbase + 3) >> 2);
    for (int c = tid; c < nchunk; c += kThreads) {
      const long long g0 = gbase + 4ll * c;
      const int l0 = static_cast<int>(g0 - g_lo);
      if (g0 >= g_lo && g0 + 4 <= g_hi) {
        *reinterpret_cast<float4*>(xyz + g0) =
            make_float4(s_xyz[l0], s_xyz[l0 + 1], s_xyz[l0 + 2], s_xyz[l0 + 3]);
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (g0 + e >= g_lo && g0 + e < g_hi) xyz[g0 + e] = s_xyz[l0 + e];
      }
    }
  }
  {
    // colour bytes [3E, 3E + 3T) from sb[0 ..)
    const long long h_lo = 3 * E, h_hi = 3 * (E + total);
    const long long hbase = h_lo & ~15ll;
    const int nchunk = static_cast<int>((h_hi - hbase + 15) >> 4);
    for (int c = tid; c < nchunk; c += kThreads) {
      const long long h0 = hbase + 16ll * c;
      const int l0 = static_cast<int>(h0 - h_lo);
      if (h0 >= h_lo && h0 + 16 <= h_hi) {
        const int a = l0 >> 2, sh = l0 & 3;
        uint32_t d[5];
#pragma unroll
        for (int i = 0; i < 5; ++i) d[i] = s_bgr[a + i];
        uint32_t o4[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) o4[i] = __builtin_amdgcn_alignbyte(d[i + 1], d[i], sh);
        *reinterpret_cast<uint4*>(p.bgr + h0) = make_uint4(o4[0], o4[1], o4[2], o4[3]);
      } else {
        for (int e = 0; e < 16; ++e)
          if (h0 + e >= h_lo && h0 + e < h_hi) p.bgr[h0 + e] = sb[l0 + e];
      }
    }
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
  double* d_nc = nullptr;
  // scratch
  Header* d_hdr = nullptr;
  ViewStats* d_stats = nullptr;
  int64_t cap_views = 0;
  unsigned* d_part = nullptr;
  int64_t cap_part = 0;
  unsigned long long* d_status = nullptr;
  int64_t cap_status = 0;
  int last_views = 0;
  int dbg = 0;
  // optional per-launch HIP-event timing of k_stats / k_decode
  std::vector<hipEvent_t> prof_ev;  // 3 events per launch slot
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
  return grow(c, &c->d_status, &c->cap_status, tiles);
}

using KernelFn = void (*)(Params);

template <int KC, int KR, int MODE>
KernelFn pick_static() {
  return k_decode<KC, KR, MODE, 1>;
}

KernelFn pick_kernel(int kc, int kr, int mode, bool vec) {
  // Specialisations for the benchmark configurations (all unaligned, Nc, f64
  // or from-map calls go to the generic instantiation).
  if (vec && !(mode & (M_XYZ64 | M_FROMMAPS | M_NC))) {
    const int m = mode;
    const int maps_cloud = M_MAPS | M_CLOUD | M_ROWS;
    if (m == maps_cloud && kc == 11 && kr == 11) return pick_static<11, 11, M_MAPS | M_CLOUD | M_ROWS>();
    if (m == maps_cloud && kc == 10 && kr == 10) return pick_static<10, 10, M_MAPS | M_CLOUD | M_ROWS>();
    if (m == maps_cloud && kc == 10 && kr == 0) return pick_static<10, 0, M_MAPS | M_CLOUD | M_ROWS>();
    if (m == M_CLOUD && kc == 11) return pick_static<11, 0, M_CLOUD>();
    if (m == M_CLOUD && kc == 10) return pick_static<10, 0, M_CLOUD>();
    if (m == (M_MAPS | M_ROWS) && kc == 11 && kr == 11) return pick_static<11, 11, M_MAPS | M_ROWS>();
  }
  return vec ? k_decode<-1, -1, -1, 1> : k_decode<-1, -1, -1, 0>;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

int launch(sl_ctx* c, Params& p, bool vec, bool do_stats, hipStream_t s) {
  const int64_t tiles = static_cast<int64_t>(p.n_views) * p.tiles_per_view;
  int r = ensure_scratch(c, p.n_views, tiles);
  if (r) return r;
  p.stats = c->d_stats;
  p.part = c->d_part;
  p.status = c->d_status;
  p.hdr = c->d_hdr;
  c->last_views = p.n_views;
  // k_stats: enough blocks to cover the views with ~2K workgroups in total
  int bx = 1;
  if (do_stats) {
    bx = static_cast<int>(std::max<int64_t>(
        1, std::min<int64_t>({static_cast<int64_t>(p.tiles_per_view), int64_t{kStatBlocks},
                              std::max<int64_t>(1, 2048 / p.n_views)})));
  } else {
    bx = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(64, (tiles + 255) / 256)));
  }
  int stats_flag = do_stats ? 1 : 0, vec_flag = vec ? 1 : 0;
  int64_t n_status = tiles;
  void* sargs[] = {&p, &n_status, &stats_flag, &vec_flag};
  hipEvent_t* ev = nullptr;
  if (!c->prof_ev.empty() && 3 * (c->prof_n + 1) <= static_cast<int>(c->prof_ev.size()))
    ev = &c->prof_ev[3 * c->prof_n++];
  if (ev) HIP_TRY(c, hipEventRecord(ev[0], s));
  HIP_TRY(c, hipLaunchKernel(reinterpret_cast<const void*>(k_stats), dim3(bx, do_stats ? p.n_views : 1),
                             dim3(kThreads), sargs, 0, s));
  if (ev) HIP_TRY(c, hipEventRecord(ev[1], s));
  KernelFn fn = pick_kernel(p.kc, (p.mode & M_ROWS) ? p.kr : 0, p.mode, vec);
  void* dargs[] = {&p};
  HIP_TRY(c, hipLaunchKernel(reinterpret_cast<const void*>(fn), dim3(static_cast<unsigned>(tiles)),
                             dim3(kThreads), dargs, 0, s));
  if (ev) HIP_TRY(c, hipEventRecord(ev[2], s));
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
                    static_cast<void*>(c->d_part),
                    static_cast<void*>(c->d_status)})
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
  c->d_planes = c->d_xn = c->d_yn = c->d_nc = nullptr;
  HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_planes), sizeof(double) * 4 * Wp));
  HIP_TRY(c, hipMemcpy(c->d_planes, planes, sizeof(double) * 4 * Wp, hipMemcpyHostToDevice));
  HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_xn), sizeof(double) * W));
  HIP_TRY(c, hipMemcpy(c->d_xn, xn.data(), sizeof(double) * W, hipMemcpyHostToDevice));
  HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_yn), sizeof(double) * H));
  HIP_TRY(c, hipMemcpy(c->d_yn, yn.data(), sizeof(double) * H, hipMemcpyHostToDevice));
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
  Params p;
  fill_common(c, p, n_views, H, W);
  p.stack = stack;
  p.stack_vs = stack_vs;
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
  p.mode = (maps ? (M_MAPS | M_ROWS) : 0) | (xyz ? M_CLOUD : 0) | (xyz_dtype == SL_XYZ_F64 && xyz ? M_XYZ64 : 0) |
           (c->d_nc && xyz ? M_NC : 0);
  const bool vec = (HW % 16 == 0) && aligned16(stack) && (stack_vs % 16 == 0) && (!tex || (aligned16(tex) && tex_vs % 16 == 0)) &&
                   (!maps || (aligned16(col_out) && aligned16(row_out) && aligned16(mask_out)));
  HIP_TRY(c, hipSetDevice(c->device));
  return launch(c, p, vec, mask_mode == SL_MASK_ADAPTIVE, static_cast<hipStream_t>(stream));
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
  p.mode = M_FROMMAPS | M_CLOUD | (xyz_dtype == SL_XYZ_F64 ? M_XYZ64 : 0) | (c->d_nc ? M_NC : 0);
  const bool vec = (HW % 16 == 0) && aligned16(col_map) && aligned16(mask) && aligned16(tex);
  HIP_TRY(c, hipSetDevice(c->device));
  return launch(c, p, vec, false, static_cast<hipStream_t>(stream));
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
  for (int i = 0; i < 3 * max_launches; ++i) {
    hipEvent_t e;
    HIP_TRY(c, hipEventCreate(&e));
    c->prof_ev.push_back(e);
  }
  return SL_OK;
}

int sl_profile_read(sl_ctx* c, double* stats_ms, double* decode_ms, int* launches) {
  if (!c) return SL_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  double a = 0.0, b = 0.0;
  for (int i = 0; i < c->prof_n; ++i) {
    hipEvent_t* ev = &c->prof_ev[3 * i];
    HIP_TRY(c, hipEventSynchronize(ev[2]));
    float t0 = 0.f, t1 = 0.f;
    HIP_TRY(c, hipEventElapsedTime(&t0, ev[0], ev[1]));
    HIP_TRY(c, hipEventElapsedTime(&t1, ev[1], ev[2]));
    a += t0;
    b += t1;
  }
  if (stats_ms) *stats_ms = a;
  if (decode_ms) *decode_ms = b;
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
