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
// Work unit: a CHUNK of 1024 consecutive pixels of one view, owned by one wave.
// A 256-thread workgroup is 4 chunks of one view; grid = (chunk groups, views).
//
// Three kernels on one HIP stream, no host synchronisation between them:
//   k_decode : streams the uint8 stack once (16-byte loads, lane = 16 contiguous
//              pixels), forms the Gray bits with a byte-SWAR compare, Gray ->
//              binary in registers; writes the col/row maps and a 2-byte record
//              (clipped column code) per pixel.  Adaptive mask: also the 256-bin
//              histogram of the black plane + max(white - black), per workgroup
//              in LDS, added to the view's histogram at the end.
//   k_count  : per wave, the float32 np.percentile(black, 95) thresholds from
//              the histogram; the mask of every pixel (mask map) and, for the
//              cloud, the |n.r| > 1e-6 decision (f32 with an exact error bound,
//              f64 where undecided) as a point bitmask + the chunk's point count
//              (also added to its 64-chunk super-block sum).
//   k_cloud  : the chunk's output offset from the super-block and chunk sums,
//              its points compacted in LDS, the ray/plane intersection in f64
//              (reference operation order, no contraction), and the stores at
//              offset + rank -- the reference's np.where order.
//
// Everything in this file is compiled with -ffp-contract=off.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <stdio.h>

#include <algorithm>
#include <cmath>
#include <initializer_list>
#include <string>
#include <type_traits>
#include <thread>
#include <vector>

#include <dlfcn.h>

#include <mutex>

#include "rccl/rccl.h"
#include "slgpu.h"

#pragma clang fp contract(off)

namespace {

constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kPx = 16;                 // pixels per lane in the streaming layout
constexpr int kChunk = 64 * kPx;        // pixels per wave (one chunk)
constexpr int kChunkNib = kChunk / 4;   // point-nibble bytes per chunk
#ifndef SLGPU_RING
#define SLGPU_RING 40
#endif
constexpr int kRing = SLGPU_RING;       // stack planes in flight per lane
#ifndef SLGPU_LOAD_AUX
#define SLGPU_LOAD_AUX 2
#endif
constexpr int kLoadAux = SLGPU_LOAD_AUX;  // cache policy of the stack loads (2 = nt)
#ifndef SLGPU_NT_MAPS
#define SLGPU_NT_MAPS 0
#endif
constexpr bool kNtMaps = SLGPU_NT_MAPS != 0;  // non-temporal col/row map stores

#ifndef SLGPU_NT_SIDE
#define SLGPU_NT_SIDE 0
#endif
#ifndef SLGPU_NT_TEX
#define SLGPU_NT_TEX 0  // (A/B) nt texture loads in k_cloud
#endif
#ifndef SLGPU_NT_STATS
#define SLGPU_NT_STATS 0  // (A/B) nt loads in the histogram pass (k_stats, pre-stats)
#endif
constexpr bool kNtSide = SLGPU_NT_SIDE != 0;  // nt loads of records / texture / white-black in k_count, k_cloud
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ld_side16(const void* p) {
  if (kNtSide) {
    const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
    return make_uint4(v.x, v.y, v.z, v.w);
  }
  return *reinterpret_cast<const uint4*>(p);
}
__device__ __forceinline__ uint2 ld_side8(const void* p) {
  if (kNtSide) {
    const v2u v = __builtin_nontemporal_load(reinterpret_cast<const v2u*>(p));
    return make_uint2(v.x, v.y);
  }
  return *reinterpret_cast<const uint2*>(p);
}
__device__ __forceinline__ uint32_t ld_side4(const void* p) {
  if (kNtSide) return __builtin_nontemporal_load(reinterpret_cast<const uint32_t*>(p));
  return *reinterpret_cast<const uint32_t*>(p);
}
typedef int v4i __attribute__((ext_vector_type(4)));
#ifndef SLGPU_MAP_AUX
#define SLGPU_MAP_AUX 0
#endif
// (measurement builds) k_decode's col / row / mask map stores as buffer stores
// with this cache policy (16: sc1, write-through); 0: plain global stores
constexpr int kMapAux = SLGPU_MAP_AUX;
#ifndef SLGPU_MAP_STAGE
#define SLGPU_MAP_STAGE 2
#endif
// k_decode's col / row map stores 1 KB contiguous per wave instruction through
// a 1-KB LDS stage per wave (2: both maps, 1: the col map only), instead of
// each lane's 64 B at a 64-B stride (0).  Config 2 120.3-120.6 -> 116.5-117.4
// us per step, config 1 15.1 -> 14.4 (profiles/r04_ab/map_stage_lines.jsonl)
constexpr bool kMapStage = SLGPU_MAP_STAGE != 0;
// 16-byte store of 4 map words at p (16-byte aligned)
__device__ __forceinline__ void st_map(int32_t* p, uint32_t a, uint32_t b, uint32_t c, uint32_t d) {
  const v4i v = {static_cast<int>(a), static_cast<int>(b), static_cast<int>(c), static_cast<int>(d)};
  if (kNtMaps) __builtin_nontemporal_store(v, reinterpret_cast<v4i*>(p));
  else *reinterpret_cast<v4i*>(p) = v;
}

// mode bits
constexpr int M_MAPS = 1;      // k_decode: col/row maps; k_count: mask map
constexpr int M_CODES = 2;     // k_decode: per-pixel records; k_count: point decision + counts
constexpr int M_XYZ64 = 4;     // k_cloud: f64 xyz output (else f32)
constexpr int M_FROMMAPS = 8;  // input is a caller's (col_map, mask) instead of the stack
constexpr int M_NC = 16;       // rays from a device Nc table instead of pinhole K
constexpr int M_ROWS = 32;     // k_decode: decode the row sequence
constexpr int M_HIST = 64;     // adaptive mask: k_decode builds the histogram, k_count reads it
constexpr int M_FAST32 = 128;  // k_cloud: f32 arithmetic for well-conditioned points (SL_XYZ_F32_FAST)
constexpr int M_PLANE_RSRC = 512;  // k_decode: a buffer descriptor per plane (a view's planes read span >= 2 GiB)
constexpr int M_TEX = 2048;    // k_cloud: a BGR texture (else the white plane replicated)
constexpr int M_VERIFY = 4096; // k_cloud, SL_XYZ_F32: a shorter f64 evaluation whose f32 rounding is proven equal
                               // to the reference's (else the operators' sequences); Oc = 0, pinhole rays
                               // (with or without a pose)
constexpr int M_FUSED = 1024;  // k_fused: k_decode's chunk group, then its cloud (look-back offsets) in one launch
constexpr int M_DECIDE = 256;  // k_decode: also the mask and the |n.r| decision (k_count's work; k_stats
                               // histograms): mask map, point nibbles, chunk counts, block sums
constexpr float kFastKappa = 16.0f;  // condition-number limit of the f32 route

constexpr int kSlot = 272;                 // histogram of one view: 256 bins + max + pad (u32)
#ifndef SLGPU_HIST_REP
#define SLGPU_HIST_REP 8
#endif
constexpr int kHistRep = SLGPU_HIST_REP;   // LDS histogram replicas (lane % kHistRep; 8 measured best of 1/4/8/16/32/64)
constexpr int kHistStride = kHistRep + 1;  // bin stride: replica r of bin b sits in bank (b + r) % 32
// Measurement-only ablations, compiled in only by -DSLGPU_ABLATE=<bits> (a
// separate build for scripts/, never the shipped library): 1 = k_cloud without
// point math, 2 = k_cloud without xyz/colour stores, 4 = k_cloud without
// operand gathers, 8 = k_cloud stops after its loads + rank scan, 16 = ... after
// the LDS compaction, 32 = k_count with the fixed thresholds, 64 = k_count
// without the |n.r| test, 128 = k_count without plane gathers, 1024 = exact k_cloud gathers
// its planes from a 32-entry table (cache footprint), 4096 = exact k_cloud without any point
// arithmetic, 8192 = k_cloud without its block prefix (each chunk writes at 1024 x its index),
// 16384 / 32768 = the exact k_cloud without its colour / xyz stores.
#ifndef SLGPU_ABLATE
#define SLGPU_ABLATE 0
#endif
constexpr int kAblate = SLGPU_ABLATE;
#ifndef SLGPU_XY_CALC
#define SLGPU_XY_CALC 1
#endif
constexpr bool kXyCalc = SLGPU_XY_CALC != 0;  // exact k_cloud: rays' x / y by xy_of where sl_set_calib verified it
constexpr int kMaxWp = 32768;              // projector columns (record codes are 15 bits)
#ifndef SLGPU_MAX_CHUNKS
#define SLGPU_MAX_CHUNKS (1 << 16)
#endif
constexpr int64_t kMaxChunks = SLGPU_MAX_CHUNKS;  // chunks per launch group: bounds k_cloud's prefix reads
#ifndef SLGPU_REC_BLK
#define SLGPU_REC_BLK 1
#endif
// 12-bit records in chunk slots (1536 B: a lane's 16 codes as 16 B at 16 lane
// + 8 B at 1024 + 8 lane), the launch group's views interleaved by chunk group
// (rec_slot), stored write-through (kRecAux = sc1).  0: pixel order, 24 B per
// lane as two 12-B stores (A/B; scripts/micro/write_mix.hip prices both shapes)
constexpr bool kRecBlk = SLGPU_REC_BLK != 0;
#ifndef SLGPU_REC_BLK_MAPS
#define SLGPU_REC_BLK_MAPS 0  // (A/B) chunk slots in the maps kernels too
#endif
#ifndef SLGPU_REC_AUX
#define SLGPU_REC_AUX 16
#endif
constexpr int kRecAux = SLGPU_REC_AUX;
constexpr int kRecSlot = 1536;

struct ViewStats {
  int thr_white;        // mask: white > thr_white
  int thr_contrast;     //       white - black > thr_contrast
  float noise_floor;    // np.percentile(black, 95) (float32)
  float dynamic_range;  // max(white - black) (float32)
  unsigned pad[12];
};
static_assert(sizeof(ViewStats) % 64 == 0, "ViewStats keeps 64-B alignment");

struct Params {
  const uint8_t* stack;
  int64_t stack_vs;
  int view_bytes;  // bytes of a view's planes k_decode reads (< 2^31 unless M_PLANE_RSRC)
  const uint8_t* tex;
  int64_t tex_vs;
  const int32_t* in_col;
  const uint8_t* in_mask;
  int64_t HW;
  int H, W;
  // px / W = (px * w_magic) >> w_shift for 0 <= px < HW: 2^w_shift > HW * W and
  // w_magic = floor(2^w_shift / W) + 1 < 2^32 (fill_common).  k_decode's row
  // of a pixel without the compiler's reciprocal, a loop invariant VGPR
  uint32_t w_magic;
  int w_shift;
  int n_views;
  int cpv;           // chunks per view
  int64_t n_chunks;  // n_views * cpv
  int nc, nr, kc, kr;  // code bits and available bit planes (pairs)
  int mode;
  int Wp;
  const double4* planes;   // (n0, n1, n2, num = n.Oc + d) per projector column
  const float4* planes32;  // f32 (n0, n1, n2, -) for the point/no-point pre-decision
  const float* planes12;   // the same (n0, n1, n2) packed, 12 B per column (+ 1 KB of slack)
  const double* xn;        // (u - cx) / fx
  const double* yn;        // (v - cy) / fy
  const float* xn32;
  const float* yn32;
  float fast_thr;          // k_count's one-compare sufficient |n.r| test (sl_set_calib)
  int xy_safe;             // every xn, yn entry is div_safe (sl_set_calib): k_cloud skips the per-point test
  int xy_calc;             // k_cloud computes xn / yn (xy_of) instead of gathering them: sl_set_calib
                           // checked on the device that xy_of gives every table entry bit for bit
  double cx, cy, fx, fy;   // cam_K's (sl_system.py:610-611), for xy_of
  double rfx, rfy;         // fl(1 / fx), fl(1 / fy): the verified route's x, y
  const double* nc_rays;   // Nc table [3][HW] or null
  double o0, o1, o2;       // Oc
  const double* poses;
  uint16_t* codes;   // [view][HW] records: min(col, Wp-1)
  const int32_t* rec_col;  // maps + cloud on the decide path: k_cloud takes min(col, Wp-1) from this col
  int rec12;               // decide path (Wp < 4096): records packed 12 bits per pixel, 24 B per 16
                           // pixels, code 0xfff = no point (1.5 B/px written, no point nibbles)
                           // map and k_decode writes no records (2 B/px less k_decode write traffic)
  int rec_blk;             // rec12 records in kRecBlk's chunk slots (k_decode without maps; else pixel order)
  uint8_t* ptnib;    // [chunk][4 steps][64 lanes] point nibbles: bit e of byte (s, l) = pixel 256 s + 4 l + e
  int32_t* col_out;
  int32_t* row_out;
  uint8_t* mask_out;
  void* xyz;
  uint8_t* bgr;
  int64_t out_cap;         // points xyz / bgr hold (k_cloud writes nothing past it)
  int64_t* view_offsets;
  ViewStats* stats;
  unsigned long long* masked;  // or null: += masked pixels of each view (sl_mask_counts_to; the
                               // "Processing N valid pixels..." of sl_system.py:601-602)
  unsigned* hist;       // [view][kSlot] accumulated by this launch's k_decode
  unsigned* hist_zero;  // [view][kSlot] zeroed by this launch's k_decode (the next launch's hist)
  const int64_t* base_in;  // points of the earlier launch groups of this call, or null
  int* chunk_counts;       // k_count -> k_cloud: points per chunk
  int* block_sums;         // k_count -> k_cloud: points per workgroup (4 chunks)
  int bs_atomic;           // k_decode M_DECIDE: block sums by the last wave to arrive (no barrier)
  int decode_dyn;          // k_decode M_DECIDE | M_CODES: chunk groups after the first round pulled from a
                           // per-view counter (super_sums' last entries), not strided (SLGPU_DECODE_DYN=1, A/B)
  // two-level block prefix: every block (workgroup of 4 chunks) also adds its
  // sum to super_sums[block >> sb_shift]; k_cloud's offset = the super-block
  // sums before its super-block + the block sums before it inside it
  unsigned* super_sums;    // zeroed before the launch (by the previous launch's k_decode)
  unsigned* super_zero;    // the next launch's super-block sums: zeroed by this launch's k_decode
  int super_cap;           // entries of each super buffer
  int sb_shift;
  unsigned long long* lb;  // k_fused: look-back granules, one per workgroup of the launch (zeroed before it)
  int64_t lb_n;            // ... their number (k_stats zeroes them)
  int cloud_gx;            // k_cloud: workgroups per view that triangulate (the grid's x beyond: pre-stats)
  // k_cloud's pre-stats workgroups (sl_stack_next): the NEXT call's histogram
  // pass (k_stats' work) for the views of its first launch group, beside this
  // call's triangulation; null pre_stack: none
  const uint8_t* pre_stack;
  int64_t pre_vs;
  unsigned* pre_hist;      // [pre_views][kHistView] accumulated (zero before the launch)
  unsigned* pre_zero;      // the following pre-stats buffer: its first pre_zero_words words zeroed
  int64_t pre_zero_words;
  int pre_views;           // views of the next call's first group
  int pre_bpv;             // workgroups per view (k_stats' grid x)
  int pre_mix;             // pre-stats workgroups spread among the triangulating ones (else after them)
  int decode_gx;           // k_decode: decoding workgroups per view (0: gridDim.x; beyond: pre-stats)
};

// ---------------------------------------------------------------- helpers ----

// kRecBlk: the 1536-B record slot of chunk civ of view `view` in its launch
// group -- chunk groups (4 chunks, one workgroup iteration) of all the group's
// views interleaved, so that the views' workgroups, progressing together, write
// one contiguous window of the buffer at a time
__device__ __forceinline__ int64_t rec_slot(const Params& p, int view, int civ) {
  return (static_cast<int64_t>(civ >> 2) * p.n_views + view) * 4 + (civ & 3);
}

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

// Bit 7 of each byte: byte k of a > byte k of b (the other bits are garbage).
// a > b  <=>  !(b >= a); d = (b | 0x80) - (a & 0x7f) stays in [1, 255] per
// byte (no borrow crosses bytes) and its bit 7 is (b & 0x7f) >= (a & 0x7f);
// with the two top bits that is one three-input boolean of (a, b, d): 4
// instructions against gt_msb's 7.  Ties give 0 (strict, sl_system.py:561).
__device__ __forceinline__ uint32_t gt_bit7(uint32_t a, uint32_t b) {
  const uint32_t H = 0x80808080u;
  const uint32_t d = (b | H) - (a & ~H);
  // ~((b & ~a) | (~(a ^ b) & d)) as one v_bitop3 (truth table over src0 = 0xf0,
  // src1 = 0xcc, src2 = 0xaa: 0x71); the compiler's own matching splits it in 3
  return __builtin_amdgcn_bitop3_b32(a, b, d, 0x71);
}

// Gray -> binary within each byte's low `bits`-bit field (zeros above it):
// the prefix xor from the field's top bit down, 4 pixels per word.
__device__ __forceinline__ uint32_t gray_to_binary_bytes(uint32_t x, int bits) {
  if (bits > 1) x ^= (x >> 1) & 0x7f7f7f7fu;
  if (bits > 2) x ^= (x >> 2) & 0x3f3f3f3fu;
  if (bits > 4) x ^= (x >> 4) & 0x0f0f0f0fu;
  return x;
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

// Row of pixel px (0 <= px < HW) of the frame: px / W by Params::w_magic (one
// 32 x 32 -> 64-bit multiply and a shift, operands in SGPRs).
__device__ __forceinline__ int row_of(const Params& p, int px) {
  return static_cast<int>((static_cast<uint64_t>(static_cast<uint32_t>(px)) * p.w_magic) >> p.w_shift);
}

// Inclusive prefix sum over the 64 lanes of a wave.
__device__ __forceinline__ int wave_incl_scan(int s, int lane) {
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(s, d, 64);
    if (lane >= d) s += t;
  }
  return s;
}

__device__ __forceinline__ long long wave_sum64(long long s) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) {
    const unsigned long long u = static_cast<unsigned long long>(s);
    const unsigned lo = static_cast<unsigned>(__shfl_xor(static_cast<int>(u & 0xffffffffull), d, 64));
    const unsigned hi = static_cast<unsigned>(__shfl_xor(static_cast<int>(u >> 32), d, 64));
    s += static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo);
  }
  return s;
}

// A wave-uniform 64-bit value moved to SGPRs (so that addresses built from it
// use scalar bases).
__device__ __forceinline__ long long uniform64(long long v) {
  const unsigned lo = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(v));
  const unsigned hi = __builtin_amdgcn_readfirstlane(static_cast<unsigned>(static_cast<unsigned long long>(v) >> 32));
  return static_cast<long long>((static_cast<unsigned long long>(hi) << 32) | lo);
}

// f64 division a / b as the compiler lowers it (v_div_scale, v_rcp_f64, two
// Newton steps, a * r, the residual, v_div_fmas, v_div_fixup), without the
// scale / fixup steps, which change nothing when both operands are normal
// numbers within 2^+-300 of 1 (no rescaling, a normal quotient): the same
// bits.  The reciprocal step depends on b only, so divisions by one b share
// it.  div_safe(v): v is such an operand (and not +-0, whose sign the
// residual step would lose).
#ifndef SLGPU_DIV_SHARE
#define SLGPU_DIV_SHARE 1
#endif
constexpr bool kDivShare = SLGPU_DIV_SHARE != 0;
__device__ __forceinline__ double recip_nr(double b) {
  double r = __builtin_amdgcn_rcp(b);
  double e = __builtin_fma(-b, r, 1.0);
  r = __builtin_fma(r, e, r);
  e = __builtin_fma(-b, r, 1.0);
  return __builtin_fma(r, e, r);
}
__device__ __forceinline__ double div_rn(double a, double b, double r) {
  const double q = a * r;
  const double e = __builtin_fma(-b, q, a);
  return __builtin_fma(e, r, q);
}
// sqrt(s) as the compiler lowers it (v_rsq_f64, then Goldschmidt / Newton
// steps on g ~ sqrt(s) and h ~ 1/(2 sqrt(s))) without its range scaling
// (by 2^256 below 2^-767, undone by 2^-128) and its +-0 / inf / NaN select:
// the same bits for s in [2^-767, 2^1000].
__device__ __forceinline__ double sqrt_nr(double s) {
  const double r = __builtin_amdgcn_rsq(s);
  double g = s * r, h = r * 0.5;
  const double e = __builtin_fma(-h, g, 0.5);
  g = __builtin_fma(g, e, g);
  double d = __builtin_fma(-g, g, s);
  h = __builtin_fma(h, e, h);
  g = __builtin_fma(d, h, g);
  d = __builtin_fma(-g, g, s);
  return __builtin_fma(d, h, g);
}
// (w - c) / f of an integer pixel coordinate w (sl_system.py:615-616) by the
// shortened division (the quotient is correctly rounded where the operands
// are in range): sl_set_calib compares it with every xn / yn table entry on
// the device (k_xy_check) before k_cloud may compute the rays' x / y instead
// of gathering them.
__device__ __forceinline__ double xy_of(int w, double c, double f) {
  return div_rn(static_cast<double>(w) - c, f, recip_nr(f));
}
__device__ __forceinline__ bool div_safe(double v) {
  const double m = fabs(v);
  return m >= 0x1p-300 && m <= 0x1p300;
}

// A wave-uniform double moved to SGPRs.
__device__ __forceinline__ double uniform_f64(double v) {
  return __longlong_as_double(uniform64(__double_as_longlong(v)));
}

__device__ __forceinline__ int wave_sum(int s) {
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) s += __shfl_xor(s, d, 64);
  return s;
}

// The same sum (every lane active) without LDS permutes or address
// registers: an inclusive scan within each row of 16 lanes by DPP row_shr
// 1 / 2 / 4 / 8 (lanes shifted in from outside the row read 0), then the four
// row totals read into a scalar.  k_decode's loop uses it: the permute
// addresses of wave_sum are loop invariants the compiler hoists and, at 168
// VGPRs, spills.
__device__ __forceinline__ int wave_sum_dpp(int v) {
  v += __builtin_amdgcn_update_dpp(0, v, 0x111, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x112, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x114, 0xf, 0xf, true);
  v += __builtin_amdgcn_update_dpp(0, v, 0x118, 0xf, 0xf, true);
  return (__builtin_amdgcn_readlane(v, 15) + __builtin_amdgcn_readlane(v, 31)) +
         (__builtin_amdgcn_readlane(v, 47) + __builtin_amdgcn_readlane(v, 63));
}

// ------------------------------------------------------------ thresholds ----
// np.percentile(black_f32, 95) and max(white - black) of one view
// (sl_system.py:526-535) from its 256-bin histogram, evaluated by one wave
// (lane l holds bins 4l..4l+3, hmax = 1024 + max(white - black)): numpy 2.x's float32 recipe -- q = f32(95) /
// f32(100); virtual index (n-1)*q in float32; neighbours floor / floor+1, both
// clamped to n-1 when the index is >= n-1 (numpy/lib/_function_base_impl.py
// _get_indexes); gamma = index - floor; _lerp a + (b-a) g, replaced by
// b - (b-a)(1-g) where g >= 0.5.  white and contrast are integers, so
// `x > t` is `x > floor(t)`: the integer thresholds returned.
struct Thresholds {
  int white, contrast;
  float noise_floor, dynamic_range;
};

__device__ Thresholds thresholds_from_bins(const uint4 b4, unsigned hmax, int64_t n, int lane) {
  const int dmax = static_cast<int>(hmax) - 1024;
  const int s4 = static_cast<int>(b4.x + b4.y + b4.z + b4.w);
  const int incl = wave_incl_scan(s4, lane);
  const long long e0 = incl - s4;  // pixels below bin 4 lane
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
  // order statistic k = the bin b with cdf[b-1] <= k < cdf[b]
  auto value_at = [&](long long k) -> int {
    const long long c1 = e0 + b4.x, c2 = c1 + b4.y, c3 = c2 + b4.z, c4 = c3 + b4.w;
    int v = -1;
    if (e0 <= k && k < c1) v = 4 * lane;
    else if (c1 <= k && k < c2) v = 4 * lane + 1;
    else if (c2 <= k && k < c3) v = 4 * lane + 2;
    else if (c3 <= k && k < c4) v = 4 * lane + 3;
    const unsigned long long m = __ballot(v >= 0);
    const int src = m ? static_cast<int>(__ffsll(static_cast<long long>(m))) - 1 : 0;
    return __shfl(v, src, 64);
  };
  const float a = static_cast<float>(value_at(kp));
  const float b = static_cast<float>(value_at(kn));
  const float diff = b - a;
  float nf = a + diff * gamma;
  if (gamma >= 0.5f) nf = b - diff * (1.0f - gamma);
  const float dr = static_cast<float>(dmax);
  Thresholds t;
  t.noise_floor = nf;
  t.dynamic_range = dr;
  t.white = static_cast<int>(floorf(nf * 1.5f));
  t.contrast = static_cast<int>(floorf(dr * 0.05f));
  return t;
}

// ------------------------------------------------------- point decision ----

// Is |n.r| > 1e-6 (sl_system.py:638-642) for the pixel (u, v) / ray index q
// with clipped column code c, in the reference's exact f64 arithmetic?
// (Out of line: the rare undecided case.  Plain pointers, so that no copy of
// the kernel arguments is made.)
__device__ __noinline__ bool has_point_f64(const double4* planes, const double* xn, const double* yn,
                                           const double* nc_rays, int64_t HW, int c, int u, int v, int64_t q) {
  double r0, r1, r2;
  if (nc_rays) {
    r0 = nc_rays[q];
    r1 = nc_rays[HW + q];
    r2 = nc_rays[2 * HW + q];
  } else {
    const double xd = xn[u], yd = yn[v];
    const double nrm = sqrt((xd * xd + yd * yd) + 1.0);
    r0 = xd / nrm;
    r1 = yd / nrm;
    r2 = 1.0 / nrm;
  }
  const double4 pl = planes[c];
  return fabs((pl.x * r0 + pl.y * r1) + pl.z * r2) > 1e-6;
}

// The same decision in f32 with a rigorous error bound B: the f32 rounding of
// the inputs, of the ray and of the dot product stay below 2^-21 of
// S = sum|n_i r_i| (B uses 2^-18), plus an absolute 2^-20 * 1e-6 that covers
// the f32 rounding of the threshold itself.  Pixels within B of the threshold
// take the exact f64 arithmetic.  (x, y, z) is the unnormalised pinhole ray
// (z = 1, inv = 1/|r|) or the Nc ray (inv = 1).
__device__ __forceinline__ bool has_point(const Params& p, int mode, const float4& f, int c, float x, float y,
                                          float z, float inv, int u, int v, int64_t q) {
  const float a = fabsf((f.x * x + f.y * y + f.z * z) * inv);
  const float S = (fabsf(f.x * x) + fabsf(f.y * y) + fabsf(f.z * z)) * inv;
  const float B = S * 3.814697265625e-06f + 9.5367431640625e-13f;  // 2^-18 S + 2^-20 * 1e-6
  if (a > 1e-6f + B) return true;
  if (a < 1e-6f - B) return false;
  return has_point_f64(p.planes, p.xn, p.yn, (mode & M_NC) ? p.nc_rays : nullptr, p.HW, c, u, v, q);
}


// sl_set_calib: does xy_of give every xn / yn table entry bit for bit?
// (*bad = 1 on any difference; one thread per entry)
__global__ __launch_bounds__(256) void k_xy_check(const double* xn, int W, const double* yn, int H, double cx,
                                                  double cy, double fx, double fy, int* bad) {
  const int i = static_cast<int>(blockIdx.x) * 256 + static_cast<int>(threadIdx.x);
  bool diff = false;
  if (i < W) diff = __double_as_longlong(xy_of(i, cx, fx)) != __double_as_longlong(xn[i]);
  else if (i < W + H) diff = __double_as_longlong(xy_of(i - W, cy, fy)) != __double_as_longlong(yn[i - W]);
  if (diff) *bad = 1;
}

// ------------------------------------------------------------------ k_stats ----
// The adaptive mask's two global reductions (sl_system.py:526-528) ahead of a
// launch group whose k_decode applies the mask itself (M_DECIDE): per view,
// the black-plane 256-bin histogram and max(white - black), per workgroup in
// LDS (bank-skewed replicas, as k_decode's), flushed into kHistRepl replicas
// of the view's histogram (block % kHistRepl: the flush atomics of all
// workgroups spread over 8 rows instead of one).
constexpr int kHistRepl = 8;
constexpr int kHistView = kHistRepl * kSlot;  // u32 per view

// One workgroup's share of a view's histogram pass: the 16-pixel groups blk,
// blk + nblk, ... of the view's white (vb) and black (vb + HW) planes into the
// LDS replicas, then flushed into replica blk % kHistRepl of the view's global
// histograms gh (kHistView words).  s_hist: 256 * kHistStride words, s_max:
// kWaves ints (holds workgroup barriers).
__device__ __forceinline__ void stats_pass(const uint8_t* vb, int64_t HW, int64_t blk, int64_t nblk, unsigned* gh,
                                           unsigned* s_hist, int* s_max) {
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (int i = tid; i < 256 * kHistStride; i += kThreads) s_hist[i] = 0u;
  __syncthreads();
  unsigned* hrow = s_hist + (lane & (kHistRep - 1));
  int mx = -1024;
  const int64_t n16 = HW / 16;  // HW % 16 == 0 on this path
  for (int64_t i = blk * kThreads + tid; i < n16; i += nblk * kThreads) {
    uint4 wq, bq;
    if (SLGPU_NT_STATS) {  // (A/B) non-temporal white / black loads
      const v4u a = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(vb + 16 * i));
      const v4u b = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(vb + HW + 16 * i));
      wq = make_uint4(a.x, a.y, a.z, a.w);
      bq = make_uint4(b.x, b.y, b.z, b.w);
    } else {
      wq = *reinterpret_cast<const uint4*>(vb + 16 * i);
      bq = *reinterpret_cast<const uint4*>(vb + HW + 16 * i);
    }
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const int bk = static_cast<int>(byte_of(bq, k));
      atomicAdd(hrow + bk * kHistStride, 1u);
      mx = max(mx, static_cast<int>(byte_of(wq, k)) - bk);
    }
  }
#pragma unroll
  for (int d = 32; d > 0; d >>= 1) mx = max(mx, __shfl_xor(mx, d, 64));
  if (lane == 0) s_max[wid] = mx;
  __syncthreads();
  gh += (blk % kHistRepl) * kSlot;
  unsigned cnt = 0u;
  const unsigned* row = s_hist + tid * kHistStride;
#pragma unroll
  for (int r = 0; r < kHistRep; ++r) cnt += row[r];
  if (cnt) atomicAdd(gh + tid, cnt);
  if (tid == 0) {
    int m = s_max[0];
#pragma unroll
    for (int w = 1; w < kWaves; ++w) m = max(m, s_max[w]);
    if (m > -1024) atomicMax(gh + 256, static_cast<unsigned>(m + 1024));
  }
}

// grid (blocks per view, views of the group); 16 pixels per thread per step.
__global__ __launch_bounds__(kThreads) void k_stats(Params p) {
  __shared__ unsigned s_hist[256 * kHistStride];
  __shared__ int s_max[kWaves];
  const int tid = threadIdx.x;
  const int view = blockIdx.y;
  if (blockIdx.x == 0)  // the next launch group's histograms of this slot (its scratch here)
    for (int i = tid; i < kHistView; i += kThreads) p.hist_zero[static_cast<int64_t>(view) * kHistView + i] = 0u;
  if (p.lb && blockIdx.x == 0 && view == 0)  // k_fused's look-back granules (it follows this launch)
    for (int64_t i = tid; i < p.lb_n; i += kThreads) p.lb[i] = 0ull;
  stats_pass(p.stack + view * p.stack_vs, p.HW, blockIdx.x, gridDim.x, p.hist + static_cast<int64_t>(view) * kHistView,
             s_hist, s_max);
}

// One pre-stats workgroup (sl_stack_next), number sx of the nsx per grid row
// that a k_cloud or k_decode launch appends: zeroes its share of the buffer
// the following pass accumulates into, then runs its share of the next call's
// histogram pass (k_stats' work) into p.pre_hist.
__device__ __forceinline__ void pre_stats_block(const Params& p, int64_t sx, int64_t nsx, unsigned* s_hist,
                                                int* s_max) {
  const int tid = threadIdx.x;
  const int64_t sblk = static_cast<int64_t>(blockIdx.y) * nsx + sx;
  const int64_t total = static_cast<int64_t>(p.pre_views) * p.pre_bpv;
  for (int64_t i = sblk * kThreads + tid; i < p.pre_zero_words; i += static_cast<int64_t>(gridDim.y) * nsx * kThreads)
    p.pre_zero[i] = 0u;
  if (sblk < total) {
    const int pv = static_cast<int>(sblk / p.pre_bpv);
    stats_pass(p.pre_stack + pv * p.pre_vs, p.HW, sblk - static_cast<int64_t>(pv) * p.pre_bpv, p.pre_bpv,
               p.pre_hist + static_cast<int64_t>(pv) * kHistView, s_hist, s_max);
  }
}

// Thresholds of a view from its kHistRepl histogram replicas (one wave).
__device__ __forceinline__ Thresholds view_thresholds(const Params& p, int view, int lane) {
  uint4 b4 = make_uint4(0u, 0u, 0u, 0u);
  unsigned hmax = 0u;
  const unsigned* h = p.hist + static_cast<int64_t>(view) * kHistView;
#pragma unroll
  for (int r = 0; r < kHistRepl; ++r) {
    const uint4 t = reinterpret_cast<const uint4*>(h + r * kSlot)[lane];
    b4.x += t.x;
    b4.y += t.y;
    b4.z += t.z;
    b4.w += t.w;
    hmax = max(hmax, h[r * kSlot + 256]);
  }
  return thresholds_from_bins(b4, hmax, p.HW, lane);
}

// Mask of 4 packed pixels (one word of white / black bytes): bit e = pixel e
// has white > tw and white - black > tc (sl_system.py:534-535); byte-SWAR in
// 16-bit lanes as k_count (tw2 = (tw + 1) * 0x10001, tc2 = (tc + 17) * 0x10001;
// exact for 0 <= tw + 1 <= 0x7000, -17 <= tc <= 0x7000: adaptive thresholds
// are in [0, 382] x [-13, 12], fixed ones 40 / 10).  *bytes: the 0/1 mask bytes.
__device__ __forceinline__ uint32_t mask4(uint32_t w, uint32_t b, uint32_t tw2, uint32_t tc2, uint32_t* bytes) {
  const uint32_t we = w & 0x00ff00ffu, wo = (w >> 8) & 0x00ff00ffu;
  const uint32_t be = b & 0x00ff00ffu, bo = (b >> 8) & 0x00ff00ffu;
  const uint32_t me = ((we | 0x80008000u) - tw2) & (((we + 0x00100010u) | 0x80008000u) - (be + tc2));
  const uint32_t mo = ((wo | 0x80008000u) - tw2) & (((wo + 0x00100010u) | 0x80008000u) - (bo + tc2));
  const uint32_t y = ((me >> 15) & 0x00010001u) | ((mo >> 7) & 0x01000100u);
  *bytes = y;
  return (y & 1u) | ((y >> 7) & 2u) | ((y >> 14) & 4u) | ((y >> 21) & 8u);
}

// k_decode M_DECIDE: the f32 plane table, xn = (u - cx) / fx and yn =
// (v - cy) / fy in LDS (host: Wp <= kDecPl, W <= kDecX, H <= kDecY; the
// launch's grid is capped at a few workgroups per CU, so the fill is cheap).
#ifndef SLGPU_DEC_YN_LDS
#define SLGPU_DEC_YN_LDS 0
#endif
constexpr bool kDecYnLds = SLGPU_DEC_YN_LDS != 0;  // yn in LDS (else one early global load per lane)
#ifndef SLGPU_DEC_GLDS
#define SLGPU_DEC_GLDS 1
#endif
constexpr bool kDecGlds = SLGPU_DEC_GLDS != 0;  // decision tables by LDS-DMA, overlapping the first stack loads
#ifndef SLGPU_DEC_PL3
#define SLGPU_DEC_PL3 0
#endif
// (measurement build, SLGPU_DEC_PL3=1: the decision's plane table as packed
// (n0, n1, n2) floats, 12 B per projector column, Wp <= 1920: 38.4 KB of
// tables, so that 4 workgroups fit a CU's LDS -- with -DSLGPU_DECODE_WAVES=4
// -DSLGPU_DECODE_PER_CU=4)
constexpr bool kDecPl3 = SLGPU_DEC_PL3 != 0;
constexpr int kDecPl = kDecPl3 ? 1920 : 2048, kDecX = 4096, kDecY = 4096;
constexpr int kDecPlWords = kDecPl3 ? (kDecPl * 12 + 1023) / 1024 * 256 : kDecPl * 4;  // LDS words of the plane table
constexpr int kBsSlots = 64;
constexpr int kSuperCap = 4096;  // super-block sums per launch group (>= sqrt of its blocks)  // k_decode M_DECIDE: chunk-group iterations per workgroup with a barrier-free block sum
constexpr int kDecodeLds = (kDecPlWords + kDecX + (kDecYnLds ? kDecY : 0)) * 4;  // bytes: > the histogram replicas
static_assert(kDecodeLds >= 256 * kHistStride * 4, "the decode LDS holds the histogram replicas too");

// ================================================================ k_decode ====
// gray_decode (sl_system.py:519-577) for one chunk per wave, in the streaming
// layout (lane l owns the chunk's pixels [16 l, 16 l + 16)): column and row
// code of every pixel, reading each plane of the uint8 stack once (M_FROMMAPS:
// a caller's col_map instead).  Outputs by mode bit:
//   M_MAPS   col/row int32 maps, full frame, unmasked (what gray_decode
//            returns), 16-byte stores;
//   M_CODES  record16 = min(col, Wp-1) (np.clip, sl_system.py:626) per pixel,
//            for k_count / k_cloud;
//   M_HIST   the view's black-plane histogram and max(white - black)
//            (sl_system.py:526-528): LDS replicas bank-skewed so that the
//            lanes of a half-wave that hit the same bin use 32 different
//            banks, added to the view's global histogram once per workgroup.
// Grid (chunk groups, views); waves past the view's last chunk run empty (the
// workgroup barriers count them).
#ifndef SLGPU_DECODE_PER_CU
#define SLGPU_DECODE_PER_CU 3
#endif
constexpr int kDecodePerCu = SLGPU_DECODE_PER_CU;  // default k_decode grid cap, workgroups per CU (0: none)
#ifndef SLGPU_DECODE_WAVES
#define SLGPU_DECODE_WAVES 3
#endif
#ifndef SLGPU_SWAR_GRAY
#define SLGPU_SWAR_GRAY 1
#endif
// Gray bits gathered MSB-first into byte lanes and converted to binary there,
// 4 pixels per instruction (0: the per-pixel conversion; measurement build)
constexpr bool kSwarGray = SLGPU_SWAR_GRAY != 0;
// k_decode's body; group_hook(col, pt, live, n_px, civ, cg, s_lds) runs at
// the end of each chunk group when the mode has M_FUSED (k_fused: the
// group's cloud in the same launch), else nothing.
struct NoGroupHook {
  template <class... A>
  __device__ void operator()(A&&...) const {}
};
template <int KC, int KR, int MODE, int VEC, class Hook>
__device__ __forceinline__ void decode_body(const Params& p, const Hook& group_hook) {
  const int mode = MODE >= 0 ? MODE : p.mode;
  const int kc = KC >= 0 ? KC : p.kc;
  const int krr = (mode & M_ROWS) ? (KR >= 0 ? KR : p.kr) : 0;
  const int nc = p.nc, nr = p.nr;
  const bool vec = VEC > 0;
  const bool hist = (mode & M_HIST) && !(mode & M_DECIDE);  // accumulate the histogram (else: k_stats did)

  // LDS: the histogram replicas (M_HIST), or the decision's tables (M_DECIDE)
  __shared__ __attribute__((aligned(16))) unsigned s_lds[kDecodeLds / 4];
  __shared__ int s_max[kWaves];
  __shared__ int s_cnt[2][kWaves];
  __shared__ unsigned s_bsum[kBsSlots];  // per iteration: points (low 16 bits) + waves arrived << 16
  __shared__ uint32_t s_thr[2];          // M_DECIDE adaptive: the view's tw2, tc2
  __shared__ unsigned s_mcount;          // M_DECIDE with p.masked: the workgroup's masked pixels
  // kMapStage: a 1-KB stage per wave for contiguous map stores (maps kernels only)
  __shared__ uint4 s_mapst[(kMapStage && (MODE < 0 || (MODE & M_MAPS))) ? 64 * kWaves : 1];
  unsigned* s_hist = s_lds;
  float4* s_pl = reinterpret_cast<float4*>(s_lds);
  const float* s_pl3 = reinterpret_cast<const float*>(s_lds);
  float* s_xn = reinterpret_cast<float*>(s_lds) + kDecPlWords;
  float* s_yn = s_xn + kDecX;
  const bool decide = (mode & M_DECIDE) != 0;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform, provably
  const int view = blockIdx.y;
  const int64_t HW = p.HW;
  // pre-stats workgroups (sl_stack_next, SLGPU_PRE_DECODE=1) after the
  // decoding ones: the next call's histograms in this launch's tail
  // (instantiations for calls with a cloud on the decide path only)
  constexpr bool kPreRole = MODE < 0 || ((MODE & M_DECIDE) && (MODE & M_CODES) && !(MODE & M_FUSED));
  if (kPreRole && p.decode_gx > 0 && static_cast<int>(blockIdx.x) >= p.decode_gx) {
    pre_stats_block(p, blockIdx.x - p.decode_gx, gridDim.x - p.decode_gx, s_lds, s_max);
    return;
  }
  const int gx = p.decode_gx > 0 ? p.decode_gx : static_cast<int>(gridDim.x);  // decoding workgroups per view
  if (decide) {
    if (tid < kBsSlots) s_bsum[tid] = 0u;
    if (tid == 0) s_mcount = 0u;  // published by the barrier of iteration 0 (or the table fill's)
    // the view's mask thresholds (k_stats' histograms), once per workgroup by
    // wave 0 while the others fill the tables: at this point no decode state
    // is live (computed inside the chunk loop they cost registers and ~9 us)
    if ((mode & M_HIST) && wid == 0) {
      const Thresholds t = view_thresholds(p, view, lane);
      if (lane == 0) {
        s_thr[0] = static_cast<uint32_t>(t.white + 1) * 0x00010001u;
        s_thr[1] = static_cast<uint32_t>(t.contrast + 17) * 0x00010001u;
        if (blockIdx.x == 0) {
          p.stats[view].thr_white = t.white;
          p.stats[view].thr_contrast = t.contrast;
          p.stats[view].noise_floor = t.noise_floor;
          p.stats[view].dynamic_range = t.dynamic_range;
        }
      }
    }
    // The decision tables exist only for a cloud (M_CODES: the host checked
    // the calibration against the frame and Wp <= kDecPl); a maps-only call
    // may run on a context without calibration, or with one for another
    // frame or a wider projector, so it loads none of them.  The fills are
    // clamped to the LDS the tables own all the same.
    const bool tables = (mode & M_CODES) != 0;
    const int wp_t = min(p.Wp, kDecPl), w_t = min(p.W, kDecX);
    if (tables && kDecGlds) {
      // the tables by LDS-DMA (16 B per lane, 1 KB per wave instruction): no
      // VGPRs, and the first chunk group's stack loads below are issued
      // while they land; the workgroup barrier before the first mask
      // (iteration 0) publishes them.  Lanes past the end repeat the last
      // entry into slack LDS (kDecPl, kDecX are multiples of 64 entries).
      typedef __attribute__((address_space(3))) void* lds_ptr_t;
      if (kDecPl3) {  // the packed 12-B table as bytes, 1 KB per wave instruction (slack: kDecPlWords)
        const uint8_t* src = reinterpret_cast<const uint8_t*>(p.planes12);
        for (int i = wid; i * 1024 < wp_t * 12; i += kWaves)
          __builtin_amdgcn_global_load_lds(src + 16 * (i * 64 + lane), (lds_ptr_t)(s_lds + i * 256), 16, 0, 0);
      } else {
        for (int i = wid; i * 64 < wp_t; i += kWaves)
          __builtin_amdgcn_global_load_lds(p.planes32 + min(i * 64 + lane, wp_t - 1), (lds_ptr_t)(s_pl + i * 64), 16, 0, 0);
      }
      for (int i = wid; i * 256 < w_t; i += kWaves)
        __builtin_amdgcn_global_load_lds(p.xn32 + min(i * 256 + 4 * lane, w_t - 4), (lds_ptr_t)(s_xn + i * 256), 16, 0, 0);
    } else if (tables) {
      for (int i = tid; i < wp_t; i += kThreads) {
        if (kDecPl3) {
          float* d = reinterpret_cast<float*>(s_lds) + 3 * i;
          d[0] = p.planes12[3 * i];
          d[1] = p.planes12[3 * i + 1];
          d[2] = p.planes12[3 * i + 2];
        } else {
          s_pl[i] = p.planes32[i];
        }
      }
      for (int i = tid; i < w_t; i += kThreads) s_xn[i] = p.xn32[i];
    }
    if (tables && kDecYnLds)
      for (int i = tid; i < min(p.H, kDecY); i += kThreads) s_yn[i] = p.yn32[i];
    if (!kDecGlds) __syncthreads();
  }
  uint32_t tw2 = static_cast<uint32_t>(40 + 1) * 0x00010001u;      // fixed mask:
  uint32_t tc2 = static_cast<uint32_t>(10 + 17) * 0x00010001u;     // multi_point_cloud_process.py:36-38
  if (!kDecGlds && decide && (mode & M_HIST)) {  // adaptive: the view's (wave 0 above; the table fill's barrier)
    tw2 = __builtin_amdgcn_readfirstlane(s_thr[0]);
    tc2 = __builtin_amdgcn_readfirstlane(s_thr[1]);
  }
  int it = 0;

  // the next launch's super-block sums (scratch of this one)
  if (p.super_zero && blockIdx.x == 0 && blockIdx.y == 0)
    for (int i = tid; i < p.super_cap; i += kThreads) p.super_zero[i] = 0u;
  // the next launch's histogram (scratch of this one)
  if (hist && blockIdx.x == 0)
    for (int i = tid; i < kSlot; i += kThreads) p.hist_zero[view * kSlot + i] = 0u;
  if (hist) {
    for (int i = tid; i < 256 * kHistStride; i += kThreads) s_hist[i] = 0u;
    __syncthreads();
  }

  // Chunk groups of the view, strided over the grid's x (one group per
  // workgroup unless the launch caps the grid, SLGPU_DECODE_GRID); the
  // workgroup-uniform loop holds no barrier.
  const int ngroups = (p.cpv + kWaves - 1) / kWaves;
  int mx_acc = -1024;
  __shared__ int s_next[2];  // decode_dyn: the workgroup's next chunk group
  const bool dyn = p.decode_dyn && decide && (mode & M_CODES) && !(mode & M_FUSED) && !p.bs_atomic;
  unsigned* const dyn_ctr = p.super_sums + (p.super_cap - 1 - view);
  for (int cg = blockIdx.x; cg < ngroups;) {
  // decode_dyn: this workgroup's claim on a later chunk group, issued now so
  // that its round trip overlaps this group's loads (published below)
  unsigned dyn_next = 0u;
  if (dyn && tid == 0) dyn_next = atomicAdd(dyn_ctr, 1u);
  const int civ = cg * kWaves + wid;  // chunk in view
  const bool live = civ < p.cpv;
  const int64_t px0 = static_cast<int64_t>(civ) * kChunk + lane * kPx;
  const int n_px = live ? static_cast<int>(min<int64_t>(max<int64_t>(HW - px0, 0), kPx)) : 0;
  const int64_t pxl = n_px > 0 ? px0 : 0;  // keep loads unconditional and in bounds
  const int64_t o = view * HW + px0;

  // M_DECIDE without yn in LDS: the row's yn first (the oldest load: waiting
  // for it never waits for this iteration's stores)
  const float ys_early = (decide && !kDecYnLds && (mode & M_CODES) && n_px > 0)
                             ? p.yn32[row_of(p, static_cast<int>(px0))] : 0.0f;
  uint32_t col[kPx];
  uint32_t pt_rec = 0xffffu;  // the lane's point bits for 12-bit records (decide path)
  if (mode & M_FROMMAPS) {
    // reconstruct_point_cloud's input col_map (clipped below, sl_system.py:626)
    const int64_t ol = view * HW + pxl;
    if (vec) {
      const int4* cm = reinterpret_cast<const int4*>(p.in_col + ol);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int4 v = cm[i];
        col[4 * i] = static_cast<uint32_t>(max(v.x, 0));
        col[4 * i + 1] = static_cast<uint32_t>(max(v.y, 0));
        col[4 * i + 2] = static_cast<uint32_t>(max(v.z, 0));
        col[4 * i + 3] = static_cast<uint32_t>(max(v.w, 0));
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPx; ++k) col[k] = k < n_px ? static_cast<uint32_t>(max(p.in_col[ol + k], 0)) : 0u;
    }
  } else {
    // Plane loads: on the vector path a buffer descriptor of the view's stack
    // (SGPRs) + the lane's 32-bit pixel offset + the plane offset in an SGPR.
    // When the planes read span 2 GiB or more (M_PLANE_RSRC), a descriptor per
    // plane instead (4 SGPRs each: 46 planes overflow the SGPR file, so this is
    // not the default).
    const uint8_t* vbase = p.stack + view * p.stack_vs;
    const int voff = static_cast<int>(pxl);
    const __amdgpu_buffer_rsrc_t rs_view =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(vbase), 0, p.view_bytes, 0x00020000);
    auto ldp = [&](int plane) -> uint4 {
      if (vec && !(mode & M_PLANE_RSRC)) {
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs_view, voff, plane * static_cast<int>(HW), kLoadAux);
        return make_uint4(v[0], v[1], v[2], v[3]);
      }
      if (vec) {
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
            const_cast<uint8_t*>(vbase) + static_cast<int64_t>(plane) * HW, 0, static_cast<int>(HW), 0x00020000);
        const auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, voff, 0, kLoadAux);
        return make_uint4(v[0], v[1], v[2], v[3]);
      }
      return ld16(vbase + pxl + static_cast<int64_t>(plane) * HW, n_px, false);
    };
    const uint4 wq = ldp(0);
    const uint4 bq = ldp(1);
    // ---- Gray bit planes: (pattern, inverse) pairs, columns then rows ----
    const int npl = 2 * (kc + krr);
    uint32_t cA[4] = {0, 0, 0, 0}, cB[4] = {0, 0, 0, 0};
    uint32_t rA[4] = {0, 0, 0, 0}, rB[4] = {0, 0, 0, 0};
    // Fold one (pattern, inverse) pair into per-byte-lane accumulators:
    // acc = (acc << 1) | bit holds at most 8 bits per byte lane, so no carry
    // crosses into the neighbouring pixel; codes of up to 16 bits use A then B.
    // (kSwarGray: each bit enters at bit 7 of its byte lane and the lane
    // shifts right, acc = (acc >> 1 & 0x7f..) | (bit7 & 0x80..): the first
    // pair ends lowest, bit-reversed below; 6 instructions per word and pair)
    auto consume = [&](const uint4& P, const uint4& I, int pair) {
      if (kSwarGray) {
        auto ins = [](uint32_t acc, uint32_t g) { return ((acc >> 1) & 0x7f7f7f7fu) | (g & 0x80808080u); };
        uint32_t g[4];
#pragma unroll
        for (int w = 0; w < 4; ++w) g[w] = gt_bit7(word(P, w), word(I, w));
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          if (pair < kc) {
            if (pair < 8) cA[w] = ins(cA[w], g[w]);
            else cB[w] = ins(cB[w], g[w]);
          } else if (pair - kc < 8) {
            rA[w] = ins(rA[w], g[w]);
          } else {
            rB[w] = ins(rB[w], g[w]);
          }
        }
        return;
      }
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
    if (KC >= 0) {
      // static plane count: unrolled, kRing planes in flight
      constexpr int NPL = 2 * (KC + (KR > 0 ? KR : 0));
      constexpr int R = kRing < NPL ? kRing : NPL;
      uint4 ring[R > 0 ? R : 1];
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (j < npl) ring[j] = ldp(2 + j);
#pragma unroll
      for (int pl = 0; pl < NPL; pl += 2) {
        if (pl < npl) {
          const uint4 P = ring[pl % R];
          const uint4 I = ring[(pl + 1) % R];
          if (pl + R < npl) {
            ring[pl % R] = ldp(2 + pl + R);
            ring[(pl + 1) % R] = ldp(3 + pl + R);
          }
          consume(P, I, pl >> 1);
        }
      }
    } else {
      constexpr int R = 16;
      uint4 ring[R];
#pragma unroll
      for (int j = 0; j < R; ++j)
        if (j < npl) ring[j] = ldp(2 + j);
      for (int base = 0; base < npl; base += R) {
#pragma unroll
        for (int j = 0; j < R; j += 2) {
          const int pl = base + j;
          if (pl < npl) {
            const uint4 P = ring[j];
            const uint4 I = ring[j + 1];
            if (pl + R < npl) {
              ring[j] = ldp(2 + pl + R);
              ring[j + 1] = ldp(3 + pl + R);
            }
            consume(P, I, pl >> 1);
          }
        }
      }
    }
    // ---- Gray -> binary ----
    const int cBn = kc > 8 ? kc - 8 : 0;
    const int rBn = krr > 8 ? krr - 8 : 0;
    const int cSh = nc - kc;
    const int rSh = nr - krr;
    uint32_t row[kPx];
    if (kSwarGray) {
      // A code's top min(k, 8) Gray bits are in A, the rest in B, each
      // bit-reversed by the right-shifting accumulators: bitreverse puts them
      // MSB-first in the low bits of each byte (pixel 4 w + e in byte 3 - e).
      // Binary per byte lane; B's bits continue A's prefix xor, so A's binary
      // lowest bit (the parity of its Gray bits) is xor-ed into B's top bit
      // before B's own conversion.
      // Codes shifted by sh = n - k bits (fewer patterns than code bits):
      // binary(g << sh) = binary(g) << sh with its lowest bit repeated below.
      auto to_binary = [](uint32_t (&A)[4], uint32_t (&B)[4], int k) {
        const int kA = k < 8 ? k : 8, kB = k - kA;
#pragma unroll
        for (int w = 0; w < 4; ++w) {
          A[w] = gray_to_binary_bytes(__builtin_bitreverse32(A[w]), kA);
          // (A's parity flips B's top bit: every bit below it follows)
          B[w] = kB > 0 ? gray_to_binary_bytes(__builtin_bitreverse32(B[w]) ^ ((A[w] & 0x01010101u) << (kB - 1)), kB)
                        : 0u;
        }
      };
      to_binary(cA, cB, kc);
#pragma unroll
      for (int q = 0; q < kPx; ++q) {
        const int w = q >> 2, sft = 8 * (3 - (q & 3));
        col[q] = (((cA[w] >> sft) & 0xffu) << cBn) | ((cB[w] >> sft) & 0xffu);
      }
      if (cSh > 0) {
#pragma unroll
        for (int q = 0; q < kPx; ++q) {
          const uint32_t lo = col[q] & 1u;
          col[q] = (col[q] << cSh) | ((lo << cSh) - lo);
        }
      }
      // rows: only the maps store reads them -- converted there, a word at a time
      if (mode & M_ROWS) to_binary(rA, rB, krr);
#pragma unroll
      for (int k = 0; k < kPx; ++k) row[k] = 0u;
    } else {
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        const int w = k >> 2, sft = 8 * (k & 3);
        const uint32_t gc = (((cA[w] >> sft) & 0xffu) << cBn) | ((cB[w] >> sft) & 0xffu);
        const uint32_t gr = (((rA[w] >> sft) & 0xffu) << rBn) | ((rB[w] >> sft) & 0xffu);
        col[k] = gray_to_binary(gc << cSh);
        row[k] = (mode & M_ROWS) ? gray_to_binary(gr << rSh) : 0u;
      }
    }
    // (kSwarGray) pixel 4 w + e's row code from the binary row words
    auto row_code = [&](int w, int e) -> uint32_t {
      const int sft = 8 * (3 - e);
      uint32_t v = (((rA[w] >> sft) & 0xffu) << rBn) | ((rB[w] >> sft) & 0xffu);
      if (rSh > 0) {
        const uint32_t lo = v & 1u;
        v = (v << rSh) | ((lo << rSh) - lo);
      }
      return v;
    };
    if (mode & M_MAPS) {
      if (vec) {
        if (n_px == kPx && kMapAux) {
          const int64_t vb = view * HW;  // (4 HW < 2^31: measurement builds only)
          const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(p.col_out + vb, 0, static_cast<int>(4 * HW), 0x00020000);
          const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(p.row_out + vb, 0, static_cast<int>(4 * HW), 0x00020000);
          const int bo = 4 * static_cast<int>(px0);
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            __builtin_amdgcn_raw_buffer_store_b128(v4u{col[4 * i], col[4 * i + 1], col[4 * i + 2], col[4 * i + 3]}, rc,
                                                   bo + 16 * i, 0, kMapAux);
            uint32_t r4[4];
#pragma unroll
            for (int e = 0; e < 4; ++e) r4[e] = kSwarGray ? row_code(i, e) : row[4 * i + e];
            __builtin_amdgcn_raw_buffer_store_b128(v4u{r4[0], r4[1], r4[2], r4[3]}, rr, bo + 16 * i, 0, kMapAux);
          }
        } else if (kMapStage && live) {
          // 1-KB contiguous map stores through a 1-KB LDS stage per wave:
          // for each quarter j of the chunk (pixels 256 j .. 256 j + 255, the
          // 16 lanes of DPP row j), those lanes put their 64 B in the stage,
          // then lane l stores bytes 16 l .. 16 l + 15 of it (pixels
          // 256 j + 4 l ..); a lane stores only where its source lane's 16
          // pixels are in the view (whole 16-pixel groups: W % 16 == 0)
          uint4* const stg = s_mapst + 64 * wid;
          const int64_t cbase = view * HW + static_cast<int64_t>(civ) * kChunk;  // the chunk's first pixel
#pragma unroll
          for (int m = 0; m < 2; ++m) {
            if (m == 1 && SLGPU_MAP_STAGE == 1) {  // (1: the col map only; the rows as below)
#pragma unroll
              for (int i = 0; i < 4; ++i) {
                uint32_t r4[4];
#pragma unroll
                for (int e = 0; e < 4; ++e) r4[e] = kSwarGray ? row_code(i, e) : row[4 * i + e];
                if (n_px == kPx) st_map(p.row_out + o + 4 * i, r4[0], r4[1], r4[2], r4[3]);
              }
              continue;
            }
            // the chunk's 4 KB of this map as a buffer (SGPRs): stores past the
            // view's end (its last, partial chunk) fall outside it and are dropped
            const __amdgpu_buffer_rsrc_t rd = __builtin_amdgcn_make_buffer_rsrc(
                (m == 0 ? p.col_out : p.row_out) + cbase, 0,
                static_cast<int>(4 * min<int64_t>(kChunk, HW - static_cast<int64_t>(civ) * kChunk)), 0x00020000);
#pragma unroll
            for (int j = 0; j < 4; ++j) {
              if ((lane >> 4) == j && n_px == kPx) {
                const int u = lane & 15;
#pragma unroll
                for (int q = 0; q < 4; ++q) {
                  uint32_t v4[4];
#pragma unroll
                  for (int e = 0; e < 4; ++e)
                    v4[e] = m == 0 ? col[4 * q + e] : (kSwarGray ? row_code(q, e) : row[4 * q + e]);
                  stg[4 * u + q] = make_uint4(v4[0], v4[1], v4[2], v4[3]);
                }
              }
              __builtin_amdgcn_wave_barrier();
              const uint4 v = stg[lane];
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_raw_buffer_store_b128(v4u{v.x, v.y, v.z, v.w}, rd, 1024 * j + 16 * lane, 0, 0);
            }
          }
        } else if (n_px == kPx) {
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            st_map(p.col_out + o + 4 * i, col[4 * i], col[4 * i + 1], col[4 * i + 2], col[4 * i + 3]);
            if (kSwarGray) {
              uint32_t r4[4];
#pragma unroll
              for (int e = 0; e < 4; ++e) r4[e] = row_code(i, e);
              st_map(p.row_out + o + 4 * i, r4[0], r4[1], r4[2], r4[3]);
            } else {
              st_map(p.row_out + o + 4 * i, row[4 * i], row[4 * i + 1], row[4 * i + 2], row[4 * i + 3]);
            }
          }
        }
      } else {
#pragma unroll
        for (int k = 0; k < kPx; ++k) {
          if (k < n_px) {
            p.col_out[o + k] = static_cast<int32_t>(col[k]);
            p.row_out[o + k] = static_cast<int32_t>(kSwarGray ? row_code(k >> 2, k & 3) : row[k]);
          }
        }
      }
    }
    if (decide) {
      if (kDecGlds && it == 0) {  // workgroup-uniform: the LDS-DMA tables and s_thr are in
        __syncthreads();
        if (mode & M_HIST) {
          tw2 = __builtin_amdgcn_readfirstlane(s_thr[0]);
          tc2 = __builtin_amdgcn_readfirstlane(s_thr[1]);
        }
      }
      // ---- mask with the view's thresholds (tw2 / tc2: computed at kernel start) ----
      uint32_t ok = 0u, mb[4];
#pragma unroll
      for (int w = 0; w < 4; ++w) ok |= mask4(word(wq, w), word(bq, w), tw2, tc2, &mb[w]) << (4 * w);
      if (n_px != kPx) ok = 0u;  // vec: whole 16-pixel groups
      if (p.masked) {  // (uniform) the chunk's masked pixels into the workgroup's count
        const int mc = wave_sum_dpp(__popc(ok));
        if (lane == 0 && mc) atomicAdd(&s_mcount, static_cast<unsigned>(mc));
      }
      if ((mode & M_MAPS) && n_px == kPx) {
        if (kMapAux) {
          const __amdgpu_buffer_rsrc_t rm =
              __builtin_amdgcn_make_buffer_rsrc(p.mask_out + view * HW, 0, static_cast<int>(HW), 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(v4u{mb[0], mb[1], mb[2], mb[3]}, rm, static_cast<int>(px0), 0, kMapAux);
        } else {
          *reinterpret_cast<uint4*>(p.mask_out + o) = make_uint4(mb[0], mb[1], mb[2], mb[3]);
        }
      }
      // ---- |n.r| > 1e-6 (sl_system.py:638-642) of the masked pixels, LDS tables ----
      uint32_t pt = 0u;
      if ((mode & M_CODES) && ok) {
        const int px0i = static_cast<int>(px0);
        const int v = row_of(p, px0i), u0 = px0i - v * p.W;  // the lane's 16 pixels share row v (W % 16 == 0)
        float4 pf[kPx];
#pragma unroll
        for (int k = 0; k < kPx; ++k) {
          const uint32_t ck = min(col[k], static_cast<uint32_t>(p.Wp - 1));
          pf[k] = kDecPl3 ? make_float4(s_pl3[3 * ck], s_pl3[3 * ck + 1], s_pl3[3 * ck + 2], 0.0f) : s_pl[ck];
        }
        float xs[kPx];
#pragma unroll
        for (int q4 = 0; q4 < 4; ++q4) {
          const float4 x4 = reinterpret_cast<const float4*>(s_xn + u0)[q4];
          xs[4 * q4] = x4.x;
          xs[4 * q4 + 1] = x4.y;
          xs[4 * q4 + 2] = x4.z;
          xs[4 * q4 + 3] = x4.w;
        }
        const float ys = kDecYnLds ? s_yn[v] : ys_early;
        uint32_t todo = ok;
        if (!(mode & M_NC)) {  // k_count's one-compare sufficient test (p.fast_thr, sl_set_calib)
#pragma unroll
          for (int k = 0; k < kPx; ++k) {
            const float a = fabsf(__builtin_fmaf(pf[k].x, xs[k], __builtin_fmaf(pf[k].y, ys, pf[k].z)));
            if (a > p.fast_thr) pt |= 1u << k;
          }
          pt &= ok;
          todo &= ~pt;
        }
#pragma unroll
        for (int k = 0; k < kPx; ++k) {  // the bounded f32 test, f64 where undecided
          if (!((todo >> k) & 1u)) continue;
          const int c = static_cast<int>(min(col[k], static_cast<uint32_t>(p.Wp - 1)));
          const int64_t q = px0 + k;
          float x, y, z, inv;
          if (mode & M_NC) {
            x = static_cast<float>(p.nc_rays[q]);
            y = static_cast<float>(p.nc_rays[HW + q]);
            z = static_cast<float>(p.nc_rays[2 * HW + q]);
            inv = 1.0f;
          } else {
            x = xs[k];
            y = ys;
            z = 1.0f;
            inv = __frsqrt_rn(x * x + y * y + 1.0f);
          }
          if (has_point(p, mode, pf[k], c, x, y, z, inv, u0 + k, v, q)) pt |= 1u << k;
        }
      }
      if (mode & M_CODES) {
        // point nibbles in k_count's layout (byte 64 s + l: pixels 256 s + 4 l + e):
        // this lane's 16 pixels are the 4 bytes at 4 lane
        const int64_t gci = static_cast<int64_t>(view) * p.cpv + civ;
        pt_rec = pt;
        if (live && !p.rec12) {  // (12-bit records carry the point bits: code 0xfff = no point)
          const uint32_t nw = (pt & 0xfu) | ((pt & 0xf0u) << 4) | ((pt & 0xf00u) << 8) | ((pt & 0xf000u) << 12);
          *reinterpret_cast<uint32_t*>(p.ptnib + gci * kChunkNib + 4 * lane) = nw;
        }
        const int cnt = wave_sum_dpp(__popc(pt));
        if (lane == 0) {
          if (live) p.chunk_counts[gci] = cnt;
          const unsigned mine = live ? static_cast<unsigned>(cnt) : 0u;
          if (p.bs_atomic) {
            // the workgroup's block sum without a barrier: the last of its
            // waves to add its count (one LDS slot per iteration) writes it
            const unsigned old = atomicAdd(&s_bsum[it], (1u << 16) | mine);
            if ((old >> 16) == kWaves - 1) {
              const int64_t blk = static_cast<int64_t>(view) * ngroups + cg;
              const unsigned t = (old & 0xffffu) + mine;
              p.block_sums[blk] = static_cast<int>(t);
              if (t) atomicAdd(p.super_sums + (blk >> p.sb_shift), t);
            }
          } else {
            s_cnt[it & 1][wid] = static_cast<int>(mine);
          }
        }
      }
    }
    if (hist) {
      unsigned* hrow = s_hist + (lane & (kHistRep - 1));
      int mx = -1024;
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        if (k < n_px) {
          const int bk = static_cast<int>(byte_of(bq, k));
          atomicAdd(hrow + bk * kHistStride, 1u);
          mx = max(mx, static_cast<int>(byte_of(wq, k)) - bk);
        }
      }
      mx_acc = max(mx_acc, mx);
    }
  }

  if ((mode & M_CODES) && !p.rec_col && !(mode & M_FUSED)) {
    // records for k_count / k_cloud: clipped column code
    uint32_t rec[kPx / 2];
#pragma unroll
    for (int i = 0; i < kPx / 2; ++i)
      rec[i] = min(col[2 * i], static_cast<uint32_t>(p.Wp - 1)) |
               (min(col[2 * i + 1], static_cast<uint32_t>(p.Wp - 1)) << 16);
    if (vec && p.rec12) {
      // (chunk slots without maps: the maps kernels keep the pixel order, whose
      // registers fit; the host sets p.rec_blk to match, for k_cloud)
      const bool blk = kRecBlk && (!(mode & M_MAPS) || SLGPU_REC_BLK_MAPS);
      if (n_px == kPx) {  // 8 codes per 3 words
        uint32_t rw[6];
        uint32_t* ro = blk ? rw : reinterpret_cast<uint32_t*>(reinterpret_cast<uint8_t*>(p.codes) + 3 * o / 2);
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const uint32_t* r = rec + 4 * h;  // codes 8 h .. 8 h + 7, two per word; 0xfff: no point
          auto cd = [&](int k, uint32_t c) { return ((pt_rec >> (8 * h + k)) & 1u) ? c : 0xfffu; };
          const uint32_t c0 = cd(0, r[0] & 0xffffu), c1 = cd(1, r[0] >> 16), c2 = cd(2, r[1] & 0xffffu);
          const uint32_t c3 = cd(3, r[1] >> 16), c4 = cd(4, r[2] & 0xffffu), c5 = cd(5, r[2] >> 16);
          const uint32_t c6 = cd(6, r[3] & 0xffffu), c7 = cd(7, r[3] >> 16);
          ro[3 * h] = c0 | (c1 << 12) | (c2 << 24);  // 4-byte aligned: one dwordx3 store
          ro[3 * h + 1] = (c2 >> 8) | (c3 << 4) | (c4 << 16) | (c5 << 28);
          ro[3 * h + 2] = (c5 >> 4) | (c6 << 8) | (c7 << 20);
        }
        if (blk) {  // the chunk's 1536-B slot (rec_slot): words 0-3 at 16 lane, 4-5 at 1024 + 8 lane
          const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
              reinterpret_cast<uint8_t*>(p.codes) + kRecSlot * rec_slot(p, view, civ), 0, kRecSlot, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b128(v4u{rw[0], rw[1], rw[2], rw[3]}, rs, 16 * lane, 0, kRecAux);
          __builtin_amdgcn_raw_buffer_store_b64(v2u{rw[4], rw[5]}, rs, 1024 + 8 * lane, 0, kRecAux);
        }
      }
    } else if (vec) {
      if (n_px == kPx) {
        uint4* ro = reinterpret_cast<uint4*>(p.codes + o);
        ro[0] = make_uint4(rec[0], rec[1], rec[2], rec[3]);
        ro[1] = make_uint4(rec[4], rec[5], rec[6], rec[7]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPx; ++k)
        if (k < n_px) p.codes[o + k] = static_cast<uint16_t>(rec[k >> 1] >> (16 * (k & 1)));
    }
  }
  if (decide && (mode & M_CODES) && !p.bs_atomic && !(mode & M_FUSED)) {  // the workgroup's block sum (k_count's, for k_cloud's offsets)
    if (dyn && tid == 0) s_next[it & 1] = static_cast<int>(dyn_next) + gx;
    __syncthreads();
    if (tid == 0) {
      int t = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) t += s_cnt[it & 1][w];
      const int64_t blk = static_cast<int64_t>(view) * ngroups + cg;
      p.block_sums[blk] = t;
      if (t) atomicAdd(p.super_sums + (blk >> p.sb_shift), static_cast<unsigned>(t));
    }
  }
  if (mode & M_FUSED) group_hook(col, pt_rec, live, n_px, civ, cg, s_lds);
  cg = dyn ? s_next[it & 1] : cg + gx;  // (dyn: published before the block-sum barrier above)
  ++it;
  }  // chunk groups

  if (decide && p.masked) {  // one global add per workgroup (its view: blockIdx.y)
    __syncthreads();
    if (tid == 0 && s_mcount) atomicAdd(p.masked + view, static_cast<unsigned long long>(s_mcount));
  }

  if (hist) {
#pragma unroll
    for (int d = 32; d > 0; d >>= 1) mx_acc = max(mx_acc, __shfl_xor(mx_acc, d, 64));
    if (lane == 0) s_max[wid] = mx_acc;
    __syncthreads();
    unsigned* gh = p.hist + view * kSlot;
    unsigned cnt = 0u;
    const unsigned* row = s_hist + tid * kHistStride;
#pragma unroll
    for (int r = 0; r < kHistRep; ++r) cnt += row[r];
    if (cnt) atomicAdd(gh + tid, cnt);
    if (tid == 0) {
      int m = s_max[0];
#pragma unroll
      for (int w = 1; w < kWaves; ++w) m = max(m, s_max[w]);
      if (m > -1024) atomicMax(gh + 256, static_cast<unsigned>(m + 1024));
    }
  }
}

template <int KC, int KR, int MODE, int VEC>
__global__ __launch_bounds__(kThreads, SLGPU_DECODE_WAVES) void k_decode(Params p) {
  decode_body<KC, KR, MODE, VEC>(p, NoGroupHook{});
}

// ================================================================= k_count ====
// Per wave (one chunk): the mask thresholds (adaptive: from the view's
// histogram; fixed: white > 40, contrast > 10), the mask of every pixel
// (M_MAPS: the mask map) and, for the cloud (M_CODES), the decision
// |n.r| > 1e-6 (sl_system.py:638-642) of every masked pixel -- f32 with an
// exact error bound, f64 where undecided -- as point bits, the chunk's point
// count and its super-block sum.
// Quad layout: in step s (0..3) lane l holds the 4 pixels 256 s + 4 l + e of
// the chunk: 4-byte white/black loads and mask stores, 8-byte record loads,
// and plane gathers of nearby columns.  Every load is issued before any is
// used (clamped, unconditional addresses).
template <int VEC>
__device__ __forceinline__ int count_chunk(const Params& p, int64_t gc, int view, int civ, int lane, bool live,
                                           int* masked) {
  const int mode = p.mode;
  const bool vec = VEC > 0;
  const int HW = static_cast<int>(p.HW);  // < 2^31: one view's stack is < 2 GiB
  const int cpx = civ * kChunk;
  const int W = p.W;
  const bool codes = (mode & M_CODES) != 0;
  const bool nc = (mode & M_NC) != 0;
  const uint8_t* vstack = p.stack + view * p.stack_vs;            // wave-uniform bases
  const uint16_t* vcodes = codes ? p.codes + static_cast<int64_t>(view) * HW : nullptr;

  // ---- loads: the view's histogram first (vmcnt is in order: the threshold
  // scan then waits for it alone), then the chunk ----
  uint4 hb = make_uint4(0u, 0u, 0u, 0u);
  unsigned hmax = 0u;
  const bool adaptive = (mode & M_HIST) && !(kAblate & 32);
  if (adaptive) {
    const unsigned* h = p.hist + view * kSlot;
    hb = reinterpret_cast<const uint4*>(h)[lane];
    hmax = h[256];
  }
  uint32_t wv[4], bv[4];  // 4 pixels per step, one byte each
  uint32_t rc[4][2];      // records: 4 x u16 per step
  const int px_hi = vec ? HW - 4 : HW - 1;  // clamp for tail loads (keeps 4-pixel alignment)
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int px = min(cpx + 256 * s + 4 * lane, px_hi);
    if (mode & M_FROMMAPS) {
      wv[s] = bv[s] = 0u;
    } else if (vec) {
      wv[s] = ld_side4(vstack + px);
      bv[s] = ld_side4(vstack + HW + px);
    } else {
      uint32_t a = 0u, b = 0u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int q = min(px + e, HW - 1);
        a |= static_cast<uint32_t>(vstack[q]) << (8 * e);
        b |= static_cast<uint32_t>(vstack[HW + q]) << (8 * e);
      }
      wv[s] = a;
      bv[s] = b;
    }
    if (codes) {
      if (vec) {
        const uint2 r = ld_side8(vcodes + px);
        rc[s][0] = r.x;
        rc[s][1] = r.y;
      } else {
        rc[s][0] = vcodes[min(px, HW - 1)] | (static_cast<uint32_t>(vcodes[min(px + 1, HW - 1)]) << 16);
        rc[s][1] = vcodes[min(px + 2, HW - 1)] | (static_cast<uint32_t>(vcodes[min(px + 3, HW - 1)]) << 16);
      }
    }
  }
  uint32_t mk[4] = {0u, 0u, 0u, 0u};  // FROMMAPS: the caller's mask bytes
  if (mode & M_FROMMAPS) {
    const uint8_t* vm = p.in_mask + static_cast<int64_t>(view) * HW;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int px = cpx + 256 * s + 4 * lane;
#pragma unroll
      for (int e = 0; e < 4; ++e) mk[s] |= (px + e < HW && vm[px + e] != 0) ? (1u << e) : 0u;
    }
  }

  *masked = 0;
  if (!live) return 0;

  // ---- thresholds (while the loads above are in flight) ----
  int thr_w = 40, thr_c = 10;  // fixed: multi_point_cloud_process.py:36-38
  if (adaptive) {
    const Thresholds t = thresholds_from_bins(hb, hmax, p.HW, lane);
    thr_w = t.white;
    thr_c = t.contrast;
    if (civ == 0 && lane == 0) {
      p.stats[view].thr_white = t.white;
      p.stats[view].thr_contrast = t.contrast;
      p.stats[view].noise_floor = t.noise_floor;
      p.stats[view].dynamic_range = t.dynamic_range;
    }
  }

  // ---- mask ----
  // vec: byte-SWAR in 16-bit lanes (even / odd pixels), two compares per 4
  // pixels: w > tw  <=>  (0x8000 + w) - (tw + 1) has bit 15, and
  // w - b > tc  <=>  (0x8000 + w + 16) - (b + tc + 17) has bit 15 -- no borrow
  // crosses lanes for 0 <= tw + 1 <= 0x7000 and -17 <= tc <= 0x7000 (adaptive:
  // tw in [0, 382], tc in [-13, 12]).
  const bool swar = vec && thr_w >= -1 && thr_w < 0x7000 && thr_c >= -17 && thr_c < 0x7000;
  const uint32_t tw2 = static_cast<uint32_t>(thr_w + 1) * 0x00010001u;
  const uint32_t tc2 = static_cast<uint32_t>(thr_c + 17) * 0x00010001u;
  uint32_t ok[4];      // bit e: pixel 256 s + 4 lane + e is valid
  uint32_t mbytes[4];  // the mask map words (vec), stored after the plane gathers below:
                       // vmcnt counts stores too, so a gather issued after a store waits for it
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int px = cpx + 256 * s + 4 * lane;
    uint32_t m = 0u, bytes = 0u;
    if (mode & M_FROMMAPS) {
      m = mk[s];
    } else if (swar) {
      const uint32_t we = wv[s] & 0x00ff00ffu, wo = (wv[s] >> 8) & 0x00ff00ffu;
      const uint32_t be = bv[s] & 0x00ff00ffu, bo = (bv[s] >> 8) & 0x00ff00ffu;
      const uint32_t me = ((we | 0x80008000u) - tw2) & (((we + 0x00100010u) | 0x80008000u) - (be + tc2));
      const uint32_t mo = ((wo | 0x80008000u) - tw2) & (((wo + 0x00100010u) | 0x80008000u) - (bo + tc2));
      bytes = px < HW ? ((me >> 15) & 0x00010001u) | ((mo >> 7) & 0x01000100u) : 0u;
      m = (bytes & 1u) | ((bytes >> 7) & 2u) | ((bytes >> 14) & 4u) | ((bytes >> 21) & 8u);
    } else {
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int w = static_cast<int>((wv[s] >> (8 * e)) & 0xffu);
        const int b = static_cast<int>((bv[s] >> (8 * e)) & 0xffu);
        m |= (px + e < HW && w > thr_w && w - b > thr_c) ? (1u << e) : 0u;
      }
      bytes = (m & 1u) | ((m & 2u) << 7) | ((m & 4u) << 14) | ((m & 8u) << 21);
    }
    ok[s] = m;
    mbytes[s] = bytes;
    if ((mode & M_MAPS) && (!vec || !codes)) {
      uint8_t* mo_ = p.mask_out + static_cast<int64_t>(view) * HW;
      if (vec) {
        if (px < HW) *reinterpret_cast<uint32_t*>(mo_ + px) = bytes;
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (px + e < HW) mo_[px + e] = static_cast<uint8_t>((m >> e) & 1u);
      }
    }
  }
  if (p.masked) *masked = __popc(ok[0]) + __popc(ok[1]) + __popc(ok[2]) + __popc(ok[3]);
  if (!codes) return 0;

  // ---- |n.r| > 1e-6 for the masked pixels ----
  // gathers per step, two steps at a time (the scheduling barrier keeps the
  // second pair's gathers out of the first pair's registers: 4 waves / SIMD)
  const int v_c = cpx / W, u_c = cpx - v_c * W;  // chunk origin
  int total = 0;
  uint32_t nibs[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    if (s == 2) __builtin_amdgcn_sched_barrier(0);
    float4 pf[4];
    float xs[4], ys;
    int us, vs;
    {
      // pixel (u, v) of cpx + 256 s + 4 lane, 32-bit stepping from the origin;
      // tail pixels past the frame are clamped to its last 4 (vec) / 1 pixel
      int u = u_c + 256 * s + 4 * lane, v = v_c;
      while (u >= W) {
        u -= W;
        ++v;
      }
      if (v >= p.H) {
        v = p.H - 1;
        u = vec ? W - 4 : W - 1;
      }
      us = u;
      vs = v;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const unsigned c = (rc[s][e >> 1] >> (16 * (e & 1))) & 0x7fffu;
        pf[e] = (kAblate & 128) ? make_float4(0.5f, 0.25f, 1.0f + 1e-3f * c, 0.0f) : p.planes32[c];
      }
      ys = 0.0f;
      if (!nc) {
        if (vec) {
          const float4 x4 = *reinterpret_cast<const float4*>(p.xn32 + us);
          xs[0] = x4.x;
          xs[1] = x4.y;
          xs[2] = x4.z;
          xs[3] = x4.w;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) xs[e] = p.xn32[(us + e) % W];
        }
        ys = p.yn32[vs];
      }
    }
    uint32_t nib = 0u;
    // Cheap sufficient test (pinhole rays): with L = |x| + |y| + 1 >= |(x, y, 1)|
    // and a = |n.(x, y, 1)| in f32 (error < sum|n_i| L 2^-20, the inputs' f32
    // rounding included), a > L (1.001e-6 + sum|n_i| 2^-20) implies |n.r| >
    // 1.001e-6 for the exact ray, clear of the reference's f64 rounding.
    // p.fast_thr is that right-hand side at the frame's largest L and the
    // table's largest sum|n_i| (sl_set_calib, rounded up): one compare per
    // pixel.  Masked pixels that fail it take the bounded test below.
    uint32_t todo = ok[s];
    if (kAblate & 64) {
      nib = todo;
      todo = 0u;
    } else if (vec && !nc) {
      uint32_t fast = 0u;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float4 f = pf[e];
        const float a = fabsf(__builtin_fmaf(f.x, xs[e], __builtin_fmaf(f.y, ys, f.z)));
        fast |= (a > p.fast_thr) ? (1u << e) : 0u;
      }
      nib = todo & fast;
      todo &= ~fast;
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      if (!((todo >> e) & 1u)) continue;
      {
        const int c = static_cast<int>((rc[s][e >> 1] >> (16 * (e & 1))) & 0x7fffu);
        int u = us + e, v = vs;
        if (!vec && u >= W) {
          u -= W;
          ++v;
        }
        const int64_t q = static_cast<int64_t>(cpx) + 256 * s + 4 * lane + e;
        float x, y, z, inv;
        if (nc) {
          x = static_cast<float>(p.nc_rays[q]);
          y = static_cast<float>(p.nc_rays[p.HW + q]);
          z = static_cast<float>(p.nc_rays[2 * p.HW + q]);
          inv = 1.0f;
        } else {
          x = xs[e];
          y = vec ? ys : p.yn32[v];
          z = 1.0f;
          inv = __frsqrt_rn(x * x + y * y + 1.0f);
        }
        if (has_point(p, mode, pf[e], c, x, y, z, inv, u, v, q)) nib |= 1u << e;
      }
    }
    total += __popc(nib);
    nibs[s] = nib;
  }
  // stores last (after every gather of the wave): the point nibbles of (step
  // s, lane), one byte each in pixel order within the chunk, and the mask map
#pragma unroll
  for (int s = 0; s < 4; ++s) p.ptnib[gc * kChunkNib + 64 * s + lane] = static_cast<uint8_t>(nibs[s]);
  if ((mode & M_MAPS) && vec) {
    uint8_t* mo_ = p.mask_out + static_cast<int64_t>(view) * HW;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int px = cpx + 256 * s + 4 * lane;
      if (px < HW) *reinterpret_cast<uint32_t*>(mo_ + px) = mbytes[s];
    }
  }
  total = wave_sum(total);
  if (lane == 0) p.chunk_counts[gc] = total;
  return total;
}

// k_count: one chunk per wave, grid (chunk groups of 4, views); the
// workgroup's point total goes to block_sums for k_cloud's offsets.
#ifndef SLGPU_COUNT_WAVES
#define SLGPU_COUNT_WAVES 1
#endif
template <int VEC>
__global__ __launch_bounds__(kThreads, SLGPU_COUNT_WAVES) void k_count(Params p) {
  __shared__ int s_sum[kWaves];
  __shared__ int s_msum[kWaves];
  const int lane = threadIdx.x & 63;
  const int wid = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave-uniform, provably
  const int view = blockIdx.y;
  const int civ = blockIdx.x * kWaves + wid;
  const int64_t gc = static_cast<int64_t>(view) * p.cpv + civ;
  int mc = 0;
  const int total = count_chunk<VEC>(p, gc, view, civ, lane, civ < p.cpv, &mc);
  if (p.masked) {  // (uniform) the workgroup's masked pixels: one global add
    mc = wave_sum(mc);
    if (lane == 0) s_msum[wid] = mc;
    __syncthreads();
    if (threadIdx.x == 0) {
      int t = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) t += s_msum[w];
      if (t) atomicAdd(p.masked + view, static_cast<unsigned long long>(t));
    }
  }
  if (!(p.mode & M_CODES)) return;  // uniform: no barrier below
  if (lane == 0) s_sum[wid] = total;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) t += s_sum[w];
    const int64_t blk = static_cast<int64_t>(view) * gridDim.x + blockIdx.x;
    p.block_sums[blk] = t;
    if (t) atomicAdd(p.super_sums + (blk >> p.sb_shift), static_cast<unsigned>(t));
  }
}

// ================================================================= k_cloud ====
// reconstruct_point_cloud's arithmetic (sl_system.py:584-653) for the points
// k_count marked, one chunk per wave:
//   0. the chunk's offset in the merged cloud: the super-block sums before its
//      super-block + the chunk counts before it inside it (+ earlier launch
//      groups);
//   1. records + colour of the lane's 16 pixels (16-byte loads); the lane's
//      point count and its exclusive prefix over the wave give every point its
//      rank in the chunk (ascending pixel order, np.where, sl_system.py:601);
//   2. each point's (pixel, column code) and BGR go to LDS at its rank -- the
//      chunk's points, compacted;
//   3. kPipe x 64 points per pass: lane j takes points j, j+64, ...; all their
//      operand gathers (ray tables or Nc, plane) are issued before any point
//      is computed, then the exact f64 arithmetic in the reference's operation
//      order, then the stores at offset + rank (64 consecutive points per store
//      instruction).
#ifndef SLGPU_PIPE
#define SLGPU_PIPE 4
#endif
constexpr int kPipe = SLGPU_PIPE;  // points per lane per pass in k_cloud
#ifndef SLGPU_POSE_COARSE
#define SLGPU_POSE_COARSE 1
#endif
constexpr bool kPoseCoarse = SLGPU_POSE_COARSE != 0;  // posed verified route: the coarse bound of M_k (A/B)
#ifndef SLGPU_SMALL_PIPE
#define SLGPU_SMALL_PIPE 4
#endif
constexpr int kSmallPipe = SLGPU_SMALL_PIPE;  // ... in launches of at most one chunk per SIMD (f32-fast)
#ifndef SLGPU_STAGE_OUT
#define SLGPU_STAGE_OUT 0
#endif
constexpr bool kStageOut = SLGPU_STAGE_OUT != 0;  // f32 points leave through an LDS stage
#ifndef SLGPU_LDS_BGR
#define SLGPU_LDS_BGR 2
#endif
// colour of a point: 1 = compacted with the entries in LDS, 2 = the chunk's
// texture bytes in LDS in pixel order (3 B/px; 12 KB less LDS per workgroup
// than 1), 0 = re-read from the texture in global memory
constexpr int kBgrMode = SLGPU_LDS_BGR;
constexpr bool kLdsBgr = kBgrMode == 1;
constexpr bool kTexLds = kBgrMode == 2;
constexpr int kBgrWords = kLdsBgr ? kChunk : kTexLds ? 3 * kChunk / 4 + 4 : 4;  // u32 per wave
#ifndef SLGPU_TEX_COAL
#define SLGPU_TEX_COAL 0
#endif
// k_cloud's texture loads as 1-KB rows of the chunk (each instruction whole
// lines) instead of each lane's own 48 bytes (kTexLds only: the LDS copy is in
// pixel order either way)
constexpr bool kTexCoal = SLGPU_TEX_COAL != 0 && kTexLds;
#ifndef SLGPU_COL_DWORD
#define SLGPU_COL_DWORD 0
#endif
// (measurement build, SLGPU_COL_DWORD=1: k_cloud's colour bytes staged per
// pass in LDS, 3 per point shifted to the pass's alignment in the output,
// then stored 8 bytes per lane.  The byte / short stores of 3-byte colours
// cost 4x the xyz stores per byte -- kbench, 8 4K views: 46 of 262 us for 157
// MB of colours, 75 us for 629 MB of xyz -- but the stage costs more: k_cloud
// 262 -> 328 us, c2 30.4 -> 46.3 us; bit-exact, 204 GPU tests)
constexpr bool kColDword = SLGPU_COL_DWORD != 0;
#ifndef SLGPU_COL_OVERLAP
#define SLGPU_COL_OVERLAP 0
#endif
// (measurement build, SLGPU_COL_OVERLAP=1: k_cloud's colours as one 4-byte
// store per point at its 3-byte slot, an unaligned buffer store whose 4th
// byte is the next point's first colour byte -- taken from the next lane by
// DPP, so both lanes writing that byte write the same value; the chunk's last
// point writes its 3 bytes alone.  One store instruction per 64 points instead
// of two, bit-exact (204 GPU tests), but slower: k_cloud 261.7 -> 264.0 us
// for 8 4K views, c2 step 120.6 -> 122.3-123.6 us)
constexpr bool kColOverlap = SLGPU_COL_OVERLAP != 0;
constexpr int kColStage = 64 * 4 * 3 + 16;  // bytes per wave: up to 4 x 64 points + alignment


// base + a 32-bit byte offset: the form global loads / stores take with an
// SGPR base (wave-uniform pointer) and a 32-bit VGPR offset
template <typename T>
__device__ __forceinline__ T* at_bytes(T* base, unsigned off) {
  using B = typename std::conditional<std::is_const<T>::value, const char, char>::type;
  return reinterpret_cast<T*>(reinterpret_cast<B*>(base) + off);
}

// Pixel (u, v) of the entry's chunk-local pixel (the chunk starts at (u_c,
// v_c)): the 16-byte path carries the row offset in the entry; otherwise one
// row wrap at most when W >= kChunk (wave-uniform test), else a loop.
__device__ __forceinline__ uint32_t ent_code(uint32_t e) { return (e >> 10) & 0x7fffu; }
// The range facts let the table gathers use 32-bit offsets.
template <int VEC>
__device__ __forceinline__ void chunk_uv(int u_c, int v_c, uint32_t e, int W, int* u, int* v) {
  const int local = static_cast<int>(e & 1023u);
  int uu = u_c + local, vv = v_c;
  if (VEC > 0) {  // the entry's row offset (cloud_chunk)
    const int dr = static_cast<int>(e >> 25);
    uu -= dr * W;
    vv += dr;
  } else if (W >= kChunk) {
    const bool wrap = uu >= W;
    uu -= wrap ? W : 0;
    vv += wrap ? 1 : 0;
  } else {
    while (uu >= W) {
      uu -= W;
      ++vv;
    }
  }
  __builtin_assume(uu >= 0 && uu < (1 << 24));
  __builtin_assume(vv >= 0 && vv < (1 << 24));
  *u = uu;
  *v = vv;
}

// A lane's inputs of one k_cloud chunk: records, colour bytes, point bits.
struct ChunkIn {
  uint32_t d[kPx / 2];  // records (clipped column codes), 2 per word
  uint4 tq[3];          // BGR bytes of the 16 pixels (or the white plane's in tq[0])
  uint32_t ptbits;      // point bits of the 16 pixels (bit k: pixel 16 lane + k)
};

// Phase 1 of a chunk (global index gc): the lane's loads, issued by k_cloud
// before its block-offset loads so that both round trips overlap.
template <int VEC>
__device__ __forceinline__ void cloud_load(const Params& p, int64_t gc, int lane, ChunkIn* in) {
  const bool vec = VEC > 0;
  const int view = static_cast<int>(gc / p.cpv);
  const int civ = static_cast<int>(gc - static_cast<int64_t>(view) * p.cpv);
  const int64_t HW = p.HW;
  const int64_t px0 = static_cast<int64_t>(civ) * kChunk + lane * kPx;
  const int n_px = static_cast<int>(min<int64_t>(max<int64_t>(HW - px0, 0), kPx));
  const int64_t pxl = n_px > 0 ? px0 : 0;
  uint32_t* d = in->d;
  if (p.rec_col) {  // the col map k_decode wrote, clipped (sl_system.py:626)
    const int32_t* src = p.rec_col + view * HW + pxl;
    const uint32_t cmax = static_cast<uint32_t>(p.Wp - 1);
    uint32_t c[kPx];
    if (vec) {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const uint4 q = ld_side16(src + 4 * i);
        c[4 * i] = q.x;
        c[4 * i + 1] = q.y;
        c[4 * i + 2] = q.z;
        c[4 * i + 3] = q.w;
      }
    } else {
#pragma unroll
      for (int k = 0; k < kPx; ++k) c[k] = k < n_px ? static_cast<uint32_t>(src[k]) : 0u;
    }
#pragma unroll
    for (int i = 0; i < kPx / 2; ++i) d[i] = min(c[2 * i], cmax) | (min(c[2 * i + 1], cmax) << 16);
  } else if (vec && p.rec12) {  // 12-bit records (k_decode): 8 codes per 3 words
    in->ptbits = 0u;
    uint32_t w[6];
    if (p.rec_blk) {  // the chunk's slot: words 0-3 at 16 lane, 4-5 at 1024 + 8 lane
      const uint8_t* cb = reinterpret_cast<const uint8_t*>(p.codes) + kRecSlot * rec_slot(p, view, civ);
      const uint4 a = ld_side16(cb + 16 * lane);
      const uint2 b = ld_side8(cb + 1024 + 8 * lane);
      w[0] = a.x; w[1] = a.y; w[2] = a.z; w[3] = a.w; w[4] = b.x; w[5] = b.y;
    } else {
      const uint2* src = reinterpret_cast<const uint2*>(reinterpret_cast<const uint8_t*>(p.codes) +
                                                        3 * (view * HW + pxl) / 2);  // 24 B, 8-byte aligned
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const uint2 q = ld_side8(src + i);
        w[2 * i] = q.x;
        w[2 * i + 1] = q.y;
      }
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const uint32_t x = w[3 * h], y = w[3 * h + 1], z = w[3 * h + 2];
      const uint32_t c0 = x & 0xfffu, c1 = (x >> 12) & 0xfffu;
      const uint32_t c2 = __builtin_amdgcn_alignbit(y, x, 24) & 0xfffu, c3 = (y >> 4) & 0xfffu;
      const uint32_t c4 = (y >> 16) & 0xfffu, c5 = __builtin_amdgcn_alignbit(z, y, 28) & 0xfffu;
      const uint32_t c6 = (z >> 8) & 0xfffu, c7 = z >> 20;
      d[4 * h] = c0 | (c1 << 16);
      d[4 * h + 1] = c2 | (c3 << 16);
      d[4 * h + 2] = c4 | (c5 << 16);
      d[4 * h + 3] = c6 | (c7 << 16);
      const uint32_t pb = (c0 != 0xfffu) | ((c1 != 0xfffu) << 1) | ((c2 != 0xfffu) << 2) | ((c3 != 0xfffu) << 3) |
                          ((c4 != 0xfffu) << 4) | ((c5 != 0xfffu) << 5) | ((c6 != 0xfffu) << 6) | ((c7 != 0xfffu) << 7);
      in->ptbits |= pb << (8 * h);
    }
    if (n_px < kPx) in->ptbits = 0u;  // lanes past the view's end (their loads read pixel 0's records)
  } else {
    const uint16_t* src = p.codes + view * HW + pxl;
    if (vec) {
      const uint4 a = ld_side16(src);
      const uint4 b = ld_side16(src + 8);
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
  }
  // colour: BGR texture, or the white plane replicated (the colour imread of a
  // single-channel file 0, sl_system.py:580)
  uint4* tq = in->tq;
  if (p.tex != nullptr) {
    const uint8_t* t = p.tex + view * p.tex_vs + 3 * pxl;
    if (vec && kTexCoal) {
      // the chunk's 3 KB of texture as three 1-KB rows (lane: 16 B at 16 lane
      // + 1024 i), so that each load instruction covers whole lines; k_cloud
      // stores them to LDS at the same offsets (pixel order, kTexLds).  Rows
      // past the view's texture (its last, partial chunk) re-read its last 16
      // bytes: those pixels make no points.
      const int64_t tv = 3 * HW;
      const uint8_t* tb = p.tex + view * p.tex_vs;
      const int64_t c0 = 3 * static_cast<int64_t>(civ) * kChunk + 16 * lane;
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const uint8_t* a = tb + min<int64_t>(c0 + 1024 * i, tv - 16);
        if (SLGPU_NT_TEX) {
          const v4u q = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(a));
          tq[i] = make_uint4(q.x, q.y, q.z, q.w);
        } else {
          tq[i] = ld_side16(a);
        }
      }
    } else if (vec && SLGPU_NT_TEX) {  // (A/B) non-temporal texture loads (read once)
#pragma unroll
      for (int i = 0; i < 3; ++i) {
        const v4u q = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(t + 16 * i));
        tq[i] = make_uint4(q.x, q.y, q.z, q.w);
      }
    } else if (vec) {
      tq[0] = ld_side16(t);
      tq[1] = ld_side16(t + 16);
      tq[2] = ld_side16(t + 32);
    } else {
      tq[0] = ld16(t, 3 * n_px, false);
      tq[1] = ld16(t + 16, 3 * n_px - 16, false);
      tq[2] = ld16(t + 32, 3 * n_px - 32, false);
    }
  } else {
    tq[0] = ld16(p.stack + view * p.stack_vs + pxl, n_px, vec);
    tq[1] = tq[2] = make_uint4(0u, 0u, 0u, 0u);
  }
  // the lane's 16 point bits (k_count): the nibbles of pixels 16 l .. 16 l + 15,
  // bytes 64 (l / 16) + 4 (l % 16) + 0..3 of the chunk
  if (!(vec && p.rec12)) {
    const uint32_t nb4 = *reinterpret_cast<const uint32_t*>(p.ptnib + gc * kChunkNib + 64 * (lane >> 4) + 4 * (lane & 15));
    in->ptbits = (nb4 & 0xfu) | ((nb4 >> 4) & 0xf0u) | ((nb4 >> 8) & 0xf00u) | ((nb4 >> 12) & 0xf000u);
  }
}

// Phases 2-3 of a chunk (global index gc, output offset base), by one wave,
// from the lane's loads.
template <int MODE, int VEC, int PIPE>
__device__ __forceinline__ void cloud_points(const Params& p, int view, int64_t cpx, long long base, int lane,
                                             int total, const uint32_t* s_ent, const uint32_t* s_bgr,
                                             float* s_sxyz, uint8_t* s_scol, bool col_stage);

template <int MODE, int VEC, int PIPE>
__device__ __forceinline__ void cloud_chunk(const Params& p, int64_t gc, long long base, int lane, const ChunkIn& in,
                                            uint32_t* s_ent, uint32_t* s_bgr, float* s_sxyz, uint8_t* s_scol, bool col_stage = false) {
  const int view = static_cast<int>(gc / p.cpv);
  const int civ = static_cast<int>(gc - static_cast<int64_t>(view) * p.cpv);
  const int64_t cpx = static_cast<int64_t>(civ) * kChunk;  // chunk's first pixel
  const int mode = MODE >= 0 ? MODE : p.mode;
  const bool has_tex = (mode & M_TEX) != 0;
  // 16-byte path (W % 16 == 0, W >= 64): a lane's 16 pixels share one image
  // row, at most 17 rows below the chunk's first; the row offset rides in
  // the entry (bits 25..29) so that cloud_points needs no division
  uint32_t drow = 0u;
  if (VEC > 0) {
    const int px = static_cast<int>(cpx) + lane * kPx;  // < HW < 2^31
    drow = static_cast<uint32_t>(px / p.W - static_cast<int>(cpx) / p.W) << 25;
  }
  const uint32_t* d = in.d;
  const uint4* tq = in.tq;
  const uint32_t ptbits = in.ptbits;
  __builtin_amdgcn_wave_barrier();  // the previous chunk's LDS reads come first
  const int n_l = __popc(ptbits);
  const int incl = wave_incl_scan(n_l, lane);
  const int total = __shfl(incl, 63, 64);
  if (lane == 0 && civ == 0) p.view_offsets[view] = base;
  // offsets past the caller's capacity can only come from scratch out of
  // phase with its launches (e.g. a captured graph replayed when its launch
  // count is not a multiple of the scratch rotations, slgpu.h): write nothing
  // (the call's total then exceeds the capacity, which the host reports)
  if (base < 0 || base + total > p.out_cap) return;
  if (kAblate & 8) {  // measurement only: stop after the loads and the rank scan
    if (total == -1) p.bgr[0] = static_cast<uint8_t>(d[0] ^ tq[0].x ^ tq[1].y ^ tq[2].z);
    return;
  }

  // ---- 2. compacted entries in LDS (and the chunk's colours, kTexLds) ----
  if (kTexLds) {
    uint4* t4 = reinterpret_cast<uint4*>(s_bgr);
    if (has_tex && kTexCoal && VEC > 0) {  // (cloud_load's 1-KB rows)
      t4[lane] = tq[0];
      t4[64 + lane] = tq[1];
      t4[128 + lane] = tq[2];
    } else if (has_tex) {
      t4[3 * lane] = tq[0];
      t4[3 * lane + 1] = tq[1];
      t4[3 * lane + 2] = tq[2];
    } else {
      t4[lane] = tq[0];  // gray bytes, one per pixel
    }
  }
  {
    int idx = incl - n_l;
#pragma unroll
    for (int k = 0; k < kPx; ++k) {
      const uint32_t code = (d[k >> 1] >> (16 * (k & 1))) & 0x7fffu;
      uint32_t bgr;
      if (has_tex) {
        const int b = 3 * k;
        bgr = byte_of(tq[b >> 4], b & 15) | (byte_of(tq[(b + 1) >> 4], (b + 1) & 15) << 8) |
              (byte_of(tq[(b + 2) >> 4], (b + 2) & 15) << 16);
      } else {
        bgr = byte_of(tq[0], k) * 0x010101u;
      }
      if ((ptbits >> k) & 1u) {
        s_ent[idx] = static_cast<uint32_t>(lane * kPx + k) | (code << 10) | drow;
        if (kLdsBgr) s_bgr[idx] = bgr;
        (void)bgr;
      }
      idx += (ptbits >> k) & 1u;
    }
  }
  __builtin_amdgcn_wave_barrier();
  if (kAblate & 16) return;  // measurement only: stop after the LDS compaction

  cloud_points<MODE, VEC, PIPE>(p, view, cpx, base, lane, total, s_ent, s_bgr, s_sxyz, s_scol, col_stage);
}

// Phase 3 of a chunk: its `total` compacted points (s_ent: pixel | code << 10
// | row offset << 25 on the 16-byte path, s_bgr: colour) -> xyz + BGR at
// offset base + rank, kPipe x 64 per pass.
template <int MODE, int VEC, int PIPE>
__device__ __forceinline__ void cloud_points(const Params& p, int view, int64_t cpx, long long base, int lane,
                                             int total, const uint32_t* s_ent, const uint32_t* s_bgr,
                                             float* s_sxyz, uint8_t* s_scol, bool col_stage) {
  constexpr int kPipe = PIPE;  // points per lane per pass
  const int mode = MODE >= 0 ? MODE : p.mode;
  const int64_t HW = p.HW;
  const bool has_tex = (mode & M_TEX) != 0;
  // r = (x, y, 1) / sqrt((x*x + y*y) + 1) (sl_system.py:614-621) or Nc
  // (:605-606), plane of the clipped code (:624-633), den = (n0 r0 + n1 r1) +
  // n2 r2 (:638), t = -(n.Oc + d) / den (:639, :643; n.Oc + d per plane,
  // precomputed in the same order), P = Oc + r t (:648); optional pose.
  const int W = p.W;
  const int u_c = static_cast<int>(cpx % W);
  const int v_c = static_cast<int>(cpx / W);
  const double* pose = p.poses ? p.poses + 16 * view : nullptr;
  // the view's pose rows, once per chunk into wave-uniform registers (read
  // through `pose` inside the point loop they were re-loaded per point)
  // (M_VERIFY: pb_k = 2^-44 sum_j |m_kj|, pt_k = 2^-44 |m_k3|, the settle
  // test's interval half-width scale, by exponent arithmetic on the uniform
  // bits (scalar registers, none of the 12 VGPRs a VALU product would hold):
  // exact, or 2^-999 where the product would be tinier -- a wider interval)
  auto scale_2m44 = [](double v) -> double {  // v >= 0, wave-uniform
    const unsigned long long b = static_cast<unsigned long long>(__double_as_longlong(v));
    const unsigned e = static_cast<unsigned>(b >> 52) & 0x7ffu;
    // (e <= 67: v < 2^-955, so 2^-44 v < 2^-999, the value returned)
    return __longlong_as_double(static_cast<long long>(e > 67u ? b - (44ull << 52) : (24ull << 52)));
  };
  double pm[12], pb[3] = {0.0, 0.0, 0.0}, pt[3] = {0.0, 0.0, 0.0};
  if (pose) {
#pragma unroll
    for (int k = 0; k < 12; ++k) pm[k] = uniform_f64(pose[k]);
#pragma unroll
    for (int k = 0; k < 3; ++k) {
      pb[k] = scale_2m44(uniform_f64((fabs(pm[4 * k]) + fabs(pm[4 * k + 1])) + fabs(pm[4 * k + 2])));
      pt[k] = scale_2m44(uniform_f64(fabs(pm[4 * k + 3])));
    }
  }
  const bool f64out = (mode & M_XYZ64) != 0;
  constexpr int dbg = kAblate;
  auto point_bgr = [&](int j, int local) -> uint32_t {
    if (kLdsBgr) return s_bgr[j];
    if (kTexLds) {
      if (has_tex) {  // bytes 3 local .. 3 local + 2 of the chunk's BGR
        const int b = 3 * local;
        const uint32_t w0 = s_bgr[b >> 2], w1 = s_bgr[(b >> 2) + 1];
        return __builtin_amdgcn_alignbyte(w1, w0, static_cast<unsigned>(b & 3)) & 0xffffffu;
      }
      return ((s_bgr[local >> 2] >> (8 * (local & 3))) & 0xffu) * 0x010101u;
    }
    if (has_tex) {
      const uint8_t* t = p.tex + view * p.tex_vs + 3 * (cpx + local);
      return t[0] | (static_cast<uint32_t>(t[1]) << 8) | (static_cast<uint32_t>(t[2]) << 16);
    }
    return static_cast<uint32_t>(p.stack[view * p.stack_vs + cpx + local]) * 0x010101u;
  };
  float* const wx = static_cast<float*>(p.xyz) + 3 * base;  // the chunk's first point (wave-uniform)
  uint8_t* const wc = p.bgr + 3 * base;
  // (kColOverlap) the chunk's colour bytes [3 base, 3 (base + total)) as a
  // buffer: SGPR base, 32-bit lane offsets, nothing written past its end
  const __amdgpu_buffer_rsrc_t rs_col = __builtin_amdgcn_make_buffer_rsrc(wc, 0, 3 * total, 0x00020000);
  for (int j0 = 0; j0 < total; j0 += 64 * kPipe) {
    if (mode & M_FAST32) {
      // SL_XYZ_F32_FAST (Oc = 0, pinhole rays, no pose; host-checked): the
      // same formula in f32 -- rsq-normalised ray, f32 plane, rcp -- for
      // points whose condition number kappa = sum|n_i r_i| / |n.r| is at most
      // kFastKappa; the rest take the exact f64 route below.  Per-coordinate
      // relative error vs the reference's f64 <= (11 + 10 kappa) 2^-24
      // ("f32-fast").
      float fx[kPipe], fy[kPipe];
      float4 fp[kPipe];
      uint32_t bgr[kPipe];
#pragma unroll
      for (int i = 0; i < kPipe; ++i) {
        const int j = min(j0 + 64 * i + lane, total - 1);
        const uint32_t e = s_ent[j];
        const int local = static_cast<int>(e & 1023u);
        bgr[i] = point_bgr(j, local);
        int uu, vv;
        chunk_uv<VEC>(u_c, v_c, e, W, &uu, &vv);
        if (kAblate & 512) {  // measurement only: no table gathers
          fx[i] = 0.001f * static_cast<float>(uu);
          fy[i] = 0.001f * static_cast<float>(vv);
          fp[i] = make_float4(0.1f, 0.2f, 0.9f, -500.0f - static_cast<float>(ent_code(e)));
          continue;
        }
        fx[i] = *at_bytes(p.xn32, 4u * static_cast<unsigned>(uu));
        fy[i] = *at_bytes(p.yn32, 4u * static_cast<unsigned>(vv));
        fp[i] = p.planes32[ent_code(e)];
      }
#pragma unroll
      for (int i = 0; i < kPipe; ++i) {
        const int j = j0 + 64 * i + lane;
        const float x = fx[i], y = fy[i];
        const float inv = __builtin_amdgcn_rsqf((x * x + y * y) + 1.0f);
        const float r0 = x * inv, r1 = y * inv;
        const float a0 = fp[i].x * r0, a1 = fp[i].y * r1, a2 = fp[i].z * inv;
        const float den = (a0 + a1) + a2;
        const float S = (fabsf(a0) + fabsf(a1)) + fabsf(a2);
        float X, Y, Z;
        if (S <= kFastKappa * fabsf(den)) {
          const float t = -fp[i].w * __builtin_amdgcn_rcpf(den);
          X = 0.0f + r0 * t;  // o + r t with o = +0: -0 becomes +0 as in f64
          Y = 0.0f + r1 * t;
          Z = 0.0f + inv * t;
        } else {  // ill-conditioned: exact f64, as the path below
          const uint32_t e = s_ent[min(j, total - 1)];
          int uu, vv;
          chunk_uv<VEC>(u_c, v_c, e, W, &uu, &vv);
          const double xd = p.xn[uu], yd = p.yn[vv];
          const double4 pd = p.planes[ent_code(e)];
          const double nrm = sqrt((xd * xd + yd * yd) + 1.0);
          const double d0 = xd / nrm, d1 = yd / nrm, d2 = 1.0 / nrm;
          const double td = -pd.w / ((pd.x * d0 + pd.y * d1) + pd.z * d2);
          X = static_cast<float>(p.o0 + d0 * td);
          Y = static_cast<float>(p.o1 + d1 * td);
          Z = static_cast<float>(p.o2 + d2 * td);
        }
        if (kAblate & 256) {  // measurement only: no point stores (results kept live)
          if (X == -1234.5f && Y == Z) p.bgr[0] = static_cast<uint8_t>(bgr[i]);
        } else if (j < total) {
          float* xyz = at_bytes(wx, 12u * static_cast<unsigned>(j));
          xyz[0] = X;
          xyz[1] = Y;
          xyz[2] = Z;
          uint8_t* cc = at_bytes(wc, 3u * static_cast<unsigned>(j));
          cc[0] = static_cast<uint8_t>(bgr[i]);
          cc[1] = static_cast<uint8_t>(bgr[i] >> 8);
          cc[2] = static_cast<uint8_t>(bgr[i] >> 16);
        }
      }
      continue;
    }
    double ra[kPipe], rb[kPipe], rcz[kPipe];  // pinhole: x, y, -; Nc: r0, r1, r2
    double4 pl[kPipe];
    uint32_t bgr[kPipe];
#pragma unroll
    for (int i = 0; i < kPipe; ++i) {
      const int j = min(j0 + 64 * i + lane, total - 1);  // past the end: repeat the last point
      const uint32_t e = s_ent[j];
      const int local = static_cast<int>(e & 1023u);
      bgr[i] = point_bgr(j, local);
      const unsigned c = ent_code(e);
      if (dbg & 4) {
        ra[i] = 0.25 + local;
        rb[i] = 0.5;
        rcz[i] = 1.0;
        pl[i] = make_double4(0.1, 0.2, 0.9, -500.0 - c);
        continue;
      }
      if (mode & M_NC) {
        const int64_t q = cpx + local;
        ra[i] = p.nc_rays[q];
        rb[i] = p.nc_rays[HW + q];
        rcz[i] = p.nc_rays[2 * HW + q];
      } else {
        int uu, vv;
        chunk_uv<VEC>(u_c, v_c, e, W, &uu, &vv);
        if (mode & M_VERIFY) {
          // the verified route's x, y: (w - c) * fl(1 / f), within 3 u of the
          // table values (its error bound allows it; the
          // fallback re-reads the tables)
          ra[i] = (static_cast<double>(uu) - p.cx) * p.rfx;
          rb[i] = (static_cast<double>(vv) - p.cy) * p.rfy;
        } else if (kXyCalc && p.xy_calc) {  // (uniform) the table values, computed: no 16 B of gathers per point
          ra[i] = xy_of(uu, p.cx, p.fx);  // (gathering x or y instead: +0.8 / +1.1 us at c2)
          rb[i] = xy_of(vv, p.cy, p.fy);
        } else {
          ra[i] = p.xn[uu];
          rb[i] = p.yn[vv];
        }
      }
      pl[i] = p.planes[(dbg & 1024) ? (c & 31u) : c];  // (1024: measurement only, a 1-KB plane table)
    }
    double X[kPipe], Y[kPipe], Z[kPipe];
    uint32_t slow = 0u;
    if (dbg & 4096) {  // measurement only: no point arithmetic at all (operands stored as the point)
#pragma unroll
      for (int i = 0; i < kPipe; ++i) {
        X[i] = ra[i];
        Y[i] = rb[i];
        Z[i] = pl[i].w + pl[i].x;
      }
    } else {
    if (mode & M_VERIFY) {
      // SL_XYZ_F32 output is float32(P_ref), P_ref the reference's f64 value
      // (sl_system.py:614-648 with Oc = 0, pinhole rays, no pose).  With
      // v = (x, y, 1) and r = v / |v|, P = r t = v q where q = -w / (n . v):
      // the ray's norm cancels, so a shorter f64 evaluation P' = v q' (q' by
      // reciprocal + two Newton steps, no sqrt, no normalisation) gives the
      // same float32 whenever no float32 rounding midpoint lies between P'
      // and P_ref.  Error bound (u = 2^-53, kappa = sum|n_i v_i| / |n . v| =
      // sum|n_i r_i| / |n . r|): the reference's chain (s2: 3u, |v|: 2.5u,
      // r: 3.5u, den: 6.5u kappa, t: +u, P: +u) is within (5.5 + 6.5 kappa) u
      // |P| of the exact P; P' (its x, y within 3u of the tables', below)
      // within (7 + 6 kappa) u |P|, so |P' - P_ref| <= (12.5 + 12.5 kappa) u
      // |P| < 2^7.8 u |P| < 2^8 f64 ulps of P for kappa <= 16.  A coordinate whose 29 dropped mantissa bits lie within 2^13
      // ulps of the midpoint pattern 2^28, or outside 2^-100 <= |P'| < 2^100
      // (zeros, signs of zero, inf / NaN), or a point with kappa > 16 goes to
      // the operators' sequences below (the host takes the route only for
      // plane tables with |w| >= 2^-500 and max|n_i| >= 2^-400, so that
      // sum|n_i v_i| >= 2^-420: planes_plain):
      // the stored float32 is the reference's bit for bit either way
      // (tests/test_gpu_parity.py compares the two routes).
      // (bitwise, not short-circuit: the tests stay branch-free VALU / SALU.
      // The host takes this route only when every table x, y has 2^-20 <=
      // |x|, |y| <= 2^20 (xy_plain), so 2^-80 <= |Z| < 2^80 puts X, Y and Z
      // in 2^-100 .. 2^100: normal float32 values, no zeros)
      auto ambiguous = [](double v) -> unsigned {
        const unsigned lo = static_cast<unsigned>(__double_as_longlong(v)) & 0x1fffffffu;
        return (lo - (0x10000000u - 8192u)) <= 16384u;
      };
      auto out_of_range = [](double v) -> unsigned {  // not 2^-80 <= |v| < 2^80 (NaN included)
        return static_cast<unsigned>(!(fabs(v) >= 0x1p-80)) | static_cast<unsigned>(!(fabs(v) < 0x1p80));
      };
#pragma unroll
      for (int i = 0; i < kPipe; ++i) {
        const double x = ra[i], y = rb[i];
        // n . v and sum |n_i v_i| by fused multiply-adds: two roundings each,
        // fewer than the products-then-sums the bound below allows for
        const double dv = fma(pl[i].x, x, fma(pl[i].y, y, pl[i].z));                       // n . v
        const double S = fma(fabs(pl[i].x), fabs(x), fma(fabs(pl[i].y), fabs(y), fabs(pl[i].z)));  // sum |n_i v_i|
        const double q = -pl[i].w * recip_nr(dv);
        X[i] = x * q;
        Y[i] = y * q;
        Z[i] = q;
        // (S >= 2^-420 and |w| >= 2^-500 hold for every point: planes_plain)
        unsigned bad = static_cast<unsigned>(S > 16.0 * fabs(dv)) | out_of_range(Z[i]);
        if (pose) {
          // the turntable pose (the epilogue's order, below) on P': each output
          // k is within (212.5 + 8) u M_k of the epilogue on P_ref, M_k =
          // sum_j |m_kj P_j| + |m_k3| (P' within 212.5 u |P_j| per coordinate,
          // the two evaluations' roundings 4 u M_k each) < 2^-45.2 M_k; the
          // point is settled when float32(v - B) == float32(v + B), B =
          // 2^-44 M_k, a normal float32 (then the reference's value, inside
          // that interval, has the same float32)
          auto unsettled = [](double v, double B) -> unsigned {
            const uint32_t a = __float_as_uint(static_cast<float>(v - B));
            const uint32_t b = __float_as_uint(static_cast<float>(v + B));
            return static_cast<unsigned>(a != b) | static_cast<unsigned>(((a >> 23) & 0xffu) - 1u >= 254u);
          };
          const double x0 = X[i], x1 = Y[i], x2 = Z[i];
          // (by fused multiply-adds: 3 roundings per output, within the
          // 4 u M_k the bound allows this evaluation)
          const double X2 = fma(pm[0], x0, fma(pm[1], x1, fma(pm[2], x2, pm[3])));
          const double Y2 = fma(pm[4], x0, fma(pm[5], x1, fma(pm[6], x2, pm[7])));
          const double Z2 = fma(pm[8], x0, fma(pm[9], x1, fma(pm[10], x2, pm[11])));
          double M0, M1, M2;  // 2^-44 M_k (the scale folded into pb / pt: exact)
          if (kPoseCoarse) {
            // M_k <= R_k max_j |P_j| + |m_k3| (R_k = sum_j |m_kj|, per view):
            // a wider interval, so as safe, at 4 operations instead of 18
            // (the slack of 2^-44 against the 2^-45.2 the bound needs covers
            // these few roundings)
            const double pmax = fmax(fmax(fabs(x0), fabs(x1)), fabs(x2));
            M0 = fma(pb[0], pmax, pt[0]);
            M1 = fma(pb[1], pmax, pt[1]);
            M2 = fma(pb[2], pmax, pt[2]);
          } else {
            M0 = 0x1p-44 * (((fabs(pm[0] * x0) + fabs(pm[1] * x1)) + fabs(pm[2] * x2)) + fabs(pm[3]));
            M1 = 0x1p-44 * (((fabs(pm[4] * x0) + fabs(pm[5] * x1)) + fabs(pm[6] * x2)) + fabs(pm[7]));
            M2 = 0x1p-44 * (((fabs(pm[8] * x0) + fabs(pm[9] * x1)) + fabs(pm[10] * x2)) + fabs(pm[11]));
          }
          bad |= unsettled(X2, M0) | unsettled(Y2, M1) | unsettled(Z2, M2);
          X[i] = X2;
          Y[i] = Y2;
          Z[i] = Z2;
        } else {
          bad |= ambiguous(X[i]) | ambiguous(Y[i]) | ambiguous(Z[i]);
        }
        slow |= (bad & 1u) << i;
      }
    }
    // The kPipe points' chains (sqrt, shared reciprocal, divisions) carry no
    // branch, so the compiler interleaves them: a point whose operands leave
    // the range where the shortened sequences are bit-identical to the
    // operators (div_safe) only sets its bit in `slow`, and is recomputed
    // with the operators after the loop (a branch the wave skips when no
    // lane needs it).  With a branch per point the chains ran one after the
    // other, each one's full f64 latency exposed.
    // (M_VERIFY: not compiled -- the points the verified route could not
    // settle take the operators' sequences below, one by one: a branch the
    // wave skips when no lane has one, and no registers held for the chains)
    uint32_t fallback = (mode & M_VERIFY) ? slow : 0u;  // points for the operators' own sequences
    slow = 0u;
    if (!(mode & M_VERIFY)) {
    // stage by stage over the kPipe points (the source order the scheduler
    // keeps): independent instructions of different points sit side by side
    double r0[kPipe], r1[kPipe], r2[kPipe];
    if (mode & M_NC) {
#pragma unroll
      for (int i = 0; i < kPipe; ++i) {
        r0[i] = ra[i];
        r1[i] = rb[i];
        r2[i] = rcz[i];
      }
    } else {
      double nrm[kPipe], rn[kPipe];
#pragma unroll
      for (int i = 0; i < kPipe; ++i) {
        const double x = ra[i], y = rb[i];
        nrm[i] = sqrt_nr((x * x + y * y) + 1.0);  // s2 in [1, 2^601] when div_safe(x), div_safe(y)
        if (!(kDivShare && (p.xy_safe || (div_safe(x) && div_safe(y))))) slow |= 1u << i;
      }
      // the three divisions by nrm share one reciprocal (div_rn: the
      // compiler's own f64 division sequence, bit for bit, where it would
      // not rescale)
#pragma unroll
      for (int i = 0; i < kPipe; ++i) rn[i] = recip_nr(nrm[i]);
#pragma unroll
      for (int i = 0; i < kPipe; ++i) {
        r0[i] = div_rn(ra[i], nrm[i], rn[i]);
        r1[i] = div_rn(rb[i], nrm[i], rn[i]);
        r2[i] = div_rn(1.0, nrm[i], rn[i]);
      }
    }
    double den[kPipe], t[kPipe];
#pragma unroll
    for (int i = 0; i < kPipe; ++i) den[i] = (pl[i].x * r0[i] + pl[i].y * r1[i]) + pl[i].z * r2[i];
#pragma unroll
    for (int i = 0; i < kPipe; ++i) {
      t[i] = div_rn(-pl[i].w, den[i], recip_nr(den[i]));
      if (!(kDivShare && div_safe(pl[i].w) && div_safe(den[i]))) slow |= 1u << i;
    }
#pragma unroll
    for (int i = 0; i < kPipe; ++i) {
      X[i] = p.o0 + r0[i] * t[i];
      Y[i] = p.o1 + r1[i] * t[i];
      Z[i] = p.o2 + r2[i] * t[i];
      if (dbg & 1) {
        X[i] = ra[i];
        Y[i] = rb[i];
        Z[i] = pl[i].w;
      }
    }
    fallback = slow;
    }  // !M_VERIFY
    if (fallback) {  // rare: the operators' own sequences (rescaling, +-0, inf / NaN; unsettled M_VERIFY points)
#pragma unroll
      for (int i = 0; i < kPipe; ++i) {
        if (!((fallback >> i) & 1u)) continue;
        // the point's operands again (M_VERIFY: re-read, so that nothing of
        // the verified route stays live across this block)
        double xa = ra[i], xb = rb[i], xc = rcz[i];
        double4 pp = pl[i];
        if ((mode & M_VERIFY) && !(dbg & 4)) {
          const uint32_t e = s_ent[min(j0 + 64 * i + lane, total - 1)];
          int uu, vv;
          chunk_uv<VEC>(u_c, v_c, e, W, &uu, &vv);
          xa = p.xn[uu];
          xb = p.yn[vv];
          pp = p.planes[(dbg & 1024) ? (ent_code(e) & 31u) : ent_code(e)];
        }
        double r0, r1, r2;
        if (mode & M_NC) {
          r0 = xa;
          r1 = xb;
          r2 = xc;
        } else {
          const double x = xa, y = xb;
          const double nrm = sqrt((x * x + y * y) + 1.0);
          r0 = x / nrm;
          r1 = y / nrm;
          r2 = 1.0 / nrm;
        }
        const double4 pq = pp;
        const double t = -pq.w / ((pq.x * r0 + pq.y * r1) + pq.z * r2);
        X[i] = p.o0 + r0 * t;
        Y[i] = p.o1 + r1 * t;
        Z[i] = p.o2 + r2 * t;
        if ((mode & M_VERIFY) && pose) {  // (M_VERIFY: its settled points are posed above)
          const double X2 = ((pm[0] * X[i] + pm[1] * Y[i]) + pm[2] * Z[i]) + pm[3];
          const double Y2 = ((pm[4] * X[i] + pm[5] * Y[i]) + pm[6] * Z[i]) + pm[7];
          const double Z2 = ((pm[8] * X[i] + pm[9] * Y[i]) + pm[10] * Z[i]) + pm[11];
          X[i] = X2;
          Y[i] = Y2;
          Z[i] = Z2;
        }
      }
    }
    }  // dbg & 4096
    if (pose && !(mode & M_VERIFY)) {
#pragma unroll
      for (int i = 0; i < kPipe; ++i) {
        const double X2 = ((pm[0] * X[i] + pm[1] * Y[i]) + pm[2] * Z[i]) + pm[3];
        const double Y2 = ((pm[4] * X[i] + pm[5] * Y[i]) + pm[6] * Z[i]) + pm[7];
        const double Z2 = ((pm[8] * X[i] + pm[9] * Y[i]) + pm[10] * Z[i]) + pm[11];
        X[i] = X2;
        Y[i] = Y2;
        Z[i] = Z2;
      }
    }
    if (dbg & 2) continue;
    if (kStageOut && !f64out) {
      // 64 points at a time through an LDS stage: their 192 xyz words and 192
      // colour bytes leave as lane-consecutive dword / byte stores
#pragma unroll
      for (int i = 0; i < kPipe; ++i) {
        const int j = j0 + 64 * i + lane;
        const int n = min(64, total - (j0 + 64 * i));
        if (n <= 0) break;
        s_sxyz[3 * lane] = static_cast<float>(X[i]);
        s_sxyz[3 * lane + 1] = static_cast<float>(Y[i]);
        s_sxyz[3 * lane + 2] = static_cast<float>(Z[i]);
        s_scol[3 * lane] = static_cast<uint8_t>(bgr[i]);
        s_scol[3 * lane + 1] = static_cast<uint8_t>(bgr[i] >> 8);
        s_scol[3 * lane + 2] = static_cast<uint8_t>(bgr[i] >> 16);
        __builtin_amdgcn_wave_barrier();
        const long long o = base + (j - lane);
        float* xyz = static_cast<float*>(p.xyz) + 3 * o;
        uint8_t* cc = p.bgr + 3 * o;
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (64 * k + lane < 3 * n) {
            xyz[64 * k + lane] = s_sxyz[64 * k + lane];
            cc[64 * k + lane] = s_scol[64 * k + lane];
          }
        }
        __builtin_amdgcn_wave_barrier();
      }
      continue;
    }
    // (col_stage: the colours through the wave's LDS stage, shifted by the
    // pass's first output byte modulo 8, then 8 bytes per lane)
    const bool cst = col_stage && !(kAblate & 16384);
    const int csh = static_cast<int>((3 * (base + j0)) & 7);
#pragma unroll
    for (int i = 0; i < kPipe; ++i) {
      const int j = j0 + 64 * i + lane;
      if (j < total) {
        const unsigned o = static_cast<unsigned>(j);  // offset from the chunk's first point
        if (f64out) {
          double* xyz = static_cast<double*>(p.xyz) + 3 * base + 3 * o;
          xyz[0] = X[i];
          xyz[1] = Y[i];
          xyz[2] = Z[i];
        } else if (kAblate & 32768) {  // measurement only: no xyz stores (kept live)
          if (X[i] == -1234.5 && Y[i] == Z[i]) p.bgr[0] = 1;
        } else {
          float* xyz = at_bytes(wx, 12u * o);
          xyz[0] = static_cast<float>(X[i]);
          xyz[1] = static_cast<float>(Y[i]);
          xyz[2] = static_cast<float>(Z[i]);
        }
        if (kAblate & 16384) {  // measurement only: no colour stores (kept live)
          if (bgr[i] == 0x12345678u) p.bgr[1] = 1;
          continue;
        }
        if (kColOverlap && !cst) {
          // the next point's colour: lane + 1 of this slot, or lane 0 of the next
          const uint32_t nx = static_cast<uint32_t>(__builtin_amdgcn_update_dpp(0, static_cast<int>(bgr[i]), 0x130, 0xf, 0xf, false));
          const uint32_t nn = (i + 1 < kPipe) ? static_cast<uint32_t>(__builtin_amdgcn_readfirstlane(static_cast<int>(bgr[i + 1 < kPipe ? i + 1 : i]))) : 0u;
          const uint32_t next = lane == 63 ? nn : nx;
          if (j + 1 < total && (lane < 63 || i + 1 < kPipe)) {
            __builtin_amdgcn_raw_buffer_store_b32((bgr[i] & 0xffffffu) | (next << 24), rs_col, 3 * static_cast<int>(o), 0, 0);
          } else {  // the chunk's last point (or a pass's last lane with no next slot): 3 bytes
            __builtin_amdgcn_raw_buffer_store_b16(static_cast<unsigned short>(bgr[i]), rs_col, 3 * static_cast<int>(o), 0, 0);
            __builtin_amdgcn_raw_buffer_store_b8(static_cast<unsigned char>(bgr[i] >> 16), rs_col, 3 * static_cast<int>(o) + 2, 0, 0);
          }
          continue;
        }
        if (cst) {
          uint8_t* sc = s_scol + csh + 3 * (64 * i + lane);
          sc[0] = static_cast<uint8_t>(bgr[i]);
          sc[1] = static_cast<uint8_t>(bgr[i] >> 8);
          sc[2] = static_cast<uint8_t>(bgr[i] >> 16);
          continue;
        }
        uint8_t* cc = at_bytes(wc, 3u * o);
        cc[0] = static_cast<uint8_t>(bgr[i]);
        cc[1] = static_cast<uint8_t>(bgr[i] >> 8);
        cc[2] = static_cast<uint8_t>(bgr[i] >> 16);
      }
    }
    if (cst) {
      // the pass's colour bytes [A, A + 3n), A = 3 (base + j0), from the stage
      // (byte k of the stage = output byte A - csh + k) to the 8-byte aligned
      // words that cover them: whole words by one 8-byte store; the first and
      // last (shared with the neighbouring passes / chunks) byte by byte
      __builtin_amdgcn_wave_barrier();
      const int nbytes = csh + 3 * min(64 * kPipe, total - j0);
      // a buffer descriptor of the pass's 8-byte aligned output (SGPRs, per
      // pass) + the lane's 32-bit offset: no 64-bit VGPR address stays live
      // across passes (one did, and spilled)
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          p.bgr + (3 * (base + j0) - csh), 0, nbytes, 0x00020000);
#pragma unroll
      for (int q0 = 0; q0 < (3 * 64 * kPipe + 7 + 7) / 8; q0 += 64) {
        const int b0 = 8 * (q0 + lane);
        if (b0 < nbytes) {
          if (b0 >= csh && b0 + 8 <= nbytes) {
            const uint2 w = *reinterpret_cast<const uint2*>(s_scol + b0);
            __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(v2u, w), rs, b0, 0, 0);
          } else {
#pragma unroll
            for (int k = 0; k < 8; ++k)
              if (b0 + k >= csh && b0 + k < nbytes) __builtin_amdgcn_raw_buffer_store_b8(s_scol[b0 + k], rs, b0 + k, 0, 0);
          }
        }
      }
      __builtin_amdgcn_wave_barrier();  // (the next pass rewrites the stage)
    }
  }
}

// k_cloud: one chunk per wave, grid as k_count.  The workgroup's output
// offset is the sum of k_count's block sums before it (+ the earlier launch
// groups of the call); each wave adds the counts of the chunks before it in
// the workgroup.
constexpr int kPrefixBatch = 4;
#ifndef SLGPU_CLOUD_HOIST
#define SLGPU_CLOUD_HOIST 0
#endif
constexpr bool kCloudHoist = SLGPU_CLOUD_HOIST != 0;  // chunk loads issued before the block-offset loads

// Points of the blocks before block b of the launch group (one workgroup;
// holds a workgroup barrier): the super-block sums before b's super-block,
// then the block sums before b inside it (both <= ~sqrt(blocks) entries; all
// loads of a batch in flight together).
__device__ __forceinline__ long long block_offset(const Params& p, int64_t b, int tid, int lane, int wid,
                                                  long long* s_wred) {
  long long acc = 0;
  const int64_t sb = b >> p.sb_shift;
  for (int64_t t0 = 0; t0 < sb; t0 += kPrefixBatch * kThreads) {
    unsigned v[kPrefixBatch];
#pragma unroll
    for (int i = 0; i < kPrefixBatch; ++i) v[i] = p.super_sums[min<int64_t>(t0 + i * kThreads + tid, sb - 1)];
#pragma unroll
    for (int i = 0; i < kPrefixBatch; ++i) acc += (t0 + i * kThreads + tid < sb) ? v[i] : 0u;
  }
  for (int64_t t0 = sb << p.sb_shift; t0 < b; t0 += kPrefixBatch * kThreads) {
    int v[kPrefixBatch];
#pragma unroll
    for (int i = 0; i < kPrefixBatch; ++i) v[i] = p.block_sums[min<int64_t>(t0 + i * kThreads + tid, b - 1)];
#pragma unroll
    for (int i = 0; i < kPrefixBatch; ++i) acc += (t0 + i * kThreads + tid < b) ? v[i] : 0;
  }
  acc = wave_sum64(acc);
  if (lane == 0) s_wred[wid] = acc;
  __syncthreads();
  long long t = 0;
#pragma unroll
  for (int w = 0; w < kWaves; ++w) t += s_wred[w];
  return t;
}

// PIPE: points per lane per pass (kPipe; launches of at most one chunk per
// SIMD take all of a chunk's points in one pass: one gather round trip)
#ifndef SLGPU_CLOUD_WAVES
#define SLGPU_CLOUD_WAVES 5
#endif
#ifndef SLGPU_EXACT_PIPE
#define SLGPU_EXACT_PIPE 2
#endif
constexpr int kExactPipe = SLGPU_EXACT_PIPE;  // points per lane per pass of the exact (f64) k_cloud<M_TEX>
#ifndef SLGPU_VERIFY_PIPE
#define SLGPU_VERIFY_PIPE 2
#endif
constexpr int kVerifyPipe = SLGPU_VERIFY_PIPE;  // ... of the verified-route k_cloud<M_VERIFY | M_TEX>
static_assert(kWaves * kChunk >= 256 * kHistStride,
              "k_cloud's pre-stats workgroups keep their LDS histogram replicas in s_ent (SLGPU_HIST_REP <= 14)");
template <int MODE, int VEC, int PIPE = kPipe>
__global__ __launch_bounds__(kThreads, PIPE > kPipe ? 1 : SLGPU_CLOUD_WAVES) void k_cloud(Params p) {
  __shared__ uint32_t s_ent[kWaves][kChunk];  // compacted points: pixel | code << 10
  __shared__ __attribute__((aligned(16))) uint32_t s_bgr[kWaves][kBgrWords];  // colours (kBgrMode)
  __shared__ float s_sxyz[kWaves][kStageOut ? 192 : 1];      // output stage: 64 points' xyz
  __shared__ __attribute__((aligned(16))) uint8_t s_scol[kWaves][kStageOut ? 192 : kColDword ? kColStage : 4];  // colour bytes
  __shared__ long long s_wred[kWaves];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform, provably
  const int view = blockIdx.y;
  // pre-stats (sl_stack_next): S = gridDim.x - cloud_gx workgroups per view
  // compute the next call's histograms, after the triangulating ones, or
  // spread evenly among them (pre_mix: x is a pre-stats workgroup where
  // floor(x S / T) steps)
  int cx = blockIdx.x;  // triangulating workgroup index in the view
  int64_t sx = -1;      // pre-stats workgroup index in the view
  if (static_cast<int>(gridDim.x) > p.cloud_gx) {
    const int64_t T = gridDim.x, S = T - p.cloud_gx, x = blockIdx.x;
    if (p.pre_mix) {
      const int64_t s0 = x * S / T, s1 = (x + 1) * S / T;
      if (s1 != s0) sx = s0;
      cx = static_cast<int>(x - s1);
    } else if (x >= p.cloud_gx) {
      sx = x - p.cloud_gx;
    }
  }
  const int civ = cx * kWaves + wid;
  if (sx >= 0) {
    pre_stats_block(p, sx, gridDim.x - p.cloud_gx, &s_ent[0][0], reinterpret_cast<int*>(s_wred));
    return;
  }
  const int64_t b = static_cast<int64_t>(view) * p.cloud_gx + cx;  // block index in the launch
  const int64_t gc = static_cast<int64_t>(view) * p.cpv + civ;
  // (SLGPU_CLOUD_HOIST: the chunk's own loads before the offset's; measured slower)
  ChunkIn in;
  if (kCloudHoist && civ < p.cpv) cloud_load<VEC>(p, gc, lane, &in);
  const int before = (lane < wid && civ < p.cpv) ? p.chunk_counts[gc - wid + lane] : 0;  // earlier waves' chunks
  long long base;
  if (kAblate & 8192) {  // measurement only: no block prefix (disjoint slots of 1024 points)
    base = static_cast<long long>(gc) * kChunk;
  } else {
    base = block_offset(p, b, tid, lane, wid, s_wred);
    base += p.base_in ? *p.base_in : 0ll;
    base += wave_sum(before);
  }
  base = uniform64(base);
  if (civ >= p.cpv) return;
  if (!kCloudHoist) cloud_load<VEC>(p, gc, lane, &in);
  if (lane == 0 && view == p.n_views - 1 && civ == p.cpv - 1)
    p.view_offsets[p.n_views] = base + p.chunk_counts[gc];
  cloud_chunk<MODE, VEC, PIPE>(p, gc, base, lane, in, &s_ent[wid][0], &s_bgr[wid][0], &s_sxyz[wid][0], &s_scol[wid][0],
                               kColDword && !kStageOut);
}

// ================================================================= k_fused ====
// k_decode + k_cloud in one launch for calls of one launch group
// (SLGPU_FUSED=1, measured A/B): every workgroup decodes its chunk group as
// k_decode does (maps, mask, decision; no records), then, after a decoupled
// look-back over the workgroups before it for its output offset, triangulates
// its own points from registers -- the codes never leave the chip and one
// kernel boundary goes.  The look-back waits only on lower-numbered
// workgroups, dispatched before it and waiting on none after them, so it
// completes whatever the residency (other calls in flight included); its
// spin is bounded all the same (a give-up writes -1 as the call's total).
// Granules (Params::lb): 8 bytes {tag, value}, stored and loaded whole at
// agent scope -- the data is the flag (tag 1: the block's own count, 2: the
// inclusive prefix) -- zeroed before the launch (k_stats, or a memset).
__device__ __forceinline__ long long lookback_prefix(const Params& p, int64_t blk, unsigned own, int lane,
                                                     bool* failed) {
  unsigned long long* lb = p.lb;
  if (lane == 0)
    __hip_atomic_store(lb + blk, ((blk == 0 ? 2ull : 1ull) << 32) | own, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  *failed = false;
  if (blk == 0) return 0;
  long long acc = 0;
  int64_t j = blk - 1;  // lane k reads block j - k
  for (unsigned spins = 0;;) {
    const int64_t jj = j - lane;
    const unsigned long long g =
        jj >= 0 ? __hip_atomic_load(lb + jj, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : (2ull << 32);
    const unsigned tag = static_cast<unsigned>(g >> 32);
    const unsigned long long incl = __ballot(tag == 2u);
    const unsigned long long ready = __ballot(tag != 0u);
    const int f = incl ? __builtin_ctzll(incl) : 63;  // the nearest inclusive prefix (or the whole window)
    const unsigned long long need = f == 63 ? ~0ull : ((2ull << f) - 1ull);
    if ((ready & need) == need) {
      acc += wave_sum64(lane <= f ? static_cast<long long>(static_cast<unsigned>(g)) : 0ll);
      if (incl) break;
      j -= 64;
      continue;
    }
    if (++spins > (1u << 22)) {  // never expected (see above): give up rather than hang
      *failed = true;
      break;
    }
    __builtin_amdgcn_s_sleep(2);
  }
  if (lane == 0)
    __hip_atomic_store(lb + blk, (2ull << 32) | static_cast<unsigned>(acc + own), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  return acc;
}

template <int KC, int KR, int MODE, int CMODE, int PIPE>
__global__ __launch_bounds__(kThreads, 2) void k_fused(Params p) {
  __shared__ long long s_base;
  __shared__ int s_wc[kWaves];
  __shared__ int s_fail;
  static_assert((MODE & M_FUSED) && (MODE & M_DECIDE) && (MODE & M_CODES), "k_fused: a decide-path cloud call");
  static_assert(kWaves * (kChunk + kBgrWords) * 4 <= kDecodeLds, "the cloud's LDS fits in the decode tables'");
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  auto group = [&](const uint32_t* col, uint32_t pt, bool live, int n_px, int civ, int cg, unsigned* s_lds) {
    const int view = blockIdx.y;
    const int64_t px0 = static_cast<int64_t>(civ) * kChunk + lane * kPx;
    const int64_t pxl = (live && n_px > 0) ? px0 : 0;
    ChunkIn in;
    // the colour first: its latency overlaps the look-back
    if (p.tex != nullptr && kTexCoal) {  // cloud_load's 1-KB rows (cloud_chunk's LDS order)
      const uint8_t* tb = p.tex + view * p.tex_vs;
      const int64_t c0 = 3 * static_cast<int64_t>(civ) * kChunk + 16 * lane;
#pragma unroll
      for (int i = 0; i < 3; ++i) in.tq[i] = ld_side16(tb + min<int64_t>(c0 + 1024 * i, 3 * p.HW - 16));
    } else if (p.tex != nullptr) {
      const uint8_t* t = p.tex + view * p.tex_vs + 3 * pxl;
      in.tq[0] = ld_side16(t);
      in.tq[1] = ld_side16(t + 16);
      in.tq[2] = ld_side16(t + 32);
    } else {
      in.tq[0] = ld16(p.stack + view * p.stack_vs + pxl, n_px, true);
      in.tq[1] = in.tq[2] = make_uint4(0u, 0u, 0u, 0u);
    }
    const uint32_t cmax = static_cast<uint32_t>(p.Wp - 1);
#pragma unroll
    for (int i = 0; i < kPx / 2; ++i) in.d[i] = min(col[2 * i], cmax) | (min(col[2 * i + 1], cmax) << 16);
    in.ptbits = (live && n_px == kPx) ? (pt & 0xffffu) : 0u;
    const int cnt = wave_sum(__popc(in.ptbits));
    if (lane == 0) s_wc[wid] = cnt;
    __syncthreads();  // (also: every wave's decision is done with the LDS tables, reused below)
    if (wid == 0) {
      const int64_t blk = static_cast<int64_t>(view) * gridDim.x + cg;  // dispatch order
      const unsigned own = static_cast<unsigned>(s_wc[0] + s_wc[1] + s_wc[2] + s_wc[3]);
      bool failed;
      const long long pre = lookback_prefix(p, blk, own, lane, &failed);
      if (lane == 0) {
        s_base = pre + (p.base_in ? *p.base_in : 0ll);
        s_fail = failed ? 1 : 0;
      }
    }
    __syncthreads();
    long long base = s_base;
    for (int w = 0; w < wid; ++w) base += s_wc[w];
    base = uniform64(base);
    if (s_fail && tid == 0) p.view_offsets[p.n_views] = -1;  // (the give-up: an invalid total)
    if (live) {
      if (lane == 0 && view == p.n_views - 1 && civ == p.cpv - 1 && !s_fail) p.view_offsets[p.n_views] = base + cnt;
      const int64_t gc = static_cast<int64_t>(view) * p.cpv + civ;
      uint32_t* s_ent = s_lds + wid * kChunk;
      uint32_t* s_bgr = s_lds + kWaves * kChunk + wid * kBgrWords;
      float dummy_xyz[1];
      uint8_t dummy_col[4];
      cloud_chunk<CMODE, 1, PIPE>(p, gc, base, lane, in, s_ent, s_bgr, dummy_xyz, dummy_col);
    }
  };
  decode_body<KC, KR, MODE, 1>(p, group);
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
  double* d_planes = nullptr;  // [Wp] (n0, n1, n2, n.Oc + d)
  double* d_xn = nullptr;
  double* d_yn = nullptr;
  float* d_f32 = nullptr;  // planes32 [Wp][4] | xn32 [W] | yn32 [H] | planes12 [Wp][3]
  size_t off12 = 0;        // floats before planes12
  float fast_thr = 0.0f;   // k_count's sufficient |n.r| threshold (Params::fast_thr)
  bool xy_safe = false;     // every xn / yn table entry is div_safe (Params::xy_safe)
  bool xy_calc = false;     // xy_of reproduces every xn / yn entry (k_xy_check; SLGPU_XY_CALC=0: gathers, A/B)
  bool xy_plain = false;    // every xn / yn entry has 2^-20 <= |v| <= 2^20 (the verified route's range premise)
  bool planes_plain = false;  // every plane has |w| >= 2^-500 and max|n_i| >= 2^-400 (ditto)
  bool xy_calc_env = true;
  double cam[4] = {0, 0, 1, 1};  // cx, cy, fx, fy
  bool verify32 = true;     // SL_XYZ_F32 by the verified shorter route (SLGPU_VERIFY32=0: the exact sequence, A/B)
  double* d_nc = nullptr;
  // scratch
  ViewStats* d_stats = nullptr;
  int64_t cap_stats = 0;
  unsigned* d_hist[2] = {nullptr, nullptr};  // per-view histograms, parity double-buffered
  int64_t cap_hist[2] = {0, 0};
  int64_t hist_dirty[2] = {0, 0};  // leading views of each buffer that may be non-zero
  int par = 0;                     // buffer the next adaptive launch accumulates into
  int* d_chunk_counts = nullptr;
  int64_t cap_cc = 0;
  int* d_block_sums = nullptr;
  int64_t cap_bs = 0;
  unsigned* d_super[2] = {nullptr, nullptr};  // super-block sums, parity double-buffered (kSuperCap each)
  int spar = 0;
  uint8_t* d_ptnib = nullptr;
  int64_t cap_ptnib = 0;
  uint16_t* d_codes = nullptr;  // k_decode -> k_count / k_cloud records
  int64_t cap_codes = 0;
  int last_views = 0;
  int decode_wgs = 0;  // k_decode grid cap in workgroups over all views (0: one workgroup per chunk group)
  // optional per-call HIP-event timing of k_decode / k_count / k_cloud
  std::vector<hipEvent_t> prof_ev;  // kProfEv events per call slot
  std::vector<int> prof_groups;     // launch groups recorded per call
  std::vector<char> prof_decide;    // per call: M_DECIDE path (events around k_stats, k_decode, k_cloud)
  int n_cu = 0;
  bool force_3k = false;            // SLGPU_PATH=3: k_decode + k_count + k_cloud for aligned frames too (A/B)
  bool rec_from_maps = false;       // maps + cloud: k_cloud reads the col map instead of the (12-bit)
                                    // records (SLGPU_RECORDS=0; A/B: 1.6 % slower per step at config 2)
  bool rec12 = true;                // cloud only: 12-bit packed records (SLGPU_REC12=0: 16-bit, A/B)
  int prof_n = 0;
  // the last launch group's kernels and arguments (sl_time_kernels)
  // RCCL gather (sl_gather_init): communicator, this rank, count scratch
  void* comm = nullptr;
  int nranks = 0, rank = 0;
  int64_t* d_gcounts = nullptr;
  int64_t cap_gcounts = 0;
  // the last call's stream: a call on another stream first waits for the work
  // queued there (the scratch above is per context)
  hipStream_t last_stream = nullptr;
  hipEvent_t done_ev = nullptr;
  bool done_valid = false;
  int64_t last_launches = 0, last_launch_px = 0;  // sl_last_launch_info
  int64_t* mc_next = nullptr;  // sl_mask_counts_to: the next sl_decode_triangulate's masked-pixel counts
  // The adaptive mask's histogram pass (k_stats) ahead of its k_decode on a
  // side stream, beside the previous launch group's k_cloud: for the later
  // launch groups of a call, and for a call's first group when the caller
  // declared the stack ready (sl_stack_ready).  Its only scratch is the
  // parity-buffered histograms, so it waits for no more than the last kernel
  // that read them (hist_ev) and the caller's readiness event.
  hipStream_t side = nullptr;
  hipEvent_t hist_ev = nullptr;   // after the latest kernel that reads the histograms (k_decode / k_count)
  hipEvent_t stats_ev = nullptr;  // after a k_stats on `side` (its k_decode waits for it)
  hipEvent_t entry_ev = nullptr;  // the side path's first use: everything queued before it
  bool hist_tracked = false;      // hist_ev is recorded after every histogram reader from now on
  bool ready_next = false;        // sl_stack_ready: armed for the next sl_decode_triangulate
  hipEvent_t ready_ev_next = nullptr;
  bool no_side = false;           // SLGPU_STATS_SIDE=0: k_stats always on the call's stream (A/B)
  bool fused = false;             // SLGPU_FUSED=1: k_fused for one-group cloud calls (A/B)
  unsigned long long* d_lb = nullptr;  // k_fused's look-back granules
  int64_t cap_lb = 0;
  bool side_groups = false;       // SLGPU_STATS_SIDE=1: also the later launch groups of every call (A/B;
                                  // off by default: a cross-stream event wait measured 10-20 us of latency,
                                  // more than the k_stats it hides)
  // Pre-stats (sl_stack_next): a call's last k_cloud also runs the histogram
  // pass of the NEXT call's first launch group (declared stack), so that call
  // starts with its k_decode.  Three buffers in rotation: the one the current
  // call's k_decode reads, the one its k_cloud accumulates into, and the one
  // that k_cloud zeroes for the following pass (last read a call earlier).
  unsigned* d_pre[3] = {nullptr, nullptr, nullptr};
  int64_t cap_pre = 0;                // words of each
  int64_t pre_dirty[3] = {0, 0, 0};   // leading words that may be non-zero
  int pre_acc = 0;                    // buffer the next pre-stats pass accumulates into
  bool decl_next = false;             // sl_stack_next armed for the coming call
  const uint8_t* decl_stack = nullptr;
  int64_t decl_vs = 0;
  int decl_views = 0;
  bool pre_armed = false;             // a pre-stats pass was queued for the next call
  int pre_buf = 0;                    // ... into this buffer
  const uint8_t* pre_stack = nullptr; // ... of this stack, stride, first-group views, frame
  int64_t pre_vs = 0, pre_hw = 0;
  int pre_views = 0;
  bool no_pre = false;                // SLGPU_PRESTATS=0: sl_stack_next ignored, no pre-stats at all (A/B)
  bool no_pre_groups = false;         // SLGPU_PRE_GROUPS=0: no pre-stats between a call's launch groups (A/B)
  int pre_mix = 0;                    // SLGPU_PRE_MIX=1: pre-stats workgroups spread among k_cloud's (A/B)
  int pre_wgs = 0;                    // SLGPU_PRE_WGS=n: pre-stats workgroups in all (A/B; 0: 8 per CU)
  bool pre_decode = false;            // SLGPU_PRE_DECODE=1: pre-stats workgroups in k_decode's tail (A/B)
  int64_t max_chunks = kMaxChunks;    // chunks per launch group (SLGPU_GROUP_CHUNKS=n, at most kMaxChunks: A/B)
  int decode_dyn = -1;                // k_decode's later rounds pulled dynamically: -1 cloud-only calls (no
                                      // maps), SLGPU_DECODE_DYN=0 never, =1 every cloud call (A/B)
  bool decode_balance = false;        // SLGPU_DECODE_BALANCE=1: the capped k_decode grid shrunk so that every
                                      // workgroup decodes the same number of chunk groups (A/B)
  struct {
    bool valid = false;
    bool decide = false;  // fn[1] = k_stats (or null) instead of k_count
    bool fused = false;   // fn[0] = k_fused (decode and cloud), fn[2] = null
    Params p[3];
    const void* fn[3] = {nullptr, nullptr, nullptr};  // k_decode, k_count, k_cloud (or null)
    dim3 grid[3];
    hipStream_t s = nullptr;
  } last;
};

// ---------------------------------------------------------------- gather ----
// The merge's one exchange: every rank's cloud to the root
// rank in rank order, over RCCL (xGMI within a node).  RCCL is opened with
// dlopen by soname, so a process that already holds one (PyTorch's) shares
// that copy.  Counts: an ncclAllGather of one int64 per rank; payloads:
// grouped ncclSend (every rank) / ncclRecv (root) straight into the root's
// merged buffers at exclusive-scan offsets (RCCL has no gatherv, and a ring
// all-gather would push every payload over every link).
namespace {

struct Rccl {
  void* lib = nullptr;
  ncclResult_t (*get_unique_id)(ncclUniqueId*) = nullptr;
  ncclResult_t (*comm_init_rank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*comm_destroy)(ncclComm_t) = nullptr;
  ncclResult_t (*all_gather)(const void*, void*, size_t, ncclDataType_t, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*group_start)() = nullptr;
  ncclResult_t (*group_end)() = nullptr;
  const char* (*error_string)(ncclResult_t) = nullptr;
};

Rccl* rccl() {  // loaded once per process; null if RCCL is missing
  static Rccl r;
  static std::once_flag once;
  std::call_once(once, [] {
    for (const char* name : {"librccl.so.1", "librccl.so", "/opt/rocm/lib/librccl.so.1"}) {
      r.lib = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (r.lib) break;
    }
    if (!r.lib) return;
    auto sym = [](const char* n) { return dlsym(r.lib, n); };
    r.get_unique_id = reinterpret_cast<decltype(r.get_unique_id)>(sym("ncclGetUniqueId"));
    r.comm_init_rank = reinterpret_cast<decltype(r.comm_init_rank)>(sym("ncclCommInitRank"));
    r.comm_destroy = reinterpret_cast<decltype(r.comm_destroy)>(sym("ncclCommDestroy"));
    r.all_gather = reinterpret_cast<decltype(r.all_gather)>(sym("ncclAllGather"));
    r.send = reinterpret_cast<decltype(r.send)>(sym("ncclSend"));
    r.recv = reinterpret_cast<decltype(r.recv)>(sym("ncclRecv"));
    r.group_start = reinterpret_cast<decltype(r.group_start)>(sym("ncclGroupStart"));
    r.group_end = reinterpret_cast<decltype(r.group_end)>(sym("ncclGroupEnd"));
    r.error_string = reinterpret_cast<decltype(r.error_string)>(sym("ncclGetErrorString"));
    if (!r.get_unique_id || !r.comm_init_rank || !r.comm_destroy || !r.all_gather || !r.send || !r.recv ||
        !r.group_start || !r.group_end || !r.error_string)
      r.lib = nullptr;
  });
  return r.lib ? &r : nullptr;
}

#define NCCL_TRY(ctx, expr)                                                                  \
  do {                                                                                       \
    ncclResult_t e_ = (expr);                                                                \
    if (e_ != ncclSuccess) return fail((ctx), SL_EHIP, std::string(#expr) + ": " + R->error_string(e_)); \
  } while (0)

}  // namespace

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

// scratch for `views` views of `px` pixels each
int ensure_scratch(sl_ctx* c, int64_t views, int64_t px, bool codes) {
  const int64_t chunks = views * ((px + kChunk - 1) / kChunk);
  int r = grow(c, &c->d_chunk_counts, &c->cap_cc, chunks);
  if (r) return r;
  r = grow(c, &c->d_block_sums, &c->cap_bs, views * (((px + kChunk - 1) / kChunk + kWaves - 1) / kWaves));
  if (r) return r;
  r = grow(c, &c->d_ptnib, &c->cap_ptnib, chunks * kChunkNib);
  if (r) return r;
  for (int b = 0; b < 2; ++b) {
    int64_t cap = c->d_super[b] ? kSuperCap : 0;
    r = grow(c, &c->d_super[b], &cap, kSuperCap);  // zeroed once; then by the kernels
    if (r) return r;
  }
  for (int b = 0; b < 2; ++b) {
    const int64_t before = c->cap_hist[b];
    r = grow(c, &c->d_hist[b], &c->cap_hist[b], views * kHistView);  // k_stats' replicas (k_decode's: kSlot)
    if (r) return r;
    if (c->cap_hist[b] != before) c->hist_dirty[b] = 0;  // fresh (zeroed) allocation
  }
  // (u16 units: 2 B/px, or kRecBlk's 1536-B slots of whole chunk groups)
  if (codes)
    return grow(c, &c->d_codes, &c->cap_codes,
                std::max<int64_t>(views * px, views * ((px + 4 * kChunk - 1) / (4 * kChunk)) * 4 * (kRecSlot / 2)) + 16);
  return SL_OK;
}

using KernelFn = void (*)(Params);
constexpr int kProfGroups = 64;            // launch groups timed per call (at most)
constexpr int kProfEv = 4 * kProfGroups;   // events per call: per group before k_decode, k_count, k_cloud, after
                                           // (M_DECIDE: before k_stats, k_decode, k_cloud, after)

// k_decode specialisations for the benchmark configurations; everything else
// (other bit counts, unaligned frames) runs the generic instantiation.
KernelFn pick_decode(int kc, int kr, int mode, bool vec) {
  if (vec && !(mode & (M_NC | M_FROMMAPS))) {
    constexpr int mrch = M_MAPS | M_ROWS | M_CODES | M_HIST, mrh = M_MAPS | M_ROWS | M_HIST,
                  ch = M_CODES | M_HIST, mrc = M_MAPS | M_ROWS | M_CODES, cc = M_CODES;
    if (mode == mrch && kc == 11 && kr == 11) return k_decode<11, 11, mrch, 1>;
    if (mode == mrch && kc == 10 && kr == 0) return k_decode<10, 0, mrch, 1>;
    if (mode == mrh && kc == 11 && kr == 11) return k_decode<11, 11, mrh, 1>;
    if (mode == ch && kc == 11) return k_decode<11, 0, ch, 1>;
    if (mode == ch && kc == 10) return k_decode<10, 0, ch, 1>;
    if (mode == mrc && kc == 11 && kr == 11) return k_decode<11, 11, mrc, 1>;
    if (mode == cc && kc == 11) return k_decode<11, 0, cc, 1>;
    constexpr int D = M_DECIDE;
    if (mode == (mrch | D) && kc == 11 && kr == 11) return k_decode<11, 11, mrch | D, 1>;
    if (mode == (mrch | D) && kc == 10 && kr == 0) return k_decode<10, 0, mrch | D, 1>;
    if (mode == (mrh | D) && kc == 11 && kr == 11) return k_decode<11, 11, mrh | D, 1>;
    if (mode == (mrh | D) && kc == 10 && kr == 0) return k_decode<10, 0, mrh | D, 1>;  // config 1 gray_decode
    if (mode == (ch | D) && kc == 11) return k_decode<11, 0, ch | D, 1>;
    if (mode == (ch | D) && kc == 10) return k_decode<10, 0, ch | D, 1>;
    if (mode == (mrc | D) && kc == 11 && kr == 11) return k_decode<11, 11, mrc | D, 1>;
    if (mode == (cc | D) && kc == 11) return k_decode<11, 0, cc | D, 1>;
  }
  if (vec && (mode & M_NC) && !(mode & (M_FROMMAPS | M_PLANE_RSRC))) {  // non-pinhole rays (an Nc table)
    constexpr int D = M_DECIDE | M_NC, mrch = M_MAPS | M_ROWS | M_CODES | M_HIST, ch = M_CODES | M_HIST;
    if (mode == (mrch | D) && kc == 11 && kr == 11) return k_decode<11, 11, mrch | D, 1>;
    if (mode == (ch | D) && kc == 11) return k_decode<11, 0, ch | D, 1>;
  }
  return vec ? k_decode<-1, -1, -1, 1> : k_decode<-1, -1, -1, 0>;
}

KernelFn pick_cloud(int mode, bool vec, bool small) {
  if (vec && small && kSmallPipe > kPipe && mode == (M_FAST32 | M_TEX)) return k_cloud<M_FAST32 | M_TEX, 1, kSmallPipe>;
  if (vec && mode == M_TEX) return k_cloud<M_TEX, 1, kExactPipe>;  // f32 xyz, pinhole rays, BGR texture
  if (vec && mode == (M_VERIFY | M_TEX)) return k_cloud<M_VERIFY | M_TEX, 1, kVerifyPipe>;  // ... verified route
  if (vec && mode == (M_FAST32 | M_TEX)) return k_cloud<M_FAST32 | M_TEX, 1>;
  return vec ? k_cloud<-1, 1, kExactPipe> : k_cloud<-1, 0, kExactPipe>;  // (f64 chains: kExactPipe points per pass)
}

// k_fused instantiations: the benchmark configurations' one-group calls
// (decode mode with M_DECIDE | M_FUSED, cloud mode), else null
KernelFn pick_fused(int kc, int kr, int dmode, int cmode) {
  constexpr int D = M_DECIDE | M_FUSED, mrch = M_MAPS | M_ROWS | M_CODES | M_HIST, ch = M_CODES | M_HIST;
  constexpr int V = M_VERIFY | M_TEX, F = M_FAST32 | M_TEX;
  if (dmode == (mrch | D) && kc == 10 && kr == 0 && cmode == V) return k_fused<10, 0, mrch | D, V, kVerifyPipe>;
  if (dmode == (mrch | D) && kc == 11 && kr == 11 && cmode == V) return k_fused<11, 11, mrch | D, V, kVerifyPipe>;
  if (dmode == (mrch | D) && kc == 11 && kr == 11 && cmode == F) return k_fused<11, 11, mrch | D, F, kPipe>;
  if (dmode == (ch | D) && kc == 11 && cmode == V) return k_fused<11, 0, ch | D, V, kVerifyPipe>;
  return nullptr;
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

// Enqueue, per launch group of views, k_decode -> k_count [-> k_cloud] on
// stream s -- or, when decode_mode has M_DECIDE, [k_stats ->] k_decode
// [-> k_cloud] (k_decode applies the mask and makes the point decision).
// decode_mode / count_mode / cloud_mode (< 0: no cloud) are the kernels' mode
// bits.  Launch groups hold at most kMaxChunks chunks (at least one view); a
// group's points follow the earlier groups' (base_in).
// The side stream and its events (created on first use).
int ensure_side(sl_ctx* c) {
  if (c->side) return SL_OK;
  for (hipEvent_t* e : {&c->hist_ev, &c->stats_ev, &c->entry_ev})
    if (!*e) HIP_TRY(c, hipEventCreateWithFlags(e, hipEventDisableTiming));
  HIP_TRY(c, hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
  return SL_OK;
}

// The one-call arms of a context (sl_stack_next's declaration, the pre-stats
// pass an earlier call queued): taken -- and cleared on the context -- at the
// entry of every call, so that a call that fails before its launch consumes
// them all the same (a later call on a refilled buffer must never take a
// histogram of its old contents).
struct PreArms {
  bool armed = false;  // the previous call's k_cloud computed histograms for this call (c->pre_*)
  bool decl = false;   // this call names the next call's stack (c->decl_*)
};
PreArms take_arms(sl_ctx* c) {
  PreArms a;
  a.armed = c->pre_armed;
  a.decl = c->decl_next;
  c->pre_armed = false;
  c->decl_next = false;
  return a;
}

// ready: the caller declared the stack ready (sl_stack_ready; ready_ev, if
// non-null, completes when it is): the first launch group's k_stats may run on
// the side stream too.
int launch(sl_ctx* c, const Params& p0, bool vec, int decode_mode, int count_mode, int cloud_mode,
           hipStream_t s, PreArms arms, bool ready = false, hipEvent_t ready_ev = nullptr) {
  const bool decide = (decode_mode & M_DECIDE) != 0;
  const int64_t cpv = p0.cpv;
  const int vpg = static_cast<int>(std::max<int64_t>(1, c->max_chunks / cpv));  // views per group
  const int n_groups = static_cast<int>((p0.n_views + vpg - 1) / vpg);
  const bool adaptive = (decode_mode & M_HIST) != 0;
  // k_stats on the side stream (never while `s` is being captured into a
  // graph: the side path waits on events recorded outside the capture)
  bool side_ok = false;
  if (decide && adaptive && c->prof_ev.empty() && (ready || (n_groups > 1 && c->side_groups)) && !c->no_side) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    HIP_TRY(c, hipStreamIsCapturing(s, &cs));
    side_ok = cs == hipStreamCaptureStatusNone;
    if (side_ok) {
      int r = ensure_side(c);
      if (r) return r;
    }
  }
  int r = ensure_scratch(c, std::min(vpg, p0.n_views), p0.HW, (decode_mode & M_CODES) != 0);
  if (r) return r;
  r = grow(c, &c->d_stats, &c->cap_stats, p0.n_views);
  if (r) return r;
  // Pre-stats (sl_stack_next): this call's first group takes the histograms
  // the previous call's k_cloud computed for it (same stack, stride, views
  // and frame), and this call's last k_cloud computes those of the call
  // declared next.  (Not with k_fused, whose look-back granules k_stats zeroes.)
  const int nv0 = std::min(vpg, p0.n_views);
  bool pre_use = arms.armed && decide && adaptive && !c->fused && p0.stack == c->pre_stack &&
                 p0.stack_vs == c->pre_vs && nv0 == c->pre_views && p0.HW == c->pre_hw;
  int pre_in = c->pre_buf;
  const bool pre_run = arms.decl && !c->no_pre && !c->fused && cloud_mode >= 0 && vec;
  const bool pre_dec = pre_run && decide && c->pre_decode;  // ... in the last k_decode instead (A/B)
  // Within a call of several launch groups: group g's k_cloud also runs group
  // g + 1's histogram pass (the same pre-stats workgroups), so only the first
  // group can need a k_stats launch (SLGPU_PRE_GROUPS=0: every group its own, A/B)
  const bool pre_groups = decide && adaptive && n_groups > 1 && !c->no_pre && !c->no_pre_groups && !c->fused &&
                          cloud_mode >= 0 && vec;
  // pre-stats workgroups per view of a pass over nv views: up to 8 per CU in
  // all (one 16-pixel step per thread at config 2; measured 0.5-1 us faster
  // per c2 step than k_stats' 2 per CU)
  auto pre_bpv_of = [&](int nv) -> int64_t {
    const int64_t per_view = (p0.HW / 16 + kThreads - 1) / kThreads;
    const int64_t wgs = c->pre_wgs > 0 ? c->pre_wgs : 8 * c->n_cu;
    return std::max<int64_t>(1, std::min<int64_t>(per_view, (wgs + nv - 1) / nv));
  };
  {
    int64_t words = 0;
    if (pre_run) words = static_cast<int64_t>(std::min(vpg, c->decl_views)) * kHistView;
    if (pre_groups) words = std::max<int64_t>(words, static_cast<int64_t>(std::min(vpg, p0.n_views - vpg)) * kHistView);
    if (words > c->cap_pre) {  // (re)allocated zeroed: nothing left to take
      pre_use = false;
      for (int b = 0; b < 3; ++b) {
        int64_t cap = c->cap_pre;
        r = grow(c, &c->d_pre[b], &cap, words);
        if (r) return r;
        if (b == 2) c->cap_pre = cap;
        c->pre_dirty[b] = 0;
      }
    }
  }
  c->last_views = p0.n_views;
  if (p0.masked)  // the caller's per-view counts, accumulated by the groups' k_decode / k_count
    HIP_TRY(c, hipMemsetAsync(p0.masked, 0, sizeof(unsigned long long) * p0.n_views, s));
  hipEvent_t* ev = nullptr;
  if (!c->prof_ev.empty() && kProfEv * (c->prof_n + 1) <= static_cast<int>(c->prof_ev.size()))
    ev = &c->prof_ev[kProfEv * c->prof_n++];
  // The pre-stats workgroups' arguments on launch parameters pc of a grid
  // with nv rows, for the pnv views of stack pst (view stride pvs): the launch
  // grows by as many workgroups per row as they need (after its own); the
  // pass accumulates into buffer c->pre_buf, for the stack recorded in c->pre_*.
  auto add_pre = [&](Params& pc, dim3& grid, int nv, const uint8_t* pst, int64_t pvs, int pnv) -> int {
    const int acc = c->pre_acc, zb = (acc + 1) % 3;
    const int64_t bpv = pre_bpv_of(pnv);
    if (c->pre_dirty[acc] > 0)
      HIP_TRY(c, hipMemsetAsync(c->d_pre[acc], 0, sizeof(unsigned) * c->pre_dirty[acc], s));
    pc.pre_stack = pst;
    pc.pre_vs = pvs;
    pc.pre_hist = c->d_pre[acc];
    pc.pre_zero = c->d_pre[zb];
    pc.pre_zero_words = c->pre_dirty[zb];
    pc.pre_views = pnv;
    pc.pre_bpv = static_cast<int>(bpv);
    pc.pre_mix = c->pre_mix;
    const int64_t total = static_cast<int64_t>(pnv) * bpv;
    grid.x += static_cast<unsigned>((total + nv - 1) / nv);
    c->pre_dirty[acc] = static_cast<int64_t>(pnv) * kHistView;
    c->pre_dirty[zb] = 0;
    c->pre_acc = zb;
    c->pre_buf = acc;
    c->pre_stack = pst;
    c->pre_vs = pvs;
    c->pre_views = pnv;
    c->pre_hw = p0.HW;
    return SL_OK;
  };
  bool next_pre = pre_use;  // the coming group's histograms were computed by the previous k_cloud
  int g = 0;  // launch group index
  for (int v0 = 0; v0 < p0.n_views; v0 += vpg, ++g) {
    hipEvent_t* gev = (ev && g < kProfGroups) ? ev + 4 * g : nullptr;
    if (gev) HIP_TRY(c, hipEventRecord(gev[0], s));
    const int nv = std::min(vpg, p0.n_views - v0);
    c->last_launch_px = static_cast<int64_t>(nv) * p0.HW;
    Params p = p0;
    p.n_views = nv;
    p.n_chunks = static_cast<int64_t>(nv) * cpv;
    if (p.stack) p.stack += v0 * p.stack_vs;
    if (p.tex) p.tex += v0 * p.tex_vs;
    if (p.in_col) p.in_col += v0 * p.HW;
    if (p.in_mask) p.in_mask += v0 * p.HW;
    if (p.col_out) p.col_out += v0 * p.HW;
    if (p.row_out) p.row_out += v0 * p.HW;
    if (p.mask_out) p.mask_out += v0 * p.HW;
    if (p.poses) p.poses += 16 * v0;
    if (p.masked) p.masked += v0;
    if (p.view_offsets) p.view_offsets += v0;
    p.base_in = (v0 > 0 && p.view_offsets) ? p.view_offsets : nullptr;
    p.stats = c->d_stats + v0;
    p.codes = c->d_codes;
    // maps + cloud on the decide path: k_cloud reads the col map (no records)
    p.rec_col = (decide && p.col_out && cloud_mode >= 0 && c->rec_from_maps) ? p.col_out : nullptr;
    p.rec12 = (decide && vec && !p.rec_col && cloud_mode >= 0 && p.Wp < 4096 && c->rec12) ? 1 : 0;
    p.rec_blk = (p.rec12 && kRecBlk && (!(decode_mode & M_MAPS) || SLGPU_REC_BLK_MAPS)) ? 1 : 0;  // (k_decode's `blk`)
    p.ptnib = c->d_ptnib;
    p.chunk_counts = c->d_chunk_counts;
    p.block_sums = c->d_block_sums;
    // this group's k_stats on the side stream: after the last reader of the
    // histograms it zeroes (the previous group's or call's k_decode) and, for
    // a call's first group, the caller's readiness event (else after
    // everything queued so far: the side path's first use)
    const bool pre_g = next_pre;  // histograms computed by the previous k_cloud (this call's or the last call's)
    next_pre = false;
    const bool ahead = !pre_g && side_ok && ((g > 0 && c->side_groups) || (g == 0 && ready));
    hipStream_t ss = ahead ? c->side : s;
    if (g == 0 && ready_ev && !ahead) HIP_TRY(c, hipStreamWaitEvent(s, ready_ev, 0));  // the promise, kept on s
    if (ahead) {
      if (g == 0 && ready_ev) HIP_TRY(c, hipStreamWaitEvent(ss, ready_ev, 0));
      if (!c->hist_tracked) {
        HIP_TRY(c, hipEventRecord(c->entry_ev, s));
        HIP_TRY(c, hipStreamWaitEvent(ss, c->entry_ev, 0));
        c->hist_tracked = true;
      } else {
        HIP_TRY(c, hipStreamWaitEvent(ss, c->hist_ev, 0));
      }
    }
    if (pre_g) {
      p.hist = c->d_pre[pre_in];
      p.hist_zero = nullptr;
    } else if (adaptive) {  // hist_dirty: leading words of a buffer that may be non-zero
      const int a = c->par, b = 1 - c->par;
      const int64_t words = static_cast<int64_t>(nv) * (decide ? kHistView : kSlot);
      if (c->hist_dirty[a] > 0)
        HIP_TRY(c, hipMemsetAsync(c->d_hist[a], 0, sizeof(unsigned) * c->hist_dirty[a], ss));
      p.hist = c->d_hist[a];
      p.hist_zero = c->d_hist[b];
      c->hist_dirty[a] = words;  // accumulated now; this launch zeroes b's leading `words`
      if (c->hist_dirty[b] <= words) c->hist_dirty[b] = 0;
      c->par = b;
    }
    const dim3 grid(static_cast<unsigned>((cpv + kWaves - 1) / kWaves), static_cast<unsigned>(nv));
    {  // super-block size: the smallest power of two >= sqrt(blocks of the group)
      const int64_t nb = static_cast<int64_t>(grid.x) * nv;
      int sh = 0;
      while ((int64_t{1} << (2 * sh)) < nb) ++sh;
      p.sb_shift = sh;
      p.super_sums = c->d_super[c->spar];
      p.super_zero = c->d_super[c->spar ^ 1];
      p.super_cap = kSuperCap;
      c->spar ^= 1;
    }
    c->last.valid = true;
    dim3 dgrid = grid;  // k_decode: chunk groups strided over a capped grid
    if (c->decode_wgs > 0) dgrid.x = std::min(grid.x, static_cast<unsigned>(std::max(1, (c->decode_wgs + nv - 1) / nv)));
    if (c->decode_balance) {  // rounds of the capped grid, and the fewest workgroups that need no more
      const unsigned rounds = (grid.x + dgrid.x - 1) / dgrid.x;
      dgrid.x = (grid.x + rounds - 1) / rounds;
    }
    c->last.grid[0] = dgrid;
    // barrier-free block sums when every k_decode workgroup iterates at most
    // kBsSlots chunk groups (4 chunks of at most 1024 points: 16-bit sums)
    p.bs_atomic = decide && (grid.x + dgrid.x - 1) / dgrid.x <= static_cast<unsigned>(kBsSlots);
    // decode_dyn (cloud-only calls; SLGPU_DECODE_DYN): a capped decode grid pulls its chunk
    // groups after the first round from per-view counters (the last entries of
    // this launch's super-block buffer, zeroed with it); block sums then take
    // the barrier path, whose barrier publishes each workgroup's next group
    const bool dyn_want = c->decode_dyn > 0 || (c->decode_dyn < 0 && !(decode_mode & M_MAPS));
    p.decode_dyn = (dyn_want && decide && (decode_mode & M_CODES) && dgrid.x < grid.x &&
                    ((static_cast<int64_t>(grid.x) * nv) >> p.sb_shift) + 1 + nv < kSuperCap) ? 1 : 0;
    if (p.decode_dyn) p.bs_atomic = 0;
    c->last.grid[1] = c->last.grid[2] = grid;
    c->last.s = s;
    c->last.fn[2] = nullptr;
    c->last.decide = decide;
    // k_fused (SLGPU_FUSED=1): a one-group cloud call's decode and cloud in
    // one launch; its look-back granules zeroed by k_stats (or a memset)
    KernelFn fusedfn = nullptr;
    if (c->fused && decide && vec && cloud_mode >= 0 && n_groups == 1)
      fusedfn = pick_fused(p.kc, (decode_mode & M_ROWS) ? p.kr : 0, decode_mode | M_FUSED, cloud_mode);
    c->last.fused = fusedfn != nullptr;
    if (fusedfn) {
      r = grow(c, &c->d_lb, &c->cap_lb, static_cast<int64_t>(grid.x) * nv);
      if (r) return r;
      p.lb = c->d_lb;
      p.lb_n = static_cast<int64_t>(grid.x) * nv;
      if (!adaptive) HIP_TRY(c, hipMemsetAsync(c->d_lb, 0, sizeof(unsigned long long) * p.lb_n, s));
    }
    if (decide) {
      c->last.fn[1] = nullptr;
      if (adaptive && !pre_g) {  // k_stats: the thresholds' histograms, before the decode applies them
        const int64_t per_view = (p0.HW / 16 + kThreads - 1) / kThreads;
        const dim3 sg(static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(per_view, (2 * c->n_cu + nv - 1) / nv))),
                      static_cast<unsigned>(nv));
        p.mode = decode_mode;
        void* args[] = {&p};
        c->last.p[1] = p;
        const void* kst = reinterpret_cast<const void*>(k_stats);
        c->last.fn[1] = kst;
        c->last.grid[1] = sg;
        HIP_TRY(c, hipLaunchKernel(kst, sg, dim3(kThreads), args, 0, ss));
        if (ahead) {
          HIP_TRY(c, hipEventRecord(c->stats_ev, ss));
          HIP_TRY(c, hipStreamWaitEvent(s, c->stats_ev, 0));
        }
      }
      if (gev) HIP_TRY(c, hipEventRecord(gev[1], s));
    }
    if (fusedfn) {  // one workgroup per chunk group (uncapped grid), then its cloud
      p.mode = decode_mode | M_FUSED;
      p.bs_atomic = 0;
      void* args[] = {&p};
      c->last.p[0] = p;
      c->last.p[0].masked = nullptr;
      c->last.fn[0] = reinterpret_cast<const void*>(fusedfn);
      c->last.grid[0] = grid;
      HIP_TRY(c, hipLaunchKernel(reinterpret_cast<const void*>(fusedfn), grid, dim3(kThreads), args, 0, s));
    } else {
      p.mode = decode_mode;
      KernelFn fn = pick_decode(p.kc, (decode_mode & M_ROWS) ? p.kr : 0, decode_mode, vec);
      c->last.p[0] = p;
      c->last.p[0].masked = nullptr;  // sl_time_kernels' re-runs leave the caller's counts alone
      c->last.fn[0] = reinterpret_cast<const void*>(fn);
      Params pd = p;
      dim3 pgrid = dgrid;
      if (pre_dec && g == n_groups - 1) {  // + the declared next call's histogram pass, in k_decode's tail
        pd.decode_gx = static_cast<int>(dgrid.x);
        r = add_pre(pd, pgrid, nv, c->decl_stack, c->decl_vs, std::min(vpg, c->decl_views));
        if (r) return r;
      }
      void* args[] = {&pd};
      HIP_TRY(c, hipLaunchKernel(reinterpret_cast<const void*>(fn), pgrid, dim3(kThreads), args, 0, s));
      if (pre_dec && g == n_groups - 1) c->pre_armed = true;
    }
    if (adaptive && decide && (c->hist_tracked || (side_ok && c->side_groups && g + 1 < n_groups))) {
      HIP_TRY(c, hipEventRecord(c->hist_ev, s));  // the last reader of this group's histograms
      c->hist_tracked = true;
    }
    if (gev) HIP_TRY(c, hipEventRecord(gev[decide ? 2 : 1], s));
    if (!decide) {
      p.mode = count_mode;
      void* args[] = {&p};
      const void* fn = vec ? reinterpret_cast<const void*>(k_count<1>) : reinterpret_cast<const void*>(k_count<0>);
      c->last.p[1] = p;
      c->last.p[1].masked = nullptr;
      c->last.fn[1] = fn;
      HIP_TRY(c, hipLaunchKernel(fn, grid, dim3(kThreads), args, 0, s));
      if (adaptive && c->hist_tracked) HIP_TRY(c, hipEventRecord(c->hist_ev, s));  // k_count reads them too
    }
    if (gev && !decide) HIP_TRY(c, hipEventRecord(gev[2], s));
    if (cloud_mode >= 0 && !fusedfn) {
      p.mode = cloud_mode;
      p.cloud_gx = static_cast<int>(grid.x);
      // at most one chunk per SIMD: all of a chunk's points in one pass
      KernelFn fn = pick_cloud(cloud_mode, vec, p.n_chunks <= 4 * static_cast<int64_t>(c->n_cu));
      c->last.p[2] = p;  // (sl_time_kernels re-runs it without the pre-stats workgroups)
      c->last.fn[2] = reinterpret_cast<const void*>(fn);
      Params pc = p;
      dim3 cgrid = grid;
      const bool last_g = g == n_groups - 1;
      const bool pre_now = pre_run && !pre_dec && last_g;
      const bool pre_grp = pre_groups && !last_g;
      if (pre_now) {  // + the declared next call's histogram pass, after this group's triangulating workgroups
        r = add_pre(pc, cgrid, nv, c->decl_stack, c->decl_vs, std::min(vpg, c->decl_views));
        if (r) return r;
      } else if (pre_grp) {  // + this call's next launch group's
        r = add_pre(pc, cgrid, nv, p0.stack + static_cast<int64_t>(v0 + vpg) * p0.stack_vs, p0.stack_vs,
                    std::min(vpg, p0.n_views - v0 - vpg));
        if (r) return r;
      }
      void* args[] = {&pc};
      HIP_TRY(c, hipLaunchKernel(reinterpret_cast<const void*>(fn), cgrid, dim3(kThreads), args, 0, s));
      if (pre_now) c->pre_armed = true;
      if (pre_grp) {
        next_pre = true;
        pre_in = c->pre_buf;
      }
    }
    if (gev) HIP_TRY(c, hipEventRecord(gev[3], s));
  }
  if (ev) {
    c->prof_groups.push_back(std::min(g, kProfGroups));
    c->prof_decide.push_back(decide);
  }
  c->last_launches = g;
  return SL_OK;
}

// The context's scratch is shared by its calls: a call on another stream than
// the previous call's first waits for the work queued on that stream (an event
// recorded there now), so calls on one context never overlap on the device.
int stream_handoff(sl_ctx* c, hipStream_t s) {
  if (c->done_valid && s != c->last_stream) {
    HIP_TRY(c, hipEventRecord(c->done_ev, c->last_stream));
    HIP_TRY(c, hipStreamWaitEvent(s, c->done_ev, 0));
  }
  c->last_stream = s;
  c->done_valid = true;
  return SL_OK;
}

}  // namespace

// helpers for slmerge.hip (same library)
int slgpu_fail(sl_ctx* c, int code, const char* msg) { return fail(c, code, msg); }
int slgpu_device(const sl_ctx* c) { return c->device; }

// ------------------------------------------------------------- PLY writer ----
// The ASCII PLY of sl_system.py:665-691 (== multi_point_cloud_process.py:
// 121-131): header, then per point f"{x:.4f} {y:.4f} {z:.4f} {r} {g} {b}\n"
// with the colour swapped from BGR.  Python formats %.4f correctly rounded
// (round-half-even on exact ties); so does fmt4 below: N = round(x * 10^4)
// computed exactly in 128-bit integers from x's binary significand, printed
// with 4 decimals.  Values beyond 2^53 / 10^4 and non-finite ones go through
// glibc's snprintf("%.4f"), which is also correctly rounded ("nan", "inf"
// as Python prints them).
namespace {

char* fmt4(char* o, double x) {
  uint64_t bits;
  memcpy(&bits, &x, 8);
  const bool neg = bits >> 63;
  const int be = static_cast<int>((bits >> 52) & 0x7ff);
  const uint64_t frac = bits & ((1ull << 52) - 1);
  if (be == 0x7ff || fabs(x) >= 9.0e11) {  // non-finite or large: libc
    if (be == 0x7ff && frac) return o + sprintf(o, "nan");
    if (be == 0x7ff) return o + sprintf(o, neg ? "-inf" : "inf");
    return o + sprintf(o, "%.4f", x);
  }
  // x = m * 2^e exactly
  const uint64_t m = be ? (frac | (1ull << 52)) : frac;
  const int e = (be ? be : 1) - 1075;
  unsigned __int128 v = static_cast<unsigned __int128>(m) * 10000u;
  uint64_t N;
  if (e >= 0) {
    N = static_cast<uint64_t>(v << e);
  } else if (-e >= 120) {
    N = 0;  // |x| * 10^4 < 2^67 * 2^-120: far below 1/2
  } else {
    const int sh = -e;
    const unsigned __int128 q = v >> sh;
    const unsigned __int128 r = v - (q << sh);
    const unsigned __int128 half = static_cast<unsigned __int128>(1) << (sh - 1);
    N = static_cast<uint64_t>(q);
    if (r > half || (r == half && (N & 1u))) ++N;  // round half to even
  }
  if (neg) *o++ = '-';
  const uint64_t ip = N / 10000u, fp = N % 10000u;
  char t[24];
  int k = 0;
  uint64_t a = ip;
  do {
    t[k++] = static_cast<char>('0' + a % 10u);
    a /= 10u;
  } while (a);
  while (k) *o++ = t[--k];
  *o++ = '.';
  o[0] = static_cast<char>('0' + fp / 1000u);
  o[1] = static_cast<char>('0' + fp / 100u % 10u);
  o[2] = static_cast<char>('0' + fp / 10u % 10u);
  o[3] = static_cast<char>('0' + fp % 10u);
  return o + 4;
}

char* fmt_u8(char* o, unsigned v) {
  if (v >= 100) *o++ = static_cast<char>('0' + v / 100u);
  if (v >= 10) *o++ = static_cast<char>('0' + v / 10u % 10u);
  *o++ = static_cast<char>('0' + v % 10u);
  return o;
}

bool ply_args_ok(const void* xyz, int xyz_dtype, const uint8_t* bgr, int64_t n) {
  return n >= 0 && (n == 0 || (xyz && bgr)) && (xyz_dtype == SL_XYZ_F32 || xyz_dtype == SL_XYZ_F64);
}

// Header + the point lines in `threads` contiguous parts (formatted in parallel).
void ply_format(const void* xyz, int xyz_dtype, const uint8_t* bgr, int64_t n, int threads, std::string& head,
                std::vector<std::vector<char>>& parts) {
  char hb[256];
  snprintf(hb, sizeof(hb),
           "ply\nformat ascii 1.0\nelement vertex %lld\nproperty float x\nproperty float y\n"
           "property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n",
           static_cast<long long>(n));
  head = hb;
  const int T = static_cast<int>(
      std::max<int64_t>(1, std::min<int64_t>(threads > 0 ? threads : 1, (n + 65535) / 65536)));
  parts.assign(T, {});
  constexpr size_t kLineMax = 3 * 330 + 16;  // worst case: three %.4f of ~1.8e308 + colours
  auto work = [&](int t) {
    const int64_t lo = n * t / T, hi = n * (t + 1) / T;
    std::vector<char>& b = parts[t];
    b.resize(static_cast<size_t>(hi - lo) * 64 + kLineMax);
    size_t used = 0;
    for (int64_t i = lo; i < hi; ++i) {
      if (used + kLineMax > b.size()) b.resize(b.size() * 2);
      char* o = b.data() + used;
      for (int k = 0; k < 3; ++k) {
        const double v = xyz_dtype == SL_XYZ_F64 ? static_cast<const double*>(xyz)[3 * i + k]
                                                 : static_cast<double>(static_cast<const float*>(xyz)[3 * i + k]);
        o = fmt4(o, v);
        *o++ = ' ';
      }
      o = fmt_u8(o, bgr[3 * i + 2]);
      *o++ = ' ';
      o = fmt_u8(o, bgr[3 * i + 1]);
      *o++ = ' ';
      o = fmt_u8(o, bgr[3 * i]);
      *o++ = '\n';
      used = static_cast<size_t>(o - b.data());
    }
    b.resize(used);
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

int sl_abi_version(void) { return SL_ABI_VERSION; }

int sl_ctx_create(int device, sl_ctx** out) {
  if (!out) return SL_EINVAL;
  *out = nullptr;
  sl_ctx* c = new sl_ctx();
  c->device = device;
  if (hipSetDevice(device) != hipSuccess) {
    delete c;
    return SL_EHIP;
  }
  // k_decode workgroups per CU when its grid is capped (SLGPU_DECODE_PER_CU,
  // default kDecodePerCu; 0 = uncapped)
  int per_cu = kDecodePerCu, n_cu = 0;
  if (const char* d = getenv("SLGPU_DECODE_PER_CU")) per_cu = atoi(d);
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n_cu < 1)
    n_cu = 256;
  c->n_cu = n_cu;
  if (per_cu > 0) c->decode_wgs = per_cu * n_cu;
  if (const char* d = getenv("SLGPU_PATH")) c->force_3k = atoi(d) == 3;
  if (const char* d = getenv("SLGPU_RECORDS")) c->rec_from_maps = atoi(d) == 0;
  if (const char* d = getenv("SLGPU_REC12")) c->rec12 = atoi(d) != 0;
  if (const char* d = getenv("SLGPU_VERIFY32")) c->verify32 = atoi(d) != 0;
  if (const char* d = getenv("SLGPU_STATS_SIDE")) {
    c->no_side = atoi(d) == 0;
    c->side_groups = atoi(d) == 1;
  }
  if (const char* d = getenv("SLGPU_XY_CALC")) c->xy_calc_env = atoi(d) != 0;
  if (const char* d = getenv("SLGPU_FUSED")) c->fused = atoi(d) != 0;
  if (const char* d = getenv("SLGPU_PRESTATS")) c->no_pre = atoi(d) == 0;
  if (const char* d = getenv("SLGPU_PRE_GROUPS")) c->no_pre_groups = atoi(d) == 0;
  if (const char* d = getenv("SLGPU_PRE_MIX")) c->pre_mix = atoi(d);
  if (const char* d = getenv("SLGPU_PRE_WGS")) c->pre_wgs = std::max(0, atoi(d));
  if (const char* d = getenv("SLGPU_PRE_DECODE")) c->pre_decode = atoi(d) != 0;
  if (const char* d = getenv("SLGPU_DECODE_BALANCE")) c->decode_balance = atoi(d) != 0;
  if (const char* d = getenv("SLGPU_DECODE_DYN")) c->decode_dyn = atoi(d) != 0 ? 1 : 0;
  if (const char* d = getenv("SLGPU_GROUP_CHUNKS"))
    c->max_chunks = std::max<int64_t>(1, std::min<int64_t>(kMaxChunks, atoll(d)));
  if (hipEventCreateWithFlags(&c->done_ev, hipEventDisableTiming) != hipSuccess) {
    delete c;
    return SL_EHIP;
  }
  *out = c;
  return SL_OK;
}

void sl_ctx_destroy(sl_ctx* c) {
  if (!c) return;
  (void)hipSetDevice(c->device);
  if (c->comm) {
    if (Rccl* R = rccl()) (void)R->comm_destroy(static_cast<ncclComm_t>(c->comm));
  }
  if (c->d_gcounts) (void)hipFree(c->d_gcounts);
  if (c->done_ev) (void)hipEventDestroy(c->done_ev);
  if (c->side) {
    (void)hipStreamSynchronize(c->side);
    (void)hipStreamDestroy(c->side);
  }
  for (hipEvent_t e : {c->hist_ev, c->stats_ev, c->entry_ev})
    if (e) (void)hipEventDestroy(e);
  for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
  for (void* ptr : {static_cast<void*>(c->d_planes), static_cast<void*>(c->d_xn), static_cast<void*>(c->d_yn),
                    static_cast<void*>(c->d_nc), static_cast<void*>(c->d_stats), static_cast<void*>(c->d_f32),
                    static_cast<void*>(c->d_codes), static_cast<void*>(c->d_hist[0]),
                    static_cast<void*>(c->d_hist[1]), static_cast<void*>(c->d_ptnib),
                    static_cast<void*>(c->d_block_sums), static_cast<void*>(c->d_chunk_counts),
                    static_cast<void*>(c->d_super[0]), static_cast<void*>(c->d_super[1]),
                    static_cast<void*>(c->d_lb), static_cast<void*>(c->d_pre[0]),
                    static_cast<void*>(c->d_pre[1]), static_cast<void*>(c->d_pre[2])})
    if (ptr) (void)hipFree(ptr);
  delete c;
}

const char* sl_ctx_last_error(const sl_ctx* c) { return c ? c->err.c_str() : "null context"; }

int sl_ctx_reserve(sl_ctx* c, int64_t max_views, int64_t max_px) {
  if (!c || max_views < 1 || max_px < 1) return fail(c, SL_EINVAL, "sl_ctx_reserve: bad sizes");
  HIP_TRY(c, hipSetDevice(c->device));
  const int64_t vpg = std::max<int64_t>(1, c->max_chunks / ((max_px + kChunk - 1) / kChunk));
  int r = ensure_scratch(c, std::min(vpg, max_views), max_px, true);
  if (r) return r;
  return grow(c, &c->d_stats, &c->cap_stats, max_views);
}

int sl_set_calib(sl_ctx* c, int H, int W, const double* K, const double* Oc, const double* planes,
                 int Wp, const double* Nc) {
  if (!c) return SL_EINVAL;
  if (H < 1 || W < 1 || Wp < 1 || !K || !Oc || !planes)
    return fail(c, SL_EINVAL, "sl_set_calib: bad arguments");
  if (Wp > kMaxWp) return fail(c, SL_EINVAL, "sl_set_calib: at most 32768 projector columns");
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
  // per plane: (n0, n1, n2, n.Oc + d) -- numer of sl_system.py:639,
  // np.dot(N.T, Oc).flatten() + d.  N.T there is planes[:, 0:3] of the
  // fancy-indexed (M, 4) C-ordered plane rows (:629-632), a strided
  // row-major operand, so numpy hands OpenBLAS a transposed dgemv: one
  // 3-term dot per row, evaluated fma(n2, o2, fma(n0, o0, n1 o1)) (measured
  // in this image on every row); then + d.  With Oc = 0
  // (calibrate_final) every order gives d exactly.
  std::vector<double> pl(4 * static_cast<size_t>(Wp));
  for (int i = 0; i < Wp; ++i) {
    const double* s = planes + 4 * static_cast<size_t>(i);
    pl[4 * i] = s[0];
    pl[4 * i + 1] = s[1];
    pl[4 * i + 2] = s[2];
    pl[4 * i + 3] = std::fma(s[2], Oc[2], std::fma(s[0], Oc[0], s[1] * Oc[1])) + s[3];
  }
  for (double* ptr : {c->d_planes, c->d_xn, c->d_yn, c->d_nc})
    if (ptr) HIP_TRY(c, hipFree(ptr));
  if (c->d_f32) HIP_TRY(c, hipFree(c->d_f32));
  c->d_planes = c->d_xn = c->d_yn = c->d_nc = nullptr;
  c->d_f32 = nullptr;
  c->has_calib = false;
  HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_planes), sizeof(double) * 4 * Wp));
  HIP_TRY(c, hipMemcpy(c->d_planes, pl.data(), sizeof(double) * 4 * Wp, hipMemcpyHostToDevice));
  HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_xn), sizeof(double) * W));
  HIP_TRY(c, hipMemcpy(c->d_xn, xn.data(), sizeof(double) * W, hipMemcpyHostToDevice));
  HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_yn), sizeof(double) * H));
  HIP_TRY(c, hipMemcpy(c->d_yn, yn.data(), sizeof(double) * H, hipMemcpyHostToDevice));
  {
    // planes32 [Wp][4] | xn32 [W] | yn32 [H] | pad to 16 B | planes12 [Wp][3] | 1 KB + 16 B of slack
    const size_t off12 = (4 * static_cast<size_t>(Wp) + W + H + 3) / 4 * 4;
    std::vector<float> f(off12 + 3 * static_cast<size_t>(Wp) + 260, 0.0f);
    for (int i = 0; i < Wp; ++i)
      for (int k = 0; k < 3; ++k) f[off12 + 3 * i + k] = static_cast<float>(pl[4 * i + k]);
    c->off12 = off12;
    for (int i = 0; i < 4 * Wp; ++i) f[i] = static_cast<float>(pl[i]);  // w: f32 of n.Oc + d
    for (int u = 0; u < W; ++u) f[4 * Wp + u] = static_cast<float>(xn[u]);
    for (int v = 0; v < H; ++v) f[4 * Wp + W + v] = static_cast<float>(yn[v]);
    // k_count's one-compare test: L (1.001e-6 + sum|n_i| 2^-20) at the largest
    // L = |x| + |y| + 1 of the frame and the largest sum|n_i| of the table
    // (of the f32 values the kernel reads), in f64, rounded up to f32
    double xm = 0.0, ym = 0.0, nm = 0.0;
    for (int u = 0; u < W; ++u) xm = std::max(xm, fabs(static_cast<double>(f[4 * Wp + u])));
    for (int v = 0; v < H; ++v) ym = std::max(ym, fabs(static_cast<double>(f[4 * Wp + W + v])));
    for (int i = 0; i < Wp; ++i)
      nm = std::max(nm, (fabs(static_cast<double>(f[4 * i])) + fabs(static_cast<double>(f[4 * i + 1]))) +
                            fabs(static_cast<double>(f[4 * i + 2])));
    const double thr = ((xm + ym) + 1.0) * (1.001e-6 + nm * 9.5367431640625e-07);
    float thr32 = static_cast<float>(thr);
    if (static_cast<double>(thr32) < thr) thr32 = nextafterf(thr32, INFINITY);
    c->fast_thr = std::isfinite(thr32) ? thr32 : INFINITY;
    HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_f32), sizeof(float) * f.size()));
    HIP_TRY(c, hipMemcpy(c->d_f32, f.data(), sizeof(float) * f.size(), hipMemcpyHostToDevice));
  }
  if (use_nc) {
    HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&c->d_nc), sizeof(double) * 3 * HW));
    HIP_TRY(c, hipMemcpy(c->d_nc, Nc, sizeof(double) * 3 * HW, hipMemcpyHostToDevice));
  }
  {  // the exact k_cloud's shared-reciprocal forms hold for every pixel's (x, y)
    auto safe = [](double v) { const double m = fabs(v); return m >= 0x1p-300 && m <= 0x1p300; };
    bool ok = true;
    for (int u = 0; u < W && ok; ++u) ok = safe(xn[u]);
    for (int v = 0; v < H && ok; ++v) ok = safe(yn[v]);
    c->xy_safe = ok;
    auto plain = [](double v) { const double m = fabs(v); return m >= 0x1p-20 && m <= 0x1p20; };
    ok = true;
    for (int u = 0; u < W && ok; ++u) ok = plain(xn[u]);
    for (int v = 0; v < H && ok; ++v) ok = plain(yn[v]);
    c->xy_plain = ok;
    ok = true;
    for (int i = 0; i < Wp && ok; ++i)
      ok = fabs(pl[4 * i + 3]) >= 0x1p-500 &&
           std::max(fabs(pl[4 * i]), std::max(fabs(pl[4 * i + 1]), fabs(pl[4 * i + 2]))) >= 0x1p-400;
    c->planes_plain = ok;
  }
  c->cam[0] = cx;
  c->cam[1] = cy;
  c->cam[2] = fx;
  c->cam[3] = fy;
  c->xy_calc = false;
  if (c->xy_calc_env) {  // may k_cloud compute the rays' x / y?  Checked on the device, entry by entry
    int* d_bad = nullptr;
    HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(&d_bad), sizeof(int)));
    int bad = 0;
    hipError_t e = hipMemcpy(d_bad, &bad, sizeof(int), hipMemcpyHostToDevice);
    if (e == hipSuccess) {
      hipLaunchKernelGGL(k_xy_check, dim3((W + H + 255) / 256), dim3(256), 0, nullptr, c->d_xn, W, c->d_yn, H, cx,
                         cy, fx, fy, d_bad);
      e = hipGetLastError();
    }
    if (e == hipSuccess) e = hipMemcpy(&bad, d_bad, sizeof(int), hipMemcpyDeviceToHost);
    (void)hipFree(d_bad);
    if (e != hipSuccess) return fail(c, SL_EHIP, hipGetErrorString(e));
    c->xy_calc = bad == 0;
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
  if (xyz && (xyz_dtype != SL_XYZ_F32 && xyz_dtype != SL_XYZ_F64 && xyz_dtype != SL_XYZ_F32_FAST))
    return fail(c, SL_EINVAL, "bad xyz_dtype");
  if (xyz && (!aligned16(xyz) || !aligned16(bgr))) return fail(c, SL_EINVAL, "xyz/bgr must be 16-byte aligned");
  if (xyz && cap < static_cast<int64_t>(n_views) * H * W)
    return fail(c, SL_ECAPACITY, "out_capacity < n_views*H*W");
  return SL_OK;
}

// k_cloud mode bits of an output dtype.  SL_XYZ_F32_FAST takes the f32 route
// only where its error bound holds as stated: Oc = 0 (P = r t, no
// cancellation), pinhole rays and no pose; otherwise it is SL_XYZ_F32.
static int xyz_mode_bits(const sl_ctx* c, int xyz_dtype, const double* poses) {
  const int nc_bit = c->d_nc ? M_NC : 0;
  if (xyz_dtype == SL_XYZ_F64) return M_XYZ64 | nc_bit;
  const bool pinhole0 = !c->d_nc && c->Oc[0] == 0.0 && c->Oc[1] == 0.0 && c->Oc[2] == 0.0;
  if (xyz_dtype == SL_XYZ_F32_FAST && pinhole0 && !poses) return M_FAST32;
  // SL_XYZ_F32 (and F32_FAST where its bound does not apply): the verified
  // shorter f64 route where P = r t (Oc = 0, pinhole rays; with or without a pose)
  return pinhole0 && c->verify32 && c->xy_plain && c->planes_plain ? M_VERIFY : nc_bit;
}

static void fill_common(sl_ctx* c, Params& p, int n_views, int H, int W) {
  memset(&p, 0, sizeof(p));
  p.HW = static_cast<int64_t>(H) * W;
  p.H = H;
  p.W = W;
  {  // n / W exact for n < HW: n * W < 2^w_shift (Granlund-Montgomery, round up)
    const uint64_t hw_w = static_cast<uint64_t>(p.HW) * static_cast<uint64_t>(W);
    int k = 0;
    while (k < 63 && (uint64_t{1} << k) <= hw_w) ++k;
    p.w_shift = k;
    p.w_magic = static_cast<uint32_t>((uint64_t{1} << k) / static_cast<uint64_t>(W) + 1);
  }
  p.n_views = n_views;
  p.cpv = static_cast<int>((p.HW + kChunk - 1) / kChunk);
  p.n_chunks = static_cast<int64_t>(n_views) * p.cpv;
  p.Wp = c->Wp;
  p.planes = reinterpret_cast<const double4*>(c->d_planes);
  p.xn = c->d_xn;
  p.yn = c->d_yn;
  p.planes32 = reinterpret_cast<const float4*>(c->d_f32);
  p.xn32 = c->d_f32 ? c->d_f32 + 4 * c->Wp : nullptr;
  p.yn32 = c->d_f32 ? c->d_f32 + 4 * c->Wp + c->W : nullptr;
  p.planes12 = c->d_f32 ? c->d_f32 + c->off12 : nullptr;
  p.fast_thr = c->fast_thr;
  p.xy_safe = c->xy_safe ? 1 : 0;
  p.xy_calc = c->xy_calc ? 1 : 0;
  p.cx = c->cam[0];
  p.cy = c->cam[1];
  p.fx = c->cam[2];
  p.fy = c->cam[3];
  p.rfx = 1.0 / c->cam[2];
  p.rfy = 1.0 / c->cam[3];
  p.nc_rays = c->d_nc;
  p.o0 = c->Oc[0];
  p.o1 = c->Oc[1];
  p.o2 = c->Oc[2];
}

int sl_decode_triangulate(sl_ctx* c, const uint8_t* stack, int64_t stack_vs, int n_views, int n_img,
                          int H, int W, int n_cols, int n_rows, const uint8_t* tex, int64_t tex_vs,
                          int mask_mode, const double* poses, int32_t* col_out, int32_t* row_out,
                          uint8_t* mask_out, void* xyz, int xyz_dtype, uint8_t* bgr, int64_t cap,
                          int64_t* view_offsets, void* stream) {
  if (!c) return SL_EINVAL;
  int64_t* masked = c->mc_next;  // armed by sl_mask_counts_to for this call only (consumed even on failure)
  c->mc_next = nullptr;
  const bool ready = c->ready_next;  // armed by sl_stack_ready for this call only (likewise)
  const hipEvent_t ready_ev = c->ready_ev_next;
  c->ready_next = false;
  c->ready_ev_next = nullptr;
  const PreArms arms = take_arms(c);  // sl_stack_next's declaration, a queued pre-stats pass (likewise)
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
  // k_decode reads each plane through a buffer descriptor of its own: a plane
  // (not a view's stack) must stay under 2 GiB; pixel offsets are 32-bit
  if (3 * HW >= (1ll << 31)) return fail(c, SL_EINVAL, "a frame must have fewer than 2^31 / 3 pixels");
  Params p;
  fill_common(c, p, n_views, H, W);
  p.stack = stack;
  p.stack_vs = stack_vs;
  const int64_t read_bytes = static_cast<int64_t>(2 + 2 * pairs) * HW;  // the planes k_decode reads
  const int plane_rsrc = read_bytes >= (1ll << 31) ? M_PLANE_RSRC : 0;
  p.view_bytes = static_cast<int>(std::min<int64_t>(read_bytes, INT32_MAX));
  p.tex = tex;
  p.tex_vs = tex_vs;
  p.nc = nc;
  p.nr = nr;
  p.kc = std::min(nc, pairs);
  p.kr = pairs - p.kc;
  p.poses = poses;
  p.col_out = col_out;
  p.row_out = row_out;
  p.mask_out = mask_out;
  p.xyz = xyz;
  p.bgr = bgr;
  p.out_cap = cap;
  p.view_offsets = view_offsets;
  p.masked = reinterpret_cast<unsigned long long*>(masked);
  const int nc_bit = (xyz && c->d_nc) ? M_NC : 0;
  const int hist_bit = mask_mode == SL_MASK_ADAPTIVE ? M_HIST : 0;
  const int decode_mode = (maps ? (M_MAPS | M_ROWS) : 0) | (xyz ? M_CODES : 0) | hist_bit | nc_bit | plane_rsrc;
  const int count_mode = (maps ? M_MAPS : 0) | (xyz ? M_CODES : 0) | hist_bit | nc_bit;
  const int cloud_mode = xyz ? (xyz_mode_bits(c, xyz_dtype, poses) | (tex ? M_TEX : 0)) : -1;
  const bool vec = (W % 16 == 0) && W >= 64 && aligned16(stack) && (stack_vs % 16 == 0) &&
                   (!tex || (aligned16(tex) && tex_vs % 16 == 0)) &&
                   (!maps || (aligned16(col_out) && aligned16(row_out) && aligned16(mask_out)));
  // aligned frames whose f32 tables fit k_decode's LDS: mask + decision in
  // k_decode ([k_stats] + k_decode + k_cloud), else k_decode + k_count + k_cloud
  // (a maps-only call reads no calibration table: k_decode loads its tables
  // only for a cloud, whose calibration common_out_checks matched to H x W)
  const bool decide = vec && !c->force_3k && W <= kDecX && H <= kDecY &&
                      (!xyz || (c->has_calib && c->W == W && c->H == H && c->Wp <= kDecPl));
  HIP_TRY(c, hipSetDevice(c->device));
  const hipStream_t s = static_cast<hipStream_t>(stream);
  r = stream_handoff(c, s);
  if (r) return r;
  return launch(c, p, vec, decide ? (decode_mode | M_DECIDE) : decode_mode, count_mode, cloud_mode, s, arms,
                ready, ready_ev);
}

int sl_stack_ready(sl_ctx* c, void* event) {
  if (!c) return SL_EINVAL;
  c->ready_next = true;
  c->ready_ev_next = static_cast<hipEvent_t>(event);
  return SL_OK;
}

int sl_stack_next(sl_ctx* c, const uint8_t* stack, int64_t stack_vs, int n_views) {
  if (!c) return SL_EINVAL;
  c->decl_next = false;
  if (!stack) {  // disarm, and drop a pass already queued for the next call (it computes its own)
    c->pre_armed = false;
    return SL_OK;
  }
  if (n_views < 1) return fail(c, SL_EINVAL, "sl_stack_next: n_views must be >= 1");
  if (!aligned16(stack) || stack_vs % 16 != 0 || stack_vs < 0)
    return fail(c, SL_EINVAL, "sl_stack_next: the stack and its view stride must be 16-byte aligned");
  c->decl_next = true;
  c->decl_stack = stack;
  c->decl_vs = stack_vs;
  c->decl_views = n_views;
  return SL_OK;
}

// A prepared sl_decode_triangulate: its arguments, kept for sl_call_run.
struct sl_call {
  sl_ctx* c;
  const uint8_t* stack;
  int64_t stack_vs;
  int n_views, n_img, H, W, n_cols, n_rows;
  const uint8_t* tex;
  int64_t tex_vs;
  int mask_mode;
  const double* poses;
  int32_t* col_out;
  int32_t* row_out;
  uint8_t* mask_out;
  void* xyz;
  int xyz_dtype;
  uint8_t* bgr;
  int64_t cap;
  int64_t* view_offsets;
};

int sl_call_prepare(sl_ctx* c, const uint8_t* stack, int64_t stack_vs, int n_views, int n_img, int H, int W,
                    int n_cols, int n_rows, const uint8_t* tex, int64_t tex_vs, int mask_mode, const double* poses,
                    int32_t* col_out, int32_t* row_out, uint8_t* mask_out, void* xyz, int xyz_dtype,
                    uint8_t* bgr, int64_t cap, int64_t* view_offsets, sl_call** out) {
  if (!c || !out) return SL_EINVAL;
  *out = nullptr;
  int r = common_out_checks(c, n_views, H, W, xyz, xyz_dtype, bgr, cap, view_offsets);
  if (r) return r;
  if (!stack) return fail(c, SL_EINVAL, "stack is NULL");
  *out = new sl_call{c, stack, stack_vs, n_views, n_img, H, W, n_cols, n_rows, tex, tex_vs, mask_mode, poses,
                     col_out, row_out, mask_out, xyz, xyz_dtype, bgr, cap, view_offsets};
  return SL_OK;
}

int sl_call_run(sl_call* k, void* stream) {
  if (!k) return SL_EINVAL;
  return sl_decode_triangulate(k->c, k->stack, k->stack_vs, k->n_views, k->n_img, k->H, k->W, k->n_cols, k->n_rows,
                               k->tex, k->tex_vs, k->mask_mode, k->poses, k->col_out, k->row_out, k->mask_out,
                               k->xyz, k->xyz_dtype, k->bgr, k->cap, k->view_offsets, stream);
}

void sl_call_destroy(sl_call* k) { delete k; }

int sl_triangulate_maps(sl_ctx* c, const int32_t* col_map, const uint8_t* mask, const uint8_t* tex,
                        int n_views, int H, int W, const double* poses, void* xyz, int xyz_dtype,
                        uint8_t* bgr, int64_t cap, int64_t* view_offsets, void* stream) {
  if (!c) return SL_EINVAL;
  const PreArms arms = take_arms(c);  // (consumed even on failure, as sl_decode_triangulate's)
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
  p.poses = poses;
  p.xyz = xyz;
  p.bgr = bgr;
  p.out_cap = cap;
  p.view_offsets = view_offsets;
  const int nc_bit = c->d_nc ? M_NC : 0;
  const int decode_mode = M_FROMMAPS | M_CODES | nc_bit;
  const int count_mode = M_FROMMAPS | M_CODES | nc_bit;
  const int cloud_mode = xyz_mode_bits(c, xyz_dtype, poses) | (tex ? M_TEX : 0);
  const bool vec = (W % 16 == 0) && W >= 64 && aligned16(col_map) && aligned16(mask) && aligned16(tex);
  HIP_TRY(c, hipSetDevice(c->device));
  const hipStream_t s = static_cast<hipStream_t>(stream);
  r = stream_handoff(c, s);
  if (r) return r;
  return launch(c, p, vec, decode_mode, count_mode, cloud_mode, s, arms);
}

int sl_mask_counts_to(sl_ctx* c, int64_t* device_counts) {
  if (!c) return SL_EINVAL;
  if (device_counts && (reinterpret_cast<uintptr_t>(device_counts) & 7u))
    return fail(c, SL_EINVAL, "sl_mask_counts_to: counts must be 8-byte aligned");
  c->mc_next = device_counts;
  return SL_OK;
}

int sl_sync(sl_ctx* c, void* stream) {
  if (!c) return SL_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  HIP_TRY(c, hipStreamSynchronize(static_cast<hipStream_t>(stream)));
  HIP_TRY(c, hipGetLastError());
  return SL_OK;
}

int sl_profile_enable(sl_ctx* c, int max_calls) {
  if (!c || max_calls < 0) return SL_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  for (hipEvent_t e : c->prof_ev) HIP_TRY(c, hipEventDestroy(e));
  c->prof_ev.clear();
  c->prof_groups.clear();
  c->prof_decide.clear();
  c->prof_n = 0;
  for (int i = 0; i < kProfEv * max_calls; ++i) {
    hipEvent_t e;
    HIP_TRY(c, hipEventCreate(&e));
    c->prof_ev.push_back(e);
  }
  return SL_OK;
}

int sl_profile_read(sl_ctx* c, double* decode_ms, double* count_ms, double* cloud_ms, int* calls) {
  if (!c) return SL_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  double t[3] = {0.0, 0.0, 0.0};
  for (int i = 0; i < c->prof_n; ++i) {
    const int ng = i < static_cast<int>(c->prof_groups.size()) ? c->prof_groups[i] : 0;
    for (int g = 0; g < ng; ++g) {
      hipEvent_t* ev = &c->prof_ev[kProfEv * i + 4 * g];
      HIP_TRY(c, hipEventSynchronize(ev[3]));
      const bool dz = i < static_cast<int>(c->prof_decide.size()) && c->prof_decide[i];
      for (int k = 0; k < 3; ++k) {
        float ms = 0.f;
        HIP_TRY(c, hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
        t[dz ? (k == 0 ? 1 : k == 1 ? 0 : 2) : k] += ms;  // M_DECIDE: (k_stats, k_decode, k_cloud)
      }
    }
  }
  c->prof_groups.clear();
  c->prof_decide.clear();
  if (decode_ms) *decode_ms = t[0];
  if (count_ms) *count_ms = t[1];
  if (cloud_ms) *cloud_ms = t[2];
  if (calls) *calls = c->prof_n;
  c->prof_n = 0;
  return SL_OK;
}

int sl_time_kernels(sl_ctx* c, int reps, double* decode_ms, double* count_ms, double* cloud_ms) {
  if (!c || reps < 1) return SL_EINVAL;
  if (!c->last.valid) return fail(c, SL_EINVAL, "sl_time_kernels: no earlier call to re-run");
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = c->last.s;
  hipEvent_t ev[4];
  for (int k = 0; k < 4; ++k) HIP_TRY(c, hipEventCreate(&ev[k]));
  int r = SL_OK;
  // k_cloud, then k_count, then k_decode: the consumers first -- k_cloud reads
  // the block and super-block sums (which the producers' re-runs add into
  // again) and k_decode's records; k_count reads the histogram k_decode's
  // re-runs accumulate into (reset below)
  // (M_DECIDE: k_cloud, then k_decode -- it reads the histograms k_stats'
  // re-runs accumulate into -- then k_stats)
  // k_cloud re-runs first in both paths: the producers' re-runs (k_count /
  // k_decode) add their block sums into the super-block sums again
  const int order3[3] = {2, 1, 0}, orderd[3] = {2, 0, 1};
  const int* order = c->last.decide ? orderd : order3;
  HIP_TRY(c, hipEventRecord(ev[0], s));
  for (int q = 0; q < 3 && r == SL_OK; ++q) {
    const int k = order[q];
    if (c->last.fn[k]) {
      Params p = c->last.p[k];
      void* args[] = {&p};
      for (int i = 0; i < reps; ++i) {
        const hipError_t e = hipLaunchKernel(c->last.fn[k], c->last.grid[k], dim3(kThreads), args, 0, s);
        if (e != hipSuccess) {
          r = fail(c, SL_EHIP, std::string("sl_time_kernels: ") + hipGetErrorString(e));
          break;
        }
      }
    }
    if (hipEventRecord(ev[q + 1], s) != hipSuccess && r == SL_OK) r = fail(c, SL_EHIP, "hipEventRecord");
  }
  double out[3] = {0.0, 0.0, 0.0};
  if (r == SL_OK && hipEventSynchronize(ev[3]) == hipSuccess) {
    for (int q = 0; q < 3; ++q) {
      float ms = 0.f;
      const int k = order[q];
      if (hipEventElapsedTime(&ms, ev[q], ev[q + 1]) == hipSuccess) out[k] = c->last.fn[k] ? ms / reps : 0.0;
    }
  }
  // a dynamic k_decode (decode_dyn) claims chunk groups from per-view counters
  // that its launch leaves exhausted: each re-run gets fresh counters (zeroed
  // outside its events) and is timed alone
  if (r == SL_OK && c->last.fn[0] && c->last.p[0].decode_dyn) {
    Params p = c->last.p[0];
    void* args[] = {&p};
    const unsigned nv = c->last.grid[0].y;
    unsigned* ctr = p.super_sums + (p.super_cap - nv);
    double sum = 0.0;
    for (int i = 0; i < reps && r == SL_OK; ++i) {
      float ms = 0.f;
      if (hipMemsetAsync(ctr, 0, sizeof(unsigned) * nv, s) != hipSuccess || hipEventRecord(ev[0], s) != hipSuccess ||
          hipLaunchKernel(c->last.fn[0], c->last.grid[0], dim3(kThreads), args, 0, s) != hipSuccess ||
          hipEventRecord(ev[1], s) != hipSuccess || hipEventSynchronize(ev[1]) != hipSuccess ||
          hipEventElapsedTime(&ms, ev[0], ev[1]) != hipSuccess) {
        r = fail(c, SL_EHIP, "sl_time_kernels: dynamic k_decode re-run");
        break;
      }
      sum += ms;
    }
    if (r == SL_OK) out[0] = sum / reps;
  }
  for (int k = 0; k < 4; ++k) (void)hipEventDestroy(ev[k]);
  // the re-runs accumulated into the histograms: the next calls start from zero
  for (int b = 0; b < 2; ++b) c->hist_dirty[b] = c->cap_hist[b];
  c->last.valid = false;
  if (decode_ms) *decode_ms = out[0];
  if (count_ms) *count_ms = out[1];
  if (cloud_ms) *cloud_ms = out[2];
  return r;
}

int sl_last_launch_info(sl_ctx* c, int* path, int64_t* launches, int64_t* last_launch_px) {
  if (!c) return SL_EINVAL;
  if (path) *path = c->last.fused ? 2 : c->last.decide ? 1 : 0;
  if (launches) *launches = c->last_launches;
  if (last_launch_px) *last_launch_px = c->last_launch_px;
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

int sl_format_ply(const void* xyz, int xyz_dtype, const uint8_t* bgr, int64_t n, int threads, char* out,
                  int64_t out_capacity, int64_t* out_len) {
  if (!out_len || !ply_args_ok(xyz, xyz_dtype, bgr, n)) return SL_EINVAL;
  std::string head;
  std::vector<std::vector<char>> parts;
  ply_format(xyz, xyz_dtype, bgr, n, threads, head, parts);
  int64_t len = static_cast<int64_t>(head.size());
  for (auto& pp : parts) len += static_cast<int64_t>(pp.size());
  *out_len = len;
  if (!out) return SL_OK;  // size query
  if (out_capacity < len) return SL_ECAPACITY;
  memcpy(out, head.data(), head.size());
  int64_t off = static_cast<int64_t>(head.size());
  for (auto& pp : parts) {
    if (!pp.empty()) memcpy(out + off, pp.data(), pp.size());
    off += static_cast<int64_t>(pp.size());
  }
  return SL_OK;
}

int sl_write_ply(const char* path, const void* xyz, int xyz_dtype, const uint8_t* bgr, int64_t n, int threads) {
  if (!path || !ply_args_ok(xyz, xyz_dtype, bgr, n)) return SL_EINVAL;
  std::string head;
  std::vector<std::vector<char>> parts;
  ply_format(xyz, xyz_dtype, bgr, n, threads, head, parts);
  FILE* f = fopen(path, "wb");
  if (!f) return SL_EIO;
  bool ok = fwrite(head.data(), 1, head.size(), f) == head.size();
  for (auto& pp : parts)
    if (ok && !pp.empty()) ok = fwrite(pp.data(), 1, pp.size(), f) == pp.size();
  ok = (fclose(f) == 0) && ok;
  return ok ? SL_OK : SL_EIO;
}

// Binary little-endian PLY with the reference header's properties (float
// x y z, uchar red green blue): 15-byte records, packed on `threads` threads.
int sl_write_ply_binary(const char* path, const void* xyz, int xyz_dtype, const uint8_t* bgr, int64_t n,
                        int threads) {
  if (!path || !ply_args_ok(xyz, xyz_dtype, bgr, n)) return SL_EINVAL;
  char hb[256];
  const int hl = snprintf(hb, sizeof(hb),
                          "ply\nformat binary_little_endian 1.0\nelement vertex %lld\nproperty float x\n"
                          "property float y\nproperty float z\nproperty uchar red\nproperty uchar green\n"
                          "property uchar blue\nend_header\n",
                          static_cast<long long>(n));
  std::vector<char> body;
  try {
    body.resize(static_cast<size_t>(n) * 15);
  } catch (const std::bad_alloc&) {
    return SL_EINVAL;
  }
  const int T = static_cast<int>(
      std::max<int64_t>(1, std::min<int64_t>(threads > 0 ? threads : 1, (n + 262143) / 262144)));
  auto work = [&](int t) {
    const int64_t lo = n * t / T, hi = n * (t + 1) / T;
    char* o = body.data() + 15 * lo;
    for (int64_t i = lo; i < hi; ++i, o += 15) {
      float v[3];
      for (int k = 0; k < 3; ++k)
        v[k] = xyz_dtype == SL_XYZ_F64 ? static_cast<float>(static_cast<const double*>(xyz)[3 * i + k])
                                       : static_cast<const float*>(xyz)[3 * i + k];
      memcpy(o, v, 12);
      o[12] = static_cast<char>(bgr[3 * i + 2]);
      o[13] = static_cast<char>(bgr[3 * i + 1]);
      o[14] = static_cast<char>(bgr[3 * i]);
    }
  };
  std::vector<std::thread> pool;
  for (int t = 1; t < T; ++t) pool.emplace_back(work, t);
  work(0);
  for (auto& th : pool) th.join();
  FILE* f = fopen(path, "wb");
  if (!f) return SL_EIO;
  bool ok = fwrite(hb, 1, static_cast<size_t>(hl), f) == static_cast<size_t>(hl);
  if (ok && n) ok = fwrite(body.data(), 1, body.size(), f) == body.size();
  ok = (fclose(f) == 0) && ok;
  return ok ? SL_OK : SL_EIO;
}

}  // extern "C"


extern "C" {

int sl_gather_unique_id(uint8_t* id_out) {
  Rccl* R = rccl();
  if (!id_out) return SL_EINVAL;
  if (!R) return SL_EHIP;
  ncclUniqueId id;
  if (R->get_unique_id(&id) != ncclSuccess) return SL_EHIP;
  memcpy(id_out, id.internal, NCCL_UNIQUE_ID_BYTES);
  return SL_OK;
}

int sl_gather_init(sl_ctx* c, int nranks, int rank, const uint8_t* id) {
  if (!c) return SL_EINVAL;
  if (nranks < 1 || rank < 0 || rank >= nranks || !id) return fail(c, SL_EINVAL, "sl_gather_init: bad rank / id");
  Rccl* R = rccl();
  if (!R) return fail(c, SL_EHIP, "sl_gather_init: RCCL (librccl.so) could not be loaded");
  HIP_TRY(c, hipSetDevice(c->device));
  if (c->comm) {
    (void)R->comm_destroy(static_cast<ncclComm_t>(c->comm));
    c->comm = nullptr;
  }
  ncclUniqueId uid;
  memcpy(uid.internal, id, NCCL_UNIQUE_ID_BYTES);
  ncclComm_t comm = nullptr;
  NCCL_TRY(c, R->comm_init_rank(&comm, nranks, uid, rank));
  c->comm = comm;
  c->nranks = nranks;
  c->rank = rank;
  return grow(c, &c->d_gcounts, &c->cap_gcounts, 2 * static_cast<int64_t>(nranks));
}

int sl_gather_counts(sl_ctx* c, int64_t n_local, int64_t* counts_out, void* stream) {
  if (!c) return SL_EINVAL;
  if (!c->comm) return fail(c, SL_EINVAL, "sl_gather_counts: sl_gather_init has not been called");
  if (n_local < 0 || !counts_out) return fail(c, SL_EINVAL, "sl_gather_counts: bad arguments");
  Rccl* R = rccl();
  hipStream_t s = static_cast<hipStream_t>(stream);
  HIP_TRY(c, hipSetDevice(c->device));
  int64_t* d_mine = c->d_gcounts + c->nranks;
  HIP_TRY(c, hipMemcpyAsync(d_mine, &n_local, sizeof(int64_t), hipMemcpyHostToDevice, s));
  NCCL_TRY(c, R->all_gather(d_mine, c->d_gcounts, 1, ncclInt64, static_cast<ncclComm_t>(c->comm), s));
  HIP_TRY(c, hipMemcpyAsync(counts_out, c->d_gcounts, sizeof(int64_t) * c->nranks, hipMemcpyDeviceToHost, s));
  HIP_TRY(c, hipStreamSynchronize(s));
  return SL_OK;
}

int sl_gather(sl_ctx* c, const void* xyz, int xyz_dtype, const uint8_t* bgr, const int64_t* counts, int root,
              void* xyz_out, uint8_t* bgr_out, void* stream) {
  if (!c) return SL_EINVAL;
  if (!c->comm) return fail(c, SL_EINVAL, "sl_gather: sl_gather_init has not been called");
  if (root < 0 || root >= c->nranks || !counts) return fail(c, SL_EINVAL, "sl_gather: bad arguments");
  if (xyz_dtype != SL_XYZ_F32 && xyz_dtype != SL_XYZ_F64) return fail(c, SL_EINVAL, "sl_gather: bad xyz_dtype");
  const int64_t n_local = counts[c->rank];
  if (n_local < 0 || (n_local && (!xyz || !bgr))) return fail(c, SL_EINVAL, "sl_gather: bad local cloud");
  int64_t total = 0;
  for (int r = 0; r < c->nranks; ++r) total += counts[r];
  if (c->rank == root && total && (!xyz_out || !bgr_out))
    return fail(c, SL_EINVAL, "sl_gather: the root needs output buffers");
  Rccl* R = rccl();
  ncclComm_t comm = static_cast<ncclComm_t>(c->comm);
  hipStream_t s = static_cast<hipStream_t>(stream);
  HIP_TRY(c, hipSetDevice(c->device));
  const size_t esz = 3 * (xyz_dtype == SL_XYZ_F64 ? sizeof(double) : sizeof(float));
  if (c->rank == root) {  // the root's own part: a device copy
    int64_t off = 0;
    for (int r = 0; r < root; ++r) off += counts[r];
    if (n_local) {
      HIP_TRY(c, hipMemcpyAsync(static_cast<uint8_t*>(xyz_out) + off * esz, xyz, n_local * esz,
                                hipMemcpyDeviceToDevice, s));
      HIP_TRY(c, hipMemcpyAsync(bgr_out + 3 * off, bgr, 3 * n_local, hipMemcpyDeviceToDevice, s));
    }
  }
  // Inside the group every failure is recorded and the group is still closed:
  // an open group would capture this thread's later RCCL calls (torch's too,
  // the library handle is shared).
  NCCL_TRY(c, R->group_start());
  ncclResult_t first = ncclSuccess;
  const char* what = "";
  auto rec = [&](ncclResult_t e, const char* op) {
    if (e != ncclSuccess && first == ncclSuccess) {
      first = e;
      what = op;
    }
  };
  int64_t off = 0;
  for (int r = 0; r < c->nranks && first == ncclSuccess; ++r) {
    const int64_t n = counts[r];
    if (c->rank == root && r != root && n) {
      rec(R->recv(static_cast<uint8_t*>(xyz_out) + off * esz, n * esz, ncclUint8, r, comm, s), "ncclRecv(xyz)");
      if (first == ncclSuccess) rec(R->recv(bgr_out + 3 * off, 3 * n, ncclUint8, r, comm, s), "ncclRecv(bgr)");
    }
    off += n;
  }
  if (c->rank != root && n_local && first == ncclSuccess) {
    rec(R->send(xyz, n_local * esz, ncclUint8, root, comm, s), "ncclSend(xyz)");
    if (first == ncclSuccess) rec(R->send(bgr, 3 * n_local, ncclUint8, root, comm, s), "ncclSend(bgr)");
  }
  const ncclResult_t ge = R->group_end();
  if (first != ncclSuccess) return fail(c, SL_EHIP, std::string(what) + ": " + R->error_string(first));
  if (ge != ncclSuccess) return fail(c, SL_EHIP, std::string("ncclGroupEnd: ") + R->error_string(ge));
  return SL_OK;
}

const char* sl_last_error(const sl_ctx* c) { return sl_ctx_last_error(c); }

int sl_decode_triangulate_batch(sl_ctx* c, const uint8_t* stack, int64_t stack_vs, int n_views, int n_img, int H,
                                int W, int n_cols, int n_rows, const uint8_t* tex, int64_t tex_vs, int mask_mode,
                                const double* poses, int32_t* col_out, int32_t* row_out, uint8_t* mask_out,
                                void* xyz, int xyz_dtype, uint8_t* bgr, int64_t cap, int64_t* view_offsets,
                                void* stream) {
  return sl_decode_triangulate(c, stack, stack_vs, n_views, n_img, H, W, n_cols, n_rows, tex, tex_vs, mask_mode,
                               poses, col_out, row_out, mask_out, xyz, xyz_dtype, bgr, cap, view_offsets, stream);
}

}  // extern "C"
