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
// Default path (aligned frames, decision tables in LDS), per launch group on
// one HIP stream, no host synchronisation between the kernels:
//   k_stats  : (adaptive mask) the black-plane histogram + max(white - black)
//              of every view -- or the same pass run by the previous call's
//              k_cloud (pre-stats, sl_stack_next);
//   k_decode : streams the uint8 stack once, Gray bits by byte-SWAR compares,
//              Gray -> binary in the byte lanes; col/row/mask maps, the mask
//              and the |n.r| > 1e-6 decision, 12-bit records, block sums;
//   k_cloud  : the chunk's output offset from the super-block and block sums,
//              its points compacted in LDS, the ray/plane intersection in the
//              reference's f64 order (or its proven-equal verified form), the
//              stores at offset + rank -- the reference's np.where order.
// Frames that do not fit it (unaligned, W or H > 4096, Wp > 2048) run
// k_decode (codes + histogram) -> k_count (mask, decision) -> k_cloud.
//
// Scratch at a launch-group boundary never depends on the host's view of the
// sequence, so a captured hipGraph replays in any phase: the histograms are
// zeroed by their last reader (k_decode / k_count, a per-view arrival
// counter); the super-block sums alternate between two buffers selected on
// the device -- the producer (k_decode / k_count) accumulates into the buffer
// selector word par[0] names and zeroes the other one (super_produce), the
// consumer (k_cloud) only flips the selector (super_consume), so the buffer it
// read keeps its sums until the next producer zeroes it.  The one thing that
// crosses a boundary is a pre-stats pass queued for the next call, which the
// host hands on only within one capture (or eager call sequence).
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
#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <condition_variable>
#include <memory>
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
constexpr int kRing = 40;               // stack planes in flight per lane
// Cache policies (measured): the stack streams with nt loads
// (aux 2); the side loads (records, texture, the histogram pass's white and
// black) keep the default policy, whose lines the next kernel finds in the
// Infinity Cache; cloud-only records leave write-through (sc1, aux 16).
constexpr int kLoadAux = 2;
constexpr int kRecAux = 16;
constexpr int kMapAux = 2;  // nt: the maps and xyz are never read back by the path
typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint4 ld_side16(const void* p) { return *reinterpret_cast<const uint4*>(p); }
__device__ __forceinline__ uint2 ld_side8(const void* p) { return *reinterpret_cast<const uint2*>(p); }
__device__ __forceinline__ uint32_t ld_side4(const void* p) { return *reinterpret_cast<const uint32_t*>(p); }

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
constexpr int M_DECIDE = 256;  // k_decode: also the mask and the |n.r| decision (k_count's work; k_stats
                               // histograms): mask map, 12-bit records, chunk counts, block sums
constexpr float kFastKappa = 16.0f;  // condition-number limit of the f32 route

constexpr int kSlot = 272;      // histogram of one view: 256 bins + max + arrival counters + pad (u32)
constexpr int kSlotArrive = 257;  // ... its readers' two-level arrival counter (9 words, arrive_last<8>)
constexpr int kHistRep = 8;     // LDS histogram replicas (lane % kHistRep; 8 measured best of 1/4/8/16/32/64)
constexpr int kHistStride = kHistRep + 1;  // bin stride: replica r of bin b sits in bank (b + r) % 32
constexpr int kMaxWp = 32768;              // projector columns (record codes are 15 bits)
constexpr int64_t kMaxChunks = 1 << 16;    // chunks per launch group: bounds k_cloud's prefix reads
// Cloud-only calls keep the 12-bit records in chunk slots (1536 B: a lane's 16
// codes as 16 B at 16 lane + 8 B at 1024 + 8 lane), the launch group's views
// interleaved by chunk group (rec_slot), stored write-through; calls with maps
// keep pixel order, 24 B per lane as two 12-B stores (their registers fit).
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
  int rec12;               // decide path (Wp <= 2048): records packed 12 bits per pixel, 24 B per 16
                           // pixels, code 0xfff = no point (1.5 B/px written, no point nibbles)
  int rec_blk;             // rec12 records in chunk slots (k_decode without maps; else pixel order)
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
  // the adaptive mask's histograms: [view][kHistView] (decide path, k_stats /
  // pre-stats replicas) or [view][kSlot] (3-kernel path, k_decode's); clean
  // before the producing launch, zeroed by the consuming kernel's last reader
  // of each view (arrival counter at word kSlotArrive of the view's first slot)
  unsigned* hist;
  const int64_t* base_in;  // points of the earlier launch groups of this call, or null
  int* chunk_counts;       // k_count -> k_cloud: points per chunk
  int* block_sums;         // k_count -> k_cloud: points per workgroup (4 chunks)
  int bs_atomic;           // k_decode M_DECIDE: block sums by the last wave to arrive (no barrier)
  int decode_dyn;          // k_decode M_DECIDE | M_CODES: chunk groups after the first round pulled from a
                           // per-view counter (super_sums' last entries), not strided (cloud-only calls)
  // two-level block prefix: every block (workgroup of 4 chunks) also adds its
  // sum to super[block >> sb_shift]; k_cloud's offset = the super-block sums
  // before its super-block + the block sums before it inside it.  Two buffers
  // of kSuperCap words (super-block sums + the dynamic grid's counters, their
  // last n_views entries) at super_base, selected on the device (super_sel).
  unsigned* super_base;
  unsigned* super_par;     // [0]: the buffer the next producer accumulates into, [1]: the one k_cloud reads
  int sb_shift;
  int rerun;               // sl_time_kernels' re-runs: consumers leave their inputs as they are
  int cloud_gx;            // k_cloud: workgroups per view that triangulate (the grid's first x: pre-stats)
  // k_cloud's pre-stats workgroups (sl_stack_next): the NEXT call's histogram
  // pass (k_stats' work) for the views of its first launch group, beside this
  // call's triangulation; null pre_stack: none
  const uint8_t* pre_stack;
  int64_t pre_vs;
  unsigned* pre_hist;      // [pre_views][kHistView] accumulated (clean before the launch)
  int pre_views;           // views of the next call's first group
  int pre_bpv;             // workgroups per view (k_stats' grid x)
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
    const uint4 wq = ld_side16(vb + 16 * i);
    const uint4 bq = ld_side16(vb + HW + 16 * i);
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
// p.hist is clean (the last consumer zeroed it, or the host did).
__global__ __launch_bounds__(kThreads) void k_stats(Params p) {
  __shared__ unsigned s_hist[256 * kHistStride];
  __shared__ int s_max[kWaves];
  const int view = blockIdx.y;
  stats_pass(p.stack + view * p.stack_vs, p.HW, blockIdx.x, gridDim.x, p.hist + static_cast<int64_t>(view) * kHistView,
             s_hist, s_max);
}

// One pre-stats workgroup (sl_stack_next), number sx of the nsx per grid row
// that a k_cloud launch appends: its share of the next call's histogram pass
// (k_stats' work) into p.pre_hist.
__device__ __forceinline__ void pre_stats_block(const Params& p, int64_t sx, int64_t nsx, unsigned* s_hist,
                                                int* s_max) {
  const int64_t sblk = static_cast<int64_t>(blockIdx.y) * nsx + sx;
  const int64_t total = static_cast<int64_t>(p.pre_views) * p.pre_bpv;
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

// Reader `id` of `readers` (ids 0 .. readers - 1, each arriving once) at a
// two-level arrival counter ctr[0 .. S]: ctr[1 + id % S] counts the readers of
// its class, the last of each class adds one at ctr[0], and the last of those
// is the last reader.  (One counter hit by every workgroup of a launch
// serialises them: k_cloud 33 -> 51 us per c2 step with a single one.)
template <int S>
__device__ __forceinline__ bool arrive_last(unsigned* ctr, unsigned id, unsigned readers) {
  const unsigned cls = id & (S - 1);
  const unsigned n_cls = (readers - cls + S - 1) / S;  // readers of this class (id < readers)
  if (atomicAdd(ctr + 1 + cls, 1u) + 1u != n_cls) return false;
  return atomicAdd(ctr, 1u) + 1u == min(readers, static_cast<unsigned>(S));
}

// One reader (a whole wave, number id of `readers`) of a view's `words`
// histogram words at h is done with them: the empty asm consumes values
// computed from them (the thresholds), so every load has returned before the
// arrival is counted at h[kSlotArrive ..]; the last reader zeroes the words,
// the counters included, so the buffer is clean for the next producer
// whatever launch comes next.
__device__ __forceinline__ void hist_release(unsigned* h, int words, unsigned id, unsigned readers, int lane,
                                             uint32_t dep0, uint32_t dep1) {
  asm volatile("" ::"v"(dep0), "v"(dep1) : "memory");
  unsigned last = 0u;
  if (lane == 0) last = arrive_last<8>(h + kSlotArrive, id, readers) ? 1u : 0u;
  if (__shfl(static_cast<int>(last), 0, 64)) {
    uint4* h4 = reinterpret_cast<uint4*>(h);
    for (int i = lane; i < words / 4; i += 64) h4[i] = make_uint4(0u, 0u, 0u, 0u);
  }
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

// k_decode M_DECIDE: the f32 plane table and xn = (u - cx) / fx in LDS, by
// LDS-DMA while the first chunk group's stack loads are in flight (host: Wp <=
// kDecPl, W <= kDecX, H <= kDecY; the launch's grid is capped at a few
// workgroups per CU, so the fill is cheap); yn = (v - cy) / fy is one early
// global load per lane.
constexpr int kDecPl = 2048, kDecX = 4096, kDecY = 4096;
constexpr int kDecPlWords = kDecPl * 4;  // LDS words of the plane table
constexpr int kBsSlots = 64;     // k_decode M_DECIDE: chunk-group iterations per workgroup with a barrier-free block sum
constexpr int kSuperCap = 4096;  // super-block sums per launch group (>= sqrt of its blocks) + dynamic-grid counters
constexpr int kSuperWords = 2 * kSuperCap + 4;  // two buffers + their selector words (super_par)

// The super-block buffers alternate from launch group to launch group, and
// the device, not the host, keeps the alternation: the producer of a group's
// block sums (k_decode on the decide path, k_count otherwise) reads selector
// word par[0], accumulates into that buffer, zeroes the other one (its last
// reader, the previous group's k_cloud, is done) and writes par[1] = its
// buffer; k_cloud reads par[1] and writes par[0] = the other buffer.  Each
// word is written only by the kernel that does not read it, so every
// workgroup of a launch sees one value, and a captured graph replays in any
// phase (no host state is baked into its launches).  Re-runs
// (sl_time_kernels) leave both alone.
__device__ __forceinline__ unsigned* super_produce(const Params& p) {
  const unsigned sel = p.super_par[0] & 1u;
  if (!p.rerun && blockIdx.x == 0 && blockIdx.y == 0) {
    unsigned* other = p.super_base + (sel ^ 1u) * kSuperCap;
    for (int i = threadIdx.x; i < kSuperCap; i += kThreads) other[i] = 0u;
    if (threadIdx.x == 0) p.super_par[1] = sel;
  }
  return p.super_base + sel * kSuperCap;
}
__device__ __forceinline__ const unsigned* super_consume(const Params& p, int bx) {
  const unsigned sel = p.super_par[1] & 1u;
  if (!p.rerun && bx == 0 && blockIdx.y == 0 && threadIdx.x == 0) p.super_par[0] = sel ^ 1u;
  return p.super_base + sel * kSuperCap;
}
constexpr int kDecodeLds = (kDecPlWords + kDecX) * 4;  // bytes: > the histogram replicas
static_assert(kDecodeLds >= 256 * kHistStride * 4, "the decode LDS holds the histogram replicas too");

// ================================================================ k_decode ====
// gray_decode (sl_system.py:519-577) for one chunk per wave, in the streaming
// layout (lane l owns the chunk's pixels [16 l, 16 l + 16)): column and row
// code of every pixel, reading each plane of the uint8 stack once (M_FROMMAPS:
// a caller's col_map instead).  Outputs by mode bit:
//   M_MAPS   col/row int32 maps, full frame, unmasked (what gray_decode
//            returns), 1 KB contiguous per store instruction through an LDS
//            stage (config 2 120.3-120.6 -> 116.5-117.4 us per step,
//            profiles/r04_ab/map_stage_lines.jsonl);
//   M_CODES  the record min(col, Wp-1) (np.clip, sl_system.py:626) per pixel
//            for k_count / k_cloud (M_DECIDE: 12 bits, 0xfff = no point);
//   M_HIST   (3-kernel path) the view's black-plane histogram and max(white -
//            black) (sl_system.py:526-528): LDS replicas bank-skewed so that
//            the lanes of a half-wave that hit the same bin use 32 different
//            banks, added to the view's global histogram once per workgroup;
//   M_DECIDE the mask from k_stats' histograms (or fixed thresholds), the mask
//            map, the |n.r| > 1e-6 decision, chunk counts and block sums.
// Grid (chunk groups, views), capped at kDecodePerCu workgroups per CU:
// chunk groups strided over the grid's x, or (decode_dyn, cloud-only calls)
// pulled from a per-view counter after the first round.
constexpr int kDecodePerCu = 3;  // k_decode grid cap, workgroups per CU
template <int KC, int KR, int MODE, int VEC>
__global__ __launch_bounds__(kThreads, 3) void k_decode(Params p) {
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
  __shared__ int s_next[2];              // decode_dyn: the workgroup's next chunk group
  // a 1-KB stage per wave for contiguous map stores (maps kernels only)
  __shared__ uint4 s_mapst[(MODE < 0 || (MODE & M_MAPS)) ? 64 * kWaves : 1];
  unsigned* s_hist = s_lds;
  float4* s_pl = reinterpret_cast<float4*>(s_lds);
  float* s_xn = reinterpret_cast<float*>(s_lds) + kDecPlWords;
  const bool decide = (mode & M_DECIDE) != 0;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform, provably
  const int view = blockIdx.y;
  const int64_t HW = p.HW;
  const int gx = static_cast<int>(gridDim.x);  // decoding workgroups per view
  if (decide) {
    if (tid < kBsSlots) s_bsum[tid] = 0u;
    if (tid == 0) s_mcount = 0u;  // published by the barrier of iteration 0
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
    // clamped to the LDS the tables own all the same.  By LDS-DMA (16 B per
    // lane, 1 KB per wave instruction): no VGPRs, and the first chunk group's
    // stack loads below are issued while they land; the workgroup barrier
    // before the first mask (iteration 0) publishes them.  Lanes past the end
    // repeat the last entry into slack LDS (kDecPl, kDecX are multiples of 64
    // entries).
    if (mode & M_CODES) {
      const int wp_t = min(p.Wp, kDecPl), w_t = min(p.W, kDecX);
      typedef __attribute__((address_space(3))) void* lds_ptr_t;
      for (int i = wid; i * 64 < wp_t; i += kWaves)
        __builtin_amdgcn_global_load_lds(p.planes32 + min(i * 64 + lane, wp_t - 1), (lds_ptr_t)(s_pl + i * 64), 16, 0, 0);
      for (int i = wid; i * 256 < w_t; i += kWaves)
        __builtin_amdgcn_global_load_lds(p.xn32 + min(i * 256 + 4 * lane, w_t - 4), (lds_ptr_t)(s_xn + i * 256), 16, 0, 0);
    }
  }
  uint32_t tw2 = static_cast<uint32_t>(40 + 1) * 0x00010001u;      // fixed mask:
  uint32_t tc2 = static_cast<uint32_t>(10 + 17) * 0x00010001u;     // multi_point_cloud_process.py:36-38
  int it = 0;

  if (hist) {
    for (int i = tid; i < 256 * kHistStride; i += kThreads) s_hist[i] = 0u;
    __syncthreads();
  }

  // Chunk groups of the view, strided over the grid's x (or pulled
  // dynamically); the workgroup-uniform loop holds no barrier but the
  // first iteration's (M_DECIDE) and the block sums' (unless bs_atomic).
  const int ngroups = (p.cpv + kWaves - 1) / kWaves;
  int mx_acc = -1024;
  const bool dyn = p.decode_dyn && decide && (mode & M_CODES) && !p.bs_atomic;
  unsigned* const sup = (decide && (mode & M_CODES)) ? super_produce(p) : nullptr;
  unsigned* const dyn_ctr = sup + (kSuperCap - 1 - view);
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

  // M_DECIDE: the row's yn first (the oldest load: waiting for it never
  // waits for this iteration's stores)
  const float ys_early = (decide && (mode & M_CODES) && n_px > 0) ? p.yn32[row_of(p, static_cast<int>(px0))] : 0.0f;
  uint32_t col[kPx];
  uint32_t pt_rec = 0xffffu;  // the lane's point bits for 12-bit records (decide path)
  uint4 wq = make_uint4(0u, 0u, 0u, 0u), bq = wq;
  // binary code words per byte lane (pixel 4 w + e in byte 3 - e): a code's
  // top min(k, 8) bits in A, the rest in B
  uint32_t rA[4] = {0, 0, 0, 0}, rB[4] = {0, 0, 0, 0};
  const int rBn = krr > 8 ? krr - 8 : 0;
  const int rSh = nr - krr;
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
    wq = ldp(0);
    bq = ldp(1);
    // ---- Gray bit planes: (pattern, inverse) pairs, columns then rows ----
    // Each (pattern, inverse) compare is one v_bitop3 per word; the bit enters
    // at bit 7 of its byte lane and the lane shifts right, acc = (acc >> 1 &
    // 0x7f..) | (bit7 & 0x80..): at most 8 bits per byte lane, so no carry
    // crosses into the neighbouring pixel; codes of up to 16 bits use A then
    // B.  The first pair ends lowest, bit-reversed below.
    const int npl = 2 * (kc + krr);
    uint32_t cA[4] = {0, 0, 0, 0}, cB[4] = {0, 0, 0, 0};
    auto consume = [&](const uint4& P, const uint4& I, int pair) {
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
    // ---- Gray -> binary in the byte lanes, 4 pixels per instruction ----
    // bitreverse puts each byte lane's bits MSB-first in its low bits (pixel
    // 4 w + e in byte 3 - e); B's bits continue A's prefix xor, so A's binary
    // lowest bit (the parity of its Gray bits) is xor-ed into B's top bit
    // before B's own conversion.  Codes shifted by sh = n - k bits (fewer
    // patterns than code bits): binary(g << sh) = binary(g) << sh with its
    // lowest bit repeated below.
    auto to_binary = [](uint32_t (&A)[4], uint32_t (&B)[4], int k) {
      const int kA = k < 8 ? k : 8, kB = k - kA;
#pragma unroll
      for (int w = 0; w < 4; ++w) {
        A[w] = gray_to_binary_bytes(__builtin_bitreverse32(A[w]), kA);
        B[w] = kB > 0 ? gray_to_binary_bytes(__builtin_bitreverse32(B[w]) ^ ((A[w] & 0x01010101u) << (kB - 1)), kB)
                      : 0u;
      }
    };
    const int cBn = kc > 8 ? kc - 8 : 0;
    const int cSh = nc - kc;
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
  }
  // pixel 4 w + e's row code from the binary row words
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
    if (vec && live) {
      // For each quarter j of the chunk (pixels 256 j .. 256 j + 255, the 16
      // lanes of DPP row j), those lanes put their 64 B in the wave's stage,
      // then lane l stores bytes 16 l .. 16 l + 15 of it (pixels 256 j + 4 l
      // ..): 1 KB contiguous per instruction.  A lane writes the stage only
      // where its 16 pixels are in the view (whole 16-pixel groups: W % 16 ==
      // 0), and the chunk's buffer descriptor drops stores past the view's end.
      uint4* const stg = s_mapst + 64 * wid;
      const int64_t cbase = view * HW + static_cast<int64_t>(civ) * kChunk;  // the chunk's first pixel
#pragma unroll
      for (int m = 0; m < 2; ++m) {
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
              for (int e = 0; e < 4; ++e) v4[e] = m == 0 ? col[4 * q + e] : row_code(q, e);
              stg[4 * u + q] = make_uint4(v4[0], v4[1], v4[2], v4[3]);
            }
          }
          __builtin_amdgcn_wave_barrier();
          const uint4 v = stg[lane];
          __builtin_amdgcn_wave_barrier();
          __builtin_amdgcn_raw_buffer_store_b128(v4u{v.x, v.y, v.z, v.w}, rd, 1024 * j + 16 * lane, 0, kMapAux);
        }
      }
    } else if (!vec) {
#pragma unroll
      for (int k = 0; k < kPx; ++k) {
        if (k < n_px) {
          __builtin_nontemporal_store(static_cast<int32_t>(col[k]), p.col_out + o + k);
          __builtin_nontemporal_store(static_cast<int32_t>(row_code(k >> 2, k & 3)), p.row_out + o + k);
        }
      }
    }
  }
  if (decide) {
    if (it == 0) {  // workgroup-uniform: the LDS-DMA tables and s_thr are in
      __syncthreads();
      if (mode & M_HIST) {
        tw2 = __builtin_amdgcn_readfirstlane(s_thr[0]);
        tc2 = __builtin_amdgcn_readfirstlane(s_thr[1]);
      }
    }
    // ---- mask with the view's thresholds ----
    uint32_t ok = 0u, mb[4];
#pragma unroll
    for (int w = 0; w < 4; ++w) ok |= mask4(word(wq, w), word(bq, w), tw2, tc2, &mb[w]) << (4 * w);
    if (n_px != kPx) ok = 0u;  // vec: whole 16-pixel groups
    if (p.masked) {  // (uniform) the chunk's masked pixels into the workgroup's count
      const int mc = wave_sum_dpp(__popc(ok));
      if (lane == 0 && mc) atomicAdd(&s_mcount, static_cast<unsigned>(mc));
    }
    if ((mode & M_MAPS) && n_px == kPx)
      __builtin_nontemporal_store(v4u{mb[0], mb[1], mb[2], mb[3]}, reinterpret_cast<v4u*>(p.mask_out + o));
    // ---- |n.r| > 1e-6 (sl_system.py:638-642) of the masked pixels, LDS tables ----
    uint32_t pt = 0u;
    if ((mode & M_CODES) && ok) {
      const int px0i = static_cast<int>(px0);
      const int v = row_of(p, px0i), u0 = px0i - v * p.W;  // the lane's 16 pixels share row v (W % 16 == 0)
      float4 pf[kPx];
#pragma unroll
      for (int k = 0; k < kPx; ++k) pf[k] = s_pl[min(col[k], static_cast<uint32_t>(p.Wp - 1))];
      float xs[kPx];
#pragma unroll
      for (int q4 = 0; q4 < 4; ++q4) {
        const float4 x4 = reinterpret_cast<const float4*>(s_xn + u0)[q4];
        xs[4 * q4] = x4.x;
        xs[4 * q4 + 1] = x4.y;
        xs[4 * q4 + 2] = x4.z;
        xs[4 * q4 + 3] = x4.w;
      }
      const float ys = ys_early;
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
      const int64_t gci = static_cast<int64_t>(view) * p.cpv + civ;
      pt_rec = pt;  // (the 12-bit records carry the point bits: code 0xfff = no point)
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
            if (t) atomicAdd(sup + (blk >> p.sb_shift), t);
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

  if (mode & M_CODES) {
    // records for k_count / k_cloud: clipped column code
    uint32_t rec[kPx / 2];
#pragma unroll
    for (int i = 0; i < kPx / 2; ++i)
      rec[i] = min(col[2 * i], static_cast<uint32_t>(p.Wp - 1)) |
               (min(col[2 * i + 1], static_cast<uint32_t>(p.Wp - 1)) << 16);
    if (decide) {
      // 12-bit records (M_DECIDE implies the vector path and Wp <= 2048):
      // chunk slots without maps, pixel order with them (the host sets
      // p.rec_blk to match, for k_cloud)
      const bool blk = !(mode & M_MAPS);
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
  if (decide && (mode & M_CODES) && !p.bs_atomic) {  // the workgroup's block sum (k_count's, for k_cloud's offsets)
    if (dyn && tid == 0) s_next[it & 1] = static_cast<int>(dyn_next) + gx;
    __syncthreads();
    if (tid == 0) {
      int t = 0;
#pragma unroll
      for (int w = 0; w < kWaves; ++w) t += s_cnt[it & 1][w];
      const int64_t blk = static_cast<int64_t>(view) * ngroups + cg;
      p.block_sums[blk] = t;
      if (t) atomicAdd(sup + (blk >> p.sb_shift), static_cast<unsigned>(t));
    }
  }
  cg = dyn ? s_next[it & 1] : cg + gx;  // (dyn: published before the block-sum barrier above)
  ++it;
  }  // chunk groups

  if (decide && p.masked) {  // one global add per workgroup (its view: blockIdx.y)
    __syncthreads();
    if (tid == 0 && s_mcount) atomicAdd(p.masked + view, static_cast<unsigned long long>(s_mcount));
  }
  // the last of the view's workgroups to have read its histograms zeroes them
  // (here at the end: wave 0 waiting on the arrival atomic at the start delayed
  // its first stack loads, k_decode +3 us per c2 step; tw2 / tc2 came from them)
  if (decide && (mode & M_HIST) && !p.rerun && wid == 0)
    hist_release(p.hist + static_cast<int64_t>(view) * kHistView, kHistView, blockIdx.x, gx, lane, tw2, tc2);

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
  const bool adaptive = (mode & M_HIST) != 0;
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
    // every wave of the view's workgroups reads the histogram: the last zeroes it
    if (!p.rerun)
      hist_release(p.hist + static_cast<int64_t>(view) * kSlot, kSlot, blockIdx.x * kWaves + (threadIdx.x >> 6),
                   kWaves * gridDim.x, lane, t.white, t.contrast);
  }
  if (!live) return 0;

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
        if (px < HW) __builtin_nontemporal_store(bytes, reinterpret_cast<uint32_t*>(mo_ + px));
      } else {
#pragma unroll
        for (int e = 0; e < 4; ++e)
          if (px + e < HW) __builtin_nontemporal_store(static_cast<uint8_t>((m >> e) & 1u), mo_ + px + e);
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
        pf[e] = p.planes32[c];
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
    if (vec && !nc) {
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
      if (px < HW) __builtin_nontemporal_store(mbytes[s], reinterpret_cast<uint32_t*>(mo_ + px));
    }
  }
  total = wave_sum(total);
  if (lane == 0) p.chunk_counts[gc] = total;
  return total;
}

// k_count: one chunk per wave, grid (chunk groups of 4, views); the
// workgroup's point total goes to block_sums for k_cloud's offsets.
template <int VEC>
__global__ __launch_bounds__(kThreads, 1) void k_count(Params p) {
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
  unsigned* const sup = super_produce(p);
  if (lane == 0) s_sum[wid] = total;
  __syncthreads();
  if (threadIdx.x == 0) {
    int t = 0;
#pragma unroll
    for (int w = 0; w < kWaves; ++w) t += s_sum[w];
    const int64_t blk = static_cast<int64_t>(view) * gridDim.x + blockIdx.x;
    p.block_sums[blk] = t;
    if (t) atomicAdd(sup + (blk >> p.sb_shift), static_cast<unsigned>(t));
  }
}

// ================================================================= k_cloud ====
// reconstruct_point_cloud's arithmetic (sl_system.py:584-653) for the points
// k_decode / k_count marked, one chunk per wave:
//   0. the chunk's offset in the merged cloud: the super-block sums before its
//      super-block + the block sums before it inside it (+ earlier launch
//      groups), + the chunk counts of the workgroup's earlier waves;
//   1. records + colour of the lane's 16 pixels (16-byte loads); the lane's
//      point count and its exclusive prefix over the wave give every point its
//      rank in the chunk (ascending pixel order, np.where, sl_system.py:601);
//   2. each point's (pixel, column code) goes to LDS at its rank -- the
//      chunk's points, compacted -- and the chunk's texture bytes to LDS in
//      pixel order;
//   3. PIPE x 64 points per pass: lane j takes points j, j+64, ...; all their
//      operand gathers (ray tables or Nc, plane) are issued before any point
//      is computed, then the arithmetic, then the stores at offset + rank (64
//      consecutive points per store instruction).
constexpr int kPipe = 4;  // points per lane per pass in the f32-fast k_cloud
constexpr int kBgrWords = 3 * kChunk / 4 + 4;  // u32 per wave: the chunk's BGR bytes in pixel order (+ slack)

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

// Phase 1 of a chunk (global index gc): the lane's loads.
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
  if (vec && p.rec12) {  // 12-bit records (k_decode M_DECIDE): 8 codes per 3 words
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
    if (vec) {
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

// Phase 3 of a chunk: its `total` compacted points (s_ent: pixel | code << 10
// | row offset << 25 on the 16-byte path, s_bgr: the chunk's colours in pixel
// order) -> xyz + BGR at offset base + rank, PIPE x 64 per pass.
template <int MODE, int VEC, int PIPE>
__device__ __forceinline__ void cloud_points(const Params& p, int view, int64_t cpx, long long base, int lane,
                                             int total, const uint32_t* s_ent, const uint32_t* s_bgr) {
  constexpr int kP = PIPE;  // points per lane per pass
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
  auto point_bgr = [&](int local) -> uint32_t {
    if (has_tex) {  // bytes 3 local .. 3 local + 2 of the chunk's BGR
      const int b = 3 * local;
      const uint32_t w0 = s_bgr[b >> 2], w1 = s_bgr[(b >> 2) + 1];
      return __builtin_amdgcn_alignbyte(w1, w0, static_cast<unsigned>(b & 3)) & 0xffffffu;
    }
    return ((s_bgr[local >> 2] >> (8 * (local & 3))) & 0xffu) * 0x010101u;
  };
  float* const wx = static_cast<float*>(p.xyz) + 3 * base;  // the chunk's first point (wave-uniform)
  uint8_t* const wc = p.bgr + 3 * base;
  // The xyz leave with nt stores, like k_decode's maps: nothing in the path
  // reads them back, and default-policy lines would push the records, the
  // texture and the next view's planes out of L2 / the Infinity Cache (c3-c5
  // 3-5 % faster per call, c2 3 %; nt colours gained nothing more:
  // profiles/r05_ab/nt_stores_lines.jsonl).
  // Colours by quads, ahead of the point arithmetic: a lane takes 4
  // consecutive points, whose 12 colour bytes start on a 4-byte boundary
  // (point m of the chunk sits at wc + 3 m: m = (wc mod 4) + 4 k), and puts
  // them out as one dwordx3 -- 768 contiguous bytes per store instruction,
  // the xyz stores' shape, one instruction per 256 points.  The <= 3 points
  // before the first quad and the <= 3 after the last go out byte by byte.
  // (Per point, a short and a byte store per lane had cost 4x the xyz per
  // byte; quads: c2 113.9-114.2 -> 112.3-112.7 us per step, c3 632.9 ->
  // 615.7 us, c4 4.047 -> 3.985 ms, c5 3.183 -> 3.146 ms, two alternating
  // runs on one box, profiles/r05_ab/colour_quad_lines.jsonl.  The
  // register-only form -- 64 points' 192 bytes assembled by lane permutes
  // into 48 dwords -- had been slower: colour_pack_lines.jsonl.)
  {
    const int a = static_cast<int>(reinterpret_cast<uintptr_t>(wc) & 3u);  // wave-uniform
    const int head = min(a, total);
    const int nq = total > a ? (total - a) >> 2 : 0;
    const int t0 = a + 4 * nq;
    int ep = -1;
    if (lane < head) ep = lane;
    else if (lane >= 4 && lane - 4 < total - max(t0, head)) ep = t0 + lane - 4;
    if (ep >= 0) {
      const uint32_t c = point_bgr(static_cast<int>(s_ent[ep] & 1023u));
      uint8_t* cc = at_bytes(wc, 3u * static_cast<unsigned>(ep));
      cc[0] = static_cast<uint8_t>(c);
      cc[1] = static_cast<uint8_t>(c >> 8);
      cc[2] = static_cast<uint8_t>(c >> 16);
    }
    for (int k = lane; k < nq; k += 64) {
      const int m = a + 4 * k;
      const uint32_t c0 = point_bgr(static_cast<int>(s_ent[m] & 1023u));
      const uint32_t c1 = point_bgr(static_cast<int>(s_ent[m + 1] & 1023u));
      const uint32_t c2 = point_bgr(static_cast<int>(s_ent[m + 2] & 1023u));
      const uint32_t c3 = point_bgr(static_cast<int>(s_ent[m + 3] & 1023u));
      uint32_t* q = reinterpret_cast<uint32_t*>(at_bytes(wc, 3u * static_cast<unsigned>(m)));  // 4-byte aligned
      q[0] = c0 | (c1 << 24);
      q[1] = (c1 >> 8) | (c2 << 16);
      q[2] = (c2 >> 16) | (c3 << 8);
    }
  }
  for (int j0 = 0; j0 < total; j0 += 64 * kP) {
    if (mode & M_FAST32) {
      // SL_XYZ_F32_FAST (Oc = 0, pinhole rays, no pose; host-checked): the
      // same formula in f32 -- rsq-normalised ray, f32 plane, rcp -- for
      // points whose condition number kappa = sum|n_i r_i| / |n.r| is at most
      // kFastKappa; the rest take the exact f64 route below.  Per-coordinate
      // relative error vs the reference's f64 <= (11 + 10 kappa) 2^-24
      // ("f32-fast").
      float fx[kP], fy[kP];
      float4 fp[kP];
#pragma unroll
      for (int i = 0; i < kP; ++i) {
        const int j = min(j0 + 64 * i + lane, total - 1);
        const uint32_t e = s_ent[j];
        int uu, vv;
        chunk_uv<VEC>(u_c, v_c, e, W, &uu, &vv);
        fx[i] = *at_bytes(p.xn32, 4u * static_cast<unsigned>(uu));
        fy[i] = *at_bytes(p.yn32, 4u * static_cast<unsigned>(vv));
        fp[i] = p.planes32[ent_code(e)];
      }
#pragma unroll
      for (int i = 0; i < kP; ++i) {
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
        if (j < total) {
          float* xyz = at_bytes(wx, 12u * static_cast<unsigned>(j));
          __builtin_nontemporal_store(X, xyz);
          __builtin_nontemporal_store(Y, xyz + 1);
          __builtin_nontemporal_store(Z, xyz + 2);
        }
      }
      continue;
    }
    double ra[kP], rb[kP], rcz[kP];  // pinhole: x, y, -; Nc: r0, r1, r2
    double4 pl[kP];
#pragma unroll
    for (int i = 0; i < kP; ++i) {
      const int j = min(j0 + 64 * i + lane, total - 1);  // past the end: repeat the last point
      const uint32_t e = s_ent[j];
      const int local = static_cast<int>(e & 1023u);
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
        } else if (p.xy_calc) {  // (uniform) the table values, computed: no 16 B of gathers per point
          ra[i] = xy_of(uu, p.cx, p.fx);  // (gathering x or y instead: +0.8 / +1.1 us at c2)
          rb[i] = xy_of(vv, p.cy, p.fy);
        } else {
          ra[i] = p.xn[uu];
          rb[i] = p.yn[vv];
        }
      }
      pl[i] = p.planes[ent_code(e)];
    }
    double X[kP], Y[kP], Z[kP];
    uint32_t slow = 0u;
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
      for (int i = 0; i < kP; ++i) {
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
          // 2^-44 M_k <= 2^-44 (R_k max_j |P_j| + |m_k3|) (R_k = sum_j |m_kj|,
          // per view, the scale folded into pb / pt: exact): a wider interval,
          // so as safe, at 4 operations instead of 18 (the slack of 2^-44
          // against the 2^-45.2 the bound needs covers these few roundings)
          const double pmax = fmax(fmax(fabs(x0), fabs(x1)), fabs(x2));
          const double M0 = fma(pb[0], pmax, pt[0]);
          const double M1 = fma(pb[1], pmax, pt[1]);
          const double M2 = fma(pb[2], pmax, pt[2]);
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
    // The kP points' chains (sqrt, shared reciprocal, divisions) carry no
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
      // stage by stage over the kP points (the source order the scheduler
      // keeps): independent instructions of different points sit side by side
      double r0[kP], r1[kP], r2[kP];
      if (mode & M_NC) {
#pragma unroll
        for (int i = 0; i < kP; ++i) {
          r0[i] = ra[i];
          r1[i] = rb[i];
          r2[i] = rcz[i];
        }
      } else {
        double nrm[kP], rn[kP];
#pragma unroll
        for (int i = 0; i < kP; ++i) {
          const double x = ra[i], y = rb[i];
          nrm[i] = sqrt_nr((x * x + y * y) + 1.0);  // s2 in [1, 2^601] when div_safe(x), div_safe(y)
          if (!(p.xy_safe || (div_safe(x) && div_safe(y)))) slow |= 1u << i;
        }
        // the three divisions by nrm share one reciprocal (div_rn: the
        // compiler's own f64 division sequence, bit for bit, where it would
        // not rescale)
#pragma unroll
        for (int i = 0; i < kP; ++i) rn[i] = recip_nr(nrm[i]);
#pragma unroll
        for (int i = 0; i < kP; ++i) {
          r0[i] = div_rn(ra[i], nrm[i], rn[i]);
          r1[i] = div_rn(rb[i], nrm[i], rn[i]);
          r2[i] = div_rn(1.0, nrm[i], rn[i]);
        }
      }
      double den[kP], t[kP];
#pragma unroll
      for (int i = 0; i < kP; ++i) den[i] = (pl[i].x * r0[i] + pl[i].y * r1[i]) + pl[i].z * r2[i];
#pragma unroll
      for (int i = 0; i < kP; ++i) {
        t[i] = div_rn(-pl[i].w, den[i], recip_nr(den[i]));
        if (!(div_safe(pl[i].w) && div_safe(den[i]))) slow |= 1u << i;
      }
#pragma unroll
      for (int i = 0; i < kP; ++i) {
        X[i] = p.o0 + r0[i] * t[i];
        Y[i] = p.o1 + r1[i] * t[i];
        Z[i] = p.o2 + r2[i] * t[i];
      }
      fallback = slow;
    }  // !M_VERIFY
    if (fallback) {  // rare: the operators' own sequences (rescaling, +-0, inf / NaN; unsettled M_VERIFY points)
#pragma unroll
      for (int i = 0; i < kP; ++i) {
        if (!((fallback >> i) & 1u)) continue;
        // the point's operands again (M_VERIFY: re-read, so that nothing of
        // the verified route stays live across this block)
        double xa = ra[i], xb = rb[i], xc = rcz[i];
        double4 pp = pl[i];
        if (mode & M_VERIFY) {
          const uint32_t e = s_ent[min(j0 + 64 * i + lane, total - 1)];
          int uu, vv;
          chunk_uv<VEC>(u_c, v_c, e, W, &uu, &vv);
          xa = p.xn[uu];
          xb = p.yn[vv];
          pp = p.planes[ent_code(e)];
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
    if (pose && !(mode & M_VERIFY)) {
#pragma unroll
      for (int i = 0; i < kP; ++i) {
        const double X2 = ((pm[0] * X[i] + pm[1] * Y[i]) + pm[2] * Z[i]) + pm[3];
        const double Y2 = ((pm[4] * X[i] + pm[5] * Y[i]) + pm[6] * Z[i]) + pm[7];
        const double Z2 = ((pm[8] * X[i] + pm[9] * Y[i]) + pm[10] * Z[i]) + pm[11];
        X[i] = X2;
        Y[i] = Y2;
        Z[i] = Z2;
      }
    }
#pragma unroll
    for (int i = 0; i < kP; ++i) {
      const int j = j0 + 64 * i + lane;
      if (j < total) {
        const unsigned o = static_cast<unsigned>(j);  // offset from the chunk's first point
        if (f64out) {
          double* xyz = static_cast<double*>(p.xyz) + 3 * base + 3 * o;
          __builtin_nontemporal_store(X[i], xyz);
          __builtin_nontemporal_store(Y[i], xyz + 1);
          __builtin_nontemporal_store(Z[i], xyz + 2);
        } else {
          float* xyz = at_bytes(wx, 12u * o);
          __builtin_nontemporal_store(static_cast<float>(X[i]), xyz);
          __builtin_nontemporal_store(static_cast<float>(Y[i]), xyz + 1);
          __builtin_nontemporal_store(static_cast<float>(Z[i]), xyz + 2);
        }
      }
    }
  }
}

// Phases 2-3 of a chunk (global index gc, output offset base), by one wave,
// from the lane's loads.
template <int MODE, int VEC, int PIPE>
__device__ __forceinline__ void cloud_chunk(const Params& p, int64_t gc, long long base, int lane, const ChunkIn& in,
                                            uint32_t* s_ent, uint32_t* s_bgr) {
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
  const int total = __builtin_amdgcn_readlane(incl, 63);
  if (lane == 0 && civ == 0) p.view_offsets[view] = base;
  // offsets past the caller's capacity (a caller's buffer smaller than its
  // declared capacity cannot be detected; this guards the declared one):
  // write nothing (the call's total then exceeds the capacity, which the host
  // reports)
  if (base < 0 || base + total > p.out_cap) return;

  // ---- 2. compacted entries in LDS, the chunk's colours in pixel order ----
  {
    uint4* t4 = reinterpret_cast<uint4*>(s_bgr);
    if (has_tex) {
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
      if ((ptbits >> k) & 1u) s_ent[idx] = static_cast<uint32_t>(lane * kPx + k) | (code << 10) | drow;
      idx += (ptbits >> k) & 1u;
    }
  }
  __builtin_amdgcn_wave_barrier();
  cloud_points<MODE, VEC, PIPE>(p, view, cpx, base, lane, total, s_ent, s_bgr);
}

// k_cloud: one chunk per wave, grid (triangulating workgroups per view +
// pre-stats workgroups, views).  The workgroup's output offset is the sum of
// the block sums before it (+ the earlier launch groups of the call); each
// wave adds the counts of the chunks before it in the workgroup.
constexpr int kPrefixBatch = 4;

// Points of the blocks before block b of the launch group (one workgroup;
// holds a workgroup barrier): the super-block sums before b's super-block,
// then the block sums before b inside it (both <= ~sqrt(blocks) entries; all
// loads of a batch in flight together).  Every wave's loads have returned
// when it returns (their sums crossed the barrier).
__device__ __forceinline__ long long block_offset(const Params& p, const unsigned* sup, int64_t b, int tid, int lane,
                                                  int wid, long long* s_wred) {
  long long acc = 0;
  const int64_t sb = b >> p.sb_shift;
  for (int64_t t0 = 0; t0 < sb; t0 += kPrefixBatch * kThreads) {
    unsigned v[kPrefixBatch];
#pragma unroll
    for (int i = 0; i < kPrefixBatch; ++i) v[i] = sup[min<int64_t>(t0 + i * kThreads + tid, sb - 1)];
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

// PIPE: points per lane per pass (the f64 chains: 2; f32-fast: kPipe)
constexpr int kExactPipe = 2;   // points per lane per pass of the exact (f64) k_cloud<M_TEX>
constexpr int kVerifyPipe = 2;  // ... of the verified-route k_cloud<M_VERIFY | M_TEX>
static_assert(kWaves * kChunk >= 256 * kHistStride,
              "k_cloud's pre-stats workgroups keep their LDS histogram replicas in s_ent");
template <int MODE, int VEC, int PIPE>
__global__ __launch_bounds__(kThreads, 5) void k_cloud(Params p) {
  __shared__ uint32_t s_ent[kWaves][kChunk];  // compacted points: pixel | code << 10
  __shared__ __attribute__((aligned(16))) uint32_t s_bgr[kWaves][kBgrWords];  // the chunks' colours
  __shared__ long long s_wred[kWaves];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform, provably
  const int view = blockIdx.y;
  // pre-stats (sl_stack_next): the first gridDim.x - cloud_gx workgroups of
  // each row compute the next call's (or launch group's) histograms; the
  // triangulating ones follow.  (Ahead of them, the pass runs beside the
  // first triangulating workgroups, and the launch ends with the
  // triangulation's own tail: c5 -1.1 %, c2 / c3 -0.2-0.3 % against the pass
  // after them, two alternating runs, profiles/r05_ab/pre_stats_front_lines.jsonl)
  const int npre = static_cast<int>(gridDim.x) - p.cloud_gx;
  if (static_cast<int>(blockIdx.x) < npre) {
    pre_stats_block(p, blockIdx.x, npre, &s_ent[0][0], reinterpret_cast<int*>(s_wred));
    return;
  }
  const int cx = static_cast<int>(blockIdx.x) - npre;  // triangulating workgroup index in the view
  const int civ = cx * kWaves + wid;
  const int64_t b = static_cast<int64_t>(view) * p.cloud_gx + cx;  // block index in the launch
  const int64_t gc = static_cast<int64_t>(view) * p.cpv + civ;
  const int before = (lane < wid && civ < p.cpv) ? p.chunk_counts[gc - wid + lane] : 0;  // earlier waves' chunks
  long long base = block_offset(p, super_consume(p, cx), b, tid, lane, wid, s_wred);
  base += p.base_in ? *p.base_in : 0ll;
  base += wave_sum(before);
  base = uniform64(base);
  if (civ >= p.cpv) return;
  ChunkIn in;
  cloud_load<VEC>(p, gc, lane, &in);
  if (lane == 0 && view == p.n_views - 1 && civ == p.cpv - 1)
    p.view_offsets[p.n_views] = base + p.chunk_counts[gc];
  cloud_chunk<MODE, VEC, PIPE>(p, gc, base, lane, in, &s_ent[wid][0], &s_bgr[wid][0]);
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
  float* d_f32 = nullptr;  // planes32 [Wp][4] | xn32 [W] | yn32 [H]
  float fast_thr = 0.0f;   // k_count's sufficient |n.r| threshold (Params::fast_thr)
  bool xy_safe = false;     // every xn / yn table entry is div_safe (Params::xy_safe)
  bool xy_calc = false;     // xy_of reproduces every xn / yn entry (k_xy_check)
  bool xy_plain = false;    // every xn / yn entry has 2^-20 <= |v| <= 2^20 (the verified route's range premise)
  bool planes_plain = false;  // every plane has |w| >= 2^-500 and max|n_i| >= 2^-400 (ditto)
  double cam[4] = {0, 0, 1, 1};  // cx, cy, fx, fy
  bool verify32 = true;     // SL_XYZ_F32 by the verified shorter route (SLGPU_VERIFY32=0: the exact sequence,
                            // a test switch: tests/test_gpu_parity.py compares the two)
  double* d_nc = nullptr;
  // scratch
  ViewStats* d_stats = nullptr;
  int64_t cap_stats = 0;
  // the adaptive mask's histograms: k_stats / pre-stats [view][kHistView], or
  // k_decode's (3-kernel path) [view][kSlot]; zeroed by their consumer.  Two
  // buffers: [0] for eager calls, [1] for calls captured into graphs -- a
  // graph replays without the host, so eager calls never share its buffer
  unsigned* d_hist[2] = {nullptr, nullptr};
  int64_t cap_hist = 0;
  int64_t hist_dirty[2] = {0, 0};  // leading words that may be non-zero (a queued pass, a failure)
  unsigned long long cap_domain = 0;  // the capture whose calls the host tracked last in d_hist[1]
  int* d_chunk_counts = nullptr;
  int64_t cap_cc = 0;
  int* d_block_sums = nullptr;
  int64_t cap_bs = 0;
  unsigned* d_super = nullptr;  // two super-block buffers (sums + dynamic-grid counters) + their selectors
  bool super_dirty = false;     // a call stopped between k_decode / k_count and k_cloud: zeroed before the next
  uint8_t* d_ptnib = nullptr;
  int64_t cap_ptnib = 0;
  uint16_t* d_codes = nullptr;  // k_decode -> k_count / k_cloud records
  int64_t cap_codes = 0;
  int last_views = 0;
  int decode_wgs = 0;  // k_decode grid cap in workgroups over all views
  int pre_wgs = 0;     // pre-stats workgroups of a pass (2 per CU)
  // optional per-call HIP-event timing of k_decode / k_count / k_cloud
  std::vector<hipEvent_t> prof_ev;  // kProfEv events per call slot
  std::vector<int> prof_groups;     // launch groups recorded per call
  std::vector<char> prof_decide;    // per call: M_DECIDE path (events around k_stats, k_decode, k_cloud)
  int n_cu = 0;
  int prof_n = 0;
  // RCCL gather (sl_gather_init): communicator, this rank, count scratch
  void* comm = nullptr;
  int nranks = 0, rank = 0;
  int64_t* d_gcounts = nullptr;
  // sl_write_ply_device: per-workgroup line bytes and offsets, the text, and
  // the pinned host buffer it comes back through (grown, kept)
  unsigned* d_ply_bsum = nullptr;
  int64_t cap_ply_bsum = 0;
  int64_t* d_ply_boff = nullptr;
  int64_t cap_ply_boff = 0;
  char* d_ply_text = nullptr;
  int64_t cap_ply_text = 0;
  char* h_ply_text = nullptr;
  int64_t cap_h_ply_text = 0;
  int64_t cap_gcounts = 0;
  // the last call's stream: a call on another stream first waits for the work
  // queued there (the scratch above is per context)
  hipStream_t last_stream = nullptr;
  hipEvent_t done_ev = nullptr;
  bool done_valid = false;
  int64_t last_launches = 0, last_launch_px = 0;  // sl_last_launch_info
  int64_t* mc_next = nullptr;  // sl_mask_counts_to: the next sl_decode_triangulate's masked-pixel counts
  bool ready_next = false;     // sl_stack_ready: armed for the next sl_decode_triangulate
  hipEvent_t ready_ev_next = nullptr;
  // Pre-stats (sl_stack_next): a call's last k_cloud also runs the histogram
  // pass of the NEXT call's first launch group (declared stack) into d_hist,
  // so that call starts with its k_decode.
  bool decl_next = false;             // sl_stack_next armed for the coming call
  const uint8_t* decl_stack = nullptr;
  int64_t decl_vs = 0;
  int decl_views = 0;
  bool pre_armed = false;             // a pass was queued for the next call: of this stack, stride, views, frame
  const uint8_t* pre_stack = nullptr;
  int64_t pre_vs = 0, pre_hw = 0;
  int pre_views = 0;
  unsigned long long pre_capture = 0;  // ... queued inside this stream capture (capture id + 1; 0: eagerly)
  // the last launch group's kernels and arguments (sl_time_kernels)
  struct {
    bool valid = false;
    bool decide = false;  // fn[1] = k_stats (or null) instead of k_count
    bool stats = false;   // decide, adaptive: p[1] / grid[1] are k_stats' (to rebuild the histograms)
    Params p[3];
    const void* fn[3] = {nullptr, nullptr, nullptr};  // k_decode, k_count / k_stats (or null), k_cloud (or null)
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

int zero_async(sl_ctx* c, void* p, int64_t words, hipStream_t s);

// *ptr grown to at least `need` elements (at least twice the old capacity),
// zeroed: on stream s when on_stream -- a kernel ordered before the work the
// caller enqueues there next -- else before returning.  (A bare hipMemset
// runs on the null stream, which non-blocking streams -- torch's pool
// streams, ReconstructorPool's lanes -- do not wait for: a call's first
// kernels could overtake the zeroing of the scratch they accumulate into.
// Seen as a wrong adaptive mask on a lane once the lanes had hardware queues
// of their own, tests/test_gpu_pool.py.)
template <typename T>
int grow(sl_ctx* c, T** ptr, int64_t* cap, int64_t need, hipStream_t s = nullptr, bool on_stream = false) {
  if (need <= *cap) return SL_OK;
  if (*ptr) HIP_TRY(c, hipFree(*ptr));
  *ptr = nullptr;
  const int64_t n = std::max<int64_t>(need, *cap * 2);
  const int64_t words = (static_cast<int64_t>(sizeof(T)) * n + 3) / 4;
  HIP_TRY(c, hipMalloc(reinterpret_cast<void**>(ptr), 4 * words));
  if (on_stream) {
    const int r = zero_async(c, *ptr, words, s);
    if (r) return r;
  } else {
    HIP_TRY(c, hipMemset(*ptr, 0, 4 * words));
    HIP_TRY(c, hipDeviceSynchronize());
  }
  *cap = n;
  return SL_OK;
}

// scratch for `views` views of `px` pixels each (histograms: for
// max(views, hist_views)); *hist_fresh: the histogram buffer was
// (re)allocated (zeroed: a pass queued in it is gone)
int ensure_scratch(sl_ctx* c, int64_t views, int64_t px, bool codes, int64_t hist_views = 0,
                   bool* hist_fresh = nullptr, hipStream_t s = nullptr, bool on_stream = false) {
  const int64_t chunks = views * ((px + kChunk - 1) / kChunk);
  int r = grow(c, &c->d_chunk_counts, &c->cap_cc, chunks, s, on_stream);
  if (r) return r;
  r = grow(c, &c->d_block_sums, &c->cap_bs, views * (((px + kChunk - 1) / kChunk + kWaves - 1) / kWaves), s,
           on_stream);
  if (r) return r;
  r = grow(c, &c->d_ptnib, &c->cap_ptnib, chunks * kChunkNib, s, on_stream);
  if (r) return r;
  int64_t scap = c->d_super ? kSuperWords : 0;
  r = grow(c, &c->d_super, &scap, kSuperWords, s, on_stream);  // zeroed once; then by the kernels (super_produce)
  if (r) return r;
  const int64_t before = c->cap_hist, need = std::max(views, hist_views) * kHistView;
  for (int d = 0; d < 2; ++d) {  // k_stats' replicas (k_decode's: kSlot)
    int64_t cap = before;
    r = grow(c, &c->d_hist[d], &cap, need, s, on_stream);
    if (r) return r;
    if (d == 1) c->cap_hist = cap;
  }
  if (c->cap_hist != before) {
    c->hist_dirty[0] = c->hist_dirty[1] = 0;
    c->pre_armed = false;
    if (hist_fresh) *hist_fresh = true;
  }
  // (u16 units: 2 B/px, or the 1536-B slots of whole chunk groups)
  if (codes)
    return grow(c, &c->d_codes, &c->cap_codes,
                std::max<int64_t>(views * px, views * ((px + 4 * kChunk - 1) / (4 * kChunk)) * 4 * (kRecSlot / 2)) + 16,
                s, on_stream);
  return SL_OK;
}

using KernelFn = void (*)(Params);
constexpr int kProfGroups = 64;            // launch groups timed per call (at most)
constexpr int kProfEv = 4 * kProfGroups;   // events per call: per group before k_decode, k_count, k_cloud, after
                                           // (M_DECIDE: before k_stats, k_decode, k_cloud, after)

// k_decode specialisations for the benchmark configurations (the decide
// path); everything else (other bit counts, the 3-kernel path of unaligned or
// very large frames) runs the generic instantiation.
KernelFn pick_decode(int kc, int kr, int mode, bool vec) {
  if (vec && !(mode & (M_NC | M_FROMMAPS))) {
    constexpr int mrch = M_MAPS | M_ROWS | M_CODES | M_HIST, mrh = M_MAPS | M_ROWS | M_HIST,
                  ch = M_CODES | M_HIST, mrc = M_MAPS | M_ROWS | M_CODES, cc = M_CODES;
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

KernelFn pick_cloud(int mode, bool vec) {
  if (vec && mode == M_TEX) return k_cloud<M_TEX, 1, kExactPipe>;  // f32 xyz, pinhole rays, BGR texture
  if (vec && mode == (M_VERIFY | M_TEX)) return k_cloud<M_VERIFY | M_TEX, 1, kVerifyPipe>;  // ... verified route
  if (vec && mode == (M_FAST32 | M_TEX)) return k_cloud<M_FAST32 | M_TEX, 1, kPipe>;
  return vec ? k_cloud<-1, 1, kExactPipe> : k_cloud<-1, 0, kExactPipe>;  // (f64 chains: kExactPipe points per pass)
}

bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

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

// Zero n words at p on stream s.  A kernel, not hipMemsetAsync: inside a
// torch process this library runs on torch's bundled HIP runtime (7.0.51831,
// loaded first under the soname libamdhip64.so.7), whose captured memset
// nodes fill their buffer, from a graph's third launch on, with the low 32
// bits of another node's pointer argument instead of their value
// (scripts/dbg/graph_memset_torch.py: every word = low half of the next
// kernel's output address; profiles/r06_memset/).  The same
// graphs on ROCm 7.2's runtime replay clean (scripts/dbg/graph_memset.hip).
// Round 5 saw exactly that in the adaptive mask's max word (thresholds 0 /
// -7.4e8).  Kernel nodes are not affected.
__global__ __launch_bounds__(256) void k_zero(unsigned* p, int64_t n) {
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n; i += 256ll * gridDim.x) p[i] = 0u;
}
int zero_async(sl_ctx* c, void* p, int64_t words, hipStream_t s) {
  if (words <= 0) return SL_OK;
  const unsigned blocks = static_cast<unsigned>(std::min<int64_t>((words + 255) / 256, 1024));
  hipLaunchKernelGGL(k_zero, dim3(blocks), dim3(256), 0, s, static_cast<unsigned*>(p), words);
  HIP_TRY(c, hipGetLastError());
  return SL_OK;
}
// The stream capture `s` is in: its id + 1, or 0 when it is not capturing.
int capture_of(sl_ctx* c, hipStream_t s, unsigned long long* out) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  HIP_TRY(c, hipStreamGetCaptureInfo(s, &st, &id));
  *out = st == hipStreamCaptureStatusActive ? id + 1 : 0;
  return SL_OK;
}

// Enqueue, per launch group of views, k_decode -> k_count [-> k_cloud] on
// stream s -- or, when decode_mode has M_DECIDE, [k_stats ->] k_decode
// [-> k_cloud] (k_decode applies the mask and makes the point decision).
// decode_mode / count_mode / cloud_mode (< 0: no cloud) are the kernels' mode
// bits.  Launch groups hold at most kMaxChunks chunks (at least one view); a
// group's points follow the earlier groups' (base_in).
//
// Scratch at every launch-group boundary: the super-block buffer the next
// producer accumulates into is zeroed by that producer itself (super_produce:
// the two buffers alternate on the device, k_cloud only flips the selector),
// and the histogram buffer is zero (k_decode / k_count zero what they read)
// except that it may hold one queued pre-stats pass for the next group or
// call.  A call takes a queued pass only when it is of its first group's
// stack, stride, views and frame AND was queued in the same stream capture
// (or both eagerly): a captured graph never depends on a pass queued outside
// it, so it replays in any phase, any number of times.  A pass not taken is
// cleared (k_zero on the stream) before the buffer is used again; so is
// anything a failed call left behind.
int launch_groups(sl_ctx* c, const Params& p0, bool vec, int decode_mode, int count_mode, int cloud_mode,
                  hipStream_t s, PreArms arms) {
  const bool decide = (decode_mode & M_DECIDE) != 0;
  const bool codes = (decode_mode & M_CODES) != 0;
  const int64_t cpv = p0.cpv;
  const int vpg = static_cast<int>(std::max<int64_t>(1, kMaxChunks / cpv));  // views per group
  const int n_groups = static_cast<int>((p0.n_views + vpg - 1) / vpg);
  const bool adaptive = (decode_mode & M_HIST) != 0;
  const bool pre_run = arms.decl && cloud_mode >= 0 && vec;
  bool hist_fresh = false;
  int r = ensure_scratch(c, std::min(vpg, p0.n_views), p0.HW, codes, pre_run ? std::min(vpg, c->decl_views) : 0,
                         &hist_fresh, s, true);
  if (r) return r;
  r = grow(c, &c->d_stats, &c->cap_stats, p0.n_views, s, true);
  if (r) return r;
  unsigned long long cap_id = 0;
  r = capture_of(c, s, &cap_id);
  if (r) return r;
  // Pre-stats (sl_stack_next): this call's first group takes the histograms
  // the previous call's k_cloud computed for it, and this call's last k_cloud
  // computes those of the call declared next.
  const int nv0 = std::min(vpg, p0.n_views);
  const bool pre_use = arms.armed && !hist_fresh && decide && adaptive && p0.stack == c->pre_stack &&
                       p0.stack_vs == c->pre_vs && nv0 == c->pre_views && p0.HW == c->pre_hw &&
                       c->pre_capture == cap_id;
  // Within a call of several launch groups: group g's k_cloud also runs group
  // g + 1's histogram pass (the same pre-stats workgroups), so only the first
  // group can need a k_stats launch.
  const bool pre_groups = decide && adaptive && n_groups > 1 && cloud_mode >= 0 && vec;
  // eager calls and captured calls keep their histograms apart: a graph's
  // replays change its buffer without the host, so the first call of every
  // capture takes that buffer as dirty (later calls of the capture follow it)
  const int dom = cap_id ? 1 : 0;
  unsigned* const hbuf = c->d_hist[dom];
  int64_t& hist_dirty = c->hist_dirty[dom];
  if (dom == 1 && c->cap_domain != cap_id) {
    c->cap_domain = cap_id;
    hist_dirty = c->cap_hist;
  }
  // what the stream's scratch may still hold: clear it before anything reads or accumulates
  if (c->super_dirty) {
    r = zero_async(c, c->d_super, kSuperWords, s);
    if (r) return r;
  }
  c->super_dirty = false;
  if (!pre_use && hist_dirty > 0) {
    r = zero_async(c, hbuf, hist_dirty, s);
    if (r) return r;
  }
  if (!pre_use) hist_dirty = 0;
  // pre-stats workgroups per view of a pass over nv views: 2 per CU in all,
  // k_stats' size (4 steps of 16 pixels per thread at config 2).  Round 3,
  // with the pass after the triangulating workgroups, 8 per CU had been
  // 0.5-1 us faster per c2 step; ahead of them, 2 per CU is: c2 111.7 / 111.3
  // -> 110.7 / 110.1 us, c5 3.211 / 3.212 -> 3.190 / 3.190 ms (4 per CU in
  // between), profiles/r05_ab/pre_stats_size_front_lines.jsonl
  auto pre_bpv_of = [&](int nv) -> int64_t {
    const int64_t per_view = (p0.HW / 16 + kThreads - 1) / kThreads;
    return std::max<int64_t>(1, std::min<int64_t>(per_view, (c->pre_wgs + nv - 1) / nv));
  };
  c->last_views = p0.n_views;
  if (p0.masked) {  // the caller's per-view counts, accumulated by the groups' k_decode / k_count
    r = zero_async(c, p0.masked, 2 * static_cast<int64_t>(p0.n_views), s);
    if (r) return r;
  }
  hipEvent_t* ev = nullptr;
  if (!c->prof_ev.empty() && kProfEv * (c->prof_n + 1) <= static_cast<int>(c->prof_ev.size()))
    ev = &c->prof_ev[kProfEv * c->prof_n++];
  // The pre-stats workgroups' arguments on launch parameters pc of a grid
  // with nv rows, for the pnv views of stack pst (view stride pvs): the launch
  // grows by as many workgroups per row as they need (ahead of its own); the
  // pass accumulates into the (clean) histogram buffer.
  auto add_pre = [&](Params& pc, dim3& grid, int nv, const uint8_t* pst, int64_t pvs, int pnv) {
    const int64_t bpv = pre_bpv_of(pnv);
    pc.pre_stack = pst;
    pc.pre_vs = pvs;
    pc.pre_hist = hbuf;
    pc.pre_views = pnv;
    pc.pre_bpv = static_cast<int>(bpv);
    const int64_t total = static_cast<int64_t>(pnv) * bpv;
    grid.x += static_cast<unsigned>((total + nv - 1) / nv);
    hist_dirty = static_cast<int64_t>(pnv) * kHistView;
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
    // the decide path's records are 12 bits (Wp <= kDecPl): chunk slots for
    // cloud-only calls, pixel order with maps (k_decode's `blk`)
    p.rec12 = (decide && cloud_mode >= 0) ? 1 : 0;
    p.rec_blk = (p.rec12 && !(decode_mode & M_MAPS)) ? 1 : 0;
    p.ptnib = c->d_ptnib;
    p.chunk_counts = c->d_chunk_counts;
    p.block_sums = c->d_block_sums;
    p.hist = hbuf;
    p.super_base = c->d_super;
    p.super_par = c->d_super + 2 * kSuperCap;
    const bool pre_g = next_pre;  // histograms computed by the previous k_cloud (this call's or the last call's)
    next_pre = false;
    const dim3 grid(static_cast<unsigned>((cpv + kWaves - 1) / kWaves), static_cast<unsigned>(nv));
    {  // super-block size: the smallest power of two >= sqrt(blocks of the group)
      const int64_t nb = static_cast<int64_t>(grid.x) * nv;
      int sh = 0;
      while ((int64_t{1} << (2 * sh)) < nb) ++sh;
      p.sb_shift = sh;
    }
    c->last.valid = true;
    dim3 dgrid = grid;  // k_decode: chunk groups strided over a capped grid
    if (c->decode_wgs > 0) dgrid.x = std::min(grid.x, static_cast<unsigned>(std::max(1, (c->decode_wgs + nv - 1) / nv)));
    c->last.grid[0] = dgrid;
    // barrier-free block sums when every k_decode workgroup iterates at most
    // kBsSlots chunk groups (4 chunks of at most 1024 points: 16-bit sums)
    p.bs_atomic = decide && (grid.x + dgrid.x - 1) / dgrid.x <= static_cast<unsigned>(kBsSlots);
    // cloud-only calls: a capped decode grid pulls its chunk groups after the
    // first round from per-view counters (the last entries of the super-block
    // buffer); block sums then take the barrier path, whose barrier publishes
    // each workgroup's next group.  (On maps calls measured slower: c2 119.4
    // -> 122.0-122.6 us)
    p.decode_dyn = (!(decode_mode & M_MAPS) && decide && codes && dgrid.x < grid.x &&
                    ((static_cast<int64_t>(grid.x) * nv) >> p.sb_shift) + 1 + nv < kSuperCap) ? 1 : 0;
    if (p.decode_dyn) p.bs_atomic = 0;
    c->last.grid[1] = c->last.grid[2] = grid;
    c->last.s = s;
    c->last.fn[1] = c->last.fn[2] = nullptr;
    c->last.decide = decide;
    c->last.stats = false;
    if (decide) {
      if (adaptive) {  // k_stats' launch (or what would rebuild the histograms for sl_time_kernels)
        const int64_t per_view = (p0.HW / 16 + kThreads - 1) / kThreads;
        const dim3 sg(static_cast<unsigned>(std::max<int64_t>(1, std::min<int64_t>(per_view, (2 * c->n_cu + nv - 1) / nv))),
                      static_cast<unsigned>(nv));
        p.mode = decode_mode;
        c->last.p[1] = p;
        c->last.grid[1] = sg;
        c->last.stats = true;
        if (!pre_g) {  // k_stats: the thresholds' histograms, before the decode applies them
          void* args[] = {&p};
          const void* kst = reinterpret_cast<const void*>(k_stats);
          c->last.fn[1] = kst;
          HIP_TRY(c, hipLaunchKernel(kst, sg, dim3(kThreads), args, 0, s));
        }
      }
      if (gev) HIP_TRY(c, hipEventRecord(gev[1], s));
    }
    if (codes) c->super_dirty = true;  // until this group's k_cloud is enqueued
    {
      p.mode = decode_mode;
      KernelFn fn = pick_decode(p.kc, (decode_mode & M_ROWS) ? p.kr : 0, decode_mode, vec);
      c->last.p[0] = p;
      c->last.p[0].masked = nullptr;  // sl_time_kernels' re-runs leave the caller's counts alone
      c->last.fn[0] = reinterpret_cast<const void*>(fn);
      void* args[] = {&p};
      HIP_TRY(c, hipLaunchKernel(reinterpret_cast<const void*>(fn), dgrid, dim3(kThreads), args, 0, s));
      // 3-kernel path, adaptive: k_decode accumulates the histograms k_count consumes
      hist_dirty = (adaptive && !decide) ? static_cast<int64_t>(nv) * kSlot : 0;
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
      hist_dirty = 0;
    }
    if (gev && !decide) HIP_TRY(c, hipEventRecord(gev[2], s));
    if (cloud_mode >= 0) {
      p.mode = cloud_mode;
      p.cloud_gx = static_cast<int>(grid.x);
      KernelFn fn = pick_cloud(cloud_mode, vec);
      c->last.p[2] = p;  // (sl_time_kernels re-runs it without the pre-stats workgroups)
      c->last.fn[2] = reinterpret_cast<const void*>(fn);
      Params pc = p;
      dim3 cgrid = grid;
      const bool last_g = g == n_groups - 1;
      const bool pre_now = pre_run && last_g;
      const bool pre_grp = pre_groups && !last_g;
      if (pre_now)  // + the declared next call's histogram pass, after this group's triangulating workgroups
        add_pre(pc, cgrid, nv, c->decl_stack, c->decl_vs, std::min(vpg, c->decl_views));
      else if (pre_grp)  // + this call's next launch group's
        add_pre(pc, cgrid, nv, p0.stack + static_cast<int64_t>(v0 + vpg) * p0.stack_vs, p0.stack_vs,
                std::min(vpg, p0.n_views - v0 - vpg));
      void* args[] = {&pc};
      HIP_TRY(c, hipLaunchKernel(reinterpret_cast<const void*>(fn), cgrid, dim3(kThreads), args, 0, s));
      c->super_dirty = false;
      if (pre_now) {
        c->pre_armed = true;
        c->pre_stack = c->decl_stack;
        c->pre_vs = c->decl_vs;
        c->pre_views = std::min(vpg, c->decl_views);
        c->pre_hw = p0.HW;
        c->pre_capture = cap_id;
      }
      next_pre = pre_grp;
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

// launch_groups, and what a failure in it leaves: scratch that may be dirty
// (cleared before the next call uses it) and no queued pass.
int launch(sl_ctx* c, const Params& p0, bool vec, int decode_mode, int count_mode, int cloud_mode, hipStream_t s,
           PreArms arms) {
  const int r = launch_groups(c, p0, vec, decode_mode, count_mode, cloud_mode, s, arms);
  if (r) {
    c->hist_dirty[0] = c->hist_dirty[1] = c->cap_hist;
    c->super_dirty = c->d_super != nullptr;
    c->pre_armed = false;
  }
  return r;
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
// as Python prints them).  The digit code is shared by the host formatter and
// the device one (k_ply_*, sl_write_ply_device): one source, the same bytes.
namespace {

// finite and |x| < 9e11: the exact integer path applies (else libc, host only)
__host__ __device__ inline bool fmt4_exact(double x) {
  return __builtin_isfinite(x) && __builtin_fabs(x) < 9.0e11;
}

// round(|x| * 10^4), ties to even, exactly (fmt4_exact(x) holds); *neg: the sign bit
__host__ __device__ inline uint64_t fmt4_scaled(double x, bool* neg) {
  const uint64_t bits = static_cast<uint64_t>(__builtin_bit_cast(int64_t, x));
  *neg = bits >> 63;
  const int be = static_cast<int>((bits >> 52) & 0x7ff);
  const uint64_t frac = bits & ((1ull << 52) - 1);
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
  return N;
}

// the length of fmt4_digits' text for x
__host__ __device__ inline int fmt4_len(double x) {
  bool neg;
  uint64_t ip = fmt4_scaled(x, &neg) / 10000u;
  int d = 1;
  while (ip >= 10u) {
    ip /= 10u;
    ++d;
  }
  return (neg ? 1 : 0) + d + 5;
}

// x with 4 decimals, correctly rounded (fmt4_exact(x) holds); -> end of text
__host__ __device__ inline char* fmt4_digits(char* o, double x) {
  bool neg;
  const uint64_t N = fmt4_scaled(x, &neg);
  if (neg) *o++ = '-';
  // the digits of ip = N / 10^4, then 4 decimals, two at a time
  auto pair = [](unsigned r, char* d) {
    d[0] = static_cast<char>('0' + r / 10u);
    d[1] = static_cast<char>('0' + r % 10u);
  };
  const uint64_t ip = N / 10000u;
  const unsigned fp = static_cast<unsigned>(N - ip * 10000u);
  char t[24];
  int k = 0;
  uint64_t a = ip;
  while (a >= 100u) {
    const unsigned r = static_cast<unsigned>(a % 100u);
    a /= 100u;
    char d[2];
    pair(r, d);
    t[k++] = d[1];
    t[k++] = d[0];
  }
  if (a >= 10u) {
    char d[2];
    pair(static_cast<unsigned>(a), d);
    t[k++] = d[1];
    t[k++] = d[0];
  } else {
    t[k++] = static_cast<char>('0' + a);
  }
  while (k) *o++ = t[--k];
  *o++ = '.';
  pair(fp / 100u, o);
  pair(fp % 100u, o + 2);
  return o + 4;
}

char* fmt4(char* o, double x) {
  if (!fmt4_exact(x)) {  // non-finite or large: libc
    if (x != x) return o + sprintf(o, "nan");
    if (__builtin_isinf(x)) return o + sprintf(o, x < 0 ? "-inf" : "inf");
    return o + sprintf(o, "%.4f", x);
  }
  return fmt4_digits(o, x);
}

__host__ __device__ inline int u8_len(unsigned v) { return v >= 100 ? 3 : v >= 10 ? 2 : 1; }

__host__ __device__ inline char* fmt_u8_hd(char* o, unsigned v) {
  if (v >= 100) *o++ = static_cast<char>('0' + v / 100u);
  if (v >= 10) *o++ = static_cast<char>('0' + v / 10u % 10u);
  *o++ = static_cast<char>('0' + v % 10u);
  return o;
}

// one point's line "x y z r g b\n" (every coordinate fmt4_exact) -> end
__host__ __device__ inline char* ply_line(char* o, double x, double y, double z, unsigned b, unsigned g,
                                          unsigned r) {
  o = fmt4_digits(o, x);
  *o++ = ' ';
  o = fmt4_digits(o, y);
  *o++ = ' ';
  o = fmt4_digits(o, z);
  *o++ = ' ';
  o = fmt_u8_hd(o, r);
  *o++ = ' ';
  o = fmt_u8_hd(o, g);
  *o++ = ' ';
  o = fmt_u8_hd(o, b);
  *o++ = '\n';
  return o;
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

// ---- the same text on the device (sl_write_ply_device) ----
// One thread per point, kPlyBlock points per workgroup.  k_ply_len: every
// line's length from the exact scaled values (no text), summed per workgroup;
// a coordinate outside fmt4_exact sets *fallback (libc's %.4f: the host
// formats that cloud).  k_ply_scan: one workgroup turns the sums into each
// workgroup's byte offset (+ the total at [nb]).  k_ply_text: every line
// written into LDS at its offset inside the workgroup's span, then the span
// to global memory, 256 consecutive bytes per store round.
constexpr int kPlyBlock = 256;
constexpr int kPlyLineMax = 72;  // longest line with every |coordinate| < 9e11: 3 x 18 + 3 + 11 + 1 = 69

template <typename T>
__device__ inline void ply_point(const T* xyz, const uint8_t* bgr, int64_t i, double* v, unsigned* c) {
  v[0] = static_cast<double>(xyz[3 * i]);
  v[1] = static_cast<double>(xyz[3 * i + 1]);
  v[2] = static_cast<double>(xyz[3 * i + 2]);
  c[0] = bgr[3 * i];
  c[1] = bgr[3 * i + 1];
  c[2] = bgr[3 * i + 2];
}

template <typename T>
__device__ inline unsigned ply_line_len(const T* xyz, const uint8_t* bgr, int64_t i, int64_t n, bool* bad) {
  *bad = false;
  if (i >= n) return 0u;
  double v[3];
  unsigned c[3];
  ply_point(xyz, bgr, i, v, c);
  if (!(fmt4_exact(v[0]) && fmt4_exact(v[1]) && fmt4_exact(v[2]))) {
    *bad = true;
    return 0u;
  }
  return static_cast<unsigned>(fmt4_len(v[0]) + fmt4_len(v[1]) + fmt4_len(v[2]) + u8_len(c[0]) + u8_len(c[1]) +
                               u8_len(c[2]) + 6);
}

// inclusive scan over the workgroup (kPlyBlock threads); *total: the sum
__device__ inline unsigned ply_block_scan(unsigned x, unsigned* s_w, unsigned* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const unsigned t = __shfl_up(x, d, 64);
    if (lane >= d) x += t;
  }
  if (lane == 63) s_w[wid] = x;
  __syncthreads();
  unsigned before = 0u, all = 0u;
#pragma unroll
  for (int w = 0; w < kPlyBlock / 64; ++w) {
    before += w < wid ? s_w[w] : 0u;
    all += s_w[w];
  }
  *total = all;
  return x + before;
}

template <typename T>
__global__ __launch_bounds__(kPlyBlock) void k_ply_len(const T* xyz, const uint8_t* bgr, int64_t n, unsigned* bsum,
                                                        unsigned* fallback) {
  __shared__ unsigned s_w[kPlyBlock / 64];
  bool bad;
  const unsigned len = ply_line_len(xyz, bgr, static_cast<int64_t>(blockIdx.x) * kPlyBlock + threadIdx.x, n, &bad);
  if (bad) atomicOr(fallback, 1u);
  unsigned total;
  (void)ply_block_scan(len, s_w, &total);
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

__global__ __launch_bounds__(1024) void k_ply_scan(const unsigned* bsum, int64_t nb, int64_t* boff) {
  __shared__ long long s_w[16];
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int64_t per = (nb + 1023) / 1024, lo = tid * per, hi = std::min<int64_t>(nb, lo + per);
  long long mine = 0;
  for (int64_t b = lo; b < hi; ++b) mine += bsum[b];
  long long x = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const long long t = __shfl_up(x, d, 64);
    if (lane >= d) x += t;
  }
  if (lane == 63) s_w[wid] = x;
  __syncthreads();
  long long before = 0;
  for (int w = 0; w < wid; ++w) before += s_w[w];
  long long off = x - mine + before;  // exclusive
  for (int64_t b = lo; b < hi; ++b) {
    boff[b] = off;
    off += bsum[b];
  }
  if (tid == 1023) boff[nb] = off;  // the text's total bytes
}

template <typename T>
__global__ __launch_bounds__(kPlyBlock) void k_ply_text(const T* xyz, const uint8_t* bgr, int64_t n,
                                                         const int64_t* boff, char* out) {
  __shared__ unsigned s_w[kPlyBlock / 64];
  __shared__ char s_txt[kPlyBlock * kPlyLineMax];
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kPlyBlock + threadIdx.x;
  bool bad;
  const unsigned len = ply_line_len(xyz, bgr, i, n, &bad);
  unsigned total;
  const unsigned end = ply_block_scan(len, s_w, &total);
  if (len) {
    double v[3];
    unsigned c[3];
    ply_point(xyz, bgr, i, v, c);
    (void)ply_line(s_txt + (end - len), v[0], v[1], v[2], c[0], c[1], c[2]);
  }
  __syncthreads();
  char* dst = out + boff[blockIdx.x];
  for (unsigned j = threadIdx.x; j < total; j += kPlyBlock) dst[j] = s_txt[j];
}

// Header + the point lines in `threads` contiguous parts (formatted in
// parallel) into per-part buffers kept across calls (grown, never zero-filled:
// a fresh 64-B-per-point buffer of a 4K view is ~420 MB whose zero fill and
// first-touch page faults had cost more than the formatting).  The buffers are
// the process's; ply_mutex() serialises their users.
struct PlyParts {
  std::string head;
  std::vector<const char*> ptr;
  std::vector<size_t> len;
};
// open(path) for writing from byte 0, as open(O_TRUNC) does -- except that a
// large regular file already there (a re-run over the same scan folder) is
// renamed away first and unlinked on another thread: truncating a 250-MB
// file's cached pages in the writer's path had cost 40 ms per file (66 ms
// against 26 for a new file; rename + the unlink beside the write 27 ms,
// scripts/dbg/overwrite_cost.py).  The new file takes the old one's mode.
// Symlinks, files with other hard links, files of another owner and small
// files are truncated in place, as open(..., 'w') does.  The unlinks still
// pending when the process exits are waited for (10 s at most).
struct PlyReaper {
  std::mutex m;
  std::condition_variable cv;
  int pending = 0;
  unsigned long seq = 0;
  const pid_t owner = getpid();  // (a forked child has none of the unlink threads: it does not wait)
  ~PlyReaper() {
    if (getpid() != owner) return;
    std::unique_lock<std::mutex> lk(m);
    cv.wait_for(lk, std::chrono::seconds(10), [this] { return pending == 0; });
  }
};
PlyReaper& ply_reaper() {
  static PlyReaper r;
  return r;
}
int open_replacing(const char* path) {
  struct stat st;
  if (lstat(path, &st) == 0 && S_ISREG(st.st_mode) && st.st_nlink == 1 && st.st_uid == geteuid() &&
      st.st_size >= (16 << 20)) {
    PlyReaper& r = ply_reaper();
    unsigned long k;
    {
      std::lock_guard<std::mutex> lk(r.m);
      k = r.seq++;
    }
    std::string old = std::string(path) + ".slgpu-old-" + std::to_string(getpid()) + "-" + std::to_string(k);
    if (rename(path, old.c_str()) == 0) {
      const int fd = open(path, O_WRONLY | O_CREAT | O_EXCL | O_CLOEXEC, st.st_mode & 07777);
      if (fd < 0) {  // (the path reappeared meanwhile): the old file back, and the plain route
        rename(old.c_str(), path);
      } else {
        fchmod(fd, st.st_mode & 07777);  // (the mode, whatever the umask)
        {
          std::lock_guard<std::mutex> lk(r.m);
          ++r.pending;
        }
        std::thread([&r, old]() {
          unlink(old.c_str());
          std::lock_guard<std::mutex> lk(r.m);
          --r.pending;
          r.cv.notify_all();
        }).detach();
        return fd;
      }
    }
  }
  return open(path, O_WRONLY | O_CREAT | O_TRUNC | O_CLOEXEC, 0666);
}

std::mutex& ply_mutex() {
  static std::mutex m;
  return m;
}
void ply_format(const void* xyz, int xyz_dtype, const uint8_t* bgr, int64_t n, int threads, PlyParts& out) {
  static std::vector<std::unique_ptr<char[]>> bufs;  // guarded by ply_mutex()
  static std::vector<size_t> caps;
  char hb[256];
  snprintf(hb, sizeof(hb),
           "ply\nformat ascii 1.0\nelement vertex %lld\nproperty float x\nproperty float y\n"
           "property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\nend_header\n",
           static_cast<long long>(n));
  out.head = hb;
  const int T = static_cast<int>(
      std::max<int64_t>(1, std::min<int64_t>(threads > 0 ? threads : 1, (n + 65535) / 65536)));
  if (static_cast<int>(bufs.size()) < T) {
    bufs.resize(T);
    caps.resize(T, 0);
  }
  out.ptr.assign(T, nullptr);
  out.len.assign(T, 0);
  constexpr size_t kLineMax = 3 * 330 + 16;  // worst case: three %.4f of ~1.8e308 + colours
  auto work = [&](int t) {
    const int64_t lo = n * t / T, hi = n * (t + 1) / T;
    auto grow = [&](size_t need) {
      if (need <= caps[t]) return;
      const size_t cap = std::max(need, 2 * caps[t]);
      std::unique_ptr<char[]> nb(new char[cap]);
      if (out.len[t]) memcpy(nb.get(), bufs[t].get(), out.len[t]);
      bufs[t] = std::move(nb);
      caps[t] = cap;
    };
    grow(static_cast<size_t>(hi - lo) * 48 + kLineMax);
    size_t used = 0;
    for (int64_t i = lo; i < hi; ++i) {
      if (used + kLineMax > caps[t]) {
        out.len[t] = used;
        grow(2 * caps[t]);
      }
      char* o = bufs[t].get() + used;
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
      used = static_cast<size_t>(o - bufs[t].get());
    }
    out.len[t] = used;
    out.ptr[t] = bufs[t].get();
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
  // k_decode's grid cap and the pre-stats grid, per CU
  int n_cu = 0;
  if (hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, device) != hipSuccess || n_cu < 1)
    n_cu = 256;
  c->n_cu = n_cu;
  c->decode_wgs = kDecodePerCu * n_cu;
  c->pre_wgs = 2 * n_cu;
  // (test switch: the exact f32 mode through the reference's own operation
  // sequence instead of the verified route, which the GPU tests compare)
  if (const char* d = getenv("SLGPU_VERIFY32")) c->verify32 = atoi(d) != 0;
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
  for (void* ptr : {static_cast<void*>(c->d_ply_bsum), static_cast<void*>(c->d_ply_boff),
                    static_cast<void*>(c->d_ply_text)})
    if (ptr) (void)hipFree(ptr);
  if (c->h_ply_text) (void)hipHostFree(c->h_ply_text);
  if (c->done_ev) (void)hipEventDestroy(c->done_ev);
  for (hipEvent_t e : c->prof_ev) (void)hipEventDestroy(e);
  for (void* ptr : {static_cast<void*>(c->d_planes), static_cast<void*>(c->d_xn), static_cast<void*>(c->d_yn),
                    static_cast<void*>(c->d_nc), static_cast<void*>(c->d_stats), static_cast<void*>(c->d_f32),
                    static_cast<void*>(c->d_codes), static_cast<void*>(c->d_hist[0]),
                    static_cast<void*>(c->d_hist[1]), static_cast<void*>(c->d_ptnib),
                    static_cast<void*>(c->d_block_sums), static_cast<void*>(c->d_chunk_counts),
                    static_cast<void*>(c->d_super)})
    if (ptr) (void)hipFree(ptr);
  delete c;
}

const char* sl_ctx_last_error(const sl_ctx* c) { return c ? c->err.c_str() : "null context"; }

int sl_ctx_reserve(sl_ctx* c, int64_t max_views, int64_t max_px) {
  if (!c || max_views < 1 || max_px < 1) return fail(c, SL_EINVAL, "sl_ctx_reserve: bad sizes");
  HIP_TRY(c, hipSetDevice(c->device));
  // (the histograms for a whole launch group: a pre-stats pass of the next
  // group or call never needs more)
  const int64_t vpg = std::max<int64_t>(1, kMaxChunks / ((max_px + kChunk - 1) / kChunk));
  int r = ensure_scratch(c, std::min(vpg, max_views), max_px, true, vpg);
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
    // planes32 [Wp][4] | xn32 [W] | yn32 [H] | 1 KB of slack
    std::vector<float> f(4 * static_cast<size_t>(Wp) + W + H + 256, 0.0f);
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
  {  // may k_cloud compute the rays' x / y?  Checked on the device, entry by entry
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
  const hipEvent_t ready_ev = c->ready_next ? c->ready_ev_next : nullptr;  // sl_stack_ready: this call only (likewise)
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
  const bool decide = vec && W <= kDecX && H <= kDecY &&
                      (!xyz || (c->has_calib && c->W == W && c->H == H && c->Wp <= kDecPl));
  HIP_TRY(c, hipSetDevice(c->device));
  const hipStream_t s = static_cast<hipStream_t>(stream);
  r = stream_handoff(c, s);
  if (r) return r;
  if (ready_ev) HIP_TRY(c, hipStreamWaitEvent(s, ready_ev, 0));  // the caller's promise, kept on the stream
  return launch(c, p, vec, decide ? (decode_mode | M_DECIDE) : decode_mode, count_mode, cloud_mode, s, arms);
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
  // Measurement only, and eager only: it waits on its events, and its clears
  // are hipMemsetAsync, which torch's bundled HIP runtime mis-replays as
  // graph nodes (k_zero).  Refused while the stream is capturing.
  {
    hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
    HIP_TRY(c, hipStreamIsCapturing(s, &st));
    if (st != hipStreamCaptureStatusNone)
      return fail(c, SL_EINVAL, "sl_time_kernels: the last call's stream is capturing (re-runs are eager only)");
  }
  // The launch consumed its inputs (its k_decode / k_count zeroed the
  // histograms they read; the super-block sums it accumulated are stale
  // until the next producer zeroes them): from clean
  // scratch they are rebuilt once, untimed, then every kernel re-runs with
  // `rerun` set (consumers leave their inputs as they are).  k_cloud first --
  // it reads the super-block sums the producers' re-runs add into again --
  // then k_decode (M_DECIDE; k_count otherwise), which reads the histograms
  // that k_stats' (k_decode's) re-runs accumulate into, then k_stats (k_decode).
  // Afterwards the scratch is cleared again: a pass queued for the next call
  // is dropped (that call computes its own histograms).
  Params pr[3];
  for (int k = 0; k < 3; ++k) {
    pr[k] = c->last.p[k];
    pr[k].rerun = 1;
  }
  auto run = [&](const void* fn, int k) -> hipError_t {
    Params q = pr[k];
    void* args[] = {&q};
    return hipLaunchKernel(fn, c->last.grid[k], dim3(kThreads), args, 0, s);
  };
  auto clear = [&]() -> hipError_t {
    hipError_t e = hipMemsetAsync(c->d_hist[0], 0, sizeof(unsigned) * c->cap_hist, s);
    if (e == hipSuccess) e = hipMemsetAsync(c->d_hist[1], 0, sizeof(unsigned) * c->cap_hist, s);
    if (e == hipSuccess) e = hipMemsetAsync(c->d_super, 0, sizeof(unsigned) * kSuperWords, s);
    return e;
  };
  hipError_t e = clear();
  if (e == hipSuccess && c->last.decide && c->last.stats) e = run(reinterpret_cast<const void*>(k_stats), 1);
  if (e == hipSuccess) e = run(c->last.fn[0], 0);
  if (e == hipSuccess && !c->last.decide && c->last.fn[1]) e = run(c->last.fn[1], 1);
  hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};
  for (int k = 0; k < 4 && e == hipSuccess; ++k) e = hipEventCreate(&ev[k]);
  int r = e == hipSuccess ? SL_OK : fail(c, SL_EHIP, std::string("sl_time_kernels: ") + hipGetErrorString(e));
  const int order3[3] = {2, 1, 0}, orderd[3] = {2, 0, 1};
  const int* order = c->last.decide ? orderd : order3;
  if (r == SL_OK && hipEventRecord(ev[0], s) != hipSuccess) r = fail(c, SL_EHIP, "hipEventRecord");
  for (int q = 0; q < 3 && r == SL_OK; ++q) {
    const int k = order[q];
    if (c->last.fn[k]) {
      for (int i = 0; i < reps; ++i) {
        e = run(c->last.fn[k], k);
        if (e != hipSuccess) {
          r = fail(c, SL_EHIP, std::string("sl_time_kernels: ") + hipGetErrorString(e));
          break;
        }
      }
    }
    if (r == SL_OK && hipEventRecord(ev[q + 1], s) != hipSuccess) r = fail(c, SL_EHIP, "hipEventRecord");
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
    const unsigned nv = c->last.grid[0].y;
    unsigned* ctr = c->d_super + (kSuperCap - nv);  // (buffer 0: the re-runs leave the selectors at 0)
    double sum = 0.0;
    for (int i = 0; i < reps && r == SL_OK; ++i) {
      float ms = 0.f;
      if (hipMemsetAsync(ctr, 0, sizeof(unsigned) * nv, s) != hipSuccess || hipEventRecord(ev[0], s) != hipSuccess ||
          run(c->last.fn[0], 0) != hipSuccess || hipEventRecord(ev[1], s) != hipSuccess ||
          hipEventSynchronize(ev[1]) != hipSuccess || hipEventElapsedTime(&ms, ev[0], ev[1]) != hipSuccess) {
        r = fail(c, SL_EHIP, "sl_time_kernels: dynamic k_decode re-run");
        break;
      }
      sum += ms;
    }
    if (r == SL_OK) out[0] = sum / reps;
  }
  for (int k = 0; k < 4; ++k)
    if (ev[k]) (void)hipEventDestroy(ev[k]);
  // the re-runs accumulated into the histograms and the super-block sums
  if (clear() != hipSuccess && r == SL_OK) r = fail(c, SL_EHIP, "sl_time_kernels: scratch reset");
  c->hist_dirty[0] = c->hist_dirty[1] = 0;
  c->super_dirty = r != SL_OK;
  c->pre_armed = false;
  c->last.valid = false;
  if (decode_ms) *decode_ms = out[0];
  if (count_ms) *count_ms = out[1];
  if (cloud_ms) *cloud_ms = out[2];
  return r;
}

int sl_last_launch_info(sl_ctx* c, int* path, int64_t* launches, int64_t* last_launch_px) {
  if (!c) return SL_EINVAL;
  if (path) *path = c->last.decide ? 1 : 0;
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
  std::lock_guard<std::mutex> lk(ply_mutex());
  PlyParts parts;
  ply_format(xyz, xyz_dtype, bgr, n, threads, parts);
  int64_t len = static_cast<int64_t>(parts.head.size());
  for (size_t l : parts.len) len += static_cast<int64_t>(l);
  *out_len = len;
  if (!out) return SL_OK;  // size query
  if (out_capacity < len) return SL_ECAPACITY;
  memcpy(out, parts.head.data(), parts.head.size());
  int64_t off = static_cast<int64_t>(parts.head.size());
  for (size_t t = 0; t < parts.len.size(); ++t) {
    if (parts.len[t]) memcpy(out + off, parts.ptr[t], parts.len[t]);
    off += static_cast<int64_t>(parts.len[t]);
  }
  return SL_OK;
}

// The parts are written in order with write(2) straight from the formatting
// buffers.  (Alternatives measured on the GPU box, a 4K view's 250 MB:
// copying the parts into a shared mapping of the file in parallel, 142 ms per
// file against 50 for one sequential write -- every page of the mapping
// faults into the page cache; write()s of one file serialise on its inode
// lock, so parallel pwrite()s gain nothing.)
int sl_write_ply(const char* path, const void* xyz, int xyz_dtype, const uint8_t* bgr, int64_t n, int threads) {
  if (!path || !ply_args_ok(xyz, xyz_dtype, bgr, n)) return SL_EINVAL;
  std::lock_guard<std::mutex> lk(ply_mutex());
  PlyParts parts;
  ply_format(xyz, xyz_dtype, bgr, n, threads, parts);
  const int fd = open_replacing(path);
  if (fd < 0) return SL_EIO;
  auto put = [fd](const char* p, size_t len) -> bool {
    while (len) {
      const ssize_t w = write(fd, p, len);
      if (w < 0 && errno == EINTR) continue;
      if (w <= 0) return false;
      p += w;
      len -= static_cast<size_t>(w);
    }
    return true;
  };
  bool ok = put(parts.head.data(), parts.head.size());
  for (size_t t = 0; ok && t < parts.len.size(); ++t) ok = put(parts.ptr[t], parts.len[t]);
  ok = (close(fd) == 0) && ok;
  return ok ? SL_OK : SL_EIO;
}

// The cloud a call left in HBM, formatted on the device and written: the
// lines' lengths and offsets, the text into device scratch, then back in
// chunks through a pinned buffer, each chunk written while the next one is
// in flight.  A cloud with a coordinate the exact path does not take (non-
// finite, |x| >= 9e11) is copied back and formatted on the host instead.
int sl_write_ply_device(sl_ctx* c, const char* path, const void* xyz, int xyz_dtype, const uint8_t* bgr, int64_t n,
                        void* stream) {
  if (!c || !path || !ply_args_ok(xyz, xyz_dtype, bgr, n)) return SL_EINVAL;
  HIP_TRY(c, hipSetDevice(c->device));
  hipStream_t s = static_cast<hipStream_t>(stream);
  const int64_t nb = std::max<int64_t>(1, (n + kPlyBlock - 1) / kPlyBlock);
  int r = grow(c, &c->d_ply_bsum, &c->cap_ply_bsum, nb + 1, s, true);  // [nb]: the fallback flag
  if (r) return r;
  r = grow(c, &c->d_ply_boff, &c->cap_ply_boff, nb + 1, s, true);
  if (r) return r;
  unsigned* flag = c->d_ply_bsum + nb;
  r = zero_async(c, flag, 1, s);
  if (r) return r;
  const bool f64 = xyz_dtype == SL_XYZ_F64;
  if (n > 0) {
    if (f64)
      hipLaunchKernelGGL(k_ply_len<double>, dim3(static_cast<unsigned>(nb)), dim3(kPlyBlock), 0, s,
                         static_cast<const double*>(xyz), bgr, n, c->d_ply_bsum, flag);
    else
      hipLaunchKernelGGL(k_ply_len<float>, dim3(static_cast<unsigned>(nb)), dim3(kPlyBlock), 0, s,
                         static_cast<const float*>(xyz), bgr, n, c->d_ply_bsum, flag);
    hipLaunchKernelGGL(k_ply_scan, dim3(1), dim3(1024), 0, s, c->d_ply_bsum, nb, c->d_ply_boff);
    HIP_TRY(c, hipGetLastError());
  }
  int64_t total = 0;
  unsigned fallback = 0;
  if (n > 0) {
    HIP_TRY(c, hipMemcpyAsync(&total, c->d_ply_boff + nb, sizeof(total), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(&fallback, flag, sizeof(fallback), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
  }
  if (fallback) {  // libc's %.4f for some coordinate: the host formatter on a host copy
    const size_t esz = f64 ? 8 : 4;
    std::vector<char> hx(static_cast<size_t>(n) * 3 * esz);
    std::vector<uint8_t> hb(static_cast<size_t>(n) * 3);
    HIP_TRY(c, hipMemcpyAsync(hx.data(), xyz, hx.size(), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipMemcpyAsync(hb.data(), bgr, hb.size(), hipMemcpyDeviceToHost, s));
    HIP_TRY(c, hipStreamSynchronize(s));
    return sl_write_ply(path, hx.data(), xyz_dtype, hb.data(), n, 16);
  }
  r = grow(c, &c->d_ply_text, &c->cap_ply_text, std::max<int64_t>(total, 1), s, true);
  if (r) return r;
  if (n > 0) {
    if (f64)
      hipLaunchKernelGGL(k_ply_text<double>, dim3(static_cast<unsigned>(nb)), dim3(kPlyBlock), 0, s,
                         static_cast<const double*>(xyz), bgr, n, c->d_ply_boff, c->d_ply_text);
    else
      hipLaunchKernelGGL(k_ply_text<float>, dim3(static_cast<unsigned>(nb)), dim3(kPlyBlock), 0, s,
                         static_cast<const float*>(xyz), bgr, n, c->d_ply_boff, c->d_ply_text);
    HIP_TRY(c, hipGetLastError());
  }
  if (total > c->cap_h_ply_text) {
    if (c->h_ply_text) HIP_TRY(c, hipHostFree(c->h_ply_text));
    c->h_ply_text = nullptr;
    c->cap_h_ply_text = 0;
    HIP_TRY(c, hipHostMalloc(reinterpret_cast<void**>(&c->h_ply_text), static_cast<size_t>(total)));
    c->cap_h_ply_text = total;
  }
  char hb[256];
  const int hl = snprintf(hb, sizeof(hb),
                          "ply\nformat ascii 1.0\nelement vertex %lld\nproperty float x\nproperty float y\n"
                          "property float z\nproperty uchar red\nproperty uchar green\nproperty uchar blue\n"
                          "end_header\n",
                          static_cast<long long>(n));
  // the text back in chunks (events on the stream), each written as it lands
  constexpr int64_t kChunkBytes = int64_t{32} << 20;
  const int nch = static_cast<int>(std::max<int64_t>(1, (total + kChunkBytes - 1) / kChunkBytes));
  std::vector<hipEvent_t> evs(nch, nullptr);
  bool ok = true;
  for (int k = 0; k < nch && ok; ++k) {
    const int64_t lo = k * kChunkBytes, len = std::min(total, lo + kChunkBytes) - lo;
    ok = hipEventCreateWithFlags(&evs[k], hipEventDisableTiming) == hipSuccess &&
         (len <= 0 || hipMemcpyAsync(c->h_ply_text + lo, c->d_ply_text + lo, static_cast<size_t>(len),
                                     hipMemcpyDeviceToHost, s) == hipSuccess) &&
         hipEventRecord(evs[k], s) == hipSuccess;
  }
  const int fd = ok ? open_replacing(path) : -1;
  auto put = [fd](const char* p, size_t len) -> bool {
    while (len) {
      const ssize_t w = write(fd, p, len);
      if (w < 0 && errno == EINTR) continue;
      if (w <= 0) return false;
      p += w;
      len -= static_cast<size_t>(w);
    }
    return true;
  };
  bool io_ok = fd >= 0 && put(hb, static_cast<size_t>(hl));
  for (int k = 0; k < nch; ++k) {
    const int64_t lo = k * kChunkBytes, len = std::min(total, lo + kChunkBytes) - lo;
    const bool landed = evs[k] && hipEventSynchronize(evs[k]) == hipSuccess;
    ok = ok && landed;
    if (io_ok && landed && len > 0) io_ok = put(c->h_ply_text + lo, static_cast<size_t>(len));
  }
  for (hipEvent_t e : evs)
    if (e) (void)hipEventDestroy(e);
  if (fd >= 0) io_ok = (close(fd) == 0) && io_ok;
  if (!ok) return fail(c, SL_EHIP, "sl_write_ply_device: device formatting or copy failed");
  return io_ok ? SL_OK : SL_EIO;
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
  const int fd = open_replacing(path);
  FILE* f = fd >= 0 ? fdopen(fd, "wb") : nullptr;
  if (!f) {
    if (fd >= 0) close(fd);
    return SL_EIO;
  }
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
