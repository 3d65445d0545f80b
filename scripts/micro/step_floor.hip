// Whole-step floor (measurement only, not part of the library):
// the byte pattern of the library's streamed steps at HEAD -- k_decode and
// k_cloud with trivial compute, on the bench's ring of resident views and
// its lanes -- timed the way bench.py times its window.  What a step of
// bench.py cannot go below with this access pattern on this chip.
//
// Per launch group of nv views (a call = groups of <= `group` views):
//   f_decode : grid (min(chunk groups, ceil(3 n_cu / nv)), nv), 3 workgroups
//              per CU (k_decode's 53.6 KB of LDS), chunk groups strided; per
//              wave one 1024-px chunk, per lane 16 px: the view's `read`
//              planes by 16-B nt buffer loads (white, black, then the pairs,
//              40 in flight), then
//                maps calls: col / row maps as 1-KB contiguous nt stores (4 +
//                4 per chunk), the mask as one 16-B nt store per lane, 12-bit
//                records in pixel order (24 B per lane, two 12-B stores);
//                cloud-only calls: 12-bit records in the 1536-B chunk slots
//                (16 + 8 B per lane, sc1), the views interleaved by chunk
//                group (rec_slot);
//   f_cloud  : grid (pre-stats workgroups + chunk groups, nv), 5 per CU
//              (k_cloud's 28.3 KB of LDS); the pre-stats workgroups (2 per CU
//              in all, ahead) read the NEXT group's / call's white and black
//              planes (16-B default loads); the others, one chunk per wave:
//              the records + texture (24 + 48 B per lane), then the chunk's
//              points at their offset -- BGR as 12-B quads (default policy),
//              xyz as 12-B nt stores, 64 points per store instruction.
// Point counts per chunk: a fixed count (a multiple of 4) so that the cloud
// holds the bench view's points; offsets are host-computed (k_cloud's
// block-prefix loads are a few KB from L2).
//
//   step_floor [--H 2160] [--W 3840] [--planes 46] [--read 46] [--maps 1]
//              [--views 1] [--group 8] [--ring 4] [--lanes 2] [--points 6548659]
//              [--steps 20] [--warmup 10] [--reps 3] [--variants full,...]
// Variants: full | no_pre (no pre-stats reads) | no_rec (no records written /
// read) | bare (neither) | decode (f_decode only) | cloud (f_cloud only) |
// lanes1 (one lane) | chain (each decode after the previous call's decode:
// decode beside cloud) | fulla (full, the point stores in windows aligned to
// 128-B lines of the output) | cloud1 / cloud1a (f_cloud alone, one lane, no
// pre-stats: k_cloud's re-run; unaligned / aligned store windows) |
// mix (one linear kernel per step reading and writing the
// step's bytes in 16-B grid-stride streams: the chip's rate for this
// read/write mix in its most favourable form).
// One JSON line per (variant, rep): µs per step, bytes, TB/s.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <string>
#include <utility>
#include <vector>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
typedef unsigned v3u __attribute__((ext_vector_type(3)));
typedef unsigned v2u __attribute__((ext_vector_type(2)));

constexpr int kThreads = 256;
constexpr int kChunk = 1024;
constexpr int kRecSlot = 1536;
constexpr int kDecodeLdsWords = (2048 * 4 + 4096) + 256;  // k_decode: tables + map stage (53.6 KB)

#define CHECK(x)                                                                            \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(2);                                                                              \
    }                                                                                       \
  } while (0)

struct P {
  const uint8_t* stack;
  int64_t stack_vs;
  int view_bytes;
  int HW, cpv, nv, ngroups;
  int maps, rec;          // maps call (pixel-order records) / records written and read
  int32_t* col;
  int32_t* row;
  uint8_t* mask;
  uint8_t* recs;
  const uint8_t* tex;
  int64_t tex_vs;
  int pts_per_chunk;      // points of every chunk (a multiple of 4)
  int64_t out_vs;         // points per view in the output (cpv * pts_per_chunk)
  float* xyz;
  uint8_t* bgr;
  int cloud_gx;
  const uint8_t* pre_stack;
  int64_t pre_vs;
  int pre_views, pre_bpv;
  unsigned* sink;
  int align;              // store windows aligned to 128-B lines of the output (xyz: 32 points, BGR: 128)
};

template <int READ>
__global__ __launch_bounds__(kThreads, 3) void f_decode(P p) {
  __shared__ __attribute__((aligned(16))) unsigned s_lds[kDecodeLdsWords];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int view = blockIdx.y;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(p.stack + view * p.stack_vs), 0, p.view_bytes, 0x00020000);
  v4u keep = {0u, 0u, 0u, 0u};
  for (int cg = blockIdx.x; cg < p.ngroups; cg += gridDim.x) {
    const int civ = cg * 4 + wid;
    if (civ >= p.cpv) continue;
    const int voff = civ * kChunk + lane * 16;
    auto ldp = [&](int pl) -> v4u { return __builtin_amdgcn_raw_buffer_load_b128(rs, voff, pl * p.HW, 2); };
    const v4u w = ldp(0), b = ldp(1);
    constexpr int NPL = READ - 2;
    constexpr int R = NPL < 40 ? NPL : 40;  // k_decode's kRing (a few loop words spill: ~20 B per lane)
    v4u ring[R];
#pragma unroll
    for (int j = 0; j < R; ++j) ring[j] = ldp(2 + j);
    v4u a = w, c = b;
#pragma unroll
    for (int pl = 0; pl < NPL; pl += 2) {
      const v4u P0 = ring[pl % R], I0 = ring[(pl + 1) % R];
      if (pl + R < NPL) {
        ring[pl % R] = ldp(2 + pl + R);
        ring[(pl + 1) % R] = ldp(3 + pl + R);
      }
      a ^= P0;
      c += I0;
    }
    const int64_t o = static_cast<int64_t>(view) * p.HW + civ * kChunk;  // the chunk's first pixel
    if (p.maps) {
      const int n = 4 * min(kChunk, p.HW - civ * kChunk);
      const __amdgpu_buffer_rsrc_t rc = __builtin_amdgcn_make_buffer_rsrc(p.col + o, 0, n, 0x00020000);
      const __amdgpu_buffer_rsrc_t rr = __builtin_amdgcn_make_buffer_rsrc(p.row + o, 0, n, 0x00020000);
#pragma unroll
      for (int j = 0; j < 4; ++j) __builtin_amdgcn_raw_buffer_store_b128(a + j, rc, 1024 * j + 16 * lane, 0, 2);
#pragma unroll
      for (int j = 0; j < 4; ++j) __builtin_amdgcn_raw_buffer_store_b128(c + j, rr, 1024 * j + 16 * lane, 0, 2);
      __builtin_nontemporal_store(a & c, reinterpret_cast<v4u*>(p.mask + o + 16 * lane));
      if (p.rec) {
        unsigned* ro = reinterpret_cast<unsigned*>(p.recs + 3 * (o + 16 * lane) / 2);
        *reinterpret_cast<v3u*>(ro) = v3u{a[0] ^ c[1], a[1], c[2]};
        *reinterpret_cast<v3u*>(ro + 3) = v3u{a[3], c[0] ^ a[2], c[3]};
      }
    } else if (p.rec) {
      const int64_t slot = (static_cast<int64_t>(civ >> 2) * p.nv + view) * 4 + (civ & 3);
      const __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc(p.recs + kRecSlot * slot, 0, kRecSlot, 0x00020000);
      __builtin_amdgcn_raw_buffer_store_b128(a ^ c, rq, 16 * lane, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b64(v2u{a[0] - c[1], a[2] + c[3]}, rq, 1024 + 8 * lane, 0, 16);
    } else {
      keep ^= a ^ c;
    }
  }
  s_lds[tid] = keep[0] ^ keep[3];  // the LDS stays allocated: 3 workgroups per CU, as k_decode
  __syncthreads();
  if (s_lds[(tid + 64) % kThreads] == 0x9e3779b9u && s_lds[kDecodeLdsWords - 1 - tid] == 1u) p.sink[0] = 1u;
}

__global__ __launch_bounds__(kThreads, 5) void f_cloud(P p) {
  __shared__ uint32_t s_ent[4][kChunk];
  __shared__ __attribute__((aligned(16))) uint32_t s_bgr[4][3 * kChunk / 4 + 4];
  const int tid = threadIdx.x, lane = tid & 63, wid = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int view = blockIdx.y;
  const int npre = static_cast<int>(gridDim.x) - p.cloud_gx;
  if (static_cast<int>(blockIdx.x) < npre) {  // the next group's histogram pass: white + black
    const int64_t sblk = static_cast<int64_t>(blockIdx.y) * npre + blockIdx.x;
    if (sblk >= static_cast<int64_t>(p.pre_views) * p.pre_bpv) return;
    const int pv = static_cast<int>(sblk / p.pre_bpv);
    const int64_t blk = sblk - static_cast<int64_t>(pv) * p.pre_bpv;
    const uint8_t* vb = p.pre_stack + pv * p.pre_vs;
    unsigned acc = 0u;
    for (int64_t i = blk * kThreads + tid; i < p.HW / 16; i += static_cast<int64_t>(p.pre_bpv) * kThreads) {
      const v4u wq = *reinterpret_cast<const v4u*>(vb + 16 * i);
      const v4u bq = *reinterpret_cast<const v4u*>(vb + p.HW + 16 * i);
      acc += (wq[0] ^ bq[1]) + (wq[2] ^ bq[3]) + (wq[1] ^ bq[0]) + (wq[3] ^ bq[2]);
    }
    s_ent[wid][lane] = acc;
    __syncthreads();
    if (s_ent[(wid + 1) & 3][lane] == 0x9e3779b9u) p.sink[1] = acc;
    return;
  }
  const int cx = static_cast<int>(blockIdx.x) - npre;
  const int civ = cx * 4 + wid;
  if (civ >= p.cpv) return;
  const int64_t px0 = static_cast<int64_t>(civ) * kChunk + lane * 16;
  v4u x = {0u, 0u, 0u, 0u};
  if (p.rec) {
    if (p.maps) {
      const v2u* src = reinterpret_cast<const v2u*>(p.recs + 3 * (static_cast<int64_t>(view) * p.HW + px0) / 2);
      const v2u r0 = src[0], r1 = src[1], r2 = src[2];
      x = v4u{r0[0] ^ r2[1], r0[1], r1[0], r1[1] ^ r2[0]};
    } else {
      const int64_t slot = (static_cast<int64_t>(civ >> 2) * p.nv + view) * 4 + (civ & 3);
      const uint8_t* cb = p.recs + kRecSlot * slot;
      const v4u a = *reinterpret_cast<const v4u*>(cb + 16 * lane);
      const v2u b = *reinterpret_cast<const v2u*>(cb + 1024 + 8 * lane);
      x = v4u{a[0] ^ b[0], a[1], a[2] ^ b[1], a[3]};
    }
  }
  const uint8_t* t = p.tex + view * p.tex_vs + 3 * px0;
  const v4u t0 = *reinterpret_cast<const v4u*>(t), t1 = *reinterpret_cast<const v4u*>(t + 16),
            t2 = *reinterpret_cast<const v4u*>(t + 32);
  // the chunk's colours through LDS, as k_cloud (keeps the loads' consumer order)
  v4u* b4 = reinterpret_cast<v4u*>(&s_bgr[wid][0]);
  b4[3 * lane] = t0 ^ x;
  b4[3 * lane + 1] = t1;
  b4[3 * lane + 2] = t2;
  __builtin_amdgcn_wave_barrier();
  const int n = p.pts_per_chunk;
  const int64_t base = static_cast<int64_t>(view) * p.out_vs + static_cast<int64_t>(civ) * n;  // 4 | base
  float* const wx = p.xyz + 3 * base;
  uint8_t* const wc = p.bgr + 3 * base;
  const int sh_c = p.align ? static_cast<int>((base & 127) >> 2) : 0;  // quads before the first 128-point boundary
  const int sh_x = p.align ? static_cast<int>(base & 31) : 0;          // points before the first 32-point boundary
  for (int k = lane - sh_c; k < n / 4; k += 64) {
    if (k < 0) continue;
    const uint32_t* s = &s_bgr[wid][(3 * 4 * k) / 4 % (3 * kChunk / 4)];
    *reinterpret_cast<v3u*>(wc + 12 * k) = v3u{s[0], s[1], s[2]};
  }
  for (int j = lane - sh_x; j < n; j += 64) {
    if (j < 0) continue;
    const unsigned f = static_cast<unsigned>(j) ^ s_bgr[wid][j % (3 * kChunk / 4)];
    float* q = wx + 3 * j;
    __builtin_nontemporal_store(__uint_as_float(f), q);
    __builtin_nontemporal_store(__uint_as_float(f + 1u), q + 1);
    __builtin_nontemporal_store(__uint_as_float(f + 2u), q + 2);
  }
}

// One linear pass: `rd` bytes read and `wr` bytes written as 16-B grid-stride
// streams (nt loads and stores), interleaved in the ratio of the two.
__global__ __launch_bounds__(kThreads) void f_mix(const v4u* src, int64_t rd16, v4u* dst, int64_t wr16, unsigned* sink) {
  const int64_t nt = static_cast<int64_t>(gridDim.x) * kThreads;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x;
  v4u acc = {0u, 0u, 0u, 0u};
  const int64_t steps = (rd16 + nt - 1) / nt;
  for (int64_t s = 0; s < steps; ++s) {
    const int64_t i = s * nt + t0;
    if (i < rd16) acc ^= __builtin_nontemporal_load(src + i);
    const int64_t w0 = (s * wr16) / steps, w1 = ((s + 1) * wr16) / steps;  // this step's share of the writes
    for (int64_t j = w0 + t0; j < w1; j += nt) __builtin_nontemporal_store(acc + static_cast<unsigned>(j), dst + j);
  }
  if (acc[0] == 0x9e3779b9u && acc[1] == 7u) sink[2] = acc[2];
}

struct Buf {
  uint8_t* p = nullptr;
  size_t n = 0;
};
static uint8_t* dalloc(size_t n, int fill) {
  uint8_t* p = nullptr;
  CHECK(hipMalloc(&p, n));
  CHECK(hipMemset(p, fill, n));
  return p;
}

int main(int argc, char** argv) {
  int H = 2160, W = 3840, planes = 46, rd = 46, maps = 1, views = 1, group = 8, ring = 4, lanes = 2;
  int steps = 20, warmup = 10, reps = 3;
  int64_t points = 6548659;
  std::string variants = "full,no_pre,no_rec,bare,lanes1,decode,cloud,mix";
  for (int i = 1; i + 1 < argc; i += 2) {
    const std::string k = argv[i];
    const char* v = argv[i + 1];
    if (k == "--H") H = atoi(v);
    else if (k == "--W") W = atoi(v);
    else if (k == "--planes") planes = atoi(v);
    else if (k == "--read") rd = atoi(v);
    else if (k == "--maps") maps = atoi(v);
    else if (k == "--views") views = atoi(v);
    else if (k == "--group") group = atoi(v);
    else if (k == "--ring") ring = atoi(v);
    else if (k == "--lanes") lanes = atoi(v);
    else if (k == "--points") points = atoll(v);
    else if (k == "--steps") steps = atoi(v);
    else if (k == "--warmup") warmup = atoi(v);
    else if (k == "--reps") reps = atoi(v);
    else if (k == "--variants") variants = v;
    else {
      fprintf(stderr, "unknown option %s\n", k.c_str());
      return 1;
    }
  }
  if (rd != 46 && rd != 24 && rd != 22) {
    fprintf(stderr, "--read: 46, 24 or 22 planes\n");
    return 1;
  }
  const int HW = H * W;
  if (HW % kChunk != 0 || (int64_t)planes * HW >= (1ll << 31)) {
    fprintf(stderr, "frame must be a multiple of 1024 px and a view < 2 GiB\n");
    return 1;
  }
  const int cpv = HW / kChunk;
  const int ngroups = (cpv + 3) / 4;
  int ppc = static_cast<int>((points + cpv - 1) / cpv);
  ppc = (ppc + 3) / 4 * 4;
  if (ppc > kChunk) ppc = kChunk;
  const int64_t out_vs = static_cast<int64_t>(cpv) * ppc;
  int n_cu = 256;
  CHECK(hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0));

  // inputs: `ring` slots of `views` views (stack + texture); outputs per
  // (slot, lane) pair that the schedule uses; records per lane (one group)
  const int64_t stack_vs = static_cast<int64_t>(planes) * HW;
  std::vector<uint8_t*> st(ring), tx(ring);
  for (int r = 0; r < ring; ++r) {
    st[r] = dalloc(stack_vs * views, 0x5a + r);
    tx[r] = dalloc(3ll * HW * views, 0x33 + r);
  }
  struct Out {
    int32_t* col = nullptr;
    int32_t* row = nullptr;
    uint8_t* mask = nullptr;
    float* xyz = nullptr;
    uint8_t* bgr = nullptr;
  };
  std::map<std::pair<int, int>, Out> outs;
  auto out_of = [&](int slot, int lane) -> Out& {
    auto key = std::make_pair(slot, lane);
    auto it = outs.find(key);
    if (it != outs.end()) return it->second;
    Out o;
    if (maps) {
      o.col = reinterpret_cast<int32_t*>(dalloc(4ll * HW * views, 0));
      o.row = reinterpret_cast<int32_t*>(dalloc(4ll * HW * views, 0));
      o.mask = dalloc(1ll * HW * views, 0);
    }
    o.xyz = reinterpret_cast<float*>(dalloc(12ll * out_vs * views + 64, 0));
    o.bgr = dalloc(3ll * out_vs * views + 64, 0);
    return outs[key] = o;
  };
  const int gmax = views < group ? views : group;
  const int64_t rec_bytes = maps ? (3ll * HW * gmax) / 2 + 64 : static_cast<int64_t>(kRecSlot) * ngroups * 4 * gmax + 64;
  std::vector<uint8_t*> recs(lanes);
  for (int l = 0; l < lanes; ++l) recs[l] = dalloc(rec_bytes, 0);
  unsigned* sink = reinterpret_cast<unsigned*>(dalloc(64, 0));
  std::vector<hipStream_t> ss(lanes);
  for (int l = 0; l < lanes; ++l) CHECK(hipStreamCreateWithFlags(&ss[l], hipStreamNonBlocking));
  hipEvent_t ev0, ev_end[8], ev_join;
  CHECK(hipEventCreate(&ev0));
  CHECK(hipEventCreate(&ev_join));
  for (int l = 0; l < 8; ++l) CHECK(hipEventCreate(&ev_end[l]));
  // the mix pass's buffers: one step's reads and writes, per ring slot
  const double pix = static_cast<double>(HW) * views;
  const double b_stack = static_cast<double>(rd) * pix, b_maps = maps ? 9.0 * pix : 0.0, b_tex = 3.0 * pix;
  const double b_rec = 1.5 * pix, b_pre = 2.0 * pix, b_pts = 15.0 * static_cast<double>(ppc) * cpv * views;
  const double algo = b_stack + b_maps + b_tex + b_pts;

  auto kdec = rd == 46 ? f_decode<46> : rd == 24 ? f_decode<24> : f_decode<22>;
  // one call (step) on lane l over ring slot r: launch groups of <= group views
  // "chain": each call's f_decode waits for the previous call's f_decode (on
  // the other lane), so a decode runs beside the other lane's cloud instead
  // of beside its decode (the read-heavy / write-heavy pairing)
  std::vector<hipEvent_t> dec_done(lanes);
  for (int l = 0; l < lanes; ++l) CHECK(hipEventCreateWithFlags(&dec_done[l], hipEventDisableTiming));
  bool chain = false, align = false;
  auto enqueue_call = [&](int step, int lanes_used, bool pre, bool rec, bool dec, bool cld) {
    const int l = step % lanes_used, r = step % ring;
    const int r_next = (step + lanes_used) % ring;  // this lane's next call's slot
    Out& o = out_of(r, l);
    for (int v0 = 0; v0 < views; v0 += group) {
      const int nv = views - v0 < group ? views - v0 : group;
      P p{};
      p.stack = st[r] + v0 * stack_vs;
      p.stack_vs = stack_vs;
      p.view_bytes = static_cast<int>(stack_vs);
      p.HW = HW;
      p.cpv = cpv;
      p.nv = nv;
      p.ngroups = ngroups;
      p.maps = maps;
      p.rec = rec ? 1 : 0;
      p.col = maps ? o.col + static_cast<int64_t>(v0) * HW : nullptr;
      p.row = maps ? o.row + static_cast<int64_t>(v0) * HW : nullptr;
      p.mask = maps ? o.mask + static_cast<int64_t>(v0) * HW : nullptr;
      p.recs = recs[l];
      p.tex = tx[r] + 3ll * HW * v0;
      p.tex_vs = 3ll * HW;
      p.pts_per_chunk = ppc;
      p.out_vs = out_vs;
      p.xyz = o.xyz + 3 * out_vs * v0;
      p.bgr = o.bgr + 3 * out_vs * v0;
      p.sink = sink;
      p.cloud_gx = ngroups;
      p.align = align ? 1 : 0;
      // the pass of the next group of this call, or of the lane's next call's first group
      const bool last = v0 + group >= views;
      const uint8_t* pst = last ? st[r_next] : st[r] + (v0 + group) * stack_vs;
      const int pnv = last ? gmax : (views - v0 - group < group ? views - v0 - group : group);
      const int64_t per_view = (HW / 16 + kThreads - 1) / kThreads;
      int64_t bpv = (2 * n_cu + pnv - 1) / pnv;
      if (bpv > per_view) bpv = per_view;
      p.pre_stack = pst;
      p.pre_vs = stack_vs;
      p.pre_views = pnv;
      p.pre_bpv = static_cast<int>(bpv);
      int dgx = (3 * n_cu + nv - 1) / nv;
      if (dgx > ngroups) dgx = ngroups;
      if (dec) {
        if (chain && step > 0 && lanes_used > 1) CHECK(hipStreamWaitEvent(ss[l], dec_done[(step - 1) % lanes_used], 0));
        hipLaunchKernelGGL(kdec, dim3(dgx, nv), dim3(kThreads), 0, ss[l], p);
        if (chain) CHECK(hipEventRecord(dec_done[l], ss[l]));
      }
      if (cld) {
        const unsigned npre = pre ? static_cast<unsigned>((pnv * bpv + nv - 1) / nv) : 0u;
        hipLaunchKernelGGL(f_cloud, dim3(ngroups + npre, nv), dim3(kThreads), 0, ss[l], p);
      }
    }
  };
  // the mix variant's buffers: one step's reads (a source per ring slot) and
  // writes (a destination per ring slot), the same bytes as a full step
  const double mix_rd = b_stack + b_tex + b_rec + b_pre, mix_wr = b_maps + b_rec + b_pts;
  const int64_t mix_rd16 = static_cast<int64_t>(mix_rd / 16), mix_wr16 = static_cast<int64_t>(mix_wr / 16);
  std::vector<uint8_t*> mix_src, mix_dst;
  if (variants.find("mix") != std::string::npos) {
    for (int r = 0; r < ring; ++r) {
      mix_src.push_back(dalloc(mix_rd16 * 16 + 64, 0x11 + r));
      mix_dst.push_back(dalloc(mix_wr16 * 16 + 64, 0));
    }
  }
  auto enqueue_mix = [&](int step, int lanes_used) {
    const int l = step % lanes_used, r = step % ring;
    hipLaunchKernelGGL(f_mix, dim3(4 * n_cu), dim3(kThreads), 0, ss[l], reinterpret_cast<const v4u*>(mix_src[r]),
                       mix_rd16, reinterpret_cast<v4u*>(mix_dst[r]), mix_wr16, sink);
  };

  auto run = [&](const std::string& var) -> double {
    const bool pre = var != "no_pre" && var != "bare" && var != "mix" && var != "cloud1" && var != "cloud1a";
    const bool rec = var != "no_rec" && var != "bare";
    const bool dec = var != "cloud" && var != "cloud1" && var != "cloud1a",
               cld = var != "decode";
    chain = var == "chain";
    align = var == "fulla" || var == "cloud1a";
    const int L = (var == "lanes1" || var == "cloud1" || var == "cloud1a") ? 1 : lanes;
    auto one = [&](int i) {
      if (var == "mix") enqueue_mix(i, L);
      else enqueue_call(i, L, pre, rec, dec, cld);
    };
    for (int i = 0; i < warmup; ++i) one(i);
    CHECK(hipDeviceSynchronize());
    // the window: every lane starts after one event, ends joined into lane 0
    CHECK(hipEventRecord(ev0, ss[0]));
    for (int l = 1; l < L; ++l) CHECK(hipStreamWaitEvent(ss[l], ev0, 0));
    for (int i = warmup; i < warmup + steps; ++i) one(i);
    for (int l = 1; l < L; ++l) {
      CHECK(hipEventRecord(ev_end[l], ss[l]));
      CHECK(hipStreamWaitEvent(ss[0], ev_end[l], 0));
    }
    CHECK(hipEventRecord(ev_join, ss[0]));
    CHECK(hipEventSynchronize(ev_join));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, ev0, ev_join));
    return 1e3 * ms / steps;
  };

  std::vector<std::string> vars;
  {
    std::string s = variants;
    size_t a = 0;
    while (a <= s.size()) {
      size_t b = s.find(',', a);
      if (b == std::string::npos) b = s.size();
      if (b > a) vars.push_back(s.substr(a, b - a));
      a = b + 1;
    }
  }
  run("full");  // pre-roll: clocks up, every buffer touched
  for (int rep = 0; rep < reps; ++rep) {
    for (const auto& var : vars) {
      const double us = run(var);
      const bool c1v = var == "cloud1" || var == "cloud1a";
      const bool pre = var != "no_pre" && var != "bare" && var != "mix" && !c1v;
      const bool rec = var != "no_rec" && var != "bare";
      double moved = 0.0;
      if (var == "mix") moved = 16.0 * (mix_rd16 + mix_wr16);
      else {
        if (var != "cloud" && !c1v) moved += b_stack + b_maps + (rec ? b_rec : 0.0);
        if (var != "decode") moved += b_tex + b_pts + (rec ? b_rec : 0.0) + (pre ? b_pre : 0.0);
      }
      printf("{\"variant\": \"%s\", \"rep\": %d, \"H\": %d, \"W\": %d, \"planes_read\": %d, \"maps\": %d, "
             "\"views_per_call\": %d, \"group\": %d, \"ring\": %d, \"lanes\": %d, \"points_per_view\": %lld, "
             "\"steps\": %d, \"us_per_step\": %.2f, \"algorithmic_MB\": %.1f, \"moved_MB\": %.1f, "
             "\"algorithmic_TBps\": %.3f, \"moved_TBps\": %.3f, \"frac_of_8TBps\": %.4f}\n",
             var.c_str(), rep, H, W, rd, maps, views, group, ring,
             (var == "lanes1" || var == "cloud1" || var == "cloud1a") ? 1 : lanes,
             static_cast<long long>(out_vs), steps, us, algo / 1e6, moved / 1e6, algo / us / 1e6, moved / us / 1e6,
             algo / us / 1e6 / 8.0);
      fflush(stdout);
    }
  }
  CHECK(hipDeviceSynchronize());
  return 0;
}
