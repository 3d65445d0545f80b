// libslgpu.so, part 2b -- global registration of merge_pro_360
// (server/processing.py:79-113, used at :146-151), included at the end of
// slmerge.hip (one translation unit: it shares that file's cell grids, scratch
// pool and fdlibm helpers).  Open3D is not in this image: the algorithms are
// restated from its published source (pipelines/registration/Feature.cpp,
// Registration.cpp, CorrespondenceChecker.cpp, TransformationEstimation.cpp,
// Eigen's umeyama / JacobiSVD), parity with Open3D is unpinned, and
// oracle/registration_oracle.py is the CPU restatement the tests check
// against bit for bit.
//
//   radius search (KDTreeFlann::SearchHybrid): the query's 27 cells of edge >=
//     radius, candidates with ((dx^2 + dy^2) + dz^2) < radius^2 compacted into
//     LDS by wave ballots, bitonic-sorted by (d2, index), the first max_nn;
//     a query with more than kNnCap candidates selects its max_nn by a radix
//     select over the d2 bits (then the index bits of the ties) instead.
//   FPFH (compute_fpfh_feature): SPFH per point from its pair features
//     (fdlibm acos / atan2: the same bits as the oracle), then the 1/d2
//     weighted sum of the neighbours' SPFH, per-third normalised to 100, plus
//     the point's own SPFH.
//   correspondences: exact nearest neighbour in the 33-D feature space
//     (nanoflann's L2 order, ties to the lower index), both ways, mutual filter.
//   RANSAC (registration_ransac_based_on_feature_matching): Open3D's loop as
//     one thread runs it -- iteration order, early exit at the estimated k --
//     evaluated in batches: a kernel draws and checks thousands of hypotheses
//     at once (3 correspondences, the edge-length checker, Umeyama by a 3x3
//     Jacobi SVD, the distance checker), the survivors are validated in
//     parallel (every moved source point's nearest target point), and the host
//     walks the results in iteration order.

namespace {
namespace reg {

constexpr double kPi = 3.14159265358979311600e+00;

// fdlibm s_atan.c (finite x)
__device__ double atan_det(double x) {
  constexpr double atanhi[4] = {4.63647609000806093515e-01, 7.85398163397448278999e-01, 9.82793723247329054082e-01,
                                1.57079632679489655800e+00};
  constexpr double atanlo[4] = {2.26987774529616870924e-17, 3.06161699786838301793e-17, 1.39033110312309984516e-17,
                                6.12323399573676603587e-17};
  constexpr double aT[11] = {3.33333333333329318027e-01,  -1.99999999998764832476e-01, 1.42857142725034663711e-01,
                             -1.11111104054623557880e-01, 9.09088713343650656196e-02,  -7.69187620504482999495e-02,
                             6.66107313738753120669e-02,  -5.83357013379057348645e-02, 4.97687799461593236017e-02,
                             -3.65315727442169155270e-02, 1.62858201153657823623e-02};
  const int hx = static_cast<int>(static_cast<unsigned long long>(__double_as_longlong(x)) >> 32);
  const int ix = hx & 0x7fffffff;
  int id;
  if (ix >= 0x44100000) {  // |x| >= 2^66
    if (x != x) return x + x;
    return hx > 0 ? atanhi[3] + atanlo[3] : -atanhi[3] - atanlo[3];
  }
  if (ix < 0x3fdc0000) {  // |x| < 0.4375
    if (ix < 0x3e200000) return x;
    id = -1;
  } else {
    x = fabs(x);
    if (ix < 0x3ff30000) {
      if (ix < 0x3fe60000) {
        id = 0;
        x = (2.0 * x - 1.0) / (2.0 + x);
      } else {
        id = 1;
        x = (x - 1.0) / (x + 1.0);
      }
    } else if (ix < 0x40038000) {
      id = 2;
      x = (x - 1.5) / (1.0 + 1.5 * x);
    } else {
      id = 3;
      x = -1.0 / x;
    }
  }
  double z = x * x;
  const double w = z * z;
  const double s1 = z * (aT[0] + w * (aT[2] + w * (aT[4] + w * (aT[6] + w * (aT[8] + w * aT[10])))));
  const double s2 = w * (aT[1] + w * (aT[3] + w * (aT[5] + w * (aT[7] + w * aT[9]))));
  if (id < 0) return x - x * (s1 + s2);
  z = atanhi[id] - ((x * (s1 + s2) - atanlo[id]) - x);
  return hx < 0 ? -z : z;
}

// fdlibm e_atan2.c for finite y, x (NaN in -> NaN out)
__device__ double atan2_det(double y, double x) {
  constexpr double pi_o_2 = 1.5707963267948965580e+00, pi_lo = 1.2246467991473531772e-16;
  if (x != x || y != y) return x + y;
  if (x == 1.0) return atan_det(y);
  const int m = (signbit(y) ? 1 : 0) | (signbit(x) ? 2 : 0);
  if (y == 0.0) {
    if (m < 2) return y;
    return m == 2 ? kPi : -kPi;
  }
  if (x == 0.0) return y < 0.0 ? -pi_o_2 : pi_o_2;
  const int hy = static_cast<int>(static_cast<unsigned long long>(__double_as_longlong(y)) >> 32) & 0x7fffffff;
  const int hx = static_cast<int>(static_cast<unsigned long long>(__double_as_longlong(x)) >> 32) & 0x7fffffff;
  const int k = (hy - hx) >> 20;
  double z;
  if (k > 60) z = pi_o_2 + 0.5 * pi_lo;
  else if (x < 0.0 && k < -60) z = 0.0;
  else z = atan_det(fabs(y / x));
  switch (m) {
    case 0: return z;
    case 1: return -z;
    case 2: return kPi - (z - pi_lo);
    default: return (z - pi_lo) - kPi;
  }
}

struct D3 {
  double x, y, z;
};
__device__ __forceinline__ double dot3(D3 a, D3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
__device__ __forceinline__ double norm3(D3 a) { return sqrt(dot3(a, a)); }
__device__ __forceinline__ D3 cross3(D3 a, D3 b) {
  return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// ComputePairFeatures (Feature.cpp) -> f0 (atan2 angle), f1, f2; all 0 for a
// degenerate pair (Open3D returns Vector4d::Zero())
__device__ void pair_features(D3 p1, D3 n1, D3 p2, D3 n2, double* f0, double* f1, double* f2) {
  D3 dp{p2.x - p1.x, p2.y - p1.y, p2.z - p1.z};
  const double f3 = norm3(dp);
  *f0 = *f1 = *f2 = 0.0;
  if (f3 == 0.0) return;
  const double a1 = dot3(n1, dp) / f3;
  const double a2 = dot3(n2, dp) / f3;
  double g2;
  if (nrm::acos_det(fabs(a1)) > nrm::acos_det(fabs(a2))) {
    const D3 t = n1;
    n1 = n2;
    n2 = t;
    dp = {-dp.x, -dp.y, -dp.z};
    g2 = -a2;
  } else {
    g2 = a1;
  }
  D3 v = cross3(dp, n1);
  const double vn = norm3(v);
  if (vn == 0.0) return;
  v = {v.x / vn, v.y / vn, v.z / vn};
  const D3 w = cross3(n1, v);
  *f1 = dot3(v, n2);
  *f2 = g2;
  *f0 = atan2_det(dot3(w, n2), dot3(n1, n2));
}

// Open3D's bin: floor(x) clamped to [0, 10] (NaN -> 0)
__device__ __forceinline__ int bin11(double x) { return !(x >= 0.0) ? 0 : (x >= 11.0 ? 10 : static_cast<int>(x)); }

// ---- Eigen::umeyama(src, dst, false) of three point pairs (3x3 JacobiSVD) ----
constexpr double kDblMin = 2.2250738585072014e-308;
constexpr double kEps2 = 2.0 * 2.220446049250313e-16;
constexpr int kSvdSweeps = 64;

__device__ __forceinline__ void rot_left(double (&M)[3][3], int p, int q, double c, double s) {
  for (int i = 0; i < 3; ++i) {
    const double x = M[p][i], y = M[q][i];
    M[p][i] = c * x + s * y;
    M[q][i] = -s * x + c * y;
  }
}
__device__ __forceinline__ void rot_right(double (&M)[3][3], int p, int q, double c, double s) {
  for (int i = 0; i < 3; ++i) {
    const double x = M[i][p], y = M[i][q];
    M[i][p] = c * x - s * y;
    M[i][q] = s * x + c * y;
  }
}
__device__ __forceinline__ void make_jacobi(double x, double y, double z, double* c, double* s) {
  const double deno = 2.0 * fabs(y);
  if (deno < kDblMin) {
    *c = 1.0;
    *s = 0.0;
    return;
  }
  const double tau = (x - z) / deno;
  const double w = sqrt(tau * tau + 1.0);
  const double t = tau > 0.0 ? 1.0 / (tau + w) : 1.0 / (tau - w);
  const double sign_t = t > 0.0 ? 1.0 : -1.0;
  const double n = 1.0 / sqrt(t * t + 1.0);
  *c = n;
  *s = -sign_t * (y / fabs(y)) * fabs(t) * n;
}

// JacobiSVD<Matrix3d>(A, ComputeFullU | ComputeFullV): U, V (the singular
// values only order the columns)
__device__ void jacobi_svd3(const double (&A)[3][3], double (&U)[3][3], double (&V)[3][3]) {
  double scale = 0.0;
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) scale = fmax(scale, fabs(A[i][j]));
  if (scale == 0.0) scale = 1.0;
  double W[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) {
      W[i][j] = A[i][j] / scale;
      U[i][j] = V[i][j] = i == j ? 1.0 : 0.0;
    }
  double max_diag = fmax(fmax(fabs(W[0][0]), fabs(W[1][1])), fabs(W[2][2]));
  for (int sweep = 0; sweep < kSvdSweeps; ++sweep) {
    bool finished = true;
    for (int p = 1; p < 3; ++p)
      for (int q = 0; q < p; ++q) {
        const double thr = fmax(kDblMin, kEps2 * max_diag);
        if (fabs(W[p][q]) > thr || fabs(W[q][p]) > thr) {
          finished = false;
          const double m00 = W[p][p], m01 = W[p][q], m10 = W[q][p], m11 = W[q][q];
          const double t = m00 + m11, d = m10 - m01;
          double c1, s1;
          if (fabs(d) < kDblMin) {
            c1 = 1.0;
            s1 = 0.0;
          } else {
            const double u = t / d;
            const double tmp = sqrt(1.0 + u * u);
            s1 = 1.0 / tmp;
            c1 = u / tmp;
          }
          const double a00 = c1 * m00 + s1 * m10, a01 = c1 * m01 + s1 * m11, a11 = -s1 * m01 + c1 * m11;
          double cr, sr;
          make_jacobi(a00, a01, a11, &cr, &sr);
          const double cl = c1 * cr - s1 * (-sr), sl = c1 * (-sr) + s1 * cr;
          rot_left(W, p, q, cl, sl);
          rot_right(U, p, q, cl, -sl);
          rot_right(W, p, q, cr, sr);
          rot_right(V, p, q, cr, sr);
          max_diag = fmax(max_diag, fmax(fabs(W[p][p]), fabs(W[q][q])));
        }
      }
    if (finished) break;
  }
  double s[3];
  for (int i = 0; i < 3; ++i) {
    const double a = W[i][i];
    s[i] = fabs(a) * scale;
    if (a < 0.0)
      for (int r = 0; r < 3; ++r) U[r][i] = -U[r][i];
  }
  for (int i = 0; i < 3; ++i) {
    int pos = i;
    for (int k = i + 1; k < 3; ++k)
      if (s[k] > s[pos]) pos = k;
    if (s[pos] == 0.0) break;
    if (pos != i) {
      const double t = s[i];
      s[i] = s[pos];
      s[pos] = t;
      for (int r = 0; r < 3; ++r) {
        double u = U[r][i];
        U[r][i] = U[r][pos];
        U[r][pos] = u;
        u = V[r][i];
        V[r][i] = V[r][pos];
        V[r][pos] = u;
      }
    }
  }
}

__device__ __forceinline__ double det3(const double (&M)[3][3]) {
  return (M[0][0] * (M[1][1] * M[2][2] - M[2][1] * M[1][2]) - M[1][0] * (M[0][1] * M[2][2] - M[2][1] * M[0][2])) +
         M[2][0] * (M[0][1] * M[1][2] - M[1][1] * M[0][2]);
}

// src[c], dst[c]: the three pairs -> T (3 rows of 4, row-major)
__device__ void umeyama3(const D3 (&src)[3], const D3 (&dst)[3], double (&T)[12]) {
  const double one_over_n = 1.0 / 3.0;
  const double sm[3] = {((src[0].x + src[1].x) + src[2].x) * one_over_n, ((src[0].y + src[1].y) + src[2].y) * one_over_n,
                        ((src[0].z + src[1].z) + src[2].z) * one_over_n};
  const double dm[3] = {((dst[0].x + dst[1].x) + dst[2].x) * one_over_n, ((dst[0].y + dst[1].y) + dst[2].y) * one_over_n,
                        ((dst[0].z + dst[1].z) + dst[2].z) * one_over_n};
  double sd[3][3], dd[3][3];
  for (int c = 0; c < 3; ++c) {
    sd[c][0] = src[c].x - sm[0];
    sd[c][1] = src[c].y - sm[1];
    sd[c][2] = src[c].z - sm[2];
    dd[c][0] = dst[c].x - dm[0];
    dd[c][1] = dst[c].y - dm[1];
    dd[c][2] = dst[c].z - dm[2];
  }
  double sigma[3][3], U[3][3], V[3][3];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j)
      sigma[i][j] = ((dd[0][i] * sd[0][j] + dd[1][i] * sd[1][j]) + dd[2][i] * sd[2][j]) * one_over_n;
  jacobi_svd3(sigma, U, V);
  const double S2 = det3(U) * det3(V) < 0.0 ? -1.0 : 1.0;
  for (int i = 0; i < 3; ++i) {
    for (int j = 0; j < 3; ++j)
      T[4 * i + j] = (U[i][0] * 1.0 * V[j][0] + U[i][1] * 1.0 * V[j][1]) + U[i][2] * S2 * V[j][2];
  }
  for (int i = 0; i < 3; ++i)
    T[4 * i + 3] = dm[i] - ((T[4 * i] * sm[0] + T[4 * i + 1] * sm[1]) + T[4 * i + 2] * sm[2]);
}

__device__ __forceinline__ D3 tp(const double* T, D3 p) {
  return {((T[0] * p.x + T[1] * p.y) + T[2] * p.z) + T[3], ((T[4] * p.x + T[5] * p.y) + T[6] * p.z) + T[7],
          ((T[8] * p.x + T[9] * p.y) + T[10] * p.z) + T[11]};
}

// the n-th random correspondence index (splitmix64 of seed + (n + 1) golden)
__device__ __forceinline__ int64_t draw(uint64_t seed, uint64_t n, uint64_t nc) {
  uint64_t z = seed + (n + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return static_cast<int64_t>(((z >> 32) * nc) >> 32);
}

__device__ __forceinline__ D3 ld3(const double* p, int64_t i) { return {p[3 * i], p[3 * i + 1], p[3 * i + 2]}; }

}  // namespace reg

constexpr int kNnCap = 1024;  // in-radius candidates a query sorts in LDS (more: the radix select)
constexpr int kNnMax = 1024;  // largest max_nn

__device__ __forceinline__ bool nn_lt(double da, uint32_t ia, double db, uint32_t ib) {
  return da < db || (da == db && ia < ib);
}

// Ascending (d2, index) bitonic sort of s_d / s_i[0..P), P a power of two >= 64
// (a one-wave workgroup; every compare-exchange pair belongs to one lane).
__device__ void nn_sort(double* s_d, uint32_t* s_i, int P, int lane) {
  for (int size = 2; size <= P; size <<= 1)
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int k = lane; k < P; k += 64) {
        const int p = k ^ stride;
        if (p > k) {
          const double a = s_d[k], b = s_d[p];
          const uint32_t ia = s_i[k], ib = s_i[p];
          const bool sw = (k & size) == 0 ? nn_lt(b, ib, a, ia) : nn_lt(a, ia, b, ib);
          if (sw) {
            s_d[k] = b;
            s_d[p] = a;
            s_i[k] = ib;
            s_i[p] = ia;
          }
        }
      }
      __syncthreads();
    }
}

struct CellSet {  // the sorted points' cell structure (slmerge.hip's cells())
  const double* sxyz;
  const uint32_t* sidx;
  const uint64_t* skeys;
  int64_t n;
  const uint64_t* ukeys;
  const uint32_t* ustart;
  int64_t m;
  const int32_t* nbr;  // 27 neighbour cells per occupied cell
};

// fn(t, dd, pass) for every candidate of the 27 cells around sorted point j,
// 64 at a time (wave-uniform calls; pass: d2 < r2 and t in range)
template <class F>
__device__ __forceinline__ void nn_scan(const CellSet& cs, int64_t j, double r2, int lane, F&& fn) {
  const double q0 = cs.sxyz[3 * j], q1 = cs.sxyz[3 * j + 1], q2 = cs.sxyz[3 * j + 2];
  const int64_t cell = find_cell(cs.ukeys, cs.m, cs.skeys[j]);
  for (int e = 0; e < 27; ++e) {
    const int32_t cc = cs.nbr[27 * cell + e];
    if (cc < 0) continue;
    const int64_t t0 = cs.ustart[cc], t1 = cc + 1 < cs.m ? static_cast<int64_t>(cs.ustart[cc + 1]) : cs.n;
    for (int64_t b = t0; b < t1; b += 64) {
      const int64_t t = b + lane;
      double dd = INFINITY;
      bool pass = false;
      if (t < t1) {
        const double d0 = q0 - cs.sxyz[3 * t], d1 = q1 - cs.sxyz[3 * t + 1], d2 = q2 - cs.sxyz[3 * t + 2];
        dd = (d0 * d0 + d1 * d1) + d2 * d2;
        pass = dd < r2;
      }
      fn(t, dd, pass);
    }
  }
}

__device__ __forceinline__ void nn_write(const CellSet& cs, int64_t j, const double* s_d, const uint32_t* s_i,
                                         int found, int max_nn, int lane, int32_t* out_idx, double* out_d2,
                                         int32_t* out_cnt) {
  const int64_t i = cs.sidx[j];
  const int cnt = min(found, max_nn);
  for (int k = lane; k < cnt; k += 64) {
    out_idx[i * max_nn + k] = static_cast<int32_t>(s_i[k]);
    out_d2[i * max_nn + k] = s_d[k];
  }
  if (lane == 0) out_cnt[i] = cnt;
}

// SearchHybrid(p, radius, max_nn) of every point: one one-wave workgroup per
// query (sorted order); in-radius candidates compacted into LDS by ballots,
// sorted, the first max_nn written -> out_idx / out_d2 [n][max_nn], out_cnt[n].
// More than kNnCap candidates: the query goes to ovf (k_radius_nn_select).
__global__ __launch_bounds__(64) void k_radius_nn(CellSet cs, double r2, int max_nn, int32_t* out_idx, double* out_d2,
                                                  int32_t* out_cnt, uint32_t* ovf, unsigned* n_ovf) {
  __shared__ double s_d[kNnCap];
  __shared__ uint32_t s_i[kNnCap];
  const int64_t j = blockIdx.x;
  const int lane = threadIdx.x;
  int found = 0;
  nn_scan(cs, j, r2, lane, [&](int64_t t, double dd, bool pass) {
    const unsigned long long bal = __ballot(pass);
    const int rank = __popcll(bal & ((1ull << lane) - 1ull));
    if (pass && found + rank < kNnCap) {
      s_d[found + rank] = dd;
      s_i[found + rank] = cs.sidx[t];
    }
    found += __popcll(bal);
  });
  if (found > kNnCap) {
    if (lane == 0) {
      const unsigned k = atomicAdd(n_ovf, 1u);
      ovf[k] = static_cast<uint32_t>(j);
    }
    return;
  }
  int P = 64;
  while (P < found) P <<= 1;
  for (int k = found + lane; k < P; k += 64) {
    s_d[k] = INFINITY;
    s_i[k] = 0xffffffffu;
  }
  __syncthreads();
  nn_sort(s_d, s_i, P, lane);
  nn_write(cs, j, s_d, s_i, found, max_nn, lane, out_idx, out_d2, out_cnt);
}

// A query with more than kNnCap candidates (max_nn <= kNnMax <= that): the
// max_nn-th smallest d2 K by a radix select over its bit pattern (d2 >= 0:
// ordered as an integer), then among the ties d2 == K the smallest indices;
// those max_nn entries sorted and written as k_radius_nn does.
__global__ __launch_bounds__(64) void k_radius_nn_select(CellSet cs, double r2, int max_nn, const uint32_t* ovf,
                                                         int32_t* out_idx, double* out_d2, int32_t* out_cnt) {
  __shared__ double s_d[kNnMax];
  __shared__ uint32_t s_i[kNnMax];
  const int64_t j = ovf[blockIdx.x];
  const int lane = threadIdx.x;
  auto count = [&](auto pred) {
    int c = 0;
    nn_scan(cs, j, r2, lane, [&](int64_t t, double dd, bool pass) {
      const bool ok = pass && pred(static_cast<uint64_t>(__double_as_longlong(dd)), cs.sidx[t]);
      c += __popcll(__ballot(ok));
    });
    return c;
  };
  uint64_t K = 0;
  for (int b = 62; b >= 0; --b) {
    const uint64_t cand = K | (1ull << b);
    if (count([&](uint64_t key, uint32_t) { return key < cand; }) < max_nn) K = cand;
  }
  const int need = max_nn - count([&](uint64_t key, uint32_t) { return key < K; });
  uint32_t U = 0;
  for (int b = 31; b >= 0; --b) {
    const uint32_t cand = U | (1u << b);
    if (count([&](uint64_t key, uint32_t id) { return key == K && id < cand; }) < need) U = cand;
  }
  int found = 0;
  nn_scan(cs, j, r2, lane, [&](int64_t t, double dd, bool pass) {
    const uint64_t key = static_cast<uint64_t>(__double_as_longlong(dd));
    const bool ok = pass && (key < K || (key == K && cs.sidx[t] <= U));
    const unsigned long long bal = __ballot(ok);
    const int rank = __popcll(bal & ((1ull << lane) - 1ull));
    if (ok && found + rank < kNnMax) {
      s_d[found + rank] = dd;
      s_i[found + rank] = cs.sidx[t];
    }
    found += __popcll(bal);
  });
  found = min(found, kNnMax);
  int P = 64;
  while (P < found) P <<= 1;
  for (int k = found + lane; k < P; k += 64) {
    s_d[k] = INFINITY;
    s_i[k] = 0xffffffffu;
  }
  __syncthreads();
  nn_sort(s_d, s_i, P, lane);
  nn_write(cs, j, s_d, s_i, found, max_nn, lane, out_idx, out_d2, out_cnt);
}

// ComputeSPFHFeature: one point per lane; its histogram in LDS (one column per lane)
__global__ __launch_bounds__(64) void k_spfh(const double* xyz, const double* nrm, int64_t n, const int32_t* nidx,
                                             const int32_t* ncnt, int max_nn, double* spfh) {
  __shared__ double s_h[33][64];
  const int lane = threadIdx.x;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 64 + lane;
  for (int b = 0; b < 33; ++b) s_h[b][lane] = 0.0;
  if (i >= n) return;
  const int cnt = ncnt[i];
  if (cnt > 1) {
    const double incr = 100.0 / static_cast<double>(cnt - 1);
    const reg::D3 p1 = reg::ld3(xyz, i), n1 = reg::ld3(nrm, i);
    for (int k = 1; k < cnt; ++k) {
      const int64_t o = nidx[i * max_nn + k];
      double f0, f1, f2;
      reg::pair_features(p1, n1, reg::ld3(xyz, o), reg::ld3(nrm, o), &f0, &f1, &f2);
      s_h[reg::bin11(11.0 * (f0 + reg::kPi) / (2.0 * reg::kPi))][lane] += incr;
      s_h[11 + reg::bin11(11.0 * (f1 + 1.0) * 0.5)][lane] += incr;
      s_h[22 + reg::bin11(11.0 * (f2 + 1.0) * 0.5)][lane] += incr;
    }
  }
  for (int b = 0; b < 33; ++b) spfh[33 * i + b] = s_h[b][lane];
}

// ComputeFPFHFeature's second pass: sum over the neighbours (the point itself
// and d2 == 0 skipped) of spfh[k] / d2, each third scaled to 100, + spfh[i]
__global__ __launch_bounds__(64) void k_fpfh(const double* spfh, int64_t n, const int32_t* nidx, const double* nd2,
                                             const int32_t* ncnt, int max_nn, double* out) {
  __shared__ double s_a[33][64];
  const int lane = threadIdx.x;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 64 + lane;
  for (int b = 0; b < 33; ++b) s_a[b][lane] = 0.0;
  if (i >= n) return;
  const int cnt = ncnt[i];
  if (cnt <= 1) {
    for (int b = 0; b < 33; ++b) out[33 * i + b] = 0.0;
    return;
  }
  double s[3] = {0.0, 0.0, 0.0};
  for (int k = 1; k < cnt; ++k) {
    const double dist = nd2[i * max_nn + k];
    if (dist == 0.0) continue;
    const double* r = spfh + 33 * static_cast<int64_t>(nidx[i * max_nn + k]);
    for (int b = 0; b < 33; ++b) {
      const double val = r[b] / dist;
      s[b / 11] += val;
      s_a[b][lane] += val;
    }
  }
  for (int t = 0; t < 3; ++t)
    if (s[t] != 0.0) s[t] = 100.0 / s[t];
  for (int b = 0; b < 33; ++b) out[33 * i + b] = s_a[b][lane] * s[b / 11] + spfh[33 * i + b];
}

// Nearest row of B for every row of A (33-D, nanoflann's L2_Adaptor order:
// four dimensions at a time, then the 33rd; ties to the lower index).  B in
// LDS tiles of 64 rows; one query per thread.
constexpr int kFnTile = 64;
constexpr int kFeatDim = 33;
// Nearest row of B (L2 over 33 dims, nanoflann's accumulation order: four
// squared differences summed per group, the groups added in turn, then the
// last dimension; ties keep the lower index) for each row i of A, over the
// rows [lo, hi) of B; -> (distance, index) of the best (index -1: none).
__device__ __forceinline__ void feature_nn_range(const double* A, int64_t na, const double* B, int64_t lo,
                                                 int64_t hi, double* s_b, double* best_out, int64_t* bi_out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  double a[kFeatDim];
#pragma unroll
  for (int d = 0; d < kFeatDim; ++d) a[d] = i < na ? A[kFeatDim * i + d] : 0.0;
  double best = INFINITY;
  int64_t bi = -1;
  for (int64_t t0 = lo; t0 < hi; t0 += kFnTile) {
    __syncthreads();
    const int rows = static_cast<int>(min<int64_t>(kFnTile, hi - t0));
    for (int k = threadIdx.x; k < rows * kFeatDim; k += kT) s_b[k] = B[kFeatDim * t0 + k];
    __syncthreads();
    if (i < na) {
      for (int r = 0; r < rows; ++r) {
        const double* b = s_b + r * kFeatDim;
        double res = 0.0;
#pragma unroll
        for (int g = 0; g < 8; ++g) {
          const double d0 = a[4 * g] - b[4 * g], d1 = a[4 * g + 1] - b[4 * g + 1];
          const double d2 = a[4 * g + 2] - b[4 * g + 2], d3 = a[4 * g + 3] - b[4 * g + 3];
          res += ((d0 * d0 + d1 * d1) + d2 * d2) + d3 * d3;
        }
        const double d32 = a[32] - b[32];
        res += d32 * d32;
        if (res < best) {
          best = res;
          bi = t0 + r;
        }
      }
    }
  }
  *best_out = best;
  *bi_out = bi;
}

__global__ __launch_bounds__(kT) void k_feature_nn(const double* A, int64_t na, const double* B, int64_t nb,
                                                   int32_t* out) {
  __shared__ double s_b[kFnTile * kFeatDim];
  double best;
  int64_t bi;
  feature_nn_range(A, na, B, 0, nb, s_b, &best, &bi);
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i < na) out[i] = static_cast<int32_t>(bi);
}

// The same over B split into gridDim.y ranges of `per` rows (one query block
// per CU was a twentieth of the chip), each range's best to (pd, pi)[y][i]...
__global__ __launch_bounds__(kT) void k_feature_nn_part(const double* A, int64_t na, const double* B, int64_t nb,
                                                        int64_t per, double* pd, int32_t* pi) {
  __shared__ double s_b[kFnTile * kFeatDim];
  const int64_t lo = static_cast<int64_t>(blockIdx.y) * per;
  double best;
  int64_t bi;
  feature_nn_range(A, na, B, lo, min<int64_t>(nb, lo + per), s_b, &best, &bi);
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i < na) {
    pd[blockIdx.y * na + i] = best;
    pi[blockIdx.y * na + i] = static_cast<int32_t>(bi);
  }
}

// ... then folded in range order: a strictly smaller distance wins, so ties
// keep the lower index, as the one sequential scan does.
__global__ __launch_bounds__(kT) void k_feature_nn_fold(const double* pd, const int32_t* pi, int64_t na, int S,
                                                        int32_t* out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (i >= na) return;
  double best = INFINITY;
  int32_t bi = -1;
  for (int y = 0; y < S; ++y) {
    const double d = pd[y * na + i];
    if (d < best) {
      best = d;
      bi = pi[y * na + i];
    }
  }
  out[i] = bi;
}

// Launch: B split so that the grid has ~2048 workgroups (ranges of whole
// 64-row tiles); scratch from the context's pool.
int feature_nn_run(sl_ctx* c, const double* a, int64_t na, const double* b, int64_t nb, int32_t* out,
                   hipStream_t s) {
  const int64_t qb = blocks(na);
  const int64_t tiles = (nb + kFnTile - 1) / kFnTile;
  int64_t S = std::min<int64_t>(256, std::max<int64_t>(1, std::min<int64_t>((2048 + qb - 1) / qb, tiles)));
  if (S <= 1) {
    hipLaunchKernelGGL(k_feature_nn, dim3(qb), dim3(kT), 0, s, a, na, b, nb, out);
    MTRY(c, hipGetLastError());
    return SL_OK;
  }
  const int64_t per = (tiles + S - 1) / S * kFnTile;
  S = (nb + per - 1) / per;
  DBuf<double> pd;
  DBuf<int32_t> pi;
  MTRY(c, pd.alloc(S * na));
  MTRY(c, pi.alloc(S * na));
  hipLaunchKernelGGL(k_feature_nn_part, dim3(qb, S), dim3(kT), 0, s, a, na, b, nb, per, pd.p, pi.p);
  hipLaunchKernelGGL(k_feature_nn_fold, dim3(qb), dim3(kT), 0, s, pd.p, pi.p, na, static_cast<int>(S), out);
  MTRY(c, hipGetLastError());
  MTRY(c, hipStreamSynchronize(s));  // (before the scratch goes back to the pool)
  return SL_OK;
}

// ---- RANSAC ----
struct RegIn {
  const double* src;
  const double* tgt;
  int64_t ns, nt;
  const int32_t* corres;  // [nc][2] (source, target)
  int64_t nc;
  uint64_t seed;
  double edge_sim, max_dist;
};

// One hypothesis per thread, iterations it0 .. it0 + count - 1: draw three
// correspondences, CorrespondenceCheckerBasedOnEdgeLength (no transformation
// needed: checked first), Umeyama, CorrespondenceCheckerBasedOnDistance ->
// flag (0: edge check failed, 1: distance check failed, 2: passed) and T.
__global__ __launch_bounds__(kT) void k_reg_hyp(RegIn in, int64_t it0, int64_t count, uint8_t* flag, double* Tout) {
  const int64_t h = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (h >= count) return;
  const uint64_t it = static_cast<uint64_t>(it0 + h);
  reg::D3 s[3], t[3];
  for (int k = 0; k < 3; ++k) {
    const int64_t c = reg::draw(in.seed, 3 * it + k, static_cast<uint64_t>(in.nc));
    s[k] = reg::ld3(in.src, in.corres[2 * c]);
    t[k] = reg::ld3(in.tgt, in.corres[2 * c + 1]);
  }
  uint8_t f = 2;
  for (int a = 0; a < 3 && f == 2; ++a)
    for (int b = a + 1; b < 3; ++b) {
      const double ds = reg::norm3({s[a].x - s[b].x, s[a].y - s[b].y, s[a].z - s[b].z});
      const double dt = reg::norm3({t[a].x - t[b].x, t[a].y - t[b].y, t[a].z - t[b].z});
      if (ds < dt * in.edge_sim || dt < ds * in.edge_sim) {
        f = 0;
        break;
      }
    }
  double T[12];
  for (int k = 0; k < 12; ++k) T[k] = (k % 5 == 0) ? 1.0 : 0.0;
  if (f == 2) {
    reg::umeyama3(s, t, T);
    for (int k = 0; k < 3; ++k) {
      const reg::D3 q = reg::tp(T, s[k]);
      if (reg::norm3({t[k].x - q.x, t[k].y - q.y, t[k].z - q.z}) > in.max_dist) {
        f = 1;
        break;
      }
    }
  }
  flag[h] = f;
  for (int k = 0; k < 12; ++k) Tout[12 * h + k] = T[k];
}

// The nearest target point (cell grid, d2 < r2; least (d2, index)) of the
// point q -> its index (-1: none), *d2.
__device__ __forceinline__ int64_t grid_nn(double q0, double q1, double q2, const Grid& g, const int32_t* dense,
                                           const uint64_t* ukeys, int64_t m, const uint32_t* ustart, int64_t nt,
                                           const double* sxyz, const uint32_t* sidx, double r2, double* d2out) {
  double bd = INFINITY;
  int64_t bi = -1;
  const double f0 = floor((q0 - g.lo0) / g.h), f1 = floor((q1 - g.lo1) / g.h), f2 = floor((q2 - g.lo2) / g.h);
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
  *d2out = bi >= 0 ? bd : 0.0;
  return bi;
}

struct TgtGrid {
  Grid g;
  const int32_t* dense;
  const uint64_t* ukeys;
  int64_t m;
  const uint32_t* ustart;
  const double* sxyz;
  const uint32_t* sidx;
};

// GetRegistrationResultAndCorrespondences for hypotheses hyp[0..P): grid
// (source points / 256, P); every moved source point's nearest target within
// max_dist -> e2 / ok [P][ns]
__global__ __launch_bounds__(kT) void k_reg_validate(RegIn in, TgtGrid tg, const int32_t* hyp, const double* Tall,
                                                     double* e2, uint8_t* ok) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  const int p = blockIdx.y;
  if (i >= in.ns) return;
  const double* T = Tall + 12 * static_cast<int64_t>(hyp[p]);
  const reg::D3 q = reg::tp(T, reg::ld3(in.src, i));
  double d2;
  const int64_t bi = grid_nn(q.x, q.y, q.z, tg.g, tg.dense, tg.ukeys, tg.m, tg.ustart, in.nt, tg.sxyz, tg.sidx,
                             in.max_dist * in.max_dist, &d2);
  e2[p * in.ns + i] = d2;
  ok[p * in.ns + i] = bi >= 0 ? 1 : 0;
}

constexpr int kRegBlock = 64;  // source points per partial sum (the oracle's REG_BLOCK)

// per (hypothesis, 64-point block): the block's squared distances summed in
// point order (+0.0 for points without a neighbour) and its inliers
__global__ __launch_bounds__(kT) void k_reg_fold(const double* e2, const uint8_t* ok, int64_t ns, int64_t nb, int P,
                                                 double* part, int32_t* pcnt) {
  const int64_t t = static_cast<int64_t>(blockIdx.x) * kT + threadIdx.x;
  if (t >= nb * P) return;
  const int64_t p = t / nb, b = t - p * nb;
  const int64_t i0 = b * kRegBlock, i1 = min<int64_t>(i0 + kRegBlock, ns);
  double s = 0.0;
  int c = 0;
  for (int64_t i = i0; i < i1; ++i) {
    s = s + e2[p * ns + i];
    c += ok[p * ns + i];
  }
  part[t] = s;
  pcnt[t] = c;
}

// per hypothesis: the blocks left to right -> (inliers, sum d2); and
// EvaluateInlierCorrespondenceRatio's count: correspondences whose moved
// source point lies within max_dist (strict d2 < max_dist^2) of its target
__global__ __launch_bounds__(kT) void k_reg_final(RegIn in, const int32_t* hyp, const double* Tall, const double* part,
                                                  const int32_t* pcnt, int64_t nb, int64_t* cnt_out, double* err_out,
                                                  int64_t* inl_out) {
  __shared__ int s_red[kT];
  const int p = blockIdx.x;
  const double* T = Tall + 12 * static_cast<int64_t>(hyp[p]);
  const double thr2 = in.max_dist * in.max_dist;
  int c = 0;
  for (int64_t k = threadIdx.x; k < in.nc; k += kT) {
    const reg::D3 q = reg::tp(T, reg::ld3(in.src, in.corres[2 * k]));
    const reg::D3 t = reg::ld3(in.tgt, in.corres[2 * k + 1]);
    const double dx = q.x - t.x, dy = q.y - t.y, dz = q.z - t.z;
    if ((dx * dx + dy * dy) + dz * dz < thr2) ++c;
  }
  s_red[threadIdx.x] = c;
  __syncthreads();
  if (threadIdx.x == 0) {
    int64_t inl = 0;
    for (int k = 0; k < kT; ++k) inl += s_red[k];
    double e = 0.0;
    int64_t n = 0;
    for (int64_t b = 0; b < nb; ++b) {
      e = e + part[p * nb + b];
      n += pcnt[p * nb + b];
    }
    cnt_out[p] = n;
    err_out[p] = e;
    inl_out[p] = inl;
  }
}

// radius neighbour lists of every point (device) -> idx / d2 [n][max_nn], cnt [n]
int radius_lists(sl_ctx* c, const double* xyz, int64_t n, double radius, int max_nn, int32_t* idx_out,
                 double* d2_out, int32_t* cnt_out, hipStream_t s) {
  const double r2 = radius * radius;
  radius = fabs(radius);
  if (!(r2 > 0.0)) {  // nothing has d2 < 0
    MTRY(c, hipMemsetAsync(cnt_out, 0, sizeof(int32_t) * n, s));
    MTRY(c, hipStreamSynchronize(s));
    return SL_OK;
  }
  double b[6];
  int r = bounds(c, xyz, n, b, s);
  if (r) return r;
  double emax = 0.0;
  for (int k = 0; k < 3; ++k) emax = std::max(emax, b[3 + k] - b[k]);
  if (!std::isfinite(emax)) return slgpu_fail(c, SL_EINVAL, "non-finite point coordinates");
  Grid g;
  if (!make_grid(b, b + 3, std::max(radius, emax / 1.0e6), &g))
    return slgpu_fail(c, SL_EINVAL, "radius-search grid is too large");
  DBuf<uint64_t> keys, ukeys;
  DBuf<uint32_t> sidx, ustart, ovf, novf;
  int64_t m = 0;
  r = cells(c, xyz, n, g, keys, sidx, ukeys, ustart, &m, s);
  if (r) return r;
  DBuf<double> sxyz;
  DBuf<int32_t> nbr;
  MTRY(c, sxyz.alloc(3 * n));
  MTRY(c, nbr.alloc(27 * m));
  MTRY(c, ovf.alloc(n));
  MTRY(c, novf.alloc(1));
  MTRY(c, hipMemsetAsync(novf.p, 0, sizeof(uint32_t), s));
  hipLaunchKernelGGL(k_gather_sorted, dim3(blocks(n)), dim3(kT), 0, s, xyz, sidx.p, n, sxyz.p);
  hipLaunchKernelGGL(k_cell_neighbours_lin, dim3(blocks(m)), dim3(kT), 0, s, ukeys.p, m, g.nx, g.ny, g.nz, nbr.p);
  const CellSet cs{sxyz.p, sidx.p, keys.p, n, ukeys.p, ustart.p, m, nbr.p};
  hipLaunchKernelGGL(k_radius_nn, dim3(static_cast<unsigned>(n)), dim3(64), 0, s, cs, r2, max_nn, idx_out, d2_out,
                     cnt_out, ovf.p, novf.p);
  MTRY(c, hipGetLastError());
  uint32_t no = 0;
  MTRY(c, hipMemcpyAsync(&no, novf.p, sizeof(no), hipMemcpyDeviceToHost, s));
  MTRY(c, hipStreamSynchronize(s));
  if (no) {
    hipLaunchKernelGGL(k_radius_nn_select, dim3(no), dim3(64), 0, s, cs, r2, max_nn, ovf.p, idx_out, d2_out, cnt_out);
    MTRY(c, hipGetLastError());
  }
  MTRY(c, hipStreamSynchronize(s));
  return SL_OK;
}

}  // namespace

extern "C" {

int sl_radius_search(sl_ctx* c, const double* xyz, int64_t n, double radius, int max_nn, int32_t* out_idx,
                     double* out_d2, int32_t* out_cnt, void* stream) {
  if (!c) return SL_EINVAL;
  if (n < 0 || (n && (!xyz || !out_idx || !out_d2 || !out_cnt)))
    return slgpu_fail(c, SL_EINVAL, "sl_radius_search: bad size or NULL arguments");
  if (max_nn < 1 || max_nn > kNnMax) return slgpu_fail(c, SL_EINVAL, "max_nn must be in [1, 1024]");
  if (std::isnan(radius)) return slgpu_fail(c, SL_EINVAL, "radius is NaN");
  if (n >= (1ll << 31)) return slgpu_fail(c, SL_EINVAL, "at most 2^31 - 1 points");
  if (n == 0) return SL_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  PoolStream pool_stream(s);
  MTRY(c, hipSetDevice(slgpu_device(c)));
  return radius_lists(c, xyz, n, radius, max_nn, out_idx, out_d2, out_cnt, s);
}

int sl_compute_fpfh(sl_ctx* c, const double* xyz, const double* normals, int64_t n, double radius, int max_nn,
                    double* feature, void* stream) {
  if (!c) return SL_EINVAL;
  if (n < 0 || (n && (!xyz || !normals || !feature)))
    return slgpu_fail(c, SL_EINVAL, "sl_compute_fpfh: bad size or NULL arguments");
  if (max_nn < 1 || max_nn > kNnMax) return slgpu_fail(c, SL_EINVAL, "max_nn must be in [1, 1024]");
  if (std::isnan(radius)) return slgpu_fail(c, SL_EINVAL, "radius is NaN");
  if (n >= (1ll << 31)) return slgpu_fail(c, SL_EINVAL, "at most 2^31 - 1 points");
  if (n == 0) return SL_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  PoolStream pool_stream(s);
  MTRY(c, hipSetDevice(slgpu_device(c)));
  DBuf<int32_t> nidx, ncnt;
  DBuf<double> nd2, spfh;
  MTRY(c, nidx.alloc(n * max_nn));
  MTRY(c, nd2.alloc(n * max_nn));
  MTRY(c, ncnt.alloc(n));
  MTRY(c, spfh.alloc(33 * n));
  int r = radius_lists(c, xyz, n, radius, max_nn, nidx.p, nd2.p, ncnt.p, s);
  if (r) return r;
  const unsigned g64 = static_cast<unsigned>((n + 63) / 64);
  hipLaunchKernelGGL(k_spfh, dim3(g64), dim3(64), 0, s, xyz, normals, n, nidx.p, ncnt.p, max_nn, spfh.p);
  hipLaunchKernelGGL(k_fpfh, dim3(g64), dim3(64), 0, s, spfh.p, n, nidx.p, nd2.p, ncnt.p, max_nn, feature);
  MTRY(c, hipGetLastError());
  MTRY(c, hipStreamSynchronize(s));
  return SL_OK;
}

int sl_feature_nn(sl_ctx* c, const double* a, int64_t na, const double* b, int64_t nb, int dim, int32_t* out,
                  void* stream) {
  if (!c) return SL_EINVAL;
  if (dim != kFeatDim) return slgpu_fail(c, SL_EINVAL, "sl_feature_nn: only 33-dimensional (FPFH) features");
  if (na < 0 || nb < 0 || (na && (!a || !out)) || (na && nb && !b))
    return slgpu_fail(c, SL_EINVAL, "sl_feature_nn: bad sizes or NULL arguments");
  if (na >= (1ll << 31) || nb >= (1ll << 31)) return slgpu_fail(c, SL_EINVAL, "at most 2^31 - 1 rows");
  if (na == 0) return SL_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  PoolStream pool_stream(s);
  MTRY(c, hipSetDevice(slgpu_device(c)));
  const int r = feature_nn_run(c, a, na, b, nb, out, s);
  if (r) return r;
  MTRY(c, hipStreamSynchronize(s));
  return SL_OK;
}

int sl_ransac_feature_matching(sl_ctx* c, const double* source, int64_t ns, const double* target, int64_t nt,
                               const double* source_feature, const double* target_feature, int mutual_filter,
                               double max_distance, double edge_similarity, int max_iteration, double confidence,
                               uint64_t seed, double* transformation, double* fitness, double* inlier_rmse,
                               int* iterations, int* validations, int64_t* n_corres, void* stream) {
  if (!c) return SL_EINVAL;
  if (ns < 0 || nt < 0 || !transformation || (ns && (!source || !source_feature)) ||
      (nt && (!target || !target_feature)))
    return slgpu_fail(c, SL_EINVAL, "sl_ransac_feature_matching: bad sizes or NULL arguments");
  if (ns >= (1ll << 31) || nt >= (1ll << 31)) return slgpu_fail(c, SL_EINVAL, "at most 2^31 - 1 points");
  double best_T[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
  double best_fit = 0.0, best_rmse = 0.0;
  int it = 0, vals = 0;
  int64_t nc = 0;
  auto finish = [&]() {
    memcpy(transformation, best_T, sizeof(best_T));
    if (fitness) *fitness = best_fit;
    if (inlier_rmse) *inlier_rmse = best_rmse;
    if (iterations) *iterations = it;
    if (validations) *validations = vals;
    if (n_corres) *n_corres = nc;
    return SL_OK;
  };
  if (ns == 0 || nt == 0) return finish();
  hipStream_t s = static_cast<hipStream_t>(stream);
  PoolStream pool_stream(s);
  MTRY(c, hipSetDevice(slgpu_device(c)));
  // CorrespondencesFromFeatures (mutual filter; fewer than 0.1f * ns mutual
  // pairs: the one-way set)
  DBuf<int32_t> ij, ji, dcor;
  MTRY(c, ij.alloc(ns));
  MTRY(c, ji.alloc(nt));
  {
    // (both directions in one pass over the pairs -- d(a, b) and d(b, a) are
    // the same bits -- with a wave reduction per target row for the column
    // bests measured no faster: RANSAC 8.55 vs 8.6 ms, 12.7 vs 12.6 ms)
    int r0 = feature_nn_run(c, source_feature, ns, target_feature, nt, ij.p, s);
    if (!r0 && mutual_filter) r0 = feature_nn_run(c, target_feature, nt, source_feature, ns, ji.p, s);
    if (r0) return r0;
  }
  std::vector<int32_t> hij(static_cast<size_t>(ns)), hji(static_cast<size_t>(mutual_filter ? nt : 0));
  MTRY(c, hipMemcpyAsync(hij.data(), ij.p, sizeof(int32_t) * ns, hipMemcpyDeviceToHost, s));
  if (mutual_filter) MTRY(c, hipMemcpyAsync(hji.data(), ji.p, sizeof(int32_t) * nt, hipMemcpyDeviceToHost, s));
  MTRY(c, hipStreamSynchronize(s));
  // (a row without a nearest neighbour -- NaN features -- makes no pair)
  std::vector<int32_t> cor;
  if (mutual_filter) {
    for (int64_t i = 0; i < ns; ++i)
      if (hij[i] >= 0 && hji[hij[i]] == i) {
        cor.push_back(static_cast<int32_t>(i));
        cor.push_back(hij[i]);
      }
  }
  if (!mutual_filter || static_cast<int64_t>(cor.size() / 2) < static_cast<int64_t>(0.1f * static_cast<float>(ns))) {
    cor.clear();
    for (int64_t i = 0; i < ns; ++i)
      if (hij[i] >= 0) {
        cor.push_back(static_cast<int32_t>(i));
        cor.push_back(hij[i]);
      }
  }
  nc = static_cast<int64_t>(cor.size() / 2);
  if (nc < 3 || !(max_distance > 0.0)) return finish();
  MTRY(c, dcor.alloc(2 * nc));
  MTRY(c, hipMemcpyAsync(dcor.p, cor.data(), sizeof(int32_t) * 2 * nc, hipMemcpyHostToDevice, s));
  // the target's cell grid (cells of edge >= max_distance)
  double bnd[6];
  int r = bounds(c, target, nt, bnd, s);
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
  r = cells(c, target, nt, g, keys, idx, ukeys, ustart, &m, s);
  if (r) return r;
  DBuf<double> sxyz;
  DBuf<int32_t> dense;
  MTRY(c, sxyz.alloc(3 * nt));
  hipLaunchKernelGGL(k_gather_sorted, dim3(blocks(nt)), dim3(kT), 0, s, target, idx.p, nt, sxyz.p);
  MTRY(c, hipGetLastError());
  const int64_t ncell = (g.nx * g.ny) * g.nz;
  if (ncell <= (int64_t{1} << 26)) {
    MTRY(c, dense.alloc(ncell));
    MTRY(c, hipMemsetAsync(dense.p, 0xff, sizeof(int32_t) * ncell, s));
    hipLaunchKernelGGL(k_icp_dense, dim3(blocks(m)), dim3(kT), 0, s, ukeys.p, m, dense.p);
    MTRY(c, hipGetLastError());
  }
  const TgtGrid tg{g, dense.p, ukeys.p, m, ustart.p, sxyz.p, idx.p};
  const RegIn in{source, target, ns, nt, dcor.p, nc, seed, edge_similarity, max_distance};
  // hypotheses in batches; validations in chunks of at most kVal (and
  // kVal * ns <= 2^25 scratch entries), walked in iteration order
  constexpr int64_t kBatch = 4096;
  const int kVal = static_cast<int>(std::max<int64_t>(1, std::min<int64_t>(256, (int64_t{1} << 25) / ns)));
  const int64_t nb = (ns + kRegBlock - 1) / kRegBlock;
  DBuf<uint8_t> flag, ok;
  DBuf<double> Tall, e2, part, err;
  DBuf<int32_t> hyp, pcnt;
  DBuf<int64_t> cnt, inl;
  MTRY(c, flag.alloc(kBatch));
  MTRY(c, Tall.alloc(12 * kBatch));
  MTRY(c, hyp.alloc(kVal));
  MTRY(c, e2.alloc(kVal * ns));
  MTRY(c, ok.alloc(kVal * ns));
  MTRY(c, part.alloc(kVal * nb));
  MTRY(c, pcnt.alloc(kVal * nb));
  MTRY(c, cnt.alloc(kVal));
  MTRY(c, err.alloc(kVal));
  MTRY(c, inl.alloc(kVal));
  std::vector<uint8_t> hflag(kBatch);
  std::vector<double> hT(12 * kBatch), herr(kVal);
  std::vector<int64_t> hcnt(kVal), hinl(kVal);
  int64_t est_k = max_iteration;
  const double log_conf = std::log(1.0 - confidence);
  bool done = false;
  while (!done && it < std::min<int64_t>(max_iteration, est_k)) {
    const int64_t it0 = it;
    const int64_t count = std::min<int64_t>(kBatch, std::min<int64_t>(max_iteration, est_k) - it0);
    hipLaunchKernelGGL(k_reg_hyp, dim3(blocks(count)), dim3(kT), 0, s, in, it0, count, flag.p, Tall.p);
    MTRY(c, hipGetLastError());
    MTRY(c, hipMemcpyAsync(hflag.data(), flag.p, count, hipMemcpyDeviceToHost, s));
    MTRY(c, hipMemcpyAsync(hT.data(), Tall.p, sizeof(double) * 12 * count, hipMemcpyDeviceToHost, s));
    MTRY(c, hipStreamSynchronize(s));
    int64_t h = 0;  // next hypothesis of the batch to walk
    while (h < count && !done) {
      // the next chunk of passing hypotheses (in iteration order)
      std::vector<int32_t> pass;
      int64_t e = h;
      for (; e < count && static_cast<int>(pass.size()) < kVal; ++e)
        if (hflag[e] == 2) pass.push_back(static_cast<int32_t>(e));
      const int P = static_cast<int>(pass.size());
      if (P) {
        MTRY(c, hipMemcpyAsync(hyp.p, pass.data(), sizeof(int32_t) * P, hipMemcpyHostToDevice, s));
        hipLaunchKernelGGL(k_reg_validate, dim3(blocks(ns), P), dim3(kT), 0, s, in, tg, hyp.p, Tall.p, e2.p, ok.p);
        hipLaunchKernelGGL(k_reg_fold, dim3(blocks(nb * P)), dim3(kT), 0, s, e2.p, ok.p, ns, nb, P, part.p, pcnt.p);
        hipLaunchKernelGGL(k_reg_final, dim3(P), dim3(kT), 0, s, in, hyp.p, Tall.p, part.p, pcnt.p, nb, cnt.p,
                           err.p, inl.p);
        MTRY(c, hipGetLastError());
        MTRY(c, hipMemcpyAsync(hcnt.data(), cnt.p, sizeof(int64_t) * P, hipMemcpyDeviceToHost, s));
        MTRY(c, hipMemcpyAsync(herr.data(), err.p, sizeof(double) * P, hipMemcpyDeviceToHost, s));
        MTRY(c, hipMemcpyAsync(hinl.data(), inl.p, sizeof(int64_t) * P, hipMemcpyDeviceToHost, s));
        MTRY(c, hipStreamSynchronize(s));
      }
      // walk iterations h .. e - 1 in order, as Open3D's loop on one thread
      int q = 0;
      for (int64_t x = h; x < e; ++x) {
        if (it0 + x >= std::min<int64_t>(max_iteration, est_k)) {
          done = true;
          break;
        }
        it = static_cast<int>(it0 + x + 1);
        if (hflag[x] != 2) continue;
        const int k = q++;
        ++vals;
        const double fit = static_cast<double>(hcnt[k]) / static_cast<double>(ns);
        const double rmse = hcnt[k] ? std::sqrt(herr[k] / static_cast<double>(hcnt[k])) : 0.0;
        const double rmse_eff = hcnt[k] ? rmse : 0.0;
        if (fit > best_fit || (fit == best_fit && rmse_eff < best_rmse)) {
          best_fit = fit;
          best_rmse = rmse_eff;
          for (int a = 0; a < 12; ++a) best_T[a] = hT[12 * x + a];
          best_T[12] = best_T[13] = best_T[14] = 0.0;
          best_T[15] = 1.0;
          const double ratio = static_cast<double>(hinl[k]) / static_cast<double>(nc);
          const double y = 1.0 - std::pow(ratio, 3.0);
          double est_d;
          if (y <= 0.0) {
            est_d = 0.0;
          } else {
            const double den = std::log(y);
            est_d = den != 0.0 ? log_conf / den : INFINITY;
          }
          if (est_d < static_cast<double>(est_k)) est_k = static_cast<int64_t>(std::ceil(est_d));
        }
      }
      h = e;
    }
  }
  return finish();
}

}  // extern "C"
