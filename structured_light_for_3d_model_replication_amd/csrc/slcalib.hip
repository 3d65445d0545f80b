// libslgpu.so, part 3 -- calibration products: what
// SLSystem.calibrate_final (server/sl_system.py:329-415) derives from the stereo
// parameters (K1, K2, R, T) once OpenCV has estimated them, and saves to
// calib.mat for every later scan:
//
//   Nc [3][h*w]    unit camera ray of every pixel v*w + u (:353-365)
//                  r = ((u - cx)/fx, (v - cy)/fy, 1) / ||.||, the norm a
//                  sequential ((x^2 + y^2) + 1) sum (np.linalg.norm on axis 2)
//   wPlaneCol [4][Wp], wPlaneRow [4][Hp]   projector planes (:367-403):
//                  the rays of a projector column's (row's) two end pixels,
//                  rotated by R^T, crossed, normalised; d = -n . (-R^T T)
//
// Operation order: the reference's NumPy/OpenBLAS evaluation.  The 3-term
// products R^T @ p, np.dot and the 1-D np.linalg.norm (= sqrt(dot(x, x))) run in
// OpenBLAS kernels that accumulate left to right with fused multiply-adds --
// fma(a2, b2, fma(a1, b1, a0 * b0)) -- which is what the fixtures made from
// the reference itself pin (tests/golden/make_calib_golden.py); np.cross and the
// divisions are separate IEEE operations.  The rest compiles with
// -ffp-contract=off, so only the explicit fma() calls below are fused.
//
// One thread per pixel (rays: 24 B written per pixel, HBM-bound) and one per
// plane.  The calibration products are computed once per rig.
#include <hip/hip_runtime.h>

#include <math.h>
#include <stdint.h>

#include <algorithm>

#include "slgpu.h"

#pragma clang fp contract(off)

// from slgpu.hip
int slgpu_fail(sl_ctx* c, int code, const char* msg);
int slgpu_device(const sl_ctx* c);

namespace {

constexpr int kT = 256;

struct CalibParams {
  double fx, fy, cx, cy;       // K1 (camera)
  double fxp, fyp, cxp, cyp;   // K2 (projector)
  double rinv[9];              // R^T, row-major
  double T[3];
  int w, h, wp, hp;
};

// k_calib_rays: Nc, sl_system.py:353-365.  Pixel i = v*w + u (the row-major
// reshape(-1, 3).T of the (h, w, 3) ray image).
__global__ __launch_bounds__(kT) void k_calib_rays(CalibParams p, double* __restrict__ nc) {
  const int64_t hw = static_cast<int64_t>(p.w) * p.h;
  for (int64_t i = blockIdx.x * static_cast<int64_t>(kT) + threadIdx.x; i < hw;
       i += static_cast<int64_t>(gridDim.x) * kT) {
    const int v = static_cast<int>(i / p.w);
    const int u = static_cast<int>(i - static_cast<int64_t>(v) * p.w);
    const double x = (static_cast<double>(u) - p.cx) / p.fx;   // :357
    const double y = (static_cast<double>(v) - p.cy) / p.fy;   // :358
    const double n = sqrt((x * x + y * y) + 1.0 * 1.0);         // :363, add.reduce over axis 2
    nc[i] = x / n;                                              // :364
    nc[hw + i] = y / n;
    nc[2 * hw + i] = 1.0 / n;
  }
}

__device__ __forceinline__ double dot3(const double* a, const double* b) {  // OpenBLAS 3-term dot
  return fma(a[2], b[2], fma(a[1], b[1], a[0] * b[0]));
}

// k_calib_planes: get_plane_from_proj_line (sl_system.py:380-395) for every
// column c (is_col: pixels (c, 0) and (c, Hp)) and row r (pixels (0, r) and
// (Wp, r)); out layout [4][n] = wPlaneCol.T / wPlaneRow.T as saved (:408-409).
__global__ __launch_bounds__(kT) void k_calib_planes(CalibParams p, double* __restrict__ col,
                                                     double* __restrict__ row) {
  const int t = blockIdx.x * kT + threadIdx.x;
  if (t >= p.wp + p.hp) return;
  const bool is_col = t < p.wp;
  const int k = is_col ? t : t - p.wp;
  double p1[3], p2[3];
  if (is_col) {  // :382-384
    p1[0] = p2[0] = (static_cast<double>(k) - p.cxp) / p.fxp;
    p1[1] = (0.0 - p.cyp) / p.fyp;
    p2[1] = (static_cast<double>(p.hp) - p.cyp) / p.fyp;
  } else {       // :386-387
    p1[0] = (0.0 - p.cxp) / p.fxp;
    p2[0] = (static_cast<double>(p.wp) - p.cxp) / p.fxp;
    p1[1] = p2[1] = (static_cast<double>(k) - p.cyp) / p.fyp;
  }
  p1[2] = p2[2] = 1.0;
  double r1[3], r2[3], cp[3];
  for (int i = 0; i < 3; ++i) {  // r = R_inv @ p (:389-390); C_p_cam = -R_inv @ T (:377)
    r1[i] = dot3(p.rinv + 3 * i, p1);
    r2[i] = dot3(p.rinv + 3 * i, p2);
    const double m[3] = {-p.rinv[3 * i], -p.rinv[3 * i + 1], -p.rinv[3 * i + 2]};
    cp[i] = dot3(m, p.T);
  }
  double n[3];  // np.cross (:393): a1 b2 - a2 b1, a2 b0 - a0 b2, a0 b1 - a1 b0
  n[0] = r1[1] * r2[2] - r1[2] * r2[1];
  n[1] = r1[2] * r2[0] - r1[0] * r2[2];
  n[2] = r1[0] * r2[1] - r1[1] * r2[0];
  const double nn = sqrt(dot3(n, n));  // np.linalg.norm of a 1-D array = sqrt(dot(x, x)) (:394)
  n[0] /= nn;
  n[1] /= nn;
  n[2] /= nn;
  const double d = -dot3(n, cp);  // :395
  double* out = is_col ? col : row;
  const int m = is_col ? p.wp : p.hp;
  if (!out) return;
  out[k] = n[0];
  out[m + k] = n[1];
  out[2 * m + k] = n[2];
  out[3 * m + k] = d;
}

}  // namespace

extern "C" {

int sl_calib_products(sl_ctx* c, const double* cam_K, const double* proj_K, const double* R, const double* T,
                      int cam_w, int cam_h, int proj_w, int proj_h, double* nc_out, double* plane_col_out,
                      double* plane_row_out, void* stream) {
  if (!c) return SL_EINVAL;
  if (!cam_K || !proj_K || !R || !T) return slgpu_fail(c, SL_EINVAL, "cam_K, proj_K, R and T are required");
  if (cam_w < 1 || cam_h < 1 || proj_w < 1 || proj_h < 1)
    return slgpu_fail(c, SL_EINVAL, "camera and projector sizes must be positive");
  if (!nc_out && !plane_col_out && !plane_row_out) return slgpu_fail(c, SL_EINVAL, "nothing to compute");
  CalibParams p;
  p.fx = cam_K[0];
  p.fy = cam_K[4];
  p.cx = cam_K[2];
  p.cy = cam_K[5];
  p.fxp = proj_K[0];
  p.fyp = proj_K[4];
  p.cxp = proj_K[2];
  p.cyp = proj_K[5];
  for (int i = 0; i < 3; ++i)
    for (int j = 0; j < 3; ++j) p.rinv[3 * i + j] = R[3 * j + i];  // R.T (:376)
  for (int i = 0; i < 3; ++i) p.T[i] = T[i];
  p.w = cam_w;
  p.h = cam_h;
  p.wp = proj_w;
  p.hp = proj_h;
  hipStream_t s = static_cast<hipStream_t>(stream);
  hipError_t e = hipSetDevice(slgpu_device(c));
  if (e == hipSuccess && nc_out) {
    const int64_t hw = static_cast<int64_t>(cam_w) * cam_h;
    const int64_t blocks = std::min<int64_t>((hw + kT - 1) / kT, 65536);
    hipLaunchKernelGGL(k_calib_rays, dim3(static_cast<unsigned>(blocks)), dim3(kT), 0, s, p, nc_out);
    e = hipGetLastError();
  }
  if (e == hipSuccess && (plane_col_out || plane_row_out)) {
    const int n = proj_w + proj_h;
    hipLaunchKernelGGL(k_calib_planes, dim3(static_cast<unsigned>((n + kT - 1) / kT)), dim3(kT), 0, s, p,
                       plane_col_out, plane_row_out);
    e = hipGetLastError();
  }
  if (e != hipSuccess) return slgpu_fail(c, SL_EHIP, hipGetErrorString(e));
  return SL_OK;
}

}  // extern "C"
