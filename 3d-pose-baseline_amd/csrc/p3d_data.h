// p3d_data.h -- the H3.6M data pipeline on the GPU, float64 like the
// reference's numpy.  Byte-moving, HBM-bound kernels: no MFMA, coalesced 8/16-B accesses, one
// read of every input byte.
//
//   k_cam_points<MODE>  per point, for every camera c of a subject (camera record uniform per
//                       loop trip: scalar loads):
//       MODE 0  world -> camera      X = R (P - T)             src/cameras.py:55-72
//       MODE 1  camera -> world      P = R^T X + T             src/cameras.py:74-90
//       MODE 2  project (radial + tangential distortion)       src/cameras.py:13-53
//   k_root_center        poses - tile(poses[:, :3])            src/data_utils.py:474-494
//   k_normalize          (x[:, use] - mean[use]) / std[use]    src/data_utils.py:260-280
//   k_unnormalize        float32 scatter, * std + mean         src/data_utils.py:283-311
//   k_col_partial/final  np.mean / np.std over axis 0          src/data_utils.py:210-211
//
// Camera record (21 float64): R row-major (9), T (3), f (2), c (2), k (3), p (2).
//
// Rounding: every product and sum is rounded separately (no FMA contraction), in the order
// numpy evaluates the reference's expressions, so the transforms, the projection and the
// (un)normalisation reproduce the reference's float64 results bit for bit (pinned by
// tests/golden/reference_goldens_data.npz); r2**3 is the correctly rounded cube.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define P3D_CAM_DOUBLES 21

struct CamArgs {
  const double* P;       // MODE 0/2: [n, 3]; MODE 1: [C, n, 3] if in_cam_stride else [n, 3]
  int64_t in_cam_stride; // doubles between cameras' inputs (0: shared input)
  int64_t n;             // points
  const double* cams;    // [C, 21]
  int C;
  double* out;           // MODE 0/1: [C, n, 3]; MODE 2: projections [C, n, 2]
  double* depth;         // MODE 2 optional [C, n] (may be null), likewise radial, tan, r2
  double* radial;
  double* tan;
  double* r2;
};

// correctly rounded x^3 (double-double x^2, then one rounding of x^2 * x)
__device__ __forceinline__ double p3d_cube(double x) {
  const double hi = x * x;
  const double lo = __fma_rn(x, x, -hi);
  const double p = hi * x;
  const double e = __fma_rn(hi, x, -p) + lo * x;
  return p + e;
}

template <int MODE>
__global__ __launch_bounds__(256) void k_cam_points(CamArgs a) {
#pragma clang fp contract(off)
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= a.n) return;
  double px = 0, py = 0, pz = 0;
  if (a.in_cam_stride == 0) { px = a.P[3 * i]; py = a.P[3 * i + 1]; pz = a.P[3 * i + 2]; }
  for (int c = 0; c < a.C; ++c) {
    const double* cm = a.cams + (int64_t)c * P3D_CAM_DOUBLES;
    if (a.in_cam_stride) {
      const double* q = a.P + c * a.in_cam_stride;
      px = q[3 * i]; py = q[3 * i + 1]; pz = q[3 * i + 2];
    }
    if (MODE == 1) {
      // R^T . X + T: column r of R dotted with X, in the order (R0r x + R1r y) + R2r z
      double* o = a.out + ((int64_t)c * a.n + i) * 3;
#pragma unroll
      for (int r = 0; r < 3; ++r) o[r] = ((cm[r] * px + cm[3 + r] * py) + cm[6 + r] * pz) + cm[9 + r];
      continue;
    }
    const double dx = px - cm[9], dy = py - cm[10], dz = pz - cm[11];
    const double X = (cm[0] * dx + cm[1] * dy) + cm[2] * dz;
    const double Y = (cm[3] * dx + cm[4] * dy) + cm[5] * dz;
    const double Z = (cm[6] * dx + cm[7] * dy) + cm[8] * dz;
    const int64_t ci = (int64_t)c * a.n + i;
    if (MODE == 0) {
      double* o = a.out + ci * 3;
      o[0] = X; o[1] = Y; o[2] = Z;
      continue;
    }
    const double u = X / Z, v = Y / Z;
    const double r2 = u * u + v * v;
    const double r4 = r2 * r2, r6 = p3d_cube(r2);
    const double radial = 1.0 + ((cm[16] * r2 + cm[17] * r4) + cm[18] * r6);
    const double tan = cm[19] * v + cm[20] * u;
    const double s = radial + tan;
    const double du = u * s + cm[20] * r2;
    const double dv = v * s + cm[19] * r2;
    double2 pr;
    pr.x = cm[12] * du + cm[14];
    pr.y = cm[13] * dv + cm[15];
    *(double2*)(a.out + ci * 2) = pr;
    if (a.depth) a.depth[ci] = Z;
    if (a.radial) a.radial[ci] = radial;
    if (a.tan) a.tan[ci] = tan;
    if (a.r2) a.r2[ci] = r2;
  }
}

// out[f, e] = in[f, e] - in[f, e % 3]; root[f, 0..2] = in[f, 0..2]   (row width W = 3 J)
__global__ __launch_bounds__(256) void k_root_center(const double* __restrict__ in, int64_t F, int W,
                                                     double* __restrict__ out, double* __restrict__ root) {
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= F * W) return;
  const int64_t f = idx / W;
  const int e = (int)(idx - f * W);
  const double v = in[idx], r = in[f * W + e % 3];
  out[idx] = v - r;
  if (root && e < 3) root[f * 3 + e] = v;
}

// out[f, u] = (x[f, use[u]] - mean[use[u]]) / std[use[u]]   (f64 or rounded to f32)
template <bool F32>
__global__ __launch_bounds__(256) void k_normalize(const double* __restrict__ x, int64_t F, int D,
                                                   const double* __restrict__ mean, const double* __restrict__ stdv,
                                                   const int32_t* __restrict__ use, int U, void* __restrict__ out) {
#pragma clang fp contract(off)
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= F * U) return;
  const int64_t f = idx / U;
  const int d = use[idx - f * U];
  const double y = (x[f * D + d] - mean[d]) / stdv[d];
  if (F32) ((float*)out)[idx] = (float)y;
  else ((double*)out)[idx] = y;
}

// orig = float32 zeros [F, D]; orig[:, use] = normalized (rounded to float32);
// out = orig * std + mean in float64 (numpy: float32 * float64 -> float64, then + mean)
template <bool INF32>
__global__ __launch_bounds__(256) void k_unnormalize(const void* __restrict__ xn, int64_t F, int U,
                                                     const double* __restrict__ mean, const double* __restrict__ stdv,
                                                     const int32_t* __restrict__ use, int D, double* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ int pos[256];
  for (int d = threadIdx.x; d < D && d < 256; d += 256) pos[d] = -1;
  __syncthreads();
  for (int u = threadIdx.x; u < U; u += 256) pos[use[u]] = u;
  __syncthreads();
  const int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (idx >= F * D) return;
  const int64_t f = idx / D;
  const int d = (int)(idx - f * D);
  const int u = pos[d];
  float v = 0.0f;
  if (u >= 0) v = INF32 ? ((const float*)xn)[f * U + u] : (float)((const double*)xn)[f * U + u];
  out[idx] = (double)v * stdv[d] + mean[d];
}

// Column sums of a row-major [F, D] float64 matrix in two deterministic levels.
// Level 1: block b sums rows [b*chunk, (b+1)*chunk) of every column (PASS 1: x, PASS 2:
// (x - mean)^2); thread = (row lane, column), rpb = 256 / D row lanes; each lane keeps 4
// independent accumulators (rows r, r+rpb, r+2rpb, r+3rpb of every group of 4 rpb) so four
// loads are in flight per thread; accumulators and lanes are folded in a fixed order.
template <int PASS>
__global__ __launch_bounds__(256) void k_col_partial(const double* __restrict__ x, int64_t F, int D, int64_t chunk,
                                                     const double* __restrict__ mean, double* __restrict__ part) {
#pragma clang fp contract(off)
  __shared__ double red[256];
  const int rpb = 256 / D;
  const int t = threadIdx.x;
  const int lane = t / D, d = t - lane * D;
  const int64_t r0 = (int64_t)blockIdx.x * chunk, r1 = min(F, r0 + chunk);
  double s = 0.0;
  if (lane < rpb) {
    const double mu = PASS == 2 ? mean[d] : 0.0;
    double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
    int64_t r = r0 + lane;
    const int64_t step = rpb;
    for (; r + 3 * step < r1; r += 4 * step) {
      double v0 = x[r * D + d], v1 = x[(r + step) * D + d], v2 = x[(r + 2 * step) * D + d],
             v3 = x[(r + 3 * step) * D + d];
      if (PASS == 2) { v0 -= mu; v1 -= mu; v2 -= mu; v3 -= mu; v0 *= v0; v1 *= v1; v2 *= v2; v3 *= v3; }
      a0 += v0; a1 += v1; a2 += v2; a3 += v3;
    }
    for (; r < r1; r += step) {
      double v = x[r * D + d];
      if (PASS == 2) { v -= mu; v *= v; }
      a0 += v;
    }
    s = (a0 + a1) + (a2 + a3);
  }
  red[t] = s;
  __syncthreads();
  if (t < D) {
    double acc = red[t];
    for (int l = 1; l < rpb; ++l) acc += red[l * D + t];
    part[(int64_t)t * gridDim.x + blockIdx.x] = acc;   // column-major: the fold reads rows
  }
}

// Level 2: block d folds column d's G block partials (part[d][g], contiguous; thread t:
// partials t, t+256, ...;
// then a fixed LDS tree); PASS 1 -> mean = sum / F, PASS 2 -> std = sqrt(sum / F).
template <int PASS>
__global__ __launch_bounds__(256) void k_col_final(const double* __restrict__ part, int G, int D, int64_t F,
                                                   double* __restrict__ out) {
#pragma clang fp contract(off)
  __shared__ double red[256];
  const int d = blockIdx.x, t = threadIdx.x;
  double s = 0.0;
  for (int g = t; g < G; g += 256) s += part[(int64_t)d * G + g];
  red[t] = s;
  __syncthreads();
#pragma unroll
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  if (t == 0) {
    const double m = red[0] / (double)F;
    out[d] = PASS == 1 ? m : sqrt(m);
  }
}
