// Evaluation epilogue of the hot path: un-normalize + (optional) per-frame Procrustes
// alignment + per-joint L2, accumulated in fp64.  src/predict_3dpose.py:399-430,
// src/procrustes.py:2-63, src/data_utils.py:283-311.
//
// One thread per frame.  The reference un-normalizes into a float32 zero buffer and
// multiplies by fp64 std/mean (data_utils.py:305-309), so an fp32 input row is exact;
// the non-Procrustes arithmetic below is the reference's operation order with no FMA
// contraction (bit-exact per frame).  The Procrustes branch solves the 3x3 orthogonal
// Procrustes problem with a cyclic Jacobi eigensolver on A^T A (fp64); the rotation is
// the unique proper-rotation solution, so it agrees with LAPACK's SVD path to rounding.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define P3D_MAX_JOINTS 17

struct MpjpeArgs {
  const float* pred; const float* gt;   // [B, D] normalized network outputs / targets
  int D;                                // 48 (17-joint protocol) or 42 (predict_14)
  int J;                                // joints scored: 17 (root prepended) or 14
  int root;                             // 1: joint 0 is the root (dims 0..2, = mean)
  const double* mean; const double* stdv; const int32_t* dims;   // [96], [96], [D]
  int64_t B;
  double* joint_sum;                    // [J] (+=)
  double* sq_sum;                       // [1] (+=) sum of (pred_n - gt_n)^2, or null
};

// joint j of one frame, un-normalized (mm)
__device__ __forceinline__ void p3d_joint(const float* row, const MpjpeArgs& a, int j, double v[3]) {
#pragma clang fp contract(off)   // x*std + mean rounded twice, as numpy computes it
#pragma unroll
  for (int d = 0; d < 3; ++d) {
    if (a.root && j == 0) {
      v[d] = __dadd_rn(__dmul_rn(0.0, a.stdv[d]), a.mean[d]);
    } else {
      const int c = 3 * (j - a.root) + d;
      const int idx = a.dims[c];
      v[d] = __dadd_rn(__dmul_rn((double)row[c], a.stdv[idx]), a.mean[idx]);
    }
  }
}

template <int P, int Q>
__device__ __forceinline__ void p3d_jrot(double M[3][3], double V[3][3]) {
  constexpr int R = 3 - P - Q;
  const double apq = M[P][Q];
  if (apq == 0.0) return;
  const double theta = (M[Q][Q] - M[P][P]) / (2.0 * apq);
  double t;
  if (fabs(theta) > 1e150) t = 0.5 / theta;
  else t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
  const double c = 1.0 / sqrt(t * t + 1.0), s = t * c;
  M[P][P] -= t * apq;
  M[Q][Q] += t * apq;
  M[P][Q] = M[Q][P] = 0.0;
  const double arp = M[R][P], arq = M[R][Q];
  M[R][P] = M[P][R] = c * arp - s * arq;
  M[R][Q] = M[Q][R] = s * arp + c * arq;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double vp = V[k][P], vq = V[k][Q];
    V[k][P] = c * vp - s * vq;
    V[k][Q] = s * vp + c * vq;
  }
}

__device__ __forceinline__ void p3d_swapcol(double l[3], double V[3][3], int i, int k) {
  if (l[k] > l[i]) {
    const double tl = l[i]; l[i] = l[k]; l[k] = tl;
#pragma unroll
    for (int r = 0; r < 3; ++r) { const double tv = V[r][i]; V[r][i] = V[r][k]; V[r][k] = tv; }
  }
}

// T (3x3) and trace of compute_similarity_transform(X, Y, compute_optimal_scale=True)
// for A = X0^T Y0 (procrustes.py:34-49): T = V diag(1,1,sign) U^T, traceTA = sum(s).
__device__ void p3d_procrustes_rot(const double A[3][3], double T[3][3], double* traceTA) {
  double M[3][3], V[3][3];
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      M[r][c] = A[0][r] * A[0][c] + A[1][r] * A[1][c] + A[2][r] * A[2][c];
      V[r][c] = (r == c) ? 1.0 : 0.0;
    }
  for (int sweep = 0; sweep < 16; ++sweep) {
    const double off = M[0][1] * M[0][1] + M[0][2] * M[0][2] + M[1][2] * M[1][2];
    const double dia = M[0][0] * M[0][0] + M[1][1] * M[1][1] + M[2][2] * M[2][2];
    if (!(off > 1e-40 * dia)) break;
    p3d_jrot<0, 1>(M, V);
    p3d_jrot<0, 2>(M, V);
    p3d_jrot<1, 2>(M, V);
  }
  double l[3] = {M[0][0], M[1][1], M[2][2]};
  p3d_swapcol(l, V, 0, 1);
  p3d_swapcol(l, V, 0, 2);
  p3d_swapcol(l, V, 1, 2);
  // AV columns; U = [Av1/s1, GS(Av2)/s2, u1 x u2] (det U = +1)
  double av[3][3];
#pragma unroll
  for (int k = 0; k < 3; ++k)
#pragma unroll
    for (int r = 0; r < 3; ++r) av[k][r] = A[r][0] * V[0][k] + A[r][1] * V[1][k] + A[r][2] * V[2][k];
  double u[3][3];
  const double s1 = sqrt(av[0][0] * av[0][0] + av[0][1] * av[0][1] + av[0][2] * av[0][2]);
  const double i1 = s1 > 0.0 ? 1.0 / s1 : 0.0;
  for (int r = 0; r < 3; ++r) u[0][r] = av[0][r] * i1;
  const double s2 = sqrt(av[1][0] * av[1][0] + av[1][1] * av[1][1] + av[1][2] * av[1][2]);
  const double p12 = u[0][0] * av[1][0] + u[0][1] * av[1][1] + u[0][2] * av[1][2];
  double w2[3];
  for (int r = 0; r < 3; ++r) w2[r] = av[1][r] - p12 * u[0][r];
  const double n2 = sqrt(w2[0] * w2[0] + w2[1] * w2[1] + w2[2] * w2[2]);
  const double i2 = n2 > 0.0 ? 1.0 / n2 : 0.0;
  for (int r = 0; r < 3; ++r) u[1][r] = w2[r] * i2;
  u[2][0] = u[0][1] * u[1][2] - u[0][2] * u[1][1];
  u[2][1] = u[0][2] * u[1][0] - u[0][0] * u[1][2];
  u[2][2] = u[0][0] * u[1][1] - u[0][1] * u[1][0];
  const double sig3 = u[2][0] * av[2][0] + u[2][1] * av[2][1] + u[2][2] * av[2][2];
  const double e = sig3 < 0.0 ? -1.0 : 1.0;
  const double detV = V[0][0] * (V[1][1] * V[2][2] - V[1][2] * V[2][1]) -
                      V[0][1] * (V[1][0] * V[2][2] - V[1][2] * V[2][0]) +
                      V[0][2] * (V[1][0] * V[2][1] - V[1][1] * V[2][0]);
  // reference: U' = U diag(1,1,e) (s3 >= 0); sign(det(V U'^T)) = sign(detV * e)
  const double g = (detV * e) < 0.0 ? -1.0 : 1.0;
  const double d3 = g * e;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) T[r][c] = V[r][0] * u[0][c] + V[r][1] * u[1][c] + d3 * V[r][2] * u[2][c];
  *traceTA = s1 + s2 + g * fabs(sig3);
}

// 64 frames per workgroup (one wave): many small workgroups spread the per-frame
// dependent loads over the whole chip.
template <bool PROC>
__global__ __launch_bounds__(64) void k_mpjpe(MpjpeArgs a) {
  __shared__ double part[P3D_MAX_JOINTS][65];
  const int64_t f = (int64_t)blockIdx.x * 64 + threadIdx.x;
  const bool live = f < a.B;
  const float* prow = a.pred + (live ? f : 0) * a.D;
  const float* grow = a.gt + (live ? f : 0) * a.D;
  double sq_frame = 0.0;
  if (a.sq_sum && live) {
    // the loss of src/linear_model.py:129 in normalized space (fp32 differences/squares)
    for (int c = 0; c < a.D; ++c) {
      const float d = prow[c] - grow[c];
      sq_frame += (double)(d * d);
    }
  }
  if (!PROC) {
#pragma clang fp contract(off)
    for (int j = 0; j < a.J; ++j) {
      double dist = 0.0;
      if (live) {
        double pv[3], gv[3], sq[3];
        p3d_joint(prow, a, j, pv);
        p3d_joint(grow, a, j, gv);
#pragma unroll
        for (int d = 0; d < 3; ++d) {
          const double df = __dsub_rn(pv[d], gv[d]);
          sq[d] = __dmul_rn(df, df);
        }
        dist = sqrt(__dadd_rn(__dadd_rn(sq[0], sq[1]), sq[2]));
      }
      part[j][threadIdx.x] = dist;
    }
  } else {
    // X = ground truth (targets), Y = prediction (procrustes.py:21-63 as called at
    // predict_3dpose.py:416-418): out = b * Y.T + c
    double muX[3] = {0, 0, 0}, muY[3] = {0, 0, 0};
    for (int j = 0; j < a.J; ++j) {
      double pv[3], gv[3];
      p3d_joint(prow, a, j, pv);
      p3d_joint(grow, a, j, gv);
      for (int d = 0; d < 3; ++d) { muX[d] += gv[d]; muY[d] += pv[d]; }
    }
    const double invJ = 1.0 / a.J;
    for (int d = 0; d < 3; ++d) { muX[d] *= invJ; muY[d] *= invJ; }
    double ssX = 0, ssY = 0, A[3][3] = {{0, 0, 0}, {0, 0, 0}, {0, 0, 0}};
    for (int j = 0; j < a.J; ++j) {
      double pv[3], gv[3];
      p3d_joint(prow, a, j, pv);
      p3d_joint(grow, a, j, gv);
      for (int d = 0; d < 3; ++d) { gv[d] -= muX[d]; pv[d] -= muY[d]; ssX += gv[d] * gv[d]; ssY += pv[d] * pv[d]; }
#pragma unroll
      for (int r = 0; r < 3; ++r)
#pragma unroll
        for (int c = 0; c < 3; ++c) A[r][c] += gv[r] * pv[c];
    }
    const double normX = sqrt(ssX), normY = sqrt(ssY);
    const double sA = (normX > 0.0 && normY > 0.0) ? 1.0 / (normX * normY) : 0.0;
    for (int r = 0; r < 3; ++r)
      for (int c = 0; c < 3; ++c) A[r][c] *= sA;
    double T[3][3], tr;
    p3d_procrustes_rot(A, T, &tr);
    const double b = normY > 0.0 ? tr * normX / normY : 0.0;
    double cc[3];
    for (int c = 0; c < 3; ++c) cc[c] = muX[c] - b * (muY[0] * T[0][c] + muY[1] * T[1][c] + muY[2] * T[2][c]);
    for (int j = 0; j < a.J; ++j) {
      double dist = 0.0;
      if (live) {
        double pv[3], gv[3], sq[3];
        p3d_joint(prow, a, j, pv);
        p3d_joint(grow, a, j, gv);
#pragma unroll
        for (int c = 0; c < 3; ++c) {
          const double o = b * (pv[0] * T[0][c] + pv[1] * T[1][c] + pv[2] * T[2][c]) + cc[c];
          const double df = o - gv[c];
          sq[c] = df * df;
        }
        dist = sqrt(sq[0] + sq[1] + sq[2]);
      }
      part[j][threadIdx.x] = dist;
    }
  }
  __syncthreads();
  if ((int)threadIdx.x < a.J) {
    double s = 0.0;
    for (int t = 0; t < 64; ++t) s += part[threadIdx.x][t];
    if (s != 0.0) atomicAdd(a.joint_sum + threadIdx.x, s);
  }
  if (a.sq_sum) {
    for (int o = 32; o > 0; o >>= 1) sq_frame += __shfl_xor(sq_frame, o, 64);
    if (threadIdx.x == 0) atomicAdd(a.sq_sum, sq_frame);
  }
}
