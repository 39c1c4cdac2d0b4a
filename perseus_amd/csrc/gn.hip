// Factor-graph consumer: one damped Gauss-Newton / LM step over each
// trajectory, from the whitened factors of pa_trajectory_linearize, on the device.
// The graph and optimizer are not in the reference (GTSAM's LM runs on the host), so
// this build defines them: per frame l the variable block is
//   x_l = [ pose tangent (6, GTSAM order [omega; v]) | angular velocity (3) | velocity (3) ]
// and the step solves (J^T J + lambda I) delta = -J^T r.  The normal matrix of one
// trajectory is block tridiagonal in 12 x 12 blocks:
//   D_l (diagonal): the K projection factors of frame l (pose), the dynamics factors
//                   (l-1, l) and (l, l+1), the constant-velocity factors around l;
//   E_l (x_l rows, x_{l+1} cols): the dynamics and constant-velocity factors (l, l+1).
// Kernel 1 (gn_assemble): one thread per frame builds D_l, E_l, g_l = J^T r from the
// factors touching it -- each block has one writer, no atomics.  Kernel 2 (gn_solve):
// one thread per trajectory, block Cholesky (L_l L_l^T = D_l + lambda I - W_l^T W_l,
// W_l = L_{l-1}^{-1} E_{l-1}), forward and back substitution.  f64 throughout.
// Jacobians are column-major per factor (include/perseus_amd.h).
#include "common.h"

namespace pa {

namespace gn {
constexpr int NV = 12;  // variables per frame
constexpr int NB = NV * NV;
}  // namespace gn

// acc[r][c] += sum_i A(i, ra + r) * B(i, cb + c) over the factor rows, where A / B are
// column-major (rows x cols) Jacobians placed at column offsets ra / cb of x
__device__ __forceinline__ void gn_atb(double* __restrict__ blk, const double* __restrict__ A, int ca, int oa,
                                       const double* __restrict__ Bm, int cb, int ob, int rows) {
  for (int c = 0; c < cb; ++c)
    for (int r = 0; r < ca; ++r) {
      double s = 0.0;
      for (int i = 0; i < rows; ++i) s += A[i + r * rows] * Bm[i + c * rows];
      blk[(oa + r) * gn::NV + ob + c] += s;
    }
}
__device__ __forceinline__ void gn_atr(double* __restrict__ g, const double* __restrict__ A, int ca, int oa,
                                       const double* __restrict__ res, int rows) {
  for (int r = 0; r < ca; ++r) {
    double s = 0.0;
    for (int i = 0; i < rows; ++i) s += A[i + r * rows] * res[i];
    g[oa + r] += s;
  }
}

struct GnArgs {
  int T, L, K;
  const double *r_proj, *j_proj;
  const int32_t* st_proj;
  const double *r_dyn, *j0, *j1, *j2, *j3, *r_cv, *jc0, *jc1;
  double lambda;
  double *D, *E, *g, *delta;
  int32_t* info;
  double* ws;
};

__global__ __launch_bounds__(64) void gn_assemble(GnArgs a) {
  using namespace gn;
  const int f = blockIdx.x * 64 + threadIdx.x;
  if (f >= a.T * a.L) return;
  const int t = f / a.L, l = f - t * a.L;
  // accumulate straight into this frame's output blocks (one writer each; L1/L2-resident):
  // private 144-double arrays would live in scratch
  const int npair = a.L - 1;
  double* Dl = a.D + (size_t)f * NB;
  double* El = l + 1 < a.L ? a.E + ((size_t)t * npair + l) * NB : nullptr;
  double* gl = a.g + (size_t)f * NV;
  for (int i = 0; i < NB; ++i) Dl[i] = 0.0;
  if (El)
    for (int i = 0; i < NB; ++i) El[i] = 0.0;
  for (int i = 0; i < NV; ++i) gl[i] = 0.0;
  // projection factors of frame f: 2 x 6 on the pose; cheirality failures are skipped
  for (int k = 0; k < a.K; ++k) {
    const size_t u = (size_t)f * a.K + k;
    if (a.st_proj && a.st_proj[u] != 0) continue;
    const double* J = a.j_proj + u * 12;
    const double* r = a.r_proj + u * 2;
    gn_atb(Dl, J, 6, 0, J, 6, 0, 2);
    gn_atr(gl, J, 6, 0, r, 2);
  }
  if (l + 1 < a.L) {  // factors (l, l+1): this frame is their first key set
    const size_t u = (size_t)t * npair + l;
    const double *J0 = a.j0 + u * 36, *J1 = a.j1 + u * 18, *J2 = a.j2 + u * 18, *J3 = a.j3 + u * 36;
    const double* r = a.r_dyn + u * 6;
    // D_l += [J0 J1 J2]^T [J0 J1 J2]; E_l += [J0 J1 J2]^T [J3 0]
    const double* Jl[3] = {J0, J1, J2};
    const int cl[3] = {6, 3, 3}, ol[3] = {0, 6, 9};
    for (int p = 0; p < 3; ++p) {
      for (int q = 0; q < 3; ++q) gn_atb(Dl, Jl[p], cl[p], ol[p], Jl[q], cl[q], ol[q], 6);
      gn_atb(El, Jl[p], cl[p], ol[p], J3, 6, 0, 6);
      gn_atr(gl, Jl[p], cl[p], ol[p], r, 6);
    }
    const double *C0 = a.jc0 + u * 9, *C1 = a.jc1 + u * 9, *rc = a.r_cv + u * 3;
    gn_atb(Dl, C0, 3, 9, C0, 3, 9, 3);
    gn_atb(El, C0, 3, 9, C1, 3, 9, 3);
    gn_atr(gl, C0, 3, 9, rc, 3);
  }
  if (l > 0) {  // factors (l-1, l): this frame is their second key set
    const size_t u = (size_t)t * npair + l - 1;
    const double* J3 = a.j3 + u * 36;
    gn_atb(Dl, J3, 6, 0, J3, 6, 0, 6);
    gn_atr(gl, J3, 6, 0, a.r_dyn + u * 6, 6);
    const double* C1 = a.jc1 + u * 9;
    gn_atb(Dl, C1, 3, 9, C1, 3, 9, 3);
    gn_atr(gl, C1, 3, 9, a.r_cv + u * 3, 3);
  }
}

// in-place lower Cholesky of a 12 x 12 row-major block; false if not positive definite
__device__ bool gn_chol(double* A) {
  using namespace gn;
  for (int j = 0; j < NV; ++j) {
    double d = A[j * NV + j];
    for (int k = 0; k < j; ++k) d -= A[j * NV + k] * A[j * NV + k];
    if (!(d > 0.0)) return false;
    d = sqrt(d);
    A[j * NV + j] = d;
    for (int i = j + 1; i < NV; ++i) {
      double s = A[i * NV + j];
      for (int k = 0; k < j; ++k) s -= A[i * NV + k] * A[j * NV + k];
      A[i * NV + j] = s / d;
    }
    for (int k = j + 1; k < NV; ++k) A[j * NV + k] = 0.0;
  }
  return true;
}

// One thread per trajectory; the blocks it works on (L_{l-1}, L_l, W_l: 3.4 KB) live in
// its own LDS slice, so the dependent read-after-write chains of the factorisation stay
// on chip (through global memory this kernel took 8.7 ms per 1000 trajectories).
// L_l and W_l are also stored to the workspace for the back substitution.
constexpr int GN_TPB = 16;
__global__ __launch_bounds__(GN_TPB) void gn_solve(GnArgs a) {
  using namespace gn;
  __shared__ double sm[GN_TPB][3][NB];
  const int t = blockIdx.x * GN_TPB + threadIdx.x;
  if (t >= a.T) return;
  const int L = a.L, npair = L - 1;
  double* ws = a.ws + (size_t)t * L * (2 * NB + NV);
  double* Lp = sm[threadIdx.x][0];
  double* Lb = sm[threadIdx.x][1];
  double* Wb = sm[threadIdx.x][2];
  double yp[NV];
  int info = 0;
  for (int l = 0; l < L && !info; ++l) {
    const size_t f = (size_t)t * L + l;
    double* Lg = ws + (size_t)l * (2 * NB + NV);
    for (int i = 0; i < NB; ++i) Lb[i] = a.D[f * NB + i];
    for (int i = 0; i < NV; ++i) Lb[i * NV + i] += a.lambda;
    double rhs[NV];
#pragma unroll
    for (int i = 0; i < NV; ++i) rhs[i] = -a.g[f * NV + i];
    if (l > 0) {
      // W = L_{l-1}^{-1} E_{l-1} (forward substitution per column)
      const double* Ep = a.E + ((size_t)t * npair + l - 1) * NB;
      for (int i = 0; i < NB; ++i) Wb[i] = Ep[i];
      for (int c = 0; c < NV; ++c)
        for (int i = 0; i < NV; ++i) {
          double s = Wb[i * NV + c];
          for (int k = 0; k < i; ++k) s -= Lp[i * NV + k] * Wb[k * NV + c];
          Wb[i * NV + c] = s / Lp[i * NV + i];
        }
      // S = D + lambda I - W^T W;  rhs -= W^T y_{l-1}
      for (int i = 0; i < NV; ++i)
        for (int j = 0; j < NV; ++j) {
          double s = 0.0;
          for (int k = 0; k < NV; ++k) s += Wb[k * NV + i] * Wb[k * NV + j];
          Lb[i * NV + j] -= s;
        }
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        double s = 0.0;
#pragma unroll
        for (int k = 0; k < NV; ++k) s += Wb[k * NV + i] * yp[k];
        rhs[i] -= s;
      }
      for (int i = 0; i < NB; ++i) Lg[NB + i] = Wb[i];
    }
    if (!gn_chol(Lb)) {
      info = l + 1;
      break;
    }
#pragma unroll
    for (int i = 0; i < NV; ++i) {  // y = L^{-1} rhs
      double s = rhs[i];
#pragma unroll
      for (int k = 0; k < i; ++k) s -= Lb[i * NV + k] * yp[k];
      yp[i] = s / Lb[i * NV + i];
    }
    for (int i = 0; i < NB; ++i) Lg[i] = Lb[i];
#pragma unroll
    for (int i = 0; i < NV; ++i) Lg[2 * NB + i] = yp[i];
    double* tmp = Lp;  // L_l becomes L_{l-1}
    Lp = Lb;
    Lb = tmp;
  }
  if (!info) {
    double xn[NV];
    for (int l = L - 1; l >= 0; --l) {
      const double* Lb = ws + (size_t)l * (2 * NB + NV);
      const double* yb = Lb + 2 * NB;
      double rhs[NV];
#pragma unroll
      for (int i = 0; i < NV; ++i) rhs[i] = yb[i];
      if (l + 1 < L) {  // rhs -= W_{l+1} delta_{l+1}
        const double* Wn = ws + (size_t)(l + 1) * (2 * NB + NV) + NB;
#pragma unroll
        for (int i = 0; i < NV; ++i) {
          double s = 0.0;
#pragma unroll
          for (int k = 0; k < NV; ++k) s += Wn[i * NV + k] * xn[k];
          rhs[i] -= s;
        }
      }
      double x[NV];
#pragma unroll
      for (int i = NV - 1; i >= 0; --i) {  // L^T x = rhs
        double s = rhs[i];
#pragma unroll
        for (int k = i + 1; k < NV; ++k) s -= Lb[k * NV + i] * x[k];
        x[i] = s / Lb[i * NV + i];
      }
      double* d = a.delta + ((size_t)t * L + l) * NV;
#pragma unroll
      for (int i = 0; i < NV; ++i) {
        d[i] = x[i];
        xn[i] = x[i];
      }
    }
  } else {
    for (int i = 0; i < L * NV; ++i) a.delta[(size_t)t * L * NV + i] = NAN;
  }
  if (a.info) a.info[t] = info;
}

}  // namespace pa

extern "C" {

size_t pa_trajectory_gn_workspace(int T, int L) {
  return (T > 0 && L > 0) ? (size_t)T * L * (2 * pa::gn::NB + pa::gn::NV) * sizeof(double) : 0;
}

int pa_trajectory_gn_step(int T, int L, int n_kp, const double* r_proj, const double* j_proj,
                          const int32_t* status_proj, const double* r_dyn, const double* j_dyn0,
                          const double* j_dyn1, const double* j_dyn2, const double* j_dyn3, const double* r_cv,
                          const double* j_cv0, const double* j_cv1, double lambda, double* D, double* E, double* g,
                          double* delta, int32_t* info, void* ws, size_t ws_bytes, void* stream) {
  PA_CHECK(T >= 0 && L >= 1 && n_kp >= 0, "gn: T %d L %d n_kp %d", T, L, n_kp);
  if (T == 0) return PA_OK;
  PA_CHECK(lambda >= 0.0, "gn: lambda %g < 0", lambda);
  PA_CHECK(D && g && delta && ws && (L == 1 || E), "gn: null output / workspace pointer");
  PA_CHECK(n_kp == 0 || (r_proj && j_proj), "gn: null projection factors");
  PA_CHECK(L == 1 || (r_dyn && j_dyn0 && j_dyn1 && j_dyn2 && j_dyn3 && r_cv && j_cv0 && j_cv1),
           "gn: null dynamics / constant-velocity factors (Jacobians are required)");
  PA_CHECK(ws_bytes >= pa_trajectory_gn_workspace(T, L), "gn: workspace %zu < %zu", ws_bytes,
           pa_trajectory_gn_workspace(T, L));
  const pa::GnArgs a{T,     L,      n_kp,   r_proj, j_proj, status_proj, r_dyn, j_dyn0, j_dyn1, j_dyn2, j_dyn3,
                     r_cv,  j_cv0,  j_cv1,  lambda, D,      E,           g,     delta,  info,   (double*)ws};
  const hipStream_t s = (hipStream_t)stream;
  const int F = T * L;
  hipLaunchKernelGGL(pa::gn_assemble, dim3((F + 63) / 64), dim3(64), 0, s, a);
  hipLaunchKernelGGL(pa::gn_solve, dim3((T + pa::GN_TPB - 1) / pa::GN_TPB), dim3(pa::GN_TPB), 0, s, a);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // extern "C"
