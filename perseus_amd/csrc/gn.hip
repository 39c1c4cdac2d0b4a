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
// Kernel 1 (gn_assemble): one wave per frame builds D_l, E_l, g_l = J^T r from the
// factors touching it -- each block has one writer, no atomics.  Kernel 2 (gn_solve):
// one wave per trajectory, block Cholesky (L_l L_l^T = D_l + lambda I - W_l^T W_l,
// W_l = L_{l-1}^{-1} E_{l-1}), forward and back substitution.  f64 throughout.
// Jacobians are column-major per factor (include/perseus_amd.h).
#include "common.h"

namespace pa {

namespace gn {
constexpr int NV = 12;  // variables per frame
constexpr int NB = NV * NV;
}  // namespace gn

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

// ---------------------------------------------------------------- assembly
// One wave per frame l (of trajectory t).  The factor rows touching x_l are stacked in
// LDS, transposed, as A^T (12 x R, in x_l coordinates; zero rows for cheirality-failed
// projections) with their residuals r, and the rows of the factors (l, l+1) also as the
// 12 x 10 pair (A_next^T, B^T) (B: their x_{l+1} part):
//   projection k of frame l   2 rows  A = [J_k | 0 | 0]
//   dynamics (l, l+1)         6 rows  A = [J0 | J1 | J2]   B = [J3 | 0 | 0]
//   const-velocity (l, l+1)   3 rows  A = [0 | 0 | C0]     B = [0 | 0 | C1]
//   dynamics (l-1, l)         6 rows  A = [J3 | 0 | 0]
//   const-velocity (l-1, l)   3 rows  A = [0 | 0 | C1]
// Then D = A^T A, E = A_next^T B, g = A^T r as 108 work items (an output row i x 3
// columns, or one g entry) over the wave's lanes, reading 2 rows per 16-B LDS read.
constexpr int GN_KMAX = 16;  // keypoints per frame supported
constexpr int GN_WSF = 2 * gn::NB + 2 * gn::NV;  // workspace doubles per frame: L_l, W_l, y_l, 1 / diag(L_l)
template <int RP>  // stacked rows, padded to even: 2 K + 18 (+1)
__global__ __launch_bounds__(64, 8) void gn_assemble(GnArgs a) {
  using namespace gn;
  __shared__ __attribute__((aligned(16))) double AT[NV][RP];
  __shared__ __attribute__((aligned(16))) double rT[RP];
  __shared__ __attribute__((aligned(16))) double ANT[NV][10];
  __shared__ __attribute__((aligned(16))) double BT[NV][10];
  const int lane = threadIdx.x;
  const long f = blockIdx.x;
  const int t = (int)(f / a.L), l = (int)(f - (long)t * a.L);
  const int npair = a.L - 1;
  const int K = a.K;
  const bool nxt = l + 1 < a.L, prv = l > 0;
  for (int e = lane; e < NV * RP; e += 64) (&AT[0][0])[e] = 0.0;
  for (int e = lane; e < NV * 10; e += 64) {
    (&ANT[0][0])[e] = 0.0;
    (&BT[0][0])[e] = 0.0;
  }
  for (int e = lane; e < RP; e += 64) rT[e] = 0.0;
  __syncthreads();
  // projections: rows 2k, 2k + 1; J column-major 2 x 6
  for (int e = lane; e < K * 12; e += 64) {
    const int k = e / 12, c = (e - k * 12) >> 1, row = e & 1;
    const long u = f * K + k;
    if (!a.st_proj || a.st_proj[u] == 0) AT[c][2 * k + row] = a.j_proj[u * 12 + c * 2 + row];
  }
  for (int e = lane; e < K * 2; e += 64) {
    const long u = f * K + (e >> 1);
    if (!a.st_proj || a.st_proj[u] == 0) rT[e] = a.r_proj[u * 2 + (e & 1)];
  }
  const int rn = 2 * K, rp = rn + 9;  // first row of the (l, l+1) / (l-1, l) blocks
  if (nxt) {
    const long u = (long)t * npair + l;
    if (lane < 36) {  // dynamics: 6 x 6 / 6 x 3 / 6 x 3, column-major
      const int c = lane / 6, row = lane - c * 6;
      const double j0 = a.j0[u * 36 + lane];
      AT[c][rn + row] = j0;
      ANT[c][row] = j0;
      BT[c][row] = a.j3[u * 36 + lane];
      if (lane < 18) {
        const double j1 = a.j1[u * 18 + lane], j2 = a.j2[u * 18 + lane];
        AT[6 + c][rn + row] = j1;
        ANT[6 + c][row] = j1;
        AT[9 + c][rn + row] = j2;
        ANT[9 + c][row] = j2;
      }
    } else if (lane < 45) {  // const velocity: 3 x 3 on the velocity block
      const int e = lane - 36, c = e / 3, row = e - c * 3;
      const double c0 = a.jc0[u * 9 + e];
      AT[9 + c][rn + 6 + row] = c0;
      ANT[9 + c][6 + row] = c0;
      BT[9 + c][6 + row] = a.jc1[u * 9 + e];
    } else if (lane < 51) {
      rT[rn + lane - 45] = a.r_dyn[u * 6 + lane - 45];
    } else if (lane < 54) {
      rT[rn + 6 + lane - 51] = a.r_cv[u * 3 + lane - 51];
    }
  }
  if (prv) {
    const long u = (long)t * npair + l - 1;
    if (lane < 36) {
      const int c = lane / 6, row = lane - c * 6;
      AT[c][rp + row] = a.j3[u * 36 + lane];
    } else if (lane < 45) {
      const int e = lane - 36, c = e / 3, row = e - c * 3;
      AT[9 + c][rp + 6 + row] = a.jc1[u * 9 + e];
    } else if (lane < 51) {
      rT[rp + lane - 45] = a.r_dyn[u * 6 + lane - 45];
    } else if (lane < 54) {
      rT[rp + 6 + lane - 51] = a.r_cv[u * 3 + lane - 51];
    }
  }
  __syncthreads();
  typedef double d2_t __attribute__((ext_vector_type(2)));
  double* Dl = a.D + f * NB;
  double* El = nxt ? a.E + ((long)t * npair + l) * NB : nullptr;
  double* gl = a.g + f * NV;
  for (int w = lane; w < 108; w += 64) {
    if (w < 96) {  // D (w < 48) or E: row i, columns j0 .. j0 + 2
      const bool isD = w < 48;
      if (!isD && !El) continue;
      const int wi = isD ? w : w - 48;
      const int i = wi >> 2, j0 = (wi & 3) * 3;
      double s[3][2] = {{0.0, 0.0}, {0.0, 0.0}, {0.0, 0.0}};
      if (isD) {
#pragma unroll 3
        for (int q = 0; q < RP; q += 2) {
          const d2_t ai = *reinterpret_cast<const d2_t*>(&AT[i][q]);
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const d2_t aj = *reinterpret_cast<const d2_t*>(&AT[j0 + c][q]);
            s[c][0] += ai[0] * aj[0];
            s[c][1] += ai[1] * aj[1];
          }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) Dl[i * NV + j0 + c] = s[c][0] + s[c][1];
      } else {
#pragma unroll
        for (int q = 0; q < 10; q += 2) {
          const d2_t ai = *reinterpret_cast<const d2_t*>(&ANT[i][q]);
#pragma unroll
          for (int c = 0; c < 3; ++c) {
            const d2_t bj = *reinterpret_cast<const d2_t*>(&BT[j0 + c][q]);
            s[c][0] += ai[0] * bj[0];
            s[c][1] += ai[1] * bj[1];
          }
        }
#pragma unroll
        for (int c = 0; c < 3; ++c) El[i * NV + j0 + c] = s[c][0] + s[c][1];
      }
    } else {  // g[i]
      const int i = w - 96;
      double s0 = 0.0, s1 = 0.0;
#pragma unroll 3
      for (int q = 0; q < RP; q += 2) {
        const d2_t ai = *reinterpret_cast<const d2_t*>(&AT[i][q]);
        const d2_t r = *reinterpret_cast<const d2_t*>(&rT[q]);
        s0 += ai[0] * r[0];
        s1 += ai[1] * r[1];
      }
      gl[i] = s0 + s1;
    }
  }
}

// ---------------------------------------------------------------- solve
// One wave per trajectory: block Cholesky of the block-tridiagonal normal matrix, frame
// by frame,
//   W_l = L_{l-1}^{-1} E_{l-1}                 lane c < 12: column c, forward substitution
//                                              with L_{l-1} read from LDS (uniform addresses)
//   S_l = D_l + lambda I - W_l^T W_l           lane i: row i (its own W column, all of W
//   rhs_l = -g_l - W_l^T y_{l-1}                from LDS)
//   L_l L_l^T = S_l                            right-looking, column j final at step j; the
//                                              raw column j reaches every lane by v_readlane
//   y_l = L_l^{-1} rhs_l
// then back substitution L_l^T delta_l = y_l - W_{l+1} delta_{l+1}.  L_l, W_l, y_l go to the
// workspace for the backward pass.  The next frame's D / E / g rows are loaded while the
// current frame is factored.  (Round 1 ran one thread per trajectory with the blocks in
// LDS, 16-thread workgroups: 2.2 ms per 1000 x 24.)
// 1 / sqrt(x) for x > 0: the hardware estimate + two Newton steps (f64 accurate; the IEEE
// sqrt + divide sequences were a third of the solve's instructions)
__device__ __forceinline__ double gn_rsqrt(double x) {
  double y = __builtin_amdgcn_rsq(x);
  const double hx = 0.5 * x;
  y = y * (1.5 - hx * y * y);
  y = y * (1.5 - hx * y * y);
  return y;
}

__device__ __forceinline__ double gn_bcast(double v, int src) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)b, src);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), src);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

__global__ __launch_bounds__(64) void gn_solve(GnArgs a) {
  using namespace gn;
  __shared__ __attribute__((aligned(16))) double Lp[NB];  // L_{l-1}, row-major
  __shared__ double Ld[NV];                                 // 1 / L_{l-1}[i][i]
  __shared__ __attribute__((aligned(16))) double Wt[NB];  // W_l^T: row c = column c of W
  __shared__ __attribute__((aligned(16))) double ys[NV];  // y_{l-1}
  const int t = blockIdx.x, i = threadIdx.x;
  const int ic = i < NV ? i : NV - 1;  // lanes >= 12 shadow row / column 11 (no stores)
  const bool act = i < NV;
  const int L = a.L, npair = L - 1;
  double* ws = a.ws + (size_t)t * L * GN_WSF;
  // frame-l operands, loaded one frame ahead: row ic of D_l, column ic of E_{l-1}, g_l[ic]
  double Dn[NV], En[NV], gn_;
  auto load = [&](int l) {
    const size_t f = (size_t)t * L + l;
#pragma unroll
    for (int j = 0; j < NV; ++j) Dn[j] = a.D[f * NB + ic * NV + j];
    gn_ = a.g[f * NV + ic];
    if (l > 0) {
      const double* Ep = a.E + ((size_t)t * npair + l - 1) * NB;
#pragma unroll
      for (int k = 0; k < NV; ++k) En[k] = Ep[k * NV + ic];
    }
  };
  load(0);
  int info = 0;
  for (int l = 0; l < L; ++l) {
    double* wl = ws + (size_t)l * GN_WSF;
    double S[NV], Ec[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      S[j] = Dn[j] + (j == ic ? a.lambda : 0.0);
      Ec[j] = En[j];
    }
    double rhs = -gn_;
    if (l + 1 < L) load(l + 1);
    if (l > 0) {
      // W column ic: L_{l-1} w = E_{l-1}[:, ic]
      double w[NV];
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        double s0 = Ec[k], s1 = 0.0;
#pragma unroll
        for (int m = 0; m < k; ++m) {
          if (m & 1)
            s1 -= Lp[k * NV + m] * w[m];
          else
            s0 -= Lp[k * NV + m] * w[m];
        }
        w[k] = (s0 + s1) * Ld[k];
      }
      if (act) {
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          Wt[i * NV + k] = w[k];
          wl[NB + k * NV + i] = w[k];  // W_l row-major in the workspace
        }
      }
      lds_barrier();  // LDS only (a full barrier would drain the stores and the prefetch)
      // S[ic][j] -= sum_k W[k][ic] W[k][j];  rhs -= sum_k W[k][ic] y_{l-1}[k]
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        double s0 = 0.0, s1 = 0.0;
#pragma unroll
        for (int k = 0; k < NV; k += 2) {
          s0 += w[k] * Wt[j * NV + k];
          s1 += w[k + 1] * Wt[j * NV + k + 1];
        }
        S[j] -= s0 + s1;
      }
      double r0 = 0.0, r1 = 0.0;
#pragma unroll
      for (int k = 0; k < NV; k += 2) {
        r0 += w[k] * ys[k];
        r1 += w[k + 1] * ys[k + 1];
      }
      rhs -= r0 + r1;
    }
    // S = L L^T, right-looking; lane ic's S becomes row ic of L (a non-positive pivot sets
    // `bad`; the loop runs on with a dummy pivot so it stays fully unrolled)
    bool bad = false;
    double invd = 1.0;  // 1 / L[ic][ic]
#pragma unroll
    for (int j = 0; j < NV; ++j) {
      double col[NV];  // raw column j: S[m][j], final for m >= j
#pragma unroll
      for (int m = j; m < NV; ++m) col[m] = gn_bcast(S[j], m);
      double d2 = col[j];
      if (!(d2 > 0.0)) {
        bad = true;
        d2 = 1.0;
      }
      const double inv = gn_rsqrt(d2);
      const double lij = S[j] * inv;  // L[ic][j] for ic > j
      if (ic >= j) S[j] = ic == j ? d2 * inv : lij;
      invd = ic == j ? inv : invd;
#pragma unroll
      for (int m = j + 1; m < NV; ++m)
        if (ic > j) S[m] -= lij * (col[m] * inv);
    }
    if (bad) {
      info = l + 1;
      break;
    }
#pragma unroll
    for (int j = 0; j < NV; ++j)
      if (j > ic) S[j] = 0.0;
    // y = L^{-1} rhs
    double y[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      if (ic == k) rhs *= invd;
      y[k] = gn_bcast(rhs, k);
      if (ic > k) rhs -= S[k] * y[k];
    }
    lds_barrier();  // every lane is past its reads of Lp / Ld / Wt / ys
    if (act) {
#pragma unroll
      for (int j = 0; j < NV; ++j) {
        Lp[i * NV + j] = S[j];
        wl[i * NV + j] = S[j];
      }
      Ld[i] = invd;
      ys[i] = y[i];
      wl[2 * NB + i] = y[i];
      wl[2 * NB + NV + i] = invd;
    }
    lds_barrier();
  }
  if (!info) {
    double xn[NV];
#pragma unroll
    for (int j = 0; j < NV; ++j) xn[j] = 0.0;
    // frame l's column ic of L_l, y_l[ic] and row ic of W_{l+1}, loaded one frame ahead
    double Lc_n[NV], Wr_n[NV], y_n = 0.0, di_n = 0.0;
    auto load_b = [&](int l) {
      const double* wl = ws + (size_t)l * GN_WSF;
#pragma unroll
      for (int k = 0; k < NV; ++k) Lc_n[k] = wl[k * NV + ic];
      y_n = wl[2 * NB + ic];
      di_n = wl[2 * NB + NV + ic];
      if (l + 1 < L) {
        const double* Wn = ws + (size_t)(l + 1) * GN_WSF + NB + ic * NV;
#pragma unroll
        for (int k = 0; k < NV; ++k) Wr_n[k] = Wn[k];
      }
    };
    load_b(L - 1);
    for (int l = L - 1; l >= 0; --l) {
      double Lc[NV], Wr[NV];  // column ic of L_l = row ic of L_l^T; row ic of W_{l+1}
#pragma unroll
      for (int k = 0; k < NV; ++k) {
        Lc[k] = Lc_n[k];
        Wr[k] = Wr_n[k];
      }
      double rhs = y_n;
      const double di = di_n;  // 1 / L_l[ic][ic]
      if (l > 0) load_b(l - 1);
      if (l + 1 < L) {  // rhs -= W_{l+1} delta_{l+1}
        double r0 = 0.0, r1 = 0.0;
#pragma unroll
        for (int k = 0; k < NV; k += 2) {
          r0 += Wr[k] * xn[k];
          r1 += Wr[k + 1] * xn[k + 1];
        }
        rhs -= r0 + r1;
      }
#pragma unroll
      for (int k = NV - 1; k >= 0; --k) {  // L^T x = rhs, right-looking from the last row
        if (ic == k) rhs *= di;
        xn[k] = gn_bcast(rhs, k);
        if (ic < k) rhs -= Lc[k] * xn[k];
      }
      if (act) a.delta[((size_t)t * L + l) * NV + i] = xn[i];
    }
  } else {
    for (int e = i; e < L * NV; e += 64) a.delta[(size_t)t * L * NV + e] = NAN;
  }
  if (a.info && i == 0) a.info[t] = info;
}

}  // namespace pa

extern "C" {

size_t pa_trajectory_gn_workspace(int T, int L) {
  return (T > 0 && L > 0) ? (size_t)T * L * pa::GN_WSF * sizeof(double) : 0;
}

int pa_trajectory_gn_step(int T, int L, int n_kp, const double* r_proj, const double* j_proj,
                          const int32_t* status_proj, const double* r_dyn, const double* j_dyn0,
                          const double* j_dyn1, const double* j_dyn2, const double* j_dyn3, const double* r_cv,
                          const double* j_cv0, const double* j_cv1, double lambda, double* D, double* E, double* g,
                          double* delta, int32_t* info, void* ws, size_t ws_bytes, void* stream) {
  PA_CHECK(T >= 0 && L >= 1 && n_kp >= 0 && n_kp <= pa::GN_KMAX, "gn: T %d L %d n_kp %d (<= %d)", T, L, n_kp,
           pa::GN_KMAX);
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
  if (n_kp == 8)
    hipLaunchKernelGGL(pa::gn_assemble<34>, dim3(F), dim3(64), 0, s, a);
  else
    hipLaunchKernelGGL(pa::gn_assemble<2 * pa::GN_KMAX + 18>, dim3(F), dim3(64), 0, s, a);
  hipLaunchKernelGGL(pa::gn_solve, dim3(T), dim3(64), 0, s, a);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // extern "C"
