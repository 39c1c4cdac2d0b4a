// Smoother factor residual + Jacobian kernels (f64), one lane per factor.
//
// Replaces the GTSAM CustomFactor callbacks of perseus/smoother/factors.py
// (PoseDynamicsFactor :54-142, ConstantVelocityFactor :160-171,
// KeypointProjectionFactor :216-275) and the GTSAM 4.2 geometry they call
// (Pose3 Expmap/Logmap/ExpmapDerivative/LogmapDerivative/compose/between/
// transformFrom/transformTo, Rot3 Logmap incl. the trace ~ -1 branch,
// PinholeCamera<Cal3_S2>::project with its cheirality check).
//
// Layout (HBM): poses are 12 f64 (R row-major, t), vectors 3 f64, pixels 2 f64,
// Jacobians column-major per factor.  A wave's 64 factors read 64 consecutive
// records, so every fetched line is fully used; the work is FP64 VALU bound,
// well below HBM.  Tangent order [omega; v], right perturbation.
#include "factors_dev.h"

namespace pa {

__global__ __launch_bounds__(64) void dyn_kernel(int n, const double* __restrict__ T1p, const double* __restrict__ wp,
                                                 const double* __restrict__ vp, const double* __restrict__ T2p,
                                                 double dt, int vel_frame, const double* __restrict__ isig,
                                                 double* __restrict__ r_out, double* __restrict__ J0,
                                                 double* __restrict__ J1, double* __restrict__ J2,
                                                 double* __restrict__ J3, double* __restrict__ err) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const size_t u = i;
  dyn_one(T1p + u * 12, wp + u * 3, vp + u * 3, T2p + u * 12, dt, vel_frame, isig, r_out + u * 6,
          J0 ? J0 + u * 36 : nullptr, J1 ? J1 + u * 18 : nullptr, J2 ? J2 + u * 18 : nullptr,
          J3 ? J3 + u * 36 : nullptr, err ? err + u : nullptr);
}

__global__ __launch_bounds__(64) void cv_kernel(int n, const double* __restrict__ v1, const double* __restrict__ v2,
                                                const double* __restrict__ isig, double* __restrict__ r,
                                                double* __restrict__ J0, double* __restrict__ J1,
                                                double* __restrict__ err) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const size_t u = i;
  cv_one(v1 + u * 3, v2 + u * 3, isig, r + u * 3, J0 ? J0 + u * 9 : nullptr, J1 ? J1 + u * 9 : nullptr,
         err ? err + u : nullptr);
}

__global__ __launch_bounds__(64) void proj_kernel(int n, const double* __restrict__ Tb, const double* __restrict__ pbp,
                                                  const double* __restrict__ zp, const double* __restrict__ Kp,
                                                  int k_stride, const double* __restrict__ Tcp, int tc_stride,
                                                  const double* __restrict__ isig, double* __restrict__ r_out,
                                                  double* __restrict__ J, double* __restrict__ err,
                                                  int32_t* __restrict__ status) {
  const int i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n) return;
  const size_t u = i;
  proj_one(Tb + u * 12, load3(pbp + u * 3), zp[u * 2], zp[u * 2 + 1], Kp + u * k_stride,
           Tcp ? Tcp + u * tc_stride : nullptr, isig, r_out + u * 2, J ? J + u * 12 : nullptr, err ? err + u : nullptr,
           status ? status + u : nullptr);
}

// one launch, the dynamics workgroups dispatched first: they hold the longest per-lane
// chains and the projection / constant-velocity waves fill the other SIMDs meanwhile.
// Round 2a: one wave per 64 dynamics factors doing all of dyn_one, 16.1 us at 1000 x 24
// (block-lower-triangular 6x6 products: 19.0 -> 17.8; two waves per SIMD 17.8 -> 16.1).
// Also measured: two launches (the projection kernel at 76 VGPRs) 16.1 + 8.9 us; the
// dynamics launch on a forked side stream 42 us; s_setprio on the dynamics waves: no
// change; a lane PAIR per factor (both lanes running the shared chain, the Jacobian
// halves as one instruction stream) 18.3 us.  Two-wave dynamics workgroups: 15.3 us
// (dynamics alone 12.7, projection / constant-velocity alone 11.3 at 45 KB of LDS per
// workgroup; four workgroups per CU since); H0 / J0 moved to wave 1 (one barrier) and four
// projection factors per lane: 14.7 us.  Three waves per SIMD does not fit (~220 VGPRs).
// mode (pa_debug_trajectory_linearize, timing only): 1 = dynamics workgroups only,
// 2 = projection / constant-velocity workgroups only
__global__ __launch_bounds__(128, 2) void traj_all_kernel(pa_traj_args a, int mode, unsigned long long* ts) {
  __shared__ __attribute__((aligned(16))) double st[trj::STAGE];
  const long wd = ((long)a.T * (a.L - 1) + 63) / 64;
  if ((long)blockIdx.x < wd) {
    if (mode == 2) return;
    traj_dyn_block(a, blockIdx.x, st, ts);
  } else if (mode == 1) {
    return;
  } else {
    const int wv = threadIdx.x >> 6;
    traj_unit_wave(a, 2 * ((long)blockIdx.x - wd) + wv, st + wv * trj::UNIT, ts);
  }
}

// ---------------------------------------------------------------------------------------
// Fixed-lag window of the streaming pose stage (config 4): the smoother loop the
// reference leaves to downstream GTSAM code (scripts/streaming.py:121-155 runs the
// detector only), restated on device so a tick's poses never leave HBM.


__global__ __launch_bounds__(256) void window_advance_kernel(int L, int n_kp, const float* __restrict__ y_new,
                                                             float* y, double* pose, double* angvel, double* vel,
                                                             double dt, int vel_frame, int32_t* nvalid) {
  window_advance_body(blockIdx.x, threadIdx.x, 256, L, n_kp, y_new, y, pose, angvel, vel, dt, vel_frame, nvalid);
}

__global__ __launch_bounds__(64) void window_retract_kernel(int T, int L, const double* __restrict__ delta,
                                                            const int32_t* __restrict__ info, double* pose,
                                                            double* angvel, double* vel, double* newest) {
  const long f = (long)blockIdx.x * 64 + threadIdx.x;
  if (f < (long)T * L) window_retract_one(f, L, delta, info, pose, angvel, vel, newest);
}

}  // namespace pa

extern "C" {

int pa_window_advance_n(int T, int L, int n_kp, const float* y_new, float* y, double* pose, double* angvel,
                        double* vel, int32_t* nvalid, double dt, int vel_frame, void* stream) {
  PA_CHECK(T >= 0 && L >= 1 && n_kp >= 1 && n_kp <= 32, "T=%d L=%d n_kp=%d", T, L, n_kp);
  if (T == 0) return PA_OK;
  PA_CHECK(y_new && y && pose && angvel && vel, "null pointer");
  PA_CHECK(vel_frame == PA_VEL_WORLD || vel_frame == PA_VEL_BODY, "vel_frame must be 'world' or 'body'.");
  hipLaunchKernelGGL(pa::window_advance_kernel, dim3(T), dim3(256), 0, (hipStream_t)stream, L, n_kp, y_new, y, pose,
                     angvel, vel, dt, vel_frame, nvalid);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int pa_window_advance(int T, int L, int n_kp, const float* y_new, float* y, double* pose, double* angvel,
                      double* vel, double dt, int vel_frame, void* stream) {
  return pa_window_advance_n(T, L, n_kp, y_new, y, pose, angvel, vel, nullptr, dt, vel_frame, stream);
}

int pa_window_retract_newest(int T, int L, const double* delta, const int32_t* info, double* pose, double* angvel,
                             double* vel, double* newest_pose, void* stream) {
  PA_CHECK(T >= 0 && L >= 1, "T=%d L=%d", T, L);
  if (T == 0) return PA_OK;
  PA_CHECK(delta && pose && angvel && vel, "null pointer");
  const long n = (long)T * L;
  hipLaunchKernelGGL(pa::window_retract_kernel, dim3((unsigned)((n + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                     T, L, delta, info, pose, angvel, vel, newest_pose);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int pa_window_retract(int T, int L, const double* delta, const int32_t* info, double* pose, double* angvel,
                      double* vel, void* stream) {
  return pa_window_retract_newest(T, L, delta, info, pose, angvel, vel, nullptr, stream);
}

int pa_dyn_linearize(int n, const double* t1, const double* w, const double* v, const double* t2, double dt,
                     int vel_frame, const double* inv_sigma, double* r, double* j0, double* j1, double* j2,
                     double* j3, double* err, void* stream) {
  PA_CHECK(n >= 0, "n %d", n);
  if (n == 0) return PA_OK;
  PA_CHECK(t1 && w && v && t2 && r, "null pointer");
  PA_CHECK(vel_frame == PA_VEL_WORLD || vel_frame == PA_VEL_BODY, "vel_frame must be 'world' or 'body'.");
  hipLaunchKernelGGL(pa::dyn_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, n, t1, w, v, t2, dt,
                     vel_frame, inv_sigma, r, j0, j1, j2, j3, err);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int pa_cv_linearize(int n, const double* v1, const double* v2, const double* inv_sigma, double* r, double* j0,
                    double* j1, double* err, void* stream) {
  PA_CHECK(n >= 0, "n %d", n);
  if (n == 0) return PA_OK;
  PA_CHECK(v1 && v2 && r, "null pointer");
  hipLaunchKernelGGL(pa::cv_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, n, v1, v2, inv_sigma, r,
                     j0, j1, err);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int pa_debug_trajectory_linearize(const pa_traj_args* a, int mode, unsigned long long* trace, void* stream) {
  PA_CHECK(a, "null args");
  PA_CHECK(a->T >= 0 && a->L >= 1 && a->n_kp >= 1, "T=%d L=%d n_kp=%d", a->T, a->L, a->n_kp);
  if (a->T == 0) return PA_OK;
  PA_CHECK(a->y && a->pose && a->vel && a->angvel && a->corners && a->K, "null input pointer");
  PA_CHECK(a->r_proj && (a->L == 1 || (a->r_dyn && a->r_cv)), "null output pointer");
  PA_CHECK(a->vel_frame == PA_VEL_WORLD || a->vel_frame == PA_VEL_BODY, "vel_frame must be 'world' or 'body'.");
  const long np = (long)a->T * a->L * a->n_kp, nd = (long)a->T * (a->L - 1);
  const long units = (np + 64 * pa::trj::PPW - 1) / (64 * pa::trj::PPW) + (nd + 63) / 64;  // projection | const-vel, two per workgroup
  hipLaunchKernelGGL(pa::traj_all_kernel, dim3((unsigned)((nd + 63) / 64 + (units + 1) / 2)), dim3(128), 0,
                     (hipStream_t)stream, *a, mode, trace);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int pa_trajectory_linearize(const pa_traj_args* a, void* stream) {
  return pa_debug_trajectory_linearize(a, 0, nullptr, stream);
}

int pa_proj_linearize(int n, const double* tbody, const double* pb, const double* z, const double* k, int k_stride,
                      const double* tcam, int tcam_stride, const double* inv_sigma, double* r, double* j, double* err,
                      int32_t* status, void* stream) {
  PA_CHECK(n >= 0, "n %d", n);
  if (n == 0) return PA_OK;
  PA_CHECK(tbody && pb && z && k && r, "null pointer");
  PA_CHECK(k_stride == 0 || k_stride == 5, "k_stride must be 0 or 5");
  PA_CHECK(tcam_stride == 0 || tcam_stride == 12, "tcam_stride must be 0 or 12");
  hipLaunchKernelGGL(pa::proj_kernel, dim3((n + 63) / 64), dim3(64), 0, (hipStream_t)stream, n, tbody, pb, z, k,
                     k_stride, tcam, tcam_stride, inv_sigma, r, j, err, status);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // extern "C"

