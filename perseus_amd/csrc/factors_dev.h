// Device code of the smoother factors (factors.hip): the GTSAM 4.2 geometry, the three
// factors' residual / Jacobian evaluations and the config-3 trajectory units, shared with
// the fused streaming pose tick (gn.hip, pa_window_pose_tick).
#pragma once
#include <cmath>

#include "common.h"

namespace pa {

struct M3 {
  double a[9];  // row-major
  __device__ double& operator()(int r, int c) { return a[r * 3 + c]; }
  __device__ double operator()(int r, int c) const { return a[r * 3 + c]; }
};
struct V3 {
  double x, y, z;
};

__device__ __forceinline__ V3 v3(double x, double y, double z) { return V3{x, y, z}; }
__device__ __forceinline__ V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
__device__ __forceinline__ V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
__device__ __forceinline__ V3 operator*(double s, V3 a) { return v3(s * a.x, s * a.y, s * a.z); }
__device__ __forceinline__ double dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
__device__ __forceinline__ V3 cross(V3 a, V3 b) {
  return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ M3 zero3() {
  M3 m;
#pragma unroll
  for (int i = 0; i < 9; ++i) m.a[i] = 0.0;
  return m;
}
__device__ __forceinline__ M3 eye3() {
  M3 m = zero3();
  m.a[0] = m.a[4] = m.a[8] = 1.0;
  return m;
}
__device__ __forceinline__ M3 skew(V3 w) {
  M3 m = zero3();
  m(0, 1) = -w.z;
  m(0, 2) = w.y;
  m(1, 0) = w.z;
  m(1, 2) = -w.x;
  m(2, 0) = -w.y;
  m(2, 1) = w.x;
  return m;
}
__device__ __forceinline__ M3 mul(const M3& A, const M3& B) {
  M3 C;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) C(r, c) = A(r, 0) * B(0, c) + A(r, 1) * B(1, c) + A(r, 2) * B(2, c);
  return C;
}
__device__ __forceinline__ M3 tr(const M3& A) {
  M3 C;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) C(r, c) = A(c, r);
  return C;
}
__device__ __forceinline__ M3 add(const M3& A, const M3& B, double sb = 1.0) {
  M3 C;
#pragma unroll
  for (int i = 0; i < 9; ++i) C.a[i] = A.a[i] + sb * B.a[i];
  return C;
}
__device__ __forceinline__ M3 scale(const M3& A, double s) {
  M3 C;
#pragma unroll
  for (int i = 0; i < 9; ++i) C.a[i] = s * A.a[i];
  return C;
}
__device__ __forceinline__ V3 mv(const M3& A, V3 v) {
  return v3(A(0, 0) * v.x + A(0, 1) * v.y + A(0, 2) * v.z, A(1, 0) * v.x + A(1, 1) * v.y + A(1, 2) * v.z,
            A(2, 0) * v.x + A(2, 1) * v.y + A(2, 2) * v.z);
}
__device__ __forceinline__ V3 mtv(const M3& A, V3 v) {  // A^T v
  return v3(A(0, 0) * v.x + A(1, 0) * v.y + A(2, 0) * v.z, A(0, 1) * v.x + A(1, 1) * v.y + A(2, 1) * v.z,
            A(0, 2) * v.x + A(1, 2) * v.y + A(2, 2) * v.z);
}

struct Pose {
  M3 R;
  V3 t;
};

__device__ __forceinline__ Pose load_pose(const double* p) {
  Pose T;
#pragma unroll
  for (int i = 0; i < 9; ++i) T.R.a[i] = p[i];
  T.t = v3(p[9], p[10], p[11]);
  return T;
}
__device__ __forceinline__ V3 load3(const double* p) { return v3(p[0], p[1], p[2]); }

constexpr double kEps = 2.220446049250313e-16;  // std::numeric_limits<double>::epsilon()

// |w| with its sine and cosine, computed once per rotation vector: the exp, its
// derivative and Barfoot's Q of one vector share them (each called sincos itself)
struct Ang {
  double th2, th, s, c;
};
__device__ __forceinline__ Ang ang(V3 w) {
  Ang a;
  a.th2 = dot(w, w);
  a.th = sqrt(a.th2);
  sincos(a.th, &a.s, &a.c);
  return a;
}

// Rot3::Expmap (so3::ExpmapFunctor)
__device__ M3 rot_exp(V3 w, const Ang& a) {
  M3 W = skew(w);
  if (a.th2 <= kEps) return add(eye3(), W);
  return add(add(eye3(), W, a.s / a.th), mul(W, W), (1.0 - a.c) / a.th2);
}
__device__ M3 rot_exp(V3 w) { return rot_exp(w, ang(w)); }

// Rot3::Logmap (SO3::Logmap), incl. the trace ~ -1 branch
__device__ V3 rot_log(const M3& R) {
  const double R11 = R(0, 0), R12 = R(0, 1), R13 = R(0, 2);
  const double R21 = R(1, 0), R22 = R(1, 1), R23 = R(1, 2);
  const double R31 = R(2, 0), R32 = R(2, 1), R33 = R(2, 2);
  const double trc = R11 + R22 + R33;
  if (trc + 1.0 < 1e-3) {
    double Wv, Q1, Q2, Q3;
    V3 vec;
    if (R33 > R22 && R33 > R11) {
      Wv = R21 - R12;
      Q1 = 2.0 + 2.0 * R33;
      Q2 = R31 + R13;
      Q3 = R23 + R32;
      vec = v3(Q2, Q3, Q1);
    } else if (R22 > R11) {
      Wv = R13 - R31;
      Q1 = 2.0 + 2.0 * R22;
      Q2 = R23 + R32;
      Q3 = R12 + R21;
      vec = v3(Q3, Q1, Q2);
    } else {
      Wv = R32 - R23;
      Q1 = 2.0 + 2.0 * R11;
      Q2 = R12 + R21;
      Q3 = R31 + R13;
      vec = v3(Q1, Q2, Q3);
    }
    const double r = sqrt(Q1);
    const double nrm = sqrt(Q1 * Q1 + Q2 * Q2 + Q3 * Q3 + Wv * Wv);
    const double sgn = Wv < 0 ? -1.0 : 1.0;
    const double mag = M_PI - (2.0 * sgn * Wv) / nrm;
    const double sc = 0.5 / r * mag;
    return (sgn * sc) * vec;
  }
  const double tr3 = trc - 3.0;
  double mag;
  if (tr3 < -1e-6) {
    const double th = acos((trc - 1.0) / 2.0);
    mag = th / (2.0 * sin(th));
  } else {
    mag = 0.5 - tr3 / 12.0 + tr3 * tr3 / 60.0;
  }
  return mag * v3(R32 - R23, R13 - R31, R21 - R12);
}

// SO3 ExpmapDerivative (right Jacobian) and LogmapDerivative (its inverse)
__device__ M3 rot_dexp(V3 w, const Ang& a) {
  M3 W = skew(w);
  if (a.th2 <= kEps) return add(eye3(), W, -0.5);
  return add(add(eye3(), W, -(1.0 - a.c) / a.th2), mul(W, W), (a.th - a.s) / (a.th2 * a.th));
}
__device__ M3 rot_dlog(V3 w, const Ang& a) {
  if (a.th2 <= kEps) return eye3();
  M3 W = skew(w);
  return add(add(eye3(), W, 0.5), mul(W, W), 1.0 / a.th2 - (1.0 + a.c) / (2.0 * a.th * a.s));
}

// Pose3::Expmap
__device__ Pose pose_exp(V3 w, V3 v, const Ang& a) {
  Pose T;
  T.R = rot_exp(w, a);
  const double th2 = a.th2;
  if (th2 > kEps) {
    V3 wxv = cross(w, v);
    T.t = (1.0 / th2) * (wxv - mv(T.R, wxv) + dot(w, v) * w);
  } else {
    T.t = v;
  }
  return T;
}

// Pose3::Logmap (Agrawal06iros eq. 14)
__device__ void pose_log(const Pose& T, V3& w, V3& u) {
  w = rot_log(T.R);
  const double th = sqrt(dot(w, w));
  if (th < 1e-10) {
    u = T.t;
    return;
  }
  M3 W = skew((1.0 / th) * w);
  const double tn = tan(0.5 * th);
  V3 WT = mv(W, T.t);
  u = T.t - (0.5 * th) * WT + (1.0 - th / (2.0 * tn)) * mv(W, WT);
}

// Pose3::ComputeQforExpmapDerivative (Barfoot14tro eq. 102, right Jacobian)
__device__ M3 compute_q(V3 w, V3 v, const Ang& a) {
  M3 V = skew(v), W = skew(w);
  M3 WV = mul(W, V), VW = mul(V, W);
  M3 WVW = mul(WV, W);
  M3 WWV = mul(W, WV), VWW = mul(VW, W);
  M3 WVWW = mul(WVW, W), WWVW = mul(W, WVW);
  const double phi = a.th;
  M3 t1 = add(add(WV, VW), WVW, -1.0);
  M3 t2 = add(add(WWV, VWW), WVW, -3.0);
  M3 t3 = add(WVWW, WWVW);
  double c1, c2, c3;
  if (fabs(phi) > 1e-5) {
    const double s = a.s, c = a.c;
    const double p2 = phi * phi, p3 = p2 * phi, p4 = p2 * p2, p5 = p4 * phi;
    c1 = (phi - s) / p3;
    c2 = (1.0 - p2 / 2.0 - c) / p4;
    c3 = -0.5 * ((1.0 - p2 / 2.0 - c) / p4 - 3.0 * (phi - s - p3 / 6.0) / p5);
  } else {
    c1 = 1.0 / 6.0;
    c2 = -1.0 / 24.0;
    c3 = 1.0 / 120.0;
  }
  M3 Q = scale(V, -0.5);
  Q = add(Q, t1, c1);
  Q = add(Q, t2, c2);
  Q = add(Q, t3, c3);
  return Q;
}

// 6x6 helpers: block matrices [[A, 0],[C, A]] (dexp / dlog / adjoint form)
struct M6 {
  double a[36];  // row-major
  __device__ double& operator()(int r, int c) { return a[r * 6 + c]; }
  __device__ double operator()(int r, int c) const { return a[r * 6 + c]; }
};
__device__ __forceinline__ M6 blk(const M3& A, const M3& C) {
  M6 m;
#pragma unroll
  for (int r = 0; r < 3; ++r)
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      m(r, c) = A(r, c);
      m(r, c + 3) = 0.0;
      m(r + 3, c) = C(r, c);
      m(r + 3, c + 3) = A(r, c);
    }
  return m;
}
__device__ __forceinline__ M6 mul6(const M6& A, const M6& B) {
  M6 C;
  for (int r = 0; r < 6; ++r)
    for (int c = 0; c < 6; ++c) {
      double s = 0.0;
#pragma unroll
      for (int k = 0; k < 6; ++k) s += A(r, k) * B(k, c);
      C(r, c) = s;
    }
  return C;
}
// block lower-triangular 6x6 [[A, 0], [C, A]]
struct BL {
  M3 A, C;
};
__device__ __forceinline__ BL mulbl(const BL& X, const BL& Y) {
  return BL{mul(X.A, Y.A), add(mul(X.C, Y.A), mul(X.A, Y.C))};
}
__device__ __forceinline__ BL adjoint_bl(const Pose& T) { return BL{T.R, mul(skew(T.t), T.R)}; }
// Pose3::AdjointMap = [[R, 0], [skew(t) R, R]]
__device__ __forceinline__ M6 adjoint(const Pose& T) { return blk(T.R, mul(skew(T.t), T.R)); }
__device__ __forceinline__ Pose inverse(const Pose& T) {
  Pose I;
  I.R = tr(T.R);
  I.t = -1.0 * mtv(T.R, T.t);
  return I;
}
__device__ __forceinline__ Pose compose(const Pose& A, const Pose& B) {
  Pose C;
  C.R = mul(A.R, B.R);
  C.t = mv(A.R, B.t) + A.t;
  return C;
}

// -------------------------------------------------------------------- kernels
__device__ __forceinline__ void store_colmajor(double* J, const M6& m, int rows, int col0, int ncols,
                                               const double* isig) {
  for (int c = 0; c < ncols; ++c)
#pragma unroll
    for (int r = 0; r < 6; ++r) J[c * rows + r] = m(r, col0 + c) * (isig ? isig[r] : 1.0);
}

struct NoMid {
  __device__ void operator()() const {}
};

// One PoseDynamicsFactor: inputs point at this factor's records, outputs at its
// slots (r 6, J0 36, J1 18, J2 18, J3 36 column-major; err 1; any J may be null).
// `mid` runs after r, J0 and J1 are written and before J2, J3 and err are (traj_kernel:
// the wave's staging buffer is flushed there and reused for the second half).
template <typename Mid = NoMid>
__device__ void dyn_one(const double* __restrict__ T1p, const double* __restrict__ wp, const double* __restrict__ vp,
                        const double* __restrict__ T2p, double dt, int vel_frame, const double* __restrict__ isig,
                        double* r_out, double* J0, double* J1, double* J2, double* J3, double* err, Mid mid = Mid{}) {
  const Pose T1 = load_pose(T1p);
  const Pose T2 = load_pose(T2p);
  const V3 w = load3(wp);
  V3 v = load3(vp);
  V3 vb = v;
  if (vel_frame == PA_VEL_WORLD) vb = mtv(T1.R, v);  // transformTo / unrotate (factors.py:100,134)
  const V3 xw = dt * w, xv = dt * vb;
  const Ang ax = ang(xw);               // |xi_w| for Expmap, ExpmapDerivative and Q below
  const Pose inc = pose_exp(xw, xv, ax);  // Expmap (:104 / :136)
  const Pose pred = compose(T1, inc);  // compose (:105)
  const Pose rel = compose(inverse(pred), T2);  // between (:108)
  V3 ew, ev;
  pose_log(rel, ew, ev);  // Logmap (:109)
  double r[6] = {ew.x, ew.y, ew.z, ev.x, ev.y, ev.z};
  double rs[6];
#pragma unroll
  for (int k = 0; k < 6; ++k) rs[k] = r[k] * (isig ? isig[k] : 1.0);
#pragma unroll
  for (int k = 0; k < 6; ++k) r_out[k] = rs[k];
  double e = 0.0;
#pragma unroll
  for (int k = 0; k < 6; ++k) e += rs[k] * rs[k];
  if (!(J0 || J1 || J2 || J3)) {
    mid();
    if (err) *err = 0.5 * e;
    return;
  }
  // Every 6x6 factor below is block lower-triangular [[A, 0], [C, A]] (dexp / dlog /
  // adjoint form), so each product is three 3x3 products (BL, mulbl).
  // dlog = LogmapDerivative(rel) (:112)
  const Ang ae = ang(ew);
  const M3 Jw = rot_dlog(ew, ae);
  const BL dlog{Jw, scale(mul(mul(Jw, compute_q(ew, ev, ae)), Jw), -1.0)};
  // A = dlog * drel_dpred, drel_dpred = -Ad(rel^-1); H0 = A * Ad(inc^-1)
  BL A = mulbl(dlog, adjoint_bl(inverse(rel)));
  A.A = scale(A.A, -1.0);
  A.C = scale(A.C, -1.0);
  const BL H0 = mulbl(A, adjoint_bl(inverse(inc)));
  // derr_dtwist = dt * dlog * drel_dpred * I * ExpmapDerivative(xi) (:117)
  BL dtw = mulbl(A, BL{rot_dexp(xw, ax), compute_q(xw, xv, ax)});
  dtw.A = scale(dtw.A, dt);
  dtw.C = scale(dtw.C, dt);
  // J0 = H0 (+ world frame: lower-left += dtw[3:, 3:] skew(vb), :122); its columns 3..5 are [0; H0.A]
  const M3 C0 = vel_frame == PA_VEL_WORLD ? add(H0.C, mul(dtw.A, skew(vb))) : H0.C;
  const double s0 = isig ? isig[0] : 1.0, s1 = isig ? isig[1] : 1.0, s2 = isig ? isig[2] : 1.0;
  const double s3 = isig ? isig[3] : 1.0, s4 = isig ? isig[4] : 1.0, s5 = isig ? isig[5] : 1.0;
  const double sw[6] = {s0, s1, s2, s3, s4, s5};
  // column-major 6 x ncols: rows 0..2 from `top`, rows 3..5 from `bot` (null = zero block)
  auto store = [&](double* J, const M3* top, const M3& bot, int ncols) __attribute__((always_inline)) {
#pragma unroll
    for (int c = 0; c < 3; ++c) {
      if (c >= ncols) break;
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        J[c * 6 + r] = (top ? (*top)(r, c) : 0.0) * sw[r];
        J[c * 6 + 3 + r] = bot(r, c) * sw[3 + r];
      }
    }
  };
  if (J0) {
    store(J0, &H0.A, C0, 3);
    store(J0 + 18, nullptr, H0.A, 3);
  }
  if (J1) store(J1, &dtw.A, dtw.C, 3);  // dtw[:, :3] (:117-118)
  mid();
  // J2 = dtw[:, 3:] @ R1^T (world, :125) or dtw[:, 3:] (body, :128); dtw[:3, 3:] = 0
  if (J2) store(J2, nullptr, vel_frame == PA_VEL_WORLD ? mul(dtw.A, tr(T1.R)) : dtw.A, 3);
  if (J3) {  // dlog * I (:130)
    store(J3, &dlog.A, dlog.C, 3);
    store(J3 + 18, nullptr, dlog.A, 3);
  }
  if (err) *err = 0.5 * e;
}


__device__ void cv_one(const double* __restrict__ v1, const double* __restrict__ v2, const double* __restrict__ isig,
                       double* __restrict__ r, double* __restrict__ J0, double* __restrict__ J1,
                       double* __restrict__ err) {
  double e = 0.0;
#pragma unroll
  for (int k = 0; k < 3; ++k) {
    const double s = isig ? isig[k] : 1.0;
    const double rk = (v2[k] - v1[k]) * s;
    r[k] = rk;
    e += rk * rk;
  }
  if (err) *err = 0.5 * e;
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int rr = 0; rr < 3; ++rr) {
      const double s = isig ? isig[rr] : 1.0;
      if (J0) J0[c * 3 + rr] = (rr == c ? -1.0 : 0.0) * s;
      if (J1) J1[c * 3 + rr] = (rr == c ? 1.0 : 0.0) * s;
    }
}


// One KeypointProjectionFactor on preloaded operands (T: body pose, C: camera pose, cal:
// fx, fy, s, u0, v0, s0 / s1: whitening), branch-free: the cheirality case (pc.z <= 0)
// is a select at the end, so the caller can interleave several factors' loads and
// arithmetic (a branch per factor kept the traj kernel's four per-lane factors in
// sequence, each waiting out its own loads).  Outputs r 2, J 12 (col-major 2x6), err,
// status.
struct Cam {
  Pose C;
  double fx, fy, sk, u0, v0, s0, s1;
};
__device__ __forceinline__ Cam load_cam(const double* __restrict__ K, const double* __restrict__ Tcp,
                                        const double* __restrict__ isig) {
  Cam c;
  if (Tcp) {
    c.C = load_pose(Tcp);
  } else {
    c.C.R = eye3();
    c.C.t = v3(0, 0, 0);
  }
  c.fx = K[0];
  c.fy = K[1];
  c.sk = K[2];
  c.u0 = K[3];
  c.v0 = K[4];
  c.s0 = isig ? isig[0] : 1.0;
  c.s1 = isig ? isig[1] : 1.0;
  return c;
}
__device__ __forceinline__ void proj_eval(const Pose& T, V3 pb, double zx, double zy, const Cam& cam, double (&r_out)[2],
                                          double (&J)[12], double& err, int32_t& status) {
  const Pose& C = cam.C;
  const double fx = cam.fx, fy = cam.fy, sk = cam.sk, u0 = cam.u0, v0 = cam.v0, s0 = cam.s0, s1 = cam.s1;
  // transformFrom (factors.py:257): pw = R pb + t, d/dpose = [R skew(-pb), R]
  const V3 pw = mv(T.R, pb) + T.t;
  // PinholeCamera::project (:260-261): pc = Rc^T (pw - tc), cheirality pc.z <= 0
  const V3 pc = mtv(C.R, pw - C.t);
  const bool ok = pc.z > 0.0;
  const double iz = 1.0 / pc.z;
  const double x = pc.x * iz, y = pc.y * iz;
  const double u = fx * x + sk * y + u0, v = fy * y + v0;
  const double r0 = (u - zx) * s0, r1 = (v - zy) * s1;
  // dproj_dpoint = Dcal * Dpn * Rc^T (2x3), Dcal = [[fx, s],[0, fy]], Dpn = 1/z [[1,0,-x],[0,1,-y]]
  double Dpn[2][3] = {{iz, 0.0, -x * iz}, {0.0, iz, -y * iz}};
  double Dp[2][3];
  for (int c = 0; c < 3; ++c) {
    Dp[0][c] = fx * Dpn[0][c] + sk * Dpn[1][c];
    Dp[1][c] = fy * Dpn[1][c];
  }
  double Dw[2][3];  // * Rc^T : (Rc^T)(k, c) = Rc(c, k)
  for (int rr = 0; rr < 2; ++rr)
    for (int c = 0; c < 3; ++c) Dw[rr][c] = Dp[rr][0] * C.R(c, 0) + Dp[rr][1] * C.R(c, 1) + Dp[rr][2] * C.R(c, 2);
  // dpc_dpose = [R skew(-pb), R]
  const M3 RS = mul(T.R, skew(-1.0 * pb));
  const double nan = __builtin_nan("");
  for (int c = 0; c < 6; ++c) {
    double h[2];
    for (int rr = 0; rr < 2; ++rr) {
      double sacc = 0.0;
      for (int k = 0; k < 3; ++k) sacc += Dw[rr][k] * (c < 3 ? RS(k, c) : T.R(k, c - 3));
      h[rr] = sacc;
    }
    J[c * 2] = ok ? h[0] * s0 : nan;  // H0 = dproj_dpoint @ dpc_dpose (:264), column-major
    J[c * 2 + 1] = ok ? h[1] * s1 : nan;
  }
  r_out[0] = ok ? r0 : nan;
  r_out[1] = ok ? r1 : nan;
  err = ok ? 0.5 * (r0 * r0 + r1 * r1) : nan;
  status = ok ? 0 : 1;
}

// One KeypointProjectionFactor.  K: 5 values; Tc: 12 values or null (identity);
// outputs r 2, J 12 (col-major 2x6) or null, err / status or null.
__device__ void proj_one(const double* __restrict__ Tb, V3 pb, double zx, double zy, const double* __restrict__ K,
                         const double* __restrict__ Tcp, const double* __restrict__ isig, double* __restrict__ r_out,
                         double* __restrict__ J, double* __restrict__ err, int32_t* __restrict__ status) {
  const Pose T = load_pose(Tb);
  const Cam cam = load_cam(K, Tcp, isig);
  double r[2], Jl[12], e;
  int32_t st;
  proj_eval(T, pb, zx, zy, cam, r, Jl, e, st);
  r_out[0] = r[0];
  r_out[1] = r[1];
  if (err) *err = e;
  if (status) *status = st;
  if (J)
    for (int k = 0; k < 12; ++k) J[k] = Jl[k];
}


// Config 3: all factors of T trajectories x L frames in one launch, measurements
// straight from the detector output y (normalized, denormalized here exactly as
// kornia's denormalize_pixel_coordinates in f32, common.h kornia_denorm).
//
// Workgroups of two waves.  A dynamics workgroup takes 64 consecutive PoseDynamicsFactors
// and splits each factor's work between its waves (below); every other workgroup runs two
// independent 64-factor units (projection, then constant-velocity).  Outputs are staged
// per wave in LDS and written as the wave's contiguous slice of each output array, 16 B
// per lane per store (a lane's own record is 16-288 B of column-major doubles: stored
// directly, one wave-store instruction would scatter over the whole 1-18 KB slice).
namespace trj {
// doubles: dynamics wave 0 staging (r | J3 | err); A, handed from wave 0 to wave 1, whose
// region then stages wave 1's J0, J1 and J2 in turn.  40 KB: four workgroups per CU, the
// two-waves-per-SIMD register limit
constexpr int W0 = 0, XA = 64 * 43, W1 = XA, STAGE = W1 + 64 * 36;
constexpr int UNIT = 64 * 22;  // projection / constant-velocity staging per wave
static_assert(2 * UNIT <= STAGE, "unit staging");
}  // namespace trj

typedef unsigned fu32x4 __attribute__((ext_vector_type(4)));

// the wave's n records of PER doubles, staged at st[lane * PER ..], -> dst[0 .. n * PER).
// A full wave (n = 64) to a 16-B aligned dst takes the unrolled path: the LDS reads of a
// batch of 6 are issued before its stores (the rolled loop waited out one LDS round trip
// per 1 KB store: ~2 us of a 36-double flush, tools/traj_exp.py --trace)
template <int PER>
__device__ __forceinline__ void wave_flush(double* __restrict__ dst, const double* st, int n) {
  const int lane = threadIdx.x & 63, nd = n * PER;
  if (!dst) return;
  if (n == 64 && ((uintptr_t)dst & 15) == 0) {
    // write-through (sc1) buffer stores, as the conv epilogues: the 54 MB of factor outputs
    // otherwise sit dirty in the XCDs' L2s and the end-of-kernel release writes them back
    // after the last wave
    constexpr int N2 = 32 * PER, NI = (N2 + 63) / 64, BT = 6;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7fffffff, 0x00020000);
#pragma unroll
    for (int b = 0; b < NI; b += BT) {
      double2 v[BT];
#pragma unroll
      for (int i = 0; i < BT; ++i)
        if (b + i < NI && (b + i) * 64 + lane < N2) v[i] = reinterpret_cast<const double2*>(st)[(b + i) * 64 + lane];
#pragma unroll
      for (int i = 0; i < BT; ++i)
        if (b + i < NI && (b + i) * 64 + lane < N2)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(fu32x4, v[i]), rs, ((b + i) * 64 + lane) * 16, 0, 16);
    }
    return;
  }
  if (((uintptr_t)dst & 15) == 0) {
    for (int c = lane; c < nd / 2; c += 64)
      reinterpret_cast<double2*>(dst)[c] = reinterpret_cast<const double2*>(st)[c];
    if ((nd & 1) && lane == 0) dst[nd - 1] = st[nd - 1];
  } else {
    for (int c = lane; c < nd; c += 64) dst[c] = st[c];
  }
}

// timing only (pa_debug_trajectory_linearize with a trace buffer): s_memrealtime (100 MHz)
// per wave, 8 slots at trace[(workgroup * 2 + wave) * 8 + slot]
__device__ __forceinline__ void traj_stamp(unsigned long long* ts, int slot) {
  if (ts && (threadIdx.x & 63) == 0) ts[(blockIdx.x * 2 + (threadIdx.x >> 6)) * 8 + slot] = __builtin_amdgcn_s_memrealtime();
}

// wave-local LDS ordering: the staging of one wave is written and flushed by that wave only,
// and one wave's LDS instructions execute in issue order, so a compiler barrier is enough
// (it was an lgkmcnt(0) wait: every stage -> flush -> restage round then drained the LDS
// queue before the next round could be issued)
__device__ __forceinline__ void wave_sync() { asm volatile("" ::: "memory"); }

// 6 x 3 column-major block of a Jacobian: rows 0..2 from `top` (zero if !has_top), rows
// 3..5 from `bot`, row-scaled by sw (references, not pointers: an address-taken M3 lives
// in scratch)
__device__ __forceinline__ void stage6x3(double* J, bool has_top, const M3& top, const M3& bot, const double* sw) {
#pragma unroll
  for (int c = 0; c < 3; ++c)
#pragma unroll
    for (int r = 0; r < 3; ++r) {
      J[c * 6 + r] = (has_top ? top(r, c) : 0.0) * sw[r];
      J[c * 6 + 3 + r] = bot(r, c) * sw[3 + r];
    }
}

// PoseDynamicsFactor (l, l+1), 64 per workgroup, factor k on lane k of BOTH waves:
//   wave 0: Expmap -> compose -> between -> Logmap (r), dlog = LogmapDerivative(rel),
//           A = -dlog Ad(rel^-1); writes r, J3, err
//   wave 1: Expmap(xi) and ExpmapDerivative(xi) = [[dexp, 0], [Q(xw, xv), dexp]] -- both
//           independent of the chain, so they run beside it on another SIMD -- then, with A:
//           dtw = dt A D and H0 = A Ad(inc^-1); writes J1, J2, J0
// A goes 0 -> 1 through LDS (one barrier).  The products and their order are dyn_one's
// (factors.py:54-142), so the values are the same; wave 0 holds only the chain and dlog.
__device__ __forceinline__ void traj_dyn_block(const pa_traj_args& a, long blk, double* st, unsigned long long* ts) {
  using namespace trj;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long nd = (long)a.T * (a.L - 1);
  const long j0 = blk * 64;
  const int n = (int)(nd - j0 < 64 ? nd - j0 : 64);
  const long jd = j0 + (lane < n ? lane : n - 1);  // tail lanes recompute the last factor, store nothing
  const long t = jd / (a.L - 1), f = t * a.L + (jd - t * (a.L - 1));
  const bool J = a.j_dyn0 || a.j_dyn1 || a.j_dyn2 || a.j_dyn3;
  const bool world = a.vel_frame == PA_VEL_WORLD;
  const double dt = a.dt;
  double sw[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) sw[i] = a.isig_dyn ? a.isig_dyn[i] : 1.0;
  traj_stamp(ts, 0);
  const Pose T1 = load_pose(a.pose + f * 12);
  const V3 w = load3(a.angvel + f * 3);
  V3 vb = load3(a.vel + f * 3);
  if (world) vb = mtv(T1.R, vb);  // transformTo / unrotate (factors.py:100,134)
  if (ts) {
    asm volatile("" ::"v"(vb.x), "v"(T1.R.a[0]), "v"(w.x));  // the loads have landed
    traj_stamp(ts, 1);
  }
  const V3 xw = dt * w, xv = dt * vb;
  const Ang ax = ang(xw);  // |xi_w| for Expmap, ExpmapDerivative and Q
  const Pose inc = pose_exp(xw, xv, ax);  // Expmap (:104 / :136)
  double* XAp = st + XA + lane * 18;
  if (wv == 0) {
    const Pose T2 = load_pose(a.pose + (f + 1) * 12);
    const Pose pred = compose(T1, inc);           // compose (:105)
    const Pose rel = compose(inverse(pred), T2);  // between (:108)
    V3 ew, ev;
    pose_log(rel, ew, ev);  // Logmap (:109)
    const double r[6] = {ew.x, ew.y, ew.z, ev.x, ev.y, ev.z};
    double e = 0.0;
#pragma unroll
    for (int i = 0; i < 6; ++i) e += (r[i] * sw[i]) * (r[i] * sw[i]);
    BL dlog{};
    if (J) {
      // dlog = LogmapDerivative(rel) (:112)
      const Ang ae = ang(ew);
      const M3 Jw = rot_dlog(ew, ae);
      dlog = BL{Jw, scale(mul(mul(Jw, compute_q(ew, ev, ae)), Jw), -1.0)};
      // A = dlog * drel_dpred, drel_dpred = -Ad(rel^-1)
      BL A = mulbl(dlog, adjoint_bl(inverse(rel)));
      A.A = scale(A.A, -1.0);
      A.C = scale(A.C, -1.0);
#pragma unroll
      for (int i = 0; i < 9; ++i) {
        XAp[i] = A.A.a[i];
        XAp[9 + i] = A.C.a[i];
      }
    }
    traj_stamp(ts, 2);
    lds_barrier();  // A -> wave 1
    traj_stamp(ts, 3);
    // r | J3 = dlog * I (:130) | err
    double* sr = st + W0 + lane * 6;
    double* s3 = st + W0 + 64 * 6 + lane * 36;
    double* se = st + W0 + 64 * 42 + lane;
    if (lane < n) {
#pragma unroll
      for (int i = 0; i < 6; ++i) sr[i] = r[i] * sw[i];
      *se = 0.5 * e;
      if (a.j_dyn3) {
        stage6x3(s3, true, dlog.A, dlog.C, sw);
        stage6x3(s3 + 18, false, dlog.A, dlog.A, sw);
      }
    }
    wave_sync();
    wave_flush<6>(a.r_dyn + j0 * 6, st + W0, n);
    if (a.j_dyn3) wave_flush<36>(a.j_dyn3 + j0 * 36, st + W0 + 64 * 6, n);
    if (a.err_dyn) wave_flush<1>(a.err_dyn + j0, st + W0 + 64 * 42, n);
    traj_stamp(ts, 4);
    if (ts) {
      __builtin_amdgcn_s_waitcnt(0);
      traj_stamp(ts, 7);
    }
  } else {
    BL D{}, Ainc{};
    if (J) {
      D = BL{rot_dexp(xw, ax), compute_q(xw, xv, ax)};  // ExpmapDerivative(xi)
      Ainc = adjoint_bl(inverse(inc));
    }
    traj_stamp(ts, 2);
    lds_barrier();  // A <- wave 0
    traj_stamp(ts, 3);
    if (!J) return;
    BL A;
#pragma unroll
    for (int i = 0; i < 9; ++i) {
      A.A.a[i] = XAp[i];
      A.C.a[i] = XAp[9 + i];
    }
    // derr_dtwist = dt * dlog * drel_dpred * I * ExpmapDerivative(xi) (:117)
    BL dtw = mulbl(A, D);
    dtw.A = scale(dtw.A, dt);
    dtw.C = scale(dtw.C, dt);
    const BL H0 = mulbl(A, Ainc);  // H0 = A * Ad(inc^-1)
    wave_sync();  // every lane has read its A slots: the region stages J0 / J1 / J2 next
    double* s1 = st + W1;
    if (a.j_dyn0) {
      // J0 = H0 (+ world frame: lower-left += dtw[3:, 3:] skew(vb), :122); columns 3..5 [0; H0.A]
      const M3 C0 = world ? add(H0.C, mul(dtw.A, skew(vb))) : H0.C;
      if (lane < n) {
        stage6x3(s1 + lane * 36, true, H0.A, C0, sw);
        stage6x3(s1 + lane * 36 + 18, false, H0.A, H0.A, sw);
      }
      wave_sync();
      wave_flush<36>(a.j_dyn0 + j0 * 36, s1, n);
      wave_sync();
    }
    if (a.j_dyn1) {  // dtw[:, :3] (:117-118)
      if (lane < n) stage6x3(s1 + lane * 18, true, dtw.A, dtw.C, sw);
      wave_sync();
      wave_flush<18>(a.j_dyn1 + j0 * 18, s1, n);
      wave_sync();
    }
    if (a.j_dyn2) {  // J2 = dtw[:, 3:] @ R1^T (world, :125) or dtw[:, 3:] (body, :128); dtw[:3, 3:] = 0
      if (lane < n) stage6x3(s1 + lane * 18, false, dtw.A, world ? mul(dtw.A, tr(T1.R)) : dtw.A, sw);
      wave_sync();
      wave_flush<18>(a.j_dyn2 + j0 * 18, s1, n);
    }
    traj_stamp(ts, 4);
    if (ts) {
      __builtin_amdgcn_s_waitcnt(0);
      traj_stamp(ts, 7);
    }
  }
}

// one projection unit of PPW x 64 factors (unit < wp: each lane evaluates PPW factors as
// independent chains, so their loads overlap, then stages and flushes them 64 at a time) or
// one 64-factor constant-velocity unit, staged in this wave's own LDS region (wave-local
// syncs only)
namespace trj {
constexpr int PPW = 4;  // projection factors per lane
}
__device__ __forceinline__ void traj_unit_wave(const pa_traj_args& a, long u, double* st, unsigned long long* ts) {
  using trj::PPW;
  const int lane = threadIdx.x & 63;
  const long F = (long)a.T * a.L;
  const long np = F * a.n_kp, nd = (long)a.T * (a.L - 1);
  const long wp = (np + 64 * PPW - 1) / (64 * PPW);
  traj_stamp(ts, 0);
  if (u < wp) {  // KeypointProjectionFactor, factor i = f * K + k
    double r[PPW][2], J[PPW][12], e[PPW];
    int32_t stt[PPW];
    int n[PPW];
    // every operand of the PPW factors is loaded before any is used (proj_eval is
    // branch-free, so the loads of all PPW chains are in flight together)
    const Cam cam = load_cam(a.K, a.tcam, a.isig_proj);
    Pose T[PPW];
    V3 pb[PPW];
    float2 yv[PPW];
    bool off[PPW];  // a.nvalid: frame before its window's filled part
#pragma unroll
    for (int h = 0; h < PPW; ++h) {
      const long ib = (u * PPW + h) * 64;
      n[h] = (int)(np - ib < 64 ? (np - ib > 0 ? np - ib : 0) : 64);
      const long i = n[h] > 0 ? ib + (lane < n[h] ? lane : n[h] - 1) : np - 1;
      const long f = i / a.n_kp;
      const int k = (int)(i - f * a.n_kp);
      const float* yf = a.y + f * 2 * a.n_kp + 2 * k;
      yv[h] = float2{yf[0], yf[1]};
      T[h] = load_pose(a.pose + f * 12);
      pb[h] = load3(a.corners + 3 * k);
      const long t = f / a.L;
      off[h] = a.nvalid ? (int)(f - t * a.L) < a.L - a.nvalid[t] : false;
    }
#pragma unroll
    for (int h = 0; h < PPW; ++h) {
      const float px = kornia_denorm(yv[h].x, a.W);
      const float py = kornia_denorm(yv[h].y, a.H);
      proj_eval(T[h], pb[h], (double)px, (double)py, cam, r[h], J[h], e[h], stt[h]);
      if (off[h]) {  // no measurement yet: status 2, zero residual / Jacobian / error
        r[h][0] = r[h][1] = 0.0;
#pragma unroll
        for (int c = 0; c < 12; ++c) J[h][c] = 0.0;
        e[h] = 0.0;
        stt[h] = 2;
      }
    }
    if (ts) {
      asm volatile("" ::"v"(r[0][0]), "v"(r[PPW - 1][1]), "v"(J[PPW - 1][11]));  // compute done
      traj_stamp(ts, 2);
    }
    int32_t* sst = reinterpret_cast<int32_t*>(st + 64 * 15);
#pragma unroll
    for (int h = 0; h < PPW; ++h) {
      if (n[h] <= 0) break;  // wave-uniform
      const long i0 = (u * PPW + h) * 64;
      if (h) wave_sync();  // the previous flush's LDS reads are done
      st[lane * 2] = r[h][0];
      st[lane * 2 + 1] = r[h][1];
      if (a.j_proj) {
#pragma unroll
        for (int c = 0; c < 12; ++c) st[64 * 2 + lane * 12 + c] = J[h][c];
      }
      if (a.err_proj) st[64 * 14 + lane] = e[h];
      sst[lane] = stt[h];
      wave_sync();
      wave_flush<2>(a.r_proj + i0 * 2, st, n[h]);
      if (a.j_proj) wave_flush<12>(a.j_proj + i0 * 12, st + 64 * 2, n[h]);
      if (a.err_proj) wave_flush<1>(a.err_proj + i0, st + 64 * 14, n[h]);
      if (a.status && lane < n[h]) a.status[i0 + lane] = sst[lane];
    }
    traj_stamp(ts, 4);
    if (ts) {
      __builtin_amdgcn_s_waitcnt(0);
      traj_stamp(ts, 7);
    }
    return;
  }
  const long c0 = (u - wp) * 64;  // ConstantVelocityFactor (l, l+1)
  if (c0 >= nd) return;
  const int n = (int)(nd - c0 < 64 ? nd - c0 : 64);
  const long jc = c0 + (lane < n ? lane : n - 1);
  const long t = jc / (a.L - 1), f = t * a.L + (jc - t * (a.L - 1));
  cv_one(a.vel + f * 3, a.vel + (f + 1) * 3, a.isig_cv, st + lane * 3, a.j_cv0 ? st + 64 * 3 + lane * 9 : nullptr,
         a.j_cv1 ? st + 64 * 12 + lane * 9 : nullptr, a.err_cv ? st + 64 * 21 + lane : nullptr);
  wave_sync();
  wave_flush<3>(a.r_cv + c0 * 3, st, n);
  if (a.j_cv0) wave_flush<9>(a.j_cv0 + c0 * 9, st + 64 * 3, n);
  if (a.j_cv1) wave_flush<9>(a.j_cv1 + c0 * 9, st + 64 * 12, n);
  if (a.err_cv) wave_flush<1>(a.err_cv + c0, st + 64 * 21, n);
  traj_stamp(ts, 4);
  if (ts) {
    __builtin_amdgcn_s_waitcnt(0);
    traj_stamp(ts, 7);
  }
}

// ---------------------------------------------------------------------------------------
// Advance: one workgroup per trajectory.  Every element of frames 1 .. L-1 (y, pose, angvel,
// vel) moves one frame towards l = 0: the workgroup's threads first load up to ADV_E elements each
// (all loads in flight at once), then, after a barrier, store them one frame down; rounds
// cover the window in increasing frame order, so no round stores into what a later round
// reads.  (Round 2's per-element loop waited out one load-store round trip per frame: 18.7
// us for 3 x 24 against ~2.)  Then thread 0 predicts the new last frame with the
// PoseDynamicsFactor model (factors.py:100-105): pose[L-1] = pose[L-2] Exp(dt [w; v_b]),
// v_b = R^T v for a world-frame velocity, v = vel[L-2] carried over; w = the angular
// velocity frame L-2 had before the shift (L >= 3), which both new last frames take.  The
// last frame's angular velocity enters no factor (ConstantVelocityFactor constrains the
// linear velocity only, factors.py:145-171), so the GN step never corrects it: carried
// from frame L-1 instead, it kept its initial value forever and every prediction used it
// (a 40-tick tracking test plateaued at 3e-4 rad; with this, 2e-7).
// nvalid (optional): frames of the window that hold a real measurement, + 1 per advance up
// to L (pa_trajectory_linearize skips the projection factors of the others)
// (the body: trajectory t, thread e of nthr, every thread of the workgroup calls it)
constexpr int ADV_E = 4;
__device__ __forceinline__ void window_advance_body(int t, int e, int nthr, int L, int n_kp,
                                                    const float* __restrict__ y_new, float* y, double* pose,
                                                    double* angvel, double* vel, double dt, int vel_frame,
                                                    int32_t* nvalid) {
  if (nvalid && e == 0) nvalid[t] = nvalid[t] < L ? nvalid[t] + 1 : L;
  // the angular velocity of frame L-2 BEFORE the shift: the newest one a dynamics factor
  // constrains (frame L-1's enters no factor, so its value holds no information); read
  // before the first barrier, i.e. before any shifted store
  V3 wc{0.0, 0.0, 0.0};
  if (e == 0 && L >= 3) wc = load3(angvel + ((size_t)t * L + L - 2) * 3);
  const int ny = 2 * n_kp;
  float* yt = y + (size_t)t * L * ny;
  double* pt = pose + (size_t)t * L * 12;
  double* wt = angvel + (size_t)t * L * 3;
  double* vt = vel + (size_t)t * L * 3;
  const int per = ny + 18;        // elements per frame: y (ny floats) | pose (12) | angvel (3) | vel (3)
  const int n = (L - 1) * per;    // elements of frames 1 .. L-1, frame-major
  // element k of source frame l + 1 (k < per): its address
  auto at = [&](int l, int k, bool& isf) -> void* {
    isf = k < ny;
    if (k < ny) return yt + (size_t)l * ny + k;
    k -= ny;
    if (k < 12) return pt + (size_t)l * 12 + k;
    k -= 12;
    if (k < 3) return wt + (size_t)l * 3 + k;
    return vt + (size_t)l * 3 + (k - 3);
  };
  for (int base = 0; base < n; base += nthr * ADV_E) {
    double v[ADV_E];
#pragma unroll
    for (int u = 0; u < ADV_E; ++u) {
      const int i = base + u * nthr + e;
      if (i < n) {
        bool isf;
        const void* src = at(i / per + 1, i % per, isf);
        v[u] = isf ? (double)*(const float*)src : *(const double*)src;
      }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < ADV_E; ++u) {
      const int i = base + u * nthr + e;
      if (i < n) {
        bool isf;
        void* dst = at(i / per, i % per, isf);
        if (isf)
          *(float*)dst = (float)v[u];  // exact: v came from a float
        else
          *(double*)dst = v[u];
      }
    }
    __syncthreads();
  }
  if (y_new && e < ny) yt[(L - 1) * ny + e] = y_new[(size_t)t * ny + e];  // (null: the split tick's post half lands it)
  __syncthreads();
  if (e == 0 && L >= 2) {
    const Pose T1 = load_pose(pt + (L - 2) * 12);
    const V3 w = L >= 3 ? wc : load3(wt + (L - 2) * 3), v = load3(vt + (L - 2) * 3);
    if (L >= 3) {  // the shifted frame L-2 takes it too
      wt[(L - 2) * 3 + 0] = w.x;
      wt[(L - 2) * 3 + 1] = w.y;
      wt[(L - 2) * 3 + 2] = w.z;
    }
    const V3 vb = vel_frame == PA_VEL_WORLD ? mtv(T1.R, v) : v;
    const V3 xw = dt * w, xv = dt * vb;
    const Pose P = compose(T1, pose_exp(xw, xv, ang(xw)));
    double* o = pt + (L - 1) * 12;
#pragma unroll
    for (int i = 0; i < 9; ++i) o[i] = P.R.a[i];
    o[9] = P.t.x;
    o[10] = P.t.y;
    o[11] = P.t.z;
    wt[(L - 1) * 3 + 0] = w.x;
    wt[(L - 1) * 3 + 1] = w.y;
    wt[(L - 1) * 3 + 2] = w.z;
    vt[(L - 1) * 3 + 0] = v.x;
    vt[(L - 1) * 3 + 1] = v.y;
    vt[(L - 1) * 3 + 2] = v.z;
  }
}

// Retract: one thread per frame.  pose <- pose Exp(delta[0:6]) (GTSAM Pose3::retract
// with the Expmap chart, tangent [omega; v]), angvel += delta[6:9], vel += delta[9:12]
// (pa_trajectory_gn_step's variable block); trajectories whose step failed (info != 0)
// keep their values.
// newest (optional): each trajectory's last-frame pose after the update (T, 12), the
// streaming tick's output, so it needs no gather of the strided window
// (d: frame f's 12 delta values, anywhere; solved: its trajectory's info == 0)
__device__ __forceinline__ void window_retract_frame(long f, int L, const double* d, bool solved, double* pose,
                                                     double* angvel, double* vel, double* newest) {
  const long t = f / L;
  double* o = pose + f * 12;
  double* no = (newest && f - t * L == L - 1) ? newest + t * 12 : nullptr;
  if (!solved) {  // unsolved: the window stays
    if (no)
#pragma unroll
      for (int i = 0; i < 12; ++i) no[i] = o[i];
    return;
  }
  const V3 dw = load3(d), dv = load3(d + 3);
  const Pose P = compose(load_pose(o), pose_exp(dw, dv, ang(dw)));
  double v[12];
#pragma unroll
  for (int i = 0; i < 9; ++i) v[i] = P.R.a[i];
  v[9] = P.t.x;
  v[10] = P.t.y;
  v[11] = P.t.z;
#pragma unroll
  for (int i = 0; i < 12; ++i) o[i] = v[i];
  if (no)
#pragma unroll
    for (int i = 0; i < 12; ++i) no[i] = v[i];
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    angvel[f * 3 + i] += d[6 + i];
    vel[f * 3 + i] += d[9 + i];
  }
}

__device__ __forceinline__ void window_retract_one(long f, int L, const double* __restrict__ delta,
                                                   const int32_t* __restrict__ info, double* pose, double* angvel,
                                                   double* vel, double* newest) {
  window_retract_frame(f, L, delta + f * 12, !(info && info[f / L] != 0), pose, angvel, vel, newest);
}

}  // namespace pa
