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
// One launch, one workgroup per trajectory.  Assembler waves build D_l, E_l, g_l = J^T r
// from the factors touching frame l (each block has one writer, no atomics) into LDS rings
// while solver waves eliminate frame by frame.  Shipped (gn_twisted_kernel, SOLVER 2): four
// waves -- a top-down and a bottom-up chain, each one assembler + one solver wave, meeting
// at frame L / 2 (block Thomas with the Schur complements inverted by the symmetric sweep
// operator, run from both ends).  Kept as variants (gn_step_kernel): SOLVER 1, the same
// elimination as one top-down chain fed by NA assembler waves; SOLVER 0, the round-2 block
// Cholesky (L_l L_l^T = D_l + lambda I - W_l^T W_l, W_l = L_{l-1}^{-1} E_{l-1}) with
// forward and back substitution.  Launches of at most as many trajectories as CUs (the
// streaming tick's T = 3) with L <= 24 run gn_cr_kernel instead: block cyclic reduction,
// 5 serial pivots at L = 24 instead of 13.  D / E / g are optional outputs.
// f64 throughout.
// Jacobians are column-major per factor (include/perseus_amd.h).
#include "common.h"
#include "factors_dev.h"

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
  unsigned long long* trace;  // timing only (pa_debug_gn_set_trace): 256 s_memrealtime stamps per trajectory
};

// slot s of trajectory t's trace (lane 0 of the calling wave only)
__device__ __forceinline__ void gn_stamp(const GnArgs& a, int t, int slot) {
  if (a.trace && (threadIdx.x & 63) == 0 && slot < 256) a.trace[(size_t)t * 256 + slot] = __builtin_amdgcn_s_memrealtime();
}

// ---------------------------------------------------------------- assembly
// One wave, frame l (of trajectory t).  The factor rows touching x_l are stacked in
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
// wave-local LDS ordering (one wave's ds ops run in order; the wait and the "memory" clobber
// keep the compiler from moving LDS accesses across it)
__device__ __forceinline__ void wave_lds_sync() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }
// compiler-only fence: one wave's LDS instructions execute in issue order, so a read
// issued after another lane's write of the same wave sees it without a wait; this only
// keeps the compiler from moving LDS accesses across it
__device__ __forceinline__ void wave_order() { asm volatile("" ::: "memory"); }

// RP factor rows padded to whole 4-row MFMA k-steps (the pad rows stay zero)
// Rows 12..15 pad the variables to the MFMA's 16 so the operand reads need no lane test:
// AT row 12 holds r (B's column 12 -> g), AT rows 13..15 are don't-care (they only feed
// output rows / columns >= 13, never stored) and take the branch-free staging's dummy writes;
// ANT / BT rows 12..15 stay zero.
template <int RP>
struct GnStage {
  static constexpr int RPP = (RP + 3) / 4 * 4;
  double AT[16][RPP];
  double ANT[16][12];
  double BT[16][12];
};

static __device__ int32_t gn_zero_i32[1];  // status source when no status array is given (zero-initialised)
static __device__ double gn_zero_f64[2];   // projection source when K == 0 (the pointers may be null then)

// Assembles frame f (of trajectory t, frame index l) with one wave: D_l, E_l (if l + 1 < L)
// and g_l to the outputs a.D / a.E / a.g and to the LDS block `blk` (D | E | g).
// The per-lane values of one frame's factors (gn_load_frame), fetched before any is used.
template <int RP>
struct GnFrameLoads {
  static constexpr int KM = (RP - 18) / 2;        // keypoints this instantiation holds
  static constexpr int JR = (KM * 12 + 63) / 64;  // projection Jacobian entries per lane
  double jv[JR];
  int js[JR];
  double rv;
  int rs;
  double n0, n3, n1, n2, p3;
};

// Loads of frame f: every value is fetched from an address clamped to a valid element, then
// selected -- one memory latency per frame (branches around guarded loads made the compiler
// wait out each load in turn: ~10 round trips).  Nothing loaded decides a branch here, so a
// caller can issue the next frame's loads before building the current one.
template <int RP>
__device__ __forceinline__ void gn_load_frame(const GnArgs& a, long f, GnFrameLoads<RP>& ld) {
  constexpr int JR = GnFrameLoads<RP>::JR;
  const int lane = threadIdx.x & 63;
  const int t = (int)(f / a.L), l = (int)(f - (long)t * a.L);
  const int npair = a.L - 1;
  const int K = a.K;
  const bool nxt = l + 1 < a.L, prv = l > 0;
  const long fk = f * K;
  // (the status pointer test is uniform)
  const bool has_st = a.st_proj != nullptr;
  const int32_t* stp = has_st ? a.st_proj : gn_zero_i32;  // always a valid address
  // K == 0: every projection load below is clamped to element 0 of a valid dummy (the
  // caller may pass null projection arrays), and no lane uses the value
  const double* jproj = K > 0 ? a.j_proj : gn_zero_f64;
  const double* rproj = K > 0 ? a.r_proj : gn_zero_f64;
#pragma unroll
  for (int q = 0; q < JR; ++q) {
    const int e = lane + 64 * q;
    const bool v = e < K * 12;
    const long u = fk + (v ? e / 12 : 0);
    ld.jv[q] = jproj[v ? fk * 12 + e : (K > 0 ? fk * 12 : 0)];  // (u, c, row) = (e / 12, (e % 12) / 2, e & 1)
    ld.js[q] = stp[has_st ? u : 0];
  }
  const bool vr = lane < 2 * K;
  const long ur = fk + (vr ? lane >> 1 : 0);
  ld.rv = rproj[vr ? fk * 2 + lane : (K > 0 ? fk * 2 : 0)];
  ld.rs = stp[has_st ? ur : 0];
  // pair factors: lane classes [0, 36) dynamics J (6 x 6 column-major; < 18 also the 6 x 3
  // J1 / J2), [36, 45) constant velocity (3 x 3), [45, 51) dynamics r, [51, 54) const-vel r
  ld.n0 = ld.n3 = ld.n1 = ld.n2 = ld.p3 = 0.0;
  if (npair > 0) {
    const long un = (long)t * npair + (nxt ? l : 0), up = (long)t * npair + (prv ? l - 1 : 0);
    const int e36 = lane < 36 ? lane : 0, e9 = lane >= 36 && lane < 45 ? lane - 36 : 0;
    const int e6 = lane >= 45 && lane < 51 ? lane - 45 : 0, e3 = lane >= 51 && lane < 54 ? lane - 51 : 0;
    const int cls = lane < 36 ? 0 : lane < 45 ? 1 : lane < 51 ? 2 : lane < 54 ? 3 : 4;
    // per lane: the (l, l+1) factor's A-part value, its B-part value, and the (l-1, l) B-part
    const double* sa = cls == 0 ? a.j0 + un * 36 + e36 : cls == 1 ? a.jc0 + un * 9 + e9
                     : cls == 2 ? a.r_dyn + un * 6 + e6 : cls == 3 ? a.r_cv + un * 3 + e3 : a.j0;
    const double* sb = cls == 0 ? a.j3 + un * 36 + e36 : cls == 1 ? a.jc1 + un * 9 + e9 : a.j3;
    const double* sp = cls == 0 ? a.j3 + up * 36 + e36 : cls == 1 ? a.jc1 + up * 9 + e9
                     : cls == 2 ? a.r_dyn + up * 6 + e6 : cls == 3 ? a.r_cv + up * 3 + e3 : a.j3;
    const int e18 = lane < 18 ? lane : 0;
    ld.n0 = *sa;
    ld.n3 = *sb;
    ld.p3 = *sp;
    ld.n1 = a.j1[un * 18 + e18];
    ld.n2 = a.j2[un * 18 + e18];
  }
}

template <int RP, bool ZERO = true>
__device__ __forceinline__ void gn_build_frame(const GnArgs& a, long f, const GnFrameLoads<RP>& ld, GnStage<RP>& st,
                                               double* blk);

// the staging zeroed once (the pad rows and every position no factor writes stay zero;
// gn_build_frame<RP, false> then writes only the factor positions, zeros included)
template <int RP>
__device__ __forceinline__ void gn_zero_stage(GnStage<RP>& st) {
  const int lane = threadIdx.x & 63;
  for (int e = lane; e < (int)(sizeof(GnStage<RP>) / sizeof(double)); e += 64) (&st.AT[0][0])[e] = 0.0;
  wave_order();
}

template <int RP>
__device__ __forceinline__ void gn_assemble_frame(const GnArgs& a, long f, GnStage<RP>& st, double* blk) {
  GnFrameLoads<RP> ld;
  gn_load_frame<RP>(a, f, ld);
  gn_build_frame<RP>(a, f, ld, st, blk);
}

template <int RP, bool ZERO>
__device__ __forceinline__ void gn_build_frame(const GnArgs& a, long f, const GnFrameLoads<RP>& ld, GnStage<RP>& st,
                                               double* blk) {
  using namespace gn;
  constexpr int RPP = GnStage<RP>::RPP;
  constexpr int JR = GnFrameLoads<RP>::JR;
  double(&AT)[16][RPP] = st.AT;
  double(&rT)[RPP] = st.AT[NV];
  double(&ANT)[16][12] = st.ANT;
  double(&BT)[16][12] = st.BT;
  const int lane = threadIdx.x & 63;
  const int t = (int)(f / a.L), l = (int)(f - (long)t * a.L);
  const int npair = a.L - 1;
  const int K = a.K;
  const bool nxt = l + 1 < a.L, prv = l > 0;
  const bool vr = lane < 2 * K;
  const double(&jv)[JR] = ld.jv;
  const int(&js)[JR] = ld.js;
  const double rv = ld.rv, n0 = ld.n0, n3 = ld.n3, n1 = ld.n1, n2 = ld.n2, p3 = ld.p3;
  const int rs = ld.rs;
  // ---- staging: zero (ZERO; else once per launch, gn_zero_stage), then fill (one wave: its LDS
  // ops run in order).  Without the per-frame zeroing every factor position is written, with
  // 0 for a missing neighbour pair (first / last frame)
  if constexpr (ZERO) {
    for (int e = lane; e < NV * RPP; e += 64) (&AT[0][0])[e] = 0.0;
    for (int e = lane; e < NV * 12; e += 64) {
      (&ANT[0][0])[e] = 0.0;
      (&BT[0][0])[e] = 0.0;
    }
    for (int e = lane; e < RPP; e += 64) rT[e] = 0.0;
    wave_order();
  }
  typedef double d4_t __attribute__((ext_vector_type(4)));
  const int li = lane & 15, lk = lane >> 4;
  d4_t cD = {0.0, 0.0, 0.0, 0.0}, cE = {0.0, 0.0, 0.0, 0.0};
  const int rn = 2 * K, rp = rn + 9;  // first row of the (l, l+1) / (l-1, l) blocks
  if constexpr (!ZERO) {
    // branch-free staging: every lane writes its fixed positions (offsets in doubles from
    // AT[0][0]; unused slots go to the don't-care row 13 + lane / RPP), selects instead of
    // lane-class branches
    double* S = &AT[0][0];
    constexpr int OA = 0, ON = 16 * RPP, OB = 16 * RPP + 16 * 12;
    const int dummy = 13 * RPP + lane;
#pragma unroll
    for (int q = 0; q < JR; ++q) {
      const int e = lane + 64 * q;
      const int k = e / 12, c = (e - k * 12) >> 1, row = e & 1;
      S[e < K * 12 ? OA + c * RPP + 2 * k + row : dummy] = js[q] == 0 ? jv[q] : 0.0;
    }
    S[vr ? OA + NV * RPP + lane : dummy] = rs == 0 ? rv : 0.0;
    const double m0 = nxt ? n0 : 0.0, m3 = nxt ? n3 : 0.0, m1 = nxt ? n1 : 0.0, m2 = nxt ? n2 : 0.0;
    const double q3 = prv ? p3 : 0.0;
    const bool d36 = lane < 36, c9 = lane >= 36 && lane < 45, r6 = lane >= 45 && lane < 51, r3 = lane >= 51 && lane < 54;
    const int c6 = lane / 6, w6 = lane - c6 * 6;                  // dynamics: column, row
    const int c3 = (lane - 36) / 3, w3 = (lane - 36) - c3 * 3;    // const velocity (lane 36..44)
    auto at_row = [&](int r0) {  // AT offset of this lane's (l, l+1) or (l-1, l) element (rows from r0)
      return d36 ? OA + c6 * RPP + r0 + w6
           : c9  ? OA + (9 + c3) * RPP + r0 + 6 + w3
           : r6  ? OA + NV * RPP + r0 + lane - 45
           : r3  ? OA + NV * RPP + r0 + 6 + lane - 51
                 : dummy;
    };
    S[at_row(rn)] = m0;
    S[d36 ? ON + c6 * 12 + w6 : c9 ? ON + (9 + c3) * 12 + 6 + w3 : dummy] = m0;
    S[d36 ? OB + c6 * 12 + w6 : c9 ? OB + (9 + c3) * 12 + 6 + w3 : dummy] = m3;
    const bool d18 = lane < 18;
    S[d18 ? OA + (6 + c6) * RPP + rn + w6 : dummy] = m1;
    S[d18 ? ON + (6 + c6) * 12 + w6 : dummy] = m1;
    S[d18 ? OA + (9 + c6) * RPP + rn + w6 : dummy] = m2;
    S[d18 ? ON + (9 + c6) * 12 + w6 : dummy] = m2;
    S[at_row(rp)] = q3;
    wave_order();
    // [D_l | g_l] = A^T [A | r], E_l = A_next^T B: the operands straight from the padded rows
#pragma unroll
    for (int q = 0; q < RPP / 4; ++q) {
      const double v = AT[li][4 * q + lk];
      cD = __builtin_amdgcn_mfma_f64_16x16x4f64(v, v, cD, 0, 0, 0);
    }
    if (nxt) {
#pragma unroll
      for (int q = 0; q < 3; ++q)
        cE = __builtin_amdgcn_mfma_f64_16x16x4f64(ANT[li][4 * q + lk], BT[li][4 * q + lk], cE, 0, 0, 0);
    }
  } else {
    // projections: rows 2k, 2k + 1; J column-major 2 x 6
#pragma unroll
    for (int q = 0; q < JR; ++q) {
      const int e = lane + 64 * q;
      if (e < K * 12) {
        const int k = e / 12, c = (e - k * 12) >> 1, row = e & 1;
        AT[c][2 * k + row] = js[q] == 0 ? jv[q] : 0.0;
      }
    }
    if (vr) rT[lane] = rs == 0 ? rv : 0.0;
    if (nxt || !ZERO) {
      const double m0 = nxt ? n0 : 0.0, m3 = nxt ? n3 : 0.0, m1 = nxt ? n1 : 0.0, m2 = nxt ? n2 : 0.0;
      if (lane < 36) {  // dynamics: 6 x 6 / 6 x 3 / 6 x 3, column-major
        const int c = lane / 6, row = lane - c * 6;
        AT[c][rn + row] = m0;
        ANT[c][row] = m0;
        BT[c][row] = m3;
        if (lane < 18) {
          AT[6 + c][rn + row] = m1;
          ANT[6 + c][row] = m1;
          AT[9 + c][rn + row] = m2;
          ANT[9 + c][row] = m2;
        }
      } else if (lane < 45) {  // const velocity: 3 x 3 on the velocity block
        const int e = lane - 36, c = e / 3, row = e - c * 3;
        AT[9 + c][rn + 6 + row] = m0;
        ANT[9 + c][6 + row] = m0;
        BT[9 + c][6 + row] = m3;
      } else if (lane < 51) {
        rT[rn + lane - 45] = m0;
      } else if (lane < 54) {
        rT[rn + 6 + lane - 51] = m0;
      }
    }
    if (prv || !ZERO) {
      const double q3 = prv ? p3 : 0.0;
      if (lane < 36) {
        const int c = lane / 6, row = lane - c * 6;
        AT[c][rp + row] = q3;
      } else if (lane < 45) {
        const int e = lane - 36, c = e / 3, row = e - c * 3;
        AT[9 + c][rp + 6 + row] = q3;
      } else if (lane < 51) {
        rT[rp + lane - 45] = q3;
      } else if (lane < 54) {
        rT[rp + 6 + lane - 51] = q3;
      }
    }
    wave_order();
    // [D_l | g_l] = A^T [A | r] and E_l = A_next^T B on the f64 matrix cores
    // (v_mfma_f64_16x16x4_f64, MI355X_MICROARCH.md / cdna_hip_programming.md fragment maps:
    // A operand lane l = (i = l & 15, k = l >> 4), B operand (k = l >> 4, j = l & 15),
    // C/D lane l, register v = (row (l >> 4) + 4 v, col l & 15)).  Rows of the staged
    // transposes are the k dimension, 4 per instruction; variables 12..15 are zero padding
    // except B's column 12, which carries r so that C[:, 12] = A^T r = g.
#pragma unroll
    for (int q = 0; q < RPP / 4; ++q) {
      const int row = 4 * q + lk;
      const double at = li < NV ? AT[li][row] : 0.0;
      const double bv = li < NV ? at : (li == NV ? rT[row] : 0.0);
      cD = __builtin_amdgcn_mfma_f64_16x16x4f64(at, bv, cD, 0, 0, 0);
    }
    if (nxt) {
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        const int row = 4 * q + lk;
        const double an = li < NV ? ANT[li][row] : 0.0;
        const double bt = li < NV ? BT[li][row] : 0.0;
        cE = __builtin_amdgcn_mfma_f64_16x16x4f64(an, bt, cE, 0, 0, 0);
      }
    }
  }
  // D / E / g go to the API outputs only when the caller asked for them (a.D null: the
  // blocks stay in the solver's LDS ring; the streaming tick and GNPlan use delta only)
  const bool out = a.D != nullptr;  // uniform
  double* Dl = out ? a.D + f * NB : nullptr;
  double* El = (out && nxt) ? a.E + ((long)t * npair + l) * NB : nullptr;
  double* gl = out ? a.g + f * NV : nullptr;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    const int i = lk + 4 * v;
    if (i >= NV) continue;
    if (li < NV) {
      if (out) Dl[i * NV + li] = cD[v];
      blk[i * NV + li] = cD[v];
      if (nxt) {
        if (out) El[i * NV + li] = cE[v];
        blk[NB + i * NV + li] = cE[v];
      }
    } else if (li == NV) {
      if (out) gl[i] = cD[v];
      blk[2 * NB + i] = cD[v];
    }
  }
}

// ---------------------------------------------------------------- solve
// The solver wave of a trajectory: block Cholesky of the block-tridiagonal normal matrix, frame
// by frame,
//   W_l = L_{l-1}^{-1} E_{l-1}                 lane c < 12: column c, forward substitution
//                                              with L_{l-1} read from LDS (uniform addresses)
//   S_l = D_l + lambda I - W_l^T W_l           lane i: row i (its own W column, all of W
//   rhs_l = -g_l - W_l^T y_{l-1}                from LDS)
//   L_l L_l^T = S_l                            right-looking, column j final at step j; the
//                                              raw column j reaches every lane by v_readlane
//   y_l = L_l^{-1} rhs_l
// then back substitution L_l^T delta_l = y_l - W_{l+1} delta_{l+1}.  L_l, W_l, y_l go to the
// workspace for the backward pass.  Frame l's D / E / g come from the LDS ring, built by
// the assembler wave during frame l - 1 (one LDS-only barrier per frame hands a slot
// over; the solver's own LDS exchanges are wave-local).  Round 2a ran assembly (one
// wave per frame) and solve (one wave per trajectory) as two launches: 54 + 175 us per
// 1000 x 24.  (Round 1 ran one thread per trajectory with the blocks in
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

__device__ __forceinline__ int lds_load_acquire(const int* p) {
  const int v = __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
  return v;
}
__device__ __forceinline__ void lds_store_release(int* p, int v) {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");  // LDS only: global stores stay in flight
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
}

// NA assembler waves (wave a builds frames a, a + NA, ...) and one solver wave per
// trajectory, handing frames over through an LDS ring of NA + 2 slots with two LDS
// counters: ready[slot] = frame + 1 once the slot holds that frame, `consumed` = frames
// the solver has finished (frame m may overwrite slot m % R once the solver is past frame
// m - R + 1, whose E block it reads last).  Every wait is satisfied by waves of the same
// workgroup that are already running, and the solver publishes `consumed` even for frames
// it skips after a failed pivot, so every wave runs to its end.
// 1 / x for x > 0: the hardware estimate + two Newton steps (f64 accurate)
__device__ __forceinline__ double gn_rcp(double x) {
  double y = __builtin_amdgcn_rcp(x);
  y = y * (2.0 - x * y);
  y = y * (2.0 - x * y);
  return y;
}

typedef double gn_d2 __attribute__((ext_vector_type(2)));
#ifndef GN_CU
#define GN_CU 3  // k-pair unroll of gn_couple's loops (6 = fully unrolled)
#endif

// One eliminated frame's state in LDS (a solver wave's own): M = S^-1 (row-major), G =
// M E' (the S update reads it across lanes), z, this frame's b, the sweep's pivot rows.
struct GnChainLds {
  double M[gn::NB];
  double G[gn::NV * 13];  // gn_couple: G (row-major 12 x 12); gn_couple_mfma: E'^T [G | zprev] (12 x 13)
  double z[gn::NV];
  double bs[gn::NV];
  double rk2[2 * gn::NV];
};

// gn_couple on the f64 matrix cores (v_mfma_f64_16x16x4f64, operand maps as in
// gn_build_frame): G = Mprev E' as 3 k-steps with A = Mprev (lane: row l & 15, k = l >> 4) and
// B = E' (k = l >> 4, column l & 15); G lands in the C layout (register v: row (l >> 4) + 4v,
// column l & 15), which for k-step q is exactly the B operand E'^T G needs (row 4q + (l >> 4)),
// and E'^T's A operand is E' read as B was -- so the second product needs no exchange.
// Column 12 of that B carries zprev, so T = E'^T [G | zprev] gives the b update too. T goes
// through LDS (xch, 12 x 13) once to reach the row layout (lane: row r, columns c0 .. c0 + 3).
// Gout (LDS, row-major) and gws (workspace) receive G when given.
template <bool MIR>
__device__ __forceinline__ void gn_couple_mfma(const double* Mprev, const double* zprev, const double* eb,
                                               double* Gout, double* gws, double* xch, int r, int c0,
                                               double (&sv)[4], double& b) {
  using namespace gn;
  typedef double d4_t __attribute__((ext_vector_type(4)));
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const bool in = li < NV;
  const int lr = in ? li : 0;  // a valid row / column for the lanes of the padding
  double e[3];
  d4_t cG = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int k = 4 * q + lk;
    const double m = in ? Mprev[lr * NV + k] : 0.0;
    e[q] = in ? (MIR ? eb[lr * NV + k] : eb[k * NV + lr]) : 0.0;  // E'(k, li)
    cG = __builtin_amdgcn_mfma_f64_16x16x4f64(m, e[q], cG, 0, 0, 0);
  }
  d4_t cT = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const double bz = li == NV ? zprev[4 * q + lk] : 0.0;
    cT = __builtin_amdgcn_mfma_f64_16x16x4f64(e[q], in ? cG[q] : bz, cT, 0, 0, 0);
  }
  wave_order();  // every lane is past its reads of xch / Gout's previous contents
#pragma unroll
  for (int v = 0; v < 3; ++v) {  // rows lk + 4v < 12
    const int i = lk + 4 * v;
    if (li <= NV) xch[i * 13 + li] = cT[v];
    if (in) {
      if (Gout) Gout[i * NV + li] = cG[v];
      if (gws) gws[i * NV + li] = cG[v];
    }
  }
  wave_order();
#pragma unroll
  for (int c = 0; c < 4; ++c) sv[c] -= xch[r * 13 + c0 + c];  // (8-byte aligned rows)
  b -= xch[r * 13 + NV];
}

// (sv, b) -= the coupling to the previously eliminated frame (lane: row r, columns c0 .. c0 + 3):
//   G = Mprev E',   sv -= E'^T G,   b -= E'^T zprev,
// with E'(k, c) = eb[k * NV + c] (MIR = false: E_{l-1}, from the previous frame's slot) or
// eb[c * NV + k] (MIR = true: the current frame's own E_l, transposed -- the bottom-up chain).
// G goes to Gout (LDS) and, when gws is given, to the workspace (row-major, back substitution).
template <bool MIR, int CU = GN_CU>
__device__ __forceinline__ void gn_couple(const double* Mprev, const double* zprev, const double* eb, double* Gout,
                                          double* gws, int r, int c0, bool act, double (&sv)[4], double& b) {
  using namespace gn;
  double pv[4] = {0.0, 0.0, 0.0, 0.0}, ph[4] = {0.0, 0.0, 0.0, 0.0};  // even / odd k
  // k in pairs, the pair loop unrolled by NU only: fully unrolled, the compiler hoists all
  // 60 LDS reads and the 4-wave workgroup's 128-VGPR budget spills
#pragma unroll CU
  for (int k2 = 0; k2 < NV; k2 += 2) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = k2 + h;
      const double m = Mprev[r * NV + k];
      double e[4];
      if constexpr (MIR) {
#pragma unroll
        for (int c = 0; c < 4; ++c) e[c] = eb[(c0 + c) * NV + k];
      } else {
        const gn_d2 e0 = *reinterpret_cast<const gn_d2*>(eb + k * NV + c0);
        const gn_d2 e1 = *reinterpret_cast<const gn_d2*>(eb + k * NV + c0 + 2);
        e[0] = e0[0];
        e[1] = e0[1];
        e[2] = e1[0];
        e[3] = e1[1];
      }
      double* acc = h ? ph : pv;
#pragma unroll
      for (int c = 0; c < 4; ++c) acc[c] += m * e[c];
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) pv[c] += ph[c];
  wave_order();  // every lane is past its reads of Gout's previous contents
  if (act) {
    *reinterpret_cast<gn_d2*>(Gout + r * NV + c0) = gn_d2{pv[0], pv[1]};
    *reinterpret_cast<gn_d2*>(Gout + r * NV + c0 + 2) = gn_d2{pv[2], pv[3]};
    if (gws)
#pragma unroll
      for (int c = 0; c < 4; ++c) gws[r * NV + c0 + c] = pv[c];
  }
  wave_order();
  double s2[2][4] = {{0.0, 0.0, 0.0, 0.0}, {0.0, 0.0, 0.0, 0.0}}, b2[2] = {0.0, 0.0};
#pragma unroll CU
  for (int k2 = 0; k2 < NV; k2 += 2) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int k = k2 + h;
      const double ek = MIR ? eb[r * NV + k] : eb[k * NV + r];
      const gn_d2 p0 = *reinterpret_cast<const gn_d2*>(Gout + k * NV + c0);
      const gn_d2 p1 = *reinterpret_cast<const gn_d2*>(Gout + k * NV + c0 + 2);
      s2[h][0] += ek * p0[0];
      s2[h][1] += ek * p0[1];
      s2[h][2] += ek * p1[0];
      s2[h][3] += ek * p1[1];
      b2[h] += ek * zprev[k];
    }
  }
#pragma unroll
  for (int c = 0; c < 4; ++c) sv[c] -= s2[0][c] + s2[1][c];
  b -= b2[0] + b2[1];
}

// M = S^-1 by the symmetric sweep operator with 2 x 2 pivot blocks K = {k, k + 1}, k = 0, 2, .., 10
// (ends with -S^-1):  S_KK <- -P^-1,  S_iK <- S_iK P^-1,  S_Kj <- P^-1 S_Kj,
// S_ij <- S_ij - S_iK P^-1 S_Kj  (P = S_KK).  P is positive definite iff a > 0 and
// det > 0 -- the two scalar pivots a, d - b^2 / a of the Cholesky / LDL^T test.  Returns
// false on a pivot block that is not positive definite; otherwise sv is row r of -M.
__device__ __forceinline__ bool gn_sweep(double (&sv)[4], double* rk2, int r, int c0, bool act) {
  using namespace gn;
  bool bad = false;
#pragma unroll 1
  for (int k = 0; k < NV; k += 2) {
    if (act && (r >> 1) == (k >> 1)) {  // rows k, k + 1 -> the pivot-row buffer
      double* dst = rk2 + (r - k) * NV + c0;
      *reinterpret_cast<gn_d2*>(dst) = gn_d2{sv[0], sv[1]};
      *reinterpret_cast<gn_d2*>(dst + 2) = gn_d2{sv[2], sv[3]};
    }
    wave_order();
    const gn_d2 pa = *reinterpret_cast<const gn_d2*>(rk2 + k);  // S[k][k], S[k][k+1]
    const double pd = rk2[NV + k + 1];                          // S[k+1][k+1]
    const double u0 = rk2[r], u1 = rk2[NV + r];                 // S[r][k], S[r][k+1] (symmetric)
    const gn_d2 x0 = *reinterpret_cast<const gn_d2*>(rk2 + c0);
    const gn_d2 x1 = *reinterpret_cast<const gn_d2*>(rk2 + c0 + 2);
    const gn_d2 y0 = *reinterpret_cast<const gn_d2*>(rk2 + NV + c0);
    const gn_d2 y1 = *reinterpret_cast<const gn_d2*>(rk2 + NV + c0 + 2);
    const double vk[4] = {x0[0], x0[1], x1[0], x1[1]};   // S[k][c0 ..]
    const double vk1[4] = {y0[0], y0[1], y1[0], y1[1]};  // S[k+1][c0 ..]
    double a0 = pa[0], b0 = pa[1], d0 = pd;
    double det = a0 * d0 - b0 * b0;
    if (!(a0 > 0.0) || !(det > 0.0)) {
      bad = true;
      a0 = 1.0;
      b0 = 0.0;
      d0 = 1.0;
      det = 1.0;
    }
    const double id = gn_rcp(det);
    const double q00 = d0 * id, q01 = -b0 * id, q11 = a0 * id;  // P^-1 (symmetric)
    // one formula for every element (branch-free): with (al0, al1) = row r - k of P^-1
    // for the pivot rows and -(S_rK P^-1) otherwise,
    //   j not in K:  S'[r][j] = (r in K ? 0 : S[r][j]) + al0 S[k][j] + al1 S[k+1][j]
    //   j in K:      S'[r][j] = -(j == k ? al0 : al1)
    const bool rk = (r >> 1) == (k >> 1);
    const double al0 = rk ? (r == k ? q00 : q01) : -(u0 * q00 + u1 * q01);
    const double al1 = rk ? (r == k ? q01 : q11) : -(u0 * q01 + u1 * q11);
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      const int j = c0 + c;
      const double gen = fma(al0, vk[c], fma(al1, vk1[c], rk ? 0.0 : sv[c]));
      sv[c] = (j >> 1) == (k >> 1) ? -(j == k ? al0 : al1) : gen;
    }
  }
  return !bad;
}

// after a successful sweep: M (= -sv) and b to LDS, z = M b (returned on every lane for its row r)
__device__ __forceinline__ double gn_finish(const double (&sv)[4], double b, GnChainLds& C, int r, int c0, bool act) {
  using namespace gn;
  wave_order();
  if (act) {
    *reinterpret_cast<gn_d2*>(C.M + r * NV + c0) = gn_d2{-sv[0], -sv[1]};
    *reinterpret_cast<gn_d2*>(C.M + r * NV + c0 + 2) = gn_d2{-sv[2], -sv[3]};
    if (c0 == 0) C.bs[r] = b;
  }
  wave_order();
  double z0 = 0.0, z1 = 0.0;
#pragma unroll
  for (int j = 0; j < NV; j += 2) {
    z0 += C.M[r * NV + j] * C.bs[j];
    z1 += C.M[r * NV + j + 1] * C.bs[j + 1];
  }
  wave_order();
  if (act && c0 == 0) C.z[r] = z0 + z1;
  return z0 + z1;
}

// Back substitution along n frames f = f0, f0 + step, ..:  delta_f = z_f - G_f delta_prev
// (lane i < 12: row i).  G_f rows and z_f come from the workspace slot of f, loaded one frame
// ahead (two register sets), except the first frame's G (G0, LDS) when given; delta_prev
// starts as d0 (LDS) or, without one, the first frame has no coupling term.
// dl: 12 doubles of LDS scratch (this wave's).
__device__ __forceinline__ void gn_backsub(const double* ws, int f0, int step, int n, const double* G0,
                                           const double* d0, double* dl, double* delta, int i) {
  using namespace gn;
  if (n <= 0) return;
  const int ir = i < NV ? i : NV - 1;
  double Gn[NV], zn;
  auto ld = [&](int u) __attribute__((always_inline)) {
    const double* wn = ws + (size_t)(f0 + u * step) * GN_WSF;
    const double* gr = (u == 0 && G0) ? G0 + ir * NV : wn + ir * NV;
#pragma unroll
    for (int k = 0; k < NV; ++k) Gn[k] = gr[k];
    zn = wn[NB + ir];
  };
  if (d0 && i < NV) dl[i] = d0[i];
  wave_order();
  ld(0);
  for (int u = 0; u < n; ++u) {
    double Gc[NV];
#pragma unroll
    for (int k = 0; k < NV; ++k) Gc[k] = Gn[k];
    double d = zn;
    if (u + 1 < n) ld(u + 1);
    if (u > 0 || d0) {
      double e0 = 0.0, e1 = 0.0;
#pragma unroll
      for (int k = 0; k < NV; k += 2) {
        e0 += Gc[k] * dl[k];
        e1 += Gc[k + 1] * dl[k + 1];
      }
      d -= e0 + e1;
    }
    wave_order();
    if (i < NV) {
      dl[i] = d;
      delta[(size_t)(f0 + u * step) * NV + i] = d;
    }
    wave_order();
  }
}

// SOLVER = 1 (round 3): block Thomas with explicit inverses, so the per-frame chain has ONE
// 12-step sequence instead of three (W solve, Cholesky, y solve):
//   G_{l-1} = M_{l-1} E_{l-1}                   (M = S^-1; 12 x 12 x 12, no chain)
//   S_l = D_l + lambda I - E_{l-1}^T G_{l-1}    (no chain)
//   b_l = -g_l - E_{l-1}^T z_{l-1}
//   M_l = S_l^-1 by the symmetric sweep operator (12 pivots; the pivots are S_l's LDL^T
//          pivots, so a pivot <= 0 <=> S_l not positive definite, as the Cholesky test)
//   z_l = M_l b_l;  backward  delta_l = z_l - G_l delta_{l+1}  (one mat-vec per frame).
// 36 lanes hold a 12 x 12 block, lane i: row i / 3, columns 4 (i % 3) .. + 3; the sweep
// hands row k round through LDS (one wave: LDS ops run in order) and uses symmetry for
// column k.
template <int RP, int NA, int SOLVER>
__global__ __launch_bounds__(64 * (NA + 1), 3) void gn_step_kernel(GnArgs a) {
  using namespace gn;
  constexpr int BLK = 2 * NB + NV;  // D | E | g of one frame
  constexpr int R = NA + 2;
  __shared__ __attribute__((aligned(16))) GnStage<RP> st[NA];  // assembler staging
  __shared__ __attribute__((aligned(16))) double blk[R][BLK];   // frame ring
  __shared__ __attribute__((aligned(16))) double Lp[NB];        // L_{l-1}, row-major
  __shared__ double Ld[NV];                                     // 1 / L_{l-1}[i][i]
  __shared__ __attribute__((aligned(16))) double Wt[NB];        // W_l^T: row c = column c of W
  __shared__ __attribute__((aligned(16))) double ys[NV];        // y_{l-1}
  __shared__ int ready[R];
  __shared__ int consumed;
  const int t = blockIdx.x;
  const int wv = threadIdx.x >> 6;
  const int i = threadIdx.x & 63;
  const int L = a.L;
  const long f0 = (long)t * L;
  if (threadIdx.x < R) ready[threadIdx.x] = 0;
  if (threadIdx.x == 0) consumed = 0;
  __syncthreads();
  if (wv < NA) {
    for (int l = wv; l < L; l += NA) {
      while (lds_load_acquire(&consumed) < l - R + 2) __builtin_amdgcn_s_sleep(2);
      gn_stamp(a, t, 2 * l);  // assembler: frame l start (slot 2 l) / published (2 l + 1)
      gn_assemble_frame<RP>(a, f0 + l, st[wv], blk[l % R]);
      if (i == 0) lds_store_release(&ready[l % R], l + 1);
      gn_stamp(a, t, 2 * l + 1);
    }
    return;
  }
  double* ws = a.ws + (size_t)t * L * GN_WSF;
  int info = 0;
  if constexpr (SOLVER == 1) {
    // the solver's chain is the launch's critical path: it wins issue arbitration against
    // the assembler waves of its own and of the CU's other workgroups
    __builtin_amdgcn_s_setprio(3);
    __shared__ __attribute__((aligned(16))) GnChainLds C;
    const bool act = i < 36;
    const int ii = act ? i : 35;
    const int r = ii / 3, c0 = 4 * (ii - 3 * (ii / 3));
    for (int l = 0; l < L; ++l) {
      const int cur = l % R, prv = (l + R - 1) % R;
      gn_stamp(a, t, 64 + 4 * l);  // solver: frame l wait start / data ready / sweep start / done
      while (lds_load_acquire(&ready[cur]) != l + 1) __builtin_amdgcn_s_sleep(1);
      gn_stamp(a, t, 65 + 4 * l);
      if (!info) {
        const double* bc = blk[cur];
        double sv[4];
#pragma unroll
        for (int c = 0; c < 4; ++c) sv[c] = bc[r * NV + c0 + c] + (r == c0 + c ? a.lambda : 0.0);
        double b = -bc[2 * NB + r];
        if (l > 0)  // G_{l-1} = M_{l-1} E_{l-1} (to the workspace for the backward pass)
          gn_couple<false>(C.M, C.z, blk[prv] + NB, C.G, ws + (size_t)(l - 1) * GN_WSF, r, c0, act, sv, b);
        gn_stamp(a, t, 66 + 4 * l);
        if (!gn_sweep(sv, C.rk2, r, c0, act)) {
          info = l + 1;  // the solver wave idles through the remaining frames' hand-overs
        } else {
          const double z = gn_finish(sv, b, C, r, c0, act);
          if (act && c0 == 0) ws[(size_t)l * GN_WSF + NB + r] = z;
        }
      }
      if (i == 0) lds_store_release(&consumed, l + 1);
      gn_stamp(a, t, 67 + 4 * l);
    }
    gn_stamp(a, t, 250);
    if (!info) {
      // backward: delta_l = z_l - G_l delta_{l+1}, l = L - 1 .. 0
      gn_backsub(ws, L - 1, -1, L, nullptr, nullptr, C.bs, a.delta + (size_t)t * L * NV, i);
    } else {
      for (int e = i; e < L * NV; e += 64) a.delta[(size_t)t * L * NV + e] = NAN;
    }
    if (a.info && i == 0) a.info[t] = info;
    gn_stamp(a, t, 251);
    return;
  }
  const int ic = i < NV ? i : NV - 1;  // lanes >= 12 shadow row / column 11 (no stores)
  const bool act = i < NV;
  for (int l = 0; l < L; ++l) {
    const int cur = l % R, prv = (l + R - 1) % R;
    while (lds_load_acquire(&ready[cur]) != l + 1) __builtin_amdgcn_s_sleep(1);
    if (!info) {
      double* wl = ws + (size_t)l * GN_WSF;
      const double* bc = blk[cur];
      const double* bp = blk[prv];
      double S[NV];
#pragma unroll
      for (int j = 0; j < NV; ++j) S[j] = bc[ic * NV + j] + (j == ic ? a.lambda : 0.0);
      double rhs = -bc[2 * NB + ic];
      if (l > 0) {
        // W column ic: L_{l-1} w = E_{l-1}[:, ic]
        double w[NV];
#pragma unroll
        for (int k = 0; k < NV; ++k) {
          double s0 = bp[NB + k * NV + ic], s1 = 0.0;
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
        wave_lds_sync();
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
        info = l + 1;  // the solver wave idles through the remaining frames' barriers
      } else {
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
        wave_lds_sync();  // every lane is past its reads of Lp / Ld / Wt / ys
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
      }
    }
    if (i == 0) lds_store_release(&consumed, l + 1);
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

// SOLVER 2 (round 3, shipped): SOLVER 1's block Thomas elimination run from BOTH ends of the
// trajectory at once (twisted / "burn at both ends" factorization).  Frames 0 .. m - 1 are
// eliminated top-down by one solver wave and frames L - 1 .. m + 1 bottom-up by another, each
// fed by its own assembler wave and LDS ring (R = 3 slots, the SOLVER 1 protocol); the top
// solver then eliminates frame m against both neighbours,
//   Z_m = D_m + lambda I - E_{m-1}^T M_{m-1} E_{m-1} - E_m N_{m+1} E_m^T,
//   z_m = Z_m^-1 (-g_m - E_{m-1}^T z_{m-1} - E_m w_{m+1}) = delta_m,
// and the two back substitutions run outward from delta_m concurrently:
//   delta_l = z_l - G_l delta_{l+1} (l < m),   delta_l = w_l - H_l delta_{l-1} (l > m),
// H_l = N_l E_{l-1}^T.  The bottom chain is the top chain's algorithm on the mirrored problem
// (frame j = L - 1 - l, coupling block E'_{j-1} = E_l^T, read transposed from frame l's own
// slot: gn_couple<true>); the merge's extra term is one more gn_couple<true> with the bottom
// chain's N_{m+1}, w_{m+1} and frame m's E_m.  m = L / 2: the serial depth is L - m + 1 frame
// eliminations (13 at L = 24) instead of L.  Workspace slot l holds G_l, z_l (l <= m) or H_l,
// w_l (l > m).  Waves: 0 / 1 top / bottom assembler, 2 / 3 top / bottom solver.  info: the
// bottom chain's failed frame if it failed, else the top chain's (1-based; 0 = solved).
// OCC workgroups per CU: 4 (k loops unrolled by pairs, <= 128 VGPRs) for launches of more
// trajectories than 2 per CU, else 2 (fully unrolled, <= 256 VGPRs: a shorter solver chain)
template <int RP, int OCC = 4>
__global__ __launch_bounds__(256, OCC) void gn_twisted_kernel(GnArgs a) {
  constexpr int CU = OCC >= 4 ? GN_CU : 6;
  using namespace gn;
  constexpr int BLK = 2 * NB + NV;
  constexpr int R = 3;
  __shared__ __attribute__((aligned(16))) GnStage<RP> st[2];
  __shared__ __attribute__((aligned(16))) double blk[2][R][BLK];  // [chain][slot]
  __shared__ __attribute__((aligned(16))) GnChainLds ch[2];
  __shared__ __attribute__((aligned(16))) double Hm[NB];  // H_{m+1} = N_{m+1} E_m^T (the merge)
  __shared__ int ready[2][R];
  __shared__ int consumed[2];
  __shared__ int bdone, binfo, mdone;
  const int t = blockIdx.x;
  const int wv = threadIdx.x >> 6;
  const int i = threadIdx.x & 63;
  const int L = a.L;
  const int m = L / 2, nb = L - 1 - m;  // merge frame; bottom-chain frames L - 1 .. m + 1
  const long f0 = (long)t * L;
  if (threadIdx.x < 2 * R) (&ready[0][0])[threadIdx.x] = 0;
  if (threadIdx.x < 2) consumed[threadIdx.x] = 0;
  if (threadIdx.x == 0) {
    bdone = 0;
    binfo = 0;
    mdone = 0;
  }
  __syncthreads();
  if (wv < 2) {  // assembler of chain wv: top frames 0 .. m, bottom frames L - 1 .. m + 1
    // the next frame's loads are issued before the current frame is built, so the
    // factors' memory latency is off the chain
    const int n = wv == 0 ? m + 1 : nb;
    gn_zero_stage<RP>(st[wv]);
    // frame j + 1's loads are issued before frame j is built (an unrolled pair of load sets
    // without the copy measured the same, 83.1 vs 84.4 us, and needs more registers)
    GnFrameLoads<RP> ld0;
    if (n > 0) gn_load_frame<RP>(a, f0 + (wv == 0 ? 0 : L - 1), ld0);
    auto step = [&](int j, const GnFrameLoads<RP>& cu, GnFrameLoads<RP>& nx) __attribute__((always_inline)) {
      const int l = wv == 0 ? j : L - 1 - j;
      if (j + 1 < n) gn_load_frame<RP>(a, f0 + (wv == 0 ? l + 1 : l - 1), nx);
      while (lds_load_acquire(&consumed[wv]) < j - R + 2) __builtin_amdgcn_s_sleep(2);
      gn_stamp(a, t, 2 * l);
      gn_build_frame<RP, false>(a, f0 + l, cu, st[wv], blk[wv][j % R]);
      if (i == 0) lds_store_release(&ready[wv][j % R], j + 1);
      gn_stamp(a, t, 2 * l + 1);
    };
    for (int j = 0; j < n; ++j) {
      const GnFrameLoads<RP> cu = ld0;
      step(j, cu, ld0);
    }
    return;
  }
  const int sc = wv - 2;  // solver chain: 0 top, 1 bottom
  if (sc == 1 && nb == 0) return;
  __builtin_amdgcn_s_setprio(3);  // the solvers' chains are the launch's critical path
  double* ws = a.ws + (size_t)t * L * GN_WSF;
  double* delta = a.delta + (size_t)t * L * NV;
  GnChainLds& C = ch[sc];
  const bool act = i < 36;
  const int ii = act ? i : 35;
  const int r = ii / 3, c0 = 4 * (ii - 3 * (ii / 3));
  int info = 0;
  const int n = sc == 0 ? m + 1 : nb;
  for (int j = 0; j < n; ++j) {
    const int l = sc == 0 ? j : L - 1 - j;
    const int cur = j % R, prv = (j + R - 1) % R;
    gn_stamp(a, t, 64 + 4 * l);
    while (lds_load_acquire(&ready[sc][cur]) != j + 1) __builtin_amdgcn_s_sleep(1);
    gn_stamp(a, t, 65 + 4 * l);
    const double* bc = blk[sc][cur];
    const bool merge = sc == 0 && j == m && nb > 0;
    bool bfail = false;
    if (merge) {  // the bottom chain's N_{m+1}, w_{m+1} (or its failure)
      int bd;
      while ((bd = lds_load_acquire(&bdone)) == 0) __builtin_amdgcn_s_sleep(1);
      bfail = bd == 2;
    }
    if (!info && !bfail) {
      double sv[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) sv[c] = bc[r * NV + c0 + c] + (r == c0 + c ? a.lambda : 0.0);
      double b = -bc[2 * NB + r];
      if (j > 0) {
        if (sc == 0)  // G_{l-1} = M_{l-1} E_{l-1} -> workspace slot l - 1
          gn_couple_mfma<false>(C.M, C.z, blk[0][prv] + NB, nullptr, ws + (size_t)(l - 1) * GN_WSF, C.G, r, c0, sv, b);
        else  // H_{l+1} = N_{l+1} E_l^T -> workspace slot l + 1
          gn_couple_mfma<true>(C.M, C.z, bc + NB, nullptr, ws + (size_t)(l + 1) * GN_WSF, C.G, r, c0, sv, b);
      }
      if (merge) gn_couple_mfma<true>(ch[1].M, ch[1].z, bc + NB, Hm, nullptr, C.G, r, c0, sv, b);
      gn_stamp(a, t, 66 + 4 * l);
      if (!gn_sweep(sv, C.rk2, r, c0, act)) {
        info = l + 1;  // idles through the remaining frames' hand-overs
      } else {
        const double z = gn_finish(sv, b, C, r, c0, act);
        if (act && c0 == 0) ws[(size_t)l * GN_WSF + NB + r] = z;
      }
    }
    if (i == 0) lds_store_release(&consumed[sc], j + 1);
    gn_stamp(a, t, 67 + 4 * l);
  }
  if (sc == 1) {
    if (i == 0) {
      binfo = info;
      lds_store_release(&bdone, info ? 2 : 1);
    }
    int md;
    while ((md = lds_load_acquire(&mdone)) == 0) __builtin_amdgcn_s_sleep(1);
    gn_stamp(a, t, 252);
    if (md == 1)  // delta_l = w_l - H_l delta_{l-1}, l = m + 1 .. L - 1, from delta_m = z_m (top's C.z)
      gn_backsub(ws, m + 1, 1, nb, Hm, ch[0].z, C.bs, delta, i);
    else
      for (int e = i; e < nb * NV; e += 64) delta[(size_t)(m + 1) * NV + e] = NAN;
    gn_stamp(a, t, 253);
    return;
  }
  // top solver: final info (the bottom chain's failure first), release the bottom solver
  if (nb > 0) {
    int bd;
    while ((bd = lds_load_acquire(&bdone)) == 0) __builtin_amdgcn_s_sleep(1);
    if (bd == 2) info = lds_load_acquire(&binfo);
  }
  if (i == 0) lds_store_release(&mdone, info ? 2 : 1);
  gn_stamp(a, t, 250);
  if (!info)  // delta_l = z_l - G_l delta_{l+1}, l = m .. 0 (delta_m = z_m)
    gn_backsub(ws, m, -1, m + 1, nullptr, nullptr, C.bs, delta, i);
  else
    for (int e = i; e < (m + 1) * NV; e += 64) delta[e] = NAN;
  if (a.info && i == 0) a.info[t] = info;
  gn_stamp(a, t, 251);
}

// ---------------------------------------------------------------- cyclic reduction (few trajectories)
// At T = 3 (the streaming tick) the two-ended elimination above is a 13-frame serial chain on
// 3 CUs.  Block cyclic reduction cuts the serial depth to log2(L) levels by eliminating every
// other active frame at once.  One workgroup of 12 waves per trajectory, all blocks in LDS:
//   assembly   the waves build frames w, w + NS, .. (gn_build_frame) straight into fb[l] = D | E | g,
//              then S_l = D_l + lambda I, b_l = -g_l, C_l = E_l (the coupling to the next
//              active frame)
//   level      active frames a_0 .. a_{n-1}; n even: the odd positions are eliminated, n odd:
//              the even ones (so every eliminated frame's neighbours survive).  Eliminated i
//              with neighbours p < i < q (either may be absent):
//                M_i = S_i^-1 (gn_sweep: the PD test of the pivot), z_i = M_i b_i,
//                PM_i = C_p M_i,  QM_i = C_i^T M_i                    (one wave each)
//              then each survivor s with eliminated neighbours h < s < i and next survivor q:
//                S_s -= QM_h C_h + PM_i C_s^T,  b_s -= C_h^T z_h + C_s z_i,
//                C_s <- -PM_i C_i                                     (one wave each)
//   last       n = 1: delta = S^-1 b
//   back       levels in reverse: delta_i = z_i - PM_i^T delta_p - QM_i^T delta_q.
// L = 24: 5 sweeps in series (24 -> 12 -> 6 -> 3 -> 1 -> solve) instead of 13; about twice
// the flops of the elimination, so it is the form for launches that leave CUs idle.  The
// 12 x 12 products run on the f64 matrix cores.  info: the 1-based frame of the first
// level's (lowest) pivot block that is not positive definite, 0 = solved.
constexpr int GN_CR_LMAX = 24;
constexpr int GN_CR_W = 12;  // waves per workgroup
typedef double gn_d4 __attribute__((ext_vector_type(4)));

// acc += A B for 12 x 12 row-major LDS blocks (A read transposed when TA, B when TB), on the
// f64 matrix cores: A operand lane l = (row l & 15, k = l >> 4), B operand (k = l >> 4,
// column l & 15), result register v = (row (l >> 4) + 4 v, column l & 15); rows / columns
// 12..15 are zero padding
template <bool TA, bool TB>
__device__ __forceinline__ gn_d4 gn_mm_acc(const double* A, const double* B, gn_d4 acc) {
  using namespace gn;
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  const bool in = li < NV;
  const int lr = in ? li : 0;
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int k = 4 * q + lk;
    const double av = in ? (TA ? A[k * NV + lr] : A[lr * NV + k]) : 0.0;
    const double bv = in ? (TB ? B[lr * NV + k] : B[k * NV + lr]) : 0.0;
    acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av, bv, acc, 0, 0, 0);
  }
  return acc;
}

// a C-layout result to a 12 x 12 row-major LDS block (scaled by s)
__device__ __forceinline__ void gn_mm_store(double* out, const gn_d4& c, double s) {
  using namespace gn;
  const int lane = threadIdx.x & 63, li = lane & 15, lk = lane >> 4;
  if (li < NV)
#pragma unroll
    for (int v = 0; v < 3; ++v) out[(lk + 4 * v) * NV + li] = s * c[v];
}

// LDS of gn_cr_run: fb (S | C | b per frame) and the pool (assembly staging, then the level data)
template <int RP, int NS, bool ROOT = false>
struct GnCrLds {
  static constexpr int BLK = 2 * gn::NB + gn::NV;
  static constexpr int LM = GN_CR_LMAX, W = GN_CR_W;
  static constexpr int CHD = (int)(sizeof(GnChainLds) / sizeof(double));
  static constexpr int STGD = (int)(sizeof(GnStage<RP>) / sizeof(double));
  static constexpr int FR = 2 * gn::NB + gn::NV;
  static constexpr bool PAIR = !ROOT && NS == W && 2 * W >= LM;
  static constexpr int SLAB0 = 2 * FR + CHD > STGD ? 2 * FR + CHD : STGD;
  static constexpr int SLAB = (SLAB0 + 1) / 2 * 2;
  static constexpr int POST = LM * FR + W * CHD;
  static constexpr int STG = NS * STGD;
  static constexpr int POOL = PAIR ? W * SLAB : (POST > STG ? POST : STG);
};

// The split streaming tick (pa_window_pose_tick_pre / _post): per trajectory, what the pre
// half leaves for the post half in the workspace a.ws (doubles): per frame B_l | a_l (the
// back substitution run on the root's delta as an unknown: delta_l = a_l + B_l delta_root),
// the root's S | b, the failure word
constexpr int GN_TICK_FRD = gn::NB + gn::NV;
constexpr int GN_TICK_WSD = GN_CR_LMAX * GN_TICK_FRD + gn::NB + gn::NV + 2;

// the level lists: frames active at each level, the parity of the eliminated positions
// (pe), the level count.  Shipped order: n even -> the odd positions, n odd -> the even ones
// (PAIR: level 0 the odd ones whatever the parity).  ROOT (the split tick): n even -> the
// even positions, n odd -> the odd ones, so position n - 1, frame L - 1, is never eliminated
// and stays as the root of the reduction (24 -> 12 -> 6 -> 3 -> 2 -> 1: one level more).
template <bool PAIR, bool ROOT>
__device__ __forceinline__ int gn_cr_lists(int L, signed char (*lst)[GN_CR_LMAX], int* lcnt, int* lpe) {
  int n = L, lv = 0;
  for (int l = 0; l < L; ++l) lst[0][l] = (signed char)l;
  while (n > 1) {
    const int pe = ROOT ? (n & 1) : ((PAIR && lv == 0) || !(n & 1) ? 1 : 0);
    int m = 0;
    for (int p = 0; p < n; ++p)
      if ((p & 1) != pe) lst[lv + 1][m++] = lst[lv][p];
    lcnt[lv] = n;
    lpe[lv] = pe;
    n = m;
    ++lv;
  }
  lcnt[lv] = 1;
  return lv;
}

// trajectory t on this workgroup (64 * GN_CR_W threads); fb / pool: GnCrLds<RP, NS, ROOT> in LDS.
// ROOT (pa_window_pose_tick_pre): the ROOT level order, and after the last level the reduced
// system goes to the workspace (GN_TICK_WSD per trajectory) instead of being solved.
template <int RP, int NS, bool ROOT = false>
__device__ __forceinline__ void gn_cr_run(const GnArgs& a, int t, double (*fb)[2 * gn::NB + gn::NV], double* pool) {
  using namespace gn;
  constexpr int BLK = 2 * NB + NV;
  constexpr int LM = GN_CR_LMAX, W = GN_CR_W;
  constexpr int CHD = (int)(sizeof(GnChainLds) / sizeof(double));
  constexpr int STGD = (int)(sizeof(GnStage<RP>) / sizeof(double));
  constexpr int FR = 2 * NB + NV;  // per eliminated frame: PM | QM | z
  // PAIR (one assembler wave per two frames, NS = W): wave w builds frames 2w, 2w + 1 and
  // eliminates 2w + 1 at once (level 0 eliminates the odd positions whatever L's parity), so
  // level 0 needs no barrier of its own.  Its slab of the pool is its staging, then the
  // PM | QM | z of frames 2w + 1 and 2w and its sweep scratch.  Otherwise (the general-K
  // instance: its staging does not fit 12 times) NS waves assemble, then every wave starts.
  constexpr bool PAIR = !ROOT && NS == W && 2 * W >= LM;
  constexpr int SLAB0 = 2 * FR + CHD > STGD ? 2 * FR + CHD : STGD;
  constexpr int SLAB = (SLAB0 + 1) / 2 * 2;
  constexpr int POST = LM * FR + W * CHD;
  constexpr int STG = NS * STGD;
  constexpr int POOL = PAIR ? W * SLAB : (POST > STG ? POST : STG);
  constexpr int NOFAIL = 0x7fffffff;
  static_assert(NS <= W, "assembler waves");
  static_assert(POOL == GnCrLds<RP, NS, ROOT>::POOL && BLK == GnCrLds<RP, NS, ROOT>::BLK, "LDS layout");
  __shared__ signed char lst[8][LM];  // active frames per level
  __shared__ int lcnt[8], lpe[8];
  __shared__ int nlev_s, fail;
  const int wv = threadIdx.x >> 6;
  const int i = threadIdx.x & 63;
  const int L = a.L;
  const long f0 = (long)t * L;
  auto fr = [&](int f) __attribute__((always_inline)) -> double* {  // PM | QM | z of frame f
    return PAIR ? pool + (f >> 1) * SLAB + ((f & 1) ? 0 : FR) : pool + f * FR;
  };
  GnChainLds& C = *reinterpret_cast<GnChainLds*>(PAIR ? pool + wv * SLAB + 2 * FR : pool + LM * FR + wv * CHD);
  auto dl = [&](int f) __attribute__((always_inline)) -> double* { return fb[f]; };
  if (threadIdx.x == 0) {
    nlev_s = gn_cr_lists<PAIR, ROOT>(L, lst, lcnt, lpe);
    fail = NOFAIL;
  }
  // the level lists and `fail` are in place before any wave eliminates or reads them (LDS
  // holds whatever the previous kernel left: an unsynchronised read of nlev_s gave waves
  // different level counts, i.e. different barrier counts -- a hang)
  __syncthreads();
  if (wv == 0) gn_stamp(a, t, 0);
  const bool act = i < 36;
  const int ii = act ? i : 35;
  const int r = ii / 3, c0 = 4 * (ii - 3 * (ii / 3));
  // eliminate frame fi (neighbours fp, fq, or -1): M = S^-1 (false if S is not PD), z = M b,
  // PM = C_p M, QM = C_fi^T M
  auto eliminate = [&](int fi, int fp, int fq) __attribute__((always_inline)) {
    double sv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) sv[c] = fb[fi][r * NV + c0 + c];
    const double b = fb[fi][2 * NB + r];
    if (!gn_sweep(sv, C.rk2, r, c0, act)) {
      if (i == 0) __hip_atomic_fetch_min(&fail, fi + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      return;
    }
    double* o = fr(fi);
    const double z = gn_finish(sv, b, C, r, c0, act);  // C.M = M
    if (act && c0 == 0) o[2 * NB + r] = z;
    if (fp >= 0) gn_mm_store(o, gn_mm_acc<false, false>(fb[fp] + NB, C.M, gn_d4{0, 0, 0, 0}), 1.0);
    if (fq >= 0) gn_mm_store(o + NB, gn_mm_acc<true, false>(fb[fi] + NB, C.M, gn_d4{0, 0, 0, 0}), 1.0);
  };
  // S = D + lambda I, b = -g (frame l; lanes < 12 of one wave)
  auto init = [&](int l) __attribute__((always_inline)) {
    if (i < NV) {
      fb[l][i * NV + i] += a.lambda;
      fb[l][2 * NB + i] = -fb[l][2 * NB + i];
    }
  };
  if constexpr (PAIR) {
    // ---- wave w: frames 2w, 2w + 1 (both loads issued before either is built), then the
    // level-0 elimination of 2w + 1
    const int la = 2 * wv, lb = 2 * wv + 1;
    if (la < L) {
      GnStage<RP>& st = *reinterpret_cast<GnStage<RP>*>(pool + wv * SLAB);
      gn_zero_stage<RP>(st);
      GnFrameLoads<RP> ld0, ld1;
      gn_load_frame<RP>(a, f0 + la, ld0);
      if (lb < L) gn_load_frame<RP>(a, f0 + lb, ld1);
      gn_build_frame<RP, false>(a, f0 + la, ld0, st, fb[la]);
      if (lb < L) gn_build_frame<RP, false>(a, f0 + lb, ld1, st, fb[lb]);
      wave_order();
      init(la);
      if (lb < L) init(lb);
      wave_order();
      if (wv == 0) gn_stamp(a, t, 2);
      if (lb < L) eliminate(lb, la, lb + 1 < L ? lb + 1 : -1);  // (the staging is dead: the slab's new use)
    }
  } else {
    if (wv < NS) {
      GnStage<RP>& st = reinterpret_cast<GnStage<RP>*>(pool)[wv];
      gn_zero_stage<RP>(st);
      GnFrameLoads<RP> ld0;
      if (wv < L) gn_load_frame<RP>(a, f0 + wv, ld0);
      for (int l = wv; l < L; l += NS) {
        const GnFrameLoads<RP> cu = ld0;
        if (l + NS < L) gn_load_frame<RP>(a, f0 + l + NS, ld0);
        gn_build_frame<RP, false>(a, f0 + l, cu, st, fb[l]);
      }
      if (wv == 0) gn_stamp(a, t, 2);
    }
    __syncthreads();
    for (int l = wv; l < L; l += W) init(l);
  }
  __syncthreads();
  const int nlev = nlev_s;  // (after a barrier: thread 0 wrote it)
  if (wv == 0) gn_stamp(a, t, 1);
  int lv = 0;
  for (; lv < nlev; ++lv) {
    const int n = lcnt[lv], pe = lpe[lv];
    const int ne = pe ? n / 2 : (n + 1) / 2;
    if (!(PAIR && lv == 0)) {
      for (int e = wv; e < ne; e += W) {  // eliminated frames
        const int pos = 2 * e + pe;
        eliminate(lst[lv][pos], pos > 0 ? lst[lv][pos - 1] : -1, pos + 1 < n ? lst[lv][pos + 1] : -1);
      }
      __syncthreads();
    }
    if (wv == 0) gn_stamp(a, t, 10 + 2 * lv);
    if (fail != NOFAIL) break;
    const int ns = n - ne;
    for (int s = wv; s < ns; s += W) {  // survivors
      const int pos = 2 * s + (1 - pe);
      const int fs = lst[lv][pos];
      const int fh = pos > 0 ? lst[lv][pos - 1] : -1;
      const int fi = pos + 1 < n ? lst[lv][pos + 1] : -1;
      const bool cq = fi >= 0 && pos + 2 < n;  // a next survivor: new coupling
      gn_d4 acc = {0.0, 0.0, 0.0, 0.0}, cn = {0.0, 0.0, 0.0, 0.0};
      if (fh >= 0) acc = gn_mm_acc<false, false>(fr(fh) + NB, fb[fh] + NB, acc);
      if (fi >= 0) acc = gn_mm_acc<false, true>(fr(fi), fb[fs] + NB, acc);
      if (cq) cn = gn_mm_acc<false, false>(fr(fi), fb[fi] + NB, cn);
      double db0 = 0.0, db1 = 0.0;
      if (i < NV) {
        if (fh >= 0) {
          const double* zh = fr(fh) + 2 * NB;
#pragma unroll
          for (int k = 0; k < NV; ++k) db0 += fb[fh][NB + k * NV + i] * zh[k];
        }
        if (fi >= 0) {
          const double* zi = fr(fi) + 2 * NB;
#pragma unroll
          for (int k = 0; k < NV; ++k) db1 += fb[fs][NB + i * NV + k] * zi[k];
        }
      }
      wave_order();  // this wave's reads of fb[fs] are issued before its writes
      const int li = i & 15, lk = i >> 4;
      if (li < NV)
#pragma unroll
        for (int v = 0; v < 3; ++v) fb[fs][(lk + 4 * v) * NV + li] -= acc[v];
      if (cq) gn_mm_store(fb[fs] + NB, cn, -1.0);
      if (i < NV) fb[fs][2 * NB + i] -= db0 + db1;
    }
    __syncthreads();
    if (wv == 0) gn_stamp(a, t, 11 + 2 * lv);
  }
  if constexpr (ROOT) {
    // the root (frame L - 1) S | b and the failure word to the workspace, then the back
    // substitution with delta_root unknown: delta_l = a_l + B_l delta_root, B_root = I, a_root = 0,
    //   B_i = -(PM_i^T B_p + QM_i^T B_q),  a_i = z_i - PM_i^T a_p - QM_i^T a_q
    // level by level in reverse (the products on the f64 matrix cores), into fb[l] (its S and C
    // are dead): B_l | a_l, then to the workspace
    constexpr int FD = GN_TICK_FRD;
    double* w = a.ws + (size_t)t * GN_TICK_WSD;
    const int rt = L - 1;
    for (int e = threadIdx.x; e < NB + NV; e += 64 * W) w[LM * FD + e] = e < NB ? fb[rt][e] : fb[rt][NB + e];
    if (threadIdx.x == 0) reinterpret_cast<int*>(w + LM * FD + NB + NV)[0] = fail == NOFAIL ? 0 : fail;
    if (fail != NOFAIL) return;  // (uniform: read after the last level's barrier)
    __syncthreads();  // every read of the root's S | b is done
    for (int e = threadIdx.x; e < FD; e += 64 * W) fb[rt][e] = (e < NB && e % (NV + 1) == 0) ? 1.0 : 0.0;
    __syncthreads();
    for (lv = nlev - 1; lv >= 0; --lv) {
      const int n = lcnt[lv], pe = lpe[lv];
      const int ne = pe ? n / 2 : (n + 1) / 2;
      for (int e = wv; e < ne; e += W) {
        const int pos = 2 * e + pe;
        const int fi = lst[lv][pos];
        const int fp = pos > 0 ? lst[lv][pos - 1] : -1, fq = pos + 1 < n ? lst[lv][pos + 1] : -1;
        const double* o = fr(fi);
        gn_d4 acc = {0.0, 0.0, 0.0, 0.0};
        if (fp >= 0) acc = gn_mm_acc<true, false>(o, fb[fp], acc);
        if (fq >= 0) acc = gn_mm_acc<true, false>(o + NB, fb[fq], acc);
        double av = 0.0;
        if (i < NV) {
          double d0 = o[2 * NB + i], d1 = 0.0;
          if (fp >= 0)
#pragma unroll
            for (int k = 0; k < NV; ++k) d0 -= o[k * NV + i] * fb[fp][NB + k];
          if (fq >= 0)
#pragma unroll
            for (int k = 0; k < NV; ++k) d1 += o[NB + k * NV + i] * fb[fq][NB + k];
          av = d0 - d1;
        }
        gn_mm_store(fb[fi], acc, -1.0);  // (fb[fi] is this wave's alone; nothing above reads it)
        if (i < NV) fb[fi][NB + i] = av;
      }
      __syncthreads();
    }
    for (int e = threadIdx.x; e < L * FD / 2; e += 64 * W) {
      const int l = e / (FD / 2), c = e - l * (FD / 2);
      reinterpret_cast<gn_d2*>(w + l * FD)[c] = reinterpret_cast<const gn_d2*>(fb[l])[c];
    }
    return;
  }
  if (fail == NOFAIL && wv == 0) {  // the last active frame: delta = S^-1 b (over its S block)
    const int ff = lst[nlev][0];
    double sv[4];
#pragma unroll
    for (int c = 0; c < 4; ++c) sv[c] = fb[ff][r * NV + c0 + c];
    const double b = fb[ff][2 * NB + r];
    if (!gn_sweep(sv, C.rk2, r, c0, act)) {
      if (i == 0) __hip_atomic_fetch_min(&fail, ff + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    } else {
      const double z = gn_finish(sv, b, C, r, c0, act);
      wave_order();  // every lane's S reads are done
      if (act && c0 == 0) dl(ff)[r] = z;
    }
  }
  __syncthreads();
  if (wv == 0) gn_stamp(a, t, 30);
  const int info = fail == NOFAIL ? 0 : fail;
  if (!info) {
    for (lv = nlev - 1; lv >= 0; --lv) {  // delta_i over S_i's first row (dead since its elimination)
      const int n = lcnt[lv], pe = lpe[lv];
      const int ne = pe ? n / 2 : (n + 1) / 2;
      for (int e = wv; e < ne; e += W) {
        const int pos = 2 * e + pe;
        const int fi = lst[lv][pos];
        const int fp = pos > 0 ? lst[lv][pos - 1] : -1, fq = pos + 1 < n ? lst[lv][pos + 1] : -1;
        const double* o = fr(fi);
        if (i < NV) {
          double d0 = o[2 * NB + i], d1 = 0.0;
          if (fp >= 0)
#pragma unroll
            for (int k = 0; k < NV; ++k) d0 -= o[k * NV + i] * dl(fp)[k];
          if (fq >= 0)
#pragma unroll
            for (int k = 0; k < NV; ++k) d1 += o[NB + k * NV + i] * dl(fq)[k];
          dl(fi)[i] = d0 - d1;
        }
      }
      __syncthreads();
      if (wv == 0) gn_stamp(a, t, 31 + lv);
    }
  }
  double* delta = a.delta + (size_t)f0 * NV;
  for (int e = threadIdx.x; e < L * NV; e += 64 * W) {
    const int l = e / NV;
    delta[e] = info ? NAN : dl(l)[e - l * NV];
  }
  if (a.info && threadIdx.x == 0) a.info[t] = info;
  if (wv == 0) gn_stamp(a, t, 40);
}

template <int RP, int NS>
__global__ __launch_bounds__(64 * GN_CR_W, 1) void gn_cr_kernel(GnArgs a) {
  using Ld = GnCrLds<RP, NS>;
  __shared__ __attribute__((aligned(16))) double fb[Ld::LM][Ld::BLK];
  __shared__ __attribute__((aligned(16))) double pool[Ld::POOL];
  gn_cr_run<RP, NS>(a, blockIdx.x, fb, pool);
}

// ---------------------------------------------------------------- the streaming pose tick, fused
// pa_window_pose_tick: one tick's pose stage (config 4) as two launches instead of four, one
// workgroup per trajectory (camera) in each:
//   pose_tick_lin_kernel (6 waves)  advance: window_advance_body (the window shifts, y_new
//        lands, frame L-1 predicted); linearize: the trajectory's factors as a T = 1 view --
//        waves 0-1 its L-1 dynamics factors (traj_dyn_block), then one wave per 256
//        projection factors and one for the constant-velocity ones (traj_unit_wave)
//   pose_tick_gn_kernel (12 waves)  the GN step (gn_cr_run, block cyclic reduction), then the
//        retract (window_retract_one per frame, the newest pose to `newest`)
// (One 12-wave launch for all four would hold the dynamics factors' ~220 VGPRs at three waves
// per SIMD: 240 spilled.)  Every phase is its separate kernel's device code, so the window,
// the factors, delta, info and the newest poses are bit for bit the four-launch sequence's
// (tests/test_streaming_pose_gpu.py).
constexpr int TICK_LIN_W = 6;
// y_new null (the split tick's pre half): the window advances without the new keypoints, and
// frame L - 1's projection factors (evaluated on the stale keypoints the slot still holds)
// are marked status 3 afterwards, so the GN assembly gives them zero rows; the post half
// evaluates them on y_new.
__global__ __launch_bounds__(64 * TICK_LIN_W) void pose_tick_lin_kernel(pa_traj_args ta, const float* __restrict__ y_new) {
  static_assert((trj::STAGE + 4 * trj::UNIT) * 8 <= 96 * 1024, "factor staging");
  __shared__ __attribute__((aligned(16))) double st[trj::STAGE + 4 * trj::UNIT];
  const int t = blockIdx.x, L = ta.L, K = ta.n_kp, wv = threadIdx.x >> 6;
  window_advance_body(t, threadIdx.x, 64 * TICK_LIN_W, L, K, y_new, const_cast<float*>(ta.y),
                      const_cast<double*>(ta.pose), const_cast<double*>(ta.angvel), const_cast<double*>(ta.vel), ta.dt,
                      ta.vel_frame, const_cast<int32_t*>(ta.nvalid));
  __syncthreads();
  // trajectory t's factors: the arrays of a T = 1 problem start at its records
  pa_traj_args a1 = ta;
  {
    const long f0 = (long)t * L, p0 = f0 * K, d0 = (long)t * (L - 1);
    auto off = [](auto* q, long n) { return q ? q + n : q; };
    a1.T = 1;
    a1.y = ta.y + f0 * 2 * K;
    a1.pose = ta.pose + f0 * 12;
    a1.vel = ta.vel + f0 * 3;
    a1.angvel = ta.angvel + f0 * 3;
    a1.r_proj = off(ta.r_proj, p0 * 2);
    a1.j_proj = off(ta.j_proj, p0 * 12);
    a1.err_proj = off(ta.err_proj, p0);
    a1.status = off(ta.status, p0);
    a1.r_dyn = off(ta.r_dyn, d0 * 6);
    a1.j_dyn0 = off(ta.j_dyn0, d0 * 36);
    a1.j_dyn1 = off(ta.j_dyn1, d0 * 18);
    a1.j_dyn2 = off(ta.j_dyn2, d0 * 18);
    a1.j_dyn3 = off(ta.j_dyn3, d0 * 36);
    a1.err_dyn = off(ta.err_dyn, d0);
    a1.r_cv = off(ta.r_cv, d0 * 3);
    a1.j_cv0 = off(ta.j_cv0, d0 * 9);
    a1.j_cv1 = off(ta.j_cv1, d0 * 9);
    a1.err_cv = off(ta.err_cv, d0);
    a1.nvalid = off(ta.nvalid, (long)t);
  }
  const int wp = (L * K + 64 * trj::PPW - 1) / (64 * trj::PPW);  // projection units (<= 2); unit wp: constant velocity
  if (wv < 2) {
    traj_dyn_block(a1, 0, st, nullptr);  // (its one LDS barrier is matched by every other wave's below)
  } else {
    if (wv - 2 <= wp) traj_unit_wave(a1, wv - 2, st + trj::STAGE + (wv - 2) * trj::UNIT, nullptr);
    lds_barrier();
  }
  if (!y_new) {  // (uniform)
    __syncthreads();  // the unit waves' status stores come first
    if ((int)threadIdx.x < K) a1.status[(long)(L - 1) * K + threadIdx.x] = 3;
  }
}

template <int RP>
__global__ __launch_bounds__(64 * GN_CR_W, 1) void pose_tick_gn_kernel(GnArgs g, double* pose, double* angvel,
                                                                        double* vel, double* newest) {
  constexpr int NS = RP <= 34 ? 12 : 8;
  using Ld = GnCrLds<RP, NS>;
  __shared__ __attribute__((aligned(16))) double fb[Ld::LM][Ld::BLK];
  __shared__ __attribute__((aligned(16))) double pool[Ld::POOL];
  const int t = blockIdx.x, L = g.L;
  gn_cr_run<RP, NS>(g, t, fb, pool);
  __syncthreads();
  if ((int)threadIdx.x < L)
    window_retract_one((long)t * L + threadIdx.x, L, g.delta, g.info, pose, angvel, vel, newest);
}

// The split tick.  pa_window_pose_tick_pre (before the keypoints exist: it runs beside the
// detector forward on a second stream of the tick's graph) = pose_tick_lin_kernel(null) +
// pose_tick_pre_kernel: every factor but the newest frame's projections, assembled and
// reduced by cyclic reduction in the ROOT order down to frame L - 1 alone.  A projection
// factor touches only its own frame's diagonal block, and the root's S and b enter the
// reduction only additively (no elimination reads them), so the newest frame's projection
// rows can be added to the reduced root at the end:
//   pose_tick_post_kernel  y_new lands in the window, its K projection factors (the factor
//        outputs, as the linearize writes them), S_root += Jp^T Jp and b_root -= Jp^T rp on the
//        pose block, delta_root = S_root^-1 b_root, back substitution, delta / info, retract.
// The same normal equations as pa_window_pose_tick, another elimination order and f64
// rounding (tests/test_streaming_pose_gpu.py: within 1e-9 of its delta).
template <int RP>
__global__ __launch_bounds__(64 * GN_CR_W, 1) void pose_tick_pre_kernel(GnArgs g) {
  constexpr int NS = RP <= 34 ? 12 : 8;
  using Ld = GnCrLds<RP, NS, true>;
  __shared__ __attribute__((aligned(16))) double fb[Ld::LM][Ld::BLK];
  __shared__ __attribute__((aligned(16))) double pool[Ld::POOL];
  gn_cr_run<RP, NS, true>(g, blockIdx.x, fb, pool);
}

__global__ __launch_bounds__(64 * GN_CR_W, 1) void pose_tick_post_kernel(pa_traj_args ta, const float* __restrict__ y_new,
                                                                          const double* __restrict__ ws, double* delta,
                                                                          int32_t* info, double* newest) {
  using namespace gn;
  constexpr int KP = 2 * GN_KMAX, FD = GN_TICK_FRD, LM = GN_CR_LMAX;
  __shared__ __attribute__((aligned(16))) double dl[LM][NV];   // delta per frame
  __shared__ __attribute__((aligned(16))) double sr[NB + NV];  // the root's S | b
  __shared__ __attribute__((aligned(16))) double jt[7][KP];    // newest frame: Jp^T (6 x 2K) | rp
  __shared__ __attribute__((aligned(16))) GnChainLds C;
  __shared__ int fail_s;
  const int t = blockIdx.x, L = ta.L, K = ta.n_kp, ny = 2 * K;
  const int wv = threadIdx.x >> 6, i = threadIdx.x & 63;
  const long f0 = (long)t * L, fn = f0 + L - 1;
  const double* w = ws + (size_t)t * GN_TICK_WSD;
  // thread (l, r) < L x 12: row r of B_l and a_l[r], loaded first (in flight with the rest)
  const int tl = (int)threadIdx.x / NV, tr = (int)threadIdx.x - tl * NV;
  const bool brow = tl < L;
  double bv[NV], av = 0.0;
  if (brow) {
    const double* src = w + tl * FD;
#pragma unroll
    for (int k = 0; k < NV; k += 2) {
      const gn_d2 v = *reinterpret_cast<const gn_d2*>(src + tr * NV + k);
      bv[k] = v[0];
      bv[k + 1] = v[1];
    }
    av = src[NB + tr];
  }
  for (int e = threadIdx.x; e < NB + NV; e += 64 * GN_CR_W) sr[e] = w[LM * FD + e];
  if (threadIdx.x == 0) fail_s = reinterpret_cast<const int*>(w + LM * FD + NB + NV)[0];
  double s = 0.0;  // wave 0, lane o < 42: entry o of [Jp^T Jp | Jp^T rp] (6 x 7, row-major)
  if (wv == 0) {
    // y_new lands (pa_window_advance's last step) and frame L - 1's projection factors:
    // lane k, traj_unit_wave's evaluation
    if (i < ny) const_cast<float*>(ta.y)[fn * ny + i] = y_new[(size_t)t * ny + i];
    if (i < K) {
      const Cam cam = load_cam(ta.K, ta.tcam, ta.isig_proj);
      const Pose T = load_pose(ta.pose + fn * 12);
      const V3 pb = load3(ta.corners + 3 * i);
      const float px = kornia_denorm(y_new[(size_t)t * ny + 2 * i], ta.W);
      const float py = kornia_denorm(y_new[(size_t)t * ny + 2 * i + 1], ta.H);
      const bool off = ta.nvalid ? L - 1 < L - ta.nvalid[t] : false;
      double r[2], J[12], e;
      int32_t st;
      proj_eval(T, pb, (double)px, (double)py, cam, r, J, e, st);
      if (off) {
        r[0] = r[1] = 0.0;
#pragma unroll
        for (int c = 0; c < 12; ++c) J[c] = 0.0;
        e = 0.0;
        st = 2;
      }
      const long u = fn * K + i;
      ta.r_proj[u * 2] = r[0];
      ta.r_proj[u * 2 + 1] = r[1];
#pragma unroll
      for (int c = 0; c < 12; ++c) ta.j_proj[u * 12 + c] = J[c];
      if (ta.err_proj) ta.err_proj[u] = e;
      ta.status[u] = st;
      // the GN assembly's rows: a failed projection (status != 0) gives zero rows
#pragma unroll
      for (int c = 0; c < 6; ++c) {
        jt[c][2 * i] = st == 0 ? J[c * 2] : 0.0;
        jt[c][2 * i + 1] = st == 0 ? J[c * 2 + 1] : 0.0;
      }
      jt[6][2 * i] = st == 0 ? r[0] : 0.0;
      jt[6][2 * i + 1] = st == 0 ? r[1] : 0.0;
    }
    wave_order();
    if (i < 42) {
      const int ra = i < 36 ? i / 6 : i - 36, cb = i < 36 ? i - 6 * (i / 6) : 6;
      for (int q = 0; q < ny; ++q) s += jt[ra][q] * jt[cb][q];
    }
  }
  __syncthreads();  // the root's S | b, the failure word
  if (wv == 0) {
    // the newest frame's projections into the root (S += Jp^T Jp on the pose block, b -= Jp^T rp)
    if (i < 36) sr[(i / 6) * NV + i - 6 * (i / 6)] += s;
    else if (i < 42) sr[NB + i - 36] -= s;
    wave_order();
    if (fail_s == 0) {  // delta_root = S^-1 b
      const bool act = i < 36;
      const int ii = act ? i : 35;
      const int r = ii / 3, c0 = 4 * (ii - 3 * (ii / 3));
      double sv[4];
#pragma unroll
      for (int c = 0; c < 4; ++c) sv[c] = sr[r * NV + c0 + c];
      const double b = sr[NB + r];
      if (!gn_sweep(sv, C.rk2, r, c0, act)) {
        if (i == 0) fail_s = L;
      } else {
        const double z = gn_finish(sv, b, C, r, c0, act);
        wave_order();
        if (act && c0 == 0) dl[L - 1][r] = z;
      }
    }
  }
  __syncthreads();
  const int inf = fail_s;
  // every frame at once: delta_l = a_l + B_l delta_root
  double dv = NAN;
  if (brow && !inf) {
    double d0 = av, d1 = 0.0;
#pragma unroll
    for (int k = 0; k < NV; k += 2) {
      d0 += bv[k] * dl[L - 1][k];
      d1 += bv[k + 1] * dl[L - 1][k + 1];
    }
    dv = d0 + d1;
  }
  __syncthreads();  // every read of delta_root is done
  if (brow) {
    dl[tl][tr] = dv;
    delta[(size_t)f0 * NV + threadIdx.x] = dv;
  }
  if (threadIdx.x == 0) info[t] = inf;
  __syncthreads();
  if ((int)threadIdx.x < L)
    window_retract_frame(f0 + threadIdx.x, L, dl[threadIdx.x], inf == 0, const_cast<double*>(ta.pose),
                         const_cast<double*>(ta.angvel), const_cast<double*>(ta.vel), newest);
}

// assembler waves per trajectory and solver (pa_debug_gn_set_assemblers: na + 8 * legacy;
// 0 = the shipped choice)
static int g_gn_na = 0;
// CUs of the CURRENT device (cached per device id: a host with GPUs of different CU counts
// gets each one's own); only the cyclic-reduction vs two-ended choice in launch_gn uses it
static int g_gn_cus() {
  static int cache[64] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) return 256;
  if (dev < 64 && cache[dev] > 0) return cache[dev];
  int n = 0;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  if (dev < 64) cache[dev] = n;
  return n;
}
static unsigned long long* g_gn_trace = nullptr;

template <int RP, int SV>
static void launch_gn_sv(const GnArgs& a, int na, hipStream_t s) {
  switch (na) {
    case 1: hipLaunchKernelGGL((gn_step_kernel<RP, 1, SV>), dim3(a.T), dim3(64 * 2), 0, s, a); break;
    case 3: hipLaunchKernelGGL((gn_step_kernel<RP, 3, SV>), dim3(a.T), dim3(64 * 4), 0, s, a); break;
    case 4: hipLaunchKernelGGL((gn_step_kernel<RP, 4, SV>), dim3(a.T), dim3(64 * 5), 0, s, a); break;
    default: hipLaunchKernelGGL((gn_step_kernel<RP, 2, SV>), dim3(a.T), dim3(64 * 3), 0, s, a); break;
  }
}

// shipped: solver 2 (the two-ended elimination); v & 16 selects solver 1 (one top-down chain of
// swept inverses) and v & 8 the round-2 block Cholesky, both with v & 7 assembler waves
// cyclic reduction for launches of few trajectories (v & 64 forces it, v & 128 never)
template <int RP>
static void launch_gn(const GnArgs& a, int v, hipStream_t s) {
  v &= 255;
  const bool cr_ok = a.L <= GN_CR_LMAX && !(v & 63);
  // (T x 24, us, two-ended / cyclic: 3: 41.3 / 33.4, 64: 41.9 / 33.9, 256: 42.6 / 34.4,
  // 512: 54.1 / 66.6, 1000: 71.3 / 130.8; profiles/r04i/gn_cr_ab.log)
  if (cr_ok && ((v & 64) || (!(v & 128) && a.T <= g_gn_cus())))
    hipLaunchKernelGGL((gn_cr_kernel<RP, RP <= 34 ? 12 : 8>), dim3(a.T), dim3(64 * GN_CR_W), 0, s, a);
  else if (v & 8)
    launch_gn_sv<RP, 0>(a, v & 7, s);
  else if (v & 16)
    launch_gn_sv<RP, 1>(a, v & 7, s);
  else if ((v & 32) || a.T > 2 * g_gn_cus())  // 32: force the 4-per-CU form
    hipLaunchKernelGGL((gn_twisted_kernel<RP, 4>), dim3(a.T), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL((gn_twisted_kernel<RP, 2>), dim3(a.T), dim3(256), 0, s, a);
}

}  // namespace pa

extern "C" {

int pa_debug_gn_set_trace(unsigned long long* trace_dev) {
  pa::g_gn_trace = trace_dev;
  return PA_OK;
}

int pa_debug_gn_set_assemblers(int na) {
  PA_CHECK((na & 7) <= 4 && na >= 0 && na < 4096 && !((na & 8) && (na & 16)) && !((na & 64) && (na & 128)),
           "gn variant %d: assembler waves (0..4) + 8 * legacy Cholesky or 16 * single-chain solver, 32: "
           "two-ended kernel in its 4-per-CU form, 64: cyclic reduction (L <= 24), 128: never cyclic "
           "reduction; pa_window_pose_tick debugging: 1024 its linearize launch only, 2048 its GN launch only",
           na);
  pa::g_gn_na = na;
  return PA_OK;
}

int pa_window_pose_tick(const pa_traj_args* ta, const float* y_new, double lambda, double* delta, int32_t* info,
                        double* newest_pose, void* stream) {
  PA_CHECK(ta && y_new && delta && info, "pose tick: null args / y_new / delta / info");
  const int T = ta->T, L = ta->L, K = ta->n_kp;
  // one workgroup per trajectory: correct at any T (the CU count is a performance choice of the
  // caller, StreamingPipeline's fused_pose / split_pose eligibility)
  PA_CHECK(T >= 0 && L >= 2 && L <= pa::GN_CR_LMAX && K >= 0 && K <= pa::GN_KMAX,
           "pose tick: T %d, L %d (2..%d), n_kp %d (<= %d)", T, L, pa::GN_CR_LMAX, K, pa::GN_KMAX);
  if (T == 0) return PA_OK;
  PA_CHECK(lambda >= 0.0, "pose tick: lambda %g < 0", lambda);
  PA_CHECK(ta->y && ta->pose && ta->vel && ta->angvel && ta->corners && ta->K && ta->nvalid,
           "pose tick: null window / model pointer");
  PA_CHECK((K == 0 || (ta->r_proj && ta->j_proj && ta->status)) && ta->r_dyn && ta->j_dyn0 && ta->j_dyn1 &&
               ta->j_dyn2 && ta->j_dyn3 && ta->r_cv && ta->j_cv0 && ta->j_cv1,
           "pose tick: the factor outputs and every Jacobian are required");
  const pa::GnArgs g{T,     L,     K,     ta->r_proj, ta->j_proj, ta->status, ta->r_dyn, ta->j_dyn0,
                     ta->j_dyn1, ta->j_dyn2, ta->j_dyn3, ta->r_cv, ta->j_cv0, ta->j_cv1, lambda, nullptr,
                     nullptr, nullptr, delta, info, nullptr, nullptr};
  const hipStream_t s = (hipStream_t)stream;
  if (!(pa::g_gn_na & 2048)) hipLaunchKernelGGL(pa::pose_tick_lin_kernel, dim3(T), dim3(64 * pa::TICK_LIN_W), 0, s, *ta, y_new);
  if (pa::g_gn_na & 1024) { PA_LAUNCH_CHECK(); return PA_OK; }
  double* pose = const_cast<double*>(ta->pose);
  double* angvel = const_cast<double*>(ta->angvel);
  double* vel = const_cast<double*>(ta->vel);
  if (K == 8)
    hipLaunchKernelGGL(pa::pose_tick_gn_kernel<34>, dim3(T), dim3(64 * pa::GN_CR_W), 0, s, g, pose, angvel, vel,
                       newest_pose);
  else
    hipLaunchKernelGGL(pa::pose_tick_gn_kernel<2 * pa::GN_KMAX + 18>, dim3(T), dim3(64 * pa::GN_CR_W), 0, s, g, pose,
                       angvel, vel, newest_pose);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

size_t pa_window_pose_tick_workspace(int T, int L) {
  return (T > 0 && L > 0) ? (size_t)T * pa::GN_TICK_WSD * sizeof(double) : 0;
}

// the checks of pa_window_pose_tick
static int pose_tick_check(const pa_traj_args* ta, const char* who) {
  PA_CHECK(ta, "%s: null args", who);
  const int T = ta->T, L = ta->L, K = ta->n_kp;
  PA_CHECK(T >= 0 && L >= 2 && L <= pa::GN_CR_LMAX && K >= 0 && K <= pa::GN_KMAX,
           "%s: T %d, L %d (2..%d), n_kp %d (<= %d)", who, T, L, pa::GN_CR_LMAX, K, pa::GN_KMAX);
  PA_CHECK(ta->y && ta->pose && ta->vel && ta->angvel && ta->corners && ta->K && ta->nvalid,
           "%s: null window / model pointer", who);
  PA_CHECK((K == 0 || (ta->r_proj && ta->j_proj && ta->status)) && ta->r_dyn && ta->j_dyn0 && ta->j_dyn1 &&
               ta->j_dyn2 && ta->j_dyn3 && ta->r_cv && ta->j_cv0 && ta->j_cv1,
           "%s: the factor outputs and every Jacobian are required", who);
  return PA_OK;
}

int pa_window_pose_tick_pre(const pa_traj_args* ta, double lambda, void* ws, size_t ws_bytes, void* stream) {
  const int rc = pose_tick_check(ta, "pose tick pre");
  if (rc != PA_OK) return rc;
  const int T = ta->T, L = ta->L, K = ta->n_kp;
  if (T == 0) return PA_OK;
  PA_CHECK(lambda >= 0.0, "pose tick pre: lambda %g < 0", lambda);
  PA_CHECK(ws && ws_bytes >= pa_window_pose_tick_workspace(T, L), "pose tick pre: workspace %zu < %zu", ws_bytes,
           pa_window_pose_tick_workspace(T, L));
  const pa::GnArgs g{T,     L,     K,     ta->r_proj, ta->j_proj, ta->status, ta->r_dyn, ta->j_dyn0,
                     ta->j_dyn1, ta->j_dyn2, ta->j_dyn3, ta->r_cv, ta->j_cv0, ta->j_cv1, lambda, nullptr,
                     nullptr, nullptr, nullptr, nullptr, (double*)ws, nullptr};
  const hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(pa::pose_tick_lin_kernel, dim3(T), dim3(64 * pa::TICK_LIN_W), 0, s, *ta, nullptr);
  if (K == 8)
    hipLaunchKernelGGL(pa::pose_tick_pre_kernel<34>, dim3(T), dim3(64 * pa::GN_CR_W), 0, s, g);
  else
    hipLaunchKernelGGL(pa::pose_tick_pre_kernel<2 * pa::GN_KMAX + 18>, dim3(T), dim3(64 * pa::GN_CR_W), 0, s, g);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

int pa_window_pose_tick_post(const pa_traj_args* ta, const float* y_new, const void* ws, size_t ws_bytes,
                             double* delta, int32_t* info, double* newest_pose, void* stream) {
  const int rc = pose_tick_check(ta, "pose tick post");
  if (rc != PA_OK) return rc;
  const int T = ta->T, L = ta->L;
  if (T == 0) return PA_OK;
  PA_CHECK(y_new && delta && info, "pose tick post: null y_new / delta / info");
  PA_CHECK(ws && ws_bytes >= pa_window_pose_tick_workspace(T, L), "pose tick post: workspace %zu < %zu", ws_bytes,
           pa_window_pose_tick_workspace(T, L));
  hipLaunchKernelGGL(pa::pose_tick_post_kernel, dim3(T), dim3(64 * pa::GN_CR_W), 0, (hipStream_t)stream, *ta, y_new,
                     (const double*)ws, delta, info, newest_pose);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

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
  PA_CHECK(delta && ws, "gn: null delta / workspace pointer");
  PA_CHECK((!D && !E && !g) || (D && g && (L == 1 || E)), "gn: D, E, g are given together (or all NULL)");
  PA_CHECK(n_kp == 0 || (r_proj && j_proj), "gn: null projection factors");
  PA_CHECK(L == 1 || (r_dyn && j_dyn0 && j_dyn1 && j_dyn2 && j_dyn3 && r_cv && j_cv0 && j_cv1),
           "gn: null dynamics / constant-velocity factors (Jacobians are required)");
  PA_CHECK(ws_bytes >= pa_trajectory_gn_workspace(T, L), "gn: workspace %zu < %zu", ws_bytes,
           pa_trajectory_gn_workspace(T, L));
  const pa::GnArgs a{T,     L,      n_kp,   r_proj, j_proj, status_proj, r_dyn, j_dyn0, j_dyn1, j_dyn2, j_dyn3,
                     r_cv,  j_cv0,  j_cv1,  lambda, D,      E,           g,     delta,  info,   (double*)ws,
                     pa::g_gn_trace};
  const hipStream_t s = (hipStream_t)stream;
  if (n_kp == 8)
    pa::launch_gn<34>(a, pa::g_gn_na, s);
  else
    pa::launch_gn<2 * pa::GN_KMAX + 18>(a, pa::g_gn_na, s);
  PA_LAUNCH_CHECK();
  return PA_OK;
}

}  // extern "C"
