/*
 * perseus_amd — C ABI of the MI355X keypoint-inference path (libperseus_amd.so).
 *
 * Plain pointers and sizes only; every array argument named *_dev is a device
 * pointer (hipMalloc / torch CUDA tensor storage) owned by the caller, every
 * `stream` is a hipStream_t passed as void* (NULL = default stream).  All entry
 * points return 0 on success and a negative PA_E* code on failure, with a
 * thread-local message in pa_last_error().  Nothing here synchronises the
 * stream; results are ready when the caller's stream work completes.
 *
 * Reference interfaces replaced (paths relative to pculbertson/perseus):
 *   detector  perseus/detector/models.py:6-40   KeypointCNN.__init__/forward
 *             perseus/detector/validate.py:92-98 ckpt load ("module." strip) + eval
 *   factors   perseus/smoother/factors.py:54-142  PoseDynamicsFactor.error_func
 *             perseus/smoother/factors.py:160-171 ConstantVelocityFactor.error_func
 *             perseus/smoother/factors.py:216-275 KeypointProjectionFactor.error_func
 */
#ifndef PERSEUS_AMD_H
#define PERSEUS_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PA_OK 0
#define PA_EINVAL -1   /* bad argument (shape, size, null pointer)           */
#define PA_EHIP -2     /* HIP runtime error (message has hipGetErrorString)   */
#define PA_ENOMEM -3   /* device allocation failed                            */

#define PA_PREC_FP16 0   /* fp16 NHWC activations/weights, fp32 MFMA accumulate     */
#define PA_PREC_FP32 1   /* fp32 NHWC, exact-f32 MFMA (reference parity mode)     */
#define PA_PREC_FP16X3 2 /* fast parity mode: hi/lo fp16 planes, 3 fp16 MFMA products
                            per MAC (x_hi w_hi + x_lo w_hi + x_hi w_lo), f32 accumulate */

#define PA_VEL_WORLD 0 /* factors.py:41 vel_frame="world" */
#define PA_VEL_BODY 1  /* vel_frame="body"                */

const char* pa_last_error(void);
const char* pa_version(void);

/* ------------------------------------------------------------------ detector */
typedef struct pa_detector pa_detector;

/* Replaces KeypointCNN(n_keypoints, num_channels, H, W) + load_state_dict + eval()
 * (models.py:9-32, validate.py:92-98).
 * weights: HOST f32 blob = the state-dict float tensors in torchvision resnet18
 * order with the "resnet." prefix and without the 20 num_batches_tracked
 * counters (conv1.weight [64,C,7,7]; bn1.{weight,bias,running_mean,running_var};
 * layer1.0.conv1.weight ... ; fc.weight [2K,512]; fc.bias [2K]) — 102 tensors,
 * nbytes must equal the sum of their sizes.  BatchNorm (eps 1e-5) is folded and
 * weights are packed for the GPU here, once.  Only H = W = 256 and
 * 1 <= in_ch <= 4 are supported (the trained configurations). */
int pa_detector_create(const float* weights, size_t nbytes, int in_ch, int n_kp, int H, int W,
                       pa_detector** out);
void pa_detector_destroy(pa_detector* d);

/* Pre-size the activation workspace for batches up to max_batch (clamped to the
 * 1,024-frame chunk a forward runs in), and for 4-channel models in fp16x3 / fp32 also
 * forward_rgbd's f32 input staging (a later set_precision keeps the reservation).
 * Without it, allocation is done lazily by the first call of a larger batch, which
 * frees the smaller buffer: capture a graph only after reserve() (or after an eager
 * call of the same batch), and reserve the largest batch any graph will replay. */
int pa_detector_reserve(pa_detector* d, int max_batch);

/* PA_PREC_FP16 (default), PA_PREC_FP32 or PA_PREC_FP16X3. */
int pa_detector_set_precision(pa_detector* d, int precision);

/* Latency mode for small batches (the streaming pose stage, streaming.py:101-166: one
 * frame per camera per tick).  fp16 and fp16x3 forwards whose whole batch is
 * B <= max_batch frames run the stem on short bands, layer1 on small tiles and the convs
 * of layers 2-4 as split-K launches + a fixed-order reduce (layer2's stride-2 entry, with
 * 64 input channels, on one-tile workgroups instead), which fills the chip at a few
 * frames (deterministic, but not bit-identical to the batched kernels: the f32 sums are
 * taken in another order; fp16x3 stays within its 1e-3 px parity bar).  Allocates
 * max_batch MiB of partials.  max_batch = 0 (default) turns it off; at most 64. */
int pa_detector_set_split_k(pa_detector* d, int max_batch);

/* Replaces KeypointCNN.forward (models.py:34-40): x (B,C,H,W) f32 NCHW contiguous
 * on the device -> y (B, 2K) f32, y[:,2k] = x_k, y[:,2k+1] = y_k in [-1,1]
 * normalized image coordinates.  B = 0 is a no-op. */
int pa_detector_forward(pa_detector* d, const float* x_dev, int B, float* y_dev, void* stream);

/* Camera frames -> keypoints: uint8 HWC RGB (bgr != 0: BGR byte order, as
 * the ZED delivers) + f32 depth in metres, both [B][Hs][Ws], centre-cropped to 256x256;
 * pa_preprocess_rgbd's arithmetic (streaming.py:68-80, deterministic near/far clip, < 0 =
 * off).  fp16: applied inside the stem's row loads, so the f32 (B,4,256,256) input is never
 * written; fp16x3 / fp32: the preprocess kernel into the handle's own f32 staging (sized by
 * pa_detector_reserve, else by the first call of a larger batch), then the forward.  Output
 * bit-identical to pa_preprocess_rgbd + pa_detector_forward.  4-channel models only. */
int pa_detector_forward_rgbd(pa_detector* d, const uint8_t* rgb_dev, const float* depth_dev, int B, int Hs, int Ws,
                             int bgr, float near_m, float far_m, float* y_dev, void* stream);

/* pa_detector_forward_rgbd + pa_keypoints_postprocess (no target) in the same launches:
 * the head also writes the pixel coordinates px (B, n_kp, 2) f32, kornia's denormalize
 * (streaming.py:128-131), bit-identical to the separate postprocess.  The streaming
 * tick's detector call (one launch fewer per tick). */
int pa_detector_forward_rgbd_px(pa_detector* d, const uint8_t* rgb_dev, const float* depth_dev, int B, int Hs, int Ws,
                                int bgr, float near_m, float far_m, float* y_dev, float* px_dev, void* stream);
/* The device address of a mapped pinned host buffer (hipHostGetDevicePointer): forward_rgbd
 * may read the camera frames straight from host memory over PCIe (zero-copy), so a tick
 * needs no H2D copy before the stem (StreamingPipeline(zero_copy=True)). */
int pa_host_device_pointer(const void* host, void** dev);

/* Same forward with a HIP event after every kernel: writes up to max_n per-kernel
 * durations (ms) into ms_out and their names into names_out (may be NULL), returns
 * the number of kernels or <0.  Synchronises the stream (diagnostics only). */
int pa_detector_profile(pa_detector* d, const float* x_dev, int B, float* y_dev, void* stream,
                        float* ms_out, const char** names_out, int max_n);

/* Average device time of ONE launch of the forward (index in pa_detector_profile
 * order): the forward runs once with that launch issued `reps` times back to back
 * between two HIP events on `stream`.  y_dev and the activations are scratch
 * afterwards (an in-place residual launch accumulates); run a normal forward before
 * using outputs.  Test/measurement entry point, not part of the drop-in surface. */
int pa_detector_time_launch(pa_detector* d, const float* x_dev, int B, float* y_dev, void* stream, int index,
                            int reps, float* avg_ms_out, const char** name_out);

/* Algorithmic FLOPs of one frame's forward (2 x MAC over the 20 convs + fc). */
double pa_detector_flops_per_frame(const pa_detector* d);

/* Fused preprocessing (streaming.py:59-82, augmentations.py:128-169
 * val mode): RGB uint8 (B,Hs,Ws,3, BGR if bgr) + f32 depth metres (B,Hs,Ws),
 * centre crop to H x W, rgb/255, depth nan/inf -> 0, depth/0.035, then the
 * deterministic near/far clip (scaled depth < near or > far -> 0; pass near<0 /
 * far<0 to skip) -> x (B,4,H,W) f32 NCHW on the device. */
int pa_preprocess_rgbd(const uint8_t* rgb_dev, const float* depth_dev, int B, int Hs, int Ws, int bgr,
                       float near_m, float far_m, int H, int W, float* x_dev, void* stream);

/* Keypoint post-processing on device (validate.py:130-153): px = (n+1)(S-1)/2 into
 * px_dev (B,K,2); if target_dev != NULL (B,2K normalized), SmoothL1(beta=1) per
 * element into loss_dev (B,2K). */
int pa_keypoints_postprocess(const float* y_dev, const float* target_dev, int B, int n_kp, int H, int W,
                             float* px_dev, float* loss_dev, void* stream);

/* Validation loss statistics (validate.py:162-168, the "Validation Loss" block):
 * over n f32 losses on the device, stats_dev[0..4] (f64, device) = mean, stdev
 * (unbiased, torch.std; NaN for n = 1), min, max, median (torch.median: the
 * element of sorted index (n-1)/2).  ws_dev: device scratch of
 * pa_loss_statistics_workspace(n) bytes, 16-byte aligned.  Stream-ordered, no
 * host sync.  n must be > 0 (torch.median raises on an empty tensor). */
size_t pa_loss_statistics_workspace(long long n);
int pa_loss_statistics(const float* loss_dev, long long n, double* stats_dev, void* ws_dev, size_t ws_bytes,
                       void* stream);

/* ------------------------------------------------------------------- factors */
/* Pose encoding: 12 f64 per pose = R row-major (9) then t (3).  Jacobians are
 * column-major per factor (Eigen/GTSAM order), tangent order [omega; v].
 * inv_sigma (may be NULL): per-dimension 1/sigma of a diagonal noise model; when
 * given, r and every J are whitened in place (A = J/sigma, r_w = r/sigma) and
 * err_dev[i] = 0.5 * ||r_w||^2 (GTSAM NoiseModelFactor::error). err_dev may be NULL. */

/* KeypointProjectionFactor (factors.py:216-275): r = pi(K, Tcam^-1 Tbody p_b) - z,
 * J = d r / d Tbody (2x6).  K = (fx, fy, s, u0, v0); k_stride / tcam_stride = 0
 * share one K / camera pose across factors, 5 / 12 give one per factor; tcam_dev
 * NULL = identity camera (factors.py:211).  status[i] = 1 on cheirality (point
 * behind the camera: GTSAM CheiralityException), r and J then hold NaN. */
int pa_proj_linearize(int n, const double* tbody_dev, const double* pb_dev, const double* z_dev,
                      const double* k_dev, int k_stride, const double* tcam_dev, int tcam_stride,
                      const double* inv_sigma_dev, double* r_dev, double* j_dev, double* err_dev,
                      int32_t* status_dev, void* stream);

/* PoseDynamicsFactor (factors.py:54-142): r = Log((T1 Exp(dt[w; v_b]))^-1 T2),
 * v_b = R1^T v if vel_frame == PA_VEL_WORLD.  J0 6x6 (pose1), J1 6x3 (ang_vel1),
 * J2 6x3 (vel1), J3 6x6 (pose2); any J pointer may be NULL (error-only). */
int pa_dyn_linearize(int n, const double* t1_dev, const double* w_dev, const double* v_dev,
                     const double* t2_dev, double dt, int vel_frame, const double* inv_sigma_dev,
                     double* r_dev, double* j0_dev, double* j1_dev, double* j2_dev, double* j3_dev,
                     double* err_dev, void* stream);

/* ConstantVelocityFactor (factors.py:160-171): r = v2 - v1, J0 = -I3, J1 = I3. */
int pa_cv_linearize(int n, const double* v1_dev, const double* v2_dev, const double* inv_sigma_dev,
                    double* r_dev, double* j0_dev, double* j1_dev, double* err_dev, void* stream);

/* Config 3: every factor of T trajectories x L frames in ONE launch,
 * keypoint measurements taken straight from the detector output y (B = T*L rows of
 * 2K normalized coordinates, denormalized on device as validate.py:144-153 does).
 * Per frame f (= t*L + l): K projection factors (corner k: p_b = corners[k], z =
 * pixel k of frame f, body pose pose[f]); per consecutive pair (l, l+1) of a
 * trajectory: one PoseDynamicsFactor (pose[f], angvel[f], vel[f], pose[f+1]) and
 * one ConstantVelocityFactor (vel[f], vel[f+1]).  Outputs use the per-factor
 * layouts of the batched entry points above; proj arrays have T*L*K rows, dyn
 * and cv arrays T*(L-1).  inv_sigma / err / J / status pointers may be NULL.
 * nvalid (may be NULL): per trajectory the number of trailing frames that hold a real
 * measurement (the streaming window before it has filled, pa_window_advance_n); the
 * projection factors of frames l < L - nvalid[t] get status 2 and r = J = err = 0, so the
 * GN step skips them. */
typedef struct pa_traj_args {
  int T, L, n_kp, H, W;
  const float* y;          /* (T*L, 2K) normalized keypoints */
  const double* pose;      /* (T*L, 12) */
  const double* vel;       /* (T*L, 3) linear velocity (vel_frame) */
  const double* angvel;    /* (T*L, 3) body angular velocity */
  const double* corners;   /* (K, 3) body-frame keypoints */
  const double* K;         /* (5) fx, fy, s, u0, v0 */
  const double* tcam;      /* (12) camera pose or NULL = identity */
  double dt;
  int vel_frame;
  const double* isig_proj; /* (2) or NULL */
  const double* isig_dyn;  /* (6) or NULL */
  const double* isig_cv;   /* (3) or NULL */
  double *r_proj, *j_proj, *err_proj;
  int32_t* status;
  double *r_dyn, *j_dyn0, *j_dyn1, *j_dyn2, *j_dyn3, *err_dyn;
  double *r_cv, *j_cv0, *j_cv1, *err_cv;
  const int32_t* nvalid;   /* (T) or NULL: frames with measurements, from the window's end */
} pa_traj_args;

int pa_trajectory_linearize(const pa_traj_args* args, void* stream);

/* Factor-graph consumer (the graph and optimizer are not in the
 * reference -- GTSAM's LM runs on the host -- so this build defines them): one damped
 * Gauss-Newton / LM step per trajectory from pa_trajectory_linearize's WHITENED outputs
 * (same layouts; every Jacobian required).  Per frame the variable block is
 * x = [pose tangent (6, [omega; v]) | angular velocity (3) | velocity (3)]; the step
 * solves (J^T J + lambda I) delta = -J^T r.  Outputs: D (T*L, 12, 12) diagonal and
 * E (T*(L-1), 12, 12) off-diagonal blocks of J^T J (E_l couples frame l rows with
 * frame l+1 columns), g (T*L, 12) = J^T r, delta (T*L, 12), info (T) = 0 or the
 * 1-based frame of a pivot block found not positive definite (delta NaN; which frame
 * depends on the elimination order: launches of few trajectories with L <= 24 run block
 * cyclic reduction, others a two-ended block elimination).  D, E and g
 * may all be NULL (then the blocks stay on chip: the step's HBM traffic is the factors in
 * and delta out).  Projection factors with status != 0 (cheirality, or a frame outside a
 * window's filled part) are skipped; with n_kp = 0 r_proj / j_proj may be NULL.
 * ws: pa_trajectory_gn_workspace. */
size_t pa_trajectory_gn_workspace(int T, int L);
int pa_trajectory_gn_step(int T, int L, int n_kp, const double* r_proj, const double* j_proj,
                          const int32_t* status_proj, const double* r_dyn, const double* j_dyn0,
                          const double* j_dyn1, const double* j_dyn2, const double* j_dyn3, const double* r_cv,
                          const double* j_cv0, const double* j_cv1, double lambda, double* D, double* E, double* g,
                          double* delta, int32_t* info, void* ws, size_t ws_bytes, void* stream);

/* Fixed-lag window of the config-4 streaming pose stage (the smoother loop the reference
 * leaves to downstream GTSAM code; scripts/streaming.py:121-155 runs the detector only).
 * Per trajectory t the window holds frames l = 0..L-1 of y (T*L, 2K) f32, pose (T*L, 12),
 * angvel and vel (T*L, 3), all device, frame f = t*L + l.
 * pa_window_advance: shifts every array one frame towards l = 0 (frame 0 dropped),
 * writes y_new[t] (T, 2K) as frame L-1 and predicts pose[L-1] = pose[L-2] Exp(dt [w; v_b])
 * (the PoseDynamicsFactor model, factors.py:100-105; v_b = R^T v for PA_VEL_WORLD), v = vel
 * of frame L-2 carried over and w = the angular velocity frame L-2 held before the shift
 * (the newest one a factor constrains; L >= 3), which frames L-2 and L-1 both take.
 * pa_window_retract: pose <- pose Exp(delta[0:6]) (Pose3 retract, Expmap chart),
 * angvel += delta[6:9], vel += delta[9:12] for pa_trajectory_gn_step's delta (T*L, 12);
 * trajectories with info[t] != 0 are left unchanged (info may be NULL). */
int pa_window_advance(int T, int L, int n_kp, const float* y_new_dev, float* y_dev, double* pose_dev,
                      double* angvel_dev, double* vel_dev, double dt, int vel_frame, void* stream);
/* pa_window_advance that also counts the window's real frames: nvalid_dev (T) int32 += 1 up
 * to L per advance (zero it with the window's reset; pa_traj_args.nvalid reads it). */
int pa_window_advance_n(int T, int L, int n_kp, const float* y_new_dev, float* y_dev, double* pose_dev,
                        double* angvel_dev, double* vel_dev, int32_t* nvalid_dev, double dt, int vel_frame,
                        void* stream);
int pa_window_retract(int T, int L, const double* delta_dev, const int32_t* info_dev, double* pose_dev,
                      double* angvel_dev, double* vel_dev, void* stream);
/* pa_window_retract that also writes each trajectory's newest (last-frame) pose after the
 * update to newest_pose_dev (T, 12) -- the streaming tick's pose output, no strided gather. */
int pa_window_retract_newest(int T, int L, const double* delta_dev, const int32_t* info_dev, double* pose_dev,
                             double* angvel_dev, double* vel_dev, double* newest_pose_dev, void* stream);

/* One streaming tick's pose stage (config 4) in two launches, bit for bit the sequence
 * pa_window_advance_n(y_new) -> pa_trajectory_linearize(args) -> pa_trajectory_gn_step
 * (lambda; delta, info; D / E / g not written) -> pa_window_retract_newest(newest_pose).
 * args: the window's pa_traj_args (args->y / pose / vel / angvel ARE the window arrays,
 * advanced and retracted in place; nvalid required; every factor output and Jacobian
 * required, whitening as the caller wants it for the GN step).  T <= the device's CU count,
 * 2 <= L <= 24, n_kp <= 16 (PA_EINVAL otherwise: use the four calls). */
int pa_window_pose_tick(const pa_traj_args* args, const float* y_new_dev, double lambda, double* delta_dev,
                        int32_t* info_dev, double* newest_pose_dev, void* stream);

/* The same tick split around the keypoints, so that most of it runs before they exist (the
 * streaming graph runs the pre half on a second stream beside the detector forward):
 *   pa_window_pose_tick_pre: the window advances WITHOUT the new keypoints, every factor but
 *     frame L-1's projections is linearized (those are marked status 3 for now), and the GN
 *     system is assembled and reduced by block cyclic reduction down to frame L-1 (the root),
 *     into ws (pa_window_pose_tick_workspace bytes);
 *   pa_window_pose_tick_post: y_new lands as frame L-1's keypoints, its projection factors
 *     are linearized into the factor outputs (as pa_trajectory_linearize writes them), added
 *     to the reduced root, and the step is solved (delta, info) and retracted (newest_pose).
 * Pre then post on the same window = pa_window_pose_tick up to f64 rounding (another
 * elimination order; the window's keypoints and factor outputs are bit-identical; info names
 * a frame whose pivot failed in that order).  Same limits as pa_window_pose_tick. */
size_t pa_window_pose_tick_workspace(int T, int L);
int pa_window_pose_tick_pre(const pa_traj_args* args, double lambda, void* ws_dev, size_t ws_bytes, void* stream);
int pa_window_pose_tick_post(const pa_traj_args* args, const float* y_new_dev, const void* ws_dev, size_t ws_bytes,
                             double* delta_dev, int32_t* info_dev, double* newest_pose_dev, void* stream);

#ifdef __cplusplus
}
#endif
#endif /* PERSEUS_AMD_H */
