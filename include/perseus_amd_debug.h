/*
 * perseus_amd — tuning / measurement hooks of libperseus_amd.so.  Not part of the
 * drop-in surface (include/perseus_amd.h); nothing in production calls these.
 * Both settings belong to one pa_detector handle and apply to that handle's
 * forwards only (another handle in the same process keeps its own).
 */
#ifndef PERSEUS_AMD_DEBUG_H
#define PERSEUS_AMD_DEBUG_H

#include "perseus_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Interleaved A/B timing (tools/layer_ab.py, tools/head_ab.py): select kernel variant
 * `variant` for layer 1..4 (stage), 0 (stem), 5-7 (stride-2 entry / head options);
 * 0 = the shipped choice. */
int pa_detector_debug_set_variant(pa_detector* d, int layer, int variant);
/* Variants that give wrong results by construction (timing experiments) exist only in a
 * measurement build (PERSEUS_AMD_TIMING_VARIANTS=1 when building); the release library
 * returns PA_EINVAL for their ids (checked before the handle).  1 in a measurement build. */
int pa_debug_timing_variants_built(void);

/* Timestamping kernel variants write s_memrealtime stamps (100 MHz) to
 * trace_dev + launch * 65536 + workgroup * 64 (launch = index in the forward, stem = 0);
 * NULL turns it off. */
int pa_detector_debug_set_trace(pa_detector* d, unsigned long long* trace_dev);

/* Timing only: pa_trajectory_linearize with mode 1 = only the dynamics workgroups,
 * 2 = only the projection / constant-velocity workgroups (the other outputs are left
 * unwritten); mode 0 is pa_trajectory_linearize itself.  A non-NULL trace_dev (8 u64
 * per wave, 2 waves per workgroup) receives s_memrealtime stamps at each wave's phases. */
int pa_debug_trajectory_linearize(const pa_traj_args* args, int mode, unsigned long long* trace_dev, void* stream);

/* Timing / debugging only, process-wide: pa_trajectory_gn_step variant = assembler waves
 * per trajectory (1..4; 0 = the shipped count) + 8: the round-2 block-Cholesky solver, 16:
 * the single-chain swept-inverse solver, 32: the two-ended kernel's 4-per-CU form, 64: block
 * cyclic reduction forced (L <= 24), 128: never cyclic reduction; pa_window_pose_tick: 1024
 * launches its linearize kernel only, 2048 its GN kernel only. */
int pa_debug_gn_set_assemblers(int na);
/* Timing only: pa_trajectory_gn_step writes s_memrealtime stamps (100 MHz), 256 per
 * trajectory, to trace_dev (assembler frame l: slots 2l, 2l+1; solver frame l: 64+4l ..
 * 67+4l; solver-1 backward 250, 251); NULL turns it off.  Process-wide. */
int pa_debug_gn_set_trace(unsigned long long* trace_dev);

#ifdef __cplusplus
}
#endif
#endif /* PERSEUS_AMD_DEBUG_H */
