// Host-side launchers, one set per robot, each compiled in its own translation unit
// (pbg_robot.hip with -DPBG_ROBOT=<Name>) so the five template instantiations build in
// parallel.  pbg_capi.hip dispatches on the robot id.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

namespace pbg {
struct Buffers;
struct StepIO;
struct ResetIO;

struct Geometry {
  int team;          // lanes per env: 1 (step_kernel), 4 (team_step_kernel, pbg_team.hip) or
                     // 16 / 32 (gang_step_kernel, pbg_gang.hip)
  int block;         // lanes per step workgroup: 16, 32 or 64
  int lds_rows;      // contact-constraint rows (gang: contacts) resident in LDS per env
  int env_words;     // gang: LDS words per env
  int gang_dist;     // gang: distributed (1) or replicated (0) unconstrained dynamics
  int force_dist;    // in: -1 = plan's choice, 0 / 1 = force gang_dist (pbg_create_debug)
  int gang_lanes;    // in: -1 = plan's choice, 16 / 32 = gang width (pbg_create_debug)
  size_t lds_bytes;  // dynamic LDS per step workgroup
  size_t scratch_words_per_env;
  int vgprs;          // the selected step kernel's registers per lane (hipFuncGetAttributes)
  int scratch_bytes;  // and its private segment per lane
  int word_bytes = 4; // bytes per constraint-row / workspace word: 4 (float32 kernels) or 8 (float64)
};

#define PBG_DECLARE_ROBOT(NAME)                                                                            \
  int plan_##NAME(int n_envs, int cus, int mode, Geometry* g);                                                       \
  int launch_step_##NAME(const Buffers& B, const StepIO& io, float* scratch, const Geometry& g, hipStream_t s); \
  int launch_reset_##NAME(const Buffers& B, const ResetIO& io, hipStream_t s);                             \
  int launch_get_state_##NAME(const Buffers& B, double* phys, double* aux, hipStream_t s);                 \
  int launch_set_state_##NAME(const Buffers& B, const double* phys, const double* aux, hipStream_t s);     \
  int launch_pack_##NAME(int n, const double* in, double* out, hipStream_t s);                              \
  int debug_stamps_##NAME(unsigned long long* host_out);                                                   \
  int plan64_##NAME(int n_envs, int cus, int mode, Geometry* g);                                             \
  int launch_step64_##NAME(const Buffers& B, const StepIO& io, float* scratch, const Geometry& g, hipStream_t s); \
  int launch_reset64_##NAME(const Buffers& B, const ResetIO& io, hipStream_t s);                           \
  int launch_get_state64_##NAME(const Buffers& B, double* phys, double* aux, hipStream_t s);               \
  int launch_set_state64_##NAME(const Buffers& B, const double* phys, const double* aux, hipStream_t s);

PBG_DECLARE_ROBOT(Pendulum)
PBG_DECLARE_ROBOT(Hopper)
PBG_DECLARE_ROBOT(HalfCheetah)
PBG_DECLARE_ROBOT(Ant)
PBG_DECLARE_ROBOT(Humanoid)
PBG_DECLARE_ROBOT(Walker2D)
PBG_DECLARE_ROBOT(PendulumSwingup)
PBG_DECLARE_ROBOT(DoublePendulum)
PBG_DECLARE_ROBOT(HumanoidFlagrun)
PBG_DECLARE_ROBOT(HopperMuJoCo)
PBG_DECLARE_ROBOT(Walker2DMuJoCo)
PBG_DECLARE_ROBOT(HalfCheetahMuJoCo)
PBG_DECLARE_ROBOT(AntMuJoCo)
PBG_DECLARE_ROBOT(HumanoidMuJoCo)
PBG_DECLARE_ROBOT(DoublePendulumMuJoCo)
PBG_DECLARE_ROBOT(HumanoidFlagrunHarder)
PBG_DECLARE_ROBOT(Atlas)
}  // namespace pbg
