// Kernel argument blocks shared by the kernels (pbg_step.hip) and the C-ABI layer.
#pragma once
#include <stdint.h>

namespace pbg {
// Scene / World parameters of a handle (include/pbg.h pbg_sim_params_t; scene_bases.py:8-18,
// 58-73), resolved once on the host at create into the constants the kernels use.  Every
// derived float is formed in float arithmetic exactly as the kernels formed it when these
// were compile-time constants, so default parameters reproduce the old bits.
struct SimP {
  float dt;          // Scene.timestep: one stepSimulation sub-step
  float gravity;     // World.gravity: setGravity(0, 0, -gravity)
  float k_sep;       // position-target slope of a separated row: -1 / dt (pos_target)
  float k_contact;   // ... of a penetrating contact normal: -contact_erp / dt
  float k_limit;     // ... of a violated joint limit: -limit_erp / dt
  float ang_max;     // [EXT] angular motion threshold / dt (exponential-map integration)
  float dt3c;        // dt^3 / 48 (small-angle quaternion series)
  int substeps;      // Scene.frame_skip = numSubSteps
  int iterations;    // World.numSolverIterations
  int flag_timeout;  // HumanoidFlagrun: 600 / frame_skip steps, rounded up (robot_locomotors.py:218-223)
  double env_dt;     // Scene.dt = timestep * frame_skip (the potential's divisor, scene_bases.py:17)
};

inline SimP resolve_sim_params(double timestep, int frame_skip, int iterations, double gravity, double contact_erp,
                               double limit_erp, double angular_motion_threshold) {
  SimP p;
  p.dt = (float)timestep;
  const float inv_dt = (float)(1.0 / timestep);
  p.gravity = (float)gravity;
  p.k_sep = -inv_dt;
  p.k_contact = -(float)contact_erp * inv_dt;
  p.k_limit = -(float)limit_erp * inv_dt;
  p.ang_max = (float)angular_motion_threshold / p.dt;
  p.dt3c = p.dt * p.dt * p.dt * 0.020833333333f;
  p.substeps = frame_skip;
  p.iterations = iterations;
  p.flag_timeout = (600 + frame_skip - 1) / frame_skip;
  p.env_dt = timestep * frame_skip;
  return p;
}

struct Buffers {
  int n;                   // envs on this device
  float* st;               // [SD][n] physical state, SoA
  double* pot;             // [n] potential
  float* z0;               // [n] initial_z
  int* elapsed;            // [n] steps in episode
  uint32_t* flags;         // [n] bit0 floor-in-parts, bits 8.. feet_contact
  uint32_t* episode;       // [n] resets so far (RNG counter)
  double* tgt;             // [2][n] walk target x, y (HumanoidFlagrun)
  int32_t* ftm;            // [2][n] flag_timeout, flag draws so far (HumanoidFlagrun RNG counter)
  double* hkd;             // [2][n] crawl_start_potential (NaN = None), crawl_ignored_potential (Harder)
  int32_t* hki;            // [3][n] frame, on_ground_frame_counter, cube launches so far (Harder)
  uint64_t seed;
  int env_offset;          // global id of env 0 (multi-GPU sharding)
  SimP sp;                 // the handle's scene parameters (kernel arguments)
};

struct StepIO {
  const float* act;        // [n][NA]
  float* obs;              // [n][OBS]
  float* rew;              // [n] float32 reward
  double* rew64;           // [n] nullable float64 reward
  uint8_t* done;           // [n] terminated | truncated
  uint8_t* trunc;          // [n] nullable, TimeLimit truncation
  float* term_obs;         // [n][OBS] nullable: obs before an auto-reset
  int32_t* ncontact;       // [n] nullable: contacts in the last sub-step
  int autoreset;
  double* rew_terms;       // [n][5] nullable: the terms the reward sums (reference self.rewards)
  uint32_t* csig;          // [n] nullable: contact-set signature (sim_params.h pbg_contact_hash)
};

struct ResetIO {
  const uint8_t* mask;     // [n] nullable = all
  const float* init_q;     // [n][NR] nullable = Philox noise U(-0.1, 0.1)
  float* obs;              // [n][OBS]
};

}  // namespace pbg
