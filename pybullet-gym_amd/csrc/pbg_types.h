// Kernel argument blocks shared by the kernels (pbg_step.hip) and the C-ABI layer.
#pragma once
#include <stdint.h>

namespace pbg {
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
  uint64_t seed;
  int env_offset;          // global id of env 0 (multi-GPU sharding)
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
