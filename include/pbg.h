/* pbg.h -- C-ABI of the MI355X batched locomotion stepper (libpbg_amd.so).
 *
 * The reference (josiahls/pybullet-gym) has no native boundary of its own: its hot path
 * calls the pybullet C extension once per query, per env, through
 * pybullet_envs.bullet.bullet_client.BulletClient (pybulletgym/envs/roboschool/
 * env_bases.py:4,51-56).  This ABI replaces that whole per-env call sequence with one
 * batched call per env step.  Each entry point names the reference interface it replaces.
 *
 * Conventions
 *   - All array arguments are DEVICE pointers (HIP / PyTorch-ROCm tensors), row-major,
 *     except where marked "host".  The caller owns every I/O buffer; the handle owns its
 *     struct-of-arrays state.  Nothing allocates or synchronises inside step/reset.
 *   - `stream` is a hipStream_t (NULL = the legacy default stream); work is async on it.
 *   - Return 0 on success, a negative PBG_E_* code on failure; pbg_last_error() gives
 *     the message (thread-local).
 *   - One handle = the envs of one GPU.  Multi-GPU: one handle per rank, env_offset =
 *     global index of the rank's first env (reset RNG streams depend on the global id).
 */
#ifndef PBG_H
#define PBG_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PBG_OK 0
#define PBG_E_ARG (-1)
#define PBG_E_ENV (-2)
#define PBG_E_HIP (-3)
#define PBG_E_NOMEM (-4)

/* Layout version of the per-env state records of pbg_get_state / pbg_set_state (reported in
 * pbg_info_t.record_version).  1: round-1 aux record (no episode counter); 2: aux ends with
 * the episodes-started counter (the reset-noise Philox counter).  A checkpoint written under
 * another version must not be passed to pbg_set_state (the aux width differs). */
#define PBG_RECORD_VERSION 2

typedef struct pbg_handle pbg_handle;

typedef struct {
  int robot_id;          /* 0 pendulum, 1 hopper, 2 halfcheetah, 3 ant, 4 humanoid, 5 walker2d,
                            6 pendulum_swingup, 7 double_pendulum, 8 humanoid_flagrun,
                            9 hopper_mujoco, 10 walker2d_mujoco, 11 halfcheetah_mujoco,
                            12 ant_mujoco, 13 humanoid_mujoco, 14 double_pendulum_mujoco,
                            15 humanoid_flagrun_harder, 16 atlas */
  int n_envs;
  int action_dim;        /* action_space.shape[0]   (robot_bases.py:24-25) */
  int obs_dim;           /* observation_space.shape[0] (robot_bases.py:26-27) */
  int n_dof;             /* generalized velocities (6 floating-base + joint dofs) */
  int n_joints;          /* joint dofs incl. `ignore*` joints */
  int n_links;
  int n_feet;
  int state_words;       /* per-env physical state record (see pbg_get_state) */
  int aux_words;         /* per-env bookkeeping record (see pbg_get_state) */
  int substeps;          /* stepSimulation sub-steps per env step (the handle's frame_skip,
                            scene_bases.py:73 numSubSteps) */
  int max_episode_steps; /* gym TimeLimit (envs/__init__.py) */
  int reset_dofs;        /* joints randomised by reset (robot_locomotors.py:18-19) */
  int floating;
  int lanes_per_env;     /* step kernel geometry: 1 (lane per env), 4 (quad) or 16 (gang) */
  int block;             /* step kernel workgroup size (lanes) */
  int lds_bytes;         /* dynamic LDS per step workgroup */
  int vgprs;             /* step kernel registers per lane (hipFuncGetAttributes numRegs) */
  int scratch_bytes;     /* step kernel private segment per lane (0: no spills to memory) */
  int lds_rows;          /* contact rows (gang: contacts) resident in LDS per env */
  int record_version;    /* PBG_RECORD_VERSION of the state / aux records (appended in round 3) */
} pbg_info_t;

typedef struct {
  const float* act;   /* [n, action_dim] float32 */
  float* obs;         /* [n, obs_dim] float32: next observation (post-reset if auto-reset) */
  float* rew;         /* [n] float32 reward (computed in float64) */
  uint8_t* done;      /* [n] terminated | truncated */
  double* rew64;      /* nullable [n] float64 reward */
  uint8_t* trunc;     /* nullable [n] TimeLimit truncation flag */
  float* term_obs;    /* nullable [n, obs_dim] observation before an auto-reset */
  int32_t* ncontact;  /* nullable [n] contact points in the last sub-step */
  int autoreset;      /* reset envs that finished, inside the same launch */
  double* rew_terms;  /* nullable [n, 5] float64: the terms the reward sums, in the order of the
                         reference's self.rewards list, zero-padded -- walkers: alive, progress,
                         electricity, joints_at_limit, feet_collision (gym_locomotion_envs.py:99-105);
                         MuJoCo Ant/Humanoid: alive, progress, joints_at_limit, feet_collision
                         (mujoco/gym_locomotion_envs.py:98-103); MuJoCo planar: potential,
                         [alive,] power_cost; pendulums: their rewards list */
  uint32_t* csig;     /* nullable [n] contact-set signature of the env step: the sum mod 2^32 of
                         fmix32((substep << 16) + candidate + 0x9E3779B9) over every active collision
                         candidate (floor slots 0..NS-1, self pairs NS + p; HumanoidFlagrunHarder's
                         cube corners NS + NPAIR + k, cube vs robot geom NS + NPAIR + 8 + g) of every
                         sub-step (sim_params.h pbg_contact_hash; for parity tests) */
} pbg_step_io_t;

/* Test / diagnostic launch options (pbg_create_debug / pbg_create_ex).  -1 = the default everywhere.
 * ABI note: round 4 appended gang_lanes (3 -> 4 ints) without a size field; the struct is frozen at
 * these four ints.  Callers that need another option use pbg_create_v2 (pbg_create_opts_t is
 * versioned by its struct_size). */
typedef struct {
  int kernel;     /* 0: one-lane-per-env kernel for every robot (PBG_E_ARG for Atlas, whose 886
                     contact slots have no lane kernel, in either precision); 2: the 16-lane gang
                     kernel for every walker (Ant included); -1 / 1: default (quad for Ant, gang
                     otherwise) */
  int lds_rows;   /* k >= 0: at most k contact rows (gang: contacts) per env resident in LDS,
                     the rest in the device workspace (bitwise-equality tests of that path) */
  int gang_dist;  /* 0 / 1: force replicated / distributed gang dynamics (PBG_E_ARG when the planned
                     kernel is no gang kernel or has no such variant: 32-lane gangs and
                     HumanoidFlagrunHarder are distributed only) */
  int gang_lanes; /* 16 / 32: gang width (32: the Humanoid family only); PBG_E_ARG when the planned
                     kernel is not a gang kernel of that width (Ant's quad plan, kernel = 0) */
} pbg_debug_opts_t;

/* Scene / World parameters (scene_bases.py:8-18 Scene(gravity, timestep, frame_skip), 58-73
 * World: setGravity, numSolverIterations, numSubSteps).  pbg_default_sim_params fills the values
 * the reference's env constructs its scene with (gym_locomotion_envs.py:18-19 StadiumScene(9.8,
 * 0.0165/4, 4); Atlas StadiumScene(9.8, 0.0165/8, 8), gym_locomotion_envs.py:187;
 * gym_pendulum_envs.py:14 SingleRobotEmptyScene(9.8, 0.0165, 1); iterations 5,
 * scene_bases.py:65) plus the solver ERPs the kernels use; pbg_create_ex takes a modified copy.
 * An env step is frame_skip sub-steps of `timestep` seconds; the potential divides by
 * Scene.dt = timestep * frame_skip (scene_bases.py:17); HumanoidFlagrun's flag timeout is
 * 600 / frame_skip steps (robot_locomotors.py:218). */
typedef struct {
  double gravity;         /* m/s^2 along -z (World.gravity; 0 = weightless) */
  double timestep;        /* seconds per physics sub-step (Scene.timestep), in (0, 0.1] */
  int frame_skip;         /* sub-steps per env step (Scene.frame_skip = numSubSteps), 1..64 */
  int solver_iterations;  /* PGS sweeps per sub-step (World.numSolverIterations), 1..1000 */
  double contact_erp;     /* [0, 1]: share of a contact penetration corrected per sub-step */
  double joint_limit_erp; /* [0, 1]: share of a joint-limit violation corrected per sub-step */
} pbg_sim_params_t;

/* Options of pbg_create_v2, versioned: set struct_size = sizeof(pbg_create_opts_t) of the header the
 * caller was built with; the library reads only the fields that size covers (fields past it take
 * their defaults), so options appended later never read past an older caller's struct. */
typedef struct {
  uint32_t struct_size;  /* sizeof(pbg_create_opts_t) at the caller's build */
  int precision;         /* physics state and arithmetic: 64 = float64 (the default since round 6,
                            as for pbg_create / pbg_create_ex: the reference's precision, pybullet's
                            btScalar is double: stepSimulation, scene_bases.py:75-76) or 32 =
                            float32, the opt-in fast kernels.  The observation / reward pack is
                            float64 in both, as in the reference.  Every env id has both
                            (AtlasPyBulletEnv-v0: the gang kernel only) */
  int kernel;            /* as in pbg_debug_opts_t.  Precision 64: 1 (default) = the quad kernel for
                            Ant, the 16-lane gang kernel for the other walkers, the lane kernel for
                            the pendulums; 0 = the lane kernel for every robot; 2 = the gang kernel
                            for every walker (Ant included) */
  int lds_rows;
  int gang_dist;
  int gang_lanes;
} pbg_create_opts_t;

/* The reference's parameters for env_id (see pbg_sim_params_t). */
int pbg_default_sim_params(const char* env_id, pbg_sim_params_t* out);

/* gym.make(env_id) for n envs (envs/__init__.py:4-103 registry entries; the env's
 * physics client is created here instead of lazily in BaseBulletEnv._reset,
 * env_bases.py:46-56), with float64 physics (the reference's precision; pbg_create_v2 selects
 * float32).  env_id (robot_id order): "InvertedPendulumPyBulletEnv-v0",
 * "HopperPyBulletEnv-v0", "HalfCheetahPyBulletEnv-v0", "AntPyBulletEnv-v0",
 * "HumanoidPyBulletEnv-v0", "Walker2DPyBulletEnv-v0", "InvertedPendulumSwingupPyBulletEnv-v0",
 * "InvertedDoublePendulumPyBulletEnv-v0", "HumanoidFlagrunPyBulletEnv-v0", "HopperMuJoCoEnv-v0",
 * "Walker2DMuJoCoEnv-v0", "HalfCheetahMuJoCoEnv-v0", "AntMuJoCoEnv-v0", "HumanoidMuJoCoEnv-v0",
 * "InvertedDoublePendulumMuJoCoEnv-v0", "HumanoidFlagrunHarderPyBulletEnv-v0",
 * "AtlasPyBulletEnv-v0" (gym_locomotion_envs.py:181-188) (the short robot names are accepted
 * too). */
int pbg_create(const char* env_id, int n_envs, int device, uint64_t seed, int env_offset, pbg_handle** out);
/* pbg_create with test / diagnostic launch options (opts NULL = pbg_create). */
int pbg_create_debug(const char* env_id, int n_envs, int device, uint64_t seed, int env_offset,
                     const pbg_debug_opts_t* opts, pbg_handle** out);
/* pbg_create with the scene built from `params` (NULL = pbg_default_sim_params) and test /
 * diagnostic launch options (NULL = defaults).  PBG_E_ARG for parameters out of range. */
int pbg_create_ex(const char* env_id, int n_envs, int device, uint64_t seed, int env_offset,
                  const pbg_sim_params_t* params, const pbg_debug_opts_t* opts, pbg_handle** out);
/* pbg_create_ex with versioned options (opts NULL = defaults: float64, the default kernels).
 * PBG_E_ARG for a bad struct_size (not a multiple of 4 in [8, sizeof]) or precision, and for a
 * launch option the planned kernel cannot honour (in either precision); PBG_E_HIP when no kernel
 * plan fits the device.  *out is NULL after every failure. */
int pbg_create_v2(const char* env_id, int n_envs, int device, uint64_t seed, int env_offset,
                  const pbg_sim_params_t* params, const pbg_create_opts_t* opts, pbg_handle** out);
/* The handle's physics precision: 32 or 64 (PBG_E_ARG for NULL). */
int pbg_precision(const pbg_handle* h);
/* The parameters a handle was created with. */
int pbg_get_sim_params(const pbg_handle* h, pbg_sim_params_t* out);
/* BaseBulletEnv._close (env_bases.py:103-107) */
void pbg_destroy(pbg_handle* h);
/* action_space / observation_space / model sizes (robot_bases.py:24-27) */
int pbg_info(const pbg_handle* h, pbg_info_t* out);

/* WalkerBaseBulletEnv._reset (gym_locomotion_envs.py:22-39) + BaseBulletEnv._reset
 * (env_bases.py:46-71) + robot_specific_reset (robot_locomotors.py:16-24):
 * restoreState snapshot, resetJointState(U(-0.1,0.1)) on the ordered joints, calc_state.
 * mask: nullable [n] uint8 (NULL = all envs).  init_q: nullable [n, reset_dofs] float32
 * joint positions to use instead of the RNG (trace replay).  obs: [n, obs_dim]. */
int pbg_reset(pbg_handle* h, const uint8_t* mask, const float* init_q, float* obs, void* stream);

/* WalkerBaseBulletEnv._step (gym_locomotion_envs.py:54-114): apply_action
 * (robot_locomotors.py:26-29) -> stepSimulation x substeps (scene_bases.py:75-76) ->
 * calc_state / potential / alive / feet contacts / costs.  No auto-reset.
 * act: [n, action_dim] float32, clipped to [-1, 1] for the torques (+-inf -> +-1, NaN -> -1: IEEE
 * max); the electricity cost takes the unclipped value (a NaN action gives a NaN reward).  The
 * reference asserts finite actions (robot_locomotors.py:27); the per-env facade does too, the
 * batch API does not check them (that would cost a host sync per step). */
int pbg_step(pbg_handle* h, const float* act, float* obs, float* rew, uint8_t* done, void* stream);
/* pbg_step with optional outputs and in-launch auto-reset (gym TimeLimit + reset). */
int pbg_step_ex(pbg_handle* h, const pbg_step_io_t* io, void* stream);

/* pybullet saveState/restoreState (gym_locomotion_envs.py:25,36) generalised to trace
 * replay / teacher forcing / checkpoints.  phys: [n, state_words] float64 records
 *   [0..2] base COM pos, [3..6] base quat (x,y,z,w), [7..9] base COM lin vel (world),
 *   [10..12] base ang vel (world), then q[n_joints], qd[n_joints], (HumanoidFlagrunHarder: the
 *   cube's 13 words in the base's layout);
 * aux: [n, aux_words] float64 = [potential, initial_z, elapsed_steps, floor_in_parts,
 *   feet_contact[n_feet], (HumanoidFlagrun / Harder: walk target x, y, flag_timeout, flag draws),
 *   (HumanoidFlagrunHarder: frame, on_ground_frame_counter, crawl_start_potential (NaN = None),
 *   crawl_ignored_potential, cube launches), episodes started (the reset-noise RNG counter)],
 *   layout PBG_RECORD_VERSION (the Harder words are new robot-specific words, not a change of
 *   any existing robot's layout).
 * set_state with aux == NULL replaces the physical state only: the handle keeps its own
 * bookkeeping -- potential, initial_z, elapsed steps, feet flags and the episode counter --
 * so later resets continue that handle's reset-noise stream, not the checkpoint's. */
int pbg_get_state(pbg_handle* h, double* phys, double* aux, void* stream);
int pbg_set_state(pbg_handle* h, const double* phys, const double* aux, void* stream);

/* Test support: fill every CU's LDS (160 KB each) with the 32-bit pattern and, when h is not NULL,
 * h's device workspace (the contact / limit rows past the LDS capacity), stream-ordered before the
 * next launch.  The kernels write everything they read in a launch, so a step after a poison must
 * give the same bits whatever the pattern (tests/test_gpu.py test_uninitialised_memory_invariance).
 * h NULL: the current device's LDS only. */
int pbg_debug_poison(pbg_handle* h, uint32_t pattern, void* stream);

/* The observation/reward/done pack alone (calc_state + the reward half of _step) on
 * explicit inputs, for golden-vector parity; layouts in pbg_pack_record_sizes. */
int pbg_pack_record_sizes(const char* env_id, int* in_words, int* out_words);
int pbg_pack(const char* env_id, int n, const double* in_rec, double* out_rec, void* stream);

/* Batched action_space.sample() (robot_bases.py:24-25 Box(-1, 1)): out[s, e, i] = U(-1, 1)
 * float32 for s < n_steps, e < n_envs, i < action_dim; Philox4x32-10, key = seed, counter =
 * (step0 + s, env_offset + e, i / 4, 0xAC7) -- the bench's random-action protocol
 * (BASELINE.md section 2), independent of the sharding.  out: device [n_steps, n_envs, action_dim];
 * the kernel runs on the device that owns `out` (pbg_pack likewise on its records' device).
 * These two handle-less entry points take device (hipMalloc) or managed memory only: a host or
 * pinned-host (hipHostMalloc) pointer has no owning device and returns PBG_E_ARG. */
int pbg_sample_actions(int action_dim, int n_envs, int n_steps, uint64_t seed, uint32_t step0, int env_offset,
                       float* out, void* stream);

const char* pbg_last_error(void);

#ifdef __cplusplus
}
#endif
#endif /* PBG_H */
