"""Drop-in mirror of the reference's env / robot / scene class surface.

The reference's user-facing API is ``gym.make('AntPyBulletEnv-v0')`` returning a
``WalkerBaseBulletEnv`` whose ``reset()`` / ``step(a)`` drive pybullet
(pybulletgym/envs/roboschool/{env_bases,gym_locomotion_envs,gym_pendulum_envs,
robot_locomotors,robot_pendula,scene_bases,scene_stadium}.py).  The same class names,
constructor signatures, class constants and return types live here; the physics and
the observation/reward pack run in the HIP step kernel (one env = a VecEnv of size 1).
For throughput use ``pybulletgym_amd.VecEnv`` directly: thousands of envs per launch.

Out of scope (not on the hot path): rendering/cameras (``render`` returns an empty array
as the reference does for non-rgb modes), multiplayer scenes, HUD.
"""
from __future__ import annotations

import numpy as np

from . import robots as _robots
from .spaces import Box


# ----------------------------------------------------------------------------- scenes
class Scene:
    """scene_bases.py:8-52.  dt = timestep * frame_skip; the sub-stepped World.step is
    fused into the step kernel, so global_step() is not callable on its own."""
    multiplayer = False

    def __init__(self, bullet_client=None, gravity=9.8, timestep=0.0165 / 4, frame_skip=4):
        self.gravity = gravity
        self.timestep = timestep
        self.frame_skip = frame_skip
        self.dt = self.timestep * self.frame_skip
        self.numSolverIterations = 5  # scene_bases.py:65

    def global_step(self):
        raise NotImplementedError("the physics step is fused into the batched kernel; call env.step(a)")


class SingleRobotEmptyScene(Scene):
    """scene_bases.py:54-55 (pendulum: no floor)."""
    multiplayer = False


class StadiumScene(Scene):
    """scene_stadium.py:10-35: the floor plane, lateral friction 0.8, restitution 0.5."""
    multiplayer = False
    zero_at_running_strip_start_line = True
    stadium_halflen = 105 * 0.25
    stadium_halfwidth = 50 * 0.25
    floor_lateral_friction = 0.8
    floor_restitution = 0.5


# ----------------------------------------------------------------------------- robots
class XmlBasedRobot:
    """robot_bases.py:10-30: action/observation spaces from the dims."""
    self_collision = True

    def __init__(self, robot_name, action_dim, obs_dim, self_collision=True):
        high = np.ones([action_dim], dtype=np.float32)
        self.action_space = Box(-high, high)
        high = np.inf * np.ones([obs_dim], dtype=np.float32)
        self.observation_space = Box(-high, high)
        self.robot_name = robot_name
        self.self_collision = self_collision


class MJCFBasedRobot(XmlBasedRobot):
    """robot_bases.py:97-129."""

    def __init__(self, model_xml, robot_name, action_dim, obs_dim, self_collision=True):
        XmlBasedRobot.__init__(self, robot_name, action_dim, obs_dim, self_collision)
        self.model_xml = model_xml


class URDFBasedRobot(XmlBasedRobot):
    """robot_bases.py:132-175 (self_collision False, floating base)."""

    def __init__(self, model_urdf, robot_name, action_dim, obs_dim, self_collision=False):
        XmlBasedRobot.__init__(self, robot_name, action_dim, obs_dim, self_collision)
        self.model_urdf = model_urdf


class WalkerBase(XmlBasedRobot):
    """robot_locomotors.py:7-79 constants (target, power)."""

    def __init__(self, power):
        self.power = power
        self.walk_target_x = 1e3
        self.walk_target_y = 0
        self.body_xyz = [0, 0, 0]


def _robot_class(key, base_cls):
    spec = _robots.spec_for(key)

    walker = spec.kind in (_robots.KIND_WALKER, _robots.KIND_MUJOCO_PLANAR, _robots.KIND_MUJOCO_3D)
    xml = URDFBasedRobot if spec.urdf else MJCFBasedRobot
    bases = (WalkerBase, xml) if walker else (xml,)

    class _R(*bases):
        foot_list = list(spec.foot_list)

        def __init__(self):
            if walker:
                WalkerBase.__init__(self, power=spec.power)
            xml.__init__(self, spec.urdf or spec.mjcf, spec.robot_name, action_dim=spec.action_dim,
                         obs_dim=spec.obs_dim)
            self.spec = spec

    _R.__name__ = base_cls
    return _R


Hopper = _robot_class("hopper", "Hopper")                    # robot_locomotors.py:82-90
Walker2D = _robot_class("walker2d", "Walker2D")              # :93-106
HalfCheetah = _robot_class("halfcheetah", "HalfCheetah")     # :109-127
Ant = _robot_class("ant", "Ant")                             # :130-138
Humanoid = _robot_class("humanoid", "Humanoid")              # :141-192
HumanoidFlagrun = _robot_class("humanoid_flagrun", "HumanoidFlagrun")  # :195-226
HumanoidFlagrunHarder = _robot_class("humanoid_flagrun_harder", "HumanoidFlagrunHarder")  # :229-302
Atlas = _robot_class("atlas", "Atlas")                                                     # :305-341
HopperMuJoCo = _robot_class("hopper_mujoco", "Hopper")                # mujoco/robot_locomotors.py:82-121
Walker2DMuJoCo = _robot_class("walker2d_mujoco", "Walker2D")          # :124-164
HalfCheetahMuJoCo = _robot_class("halfcheetah_mujoco", "HalfCheetah")  # :167-207
AntMuJoCo = _robot_class("ant_mujoco", "Ant")                          # :210-239
HumanoidMuJoCo = _robot_class("humanoid_mujoco", "Humanoid")           # :242-319
InvertedPendulum = _robot_class("pendulum", "InvertedPendulum")  # robot_pendula.py:5-51
InvertedPendulumSwingup = _robot_class("pendulum_swingup", "InvertedPendulumSwingup")  # robot_pendula.py:54-55
InvertedDoublePendulum = _robot_class("double_pendulum", "InvertedDoublePendulum")      # robot_pendula.py:58-88
InvertedDoublePendulumMuJoCo = _robot_class("double_pendulum_mujoco", "InvertedDoublePendulum")  # mujoco/robot_pendula.py:51-89
InvertedPendulum.swingup = False
InvertedPendulumSwingup.swingup = True


def _alive_bonus_hopper(self, z, pitch):
    return +1 if z > 0.8 and abs(pitch) < 1.0 else -1


def _alive_bonus_ant(self, z, pitch):
    return +1 if z > 0.26 else -1


def _alive_bonus_humanoid(self, z, pitch):
    return +2 if z > 0.78 else -1


Hopper.alive_bonus = _alive_bonus_hopper
Walker2D.alive_bonus = _alive_bonus_hopper  # robot_locomotors.py:100-101 (same rule as Hopper)
Ant.alive_bonus = _alive_bonus_ant
Humanoid.alive_bonus = _alive_bonus_humanoid
HumanoidFlagrun.alive_bonus = _alive_bonus_humanoid
# HumanoidFlagrunHarder.alive_bonus (robot_locomotors.py:250-273) moves the cube and counts
# frames; it runs inside the step kernel (the per-env bookkeeping lives in the aux record)


# ----------------------------------------------------------------------------- envs
class BaseBulletEnv:
    """env_bases.py:9-121 surface: reset() -> obs, step(a) -> (obs, reward, done, {}),
    seed(), render(), close().  One env on one GPU via the batched kernel.

    ``precision`` is the physics scalar: 64 (the default) steps in float64 like the reference's
    pybullet (btScalar is double; scene_bases.py:75-76 -> stepSimulation), 32 runs the float32
    fast-mode kernels.  The handle (``_vec``, a one-env VecEnv) is created on first use -- the
    reference connects its physics client in reset() (env_bases.py:60-67) -- and again after seed()."""
    metadata = {"render.modes": ["human", "rgb_array"], "video.frames_per_second": 60}
    env_id = None

    def __init__(self, robot, render=False, device="cuda:0", precision=64):
        self.robot = robot
        self.isRender = render
        self.action_space = robot.action_space
        self.observation_space = robot.observation_space
        self.device = device
        self.precision = int(precision)
        if self.precision not in (32, 64):
            raise ValueError(f"precision must be 32 or 64, not {precision!r}")
        self._seed_value = 0
        self._vec_h = None
        self.scene = None
        self.reward = 0.0
        self.frame = 0

    @property
    def _vec(self):
        if self._vec_h is None:
            from .vec_env import VecEnv
            self._vec_h = VecEnv(self.env_id, 1, device=self.device, seed=self._seed_value, autoreset=False,
                                 precision=self.precision)
        return self._vec_h

    @property
    def unwrapped(self):
        return self  # gym.Env.unwrapped

    def seed(self, seed=None):
        self._seed_value = 0 if seed is None else int(seed)
        self.action_space.seed(seed)
        self.close()
        return [self._seed_value]

    def reset(self):
        self.frame = 0
        self.reward = 0.0
        obs = self._vec.reset()
        return self._obs_out(obs)

    def step(self, a):
        import torch
        if self._vec_h is None:
            raise RuntimeError("call reset() before step()")
        a = np.asarray(a, dtype=np.float32).reshape(1, -1)
        assert np.isfinite(a).all()  # robot_locomotors.py:27
        res = self._vec.step(torch.from_numpy(a), want_reward64=True)
        r = float(self._vec.reward64[0])
        # termination only (gym_locomotion_envs.py:61-65): the kernel's own TimeLimit marks a
        # 1000th step done + truncated; the time limit belongs to the TimeLimit wrapper
        done = bool(res.done[0]) and not bool(res.truncated[0])
        self.frame += 1
        self.reward += r
        return self._obs_out(res.obs), r, done, {}

    def _obs_out(self, obs):
        return obs[0].cpu().numpy()

    def render(self, mode="human", close=False):
        return np.array([])  # env_bases.py:73-77 for non-rgb modes; rendering is out of scope

    def close(self):
        if self._vec_h is not None:
            self._vec_h.close()
            self._vec_h = None

    def HUD(self, state, a, done):
        pass

    # gym < 0.9.6 spelling used by the reference (env_bases.py:114-121)
    _reset = reset
    _step = step
    _seed = seed
    _close = close
    _render = render


class WalkerBaseBulletEnv(BaseBulletEnv):
    """gym_locomotion_envs.py:8-119: reward-term constants as class attributes."""
    electricity_cost = -2.0
    stall_torque_cost = -0.1
    foot_collision_cost = -1.0
    foot_ground_object_names = set(["floor"])
    joints_at_limit_cost = -0.1

    def __init__(self, robot, render=False, device="cuda:0", precision=64):
        BaseBulletEnv.__init__(self, robot, render, device, precision)
        self.camera_x = 0
        self.walk_target_x = 1e3
        self.walk_target_y = 0
        self.stateId = -1
        self.scene = self.create_single_player_scene(None)

    def create_single_player_scene(self, bullet_client):
        self.stadium_scene = StadiumScene(bullet_client, gravity=9.8, timestep=0.0165 / 4, frame_skip=4)
        return self.stadium_scene


class HopperBulletEnv(WalkerBaseBulletEnv):
    env_id = "HopperPyBulletEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        self.robot = Hopper()
        WalkerBaseBulletEnv.__init__(self, self.robot, render, device, precision)


class Walker2DBulletEnv(WalkerBaseBulletEnv):
    env_id = "Walker2DPyBulletEnv-v0"  # gym_locomotion_envs.py:128-131

    def __init__(self, render=False, device="cuda:0", precision=64):
        self.robot = Walker2D()
        WalkerBaseBulletEnv.__init__(self, self.robot, render, device, precision)


class HalfCheetahBulletEnv(WalkerBaseBulletEnv):
    env_id = "HalfCheetahPyBulletEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        self.robot = HalfCheetah()
        WalkerBaseBulletEnv.__init__(self, self.robot, render, device, precision)


class AntBulletEnv(WalkerBaseBulletEnv):
    env_id = "AntPyBulletEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        self.robot = Ant()
        WalkerBaseBulletEnv.__init__(self, self.robot, render, device, precision)


class HumanoidBulletEnv(WalkerBaseBulletEnv):
    env_id = "HumanoidPyBulletEnv-v0"

    def __init__(self, robot=None, render=False, device="cuda:0", precision=64):
        # gym_locomotion_envs.py:147 shares one default Humanoid() between instances; each
        # env here owns its own robot record (the batched state is per env anyway).
        self.robot = robot if robot is not None else Humanoid()
        WalkerBaseBulletEnv.__init__(self, self.robot, render, device, precision)
        self.electricity_cost = 4.25 * WalkerBaseBulletEnv.electricity_cost
        self.stall_torque_cost = 4.25 * WalkerBaseBulletEnv.stall_torque_cost


class HumanoidFlagrunBulletEnv(HumanoidBulletEnv):
    """gym_locomotion_envs.py:154-164: the Humanoid chasing a flag that is re-drawn
    (U(+-13.125) x U(+-6.25)) when reached within 1 m or after 150 steps; the walk target and
    flag_timeout live in the device state (aux words), the draws are Philox (not np_random)."""
    env_id = "HumanoidFlagrunPyBulletEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        HumanoidBulletEnv.__init__(self, HumanoidFlagrun(), render, device, precision)


class HumanoidFlagrunHarderBulletEnv(HumanoidBulletEnv):
    """gym_locomotion_envs.py:167-178: HumanoidFlagrun plus an attacking 1.2 kg, 5 cm cube
    (gym_utils.get_cube) launched at the robot every 30 frames after frame 100 while it is up,
    an alive bonus / potential that leak with the torso height, crawl disabled, and the episode
    ended after 170 frames on the ground (robot_locomotors.py:229-302).  The cube is a second
    free body of the env's physics state; its launches are Philox draws (not np_random).
    The env's ``electricity_cost /= 4`` (:172) is overwritten by HumanoidBulletEnv.__init__
    (:150), so the Humanoid's costs stand, as in the reference."""
    env_id = "HumanoidFlagrunHarderPyBulletEnv-v0"
    random_lean = True  # :168 (a class attribute of the env; the robot never reads it)

    def __init__(self, render=False, device="cuda:0", precision=64):
        HumanoidBulletEnv.__init__(self, HumanoidFlagrunHarder(), render, device, precision)


class AtlasBulletEnv(WalkerBaseBulletEnv):
    """gym_locomotion_envs.py:181-191: the Atlas URDF robot (30 actuated joints, power 2.9),
    StadiumScene with 8 sub-steps of 0.0165/8 s; alive_bonus +4 minus the knees at their limit
    while the head is above 1.3 m, else -1 (robot_locomotors.py:313-324); runs on the gang
    kernel."""
    env_id = "AtlasPyBulletEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        self.robot = Atlas()
        WalkerBaseBulletEnv.__init__(self, self.robot, render, device, precision)


class WalkerBaseMuJoCoEnv(WalkerBaseBulletEnv):
    """envs/mujoco/gym_locomotion_envs.py:8-118 (MuJoCo-style observations on the same
    pybullet physics)."""


class HopperMuJoCoEnv(WalkerBaseMuJoCoEnv):
    """mujoco/gym_locomotion_envs.py:121-160: obs [qpos[1:], clip(qvel, -10, 10)] (11),
    reward x-progress + 1 - 1e-3 sum(a^2), done unless height > -0.3 and |angle| < .2."""
    env_id = "HopperMuJoCoEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        WalkerBaseMuJoCoEnv.__init__(self, HopperMuJoCo(), render, device, precision)


class Walker2DMuJoCoEnv(WalkerBaseMuJoCoEnv):
    """mujoco/gym_locomotion_envs.py:163-203: obs (17); done unless 1 > height > -0.2 and
    -1 < angle < 1."""
    env_id = "Walker2DMuJoCoEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        WalkerBaseMuJoCoEnv.__init__(self, Walker2DMuJoCo(), render, device, precision)


class HalfCheetahMuJoCoEnv(WalkerBaseMuJoCoEnv):
    """mujoco/gym_locomotion_envs.py:206-240: obs [qpos[1:], qvel] (17), reward x-progress
    - 0.1 sum(a^2), never done."""
    env_id = "HalfCheetahMuJoCoEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        WalkerBaseMuJoCoEnv.__init__(self, HalfCheetahMuJoCo(), render, device, precision)


class AntMuJoCoEnv(WalkerBaseMuJoCoEnv):
    """mujoco/gym_locomotion_envs.py:243-246: obs float64 [qpos[2:], qvel, cfrc_ext zeros] (111),
    reward alive(state[0] + initial_z) + progress - 0.1 joints_at_limit."""
    env_id = "AntMuJoCoEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        WalkerBaseMuJoCoEnv.__init__(self, AntMuJoCo(), render, device, precision)

    def _obs_out(self, obs):
        return obs[0].cpu().numpy().astype(np.float64)


class HumanoidMuJoCoEnv(WalkerBaseMuJoCoEnv):
    """mujoco/gym_locomotion_envs.py:249-255: obs float64 [qpos[2:], qvel, cinert, cvel,
    qfrc_actuator, cfrc_ext] (376; the last four are zeros in the reference)."""
    env_id = "HumanoidMuJoCoEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        WalkerBaseMuJoCoEnv.__init__(self, HumanoidMuJoCo(), render, device, precision)

    def _obs_out(self, obs):
        return obs[0].cpu().numpy().astype(np.float64)


class InvertedPendulumBulletEnv(BaseBulletEnv):
    """gym_pendulum_envs.py:7-42: obs float64 [x, vx, cos(theta), sin(theta), theta_dot]."""
    env_id = "InvertedPendulumPyBulletEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        self.robot = InvertedPendulum()
        BaseBulletEnv.__init__(self, self.robot, render, device, precision)
        self.stateId = -1
        self.scene = self.create_single_player_scene(None)

    def create_single_player_scene(self, bullet_client):
        return SingleRobotEmptyScene(bullet_client, gravity=9.8, timestep=0.0165, frame_skip=1)

    def _obs_out(self, obs):
        return obs[0].cpu().numpy().astype(np.float64)


class InvertedPendulumSwingupBulletEnv(InvertedPendulumBulletEnv):
    """gym_pendulum_envs.py:45-49: hinge reset at 3.1415 + U(-.1, .1); reward cos(theta),
    never done (the TimeLimit ends episodes)."""
    env_id = "InvertedPendulumSwingupPyBulletEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        self.robot = InvertedPendulumSwingup()
        BaseBulletEnv.__init__(self, self.robot, render, device, precision)
        self.stateId = -1
        self.scene = self.create_single_player_scene(None)


class InvertedDoublePendulumBulletEnv(BaseBulletEnv):
    """gym_pendulum_envs.py:52-86: obs float64 [x, vx, pole2 x, cos th, sin th, th', cos g,
    sin g, g']; reward 10 - (0.01 x2^2 + (y2 + 0.3 - 2)^2); done y2 + 0.3 <= 1."""
    env_id = "InvertedDoublePendulumPyBulletEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        self.robot = InvertedDoublePendulum()
        BaseBulletEnv.__init__(self, self.robot, render, device, precision)
        self.stateId = -1
        self.scene = self.create_single_player_scene(None)

    def create_single_player_scene(self, bullet_client):
        return SingleRobotEmptyScene(bullet_client, gravity=9.8, timestep=0.0165, frame_skip=1)

    def _obs_out(self, obs):
        return obs[0].cpu().numpy().astype(np.float64)


class InvertedDoublePendulumMuJoCoEnv(InvertedDoublePendulumBulletEnv):
    """mujoco/gym_pendulum_envs.py:44-75: obs float64 [x, sin th, sin g, cos th, cos g,
    clip(vx, th', g'), zeros(3)]; reward 10 - dist_penalty - (1e-3 th'^2 + 5e-3 g'^2)."""
    env_id = "InvertedDoublePendulumMuJoCoEnv-v0"

    def __init__(self, render=False, device="cuda:0", precision=64):
        self.robot = InvertedDoublePendulumMuJoCo()
        BaseBulletEnv.__init__(self, self.robot, render, device, precision)
        self.stateId = -1
        self.scene = self.create_single_player_scene(None)


ENV_CLASSES = {
    "InvertedPendulumPyBulletEnv-v0": InvertedPendulumBulletEnv,
    "InvertedPendulumSwingupPyBulletEnv-v0": InvertedPendulumSwingupBulletEnv,
    "InvertedDoublePendulumPyBulletEnv-v0": InvertedDoublePendulumBulletEnv,
    "HopperPyBulletEnv-v0": HopperBulletEnv,
    "Walker2DPyBulletEnv-v0": Walker2DBulletEnv,
    "HalfCheetahPyBulletEnv-v0": HalfCheetahBulletEnv,
    "AntPyBulletEnv-v0": AntBulletEnv,
    "HumanoidPyBulletEnv-v0": HumanoidBulletEnv,
    "HumanoidFlagrunPyBulletEnv-v0": HumanoidFlagrunBulletEnv,
    "HumanoidFlagrunHarderPyBulletEnv-v0": HumanoidFlagrunHarderBulletEnv,
    "AtlasPyBulletEnv-v0": AtlasBulletEnv,
    "HopperMuJoCoEnv-v0": HopperMuJoCoEnv,
    "Walker2DMuJoCoEnv-v0": Walker2DMuJoCoEnv,
    "HalfCheetahMuJoCoEnv-v0": HalfCheetahMuJoCoEnv,
    "AntMuJoCoEnv-v0": AntMuJoCoEnv,
    "HumanoidMuJoCoEnv-v0": HumanoidMuJoCoEnv,
    "InvertedDoublePendulumMuJoCoEnv-v0": InvertedDoublePendulumMuJoCoEnv,
}
# envs/__init__.py:4-103 registry facts
MAX_EPISODE_STEPS = {k: 1000 for k in ENV_CLASSES}
REWARD_THRESHOLD = {"InvertedPendulumPyBulletEnv-v0": 950.0, "HopperPyBulletEnv-v0": 2500.0,
                    "InvertedPendulumSwingupPyBulletEnv-v0": 800.0, "InvertedDoublePendulumPyBulletEnv-v0": 9100.0,
                    "InvertedDoublePendulumMuJoCoEnv-v0": 9100.0,
                    "Walker2DPyBulletEnv-v0": 2500.0, "Walker2DMuJoCoEnv-v0": 2500.0,
                    "HalfCheetahMuJoCoEnv-v0": 3000.0, "HopperMuJoCoEnv-v0": 2500.0, "AntMuJoCoEnv-v0": 2500.0,
                    "HalfCheetahPyBulletEnv-v0": 3000.0, "AntPyBulletEnv-v0": 2500.0,
                    "HumanoidFlagrunPyBulletEnv-v0": 2000.0}  # envs/__init__.py:90


class TimeLimit:
    """gym's TimeLimit wrapper as applied by the registry (max_episode_steps)."""

    def __init__(self, env, max_episode_steps):
        self.env = env
        self._max = max_episode_steps
        self._elapsed = 0
        self.action_space, self.observation_space = env.action_space, env.observation_space

    def reset(self):
        self._elapsed = 0
        return self.env.reset()

    def step(self, a):
        obs, r, done, info = self.env.step(a)
        self._elapsed += 1
        if self._elapsed >= self._max:
            info["TimeLimit.truncated"] = not done
            done = True
        return obs, r, done, info

    def seed(self, seed=None):
        return self.env.seed(seed)

    def close(self):
        return self.env.close()

    def __getattr__(self, k):
        return getattr(self.env, k)


def make(env_id: str, device="cuda:0", precision: int = 64):
    """gym.make(env_id) equivalent: the env class behind gym's TimeLimit.  precision 64 (the
    default) is the reference's double-precision physics; 32 the float32 fast mode."""
    if env_id not in ENV_CLASSES:
        raise KeyError(f"unknown env id {env_id!r}; known: {sorted(ENV_CLASSES)}")
    return TimeLimit(ENV_CLASSES[env_id](device=device, precision=precision), MAX_EPISODE_STEPS[env_id])


def register_with_gym():
    """Register the ids with gym's registry when gym is importable (it is optional)."""
    try:
        from gym.envs.registration import register
    except Exception:
        return False
    for env_id, cls in ENV_CLASSES.items():
        kw = dict(id=env_id, entry_point=f"pybulletgym_amd.envs:{cls.__name__}",
                  max_episode_steps=MAX_EPISODE_STEPS[env_id])
        if env_id in REWARD_THRESHOLD:
            kw["reward_threshold"] = REWARD_THRESHOLD[env_id]
        try:
            register(**kw)
        except Exception:
            pass
    return True
