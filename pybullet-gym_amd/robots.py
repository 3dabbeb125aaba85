"""Per-robot environment constants, restated from the reference's robot/env classes.

Every constant cites the reference line it restates.  These feed the model tables
(``codegen.py``) that the HIP kernel and the CPU oracle share.
"""
from __future__ import annotations

import os
from collections import OrderedDict
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from . import mjcf

ALIVE_HOPPER = 0       # robot_locomotors.py:89-90   (+1 if z>0.8 and |pitch|<1 else -1)
ALIVE_HALFCHEETAH = 1  # robot_locomotors.py:116-118 (+1 if |pitch|<1 and no contact on feet 1,2,4,5)
ALIVE_ANT = 2          # robot_locomotors.py:137-138 (+1 if z>0.26 else -1)
ALIVE_HUMANOID = 3     # robot_locomotors.py:191-192 (+2 if z>0.78 else -1)
ALIVE_PENDULUM = 4     # gym_pendulum_envs.py:35-39  (reward 1, done |theta|>0.2)
ALIVE_SWINGUP = 5      # gym_pendulum_envs.py:31-34  (reward cos(theta), never done)
ALIVE_DOUBLE = 6       # gym_pendulum_envs.py:69-80  (reward 10 - dist_penalty, done pos_y+0.3<=1)
ALIVE_DOUBLE_MJ = 7    # mujoco/gym_pendulum_envs.py:60-72 (also - vel_penalty; MuJoCo obs)

KIND_WALKER = 0
KIND_PENDULUM = 1
KIND_MUJOCO_PLANAR = 2  # envs/mujoco Hopper / Walker2D / HalfCheetah: qpos/qvel obs, x-progress
KIND_MUJOCO_3D = 3      # envs/mujoco Ant / Humanoid: qpos[2:]/qvel (+ zero padding) obs, walker reward

ALIVE_MJ_HOPPER = 10    # mujoco/gym_locomotion_envs.py:127-137 (height > -0.3, |ang| < .2)
ALIVE_MJ_WALKER = 11    # :171-181 (1 > height > -0.2, -1 < ang < 1)
ALIVE_MJ_CHEETAH = 12   # :214-222 (never done, no alive bonus)
ALIVE_ATLAS = 13        # robot_locomotors.py:313-324 (+4 - knees at limit if head z > 1.3 else -1)


@dataclass
class RobotSpec:
    env_id: str
    key: str
    mjcf: str
    robot_name: str
    action_dim: int
    obs_dim: int
    kind: int
    power: float = 1.0
    foot_list: List[str] = field(default_factory=list)
    alive: int = ALIVE_ANT
    power_coef: Dict[str, float] = field(default_factory=dict)   # overrides of 100.0
    motor_order: Optional[List[str]] = None                      # Humanoid.apply_action order
    initial_z: Optional[float] = None                            # fixed z0 (Humanoid 0.8)
    electricity_cost: float = -2.0                               # gym_locomotion_envs.py:48
    stall_torque_cost: float = -0.1                              # gym_locomotion_envs.py:49
    joints_at_limit_cost: float = -0.1                           # gym_locomotion_envs.py:52
    timestep: float = 0.0165 / 4                                 # gym_locomotion_envs.py:19
    frame_skip: int = 4
    floor: bool = True
    max_episode_steps: int = 1000                                # envs/__init__.py
    self_collision: bool = True
    reset_offset: float = 0.0                                    # swingup hinge 3.1415 + u
    flagrun: bool = False                                        # HumanoidFlagrun walk target
    harder: bool = False                                         # HumanoidFlagrunHarder attacking cube
    urdf: Optional[str] = None                                   # URDF asset under assets/robots (Atlas)
    base_pos: Optional[List[float]] = None                       # reset snapshot base COM (URDF robots)
    head: Optional[str] = None                                   # Atlas alive_bonus: the head part
    knees: Optional[List[str]] = None                            # Atlas alive_bonus: the knee joints
    power_cost: float = 0.0                                      # MuJoCo planar: coef of sum(a^2)
    qvel_clip: float = 0.0                                       # MuJoCo planar: obs qvel clip (0: none)
    # the robot links' changeDynamics material (mujoco HalfCheetah, robot_locomotors.py:210); the
    # defaults are btCollisionObject's (restitution, spinning and rolling friction 0)
    restitution: float = 0.0
    spinning_friction: float = 0.0
    rolling_friction: float = 0.0


SPECS: Dict[str, RobotSpec] = OrderedDict()


def _add(s: RobotSpec):
    SPECS[s.key] = s


# InvertedPendulum: robot_pendula.py:5-51, gym_pendulum_envs.py:7-42, envs/__init__.py:4-9
_add(RobotSpec("InvertedPendulumPyBulletEnv-v0", "pendulum", "inverted_pendulum.xml", "cart",
               action_dim=1, obs_dim=5, kind=KIND_PENDULUM, power=1.0, alive=ALIVE_PENDULUM,
               timestep=0.0165, frame_skip=1, floor=False))
# InvertedPendulumSwingup: robot_pendula.py:11-18,54-55 (hinge reset 3.1415 + u),
# gym_pendulum_envs.py:26-34 (reward cos(theta), done False), envs/__init__.py:18-23
_add(RobotSpec("InvertedPendulumSwingupPyBulletEnv-v0", "pendulum_swingup", "inverted_pendulum.xml", "cart",
               action_dim=1, obs_dim=5, kind=KIND_PENDULUM, power=1.0, alive=ALIVE_SWINGUP,
               timestep=0.0165, frame_skip=1, floor=False, reset_offset=3.1415))
# InvertedDoublePendulum: robot_pendula.py:58-88, gym_pendulum_envs.py:45-86, envs/__init__.py:11-16
_add(RobotSpec("InvertedDoublePendulumPyBulletEnv-v0", "double_pendulum", "inverted_double_pendulum.xml", "cart",
               action_dim=1, obs_dim=9, kind=KIND_PENDULUM, power=2.0, alive=ALIVE_DOUBLE,
               timestep=0.0165, frame_skip=1, floor=False))
# InvertedDoublePendulumMuJoCoEnv: mujoco/robot_pendula.py:51-89, mujoco/gym_pendulum_envs.py:44-75,
# envs/__init__.py:113-118 (InvertedPendulumMuJoCoEnv-v0 is not built: its reset reads
# `self.swingup`, which the mujoco InvertedPendulum never defines -> AttributeError)
_add(RobotSpec("InvertedDoublePendulumMuJoCoEnv-v0", "double_pendulum_mujoco", "inverted_double_pendulum.xml",
               "cart", action_dim=1, obs_dim=11, kind=KIND_PENDULUM, power=2.0, alive=ALIVE_DOUBLE_MJ,
               timestep=0.0165, frame_skip=1, floor=False))
# Hopper: robot_locomotors.py:82-90, envs/__init__.py:73-78
_add(RobotSpec("HopperPyBulletEnv-v0", "hopper", "hopper.xml", "torso", action_dim=3, obs_dim=15,
               kind=KIND_WALKER, power=0.75, foot_list=["foot"], alive=ALIVE_HOPPER))
# HalfCheetah: robot_locomotors.py:109-127, envs/__init__.py:59-64
_add(RobotSpec("HalfCheetahPyBulletEnv-v0", "halfcheetah", "half_cheetah.xml", "torso", action_dim=6,
               obs_dim=26, kind=KIND_WALKER, power=0.90,
               foot_list=["ffoot", "fshin", "fthigh", "bfoot", "bshin", "bthigh"], alive=ALIVE_HALFCHEETAH,
               power_coef={"bthigh": 120.0, "bshin": 90.0, "bfoot": 60.0, "fthigh": 140.0,
                           "fshin": 60.0, "ffoot": 30.0}))
# Ant: robot_locomotors.py:130-138, envs/__init__.py:66-71
_add(RobotSpec("AntPyBulletEnv-v0", "ant", "ant.xml", "torso", action_dim=8, obs_dim=28,
               kind=KIND_WALKER, power=2.5,
               foot_list=["front_left_foot", "front_right_foot", "left_back_foot", "right_back_foot"],
               alive=ALIVE_ANT))
# Walker2D: robot_locomotors.py:93-106 (foot power_coef 30 set in robot_specific_reset),
# gym_locomotion_envs.py:128-131, envs/__init__.py:53-58
_add(RobotSpec("Walker2DPyBulletEnv-v0", "walker2d", "walker2d.xml", "torso", action_dim=6, obs_dim=22,
               kind=KIND_WALKER, power=0.40, foot_list=["foot", "foot_left"], alive=ALIVE_HOPPER,
               power_coef={"foot_joint": 30.0, "foot_left_joint": 30.0}))
# Humanoid: robot_locomotors.py:141-192, gym_locomotion_envs.py:146-151, envs/__init__.py:80-84
_add(RobotSpec("HumanoidPyBulletEnv-v0", "humanoid", "humanoid_symmetric.xml", "torso", action_dim=17,
               obs_dim=44, kind=KIND_WALKER, power=0.41, foot_list=["right_foot", "left_foot"],
               alive=ALIVE_HUMANOID,
               motor_order=["abdomen_z", "abdomen_y", "abdomen_x",
                            "right_hip_x", "right_hip_z", "right_hip_y", "right_knee",
                            "left_hip_x", "left_hip_z", "left_hip_y", "left_knee",
                            "right_shoulder1", "right_shoulder2", "right_elbow",
                            "left_shoulder1", "left_shoulder2", "left_elbow"],
               power_coef={"abdomen_z": 100, "abdomen_y": 100, "abdomen_x": 100,
                           "right_hip_x": 100, "right_hip_z": 100, "right_hip_y": 300, "right_knee": 200,
                           "left_hip_x": 100, "left_hip_z": 100, "left_hip_y": 300, "left_knee": 200,
                           "right_shoulder1": 75, "right_shoulder2": 75, "right_elbow": 75,
                           "left_shoulder1": 75, "left_shoulder2": 75, "left_elbow": 75},
               initial_z=0.8, electricity_cost=4.25 * -2.0, stall_torque_cost=4.25 * -0.1))

# HumanoidFlagrun: robot_locomotors.py:195-226 (flag_reposition / calc_state), the Humanoid
# physics and rewards (gym_locomotion_envs.py:146-163), envs/__init__.py:86-91
_add(RobotSpec("HumanoidFlagrunPyBulletEnv-v0", "humanoid_flagrun", "humanoid_symmetric.xml", "torso",
               action_dim=17, obs_dim=44, kind=KIND_WALKER, power=0.41, foot_list=["right_foot", "left_foot"],
               alive=ALIVE_HUMANOID, motor_order=SPECS["humanoid"].motor_order,
               power_coef=dict(SPECS["humanoid"].power_coef), initial_z=0.8,
               electricity_cost=4.25 * -2.0, stall_torque_cost=4.25 * -0.1, flagrun=True))

# MuJoCo-observation planar walkers (envs/mujoco, add_ignored_joints=True): obs
# qpos[1:] + qvel of every ordered joint incl. the ignored root joints, reward
# x-progress (+1 alive) + power cost; robot_locomotors.py (mujoco) :82-196,
# gym_locomotion_envs.py (mujoco) :121-252, envs/__init__.py:121-146
_add(RobotSpec("HopperMuJoCoEnv-v0", "hopper_mujoco", "hopper.xml", "torso", action_dim=3, obs_dim=11,
               kind=KIND_MUJOCO_PLANAR, power=0.75, alive=ALIVE_MJ_HOPPER, power_cost=-1e-3, qvel_clip=10.0))
_add(RobotSpec("Walker2DMuJoCoEnv-v0", "walker2d_mujoco", "walker2d.xml", "torso", action_dim=6, obs_dim=17,
               kind=KIND_MUJOCO_PLANAR, power=0.40, alive=ALIVE_MJ_WALKER,
               power_coef={"foot_joint": 30.0, "foot_left_joint": 30.0}, power_cost=-1e-3, qvel_clip=10.0))
_add(RobotSpec("HalfCheetahMuJoCoEnv-v0", "halfcheetah_mujoco", "half_cheetah.xml", "torso", action_dim=6,
               obs_dim=17, kind=KIND_MUJOCO_PLANAR, power=1.0, alive=ALIVE_MJ_CHEETAH,
               power_coef={"bthigh": 120.0, "bshin": 90.0, "bfoot": 60.0, "fthigh": 140.0,
                           "fshin": 60.0, "ffoot": 30.0}, power_cost=-0.1, qvel_clip=0.0,
               # robot_specific_reset :207-210: changeDynamics(lateralFriction=0.8,
               # spinningFriction=0.1, rollingFriction=0.1, restitution=0.5) on every part
               restitution=0.5, spinning_friction=0.1, rolling_friction=0.1))

# MuJoCo-observation floating-base walkers: obs [qpos[2:], qvel, zeros] (float64 in the
# reference), reward alive(state[0] + initial_z) + progress + joints_at_limit (no electricity);
# mujoco robot_locomotors.py:210-319, gym_locomotion_envs.py:39-118,243-260, envs/__init__.py:134-152
_add(RobotSpec("AntMuJoCoEnv-v0", "ant_mujoco", "ant.xml", "torso", action_dim=8, obs_dim=111,
               kind=KIND_MUJOCO_3D, power=2.5,
               foot_list=["front_left_foot", "front_right_foot", "left_back_foot", "right_back_foot"],
               alive=ALIVE_ANT))
_add(RobotSpec("HumanoidMuJoCoEnv-v0", "humanoid_mujoco", "humanoid_symmetric.xml", "torso", action_dim=17,
               obs_dim=376, kind=KIND_MUJOCO_3D, power=0.41, foot_list=["right_foot", "left_foot"],
               alive=ALIVE_HUMANOID, motor_order=SPECS["humanoid"].motor_order,
               power_coef=dict(SPECS["humanoid"].power_coef), initial_z=0.8))

# HumanoidFlagrunHarder: robot_locomotors.py:230-302 (the attacking cube of gym_utils.py:9-15,
# alive_bonus / potential_leak / crawl-disabling calc_potential), gym_locomotion_envs.py:167-178,
# envs/__init__.py:93-97.  The env's `self.electricity_cost /= 4` (:172) runs before
# HumanoidBulletEnv.__init__ sets electricity_cost = 4.25 * -2.0 (:150), which overwrites it: the
# Humanoid's costs stand (pinned by tests/golden/pack_humanoid_flagrun_harder.npz).
_add(RobotSpec("HumanoidFlagrunHarderPyBulletEnv-v0", "humanoid_flagrun_harder", "humanoid_symmetric.xml", "torso",
               action_dim=17, obs_dim=44, kind=KIND_WALKER, power=0.41, foot_list=["right_foot", "left_foot"],
               alive=ALIVE_HUMANOID, motor_order=SPECS["humanoid"].motor_order,
               power_coef=dict(SPECS["humanoid"].power_coef), initial_z=0.8,
               electricity_cost=4.25 * -2.0, stall_torque_cost=4.25 * -0.1, flagrun=True, harder=True))

# Atlas: robot_locomotors.py:305-341 (URDFBasedRobot atlas_v4_with_multisense.urdf, pelvis,
# power 2.9, robot_specific_reset -> reset_pose([0, 0, 0 + 1.0], yaw 0: random_yaw False),
# initial_z 1.5, alive_bonus from the head height and the knees), gym_locomotion_envs.py:181-191
# (StadiumScene timestep 0.0165/8, frame_skip 8), envs/__init__.py:99-103
_add(RobotSpec("AtlasPyBulletEnv-v0", "atlas", "", "pelvis", action_dim=30, obs_dim=70, kind=KIND_WALKER,
               power=2.9, foot_list=["r_foot", "l_foot"], alive=ALIVE_ATLAS, initial_z=1.5,
               timestep=0.0165 / 8, frame_skip=8, self_collision=False,
               urdf="atlas/atlas_description/atlas_v4_with_multisense.urdf", base_pos=[0.0, 0.0, 1.0],
               head="head", knees=["l_leg_kny", "r_leg_kny"]))

ENV_IDS = {s.env_id: s for s in SPECS.values()}


def spec_for(name: str) -> RobotSpec:
    if name in SPECS:
        return SPECS[name]
    if name in ENV_IDS:
        return ENV_IDS[name]
    raise KeyError(f"unknown robot/env id {name!r}; known: {list(ENV_IDS)}")


def add_to_scene_order(model: mjcf.RobotModel, robot_name: str):
    """Restates XmlBasedRobot.addToScene (robot_bases.py:54-91) on the compiled topology.

    Returns (parts, ordered_joint_links, robot_body) where parts is an ordered mapping
    part_name -> link index (-1 = base), in Python dict insertion order."""
    parts: "OrderedDict[str, int]" = OrderedDict()
    ordered: List[int] = []
    robot_body: Optional[int] = None
    for j, link in enumerate(model.links):
        parts[link.name] = j                                   # :72
        if link.name == robot_name:                            # :74-75
            robot_body = j
        if j == 0 and robot_body is None:                      # :77-79
            parts[robot_name] = -1
            robot_body = -1
        if link.joint_name[:6] == "ignore":                    # :81-83
            continue
        if link.joint_name[:8] != "jointfix":                  # :85-89
            ordered.append(j)
    return parts, ordered, robot_body


def reference_asset_dir() -> str:
    return os.path.join("/root/reference", "pybulletgym", "envs", "assets", "mjcf")


def reference_robot_dir() -> str:
    return os.path.join("/root/reference", "pybulletgym", "envs", "assets", "robots")


def compile_model(spec: RobotSpec, asset_dir: str = None):
    """The spec's robot compiled from its reference asset (MJCF, or URDF for Atlas)."""
    if spec.urdf:
        from . import urdf
        return urdf.compile_urdf(os.path.join(reference_robot_dir(), spec.urdf), spec.key, spec.base_pos)
    return mjcf.compile_mjcf(os.path.join(asset_dir or reference_asset_dir(), spec.mjcf), spec.key)
