"""pybulletgym_amd: MI355X-native batched stepper for the roboschool locomotion envs of
josiahls/pybullet-gym (InvertedPendulum, InvertedPendulumSwingup, InvertedDoublePendulum,
Hopper, HalfCheetah, Ant, Humanoid, HumanoidFlagrun, HumanoidFlagrunHarder, Walker2D, Atlas
``*PyBulletEnv-v0``, and the MuJoCo-observation variants).  Import as ``import pybulletgym_amd``.

    from pybulletgym_amd import VecEnv, make
    envs = VecEnv("AntPyBulletEnv-v0", 16384)      # device-resident batch, one launch per step
    env = make("AntPyBulletEnv-v0")                  # single env, gym.Env-style surface
"""
ENV_IDS = ("InvertedPendulumPyBulletEnv-v0", "HopperPyBulletEnv-v0", "HalfCheetahPyBulletEnv-v0",
           "AntPyBulletEnv-v0", "HumanoidPyBulletEnv-v0", "Walker2DPyBulletEnv-v0",
           "InvertedPendulumSwingupPyBulletEnv-v0", "InvertedDoublePendulumPyBulletEnv-v0",
           "HumanoidFlagrunPyBulletEnv-v0", "HopperMuJoCoEnv-v0", "Walker2DMuJoCoEnv-v0", "HalfCheetahMuJoCoEnv-v0",
           "AntMuJoCoEnv-v0", "HumanoidMuJoCoEnv-v0", "InvertedDoublePendulumMuJoCoEnv-v0",
           "HumanoidFlagrunHarderPyBulletEnv-v0", "AtlasPyBulletEnv-v0")


def __getattr__(name):
    # lazy: keep `import pybulletgym_amd` cheap and torch-free for the model compiler
    if name == "VecEnv":
        from .vec_env import VecEnv
        return VecEnv
    if name in ("make", "register_with_gym"):
        from . import envs
        return getattr(envs, name)
    raise AttributeError(name)
